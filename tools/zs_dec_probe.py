import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import tiflash_amd as tfa
rng = np.random.default_rng(13)
ids = rng.integers(0, 10_000_000, (256 << 20) // 10)
body = b"".join(b"k%08d\0" % i for i in ids.tolist())[:256 << 20]
pkt = torch.frombuffer(bytearray(b"\x02" + body), dtype=torch.uint8).to("cuda")
with tfa.Context(0) as ctx:
    z = tfa.codec_compress(ctx, pkt, method=tfa.COMPRESSION_ZSTD)
    for _ in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        back = tfa.codec_decompress(ctx, z)
        torch.cuda.synchronize(); print("decode ms", (time.perf_counter() - t0) * 1e3, flush=True)
    assert torch.equal(back, pkt)
