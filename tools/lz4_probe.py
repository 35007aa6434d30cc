"""LZ4 packet compress / decompress probe (development tool): a NONE packet of k%08d rows
(V1 String chars) compressed and decompressed on the device, checked, timed.
usage: python tools/lz4_probe.py [MB] [steps] [library: a variant build]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tiflash_amd as tfa  # noqa: E402


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    if len(sys.argv) > 3:
        tfa.LIB_PATH = sys.argv[3]
    rng = np.random.default_rng(13)
    ids = rng.integers(0, 10_000_000, (mb << 20) // 10)
    body = b"".join(b"k%08d\0" % i for i in ids.tolist())[:mb << 20]
    pkt = torch.frombuffer(bytearray(b"\x02" + body), dtype=torch.uint8).to("cuda")
    with tfa.Context(0) as ctx:
        z = tfa.codec_compress(ctx, pkt)
        back = tfa.codec_decompress(ctx, z)
        assert torch.equal(back, pkt), "LZ4 round trip"
        tc, td = [], []
        for _ in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            z = tfa.codec_compress(ctx, pkt)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            tfa.codec_decompress(ctx, z)
            torch.cuda.synchronize()
            tc.append(t1 - t0)
            td.append(time.perf_counter() - t1)
    c, d = sorted(tc)[steps // 2], sorted(td)[steps // 2]
    print(f"lz4 {mb} MB: ratio {len(body) / z.numel():.3f}, compress {c * 1e3:.2f} ms {len(body) / c / 1e9:.2f} GB/s, "
          f"decompress {d * 1e3:.2f} ms {len(body) / d / 1e9:.2f} GB/s")


if __name__ == "__main__":
    main()
