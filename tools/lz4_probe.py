"""Times the LZ4 packet kernels on a bench-shaped packet (StringV2 "k%08d" + Decimal + Int64, 20M
rows) with the library's per-phase HIP-event profiler; run under rocprofv3 for kernel stats."""
import sys
import time

import torch

sys.path.insert(0, ".")
import tiflash_amd as tfa  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = tfa.Context(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(13)
    ids = torch.randint(0, 10_000_000, (n,), device=dev, generator=g, dtype=torch.int64)
    chars = torch.empty((n, 10), dtype=torch.uint8, device=dev)
    chars[:, 0] = ord("k")
    x = ids.clone()
    for j in range(8, 0, -1):
        chars[:, j] = (48 + x % 10).to(torch.uint8)
        x //= 10
    chars[:, 9] = 0
    offs = torch.arange(1, n + 1, device=dev, dtype=torch.int64) * 10
    v = torch.randint(0, 10**9, (n,), device=dev, generator=g, dtype=torch.int64)
    cols = [("k", "StringV2", chars.reshape(-1), offs, None), ("v", "Decimal(15,2)", v, None, None),
            ("id", "Int64", ids, None, None)]
    pkt = tfa.codec_encode(ctx, cols, n)
    for _ in range(2):
        lz = tfa.codec_compress(ctx, pkt)
        back = tfa.codec_decompress(ctx, lz)
    ctx.profile(True)
    ctx.profile_reset()
    t = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lz = tfa.codec_compress(ctx, pkt)
        t1 = time.perf_counter()
        back = tfa.codec_decompress(ctx, lz)
        t2 = time.perf_counter()
        t.append((t1 - t0, t2 - t1))
    prof = ctx.profile_read()
    assert torch.equal(back, pkt)
    print(f"packet {pkt.numel()} B -> {lz.numel()} B; compress {min(a for a, _ in t) * 1e3:.2f} ms, "
          f"decompress {min(b for _, b in t) * 1e3:.2f} ms")
    for k, (ms, cnt) in sorted(prof.items()):
        print(f"  {k}: {ms / max(cnt, 1):.3f} ms x {cnt}")


if __name__ == "__main__":
    main()
