"""ZSTD sender probe (development tool): compression ratio of the device ZSTD sender on several
payload shapes (next to libzstd level 1 on the same 64 KB frames and the device LZ4 sender) and its
throughput on a 256 MB NONE packet of k%08d rows; every output checked by the device decoder.
usage: python tools/zenc_probe.py [library ...]   (variant builds; default: the in-tree library)"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tiflash_amd as tfa  # noqa: E402


def payloads():
    rng = np.random.default_rng(7)
    mb = 4 << 20
    yield "k%08d rows", b"".join(b"k%08d\0" % i for i in rng.integers(0, 10_000_000, mb // 10).tolist())[:mb]
    yield "key%08d| (1000 keys)", b"".join(b"key%08d|" % i for i in rng.integers(0, 1000, mb // 12).tolist())[:mb]
    yield "4-symbol random", bytes(rng.integers(0, 4, mb, dtype=np.uint8))
    yield "Int64 0..999", rng.integers(0, 1000, mb // 8).astype(np.int64).tobytes()
    yield "Float64 prices", np.round(rng.random(mb // 8) * 1000, 2).tobytes()
    words = [b"alpha", b"beta", b"gamma", b"delta", b"epsilon", b"zeta", b"eta", b"theta"]
    yield "text-ish", b" ".join(words[i] for i in rng.integers(0, 8, mb // 6).tolist())[:mb]
    yield "geometric bytes", (rng.geometric(0.02, mb) % 256).astype(np.uint8).tobytes()


def zstd1(raw):
    try:
        z = ctypes.CDLL("libzstd.so.1")
    except OSError:
        return None
    z.ZSTD_compress.restype = ctypes.c_size_t
    total = 0
    out = ctypes.create_string_buffer(70000)
    for i in range(0, len(raw), 65536):
        c = raw[i:i + 65536]
        total += z.ZSTD_compress(out, ctypes.c_size_t(70000), c, ctypes.c_size_t(len(c)), 1) + 9
    return total


def frame_stats(pkt: bytes):
    """block / literal / sequence-table modes of the sender's frames (one block each)"""
    from collections import Counter
    st, pos = Counter(), 0
    while pos < len(pkt):
        fb = int.from_bytes(pkt[pos + 1:pos + 5], "little")
        c = pkt[pos + 18:pos + fb]
        bh = int.from_bytes(c[:3], "little")
        c = c[3:]
        btype = (bh >> 1) & 3
        if btype == 0:
            st["raw block"] += 1
        else:
            lt, fmt = c[0] & 3, (c[0] >> 2) & 3
            if lt == 0:
                st["lit raw"] += 1
                lsz = 3 + (int.from_bytes(c[:3], "little") >> 4)
            elif lt == 1:
                st["lit rle"] += 1
                lsz = 4
            else:
                h = 5 if fmt == 3 else 4 if fmt == 2 else 3
                v = int.from_bytes(c[:h], "little")
                csz = (v >> 22) & 0x3FFFF if fmt == 3 else (v >> 14) & 0x3FF
                st["lit huf " + ("fse" if c[h] < 128 else "direct")] += 1
                lsz = h + csz
            q = c[lsz:]
            ns = q[0] if q[0] < 128 else ((q[0] - 128) << 8) + q[1]
            if ns:
                m = q[1 if q[0] < 128 else 2]
                st["seq modes %d%d%d" % (m >> 6, (m >> 4) & 3, (m >> 2) & 3)] += 1
            else:
                st["no sequences"] += 1
        pos += fb
    return dict(st)


def main():
    libs = sys.argv[1:] or [None]
    data = list(payloads())
    refs = [zstd1(raw) for _, raw in data]
    rng = np.random.default_rng(13)
    big = b"".join(b"k%08d\0" % i for i in rng.integers(0, 10_000_000, (256 << 20) // 10).tolist())[:256 << 20]
    for lib in libs:
        if lib:
            tfa.LIB_PATH = lib
            tfa._lib = None
        with tfa.Context(0) as ctx:
            print(f"== {lib or 'in-tree'}")
            for (name, raw), ref in zip(data, refs):
                pkt = torch.frombuffer(bytearray(b"\x02" + raw), dtype=torch.uint8).to("cuda")
                z = tfa.codec_compress(ctx, pkt, method=tfa.COMPRESSION_ZSTD)
                assert torch.equal(tfa.codec_decompress(ctx, z), pkt), name
                lz = tfa.codec_compress(ctx, pkt).numel()
                print(f"  {name:24s} zstd {len(raw) / z.numel():6.3f}  libzstd-1 {len(raw) / ref if ref else 0:6.3f}"
                      f"  lz4 {len(raw) / lz:6.3f}  {frame_stats(z.cpu().numpy().tobytes())}")
            pkt = torch.frombuffer(bytearray(b"\x02" + big), dtype=torch.uint8).to("cuda")
            ts = []
            if hasattr(tfa.lib(), "tfg_zenc_prof"):
                tfa.lib().tfg_zenc_prof((ctypes.c_ulonglong * 8)())
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                z = tfa.codec_compress(ctx, pkt, method=tfa.COMPRESSION_ZSTD)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            t = sorted(ts)[2]
            L = tfa.lib()
            if hasattr(L, "tfg_zenc_prof"):  # a TFG_ZE_PROF build: phase totals over the last 5 calls
                ph = (ctypes.c_ulonglong * 8)()
                L.tfg_zenc_prof(ph)
                names = ["match", "seq counts", "literals", "tables", "sequences", "headers"]
                tot = sum(ph[:6]) or 1
                print("  phases (share of wave time): " + ", ".join(f"{n} {ph[i] / tot:.1%}" for i, n in enumerate(names)))
                print(f"  per frame: {tot / 100e6 / (5 * ((len(big) + 65535) // 65536)) * 1e6:.1f} us of wave time")
            print(f"  256 MB k%08d rows: ratio {len(big) / z.numel():.3f}, compress {t * 1e3:.2f} ms, "
                  f"{len(big) / t / 1e9:.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()
