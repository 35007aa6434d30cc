"""ZSTD packet decode probe (development tool): the bench's ZSTD leg alone — 64 MB of a StringV2
V1 packet body compressed by the system libzstd in 1 MB frames, decoded on the device, checked,
timed.  usage: python tools/zstd_probe.py [level] [frame_bytes] [steps] [library: a variant build,
timed without the output check]"""
import ctypes
import os
import struct
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tiflash_amd as tfa  # noqa: E402


def main():
    level = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    fsz = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    variant = sys.argv[4] if len(sys.argv) > 4 else None  # a measurement build (no output check)
    if variant:
        tfa.LIB_PATH = variant
    z = ctypes.CDLL("libzstd.so.1")
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compress.restype = ctypes.c_size_t
    # k%08d rows with '\0' terminators (the C5 / codec String column's chars), random ids
    rng = np.random.default_rng(13)
    ids = rng.integers(0, 10_000_000, (64 << 20) // 10)
    body = b"".join(b"k%08d\0" % i for i in ids.tolist())[:64 << 20]
    frames = []
    for i in range(0, len(body), fsz):
        chunk = body[i:i + fsz]
        cap = z.ZSTD_compressBound(ctypes.c_size_t(len(chunk)))
        buf = ctypes.create_string_buffer(cap)
        n = z.ZSTD_compress(buf, ctypes.c_size_t(cap), chunk, ctypes.c_size_t(len(chunk)), level)
        frames.append(b"\x90" + struct.pack("<II", n + 9, len(chunk)) + buf.raw[:n])
    zpkt = b"".join(frames)
    dev = torch.device("cuda", 0)
    dz = torch.frombuffer(bytearray(zpkt), dtype=torch.uint8).to(dev)
    with tfa.Context(0) as ctx:
        def run():
            try:
                return tfa.codec_decompress(ctx, dz)
            except tfa.TfgError:
                if not variant:
                    raise
        back = run()
        if not variant:
            assert back[1:].cpu().numpy().tobytes() == body, "ZSTD decompress mismatch"
        ts = []
        for _ in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    print(f"zstd level {level}: {len(frames)} frames, ratio {len(body) / len(zpkt):.3f}, {t * 1e3:.2f} ms, "
          f"{len(body) / t / 1e9:.3f} GB/s")


if __name__ == "__main__":
    main()
