"""Times the single-pass C2 design (tools/singlepass_probe.hip: global atomics straight into a
1M-group table, no staging) on the bench's C2 input, and checks its counts.  Measurement only.
usage: python3 tools/singlepass_probe.py  (after building tools/_singlepass.so)"""
import ctypes
import json
import os

import torch


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    lib = ctypes.CDLL(os.path.join(here, "_singlepass.so"))
    dev = torch.device("cuda:0")
    n, groups = 100_000_000, 1_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    f = torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 100
    k = torch.randint(0, groups, (n,), device=dev, generator=g, dtype=torch.int64)
    v = torch.randint(0, 1 << 20, (n,), device=dev, generator=g).to(torch.float64) / 64
    s = torch.empty(groups, dtype=torch.float64, device=dev)
    c = torch.empty(groups, dtype=torch.int64, device=dev)
    ms = ctypes.c_float()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = lib.sp_run(p(f), p(k), p(v), ctypes.c_int64(n), ctypes.c_double(96.0), p(s), p(c), ctypes.c_int64(groups),
                    6, ctypes.byref(ms))
    torch.cuda.synchronize()
    kept = int((f < 96).sum())
    print(json.dumps({"design": "single pass, device-scope global atomics (sum f64 + count u64) into a dense "
                                "1M-group table", "rc": rc, "ms": round(ms.value, 4), "rows": n, "kept": kept,
                      "count_ok": int(c.sum()) == kept,
                      "input_GBps": round(24 * n / (ms.value * 1e-3) / 1e9, 1) if ms.value else None}))


if __name__ == "__main__":
    main()
