"""Times the non-partitioned C3 probe against an Infinity-Cache-sized bucketised build table
(tools/ic_probe.hip) on the bench's C3 input (10M build x 100M probe, ~50% hit), beside the
partitioned v1 probe of the library, and checks the match counts.  Measurement only.
usage: python3 tools/ic_probe.py  (after building tools/_ic_probe.so)"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import tiflash_amd as tfa
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_ic_probe.so"))
    dev = torch.device("cuda:0")
    nb, npr = 10_000_000, 100_000_000
    g2 = torch.Generator(device=dev)
    g2.manual_seed(7)  # bench.py's C3 data
    bk = torch.randperm(nb, device=dev, generator=g2).to(torch.int64) * 4 + 1
    bpay = torch.randint(0, 1 << 40, (nb,), device=dev, generator=g2, dtype=torch.int64)
    hit = torch.rand(npr, device=dev, generator=g2) < 0.5
    pk = torch.where(hit, bk[torch.randint(0, nb, (npr,), device=dev, generator=g2)],
                     torch.randint(0, 1 << 40, (npr,), device=dev, generator=g2) * 4 + 3)
    ppay = torch.randint(0, 1 << 40, (npr,), device=dev, generator=g2, dtype=torch.int64)
    del hit
    expect = int(torch.isin(pk, bk).sum().item())
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    out = {"rows": npr, "build": nb, "expected_matches": expect, "runs": []}
    cap = npr
    o = [torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(3)]
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    for bits in (20, 21):
        table = torch.empty((16 << bits,), dtype=torch.int64, device=dev)
        ms = ctypes.c_float()
        rc = lib.icp_build(p(bk), ctypes.c_int64(nb), bits, p(table), p(ovf), ctypes.byref(ms))
        torch.cuda.synchronize()
        run = {"bucket_bits": bits, "table_MB": (16 << bits) * 8 / 2**20, "build_rc": rc,
               "build_ms": round(ms.value, 3), "overflow_rows": int(ovf.item())}
        for mode in (0, 1):
            for grid in (2048, 8192):
                rc = lib.icp_probe(mode, p(pk), p(ppay), ctypes.c_int64(npr), bits, p(table), p(bk), p(bpay), p(cnt),
                                   p(o[0]), p(o[1]), p(o[2]), ctypes.c_uint64(cap), grid, 5, ctypes.byref(ms))
                torch.cuda.synchronize()
                run[f"mode{mode}_grid{grid}"] = {"rc": rc, "ms": round(ms.value, 4), "matches": int(cnt.item()),
                                                 "ok": int(cnt.item()) == expect}
        if run["mode1_grid8192"]["ok"]:  # the materialised rows: build payload of the probe key
            m = expect
            pos = torch.searchsorted(torch.sort(bk).values, o[0][:m])
            order = torch.argsort(bk)
            run["rows_ok"] = bool(torch.equal(bpay[order][pos], o[2][:m]))
        out["runs"].append(run)
        del table
    # the partitioned v1 probe (bench.py's C3 leg) on the same input, same process
    with tfa.Context(0) as ctx:
        j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
        j.build(bk, payload=[bpay])
        j.finalize()
        outs = ([torch.empty(npr, dtype=torch.int64, device=dev) for _ in range(2)],
                [torch.empty(npr, dtype=torch.int64, device=dev)], torch.empty(npr, dtype=torch.uint8, device=dev))
        for _ in range(2):
            j.probe_rows(pk, [pk, ppay], 1, capacity=npr, outs=outs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            op, ob, _ = j.probe_rows(pk, [pk, ppay], 1, capacity=npr, outs=outs)
        torch.cuda.synchronize()
        out["v1_ms"] = round((time.perf_counter() - t0) / 5 * 1e3, 4)
        out["v1_matches"] = int(op[0].shape[0])
        j.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
