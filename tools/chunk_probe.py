#!/usr/bin/env python3
"""Experiment: the C2 step consumed in K chunks (K consume calls into one Aggregator), to see
whether a chunk's staged records are re-read from the Infinity Cache (MALL) instead of HBM.
Prints per-kernel ms per step for each K."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import tiflash_amd as tfa

N, G = 100_000_000, 1_000_000
dev = torch.device("cuda", 0)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
f = torch.randint(0, 100, (N,), device=dev, generator=gen, dtype=torch.int64)
k = torch.randint(0, G, (N,), device=dev, generator=gen, dtype=torch.int64)
v = torch.randint(0, 1 << 20, (N,), device=dev, generator=gen, dtype=torch.int64).double() / 256.0
ctx = tfa.Context(0)
aggs = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
agg = tfa.Aggregator(ctx, tfa.INT64, aggs, expected_groups=G)
for K in [int(x) for x in (sys.argv[1:] or ["1", "4", "8", "16"])]:
    c = N // K

    def step():
        agg.reset()
        for i in range(K):
            agg.consume_filtered(f[i * c:(i + 1) * c], tfa.LT, 96, k[i * c:(i + 1) * c], [v[i * c:(i + 1) * c], None])
        return agg.result()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(5):
        res = step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / 5
    prof = ctx.profile_read()
    ctx.profile(False)
    print(json.dumps({"K": K, "ms": round(el * 1e3, 3), "groups": agg.size(),
                      "kernels": {n: round(x[0] / 5, 4) for n, x in sorted(prof.items())}}), flush=True)
