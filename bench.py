#!/usr/bin/env python3
"""bench.py — TPC-H Q1-shaped filter -> hash GROUP BY (BASELINE.json configs[1]) on MI355X.

One "step" = one pass of the hot path over one batch of synthetic rows already resident in HBM:
    Aggregator reset -> fused (f < 96) filter + GROUP BY k: sum(v), count(*) -> final Block (result
    columns materialised on the device).
`--gpus N` (N > 1) without a torchrun environment starts N ranks itself (torch.distributed.run
as a child process, before this process touches the GPU).  Every rank aggregates its own 100M
rows (weak scaling), the partial (key, sum, count) rows are hash-repartitioned with fillSelector
and exchanged with an RCCL all-to-all (the MPP ExchangeSender/Receiver of a two-phase
aggregation), then merged by a final aggregation.  value = rows of all ranks / max-over-ranks time.

Extras in the same JSON line: the §8(d) variants (selectivity sweep 0/1/10/50/100 %, Int64 value
column), the hash-join probe (configs[2] shape, N=1), the repartitioned join (configs[3], N>1),
the String + Decimal GROUP BY (configs[4]), the packet codec, the per-kernel roofline of the
dominant kernel from HIP events recorded on the library's stream, and the CPU baseline (oracle
restatement of the reference's algorithm) on the host cores.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--threshold", type=int, default=96)
    ap.add_argument("--join-build", type=int, default=10_000_000)
    ap.add_argument("--join-probe", type=int, default=100_000_000)
    ap.add_argument("--no-join", action="store_true")
    ap.add_argument("--join-v2", action="store_true",
                    help="also time the C3 probe through JoinV2's pointer table (off by default: DESIGN §5)")
    ap.add_argument("--no-variants", action="store_true", help="skip the selectivity sweep / Int64-value legs")
    ap.add_argument("--c5-rows", type=int, default=100_000_000, help="C5 String-key GROUP BY rows per GPU (0 = skip)")
    ap.add_argument("--c5-groups", type=int, default=10_000_000)
    ap.add_argument("--codec-rows", type=int, default=20_000_000, help="packet codec leg rows (0 = skip)")
    ap.add_argument("--c4", type=int, default=-1, help="repartitioned join leg (configs[3]): 1 on, 0 off, -1 = on when N > 1")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: every rank holds --rows (and the other legs' sizes); strong: the sizes are job "
                         "totals, split evenly over the ranks")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--value-int64", action="store_true", help="Int64 value column instead of Float64 (headline leg)")
    ap.add_argument("--bucket-bits", type=int, default=0, help="aggregation radix buckets (0 = from --groups)")
    ap.add_argument("--c5-bucket-bits", type=int, default=0, help="C5 aggregation radix buckets (0 = from --c5-groups)")
    ap.add_argument("--c5-expected-groups", type=int, default=0,
                    help="C5 aggregators' expected_groups (their table sizing; 0 = --c5-groups)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, production) or gloo (rehearsal: all ranks may share one GPU)")
    return ap.parse_args()


def launch_ranks(args) -> int:
    """--gpus N > 1 outside torchrun: start N ranks (one process per GPU) with torch.distributed.run
    as a CHILD process and return its exit code.  Nothing here touches the GPU."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# Algorithmic HBM bytes of each kernel: the bytes a perfect implementation must
# move — every input byte once (f, k, v = 24 B per input row for C2) plus the output.  Staging
# records a kernel writes and a later kernel re-reads are the implementation's cost, reported
# separately as moved_bytes (and measured by the PMC passes as traffic).
def kernel_bytes(name, n_in, n_kept, n_groups):
    alg = {
        "agg.part.tiled": 24 * n_in,
        "agg.part.hist": 16 * n_in,
        "agg.part.scatter": 24 * n_in,
        "agg.bucket": 24 * n_groups,
        "join.part.hist": 8 * n_in,
        "join.part.scatter": 16 * n_in,
        "join.probe": 0,
    }.get(name)
    moved = {
        "agg.part.tiled": 24 * n_in + 16 * n_kept,
        "agg.part.hist": 16 * n_in,
        "agg.part.scatter": 24 * n_in + 16 * n_kept,
        "agg.bucket": 16 * n_kept + 24 * n_groups,
    }.get(name)
    return alg, moved


def roofline_from_profile(prof, steps, n_in, n_kept, n_groups):
    if not prof:
        return None
    name, (ms, cnt) = max(prof.items(), key=lambda kv: kv[1][0])
    per_launch_ms = ms / max(cnt, 1)
    alg, moved = kernel_bytes(name, n_in, n_kept, n_groups)
    launches_per_step = cnt / max(steps, 1)
    if not alg or per_launch_ms <= 0:
        return {"kernel": name, "avg_ms": per_launch_ms}
    b_launch = alg / launches_per_step
    ach = b_launch / (per_launch_ms * 1e-3) / 1e9
    out = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "avg_ms": round(per_launch_ms, 4),
           "algorithmic_bytes_per_launch": int(b_launch),
           "algorithmic_basis": "SURVEY 8(d): 24 B per input row (f, k, v) read once (+ 24 B per group out)"}
    if moved:
        out["moved_bytes_per_launch"] = int(moved / launches_per_step)
        out["moved_GBps"] = round(moved / launches_per_step / (per_launch_ms * 1e-3) / 1e9, 1)
    return out


def load_pmc_traffic(kernel):
    """HBM bytes per launch measured by the rocprofv3 PMC passes (profiles/pmc_traffic.json), if any."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def pmc_source():
    """Which profile run (tools/profile.sh tag) and commit the PMC traffic figures come from."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            c = json.load(f).get("_calibration", {})
        return {"file": "profiles/pmc_traffic.json", "tag": c.get("tag"), "commit": c.get("commit")}
    except Exception:
        return None


def load_pmc_step(leg):
    """HBM bytes per bench step of a leg from the same PMC passes (profiles/pmc_traffic.json)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get("_per_step", {}).get(leg, {}).get("hbm_bytes")
    except Exception:
        return None


def host_cores():
    """Host CPUs this process may use: affinity mask, capped by a cgroup CPU quota and by the
    OMP_NUM_THREADS the GPU box sets to its per-GPU CPU share."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except Exception:
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        cores = min(cores, int(omp))
    return cores, {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                   "omp_num_threads": omp}


def cpu_baseline(args):
    import numpy as np
    from oracle import oracle as orc
    cores, host = host_cores()
    threads = args.cpu_threads or cores
    n = args.rows  # the full C2 batch
    rng = np.random.default_rng(1)
    f = rng.integers(0, 100, n, dtype=np.int64)
    k = rng.integers(0, args.groups, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0
    times = []
    t_end = time.time() + 20.0
    while len(times) < 3 or (time.time() < t_end and len(times) < 5):
        t0 = time.perf_counter()
        orc.bench_filter_agg_ref(f, args.threshold, k, v, threads, 65536)
        times.append(time.perf_counter() - t0)
        if time.time() > t_end and len(times) >= 1:
            break
    med = statistics.median(times)
    out = {"value": round(n / med, 1), "unit": "rows/s", "cores": threads, "kind": "port", "host": host,
           "sample": f"{n} rows (the full C2 batch) x {len(times)} runs (median), same distribution, 65536-row blocks, "
                     f"per-thread key64 HashMap (CRC32-C, arena states, prefetch, two-level at 100k keys) + "
                     f"bucket-parallel merge + result conversion (reference-algorithm CPU restatement, "
                     f"oracle/cpu_baseline.c)"}
    return out


def cpu_join_baseline(args):
    import numpy as np
    from oracle import oracle as orc
    cores, host = host_cores()
    threads = args.cpu_threads or cores
    nb, npr = args.join_build, args.join_probe  # the full C3 sizes
    rng = np.random.default_rng(7)
    bk = rng.permutation(nb).astype(np.int64) * 4 + 1
    bpay = rng.integers(0, 1 << 40, nb, dtype=np.int64)
    pk = np.where(rng.random(npr) < 0.5, bk[rng.integers(0, nb, npr)], rng.integers(0, 1 << 40, npr) * 4 + 3)
    pk = pk.astype(np.int64)
    ppay = rng.integers(0, 1 << 40, npr, dtype=np.int64)
    t0 = time.perf_counter()
    jb = orc.JoinBench(bk, bpay, threads)
    build_s = time.perf_counter() - t0
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        jb.probe(pk, ppay)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(npr / med, 1), "unit": "probe rows/s", "cores": threads, "kind": "port", "host": host,
            "build_s": round(build_s, 3),
            "sample": f"build {nb} rows into {threads} segment HashMaps of RowRefList cells (not timed), "
                      f"probe {npr} rows x 3 runs (median) with materialised output blocks "
                      f"(reference-algorithm CPU restatement, oracle/cpu_baseline.c)"}


def cpu_string_baseline(args):
    import numpy as np
    from oracle import oracle as orc
    cores, host = host_cores()
    threads = args.cpu_threads or cores
    n = args.c5_rows  # the full batch (~10 s a run at the restatement's ~10M rows/s on 16 threads)
    rng = np.random.default_rng(11)
    ids = rng.integers(0, args.c5_groups, n)
    chars = np.empty((n, 10), np.uint8)
    chars[:, 0] = ord("k")
    x = ids.copy()
    for j in range(8, 0, -1):
        chars[:, j] = 48 + x % 10
        x //= 10
    chars[:, 9] = 0
    chars = chars.reshape(-1)
    offs = (np.arange(1, n + 1, dtype=np.uint64) * 10)
    v = rng.integers(0, 10**9, n, dtype=np.int64)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        orc.bench_string_agg(chars, offs, v, threads)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(n / med, 1), "unit": "rows/s", "cores": threads, "kind": "port", "host": host,
            "sample": f"{n} rows x 3 runs (median), k%08d keys over {args.c5_groups} ids, per-thread StringHashMap "
                      f"StringKey16 sub-maps (CRC32-C, arena Decimal128+count states, prefetch, two-level at 100k keys) "
                      f"+ bucket-parallel merge + result conversion (reference-algorithm CPU restatement, "
                      f"oracle/cpu_baseline_str.c)"}


def c4_leg(args, ctx, dev, world, rank):
    """configs[3]: hash-repartitioned join.  Every rank holds join_build build rows and join_probe
    probe rows (C3 distributions over the global key space); a step repartitions both sides by the
    reference's weak hash + fillSelector (ExchangeSender, HashPartitionWriter) with an RCCL
    all-to-all, builds the local hash table and runs the materialising probe.  value = probe rows
    of all ranks / max-over-ranks step time (weak scaling)."""
    import torch
    import torch.distributed as dist

    import tiflash_amd as tfa
    from tiflash_amd.exchange import exchange_sides
    nb, npr = args.join_build, args.join_probe
    g = torch.Generator(device=dev)
    g.manual_seed(7 + 1000 * rank)
    bk = (torch.randperm(nb, device=dev, generator=g).to(torch.int64) + rank * nb) * 4 + 1
    bpay = torch.randint(0, 1 << 40, (nb,), device=dev, generator=g, dtype=torch.int64)
    hit = torch.rand(npr, device=dev, generator=g) < 0.5
    pk = torch.where(hit, torch.randint(0, nb * world, (npr,), device=dev, generator=g) * 4 + 1,
                     torch.randint(0, 1 << 40, (npr,), device=dev, generator=g) * 4 + 3)
    ppay = torch.randint(0, 1 << 40, (npr,), device=dev, generator=g, dtype=torch.int64)
    del hit
    cap = npr * 3 // 4 + (1 << 20)
    outs = ([torch.empty(cap, dtype=torch.int64, device=dev) for _ in range(2)],
            [torch.empty(cap, dtype=torch.int64, device=dev)], torch.empty(cap, dtype=torch.uint8, device=dev))
    state = {}

    def step():
        if world > 1:  # both sides repartitioned, then ONE fused exchange (one counts + one data all-to-all)
            bcols, boffs = tfa.hash_partition(ctx, [bk, bpay], [0], world)
            pcols, poffs = tfa.hash_partition(ctx, [pk, ppay], [0], world)
            lb, lp = exchange_sides([(bcols, boffs), (pcols, poffs)])
        else:
            lb, lp = [bk, bpay], [pk, ppay]
        j = tfa.Join(ctx, tfa.INT64, expected_build_rows=lb[0].shape[0])
        j.build(lb[0], payload=[lb[1]])
        j.finalize()
        n_out = lp[0].shape[0] * 3 // 4 + (1 << 20)
        o = outs if n_out <= cap else None
        op, ob, _ = j.probe_rows(lp[0], [lp[0], lp[1]], 1, capacity=cap if o else None, outs=o)
        state["matches"] = op[0].shape[0]
        state["probe_rows"] = lp[0].shape[0]
        state["join"] = j  # freed at the next step (after its kernels are done)
        return op

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    inv = torch.tensor([float(state["matches"]), float(state["probe_rows"])], dtype=torch.float64, device=red_dev)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        dist.all_reduce(inv)
    matches, probe_total = (int(z) for z in inv.tolist())
    ms = el / args.steps * 1e3
    state.clear()
    return {"metric": "probe rows/s on the hash-repartitioned join (C3 per GPU: 10M build x 100M probe, "
                      "weak hash + fillSelector + RCCL all-to-all of both sides, local build + materialising probe)",
            "value": round(npr * world * args.steps / el, 1), "unit": "rows/s", "ms_per_step": round(ms, 3),
            "scaling": args.scaling, "config": {"workload": "configs[3] repartitioned join", "build_rows_per_gpu": nb,
                                          "probe_rows_per_gpu": npr, "parallelism": f"dp{world}"},
            "check": {"probe_rows_total": probe_total, "expected_probe_rows": npr * world, "matches": matches,
                      "ok": probe_total == npr * world},
            "kernels_ms_per_step": {kname: round(vv[0] / args.steps, 4) for kname, vv in sorted(prof.items())}}


def c5_leg(args, ctx, dev, world, rank):
    """configs[4]: GROUP BY a String key ("k%08d", c5_groups distinct) with sum(Decimal(15,2)) ->
    Decimal(37,2) and count(*); N>1: partial -> packed-key RCCL exchange -> final (two-phase)."""
    import torch
    import torch.distributed as dist

    import tiflash_amd as tfa
    from tiflash_amd.exchange import two_phase_merge_keys
    n, G = args.c5_rows, args.c5_groups
    g = torch.Generator(device=dev)
    g.manual_seed(11 + rank)
    ids = torch.randint(0, G, (n,), device=dev, generator=g, dtype=torch.int64)
    chars = torch.empty((n, 10), dtype=torch.uint8, device=dev)
    chars[:, 0] = ord("k")
    x = ids.clone()
    for j in range(8, 0, -1):
        chars[:, j] = (48 + x % 10).to(torch.uint8)
        x //= 10
    chars[:, 9] = 0
    del x, ids
    chars = chars.reshape(-1)
    offs = torch.arange(1, n + 1, device=dev, dtype=torch.int64) * 10
    v = torch.randint(0, 10**9, (n,), device=dev, generator=g, dtype=torch.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    eg = args.c5_expected_groups or G
    part = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=eg, bucket_bits=args.c5_bucket_bits)
    fin = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=eg, bucket_bits=args.c5_bucket_bits) if world > 1 else None

    hint = min(G, n)  # the result's buffers before its count is read (<= G groups)

    def step():
        part.reset()
        part.consume([(chars, offs)], [v, None])
        if world == 1:
            return part.result(capacity_hint=hint)
        fin.reset()
        two_phase_merge_keys(ctx, part, fin)
        return fin.result(capacity_hint=hint)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    inv = torch.tensor([float(res["states"][1].view(torch.int64).sum().item()), float(res["states"][1].shape[0])],
                       dtype=torch.float64, device=red_dev)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        dist.all_reduce(inv)
    cnt_total, groups_total = (int(z) for z in inv.tolist())
    ms = el / args.steps * 1e3
    alg = n * (8 + 10 + 8)  # offsets + chars + value per row
    out = {"metric": "rows/s on GROUP BY String key (k%08d) sum(Decimal64)->Decimal128 + count" +
                     (" two-phase + RCCL all-to-all" if world > 1 else ""),
           "value": round(n * world * args.steps / el, 1), "unit": "rows/s", "ms_per_step": round(ms, 3),
           "scaling": args.scaling,
           "config": {"workload": "configs[4] String + Decimal GROUP BY", "rows_per_gpu": n, "groups": G},
           "check": {"count_total": cnt_total, "rows_total": n * world, "groups_total": groups_total,
                     "ok": cnt_total == n * world and groups_total <= G},
           "pipeline_roofline": {"algorithmic_bytes_per_step": alg, "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
           "kernels_ms_per_step": {kname: round(vv[0] / args.steps, 4) for kname, vv in sorted(prof.items())}}
    for o in (part, fin):
        if o is not None:
            o.close()
    del chars, offs, v
    if world == 1 and not args.no_variants:
        out["var_len_keys"] = c5_var_len_leg(args, ctx, dev)
    return out


def var_len_keys_torch(ids):
    """SURVEY §8(d)'s C5 variant, 1- to 11-byte keys: group id -> every 1-, 2- and 3-byte key of
    the 94 printable characters, then lengths 4..11 in turn, the id's value in base 94 (no key
    is hot: c5_groups distinct keys, ~10 rows each).  tests/test_gpu_full_scale.py var_len_keys is
    the same map in numpy.  Returns (chars, end offsets) of the ColumnString."""
    import torch
    c1, c2, c3 = 94, 94 + 94**2, 94 + 94**2 + 94**3
    r = ids - c3
    L = torch.where(ids < c1, 1, torch.where(ids < c2, 2, torch.where(ids < c3, 3, 4 + r % 8)))
    q = torch.where(ids < c1, ids, torch.where(ids < c2, ids - c1, torch.where(ids < c3, ids - c2, r // 8)))
    del r
    offs = torch.cumsum(L + 1, 0)
    starts = offs - (L + 1)
    chars = torch.zeros(int(offs[-1].item()), dtype=torch.uint8, device=ids.device)
    for k in range(11):
        sel = L > k
        chars[(starts + L - 1 - k)[sel]] = (33 + q[sel] % 94).to(torch.uint8)
        q = q // 94
    return chars, offs


def c5_var_len_leg(args, ctx, dev):
    """The C5 step over 1- to 11-byte String keys (StringHashMap's size classes, reference
    Common/HashTable/StringHashTable.h:211-310), c5_rows rows over c5_groups ids (
    c5_groups distinct keys of every length 1-11), with its CPU restatement beside it."""
    import torch

    import tiflash_amd as tfa
    n, G = args.c5_rows, args.c5_groups
    g = torch.Generator(device=dev)
    g.manual_seed(17)
    ids = torch.randint(0, G, (n,), device=dev, generator=g, dtype=torch.int64)
    chars, offs = var_len_keys_torch(ids)
    del ids
    v = torch.randint(0, 10**9, (n,), device=dev, generator=g, dtype=torch.int64)
    aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
    part = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=G)
    hint = min(G, n)

    def step():
        part.reset()
        part.consume([(chars, offs)], [v, None])
        return part.result(capacity_hint=hint)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    cnt_total = int(res["states"][1].view(torch.int64).sum().item())
    groups = int(res["states"][1].shape[0])
    ms = el / args.steps * 1e3
    alg = 8 * n + int(chars.numel()) + 8 * n  # offsets + chars + value
    out = {"metric": "rows/s on GROUP BY a 1- to 11-byte String key sum(Decimal64)->Decimal128 + count",
           "value": round(n * args.steps / el, 1), "unit": "rows/s", "ms_per_step": round(ms, 3),
           "config": {"rows": n, "ids": G, "key_bytes": "1-11 (mean %.1f)" % (chars.numel() / n - 1)},
           "check": {"count_total": cnt_total, "rows_total": n, "groups": groups, "ok": cnt_total == n},
           "pipeline_roofline": {"algorithmic_bytes_per_step": alg, "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
           "kernels_ms_per_step": {kname: round(vv[0] / args.steps, 4) for kname, vv in sorted(prof.items())}}
    part.close()
    del chars, offs, v
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_var_len_baseline(args)
    return out


def cpu_var_len_baseline(args):
    """oracle/cpu_baseline_str.c over the same 1-11-byte key distribution (numpy copy of
    var_len_keys_torch), its full batch, median of 3."""
    import numpy as np
    from oracle import oracle as orc
    cores, host = host_cores()
    threads = args.cpu_threads or cores
    n, G = args.c5_rows, args.c5_groups
    rng = np.random.default_rng(17)
    ids = rng.integers(0, G, n)
    c1, c2, c3 = 94, 94 + 94**2, 94 + 94**2 + 94**3
    r = ids - c3
    L = np.where(ids < c1, 1, np.where(ids < c2, 2, np.where(ids < c3, 3, 4 + r % 8)))
    q = np.where(ids < c1, ids, np.where(ids < c2, ids - c1, np.where(ids < c3, ids - c2, r // 8)))
    del r, ids
    offs = np.cumsum(L + 1).astype(np.uint64)
    starts = offs.astype(np.int64) - (L + 1)
    chars = np.zeros(int(offs[-1]), np.uint8)
    for k in range(11):
        sel = L > k
        chars[(starts + L - 1 - k)[sel]] = 33 + q[sel] % 94
        q //= 94
    del L, q, starts
    v = rng.integers(0, 10**9, n, dtype=np.int64)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        orc.bench_string_agg(chars, offs, v, threads)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round(n / med, 1), "unit": "rows/s", "cores": threads, "kind": "port", "host": host,
            "sample": f"{n} rows x 3 runs (median), 1-11-byte keys over {G} ids, the same StringHashMap "
                      f"restatement as the k%08d leg (oracle/cpu_baseline_str.c)"}


def lz4_leg(args, ctx, pkt):
    """LZ4 packets (CompressionMethod::LZ4, MPPTunnelSetHelper::ToCompressedPacket): compress the
    uncompressed V1 packet into LZ4 frames, then decompress it; rates in packet bytes per second.
    The decompressed bytes are checked against the packet."""
    import torch

    import tiflash_amd as tfa
    for _ in range(2):
        lz = tfa.codec_compress(ctx, pkt)
        back = tfa.codec_decompress(ctx, lz)
    tc, td = [], []
    for _ in range(max(args.steps, 3)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lz = tfa.codec_compress(ctx, pkt)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        back = tfa.codec_decompress(ctx, lz)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        tc.append(t1 - t0)
        td.append(t2 - t1)
    assert torch.equal(back, pkt), "LZ4 round trip"
    c, d = statistics.median(tc), statistics.median(td)
    out = {"packet_bytes": int(pkt.numel()), "lz4_bytes": int(lz.numel()),
           "ratio": round(pkt.numel() / max(lz.numel(), 1), 3), "compress_ms": round(c * 1e3, 3),
           "decompress_ms": round(d * 1e3, 3), "compress_GBps": round(pkt.numel() / c / 1e9, 1),
           "decompress_GBps": round(pkt.numel() / d / 1e9, 1)}
    if not args.no_cpu:  # oracle/lz4.c, one host thread, on a 64 MB prefix of the same packet
        from oracle import oracle as orc
        host = pkt[:64 << 20].cpu().numpy().tobytes()
        t0 = time.perf_counter()
        hz = orc.lz4_packet_compress(host, 65536)
        t1 = time.perf_counter()
        orc.lz4_packet_decompress(hz)
        t2 = time.perf_counter()
        out["cpu_baseline"] = {"compress_GBps": round(len(host) / (t1 - t0) / 1e9, 3),
                               "decompress_GBps": round(len(host) / (t2 - t1) / 1e9, 3), "cores": 1,
                               "kind": "port", "sample": f"{len(host)} bytes of the packet, oracle/lz4.c"}
    del lz, back
    return out


def zstd_leg(args, ctx, pkt):
    """ZSTD packets (CompressionMethod::ZSTD, the HIGH_COMPRESSION mode): a 64 MB slice of the
    uncompressed V1 packet body compressed on the host by the system libzstd (level 1, one frame
    per 1 MB CompressedWriteBuffer block, as the reference's sender writes them), then decompressed
    on the device (zstd.hip: header scan, per-block entropy, resolve, byte-parallel execution);
    checked against the packet.  The device sender (zstd_enc.hip) then compresses the whole
    packet into ZSTD frames, and the device decodes its own frames; both checked.  The host
    compress / decompress of the same 64 MB by libzstd on one thread is reported beside it."""
    import ctypes
    import struct

    import torch

    import tiflash_amd as tfa
    try:
        z = ctypes.CDLL("libzstd.so.1")
    except OSError:
        return {"skipped": "libzstd.so.1 not present"}
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_decompress.restype = ctypes.c_size_t
    # 64 MB from a quarter into the packet: String chars, not the constant StringV2 sizes column
    # that opens the body (which compresses ~245x and would make a misleading sample)
    start = max(1, int(pkt.numel()) // 4)
    body = pkt[start:start + (64 << 20)].cpu().numpy().tobytes()
    frames, fsz = [], 1 << 20
    tz0 = time.perf_counter()
    for i in range(0, len(body), fsz):
        chunk = body[i:i + fsz]
        cap = z.ZSTD_compressBound(ctypes.c_size_t(len(chunk)))
        buf = ctypes.create_string_buffer(cap)
        n = z.ZSTD_compress(buf, ctypes.c_size_t(cap), chunk, ctypes.c_size_t(len(chunk)), 1)
        frames.append(b"\x90" + struct.pack("<II", n + 9, len(chunk)) + buf.raw[:n])
    host_compress = time.perf_counter() - tz0
    zpkt = b"".join(frames)
    dz = torch.frombuffer(bytearray(zpkt), dtype=torch.uint8).to(pkt.device)
    for _ in range(2):
        back = tfa.codec_decompress(ctx, dz)
    td = []
    for _ in range(max(args.steps, 3)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        back = tfa.codec_decompress(ctx, dz)
        torch.cuda.synchronize()
        td.append(time.perf_counter() - t0)
    assert back[1:].cpu().numpy().tobytes() == body, "ZSTD decompress"
    d = statistics.median(td)
    out = {"raw_bytes": len(body), "zstd_bytes": len(zpkt), "frames": len(frames), "ratio": round(len(body) / len(zpkt), 3),
           "decompress_ms": round(d * 1e3, 3), "decompress_GBps": round(len(body) / d / 1e9, 2)}
    del dz, back
    # the device sender over the whole packet, and the device decode of its frames
    for _ in range(2):
        zs = tfa.codec_compress(ctx, pkt, method=tfa.COMPRESSION_ZSTD)
    tc, tu = [], []
    for _ in range(max(args.steps, 3)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        zs = tfa.codec_compress(ctx, pkt, method=tfa.COMPRESSION_ZSTD)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        back = tfa.codec_decompress(ctx, zs)
        torch.cuda.synchronize()
        tc.append(t1 - t0)
        tu.append(time.perf_counter() - t1)
    assert torch.equal(back, pkt), "ZSTD sender round trip"
    c, u = statistics.median(tc), statistics.median(tu)
    out["sender"] = {"packet_bytes": int(pkt.numel()), "zstd_bytes": int(zs.numel()),
                     "ratio": round(pkt.numel() / max(zs.numel(), 1), 3), "compress_ms": round(c * 1e3, 3),
                     "compress_GBps": round(pkt.numel() / c / 1e9, 2), "decompress_ms": round(u * 1e3, 3),
                     "decompress_GBps": round(pkt.numel() / u / 1e9, 2)}
    del zs, back
    if not args.no_cpu:
        out["cpu_compress"] = {"compress_GBps": round(len(body) / host_compress / 1e9, 3), "cores": 1,
                               "kind": "library", "sample": f"{len(body)} bytes, system libzstd ZSTD_compress "
                               "level 1, 1 MB frames, one host thread"}
        dst = ctypes.create_string_buffer(fsz)
        t0 = time.perf_counter()
        for f in frames:
            z.ZSTD_decompress(dst, ctypes.c_size_t(fsz), f[9:], ctypes.c_size_t(len(f) - 9))
        t1 = time.perf_counter()
        out["cpu_baseline"] = {"decompress_GBps": round(len(body) / (t1 - t0) / 1e9, 3), "cores": 1,
                               "kind": "library", "sample": f"the same {len(frames)} frames, system libzstd "
                               "ZSTD_decompress (the reference's codec library), one host thread"}
    return out


def codec_leg(args, ctx, dev):
    """§8 f1: CHBlockChunkCodecV1 (NONE) encode + decode of a C5-shaped block on the device:
    String "k%08d" key (legacy size-prefixed String, the pre-V2 MPP packet form), Decimal(15,2)
    value, Int64 row id.  value = rows / (encode + decode time); packet bytes per second beside it."""
    import numpy as np
    import torch

    import tiflash_amd as tfa
    n = args.codec_rows
    g = torch.Generator(device=dev)
    g.manual_seed(13)
    ids = torch.randint(0, args.c5_groups, (n,), device=dev, generator=g, dtype=torch.int64)
    chars = torch.empty((n, 10), dtype=torch.uint8, device=dev)
    chars[:, 0] = ord("k")
    x = ids.clone()
    for j in range(8, 0, -1):
        chars[:, j] = (48 + x % 10).to(torch.uint8)
        x //= 10
    chars[:, 9] = 0
    chars = chars.reshape(-1)
    offs = torch.arange(1, n + 1, device=dev, dtype=torch.int64) * 10
    v = torch.randint(0, 10**9, (n,), device=dev, generator=g, dtype=torch.int64)
    cols = [("k", "String", chars, offs, None), ("v", "Decimal(15,2)", v, None, None), ("id", "Int64", ids, None, None)]
    res = {}
    for label, tn in (("string", "String"), ("string_v2", "StringV2")):
        cols[0] = ("k", tn, chars, offs, None)
        for _ in range(2):
            pkt = tfa.codec_encode(ctx, cols, n)
            tfa.codec_decode(ctx, pkt)
        te, td = [], []
        for _ in range(max(args.steps, 3)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pkt = tfa.codec_encode(ctx, cols, n)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            rows, dec = tfa.codec_decode(ctx, pkt)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            te.append(t1 - t0)
            td.append(t2 - t1)
        assert rows == n and torch.equal(dec[0]["offsets"], offs) and torch.equal(dec[2]["data"], ids)
        e, d = statistics.median(te), statistics.median(td)
        res[label] = {"encode_ms": round(e * 1e3, 3), "decode_ms": round(d * 1e3, 3),
                      "packet_bytes": int(pkt.numel()), "rows_per_s": round(n / (e + d), 1),
                      "packet_GBps": round(2 * pkt.numel() / (e + d) / 1e9, 1)}
        if label == "string_v2":
            res["lz4"] = lz4_leg(args, ctx, pkt)
            res["zstd"] = zstd_leg(args, ctx, pkt)
        del pkt, dec
    out = {"metric": "rows/s CHBlockChunkCodecV1 encode + decode (String k%08d, Decimal(15,2), Int64)",
           "value": res["string"]["rows_per_s"], "unit": "rows/s", "rows": n, "legs": res}
    if not args.no_cpu:  # oracle/codec.c: the reference's serialisation restated, one host thread
        from oracle import oracle as orc
        m = min(n, 5_000_000)
        hc = [("k", "String", chars[:m * 10].cpu().numpy(), offs[:m].cpu().numpy().astype(np.uint64), None),
              ("v", "Decimal(15,2)", v[:m].cpu().numpy(), None, None), ("id", "Int64", ids[:m].cpu().numpy(), None, None)]
        t0 = time.perf_counter()
        pk = orc.codec_encode(hc, m)
        t1 = time.perf_counter()
        hdr = len(pk) - (m * 10 + 16 * m)  # fixed part of the packet before the String rows
        orc.codec_decode_strings(pk[hdr:], m, m * 10)
        t2 = time.perf_counter()
        out["cpu_baseline"] = {"value": round(m / (t2 - t0), 1), "unit": "rows/s", "cores": 1, "kind": "port",
                               "sample": f"{m} rows: oracle/codec.c encode of the 3 columns + legacy String decode "
                                         f"(deserializeBinarySSE2 restated), one host thread"}
    del chars, offs, v, ids
    return out


def timed(step, args, ctx, world):
    """W warmup steps, then exactly K timed steps bracketed by barrier + synchronize; returns
    (elapsed seconds of this rank, last result, {kernel phase: (ms, launches)})."""
    import torch
    import torch.distributed as dist
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    return el, res, prof


def variants_leg(args, ctx, dev, f, k, v):
    """SURVEY 8(d) extras of C2 at N=1: the selectivity sweep f < t for t in 0/1/10/50/100 %
    (bench_column_filter.cpp:251-290) and the Int64 value column, each a separate timed run."""
    import torch

    import tiflash_amd as tfa
    out = {}
    N, G = args.rows, args.groups
    sweep = {}
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)],
                         bucket_bits=args.bucket_bits, expected_groups=G)
    for t in (0, 1, 10, 50, 100):
        def step():
            agg.reset()
            agg.consume_filtered(f, tfa.LT, t, k, [v, None])
            return agg.result(capacity_hint=G)
        el, res, prof = timed(step, args, ctx, 1)
        ms = el / args.steps * 1e3
        kept = int((f < t).sum().item())
        cnt = int(res["states"][1].view(torch.int64).sum().item()) if res["keys"] is not None else 0
        sweep[f"{t}%"] = {"value": round(N * args.steps / el, 1), "ms_per_step": round(ms, 3), "kept_rows": kept,
                          "check_ok": cnt == kept, "pipeline_frac": round(24 * N / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "kernels_ms_per_step": {kn: round(vv[0] / args.steps, 4) for kn, vv in sorted(prof.items())}}
    agg.close()
    out["selectivity_sweep"] = sweep
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    vi = torch.randint(0, 1 << 20, (N,), device=dev, generator=gen, dtype=torch.int64)
    agg = tfa.Aggregator(ctx, tfa.INT64, [(tfa.AGG_SUM, tfa.INT64), (tfa.AGG_COUNT_ALL, 0)],
                         bucket_bits=args.bucket_bits, expected_groups=G)

    def istep():
        agg.reset()
        agg.consume_filtered(f, tfa.LT, args.threshold, k, [vi, None])
        return agg.result(capacity_hint=G)
    el, res, _ = timed(istep, args, ctx, 1)
    ms = el / args.steps * 1e3
    kept = int((f < args.threshold).sum().item())
    exact = int(vi[f < args.threshold].sum().item()) == int(res["states"][0].sum().item())
    out["int64_value"] = {"metric": "rows/s filter + GROUP BY, sum(Int64) + count (exact)",
                          "value": round(N * args.steps / el, 1), "ms_per_step": round(ms, 3),
                          "check_ok": exact and int(res["states"][1].sum().item()) == kept,
                          "pipeline_frac": round(24 * N / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    agg.close()
    del vi
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    import tiflash_amd as tfa
    from tiflash_amd.exchange import exchange_partitions

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    if args.scaling == "strong" and world > 1:  # job totals -> per-rank shares
        args.rows //= world
        args.join_build //= world
        args.join_probe //= world
        args.c5_rows //= world
    N, G = args.rows, args.groups
    gen = torch.Generator(device=dev)
    gen.manual_seed(1 + rank)
    f = torch.randint(0, 100, (N,), device=dev, generator=gen, dtype=torch.int64)
    k = torch.randint(0, G, (N,), device=dev, generator=gen, dtype=torch.int64)
    if args.value_int64:
        v = torch.randint(0, 1 << 20, (N,), device=dev, generator=gen, dtype=torch.int64)
        vtype = tfa.INT64
    else:  # dyadic m * 2^-8, m < 2^20: partial sums exact, so any summation order is bit-exact
        v = torch.randint(0, 1 << 20, (N,), device=dev, generator=gen, dtype=torch.int64).double() / 256.0
        vtype = tfa.FLOAT64
    n_kept = int((f < args.threshold).sum().item())

    ctx = tfa.Context(local)
    aggs = [(tfa.AGG_SUM, vtype), (tfa.AGG_COUNT_ALL, 0)]
    agg = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=args.bucket_bits, expected_groups=G)
    final = tfa.Aggregator(ctx, tfa.INT64, aggs, bucket_bits=args.bucket_bits, expected_groups=G) if world > 1 else None

    def step():
        agg.reset()
        agg.consume_filtered(f, tfa.LT, args.threshold, k, [v, None])
        # final Block of this rank (or its partial states); the key domain [0, G) bounds the group
        # count, so the result buffers go over before the count is read (no mid-step round trip)
        res = agg.result(capacity_hint=G)
        if world == 1:
            return res
        # ExchangeSender: hash-repartition partial rows by key, RCCL all-to-all, final merge
        cols, offs = tfa.hash_partition(ctx, [res["keys"], res["states"][0], res["states"][1]], [0], world)
        outs = exchange_partitions(cols, offs)
        final.reset()
        final.consume_partial(outs[0], [outs[1], outs[2]])
        return final.result()

    el, res, prof = timed(step, args, ctx, world)
    # invariant of the last step's result: every kept row is counted exactly once over all ranks
    red_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    inv = torch.tensor([float(res["states"][1].view(torch.int64).sum().item()), float(n_kept),
                        float(res["keys"].shape[0])], dtype=torch.float64, device=red_dev)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
        dist.all_reduce(inv)
    count_total, kept_total, groups_total = (int(x) for x in inv.tolist())
    groups = agg.size() if world == 1 else final.size()
    ms = el / args.steps * 1e3
    value = N * world * args.steps / el

    line = {
        "metric": "rows/sec on filter->hash-agg (TPC-H Q1 shape: 100M rows, 1M-key GROUP BY)",
        "value": round(value, 1), "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
        "dtype": "int64/f64" if vtype == tfa.FLOAT64 else "int64",
        "data": "synthetic: f~U[0,100) (pred f<96), k~U[0,1e6), v dyadic f64; seed 1+rank",
        "config": {"workload": "configs[1] filter + GROUP BY 1M keys" + (" two-phase + RCCL all-to-all" if world > 1 else ""),
                   "rows_per_gpu": N, "total_rows": N * world, "groups": G, "kept_rows_per_gpu": n_kept,
                   "groups_out": groups,
                   "parallelism": f"dp{world}", "dist_backend": args.dist_backend if world > 1 else None},
        "check": {"count_total": count_total, "kept_total": kept_total, "groups_total": groups_total,
                  "ok": count_total == kept_total and groups_total <= G},
    }
    if rank == 0:
        rf = roofline_from_profile(prof, args.steps, N, n_kept, agg.size())
        if rf and "bound" in rf:
            rf["traffic"] = load_pmc_traffic(rf["kernel"])
            if rf["traffic"]:
                rf["traffic_over_algorithmic"] = round(rf["traffic"] / rf["algorithmic_bytes_per_launch"], 3)
                rf["traffic_source"] = pmc_source()
        line["roofline"] = rf
        line["pipeline_roofline"] = {"algorithmic_bytes_per_step": 24 * N, "achieved": round(24 * N / (ms * 1e-3) / 1e9, 1),
                                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(24 * N / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "traffic": load_pmc_step("C2")}
        if line["pipeline_roofline"]["traffic"]:
            line["pipeline_roofline"]["traffic_over_algorithmic"] = round(
                line["pipeline_roofline"]["traffic"] / (24 * N), 3)
            line["pipeline_roofline"]["traffic_source"] = pmc_source()
        line["kernels_ms_per_step"] = {kname: round(v[0] / args.steps, 4) for kname, v in sorted(prof.items())}

    if world == 1 and not args.no_variants:
        line["c2_variants"] = variants_leg(args, ctx, dev, f, k, v)

    # ---- hash join probe (configs[2] shape) at N=1
    if world == 1 and not args.no_join:
        nb, npr = args.join_build, args.join_probe
        g2 = torch.Generator(device=dev)
        g2.manual_seed(7)
        bk = torch.randperm(nb, device=dev, generator=g2).to(torch.int64) * 4 + 1
        bpay = torch.randint(0, 1 << 40, (nb,), device=dev, generator=g2, dtype=torch.int64)
        hit = torch.rand(npr, device=dev, generator=g2) < 0.5
        pk = torch.where(hit, bk[torch.randint(0, nb, (npr,), device=dev, generator=g2)],
                         torch.randint(0, 1 << 40, (npr,), device=dev, generator=g2) * 4 + 3)
        ppay = torch.randint(0, 1 << 40, (npr,), device=dev, generator=g2, dtype=torch.int64)
        del hit
        j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb)
        tb0 = time.perf_counter()
        j.build(bk, payload=[bpay])
        j.finalize()
        torch.cuda.synchronize()
        build_s = time.perf_counter() - tb0
        outs = ([torch.empty(npr, dtype=torch.int64, device=dev) for _ in range(2)],
                [torch.empty(npr, dtype=torch.int64, device=dev)], torch.empty(npr, dtype=torch.uint8, device=dev))

        def jstep():
            # the joined block (probe key, probe payload, build payload), materialised by the probe
            op, ob, _ = j.probe_rows(pk, [pk, ppay], 1, capacity=npr, outs=outs)
            return op + ob

        for _ in range(args.warmup):
            jstep()
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            outj = jstep()
        torch.cuda.synchronize()
        jel = time.perf_counter() - t0
        jprof = ctx.profile_read()
        ctx.profile(False)
        matches = outj[0].shape[0]
        jms = jel / args.steps * 1e3
        alg = 16 * npr + 24 * matches
        line["join_probe"] = {
            "metric": "probe rows/s (hash join 10M build x 100M probe, Int64 keys, ~50% hit, materialised)",
            "value": round(npr / (jel / args.steps), 1), "unit": "rows/s", "ms_per_step": round(jms, 3),
            "build_s": round(build_s, 4), "matches": matches,
            "pipeline_roofline": {"algorithmic_bytes_per_step": alg, "achieved": round(alg / (jms * 1e-3) / 1e9, 1),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(alg / (jms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "kernels_ms_per_step": {kname: round(vv[0] / args.steps, 4) for kname, vv in sorted(jprof.items())},
        }
        # the same probe through JoinV2's tagged pointer table (no probe-side partitioning): a parity
        # path, not a timed leg by default (latency-bound random walks, 8x v1)
        del j
    if world == 1 and not args.no_join and args.join_v2:
        j = tfa.Join(ctx, tfa.INT64, expected_build_rows=nb, v2=True, tagged=True)
        tb0 = time.perf_counter()
        j.build(bk, payload=[bpay])
        j.finalize()
        torch.cuda.synchronize()
        build2_s = time.perf_counter() - tb0
        for _ in range(args.warmup):
            jstep()
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            outj = jstep()
        torch.cuda.synchronize()
        jel2 = time.perf_counter() - t0
        jprof2 = ctx.profile_read()
        ctx.profile(False)
        jms2 = jel2 / args.steps * 1e3
        line["join_probe"]["join_v2"] = {
            "metric": "probe rows/s through the JoinV2 tagged pointer table", "value": round(npr / (jel2 / args.steps), 1),
            "ms_per_step": round(jms2, 3), "build_s": round(build2_s, 4), "matches": outj[0].shape[0],
            "check_ok": outj[0].shape[0] == matches,
            "pipeline_frac": round(alg / (jms2 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "kernels_ms_per_step": {kname: round(vv[0] / args.steps, 4) for kname, vv in sorted(jprof2.items())},
        }

    if args.c4 == 1 or (args.c4 == -1 and world > 1):
        c4 = c4_leg(args, ctx, dev, world, rank)
        if rank == 0:
            line["repartitioned_join"] = c4
    if world == 1 and args.codec_rows > 0:
        line["packet_codec"] = codec_leg(args, ctx, dev)
    if args.c5_rows > 0:
        c5 = c5_leg(args, ctx, dev, world, rank)
        if rank == 0:
            line["string_agg"] = c5

    if rank == 0 and world == 1 and not args.no_cpu:
        if "string_agg" in line:
            line["string_agg"]["cpu_baseline"] = cpu_string_baseline(args)
        cb = cpu_baseline(args)
        line["cpu_baseline"] = cb
        line["gpu_vs_cpu"] = round(value / cb["value"], 1)
        if "join_probe" in line:
            jb = cpu_join_baseline(args)
            line["join_probe"]["cpu_baseline"] = jb
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    for o in (agg, final):
        if o is not None:
            o.close()
    ctx.close()


if __name__ == "__main__":
    main()
