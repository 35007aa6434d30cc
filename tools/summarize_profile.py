#!/usr/bin/env python3
"""Turn a tools/profile.sh run (gpurun_out/prof_<tag>/) into the committed evidence under profiles/.

Outputs
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the default bench command
  profiles/<tag>_summary.md         per-kernel average duration + PMC bytes per launch, human-readable
  profiles/pmc_traffic.json         HBM bytes per launch per pipeline kernel (bench.py's roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE come from separate --pmc passes.
FETCH_SIZE reports exactly half the bytes of wide coalesced streaming reads on gfx950 (the guide's
HBM/rocprofv3 section), so it is doubled.  The factor was cross-checked on a kernel with a known
byte count (agg.part.hist, 16 B per input row: measured 2.000, r01); when that kernel is in the
run it is re-measured and reported next to the guide's factor.  WRITE_SIZE is used as reported
(exact for 16-B/lane streaming stores, the record stores of the partition).
"""
import argparse
import collections
import csv
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# demangled kernel name -> pipeline scope name used by bench.py / the library profiler
NAME_MAP = [
    (r"part_hist_kernel<tfg::SelWide", "agg.wide.part.hist"),
    (r"part_scatter.*<tfg::SelWide", "agg.wide.part.scatter"),
    (r"agg_bucket_kernel<tfg::WideOps", "agg.wide.bucket"),
    (r"pack_keys_kernel", "agg.pack_keys"),
    (r"part_hist_kernel<tfg::SelBucket", "agg.part.hist"),
    (r"part_scatter_staged_kernel<tfg::SelBucket.*true, true>", "agg.part.tiled"),
    (r"part_scatter_staged_kernel<tfg::SelBucket", "agg.part.scatter"),
    (r"part_scatter_kernel<tfg::SelBucket", "agg.part.scatter"),
    (r"agg_bucket_kernel", "agg.bucket"),
    (r"agg_bucket_tiled_kernel", "agg.bucket"),
    (r"agg_compact_kernel", "agg.compact"),
    (r"agg_result_kernel", "agg.result"),
    (r"scan_", "scan"),
    (r"part_hist_kernel<tfg::SelRec8", "part.hist.pass2"),
    (r"part_scatter_staged_kernel<tfg::SelRec8", "part.scatter.pass2"),
    (r"part_hist_kernel<tfg::SelJoin", "join.part.hist"),
    (r"part_scatter.*<tfg::SelJoin", "join.part.scatter"),
    (r"join_probe_kernel", "join.probe"),
    (r"gather_kernel", "gather"),
]


def short(name):
    for pat, s in NAME_MAP:
        if re.search(pat, name):
            return s
    return name.split("(")[0][:60]


def per_launch(path, counter):
    """avg counter value per dispatch, per short kernel name (sums over XCD/instance rows)."""
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = short(r["Kernel_Name"])
            tot[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: tot[k] / max(len(disp[k]), 1) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--kept", type=int, default=0, help="kept rows (from the bench log if 0)")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "kt", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    kept = a.kept
    bench_line = None
    for log in ("kt_bench.log", "fetch_bench.log"):
        p = os.path.join(src, log)
        if os.path.exists(p):
            for line in open(p):
                if line.startswith("{"):
                    bench_line = bench_line or json.loads(line)
    if not kept and bench_line:
        kept = bench_line["config"]["kept_rows_per_gpu"]
    fetch = per_launch(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_launch(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    # FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters)
    fetch = {k: v * 1024 for k, v in fetch.items()}
    write = {k: v * 1024 for k, v in write.items()}
    factor = 2.0  # MI355X_MICROARCH.md: FETCH_SIZE = 1/2 of the bytes of wide streaming reads
    measured = 16 * a.rows / fetch["agg.part.hist"] if fetch.get("agg.part.hist") else None
    alg = {"agg.part.hist": 16 * a.rows, "agg.part.scatter": 24 * a.rows + 16 * kept,
           "agg.part.tiled": 24 * a.rows + 16 * kept, "agg.bucket": 16 * kept}
    traffic = {"_calibration": {"fetch_factor": factor, "basis": "MI355X_MICROARCH.md HBM section (x2 on gfx950)",
                                "measured_on_agg_part_hist": round(measured, 4) if measured else None,
                                "rows": a.rows, "kept": kept}}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * factor
        wb = write.get(k, 0.0)
        traffic[k] = {"fetch_bytes_raw": int(fetch.get(k, 0.0)), "fetch_bytes": int(fb), "write_bytes": int(wb),
                      "hbm_bytes_per_launch": int(fb + wb), "algorithmic_bytes": alg.get(k)}
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    # duration table
    rows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            rows.append((short(r["Name"]), int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6,
                         float(r["Percentage"])))
    with open(os.path.join(out, f"{a.tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary ({a.tag})\n\n")
        f.write("Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --steps 5 --warmup 2` "
                "(tools/profile.sh); PMC from separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes "
                "over `bench.py --no-cpu --no-join --steps 2 --warmup 1`.\n\n")
        if bench_line:
            f.write(f"Bench line of the traced run: value {bench_line['value']:.4g} {bench_line['unit']}, "
                    f"{bench_line['ms_per_step']} ms/step.\n\n")
        f.write("| kernel | calls | avg ms | total ms | % |\n|---|---|---|---|---|\n")
        for name, calls, avg, tot, pct in sorted(rows, key=lambda x: -x[3])[:20]:
            f.write(f"| {name} | {calls} | {avg:.4f} | {tot:.3f} | {pct:.1f} |\n")
        f.write(f"\nFETCH_SIZE factor {factor} (guide); re-measured on agg.part.hist: {measured}\n\n")
        f.write("| kernel | fetch B/launch (corrected) | write B/launch | HBM B/launch | algorithmic B |\n|---|---|---|---|---|\n")
        for k, v in sorted(traffic.items()):
            if k.startswith("_"):
                continue
            f.write(f"| {k} | {v['fetch_bytes']:.4g} | {v['write_bytes']:.4g} | {v['hbm_bytes_per_launch']:.4g} | "
                    f"{v['algorithmic_bytes'] if v['algorithmic_bytes'] else '-'} |\n")
    print(json.dumps({k: v for k, v in traffic.items() if k in alg or k.startswith("_")}, indent=1))


if __name__ == "__main__":
    main()
