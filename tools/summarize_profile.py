#!/usr/bin/env python3
"""Turn one tools/profile.sh run (gpurun_out/prof_<tag>/) into the committed evidence under profiles/.

Outputs
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the traced bench run
  profiles/<tag>_summary.md         the commands that ran, per-kernel durations, PMC bytes per launch
                                    and per bench step for each leg (C2, C3, C5, codec)
  profiles/pmc_traffic.json         HBM bytes per launch per kernel (bench.py's roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE come from separate --pmc passes
and are reported in KB.  FETCH_SIZE reports half the bytes of wide coalesced streaming reads on
gfx950, so it is doubled; the factor is re-measured on agg.part.tiled, whose reads are the 24 B
input rows plus nothing else (reported next to the guide's factor).  WRITE_SIZE is used as is.
Dispatches are assigned to a bench leg by the most recent leg-specific kernel before them (legs
run one after another), so shared kernels (scan, compact, result, gather) land in their leg.
"""
import argparse
import collections
import csv
import json
import os
import re
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# demangled name -> short name (first match wins)
NAME_MAP = [
    (r"part_hist_kernel<tfg::SelBucket", "agg.part.hist"),
    (r"part_scatter_staged_kernel<tfg::SelBucket.*true, true(, (true|false))?>", "agg.part.tiled"),
    (r"part_scatter.*<tfg::SelBucket", "agg.part.scatter"),
    (r"agg_bucket_tiled_kernel<tfg::WideFastOps", "agg.wide.bucket.tiled"),
    (r"agg_bucket_tiled_kernel<tfg::FastOps", "agg.bucket.tiled"),
    (r"agg_bucket_tiled_kernel", "agg.bucket.tiled.other"),
    (r"part_hist_kernel<tfg::SelWide", "agg.wide.part.hist"),
    (r"part_scatter.*<tfg::SelWide", "agg.wide.part.scatter"),
    (r"agg_bucket_kernel<tfg::WideOps", "agg.wide.bucket"),
    (r"agg_bucket_kernel", "agg.bucket"),
    (r"pack_keys_kernel", "agg.pack_keys"),
    (r"unpack_keys_kernel", "agg.unpack_keys"),
    (r"agg_compact_kernel", "agg.compact"),
    (r"agg_result_kernel", "agg.result"),
    (r"part_hist_kernel<tfg::SelRec8", "part.hist.pass2"),
    (r"part_scatter_staged_kernel<tfg::SelRec8", "part.scatter.pass2"),
    (r"part_scatter_staged_kernel<tfg::SelJoin.*true, true(, (true|false))?>", "join.part.tiled"),
    (r"regroup_scatter_kernel", "join.part.regroup"),
    (r"part_hist_kernel<tfg::SelJoin", "join.part.hist"),
    (r"part_scatter.*<tfg::SelJoin", "join.part.scatter"),
    (r"join_probe_kernel", "join.probe"),
    (r"join_build", "join.build"),
    (r"zstd_scan_kernel", "codec.zstd.scan"),
    (r"zstd_block_kernel", "codec.zstd.block"),
    (r"zstd_resolve_kernel", "codec.zstd.resolve"),
    (r"zstd_expand_kernel", "codec.zstd.expand"),
    (r"zstd_jump_kernel", "codec.zstd.jump"),
    (r"zstd_gather_kernel", "codec.zstd.gather"),
    (r"zstd_check_kernel", "codec.zstd.check"),
    (r"gather_kernel", "gather"),
    (r"scan_", "scan"),
]
# leg-specific kernels (by short name or raw-name regex)
LEGS = [
    ("C3v2", r"join_v2_"),
    ("C2", r"^(agg\.part\.(hist|tiled|scatter)|agg\.bucket\.tiled)$"),
    ("C3", r"^(join\.|part\.(hist|scatter)\.pass2)"),
    ("codec", r"tfg::str_|codec|lz4_|zstd_"),
    ("C5", r"^(agg\.wide\.|agg\.(pack|unpack)_keys|agg\.bucket$)|wide_str|regroup_"),
]


def short(name):
    for pat, s in NAME_MAP:
        if re.search(pat, name):
            return s
    m = re.search(r"tfg::(?:\(anonymous namespace\)::)?(\w+)", name)
    return ("tfg::" + m.group(1)) if m else name.split("(")[0][:60]


# the kernel that ends one bench step of a leg: a leg's steady-state step is the window of its
# dispatches after one step-end kernel up to and including the next (the first window also holds
# one-off work such as the join build, so it is not used when a later window exists)
STEP_END = {"C2": r"^agg\.result$", "C5": r"^agg\.result$", "C3": r"^join\.probe$",
            "C3v2": r"join_v2_probe_kernel"}


def step_windows(ds):
    """{leg: [bytes of each complete step window, in order]} from one counter's dispatch list."""
    acc, wins = collections.defaultdict(float), collections.defaultdict(list)
    for _, s, leg, v in ds:
        acc[leg] += v
        pat = STEP_END.get(leg)
        if pat and re.search(pat, s):
            wins[leg].append(acc[leg])
            acc[leg] = 0.0
    return wins


def leg_of(short_name, raw):
    for leg, pat in LEGS:
        if re.search(pat, short_name) or re.search(pat, raw):
            return leg
    return None


def dispatches(path, counter=None):
    """[(dispatch_id, short name, leg-marker or None, value)] in dispatch order; tfg kernels only."""
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if "tfg::" not in name:
                continue
            if counter and r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            val = float(r["Counter_Value"]) if counter else 0.0
            s = short(name)
            if d in rows:
                rows[d][3] += val  # per-XCD / instance rows of one dispatch
            else:
                rows[d] = [d, s, leg_of(s, name), val]
    out, leg = [], None
    for d in sorted(rows):
        _, s, marker, val = rows[d]
        leg = marker or leg
        out.append((d, s, leg or "C2", val))
    return out


def commands(src):
    p = os.path.join(src, "commands.txt")
    return open(p).read().strip().splitlines() if os.path.exists(p) else []


def bench_line(src, log):
    p = os.path.join(src, log)
    if os.path.exists(p):
        for line in open(p):
            if line.startswith("{"):
                return json.loads(line)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--commit", default=None, help="commit the profiled tree was at (default: HEAD)")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    out = os.path.join(ROOT, "profiles")
    stats = os.path.join(src, "kt", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{a.tag}_kernel_stats.csv"))
    cmds = commands(src)
    kt_line = bench_line(src, "kt_bench.log")
    pmc_line = bench_line(src, "fetch_bench.log") or kt_line
    cfg = pmc_line["config"]
    rows, kept, groups = cfg["rows_per_gpu"], cfg["kept_rows_per_gpu"], cfg["groups"]
    runs = pmc_line["steps"] + pmc_line["warmup"]
    fetch = dispatches(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = dispatches(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    factor = 2.0  # MI355X_MICROARCH.md: FETCH_SIZE = 1/2 of the bytes of wide streaming reads

    def per_kernel(ds):  # (leg, short) -> (launches, total KB)
        acc = collections.defaultdict(lambda: [0, 0.0])
        for _, s, leg, v in ds:
            acc[(leg, s)][0] += 1
            acc[(leg, s)][1] += v
        return acc

    fk, wk = per_kernel(fetch), per_kernel(write)
    t2 = fk.get(("C2", "agg.part.tiled"))
    measured = (24 * rows) / (t2[1] * 1024 / t2[0]) if t2 else None
    # algorithmic bytes per launch where a kernel carries a leg's whole input
    alg = {("C2", "agg.part.tiled"): 24 * rows,
           ("C2", "agg.part.hist"): 16 * rows}
    commit = a.commit
    try:
        commit = commit or subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None
    except OSError:
        commit = None
    traffic = {"_calibration": {"tag": a.tag, "commit": commit, "fetch_factor": factor, "basis": "MI355X_MICROARCH.md HBM section (x2 on gfx950)",
                                "measured_on_agg_part_tiled": round(measured, 4) if measured else None,
                                "rows": rows, "kept": kept, "groups": groups, "pmc_runs_per_leg": runs,
                                "commands": cmds}}
    legs = collections.defaultdict(float)
    for key in sorted(set(fk) | set(wk)):
        leg, s = key
        fn, fkb = fk.get(key, [0, 0.0])
        wn, wkb = wk.get(key, [0, 0.0])
        fb = fkb * 1024 / max(fn, 1) * factor
        wb = wkb * 1024 / max(wn, 1)
        name = s if leg == "C2" else f"{leg}:{s}"
        traffic[name] = {"launches": max(fn, wn), "fetch_bytes_raw": int(fkb * 1024 / max(fn, 1)),
                         "fetch_bytes": int(fb), "write_bytes": int(wb), "hbm_bytes_per_launch": int(fb + wb),
                         "algorithmic_bytes": alg.get(key)}
        legs[leg] += (fkb * 1024 * factor + wkb * 1024) / runs
    leg_alg = {"C2": 24 * rows + 24 * groups}
    jl = (kt_line or {}).get("join_probe")
    if jl:
        leg_alg["C3"] = jl["pipeline_roofline"]["algorithmic_bytes_per_step"]
    sl = (kt_line or {}).get("string_agg")
    if sl:
        leg_alg["C5"] = sl["pipeline_roofline"]["algorithmic_bytes_per_step"]
    if jl and jl.get("join_v2"):
        leg_alg["C3v2"] = leg_alg["C3"]
    fw, ww = step_windows(fetch), step_windows(write)
    per_step = {}
    for leg, b in legs.items():
        e = {"hbm_bytes_avg_over_runs": int(b)}
        if fw.get(leg) and ww.get(leg):
            # steady state: the last complete step window of each counter pass
            b = fw[leg][-1] * 1024 * factor + ww[leg][-1] * 1024
            e.update({"fetch_bytes": int(fw[leg][-1] * 1024 * factor), "write_bytes": int(ww[leg][-1] * 1024),
                      "basis": "last complete step window (dispatches after one step-end kernel up to the next)"})
        else:
            e["basis"] = "all dispatches of the leg / runs (build included once)"
        e.update({"hbm_bytes": int(b), "algorithmic_bytes": leg_alg.get(leg),
                  "traffic_over_algorithmic": round(b / leg_alg[leg], 3) if leg_alg.get(leg) else None})
        per_step[leg] = e
    traffic["_per_step"] = per_step
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    # ---- summary
    srows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            srows.append((short(r["Name"]), r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e6,
                          float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
    with open(os.path.join(out, f"{a.tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary ({a.tag})\n\nCommands that ran (tools/profile.sh {a.tag}, verbatim):\n\n")
        for c in cmds:
            f.write(f"    {c}\n")
        for nm, line in (("traced", kt_line), ("PMC (FETCH_SIZE pass)", pmc_line)):
            if line:
                f.write(f"\nBench line of the {nm} run: {line['value']:.4g} {line['unit']}, {line['ms_per_step']} ms/step")
                if line.get("join_probe"):
                    f.write(f"; join {line['join_probe']['value']:.4g} probe rows/s")
                if line.get("string_agg"):
                    f.write(f"; C5 {line['string_agg']['value']:.4g} rows/s")
                f.write(".\n")
        f.write("\n## Kernel trace (top 24 by total time; tfg:: kernels are this library's)\n\n")
        f.write("| kernel | calls | avg ms | total ms | % |\n|---|---|---|---|---|\n")
        for s, raw, calls, avg, tot, pct in sorted(srows, key=lambda x: -x[4])[:24]:
            label = s if "tfg::" in raw else "(torch) " + s[:40]
            f.write(f"| {label} | {calls} | {avg:.4f} | {tot:.3f} | {pct:.1f} |\n")
        f.write(f"\n## HBM traffic (PMC)\n\nFETCH_SIZE factor {factor} (guide); re-measured on agg.part.tiled "
                f"(24 B/row input only): {round(measured, 3) if measured else None}.\n\n")
        f.write("| leg:kernel | launches | fetch B/launch (x2) | write B/launch | HBM B/launch | algorithmic B |\n"
                "|---|---|---|---|---|---|\n")
        for k, v in sorted(traffic.items()):
            if k.startswith("_"):
                continue
            f.write(f"| {k} | {v['launches']} | {v['fetch_bytes']:.4g} | {v['write_bytes']:.4g} | "
                    f"{v['hbm_bytes_per_launch']:.4g} | {v['algorithmic_bytes'] or '-'} |\n")
        f.write(f"\nPer bench step (the last complete step window of each leg; C3 = partitioned v1 join, "
                f"C3v2 = JoinV2 pointer table):\n\n"
                "| leg | HBM bytes / step | algorithmic bytes / step | ratio |\n|---|---|---|---|\n")
        for leg, v in sorted(traffic["_per_step"].items()):
            f.write(f"| {leg} | {v['hbm_bytes']:.4g} | {v['algorithmic_bytes'] or '-'} | {v['traffic_over_algorithmic']} |\n")
    print(json.dumps(traffic["_per_step"], indent=1))


if __name__ == "__main__":
    main()
