#!/bin/bash
# rocprofv3 evidence for bench.py, one tagged run (on the GPU box, from the repo root):
#   1. kernel trace + stats of the bench legs (C2 filter -> GROUP BY,
#      C3 join, packet codec, C5 String GROUP BY; CPU baselines skipped);
#   2. two PMC passes over the same legs (variants off), FETCH_SIZE and WRITE_SIZE each in a run
#      of its own, never combined with sys / runtime tracing.
# Every command is recorded verbatim in $OUT/commands.txt; tools/summarize_profile.py <tag>
# turns the directory into profiles/<tag>_summary.md, profiles/<tag>_kernel_stats.csv and
# profiles/pmc_traffic.json.
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_${TAG}
export TMPDIR=/tmp
mkdir -p "$OUT"
: > "$OUT/commands.txt"
run() { # run <name> <timeout> <cmd...>: records the command, runs it with its log in $OUT/<name>_bench.log
    local name=$1 limit=$2
    shift 2
    echo "$name: $*" >> "$OUT/commands.txt"
    timeout -k 10 "$limit" "$@" > "$OUT/${name}_bench.log" 2>&1
}
run kt 420 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -f csv -- python3 bench.py --no-cpu --no-variants --steps 5 --warmup 2
run fetch 420 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run -f csv -- python3 bench.py --no-cpu --no-variants --steps 2 --warmup 1
run write 420 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run -f csv -- python3 bench.py --no-cpu --no-variants --steps 2 --warmup 1
echo PROFILE_DONE
