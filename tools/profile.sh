#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench command (per-kernel average durations);
#   2. separate PMC passes for HBM traffic (FETCH_SIZE, WRITE_SIZE; one counter group per pass,
#      never combined with sys/runtime tracing), on the filter -> GROUP BY step only.
# Results land in gpurun_out/prof_<tag>/; tools/summarize_profile.py turns them into profiles/.
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run -f csv -- python3 bench.py --no-cpu --c5-rows 0 --c4 0 --codec-rows 0 --steps 5 --warmup 2 > "$OUT/kt_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run -f csv -- python3 bench.py --no-cpu --no-join --c5-rows 0 --c4 0 --codec-rows 0 --steps 2 --warmup 1 > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run -f csv -- python3 bench.py --no-cpu --no-join --c5-rows 0 --c4 0 --codec-rows 0 --steps 2 --warmup 1 > "$OUT/write_bench.log" 2>&1
echo PROFILE_DONE
