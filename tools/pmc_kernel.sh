#!/bin/bash
# One PMC pass (SQ counters) over the kernels matching $1, on a short bench run.
# usage: tools/pmc_kernel.sh <kernel-regex> <tag> [bench args...]
set -euo pipefail
RE=$1; TAG=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
timeout -s KILL 150 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
  -d "$OUT" -o run -f csv -- python3 bench.py --no-cpu --no-join --steps 2 --warmup 1 "$@" > "$OUT/bench.log" 2>&1
echo PMC_DONE
