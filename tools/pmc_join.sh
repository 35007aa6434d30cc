#!/bin/bash
# SQ counters of the join kernels on a short bench run (join leg only matters).
set -euo pipefail
TAG=${1:-join}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "join_probe|part_scatter|part_hist" \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
  -d "$OUT" -o run -f csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 --rows 1000000 > "$OUT/bench.log" 2>&1
echo PMC_DONE
