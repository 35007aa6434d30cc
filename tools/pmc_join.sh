#!/bin/bash
# PMC passes over the join kernels on a short bench run (join leg only; C2 shrunk, C5 / codec off).
# usage: tools/pmc_join.sh <tag>
set -euo pipefail
TAG=${1:-join}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
RE="join_probe|SelJoin|regroup_scatter"
ARGS="--no-cpu --steps 2 --warmup 1 --rows 1000000 --c5-rows 0 --codec-rows 0 --no-variants"
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES \
  -d "$OUT/a" -o run -f csv -- python3 bench.py $ARGS > "$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$RE" \
  --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  -d "$OUT/b" -o run -f csv -- python3 bench.py $ARGS > "$OUT/b.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --pmc FETCH_SIZE \
  -d "$OUT/f" -o run -f csv -- python3 bench.py $ARGS > "$OUT/f.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --pmc WRITE_SIZE \
  -d "$OUT/w" -o run -f csv -- python3 bench.py $ARGS > "$OUT/w.log" 2>&1
echo PMC_DONE
