#!/bin/bash
# Timing sweep of the C2 step under environment knobs (run on the GPU box from the repo root):
#   bash tools/sweep.sh name1 "ENV=1 ENV2=2" name2 "ENV=3" ...
# Each run: bench.py --no-cpu --no-join --c5-rows 0, value + per-kernel ms printed per line.
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  name=$1; envs=$2; shift 2
  env $envs timeout -k 10 120 python -u bench.py --no-cpu --no-join --c5-rows 0 --steps 5 --warmup 2 \
      > gpurun_out/sw_$name.log 2>&1 || exit 1
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/sw_$name.log | head -1) $(grep -o 'kernels_ms_per_step[^}]*}' gpurun_out/sw_$name.log)"
done
