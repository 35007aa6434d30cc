# C2 bucket kernel at 3 rows per thread per step (no spilled VGPRs) against 4: alternating, three
# rounds, plus the selectivity sweep of each
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 20 --warmup 5 --no-join --c5-rows 0"
X=$PWD/tiflash_amd/exp/lib_TFG_EXP_RT3.so
for i in 1 2 3; do
  timeout -k 10 200 $B --no-variants >> gpurun_out/r05ab_main.jsonl 2>> gpurun_out/r05ab.err
  TFA_LIB_PATH=$X timeout -k 10 200 $B --no-variants >> gpurun_out/r05ab_rt3.jsonl 2>> gpurun_out/r05ab.err
done
TFA_LIB_PATH=$X timeout -k 10 300 $B >> gpurun_out/r05ab_rt3_sweep.jsonl 2>> gpurun_out/r05ab.err
echo R05AB_DONE
