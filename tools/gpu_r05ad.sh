# sparse all-false check with four tiles a round against two: C2's selectivity sweep, alternating
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 20 --warmup 5 --no-join --c5-rows 0"
X=$PWD/tiflash_amd/exp/lib_TFG_EXP_SKIP4.so
for i in 1 2; do
  timeout -k 10 300 $B >> gpurun_out/r05ad_main.jsonl 2>> gpurun_out/r05ad.err
  TFA_LIB_PATH=$X timeout -k 10 300 $B >> gpurun_out/r05ad_skip4.jsonl 2>> gpurun_out/r05ad.err
done
echo R05AD_DONE
