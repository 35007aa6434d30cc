# C5 with the partition's tiles cut to whole half-batches (5120 -> 4096 rows) against 5120
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 --no-join --no-variants --rows 1000000"
X=$PWD/tiflash_amd/exp/lib_TFG_EXP_TRHALF.so
for i in 1 2 3; do
  timeout -k 10 200 $B >> gpurun_out/r05ah_main.jsonl 2>> gpurun_out/r05ah.err
  TFA_LIB_PATH=$X timeout -k 10 200 $B >> gpurun_out/r05ah_half.jsonl 2>> gpurun_out/r05ah.err
done
echo R05AH_DONE
