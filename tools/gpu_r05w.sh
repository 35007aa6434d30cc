# bucket-kernel prologue A/B (tile column loaded once, cursor atomics overlapped with the table
# clear): C2 + C5, alternating main / experiment library, three rounds
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 20 --warmup 5 --no-join --no-variants"
X=$PWD/tiflash_amd/exp/lib_TFG_EXP_PROLOGUE.so
for i in 1 2 3; do
  timeout -k 10 200 $B >> gpurun_out/r05w_main.jsonl 2>> gpurun_out/r05w.err
  TFA_LIB_PATH=$X timeout -k 10 200 $B >> gpurun_out/r05w_exp.jsonl 2>> gpurun_out/r05w.err
done
echo R05W_DONE
