# join probe with per-wave output claims (no block scan / barrier a step) against the block form:
# the join parity tests on the experiment library, then C3 alternating, three rounds
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
X=$PWD/tiflash_amd/exp/lib_TFG_EXP_WAVECLAIM.so
TFA_LIB_PATH=$X timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_hash_agg_join.py tests/test_gpu_join_keys.py tests/test_gpu_full_scale.py -k "join or c3 or probe" > gpurun_out/r05af_tests.log 2>&1 || { echo TESTS_FAIL; tail -8 gpurun_out/r05af_tests.log; exit 0; }
tail -1 gpurun_out/r05af_tests.log
B="python3 bench.py --no-cpu --no-variants --c5-rows 0 --codec-rows 0 --rows 1000000 --steps 20 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 $B >> gpurun_out/r05af_main.jsonl 2>> gpurun_out/r05af.err
  TFA_LIB_PATH=$X timeout -k 10 200 $B >> gpurun_out/r05af_wave.jsonl 2>> gpurun_out/r05af.err
done
echo R05AF_DONE
