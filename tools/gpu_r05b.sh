# bucket-kernel cost attribution (instrumented variants, tools/build_exp.sh) + the sampled-index search
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_host_cpp.py tests/test_gpu_minmax_wide.py::test_without_key_wide_and_empty > gpurun_out/r05b_tests.log 2>&1 || true
for v in TFG_EXP_BASE TFG_EXP_NOATOM TFG_EXP_NOPROBE TFG_EXP_NOATOM_TFG_EXP_NOPROBE; do
  TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_$v.so timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/exp_$v.json 2> gpurun_out/exp_$v.err
done
timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/exp_main.json 2> gpurun_out/exp_main.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c2_full.py tests/test_gpu_hash_agg_join.py > gpurun_out/r05b_c2tests.log 2>&1
for bb in 9 10; do
  timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 --bucket-bits $bb > gpurun_out/sweep_bb$bb.json 2> gpurun_out/sweep_bb$bb.err
done
