# C++ suite (two-phase first_row diagnosis), the zero-copy exchange and a15 two-phase variants, then
# the packed run-record bucket experiment vs its baseline build
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05d_cpp.log 2>&1 || true
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_exchange_slices.py tests/test_gpu_multirank.py "tests/test_gpu_minmax_wide.py::test_mixed_two_phase_with_count" > gpurun_out/r05d_tests.log 2>&1 || true
for v in TFG_EXP_BASE TFG_EXP_RUNS; do
  TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_$v.so timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/exp5d_$v.json 2> gpurun_out/exp5d_$v.err
done
