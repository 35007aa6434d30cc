# a15 tests through the C ABI, the C2 kernels with the pending state + consecutive-row loads, then the C++ suite
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_minmax_wide.py tests/test_gpu_minmax.py tests/test_gpu_c2_full.py tests/test_gpu_keys_agg.py tests/test_gpu_hash_agg_join.py > gpurun_out/r05c_tests.log 2>&1
timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05c_cpp.log 2>&1
