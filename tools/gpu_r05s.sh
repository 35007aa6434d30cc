# sparse-filter (memset tile table, all words in flight) and short-last-segment tests, the C++
# suite once more, C2 with its selectivity sweep
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_sparse_filter.py tests/test_gpu_tiled_tail.py tests/test_gpu_c2_full.py > gpurun_out/r05s_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 gpurun_out/r05s_tests.log; exit 0; }
timeout -k 10 300 tiflash_amd/host/build/test_host $PWD > gpurun_out/r05s_cpp.log 2>&1 || true
if grep -q "HIP error" gpurun_out/r05s_cpp.log; then echo FAULT_SEEN; exit 0; fi
timeout -k 10 300 python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 --no-join --c5-rows 0 > gpurun_out/r05s_c2.json 2> gpurun_out/r05s_c2.err
echo R05S_DONE
