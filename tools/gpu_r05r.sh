# the C++ operator suite without TFG_SYNC_CHECK (collation sort keys out of the stream-ordered
# pool, guarded row references), the sparse-filter / capacity-hint / wide mirror tests, C2 with
# its selectivity sweep (adaptive vector all-false check), C5 at 15 / 16 bucket bits
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 tiflash_amd/host/build/test_host $PWD > gpurun_out/r05r_cpp.log 2>&1 || true
if grep -q "HIP error" gpurun_out/r05r_cpp.log; then echo FAULT_SEEN; exit 0; fi
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_sparse_filter.py tests/test_gpu_minmax_wide.py tests/test_gpu_result_hint.py > gpurun_out/r05r_tests.log 2>&1 || { echo TESTS_FAIL; tail -5 gpurun_out/r05r_tests.log; exit 0; }
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3"
timeout -k 10 300 $B --no-join --c5-rows 0 > gpurun_out/r05r_c2.json 2> gpurun_out/r05r_c2.err
for bb in 15 16; do
  timeout -k 10 200 $B --no-join --no-variants --rows 1000000 --c5-bucket-bits $bb > gpurun_out/r05r_c5bb$bb.json 2> gpurun_out/r05r_c5bb$bb.err
done
echo R05R_DONE
