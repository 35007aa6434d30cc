# the C++ operator suite (log kept), the wide min/max mirror case, the GPU suite without the C++
# driver, the default bench line, the rocprof evidence and the wide bucket kernel PMC pass
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 tiflash_amd/host/build/test_host $PWD > gpurun_out/r05m_cpp.log 2>&1 || true
timeout -k 10 200 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_minmax_wide.py -k "mixed_collators or two_phase" > gpurun_out/r05m_wide.log 2>&1 || true
bash tools/gpu_suite.sh r05m "not host_operators_cpp"
timeout -k 10 600 python3 bench.py > gpurun_out/r05m_bench.json 2> gpurun_out/r05m_bench.err
bash tools/profile.sh r05m
bash tools/pmc_kernel.sh WideFastOps r05m_wide --no-variants --rows 1000000 --codec-rows 0 > /dev/null
echo R05M_DONE
