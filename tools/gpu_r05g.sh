# C++ suite diagnostics + the two-rank C++ exchange, the negative-value two-phase first_row case,
# C2 (sweep kernels) / C5 benches of main vs cheap slot hash vs no wide home path, bucket PMC
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05g_cpp.log 2>&1 || true
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_minmax_wide.py -k "two_phase" > gpurun_out/r05g_tests.log 2>&1 || true
timeout -k 10 300 python3 bench.py --no-cpu --no-join --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05g_main.json 2> gpurun_out/r05g_main.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_CHEAP_SLOT.so timeout -k 10 300 python3 bench.py --no-cpu --no-join --no-variants --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05g_cheap.json 2> gpurun_out/r05g_cheap.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_NO_WIDE_HOME.so timeout -k 10 300 python3 bench.py --no-cpu --no-join --no-variants --codec-rows 0 --rows 1000000 --steps 10 --warmup 3 > gpurun_out/r05g_nowh.json 2> gpurun_out/r05g_nowh.err
bash tools/pmc_kernel.sh agg_bucket_tiled r05g --no-variants --c5-rows 0 --codec-rows 0 > /dev/null
echo R05G_DONE
