# C++ suite, parity of the adaptive key skip / wide home fast path / nontemporal probe, the full
# bench (main) + C3 with temporal probe stores (A/B), then the probe FETCH attribution passes
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05f_cpp.log 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_c2_full.py tests/test_gpu_full_scale.py tests/test_gpu_keys_agg.py tests/test_gpu_hash_agg_join.py tests/test_gpu_join_keys.py tests/test_gpu_filter.py > gpurun_out/r05f_tests.log 2>&1
timeout -k 10 400 python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05f_main.json 2> gpurun_out/r05f_main.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_JOIN_TEMPORAL.so timeout -k 10 300 python3 bench.py --no-cpu --no-variants --c5-rows 0 --codec-rows 0 --rows 1000000 --steps 10 --warmup 3 > gpurun_out/r05f_jt.json 2> gpurun_out/r05f_jt.err
timeout -k 10 120 python3 tools/singlepass_probe.py > gpurun_out/r05f_singlepass.json 2> gpurun_out/r05f_singlepass.err
mkdir -p gpurun_out/pmc_r05f
for v in full nobuild miss; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex join_probe --pmc FETCH_SIZE -d gpurun_out/pmc_r05f/${v} -o run -f csv -- python3 tools/join_traffic.py $v > gpurun_out/pmc_r05f/${v}.log 2>&1
done
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_JOIN_TEMPORAL.so timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex join_probe --pmc FETCH_SIZE -d gpurun_out/pmc_r05f/full_temporal -o run -f csv -- python3 tools/join_traffic.py full > gpurun_out/pmc_r05f/full_temporal.log 2>&1
echo R05F_DONE
