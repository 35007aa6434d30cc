# C++ suite (crash handler), bucket-kernel / pred-first partition parity, C2 bench (main vs keys-with-pred),
# then the C3 probe FETCH / WRITE attribution passes
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05e_cpp.log 2>&1 || true
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c2_full.py tests/test_gpu_keys_agg.py tests/test_gpu_hash_agg_join.py tests/test_gpu_minmax_wide.py tests/test_gpu_agg_three_aggs.py tests/test_gpu_agg_count_only.py > gpurun_out/r05e_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05e_main.json 2> gpurun_out/r05e_main.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_KEYS_WITH_PRED.so timeout -k 10 300 python3 bench.py --no-cpu --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05e_kwp.json 2> gpurun_out/r05e_kwp.err
mkdir -p gpurun_out/pmc_r05e
for v in full nobuild miss; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --kernel-include-regex join_probe --pmc $c -d gpurun_out/pmc_r05e/${v}_$c -o run -f csv -- python3 tools/join_traffic.py $v > gpurun_out/pmc_r05e/${v}_$c.log 2>&1
  done
done
echo R05E_DONE
