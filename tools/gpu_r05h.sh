# first_row bisect (C++), parity of the skip-ahead partition / dense run index, benches: main,
# no wide home path (C5), nontemporal partition stores (C2 + C3), then the bucket PMC pass
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 tiflash_amd/host/build/test_host $PWD PlanAggregateMinMaxFirstRow > gpurun_out/r05h_cpp_one.log 2>&1 || true
timeout -k 10 300 python -u -m pytest -v --timeout 250 --timeout-method thread tests/test_gpu_host_cpp.py > gpurun_out/r05h_cpp.log 2>&1 || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_c2_full.py tests/test_gpu_keys_agg.py tests/test_gpu_hash_agg_join.py tests/test_gpu_filter.py tests/test_gpu_agg_three_aggs.py tests/test_gpu_minmax_wide.py > gpurun_out/r05h_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05h_main.json 2> gpurun_out/r05h_main.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_NO_WIDE_HOME.so timeout -k 10 200 python3 bench.py --no-cpu --no-join --no-variants --codec-rows 0 --rows 1000000 --steps 10 --warmup 3 > gpurun_out/r05h_nowh.json 2> gpurun_out/r05h_nowh.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_PART_NT.so timeout -k 10 200 python3 bench.py --no-cpu --no-variants --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05h_pnt.json 2> gpurun_out/r05h_pnt.err
bash tools/pmc_kernel.sh agg_bucket_tiled r05h --no-variants --c5-rows 0 --codec-rows 0 > /dev/null
echo R05H_DONE
