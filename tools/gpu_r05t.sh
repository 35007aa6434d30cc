# fused String-key result (C5) and two-tile sparse check: the keys / C5 / sparse / hint tests, the
# C5 leg, C2 with its selectivity sweep
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_sparse_filter.py tests/test_gpu_result_hint.py tests/test_gpu_keys_agg.py tests/test_gpu_full_scale.py -k "c5 or keys or sparse or hint or tail or short" tests/test_gpu_tiled_tail.py > gpurun_out/r05t_tests.log 2>&1 || { echo TESTS_FAIL; tail -8 gpurun_out/r05t_tests.log; exit 0; }
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3"
timeout -k 10 300 $B --no-join > gpurun_out/r05t_c2c5.json 2> gpurun_out/r05t_c2c5.err
echo R05T_DONE
