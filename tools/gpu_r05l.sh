# the bench legs after reverting the two-tile skip-ahead and the persistent bucket loop
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c2_full.py tests/test_gpu_keys_agg.py tests/test_gpu_result_hint.py > gpurun_out/r05l_tests.log 2>&1
echo R05L_DONE
