# round 5: new min / max / first_row tests, the existing agg suites, then the C2 bucket-bits sweep
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_minmax_wide.py tests/test_gpu_minmax.py tests/test_gpu_keys_agg.py tests/test_gpu_agg_three_aggs.py tests/test_gpu_host_cpp.py > gpurun_out/r05a_tests.log 2>&1
for bb in 8 9 10; do
  timeout -k 10 240 python3 bench.py --no-cpu --no-variants --no-join --c5-rows 0 --codec-rows 0 --steps 10 --warmup 3 --bucket-bits $bb > gpurun_out/sweep_bb$bb.json 2> gpurun_out/sweep_bb$bb.err
done
