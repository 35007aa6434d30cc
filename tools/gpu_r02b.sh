set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02b_multirank.log 2>&1 || { echo MULTIRANK_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --rows 20000000 --c5-rows 10000000 --c5-groups 1000000 --join-build 2000000 --join-probe 20000000 --no-cpu --steps 3 --warmup 1 > gpurun_out/r02b_bench_gloo2.log 2>&1 || { echo GLOO2_FAIL; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r02b_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
