set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_hash_agg_join.py tests/test_gpu_host_cpp.py -m gpu -x -q -k "join or Join or host" > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/b.log | head -1; grep -o '"join_probe": {.*' gpurun_out/b.log | cut -c1-700
