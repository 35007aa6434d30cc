set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/b.log | head -1; grep -o '"join_probe": {.*' gpurun_out/b.log | cut -c1-700
timeout -k 10 200 python bench.py --no-cpu --no-join --groups 10000000 > gpurun_out/b10m.log 2>&1 || { tail -20 gpurun_out/b10m.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/b10m.log | head -1; grep -o '"check": {[^}]*}' gpurun_out/b10m.log; grep -o '"kernels_ms_per_step": {[^}]*}' gpurun_out/b10m.log
