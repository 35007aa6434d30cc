set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_hash_agg_join.py -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for cfg in "0 8" "0 9" "0 10"; do set -- $cfg
TFG_DBG_SCATTER=$1 timeout -k 10 120 python bench.py --no-cpu --no-join --bucket-bits $2 > gpurun_out/s_$1_$2.log 2>&1
echo "dbg=$1 bb=$2 $(grep -o '"value": [0-9.]*' gpurun_out/s_$1_$2.log | head -1) $(grep -o '"kernels_ms_per_step": {[^}]*}' gpurun_out/s_$1_$2.log)"
done
