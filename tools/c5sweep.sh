set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_hash_agg_join.py tests/test_gpu_join_keys.py tests/test_gpu_full_scale.py -x -q --timeout 200 --timeout-method thread -k "join or c3 or Join" > gpurun_out/t_join.log 2>&1; echo "join rc=$?"; tail -3 gpurun_out/t_join.log
timeout -k 10 200 python bench.py --no-cpu --c5-rows 0 --codec-rows 0 --no-variants --rows 10000000 > gpurun_out/c3.json 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/c3.json').read().strip().splitlines()[-1])['join_probe']
print(d['ms_per_step'], d['matches'], d['kernels_ms_per_step'], d['join_v2']['check_ok'])
"
timeout -k 10 400 python -u -m pytest tests/test_gpu_arith_wide.py tests/test_gpu_arith.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_arith.log 2>&1; echo "arith rc=$?"; tail -3 gpurun_out/t_arith.log
