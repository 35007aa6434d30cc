set -o pipefail
run() { timeout -k 10 200 python bench.py --no-cpu --no-join --codec-rows 0 --no-variants --rows 10000000 > gpurun_out/c5_$1.json 2>&1 || exit 1
python -c "
import json,sys
d=json.loads(open('gpurun_out/c5_$1.json').read().strip().splitlines()[-1])['string_agg']
print('$1', d['ms_per_step'], d['check']['ok'], d['kernels_ms_per_step'])
"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_keys_agg.py tests/test_gpu_full_scale.py -x -q --timeout 200 --timeout-method thread -k "string or fixed_keys or c5" > gpurun_out/t_rg.log 2>&1; echo "rg1536 tests rc=$?"; tail -1 gpurun_out/t_rg.log
run rg1536
cp tiflash_amd/exp_a/libtiflash_amd.so tiflash_amd/libtiflash_amd.so
run rg1024
