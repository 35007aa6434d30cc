set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_arith_wide.py tests/test_gpu_arith.py tests/test_gpu_host_cpp.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_arith.log 2>&1; echo "arith rc=$?"; tail -3 gpurun_out/t_arith.log
run() { timeout -k 10 200 python bench.py --no-cpu --no-join --codec-rows 0 --no-variants --rows 10000000 > gpurun_out/c5_$1.json 2>&1 || exit 1
python -c "
import json,sys
d=json.loads(open('gpurun_out/c5_$1.json').read().strip().splitlines()[-1])['string_agg']
print('$1', d['ms_per_step'], d['check']['ok'], d['kernels_ms_per_step'])
"; }
run auto
cp tiflash_amd/exp/libtiflash_amd.so tiflash_amd/libtiflash_amd.so
run rg2048
