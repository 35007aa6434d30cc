set -o pipefail
run() { timeout -k 10 200 python bench.py --no-cpu --no-join --codec-rows 0 --no-variants --rows 10000000 > gpurun_out/c5_$1.json 2>&1 || exit 1
python -c "
import json,sys
d=json.loads(open('gpurun_out/c5_$1.json').read().strip().splitlines()[-1])['string_agg']
print('$1', d['ms_per_step'], d['check']['ok'], d['kernels_ms_per_step'])
"; }
run auto
cp tiflash_amd/exp/libtiflash_amd.so tiflash_amd/libtiflash_amd.so
run rg2048
