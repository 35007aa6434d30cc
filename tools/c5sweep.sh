set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_zstd.py tests/test_codec.py tests/test_codec_lz4.py tests/test_gpu_hash_agg_join.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_zk.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/t_zk.log
timeout -k 10 300 python bench.py --rows 1000000 --no-variants --no-cpu --no-join --c5-rows 0 > gpurun_out/zb.json 2>&1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/zb.json').read().strip().splitlines()[-1]); print(d['packet_codec']['legs']['zstd'])"
