# the final tree (512-thread bucket kernel held to 128 VGPRs): full GPU suite + smoke, the default
# bench line, then C5 with 1280- / 1024-cell tables (two 8-wave workgroups per CU) against 2048
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05y
timeout -k 10 600 python3 bench.py > gpurun_out/r05y_bench.json 2> gpurun_out/r05y_bench.err
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 --no-join --no-variants --rows 1000000"
for c in 1280 1024 2048; do
  TFG_AGG_TABLE_CELLS=$c timeout -k 10 200 $B >> gpurun_out/r05y_c5cells.jsonl 2>> gpurun_out/r05y_c5cells.err
done
echo R05Y_DONE
