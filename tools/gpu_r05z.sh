# C5 table cells (two 8-wave workgroups per CU up to ~1500 cells of 48 B) and C2 at 1024 buckets
# with the 128-VGPR 512-thread kernel
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3 --no-join --no-variants"
for c in 1280 1408 1472 2048 1472 1280; do
  TFG_AGG_TABLE_CELLS=$c timeout -k 10 200 $B --rows 1000000 >> gpurun_out/r05z_c5cells.jsonl 2>> gpurun_out/r05z.err
done
timeout -k 10 200 $B --c5-rows 0 --bucket-bits 10 >> gpurun_out/r05z_c2bb10.jsonl 2>> gpurun_out/r05z.err
echo R05Z_DONE
