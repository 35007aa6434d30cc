# C2 at 256 (default) / 512 / 1024 aggregation buckets (two bucket workgroups per CU below ~80 KB
# of table), three repeats of the default for the step's spread
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="python3 bench.py --no-cpu --codec-rows 0 --steps 20 --warmup 5 --no-join --c5-rows 0 --no-variants"
for bb in 0 9 10 0 0; do
  timeout -k 10 200 $B --bucket-bits $bb >> gpurun_out/r05u_c2.jsonl 2>> gpurun_out/r05u_c2.err
done
echo R05U_DONE
