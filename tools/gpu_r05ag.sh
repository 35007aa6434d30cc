# the round-end artifact: default bench line, rocprof kernel trace and FETCH / WRITE PMC passes
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > gpurun_out/r05ag_bench.json 2> gpurun_out/r05ag_bench.err
bash tools/profile.sh r05ag
echo R05AG_DONE
