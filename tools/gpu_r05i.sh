# full GPU suite + smoke on the round-5 tree, the default bench line, then the rocprof evidence
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05i
timeout -k 10 600 python3 bench.py > gpurun_out/r05i_bench.json 2> gpurun_out/r05i_bench.err
bash tools/profile.sh r05i
echo R05I_DONE
