# the final tree: full GPU suite (C++ driver included) + smoke, then the default bench line
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05x
timeout -k 10 600 python3 bench.py > gpurun_out/r05x_bench.json 2> gpurun_out/r05x_bench.err
echo R05X_DONE
