# round-5 evidence: the full GPU suite (C++ operator driver included) + smoke, the default bench
# line, the rocprof kernel trace and the FETCH / WRITE PMC passes
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05v
timeout -k 10 600 python3 bench.py > gpurun_out/r05v_bench.json 2> gpurun_out/r05v_bench.err
bash tools/profile.sh r05v
echo R05V_DONE
