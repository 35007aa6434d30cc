# round-5 final tree (wide-key tables sized for two workgroups per CU): full GPU suite (C++ driver
# included) + smoke, the default bench line, the rocprof trace and the FETCH / WRITE PMC passes
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05aa
timeout -k 10 600 python3 bench.py > gpurun_out/r05aa_bench.json 2> gpurun_out/r05aa_bench.err
bash tools/profile.sh r05aa
echo R05AA_DONE
