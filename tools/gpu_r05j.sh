# the C++ operator suite first (its log kept whatever the outcome), then the full GPU suite + smoke,
# the default bench line and the rocprof evidence of the round-5 tree
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 tiflash_amd/host/build/test_host $PWD > gpurun_out/r05j_cpp.log 2>&1 || true
bash tools/gpu_suite.sh r05j
timeout -k 10 600 python3 bench.py > gpurun_out/r05j_bench.json 2> gpurun_out/r05j_bench.err
bash tools/profile.sh r05j
bash tools/pmc_kernel.sh WideFastOps r05j_wide --no-variants --rows 1000000 --codec-rows 0 > /dev/null
echo R05J_DONE
