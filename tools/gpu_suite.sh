#!/bin/bash
# Full GPU parity suite + smoke on the box (one process, per-test timeout), results under gpurun_out/.
# usage: bash tools/gpu_suite.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_gputests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { echo GPU_TESTS_FAIL; tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
fi
tail -3 gpurun_out/${TAG}_gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
echo SUITE_OK
