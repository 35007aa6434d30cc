# the round-end artifact as it stands: full GPU suite + smoke
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash tools/gpu_suite.sh r05ae
echo R05AE_DONE
