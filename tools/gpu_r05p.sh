# the C++ operator suite with TFG_SYNC_CHECK=1 (every checked launch waits: a kernel fault is
# reported at the launch site after it); then, when it passed: C5 at 12 / 13 / 14 bucket bits
# (Int128 sums without the zero high-word atomics), C3 with and without nontemporal regroup
# loads, C2's selectivity sweep with and without the vector all-false tile check
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TFG_SYNC_CHECK=1 timeout -k 10 300 tiflash_amd/host/build/test_host $PWD > gpurun_out/r05p_cpp.log 2>&1 || true
if grep -q "HIP error" gpurun_out/r05p_cpp.log; then echo FAULT_SEEN; exit 0; fi
timeout -k 10 200 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_minmax_wide.py tests/test_gpu_result_hint.py -k "three_slices or mixed_collators or hint" > gpurun_out/r05p_wide.log 2>&1 || { echo WIDE_FAIL; tail -5 gpurun_out/r05p_wide.log; exit 0; }
B="python3 bench.py --no-cpu --codec-rows 0 --steps 10 --warmup 3"
for bb in 12 13 14; do
  timeout -k 10 200 $B --no-join --no-variants --rows 1000000 --c5-bucket-bits $bb > gpurun_out/r05p_c5bb$bb.json 2> gpurun_out/r05p_c5bb$bb.err
done
timeout -k 10 200 $B --no-variants --c5-rows 0 --rows 1000000 > gpurun_out/r05p_c3.json 2> gpurun_out/r05p_c3.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_RG_NT.so timeout -k 10 200 $B --no-variants --c5-rows 0 --rows 1000000 > gpurun_out/r05p_c3rg.json 2> gpurun_out/r05p_c3rg.err
timeout -k 10 300 $B --no-join --c5-rows 0 > gpurun_out/r05p_c2.json 2> gpurun_out/r05p_c2.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_SKIPVEC.so timeout -k 10 300 $B --no-join --c5-rows 0 > gpurun_out/r05p_c2sv.json 2> gpurun_out/r05p_c2sv.err
echo R05P_DONE
