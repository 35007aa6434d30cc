# C5 radix sweep (12 / 13 bucket bits against the default 14) and the regroup nontemporal-load A/B on C3
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for bb in 12 13; do
  timeout -k 10 200 python3 bench.py --no-cpu --no-join --no-variants --codec-rows 0 --rows 1000000 --c5-bucket-bits $bb --steps 10 --warmup 3 > gpurun_out/r05n_c5bb$bb.json 2> gpurun_out/r05n_c5bb$bb.err
done
timeout -k 10 200 python3 bench.py --no-cpu --no-variants --c5-rows 0 --codec-rows 0 --rows 1000000 --steps 10 --warmup 3 > gpurun_out/r05n_c3.json 2> gpurun_out/r05n_c3.err
TFA_LIB_PATH=$PWD/tiflash_amd/exp/lib_TFG_EXP_RG_NT.so timeout -k 10 200 python3 bench.py --no-cpu --no-variants --c5-rows 0 --codec-rows 0 --rows 1000000 --steps 10 --warmup 3 > gpurun_out/r05n_c3rg.json 2> gpurun_out/r05n_c3rg.err
echo R05N_DONE
