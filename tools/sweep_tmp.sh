mkdir -p gpurun_out
run() { # name env...
  name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --no-cpu --no-join --c5-rows 0 --steps 5 --warmup 2 > gpurun_out/sw_$name.log 2>&1 || return 1
  echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/sw_$name.log | head -1) $(grep -o 'kernels_ms_per_step[^}]*}' gpurun_out/sw_$name.log)"
}
run d1 TFG_X=0 && run dbg5 TFG_DBG_BUCKET=5 && run dbg6 TFG_DBG_BUCKET=6 && true
