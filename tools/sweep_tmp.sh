set -e
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-join > gpurun_out/b1.log 2>&1 || { tail -20 gpurun_out/b1.log; exit 1; }
tail -1 gpurun_out/b1.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --dist-backend gloo --rows 20000000 --steps 3 --warmup 1 --no-cpu --no-join > gpurun_out/b2.log 2>&1 || { tail -30 gpurun_out/b2.log; exit 1; }
grep '^{' gpurun_out/b2.log | cut -c1-300; grep -o '"check": {[^}]*}' gpurun_out/b2.log
