# rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks share cuda:0 over gloo (not a measurement)
set -eu
mkdir -p gpurun_out
SDMOE_SAME_DEVICE_REHEARSAL=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --inference-steps 3 \
  --no-cpu-baseline --mask union > gpurun_out/dp2.log 2>&1 || { tail -40 gpurun_out/dp2.log; exit 1; }
grep -a '"metric"' gpurun_out/dp2.log | cut -c1-700
