#!/bin/bash
# halo conv: kernel tests, conv micro rows (halo on / off), pipeline bench (halo on / off, same box)
set -u
mkdir -p gpurun_out/r04h
bash tools/gpu_tests.sh tests/test_gpu_kernels.py -k "conv" || exit 1
for h in 1 0; do
  echo "== conv rows halo=$h"
  SDMOE_TUNE="16=$h" timeout -k 10 300 python tools/gemm_bench.py --only conv --iters 10 > gpurun_out/r04h/conv_h$h.log 2>&1 || { echo "FAILED conv rows"; tail -5 gpurun_out/r04h/conv_h$h.log; exit 1; }
  grep conv gpurun_out/r04h/conv_h$h.log
done
BA="--no-cpu-baseline --e2e-steps 0"
for h in 1 0 1 0; do
  SDMOE_TUNE="16=$h" timeout -k 10 600 python bench.py --steps 3 --warmup 1 $BA > gpurun_out/r04h/b8_h$h.log 2>&1 || { echo "FAILED bench"; tail -20 gpurun_out/r04h/b8_h$h.log; exit 1; }
  echo "halo=$h $(grep -a '^{' gpurun_out/r04h/b8_h$h.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["avg_launch_ms"])')"
done
