#!/bin/bash
# in-kernel GroupNorm: kernel tests + U-Net pipeline tests, then the metric bench with / without it (same box)
set -u
mkdir -p gpurun_out/r04n
bash tools/gpu_tests.sh tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_metric_parity.py || exit 1
BA="--no-cpu-baseline --e2e-steps 0"
for f in 1 0 1 0; do
  SDMOE_FUSED_GN=$f timeout -k 10 600 python bench.py --steps 3 --warmup 1 $BA > gpurun_out/r04n/b8_gn$f.log 2>&1 || { echo "FAILED bench"; tail -20 gpurun_out/r04n/b8_gn$f.log; exit 1; }
  echo "fused_gn=$f $(grep -a '^{' gpurun_out/r04n/b8_gn$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"], d["roofline"]["avg_launch_ms"])')"
done
