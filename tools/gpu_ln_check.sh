#!/bin/bash
# LN-fold check on the GPU box: new kernel tests, the U-Net/SDXL pipeline tests, gemm_bench LN rows, then the metric
# bench with the fold on / off (SDMOE_FUSED_LN), interleaved. Every step under its own limit; stop at the first failure.
set -u
mkdir -p gpurun_out/ln
O=gpurun_out/ln
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "ln or geglu" --timeout 300 --timeout-method thread > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -3 $O/kern.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/unet.log 2>&1 || { tail -30 $O/unet.log; exit 1; }
tail -3 $O/unet.log
timeout -k 10 300 python tools/gemm_bench.py > $O/gb.log 2>&1 || { tail -20 $O/gb.log; exit 1; }
grep -E "ln|geglu-gemm|layernorm" $O/gb.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/b_on.log 2>&1 || { tail -20 $O/b_on.log; exit 1; }
  echo "ln-fold  $(grep -a -o '"value": [0-9.]*' $O/b_on.log)"
  SDMOE_FUSED_LN=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/b_off.log 2>&1 || { tail -20 $O/b_off.log; exit 1; }
  echo "explicit $(grep -a -o '"value": [0-9.]*' $O/b_off.log)"
done
