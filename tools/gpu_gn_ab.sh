#!/bin/bash
# GroupNorm small-path block size A/B on one box: gemm_bench GN rows and the metric bench, SDMOE_TUNE 7=1024 vs 7=256.
set -u
mkdir -p gpurun_out/gn
O=gpurun_out/gn
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "groupnorm" --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for nt in 1024 256; do
  timeout -k 10 300 python tools/gemm_bench.py --gnt $nt --only gn-stats > $O/gb$nt.log 2>&1 || exit 1
done
paste -d'|' <(grep gn-stats $O/gb1024.log | cut -c1-60) <(grep gn-stats $O/gb256.log | awk '{print $(NF-3)}')
for i in 1 2; do
  for nt in 1024 256; do
    SDMOE_TUNE=7=$nt timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/b$nt.log 2>&1 || exit 1
    echo "gn $nt $(grep -a -o '"value": [0-9.]*' $O/b$nt.log)"
  done
done
