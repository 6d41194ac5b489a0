#!/bin/bash
# A/B two builds of libsdmoe_hip.so on one box: the current one vs sdmoe/libsdmoe_hip_prev.so (SDMOE_LIB), each
# step under its own limit: kernel microbench rows (optional filter $1) then the metric bench, interleaved twice.
set -u
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
ONLY=${1:-}
timeout -k 10 300 python tools/gemm_bench.py --only "$ONLY" > gpurun_out/ab_gb_cur.log 2>&1 || exit 1
SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python tools/gemm_bench.py --only "$ONLY" > gpurun_out/ab_gb_prev.log 2>&1 || exit 1
paste -d'|' <(grep -E "us " gpurun_out/ab_gb_cur.log) <(grep -E "us " gpurun_out/ab_gb_prev.log | awk '{print $(NF-3), $(NF-2)}')
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_prev.log)"
done
