#!/bin/bash
# Full -m gpu suite (stop at the first failure, parity report), then the metric bench current vs
# sdmoe/libsdmoe_hip_prev.so, interleaved twice. Each step under its own limit.
set -u
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/sab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' gpurun_out/sab_cur.log)"
  SDMOE_LIB=$P SDMOE_FUSED_LN=${PREV_LN:-1} timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/sab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' gpurun_out/sab_prev.log)"
done
