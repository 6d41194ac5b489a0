#!/bin/bash
# r05ab: split-K reduce with 8 slabs in flight per thread -- GEMM / conv tests (bit-identity tests included), B = 1 and
# B = 8 A/B against the previous build (3d47626) on one box
set -u
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_prev$i SDMOE_AB=1 SDMOE_LIB=$P python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_cur$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
for i in 1 2; do
  run b8_prev$i SDMOE_AB=1 SDMOE_LIB=$P python bench.py --steps 4 --warmup 1 $BA
  run b8_cur$i python bench.py --steps 4 --warmup 1 $BA
done
