#!/bin/bash
# r05p: one-launch GroupNorm statistics v2 (parallel finalizer loads, <= 32 slices) -- GN tests, per-launch A/B at
# 2 and 16 images, B = 1 bench A/B
set -u
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "groupnorm or gn" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/micro_ab.py gn --nimg 2 --tune "24=0" --tune "24=1" > $O/gn2.log 2>&1 || { tail $O/gn2.log; exit 1; }
timeout -k 10 300 python tools/micro_ab.py gn --nimg 16 --tune "24=0" --tune "24=1" > $O/gn16.log 2>&1 || { tail $O/gn16.log; exit 1; }
grep stats $O/gn2.log $O/gn16.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_old$i SDMOE_TUNE=24=0 python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_gn$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
