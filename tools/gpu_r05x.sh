#!/bin/bash
# r05x: single-launch GroupNorm (statistics + apply) up to 32x32 for calls of <= 4096 rows (knob 24) -- GN tests with
# the knob on, per-launch A/B at 2 images, B = 1 bench A/B
set -u
O=gpurun_out/r05x; mkdir -p $O
SDMOE_TUNE=24=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "groupnorm" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/micro_ab.py gn --nimg 2 --tune "24=0" --tune "24=4096" > $O/gn2.log 2>&1 || { tail $O/gn2.log; exit 1; }
grep "silu HW=1024" $O/gn2.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_off$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_on$i SDMOE_TUNE=24=4096 python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
