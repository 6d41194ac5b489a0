#!/bin/bash
# r05t: ping-pong routed GEGLU (knob 25) -- bit-identity test, per-launch A/B, metric A/B on one box
set -u
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "pingpong" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 300 python tools/micro_ab.py geglu --iters 30 --tune "25=0" --tune "25=1" > $O/geglu.log 2>&1 || { tail $O/geglu.log; exit 1; }
grep geglu $O/geglu.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b8_old$i python bench.py --steps 4 --warmup 1 $BA
  run b8_pp$i SDMOE_TUNE=25=1 python bench.py --steps 4 --warmup 1 $BA
done
