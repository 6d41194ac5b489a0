#!/bin/bash
# r05o: one-launch GroupNorm statistics (knob 24) + LayerNorm folded into the GEGLU at small M -- GN tests, B = 1 and
# B = 8 A/B on one box (knob 24 = 0 is the previous statistics path)
set -u
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "groupnorm or gn" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env... -- args
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_old$i SDMOE_TUNE=24=0 python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_gn$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_gnln$i SDMOE_LN_FFN_MAXM=8192 python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
for i in 1 2; do
  run b8_old$i SDMOE_TUNE=24=0 python bench.py --steps 4 --warmup 1 $BA
  run b8_gn$i python bench.py --steps 4 --warmup 1 $BA
done
run b8_gnln SDMOE_LN_FFN_MAXM=8192 python bench.py --steps 4 --warmup 1 $BA
bash tools/gpu_measure.sh r05o trace_b1
