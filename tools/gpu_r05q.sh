#!/bin/bash
# r05q: 32-wide halo convs (knob 16 = 3) at one prompt per call: per-launch conv A/B at 2 and 16 images, B = 1 bench
set -u
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 --tune "16=1" --tune "16=3" > $O/conv2.log 2>&1 || { tail $O/conv2.log; exit 1; }
cat $O/conv2.log
timeout -k 10 300 python tools/micro_ab.py conv --nimg 16 --tune "16=1" --tune "16=3" > $O/conv16.log 2>&1 || { tail $O/conv16.log; exit 1; }
cat $O/conv16.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_def$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_h3$i SDMOE_TUNE=16=3 python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
# GEGLU / linear time split by the diagnostic knob 6 (1 no K-loop loads, 2 no MFMAs, 4 no epilogue)
timeout -k 10 300 python tools/micro_ab.py geglu --tune "6=0" --tune "6=4" --tune "6=1" --tune "6=3" --tune "6=2" > $O/geglu_diag.log 2>&1 || { tail $O/geglu_diag.log; exit 1; }
cat $O/geglu_diag.log
