#!/bin/bash
# conv tile sweep at the 32x32 / 8x8 / 16x16 levels: knob 1 (tile) x knob 9 (split-K)
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04t; mkdir -p $O
for t in "0" "1=3" "1=5" "1=4" "1=3,9=2" "1=3,9=4" "1=4,9=4" "1=5,9=4" "1=1,9=2" "1=1,9=8" "1=7" "1=8" "1=3,9=8" "1=5,9=8" "1=2"; do
  SDMOE_TUNE="$t" timeout -k 10 120 python tools/gemm_bench.py --only conv --iters 10 > $O/conv_$t.log 2>&1 || { echo "FAILED $t"; tail -5 $O/conv_$t.log; continue; }
  echo "== $t"; grep -E "conv (32x32|8x8|16x16) [0-9]+->[0-9]+ s1 " $O/conv_$t.log
done
