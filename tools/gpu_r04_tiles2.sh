#!/bin/bash
# 32x32-level conv tiles, same box, interleaved: default vs 256x320 (2x4), 256x160 (4x2), 256x320 (4x2)
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04t2; mkdir -p $O
for rep in 1 2; do
for t in "16=1" "1=6" "1=6,0=2" "1=3"; do
  SDMOE_TUNE="$t" timeout -k 10 120 python tools/gemm_bench.py --only "conv" --iters 20 > $O/conv_${t}_$rep.log 2>&1 || { echo "FAILED $t"; tail -5 $O/conv_${t}_$rep.log; continue; }
  echo "== $t"; grep -E "conv 32x32" $O/conv_${t}_$rep.log
done
done
