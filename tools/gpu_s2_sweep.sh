#!/bin/bash
# stride-2 (downsampler) conv tile / split sweep: knob 1 (tile) x knob 9 (split-K)
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/s2; mkdir -p $O
for t in "16=1" "1=1" "1=2" "1=3" "1=4" "1=5" "1=7" "1=8" "1=7,9=8" "1=7,9=4" "1=3,9=4" "1=1,9=4" "1=2,9=4" "1=2,9=8"; do
  SDMOE_TUNE="$t" timeout -k 10 120 python tools/gemm_bench.py --only " s2" --iters 20 > "$O/c$t.log" 2>&1 || { echo "FAILED $t"; tail -3 "$O/c$t.log"; continue; }
  echo "$t $(grep -E 's2' "$O/c$t.log" | awk '{for(i=1;i<=NF;i++) if($i=="us") printf "%s:%s ", $2, $(i-1)}')"
done
