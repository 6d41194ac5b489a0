#!/bin/bash
# same-box A/B: this round's final build vs the round-2 final build (git worktree r2tree at 24fb2ef)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abr2
mkdir -p $O
BA="--steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-roofline"
for i in 1 2 3; do
  cd $R && timeout -k 10 300 python bench.py $BA > $O/r3_$i.log 2>&1 || { echo FAIL r3; tail -20 $O/r3_$i.log; exit 1; }
  cd $R/r2tree && timeout -k 10 300 python bench.py $BA > $O/r2_$i.log 2>&1 || { echo FAIL r2; tail -20 $O/r2_$i.log; exit 1; }
  echo "round3 $(grep -a -o '"value": [0-9.]*' $O/r3_$i.log)  round2 $(grep -a -o '"value": [0-9.]*' $O/r2_$i.log)"
done
