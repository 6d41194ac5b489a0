#!/bin/bash
# roofline event sampling A/B: every conv launch timed (--roofline-sample 1, the round-2 bench) vs every 10th U-Net
# evaluation (default) vs no roofline timing, interleaved twice on one box
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3
mkdir -p $O
cd $R
BA="--steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0"
for i in 1 2; do
  for arm in "s1:--roofline-sample 1" "s10:" "none:--no-roofline"; do
    n=${arm%%:*}; a=${arm#*:}
    timeout -k 10 300 python bench.py $BA $a > $O/ab_${n}_$i.log 2>&1 || { echo FAIL $n; tail -20 $O/ab_${n}_$i.log; exit 1; }
    echo "$n $(grep -a '^{' $O/ab_${n}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"] or {}; print(d["value"], d["ms_per_step"], r.get("achieved"), r.get("avg_launch_ms"), r.get("launches"), r.get("sampled"))')"
  done
done
