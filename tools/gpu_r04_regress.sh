#!/bin/bash
# same-box A/B: this build vs the round-3 library (libsdmoe_hip_r03.so) on the metric bench, then a kernel profile
set -u
mkdir -p gpurun_out/r04r
BA="--no-cpu-baseline --e2e-steps 0"
for lib in cur r03 cur r03; do
  if [ $lib = r03 ]; then export SDMOE_LIB=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_r03.so; else unset SDMOE_LIB; fi
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 $BA > gpurun_out/r04r/b8_$lib.log 2>&1 || { echo "FAILED $lib"; tail -20 gpurun_out/r04r/b8_$lib.log; exit 1; }
  echo "$lib $(grep -a '^{' gpurun_out/r04r/b8_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"])')"
done
unset SDMOE_LIB
nproc; cat /proc/loadavg
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04r/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-roofline $BA > $GRAFT_REPO_ROOT/gpurun_out/r04r/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04r/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -a '^{' gpurun_out/r04r/prof.log | cut -c1-200
f=$(find gpurun_out/r04r/prof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py $f 25
