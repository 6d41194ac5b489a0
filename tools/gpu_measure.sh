#!/bin/bash
# One GPU call of round evidence, each step under its own limit, stopping at the first failure:
#   bench lines (default metric run; --mask union = config 4; optional SDXL = config 5) and a rocprofv3
#   --kernel-trace --stats profile of each. usage: gpurun -- bash tools/gpu_measure.sh TAG [sdxl] [pmc]
set -u
TAG=${1:-rXX}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
step() {  # step NAME SECONDS CMD...: run, keep the log, stop everything on failure
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED $name rc=$rc"; tail -30 $O/$name.log; exit $rc; fi
  grep -a '^{' $O/$name.log | tail -1 | cut -c1-600
}
cd $R
step bench 600 python bench.py --steps 10 --warmup 2
step bench_union 600 python bench.py --mask union --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0
if [ "${2:-}" = "sdxl" ]; then
  step bench_sdxl 600 python bench.py --model sdxl --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0
fi
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --e2e-steps 0
step prof_union 600 rocprofv3 --kernel-trace --stats -d $O/prof_union -o run --output-format csv -- python3 $R/bench.py --mask union --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0
if [ "${2:-}" = "sdxl" ]; then
  step prof_sdxl 600 rocprofv3 --kernel-trace --stats -d $O/prof_sdxl -o run --output-format csv -- python3 $R/bench.py --model sdxl --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 0
fi
if [ "${3:-}" = "pmc" ] || [ "${2:-}" = "pmc" ]; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0 > $O/pmcf.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0 > $O/pmcw.log 2>&1 || { echo "pmc write failed"; exit 1; }
fi
cd $R
for p in prof prof_union prof_sdxl; do
  f=$(find $O/$p -name '*kernel_stats.csv' 2>/dev/null | head -1)
  [ -n "$f" ] && python tools/prof_summary.py $f 45 > $O/${p}_summary.txt && head -14 $O/${p}_summary.txt
done
if [ -d $O/pmcf ]; then
  python tools/pmc_traffic.py $(find $O/pmcf -name '*counter_collection.csv' | head -1) $(find $O/pmcw -name '*counter_collection.csv' | head -1) --out $O/pmc_conv_traffic.json --build "$(cat $R/.build_rev 2>/dev/null)"
fi
exit 0
