#!/bin/bash
# Round evidence on the GPU box, each step under its own limit, stopping at the first failure:
#   bench        the metric run (bench line with roofline + cpu_baseline)
#   union        --mask union (config 4)            sdxl       --model sdxl (config 5, GELU)
#   none         --mask none (config 2, MOEFy)       b1 / b1none  --batch 1 with / without the mask (configs 3 / 2 at
#                                                    the reference's one-prompt-per-call shape, base_receiver.py:73)
#   prof         rocprofv3 --kernel-trace --stats of the metric run (prof_union / prof_sdxl likewise)
#   pmc / pmc_b1 FETCH_SIZE / WRITE_SIZE passes of a 2-step metric run (8 / 1 prompts per GPU) ->
#                pmc_conv_traffic.json / pmc_conv_traffic_b1.json (bench.py picks the one of its --batch)
# usage: gpurun -- bash tools/gpu_measure.sh TAG STEP...   (default steps: bench union prof)
set -u
TAG=${1:-rXX}
shift
STEPS=${@:-bench union prof}
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
BA="--no-cpu-baseline --e2e-steps 0"
for s in $STEPS; do
  cd $R
  case $s in
    bench) step bench 600 python bench.py --steps 10 --warmup 2 ;;
    union) step bench_union 600 python bench.py --mask union --steps 5 --warmup 1 $BA ;;
    sdxl) step bench_sdxl 600 python bench.py --model sdxl --steps 2 --warmup 1 $BA ;;
    none) step bench_none 600 python bench.py --mask none --steps 5 --warmup 1 $BA ;;
    b1) step bench_b1 600 python bench.py --batch 1 --steps 10 --warmup 2 $BA ;;
    b1none) step bench_b1none 600 python bench.py --batch 1 --mask none --steps 10 --warmup 2 $BA ;;
    prof|prof_union|prof_sdxl|prof_none|prof_b1|prof_b1none)
      case $s in
        prof) args="--steps 5 --warmup 1" ;;
        prof_union) args="--mask union --steps 3 --warmup 1" ;;
        prof_sdxl) args="--model sdxl --steps 1 --warmup 1" ;;
        prof_none) args="--mask none --steps 3 --warmup 1" ;;
        prof_b1) args="--batch 1 --steps 5 --warmup 1" ;;
        prof_b1none) args="--batch 1 --mask none --steps 5 --warmup 1" ;;
      esac
      cd /tmp && export TMPDIR=/tmp
      step $s 600 rocprofv3 --kernel-trace --stats -d $O/$s -o run --output-format csv -- python3 $R/bench.py $args $BA
      cd $R
      f=$(find $O/$s -name '*kernel_stats.csv' 2>/dev/null | head -1)
      [ -n "$f" ] && python tools/prof_summary.py $f 45 > $O/${s}_summary.txt && cp $f $O/${s}_kernel_stats.csv && head -14 $O/${s}_summary.txt
      rm -rf $O/$s ;;  # the raw traces would push gpurun_out past the 64 MiB copy-back limit
    trace|trace_b1)  # one denoising step's dispatch sequence (durations, gaps, grids) -> ${s}_seq.txt
      [ $s = trace_b1 ] && bb="--batch 1" || bb=""
      cd /tmp && export TMPDIR=/tmp
      step $s 600 rocprofv3 --kernel-trace -d $O/$s -o run --output-format csv -- python3 $R/bench.py $bb --inference-steps 3 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0
      cd $R
      python tools/trace_seq.py $(find $O/$s -name '*kernel_trace.csv' | head -1) --out $O/${s}_seq.txt > /dev/null && head -3 $O/${s}_seq.txt
      rm -rf $O/$s ;;
    pmc|pmc_b1)  # FETCH_SIZE / WRITE_SIZE passes of the metric workload (pmc: 8 prompts/GPU; pmc_b1: one prompt)
      [ $s = pmc_b1 ] && { bb=1; sfx=_b1; } || { bb=8; sfx=; }
      cd /tmp && export TMPDIR=/tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c -d $O/${s}_$c -o run --output-format csv -- python3 $R/bench.py --batch $bb --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0 > $O/${s}_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
      done
      cd $R
      python tools/pmc_traffic.py $(find $O/${s}_FETCH_SIZE -name '*counter_collection.csv' | head -1) $(find $O/${s}_WRITE_SIZE -name '*counter_collection.csv' | head -1) --out $O/pmc_conv_traffic$sfx.json --build "$(cat $R/.build_rev 2>/dev/null)" --model sd14 --batch $bb --mask remove
      for c in FETCH_SIZE WRITE_SIZE; do gzip -c $(find $O/${s}_$c -name '*counter_collection.csv' | head -1) > $O/${s}_$c.csv.gz; rm -rf $O/${s}_$c; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
