#!/bin/bash
# kernel breakdown of a short metric run + the full microbenchmark table (diagnosing a pipeline slowdown)
set -u
mkdir -p gpurun_out/r04p
timeout -k 10 300 python tools/gemm_bench.py --iters 10 > gpurun_out/r04p/gemm_bench.log 2>&1 || { echo "gemm_bench failed"; tail gpurun_out/r04p/gemm_bench.log; exit 1; }
cat gpurun_out/r04p/gemm_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04p/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/r04p/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r04p/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -a '^{' gpurun_out/r04p/prof.log | cut -c1-300
f=$(find gpurun_out/r04p/prof -name '*kernel_stats.csv' | head -1)
python tools/prof_summary.py $f 30
