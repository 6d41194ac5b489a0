# Round evidence in one GPU call: all GPU tests, the default bench line (with CPU baseline), a kernel-trace
# profile of the bench command, the two PMC traffic passes, and the per-op breakdown. Every step has its own
# time limit; the chain stops at the first failure.
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r1_test.log 2>&1 \
  || { tail -40 gpurun_out/r1_test.log; exit 1; }
tail -1 gpurun_out/r1_test.log
timeout -k 10 600 python bench.py > gpurun_out/r1_bench.log 2>&1 || { tail -20 gpurun_out/r1_bench.log; exit 1; }
tail -1 gpurun_out/r1_bench.log | cut -c1-400
timeout -k 10 300 python tools/op_breakdown.py > gpurun_out/r1_breakdown.log 2>&1 || { tail -20 gpurun_out/r1_breakdown.log; exit 1; }
head -12 gpurun_out/r1_breakdown.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --e2e-steps 0 > $R/gpurun_out/r1_prof_bench.log 2>&1
tail -1 $R/gpurun_out/r1_prof_bench.log | cut -c1-300
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r1_pmcf -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0 > $R/gpurun_out/r1_pmcf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r1_pmcw -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --e2e-steps 0 > $R/gpurun_out/r1_pmcw.log 2>&1
cd $R
python tools/prof_summary.py $(find gpurun_out/r1_prof -name '*kernel_stats.csv' | head -1) 40 > gpurun_out/r1_prof_summary.txt
head -20 gpurun_out/r1_prof_summary.txt
python tools/pmc_traffic.py $(find gpurun_out/r1_pmcf -name '*counter_collection.csv' | head -1) $(find gpurun_out/r1_pmcw -name '*counter_collection.csv' | head -1) --out gpurun_out/r1_pmc_conv_traffic.json
