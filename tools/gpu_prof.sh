# kernel-trace profile of a short bench run -> gpurun_out/profq
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profq -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-roofline --inference-steps 10 --steps 1 --warmup 1 > $R/gpurun_out/profq.log 2>&1
tail -1 $R/gpurun_out/profq.log | cut -c1-200
cd $R && python tools/prof_summary.py $(find gpurun_out/profq -name '*kernel_stats.csv' | head -1) 40
