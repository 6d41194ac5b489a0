# kernel-trace profiles of the two top-k mask placements (short bench), summaries side by side
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in down pass; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pk_$m -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-roofline --inference-steps 10 --steps 1 --warmup 1 --topk-mask $m > $R/gpurun_out/pk_$m.log 2>&1
done
cd $R
for m in down pass; do
  echo "== $m"
  python tools/prof_summary.py $(find gpurun_out/pk_$m -name '*kernel_stats.csv' | head -1) 60 | grep -E "topk|gemm_kernel<[0-9]+, [0-9]+, [0-9]+, [0-9]+, [04],|total"
done
