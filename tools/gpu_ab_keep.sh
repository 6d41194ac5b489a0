# A/B in one box: top-k mask in the down projection vs a separate pass (bench twice each, interleaved)
set -eu
mkdir -p gpurun_out
for i in 1 2; do
  for m in down pass; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --topk-mask $m > gpurun_out/ab_$m.log 2>&1
    echo "$m $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_$m.log)"
  done
done
