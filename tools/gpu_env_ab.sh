#!/bin/bash
# Same-box A/B of two environment settings on the metric bench (interleaved, twice), after optional pytest files.
# usage: gpurun -- bash tools/gpu_env_ab.sh "ENV_A=.." "ENV_B=.." [pytest file ...]
set -u
mkdir -p gpurun_out/envab
O=gpurun_out/envab
A=$1; B=$2; shift 2
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for i in 1 2; do
  env $A timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
  echo "A [$A] $(grep -a -o '"value": [0-9.]*' $O/a.log)"
  env $B timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
  echo "B [$B] $(grep -a -o '"value": [0-9.]*' $O/b.log)"
done
