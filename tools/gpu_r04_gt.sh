#!/bin/bash
# table-GELU GEGLU on 256x320 tiles (knob 20): parity, micro rows, SDXL pipeline A/B
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04gt; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_route_parity.py -k "gelu" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 0 1 0 1; do
  SDMOE_TUNE="20=$k" timeout -k 10 120 python tools/geglu_gelu_bench.py --iters 20 > $O/g$k.log 2>&1 || { echo FAILED; tail -5 $O/g$k.log; exit 1; }
  echo "20=$k"; grep -v amdgpu $O/g$k.log
done
BA="--no-cpu-baseline --e2e-steps 0 --no-roofline"
for k in 0 1 0 1; do
  SDMOE_TUNE="20=$k" timeout -k 10 600 python bench.py --model sdxl --steps 2 --warmup 1 $BA > $O/sdxl$k.log 2>&1 || { echo FAILED sdxl; tail -20 $O/sdxl$k.log; exit 1; }
  echo "sdxl 20=$k $(grep -a '^{' $O/sdxl$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
