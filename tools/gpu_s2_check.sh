#!/bin/bash
# downsampler split-K default: conv tests, the s2 rows, 16x16 halo with 6 / 8 splits (knob 19), pipeline line
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/s2c; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "conv" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 0 6 8 0; do
  SDMOE_TUNE="19=$k" timeout -k 10 120 python tools/gemm_bench.py --only conv --iters 20 > $O/c$k.log 2>&1 || { echo FAILED; tail -3 $O/c$k.log; exit 1; }
  echo "19=$k $(grep -E 'conv (16x16 (1280|2560)->1280 s1 |.* s2)' $O/c$k.log | awk '{for(i=1;i<=NF;i++) if($i=="us") printf "%s/%s:%s ", $2, $3, $(i-1)}')"
done
timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-roofline > $O/b.log 2>&1 || { echo FAILED bench; tail -20 $O/b.log; exit 1; }
echo "bench $(grep -a '^{' $O/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
