#!/bin/bash
# quad top-k (FULL form) + GroupNorm finalize-and-apply: tests, timings, pipeline A/B (knob 17), metric bench line
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04q2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_route_parity.py tests/test_gpu_kernels.py -k "topk or keep or halo or groupnorm" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 0 4; do
  SDMOE_TUNE="15=$t" timeout -k 10 120 python tools/gemm_bench.py --only topk-keep --iters 20 > $O/topk_$t.log 2>&1 || { echo FAILED topk bench; tail -20 $O/topk_$t.log; exit 1; }
  echo "knob15=$t"; grep -i topk-keep $O/topk_$t.log
done
for g in 1 0 1 0; do
  SDMOE_TUNE="17=$g" timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-roofline --e2e-steps 0 > $O/ab_gn$g.log 2>&1 || { echo FAILED ab; tail -20 $O/ab_gn$g.log; exit 1; }
  echo "knob17=$g $(grep -a '^{' $O/ab_gn$g.log | tail -1 | cut -c1-150)"
done
