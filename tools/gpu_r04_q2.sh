#!/bin/bash
# quad top-k (FULL form) tests + timing, halo tests under every knob, metric bench line
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04q2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_route_parity.py tests/test_gpu_kernels.py -k "topk or keep or halo or groupnorm" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in 0 4; do
  SDMOE_TUNE="15=$t" timeout -k 10 120 python tools/gemm_bench.py --only topk --iters 20 > $O/topk_$t.log 2>&1 || { echo FAILED topk bench; tail -20 $O/topk_$t.log; exit 1; }
  echo "knob15=$t"; grep -i topk-keep $O/topk_$t.log
done
SDMOE_TUNE="16=1" timeout -k 10 120 python tools/gemm_bench.py --only up --iters 10 > $O/up.log 2>&1 && grep conv $O/up.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-steps 0 > $O/bench.log 2>&1 || { echo FAILED bench; tail -30 $O/bench.log; exit 1; }
grep -a '^{' $O/bench.log | tail -1 | cut -c1-400
