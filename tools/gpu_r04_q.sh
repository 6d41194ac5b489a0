#!/bin/bash
# MFMA rate micro-benchmark, the quad top-k keep kernel's parity tests + its timing, then the knob-16 = 3 sweep
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 60 ./tools/micro/mfma_rate > $O/mfma_rate.log 2>&1 || { echo FAILED mfma; cat $O/mfma_rate.log; exit 1; }
cat $O/mfma_rate.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_route_parity.py -k "topk or keep" > $O/topk_tests.log 2>&1 || { echo FAILED topk tests; tail -30 $O/topk_tests.log; exit 1; }
tail -2 $O/topk_tests.log
for t in 0 4; do
  SDMOE_TUNE="15=$t" timeout -k 10 120 python tools/gemm_bench.py --only topk --iters 20 > $O/topk_$t.log 2>&1 || { echo FAILED topk bench; tail -20 $O/topk_$t.log; exit 1; }
  echo "knob15=$t"; grep -i topk $O/topk_$t.log
done
bash tools/gpu_r04_h3.sh
