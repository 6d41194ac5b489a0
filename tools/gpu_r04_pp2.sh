#!/bin/bash
# attention priority variants: tests, then d = 40 rows under knob 4 = 0 / 32 / 33 / 34
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04pp2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1 || { echo FAILED attn tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 32 33 34 0 34 33; do
  SDMOE_TUNE="4=$v" timeout -k 10 120 python tools/gemm_bench.py --only "d=40" --iters 10 > $O/attn_$v.log 2>&1 || { echo FAILED attn bench; tail -20 $O/attn_$v.log; exit 1; }
  echo "knob4=$v $(grep 'attn N=4096 d=40 Nk=4096' $O/attn_$v.log)"
done
