#!/bin/bash
# ping-pong attention (knob 4 = 32): attention tests, attention rows default vs 32, then the GN / top-k script
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04pp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1 || { echo FAILED attn tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 32 0 32; do
  SDMOE_TUNE="4=$v" timeout -k 10 120 python tools/gemm_bench.py --only attn --iters 10 > $O/attn_$v.log 2>&1 || { echo FAILED attn bench; tail -20 $O/attn_$v.log; exit 1; }
  echo "knob4=$v"; grep "attn N" $O/attn_$v.log
done
bash tools/gpu_r04_q2.sh
