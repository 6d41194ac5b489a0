#!/bin/bash
# time decomposition of the conv family by GEMM diagnostics (knob 6 bits): 0 full, 4 no epilogue, 8 epilogue without
# global stores, 2 no MFMA, 1 no K-loop loads, 3 neither, 5 no loads no epilogue
# usage: bash tools/gpu_conv_diag.sh [gemm_bench --only filter, default "conv"]
set -u
ONLY=${1:-conv}
O=gpurun_out/conv_diag; mkdir -p $O
for d in 0 4 8 2 1 5 3 0; do
  timeout -k 10 120 python tools/gemm_bench.py --diag $d --iters 20 --only "$ONLY" > $O/d$d.log 2>&1 || { echo "FAILED $d"; tail -5 $O/d$d.log; exit 1; }
  echo "== diag $d"; grep -E "^conv" $O/d$d.log
done
