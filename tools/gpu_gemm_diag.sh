#!/bin/bash
# time decomposition of the routed GEGLU and the K = 320 / 1280 projections by GEMM diagnostics (knob 6 bits):
# 0 full, 4 no epilogue, 8 epilogue without global stores, 2 no MFMA, 1 no K-loop loads (prologue stages only), 3, 6
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/gemm_diag; mkdir -p $O
for d in 0 4 8 2 1 3 6 0; do
  timeout -k 10 120 python tools/gemm_bench.py --diag $d --iters 20 > $O/d$d.log 2>&1 || { echo "FAILED $d"; tail -5 $O/d$d.log; continue; }
  echo "== diag $d"; grep -E "^(geglu-gemm |down-keep |linear M|linear+res M)" $O/d$d.log | head -14
done
