#!/bin/bash
# conv_out on 128x32 tiles (knob 21): tests, conv rows, pipeline
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/narrow; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "narrow or conv3x3 or unet_forward" tests/test_gpu_unet.py > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 0 1 0; do
  SDMOE_TUNE="21=$k" timeout -k 10 120 python tools/gemm_bench.py --only "320->8" --iters 20 > $O/c$k.log 2>&1 || { echo FAILED; tail -3 $O/c$k.log; exit 1; }
  echo "21=$k $(grep '320->8' $O/c$k.log)"
done
