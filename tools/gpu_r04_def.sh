#!/bin/bash
# Halo default change: kernel + U-Net + metric-parity tests, then the metric bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04def; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_unet.py tests/test_gpu_metric_parity.py > $O/tests.log 2>&1 || { echo FAILED tests; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { echo FAILED bench; tail -30 $O/bench.log; exit 1; }
grep -a '^{' $O/bench.log | tail -1 | cut -c1-900
