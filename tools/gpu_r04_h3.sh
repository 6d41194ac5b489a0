#!/bin/bash
# knob 16 = 3 (32-wide halo on 256-row tiles): halo parity tests, then conv rows under knobs 1 / 3 / 0
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04h3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "halo or groupnorm" > gpurun_out/r04h3/tests.log 2>&1 || { echo FAILED tests; tail -30 gpurun_out/r04h3/tests.log; exit 1; }
tail -2 gpurun_out/r04h3/tests.log
HALO_KNOBS="1 3 0" bash tools/gpu_r04_halo2.sh
