#!/bin/bash
# SDXL parity tests on the current build, then the config-5 bench line + rocprof
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sdxl.py > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_measure.sh r04x sdxl prof_sdxl
