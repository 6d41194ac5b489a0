#!/bin/bash
# r05y: one-prompt (2 images) conv split sweep incl. the upsample convs, then the B = 1 dispatch trace
set -u
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 400 python tools/micro_ab.py conv --nimg 2 --iters 30 --tune "9=0" --tune "9=4" --tune "9=8" --tune "9=12" --tune "9=16" > $O/conv2.log 2>&1 || { tail $O/conv2.log; exit 1; }
grep conv $O/conv2.log
bash tools/gpu_measure.sh r05y trace_b1
