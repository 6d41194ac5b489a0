#!/bin/bash
# r05ah: 128-row halo tiles everywhere (knob 16 = 2) vs the default at one prompt (2 images), per launch
set -u
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 --iters 30 --tune "16=1" --tune "16=2" > $O/conv2.log 2>&1 || { tail $O/conv2.log; exit 1; }
grep conv $O/conv2.log
