#!/bin/bash
# r05aj: one-prompt (2 images) linear shapes: tile (knob 1) / split (knob 9) sweep, us per launch incl. the reduce
set -u
O=gpurun_out/r05aj; mkdir -p $O
timeout -k 10 400 python tools/micro_ab.py linear --nimg 2 --iters 40 --tune "1=0" --tune "1=1" --tune "1=2" --tune "1=6" --tune "1=7" --tune "1=8" --tune "1=2,9=8" --tune "1=8,9=4" > $O/linear2.log 2>&1 || { tail $O/linear2.log; exit 1; }
grep linear $O/linear2.log
