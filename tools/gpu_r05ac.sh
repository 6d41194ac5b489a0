#!/bin/bash
# r05ac: tile / split sweep of the keep-masked FFN down projection at 16 images (micro_ab keep)
set -u
O=gpurun_out/r05ac; mkdir -p $O
timeout -k 10 400 python tools/micro_ab.py keep --iters 30 --tune "1=0" --tune "1=1" --tune "1=3" --tune "1=4" --tune "1=5" --tune "1=2" --tune "1=2,9=2" > $O/keep.log 2>&1 || { tail $O/keep.log; exit 1; }
grep keep $O/keep.log
