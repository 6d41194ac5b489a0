#!/bin/bash
# r05al: one-prompt (2 images) routed GEGLU / LN-folded projection / keep-masked down projection tile sweep
set -u
O=gpurun_out/r05al; mkdir -p $O
timeout -k 10 400 python tools/micro_ab.py geglu --nimg 2 --iters 40 --tune "1=0" --tune "1=1" --tune "1=2" --tune "1=7" > $O/geglu2.log 2>&1 || { tail $O/geglu2.log; exit 1; }
grep -E "geglu|linear_ln" $O/geglu2.log
timeout -k 10 400 python tools/micro_ab.py keep --nimg 2 --iters 40 --tune "1=0" --tune "1=1" --tune "1=2" --tune "1=4" --tune "1=5" > $O/keep2.log 2>&1 || { tail $O/keep2.log; exit 1; }
grep keep $O/keep2.log
