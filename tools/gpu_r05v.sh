#!/bin/bash
# r05v: split-K / tile sweep of the VERDICT #5 projection shapes (micro_ab linear, warm L2)
set -u
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 400 python tools/micro_ab.py linear --iters 40 --tune "9=0" --tune "9=2" --tune "9=3" --tune "9=4" --tune "1=6" --tune "1=6,9=2" --tune "1=7" --tune "1=7,9=2" > $O/linear.log 2>&1 || { tail $O/linear.log; exit 1; }
grep linear $O/linear.log
