#!/bin/bash
# GroupNorm statistics chunk width (knob 18) and the split path (knob 17): per-launch times at the bench shapes
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04gn2; mkdir -p $O
timeout -k 10 300 python tools/micro_ab.py gn --tune "18=80" --tune "18=40" --tune "18=16" --tune "17=1" --iters 50 > $O/gn.log 2>&1 || { echo FAILED; tail -20 $O/gn.log; exit 1; }
grep -v amdgpu.ids $O/gn.log
