#!/bin/bash
# GEGLU [v 2 | g 2] interleave: parity tests, geglu micro rows and pipeline vs the previous library (same box),
# GT on 256x320 tiles (knob 1 = 3) for SDXL
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r04il; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_route_parity.py tests/test_gpu_unet.py tests/test_gpu_kernels.py -k "geglu or fused or keep or gelu or route or pipeline or ln" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PREV=$GRAFT_REPO_ROOT/ab/libsdmoe_prev.so
for rep in 1 2; do
  timeout -k 10 120 python tools/gemm_bench.py --only geglu --iters 20 > $O/g_cur$rep.log 2>&1 && echo "cur  $(grep -E '^geglu-gemm M' $O/g_cur$rep.log | awk '{print $2, $5}' | tr '\n' ' ')"
  SDMOE_LIB=$PREV timeout -k 10 120 python tools/gemm_bench.py --only geglu --iters 20 > $O/g_prev$rep.log 2>&1 && echo "prev $(grep -E '^geglu-gemm M' $O/g_prev$rep.log | awk '{print $2, $5}' | tr '\n' ' ')"
done
BA="--no-cpu-baseline --e2e-steps 0 --no-roofline"
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" $BA > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -20 $O/$n.log; exit 1; }; echo "$n $(grep -a '^{' $O/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
run cur --steps 3 --warmup 1
SDMOE_LIB=$PREV run prev --steps 3 --warmup 1
run cur2 --steps 3 --warmup 1
SDMOE_LIB=$PREV run prev2 --steps 3 --warmup 1
run sdxl --model sdxl --steps 2 --warmup 1
SDMOE_TUNE="1=3" run sdxl_t3 --model sdxl --steps 2 --warmup 1
