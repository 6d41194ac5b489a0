#!/bin/bash
# Session-1 probe: new GEMM tiles / GN fold kernel tests, tile x split-K sweep, bench kernel trace (dispatch gaps),
# GN-fold same-box A/B of the metric bench. Each step under its own limit; stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s1
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "forced_tiles or gn_fold or single_launch or groupnorm or full_size" > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/tile_sweep.py --only conv --cfgs "0:0:0 3:0:1 3:0:2 3:0:4 3:0:8 1:3:1 1:3:2 1:3:4 4:0:1 4:0:2 4:0:4 4:0:8 7:2:1 7:2:2 7:2:4 7:3:2 7:3:4 8:2:1 8:2:2 8:2:4 2:2:1 2:2:2 2:2:4" > $O/sweep_conv.log 2>&1 || { echo FAIL conv; tail -20 $O/sweep_conv.log; exit 1; }
cut -c1-150 $O/sweep_conv.log
timeout -k 10 300 python tools/tile_sweep.py --only "linear|down|geglu" --cfgs "0:0:0 1:2:0 1:3:0 2:2:0 3:0:0 4:0:0 5:0:0 6:0:0 7:2:0 7:3:0 8:2:0 8:3:0" > $O/sweep_lin.log 2>&1 || { echo FAIL lin; tail -20 $O/sweep_lin.log; exit 1; }
cut -c1-150 $O/sweep_lin.log
timeout -k 10 300 python tools/micro_ab.py gn --tune "7=2" --tune "7=1" > $O/gn_ab.log 2>&1 || { echo FAIL gnab; tail -20 $O/gn_ab.log; exit 1; }
cat $O/gn_ab.log
for i in 1 2; do
  SDMOE_FUSED_GN=0 SDMOE_TUNE=7=2 timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/ab_gn0_$i.log 2>&1 || { echo FAIL ab0; tail -20 $O/ab_gn0_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/ab_gn1_$i.log 2>&1 || { echo FAIL ab1; tail -20 $O/ab_gn1_$i.log; exit 1; }
  echo "gn0 $(grep -a '^{' $O/ab_gn0_$i.log | cut -c1-160)"
  echo "gn1 $(grep -a '^{' $O/ab_gn1_$i.log | cut -c1-160)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 > $O/trace.log 2>&1 || { echo FAIL trace; tail -20 $O/trace.log; exit 1; }
cd $R
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python tools/trace_gaps.py $f
