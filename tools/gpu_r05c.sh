#!/bin/bash
# r05c: halo-conv staggered wave groups -- conv parity subset, then cur (knob 22 = 1 / 0) vs prev lib A/B
set -u
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only conv > $O/gb_cur$i.log 2>&1 || { tail $O/gb_cur$i.log; exit 1; }
  SDMOE_TUNE=22=0 timeout -k 10 200 python tools/gemm_bench.py --only conv > $O/gb_lock$i.log 2>&1 || { tail $O/gb_lock$i.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py --only conv > $O/gb_prev$i.log 2>&1 || { tail $O/gb_prev$i.log; exit 1; }
done
echo "cur | lock | prev | cur | lock | prev"
paste -d'|' <(grep -E "us " $O/gb_cur1.log | cut -c1-52) <(grep -E "us " $O/gb_lock1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_cur2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_lock2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev2.log | awk '{print $(NF-3)}')
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' $O/ab_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' $O/ab_prev.log)"
done
