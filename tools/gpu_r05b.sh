#!/bin/bash
# r05b: conv DMA placement A/B (cur vs prev lib), VALU issue-rate micro, conv diag decomposition
set -u
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 60 ./tools/micro/valu_rate > $O/valu_rate.txt 2>&1 || { cat $O/valu_rate.txt; exit 1; }
cat $O/valu_rate.txt
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only conv > $O/gb_cur$i.log 2>&1 || { tail $O/gb_cur$i.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py --only conv > $O/gb_prev$i.log 2>&1 || { tail $O/gb_prev$i.log; exit 1; }
done
paste -d'|' <(grep -E "us " $O/gb_cur1.log) <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3), $(NF-2)}') <(grep -E "us " $O/gb_cur2.log | awk '{print $(NF-3), $(NF-2)}') <(grep -E "us " $O/gb_prev2.log | awk '{print $(NF-3), $(NF-2)}')
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' $O/ab_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' $O/ab_prev.log)"
done
bash tools/gpu_conv_diag.sh
