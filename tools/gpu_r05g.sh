#!/bin/bash
# r05g: late DMA only for 3-stage rings -- full gpu suite, then metric B = 8 / B = 1 and GEMM rows A/B vs prev
set -u
O=gpurun_out/r05g; mkdir -p $O
export SDMOE_PARITY_REPORT=$O/parity_report.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
timeout -k 10 200 python tools/gemm_bench.py > $O/gb_cur1.log 2>&1 || { tail $O/gb_cur1.log; exit 1; }
SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py > $O/gb_prev1.log 2>&1 || { tail $O/gb_prev1.log; exit 1; }
echo "cur | prev"
paste -d'|' <(grep -E "us " $O/gb_cur1.log | cut -c1-52) <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3)}') | head -60
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' $O/ab_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' $O/ab_prev.log)"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --batch 1 --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 4 --warmup 1 > $O/b1_cur.log 2>&1 || exit 1
  echo "b1 cur  $(grep -a -o '"value": [0-9.]*' $O/b1_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --batch 1 --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 4 --warmup 1 > $O/b1_prev.log 2>&1 || exit 1
  echo "b1 prev $(grep -a -o '"value": [0-9.]*' $O/b1_prev.log)"
done
