#!/bin/bash
# r05e: direct fp16 epilogue (knob 23 default: no residual) + GEGLU register expert sums -- full gpu suite,
# A/B vs prev lib (DMA-late build), GEGLU rows, B = 1 split sweep
set -u
O=gpurun_out/r05e; mkdir -p $O
export SDMOE_PARITY_REPORT=$O/parity_report.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only geglu > $O/gb_cur$i.log 2>&1 || { tail $O/gb_cur$i.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py --only geglu > $O/gb_prev$i.log 2>&1 || { tail $O/gb_prev$i.log; exit 1; }
done
echo "cur | prev | cur | prev"
paste -d'|' <(grep -E "us " $O/gb_cur1.log | cut -c1-52) <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_cur2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev2.log | awk '{print $(NF-3)}')
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' $O/ab_cur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' $O/ab_prev.log)"
done
bash tools/gpu_b1_split_sweep.sh
