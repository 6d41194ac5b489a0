#!/bin/bash
# r05f: direct fp16 epilogue (host-decided) + main-loop DMA after first reads + B = 1 split policy:
# kernel tests, gemm_bench A/B vs prev (round-5 DMA-late build), metric B = 8 and B = 1 A/B
set -u
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_route_parity.py tests/test_gpu_wanda.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py > $O/gb_cur$i.log 2>&1 || { tail $O/gb_cur$i.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py > $O/gb_prev$i.log 2>&1 || { tail $O/gb_prev$i.log; exit 1; }
done
echo "cur | prev | cur | prev"
paste -d'|' <(grep -E "us " $O/gb_cur1.log | cut -c1-52) <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_cur2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev2.log | awk '{print $(NF-3)}') | head -60
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
