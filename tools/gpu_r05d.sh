#!/bin/bash
# r05d: register-resident GEGLU epilogue + direct fp16 epilogue (knob 23) -- parity, then cur vs prev lib
set -u
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_route_parity.py tests/test_gpu_kernels.py -m gpu -x -q -k "geglu or route or gelu or fused or topk or keep" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SDMOE_TUNE=23=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "linear or conv or keep or masked or per_image or ln" --timeout 300 --timeout-method thread > $O/tests_direct.log 2>&1 || { tail -30 $O/tests_direct.log; exit 1; }
tail -2 $O/tests_direct.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py > $O/gb_cur$i.log 2>&1 || { tail $O/gb_cur$i.log; exit 1; }
  SDMOE_TUNE=23=1 timeout -k 10 200 python tools/gemm_bench.py > $O/gb_dir$i.log 2>&1 || { tail $O/gb_dir$i.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 200 python tools/gemm_bench.py > $O/gb_prev$i.log 2>&1 || { tail $O/gb_prev$i.log; exit 1; }
done
echo "cur | direct | prev | cur | direct | prev"
paste -d'|' <(grep -E "us " $O/gb_cur1.log | cut -c1-52) <(grep -E "us " $O/gb_dir1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev1.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_cur2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_dir2.log | awk '{print $(NF-3)}') <(grep -E "us " $O/gb_prev2.log | awk '{print $(NF-3)}')
for d in 4 8; do
  timeout -k 10 200 python tools/gemm_bench.py --only geglu --diag $d > $O/gb_d$d.log 2>&1 || { tail $O/gb_d$d.log; exit 1; }
  echo "diag $d"; grep -E "us " $O/gb_d$d.log
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_cur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' $O/ab_cur.log)"
  SDMOE_TUNE=23=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_dir.log 2>&1 || exit 1
  echo "dir  $(grep -a -o '"value": [0-9.]*' $O/ab_dir.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > $O/ab_prev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' $O/ab_prev.log)"
done
