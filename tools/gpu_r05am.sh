#!/bin/bash
# r05am: one-prompt tile rules for the routed GEGLU (M <= 1024) and the keep-masked down projection -- tests, B = 1 A/B against the previous build
# (1eead31) on one box, B = 8 check
set -u
O=gpurun_out/r05am; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "geglu or keep or route or linear" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 $BA > $O/b1_cur$i.log 2>&1 || exit 1
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 $BA > $O/b1_prev$i.log 2>&1 || exit 1
  echo "b1 cur $(grep -a -o '"value": [0-9.]*' $O/b1_cur$i.log) prev $(grep -a -o '"value": [0-9.]*' $O/b1_prev$i.log)"
done
timeout -k 10 300 python bench.py --steps 4 --warmup 1 $BA > $O/b8.log 2>&1 || exit 1
echo "b8 $(grep -a -o '"value": [0-9.]*' $O/b8.log)"
