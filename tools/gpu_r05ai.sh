#!/bin/bash
# r05ai: 128-row halo tiles for the 16-wide / narrow 32-wide / 16->32 upsample convs at one prompt -- conv / GN
# tests, per-launch check, B = 1 A/B against the previous build (e8e4813) on one box, B = 8 check
set -u
O=gpurun_out/r05ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gn or conv or halo" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 > $O/conv_cur.log 2>&1 || { tail $O/conv_cur.log; exit 1; }
SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 > $O/conv_prev.log 2>&1 || { tail $O/conv_prev.log; exit 1; }
paste -d'|' <(grep conv $O/conv_cur.log | cut -c1-60) <(grep conv $O/conv_prev.log | cut -c38-60)
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 $BA > $O/b1_cur$i.log 2>&1 || exit 1
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 $BA > $O/b1_prev$i.log 2>&1 || exit 1
  echo "b1 cur $(grep -a -o '"value": [0-9.]*' $O/b1_cur$i.log) prev $(grep -a -o '"value": [0-9.]*' $O/b1_prev$i.log)"
done
timeout -k 10 300 python bench.py --steps 4 --warmup 1 $BA > $O/b8.log 2>&1 || exit 1
echo "b8 $(grep -a -o '"value": [0-9.]*' $O/b8.log)"
