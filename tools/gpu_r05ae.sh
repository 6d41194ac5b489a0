#!/bin/bash
# r05ae: 32-wide halo tiles for the Cin >= 1280 32x32 convs by default -- conv tests, per-launch conv A/B (prev =
# 6130b8b's library), metric check
set -u
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for n in 16 2; do
  timeout -k 10 300 python tools/micro_ab.py conv --nimg $n > $O/conv_cur$n.log 2>&1 || { tail $O/conv_cur$n.log; exit 1; }
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python tools/micro_ab.py conv --nimg $n > $O/conv_prev$n.log 2>&1 || { tail $O/conv_prev$n.log; exit 1; }
  paste -d'|' <(grep "conv 32x32" $O/conv_cur$n.log | cut -c1-60) <(grep "conv 32x32" $O/conv_prev$n.log | cut -c38-60)
done
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 $BA > $O/b8_cur$i.log 2>&1 || exit 1
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --steps 4 --warmup 1 $BA > $O/b8_prev$i.log 2>&1 || exit 1
  echo "b8 cur $(grep -a -o '"value": [0-9.]*' $O/b8_cur$i.log) prev $(grep -a -o '"value": [0-9.]*' $O/b8_prev$i.log)"
done
