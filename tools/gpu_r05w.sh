#!/bin/bash
# r05w: latency-regime split for the 8x8 convs and the 16x16 -> 8x8 downsampler at one prompt per call -- conv tests,
# per-launch conv A/B at 2 images (prev = the r05z build), B = 1 and B = 8 bench A/B on one box
set -u
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 > $O/conv_cur.log 2>&1 || { tail $O/conv_cur.log; exit 1; }
SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python tools/micro_ab.py conv --nimg 2 > $O/conv_prev.log 2>&1 || { tail $O/conv_prev.log; exit 1; }
paste -d'|' <(grep conv $O/conv_cur.log | cut -c1-60) <(grep conv $O/conv_prev.log | cut -c38-60)
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_cur$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_prev$i SDMOE_AB=1 SDMOE_LIB=$P python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
run b8_cur python bench.py --steps 4 --warmup 1 $BA
run b8_prev SDMOE_AB=1 SDMOE_LIB=$P python bench.py --steps 4 --warmup 1 $BA
