#!/bin/bash
# r05aa: whole-round halo splits at one prompt -- conv tests, B = 1 A/B against the previous build, B = 8 check
# (the run recorded in profiles/r05_b1_policy_ab.txt also A/B'd a 4-stage 64x160 ring, knob 26, since removed)
set -u
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv" --timeout 300 --timeout-method thread > $O/tests_conv.log 2>&1 || { tail -30 $O/tests_conv.log; exit 1; }
tail -1 $O/tests_conv.log
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
run() {  # tag env...
  local tag=$1; shift
  timeout -k 10 300 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep -a -o '"value": [0-9.]*' $O/$tag.log)"
}
for i in 1 2; do
  run b1_prev$i SDMOE_AB=1 SDMOE_LIB=$P python bench.py --batch 1 --steps 10 --warmup 2 $BA
  run b1_cur$i python bench.py --batch 1 --steps 10 --warmup 2 $BA
done
run b8_cur python bench.py --steps 4 --warmup 1 $BA
