#!/bin/bash
# attention variants (same box): parity tests, per-launch micro A/B (previous library vs current, sdmoe_tune knob 4
# values), metric bench A/B. usage: tools/gpu_attn_ab.sh ["tune1" "tune2" ...] (bench arms besides default)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn
P=$R/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k attention > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SDMOE_LIB=$P timeout -k 10 300 python tools/micro_ab.py attn > $O/micro_prev.log 2>&1 || { tail -20 $O/micro_prev.log; exit 1; }
echo "== previous library"; grep -v amdgpu.ids $O/micro_prev.log
timeout -k 10 300 python tools/micro_ab.py attn --tune "" ${MICRO_TUNES:---tune 4=8 --tune 4=16} > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
echo "== current"; grep -v amdgpu.ids $O/micro.log
BA="--steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-roofline"
for i in 1 2 3; do
  line=""
  SDMOE_LIB=$P timeout -k 10 300 python bench.py $BA > $O/bp_$i.log 2>&1 || { tail -20 $O/bp_$i.log; exit 1; }
  line="prev $(grep -a -o '"value": [0-9.]*' $O/bp_$i.log | cut -d' ' -f2)"
  timeout -k 10 300 python bench.py $BA > $O/b0_$i.log 2>&1 || { tail -20 $O/b0_$i.log; exit 1; }
  line="$line  cur $(grep -a -o '"value": [0-9.]*' $O/b0_$i.log | cut -d' ' -f2)"
  for t in "$@"; do
    SDMOE_TUNE=$t timeout -k 10 300 python bench.py $BA > $O/bt_$i.log 2>&1 || { tail -20 $O/bt_$i.log; exit 1; }
    line="$line  [$t] $(grep -a -o '"value": [0-9.]*' $O/bt_$i.log | cut -d' ' -f2)"
  done
  echo "$line"
done
