#!/bin/bash
# Same-box A/B of the current library vs sdmoe/libsdmoe_hip_prev.so: parity tests ($TESTS, pytest args), per-launch
# micro rows of one family ($FAMILY, tools/micro_ab.py; $MICRO_TUNES adds sdmoe_tune arms), then the metric bench
# interleaved three times (plus one bench arm per positional argument, an SDMOE_TUNE string).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
P=$R/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
F=${FAMILY:-attn}
SDMOE_LIB=$P timeout -k 10 300 python tools/micro_ab.py $F > $O/micro_prev.log 2>&1 || { tail -20 $O/micro_prev.log; exit 1; }
echo "== previous library"; grep -v amdgpu.ids $O/micro_prev.log
timeout -k 10 300 python tools/micro_ab.py $F --tune "" ${MICRO_TUNES:-} > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
echo "== current"; grep -v amdgpu.ids $O/micro.log
BA="--steps 4 --warmup 1 --no-cpu-baseline --e2e-steps 0 --no-roofline"
for i in 1 2 3; do
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
