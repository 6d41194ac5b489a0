#!/bin/bash
# Same-box A/B of the current libsdmoe_hip.so vs sdmoe/libsdmoe_hip_prev.so: tools/gemm_bench.py rows matching the
# egrep pattern $1 (both builds, twice, interleaved), then the metric bench twice each. Every step under its own limit.
set -u
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
PAT=${1:-.}
for i in 1 2; do
  timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/abr_cur$i.log 2>&1 || exit 1
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/abr_prev$i.log 2>&1 || exit 1
done
echo "row | cur1 us | prev1 | cur2 | prev2"
paste -d'|' <(grep -E "$PAT" gpurun_out/abr_cur1.log | cut -c1-56) <(grep -E "$PAT" gpurun_out/abr_prev1.log | awk '{print $(NF-3)}') \
  <(grep -E "$PAT" gpurun_out/abr_cur2.log | awk '{print $(NF-3)}') <(grep -E "$PAT" gpurun_out/abr_prev2.log | awk '{print $(NF-3)}')
[ "${2:-bench}" = "nobench" ] && exit 0
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/abr_bcur.log 2>&1 || exit 1
  echo "cur  $(grep -a -o '"value": [0-9.]*' gpurun_out/abr_bcur.log)"
  SDMOE_AB=1 SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 --steps 5 --warmup 1 > gpurun_out/abr_bprev.log 2>&1 || exit 1
  echo "prev $(grep -a -o '"value": [0-9.]*' gpurun_out/abr_bprev.log)"
done
