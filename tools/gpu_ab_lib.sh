# A/B two builds of libsdmoe_hip.so on one box: the current one vs sdmoe/libsdmoe_hip_prev.so (SDMOE_LIB)
set -eu
mkdir -p gpurun_out
P=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_prev.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 > gpurun_out/ab_cur.log 2>&1
  echo "cur  $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_cur.log)"
  SDMOE_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 > gpurun_out/ab_prev.log 2>&1
  echo "prev $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_prev.log)"
done
