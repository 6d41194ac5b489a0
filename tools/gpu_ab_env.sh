# full GPU test suite, then a same-box A/B of one build under two environments: $AB_ENV (e.g. SDMOE_FUSED_GN=0) vs default
set -eu
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1 || { tail -40 gpurun_out/full_t.log; exit 1; }
tail -1 gpurun_out/full_t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 > gpurun_out/ab_cur.log 2>&1
  echo "cur  $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_cur.log)"
  env $AB_ENV timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --e2e-steps 0 > gpurun_out/ab_prev.log 2>&1
  echo "alt  $(grep -a -o '"value": [0-9.]*' gpurun_out/ab_prev.log)"
done
