# full GPU test suite, then the same-box library A/B (current vs sdmoe/libsdmoe_hip_prev.so)
set -eu
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_t.log 2>&1 || { tail -40 gpurun_out/full_t.log; exit 1; }
tail -1 gpurun_out/full_t.log
bash tools/gpu_ab_lib.sh
