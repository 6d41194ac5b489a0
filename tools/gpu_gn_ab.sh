set -eu
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "groupnorm or gn or unet or vae or sdxl or clip" > gpurun_out/gn_t.log 2>&1 || { tail -40 gpurun_out/gn_t.log; exit 1; }
tail -1 gpurun_out/gn_t.log
bash tools/gpu_ab_lib.sh
