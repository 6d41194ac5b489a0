# all GPU tests, then the A/B of the two top-k mask placements on the same box
set -eu
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f2_test.log 2>&1 || { tail -40 gpurun_out/f2_test.log; exit 1; }
tail -1 gpurun_out/f2_test.log
bash tools/gpu_ab_keep.sh
