set -eu
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_unet.py -x -q -k fused > gpurun_out/f_test.log 2>&1 || { tail -30 gpurun_out/f_test.log; exit 1; }
tail -2 gpurun_out/f_test.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/f_bench.log 2>&1
tail -1 gpurun_out/f_bench.log | cut -c1-400
