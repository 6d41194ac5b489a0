set -eu
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/tiles_test.log 2>&1
tail -2 gpurun_out/tiles_test.log
for t in 0 1 3 4; do
  timeout -k 10 300 python tools/gemm_bench.py --tile $t > gpurun_out/tiles_$t.log 2>&1
done
paste gpurun_out/tiles_0.log gpurun_out/tiles_3.log gpurun_out/tiles_4.log | cut -c1-220
