# quick GPU check: kernel tests, microbench (auto tiles), bench without CPU baseline
set -eu
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/q_test.log 2>&1
tail -1 gpurun_out/q_test.log
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/q_gemm.log 2>&1
cat gpurun_out/q_gemm.log | grep -v amdgpu.ids
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/q_bench.log 2>&1
tail -1 gpurun_out/q_bench.log
