set -eu
mkdir -p gpurun_out
timeout -k 10 120 python tools/attn_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "attention" > gpurun_out/a_test.log 2>&1 || { tail -30 gpurun_out/a_test.log; exit 1; }
tail -1 gpurun_out/a_test.log
timeout -k 10 300 python tools/gemm_bench.py --only attn 2>&1 | grep -v amdgpu.ids
