set -eu
mkdir -p gpurun_out
timeout -k 10 120 python tools/keep_debug.py
timeout -k 10 600 python -u -m pytest tests/test_gpu_route_parity.py tests/test_gpu_unet.py -x -q --timeout 300 --timeout-method thread -k "keep or fused or route or remove or moefy" > gpurun_out/k_test.log 2>&1 || { tail -40 gpurun_out/k_test.log; exit 1; }
tail -1 gpurun_out/k_test.log
timeout -k 10 200 python tools/gemm_bench.py --only "-" 2>&1 | grep -v amdgpu
bash tools/gpu_ab_keep.sh
