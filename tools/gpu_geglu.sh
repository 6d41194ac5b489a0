set -eu
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_route_parity.py -x -q -k fused > gpurun_out/g_test.log 2>&1 || { tail -30 gpurun_out/g_test.log; exit 1; }
tail -1 gpurun_out/g_test.log
timeout -k 10 300 python tools/gemm_bench.py 2>&1 | grep -E 'geglu|topk|unfused'
