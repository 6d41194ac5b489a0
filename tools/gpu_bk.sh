set -eu
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_route_parity.py -x -q -k fused > gpurun_out/bk_test.log 2>&1 || { tail -30 gpurun_out/bk_test.log; exit 1; }
tail -1 gpurun_out/bk_test.log
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/t0.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py --tile 5 > gpurun_out/t5.log 2>&1
timeout -k 10 300 python tools/gemm_bench.py --tile 3 > gpurun_out/t3.log 2>&1
paste gpurun_out/t0.log gpurun_out/t5.log gpurun_out/t3.log | grep -v amdgpu | grep -v attn | awk -F'\t' '{printf "%-60s | %-22s | %s\n", $1, substr($2,43), substr($3,43)}'
