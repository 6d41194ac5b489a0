# attention A/B: query fragments per wave 2 vs 4 (sdmoe_tune knob 4), parity tests first
set -eu
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "attention" > gpurun_out/a_test.log 2>&1 || { tail -30 gpurun_out/a_test.log; exit 1; }
tail -1 gpurun_out/a_test.log
for q in 2 4 0; do
  echo "== nqf $q"
  timeout -k 10 120 python tools/gemm_bench.py --only attn --nqf $q 2>&1 | grep -v amdgpu.ids
done
