# auto vs forced 64x160 / 128x160 over every microbenchmark row (convs, linears, residual epilogues)
set -eu
mkdir -p gpurun_out
for t in 0 2 1; do
  timeout -k 10 300 python tools/gemm_bench.py --tile $t > gpurun_out/ta_$t.log 2>&1
done
paste -d'|' gpurun_out/ta_0.log gpurun_out/ta_2.log gpurun_out/ta_1.log | grep -v "amdgpu.ids" | cut -c1-220
