# forced-tile comparison of the GEMM microbenchmark on linear rows (auto, 128x160, 64x160, 256x160-8w)
set -eu
mkdir -p gpurun_out
for t in 0 1 2 4; do
  timeout -k 10 300 python tools/gemm_bench.py --tile $t --only "linear" > gpurun_out/tk_$t.log 2>&1
done
for t in 0 1 2 4; do echo "== tile $t"; cat gpurun_out/tk_$t.log; done
