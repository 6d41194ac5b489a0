# forced-tile sweep of the GEMM microbenchmark (rows matching $1)
set -eu
mkdir -p gpurun_out
for t in 0 1 2 3 4 5; do
  timeout -k 10 300 python tools/gemm_bench.py --tile $t --only "${1:-}" > gpurun_out/tiles_$t.log 2>&1
done
paste gpurun_out/tiles_0.log gpurun_out/tiles_1.log gpurun_out/tiles_2.log | cut -c1-240
paste gpurun_out/tiles_3.log gpurun_out/tiles_4.log gpurun_out/tiles_5.log | cut -c1-240
