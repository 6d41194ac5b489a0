#!/bin/bash
# Round-4 check: GELU table + step-graph tests, then B=1 / B=8 bench with and without --graphs (same box).
set -u
mkdir -p gpurun_out/r04g
bash tools/gpu_tests.sh tests/test_gpu_graphs.py tests/test_gpu_route_parity.py tests/test_gpu_sdxl.py || exit 1
BA="--no-cpu-baseline --e2e-steps 0 --no-roofline"
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" $BA > gpurun_out/r04g/$n.log 2>&1 || { echo "FAILED $n"; tail -20 gpurun_out/r04g/$n.log; exit 1; }; grep -a '^{' gpurun_out/r04g/$n.log | cut -c1-200; }
run b1_eager --batch 1 --steps 6 --warmup 1
run b1_graphs --batch 1 --steps 6 --warmup 1 --graphs
run b8_eager --steps 3 --warmup 1
run b8_graphs --steps 3 --warmup 1 --graphs
run sdxl --model sdxl --steps 2 --warmup 1
# conv load-cost decomposition (diag bits: 16 = no A pieces, 32 = no B pieces, 1 = no loads at all)
for d in 0 16 32 1; do
  echo "== conv diag $d"
  timeout -k 10 300 python tools/gemm_bench.py --only conv --diag $d --iters 10 > gpurun_out/r04g/conv_diag$d.log 2>&1 || { echo "FAILED diag $d"; tail -5 gpurun_out/r04g/conv_diag$d.log; exit 1; }
  grep conv gpurun_out/r04g/conv_diag$d.log
done
