# forced-tile comparison of the fused GEGLU GEMM rows (auto, 128x160, 256x320 2x4 waves, 256x160 8 waves)
set -eu
mkdir -p gpurun_out
for t in 0 1 3 4; do
  timeout -k 10 300 python tools/gemm_bench.py --tile $t --only "geglu" > gpurun_out/tg_$t.log 2>&1
done
for t in 0 1 3 4; do echo "== tile $t"; grep geglu gpurun_out/tg_$t.log; done
