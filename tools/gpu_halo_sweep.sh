#!/bin/bash
# conv rows under the halo knob settings (16 = 0 off, 1 default, 2 all 128-row tiles, 3 32-wide on 256-row tiles too)
set -u
mkdir -p gpurun_out/halo_sweep
for h in ${HALO_KNOBS:-1 3 0}; do
  echo "== halo knob $h"
  SDMOE_TUNE="16=$h" timeout -k 10 300 python tools/gemm_bench.py --only conv --iters 10 > gpurun_out/halo_sweep/conv_h$h.log 2>&1 || { echo "FAILED"; tail -5 gpurun_out/halo_sweep/conv_h$h.log; exit 1; }
  grep conv gpurun_out/halo_sweep/conv_h$h.log
done
