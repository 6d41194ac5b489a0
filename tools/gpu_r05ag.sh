#!/bin/bash
# r05ag: verification of the 128-row 64-wide halo default at one prompt -- conv / GroupNorm tests, smoke, B = 1 and
# B = 8 bench lines
set -u
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "gn or conv or halo" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
BA="--no-cpu-baseline --no-roofline --e2e-steps 0"
timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 $BA > $O/b1.log 2>&1 || exit 1
echo "b1 $(grep -a -o '"value": [0-9.]*' $O/b1.log)"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 $BA > $O/b8.log 2>&1 || exit 1
echo "b8 $(grep -a -o '"value": [0-9.]*' $O/b8.log)"
