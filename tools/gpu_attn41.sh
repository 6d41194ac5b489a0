#!/bin/bash
# attention with -m through a spare K column (knob 4 = 41) vs the 8-wave default: tests, d = 40 rows, pipeline
set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/a41; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1 || { echo FAILED tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 41 0 41; do
  SDMOE_TUNE="4=$v" timeout -k 10 120 python tools/gemm_bench.py --only "d=40" --iters 20 > $O/a$v.log 2>&1 || { echo FAILED; tail -3 $O/a$v.log; exit 1; }
  echo "4=$v $(grep 'attn N=4096 d=40 Nk=4096' $O/a$v.log)"
done
BA="--no-cpu-baseline --e2e-steps 0 --no-roofline"
for v in 0 41 0 41; do
  SDMOE_TUNE="4=$v" timeout -k 10 600 python bench.py --steps 3 --warmup 1 $BA > $O/b$v.log 2>&1 || { echo FAILED bench; tail -20 $O/b$v.log; exit 1; }
  echo "bench 4=$v $(grep -a '^{' $O/b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
