#!/bin/bash
# Full -m gpu suite on the GPU box (stop at the first failure), with the near-tie/flip parity report.
# usage: gpurun -- bash tools/gpu_tests.sh [pytest selection args]
set -u
mkdir -p gpurun_out
export SDMOE_PARITY_REPORT=gpurun_out/parity_report.json
timeout -k 10 1100 python -u -m pytest ${@:-tests} -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
tail -25 gpurun_out/gputests.log
exit $rc
