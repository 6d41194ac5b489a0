#!/bin/bash
# Selected -m gpu tests (stop at the first failure) with the parity report, e.g. the tests added this round.
# usage: gpurun -- bash tools/gpu_new_tests.sh LOGNAME test_file[::test] ...
set -u
mkdir -p gpurun_out
LOG=gpurun_out/$1.log; shift
export SDMOE_PARITY_REPORT=gpurun_out/parity_report_new.json
timeout -k 10 1100 python -u -m pytest "$@" -m gpu -x -v -s --durations=25 --timeout 600 --timeout-method thread \
  > $LOG 2>&1
rc=$?
tail -30 $LOG
exit $rc
