#!/bin/bash
# Round-end evidence on one box (two calls, each within gpurun's 20-minute limit), stopping at the first failure:
#   suite   full -m gpu suite with the parity report (tools/gpu_tests.sh)
#   measure tools/gpu_measure.sh (bench, union, sdxl, prof, pmc), PMC utilisation counters, per-op breakdown
# usage: gpurun -- bash tools/gpu_final.sh TAG suite|measure
set -u
TAG=${1:-rXX}
case ${2:-measure} in
  suite) bash tools/gpu_tests.sh ;;
  measure)
    bash tools/gpu_measure.sh $TAG bench union sdxl prof pmc || exit 1
    bash tools/gpu_pmc_util.sh $TAG > /dev/null || { echo "pmc util failed"; exit 1; }
    timeout -k 10 300 python tools/op_breakdown.py > gpurun_out/${TAG}_op_breakdown.txt 2>&1 || { echo "op breakdown failed"; exit 1; }
    head -12 gpurun_out/${TAG}_op_breakdown.txt ;;
esac
