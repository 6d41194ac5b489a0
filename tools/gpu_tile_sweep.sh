#!/bin/bash
# GEMM tile x stage sweep of tools/gemm_bench.py rows matching $1 (egrep), every run under its own limit.
# usage: gpurun -- bash tools/gpu_tile_sweep.sh 'linear|down' "0:0 1:2 1:3 2:2 3:0 4:0 5:0" [extra gemm_bench args]
set -u
mkdir -p gpurun_out/sweep
PAT=${1:-linear}
CFGS=${2:-"0:0 1:2 1:3 2:2 2:3 3:0 4:0 5:0"}
EXTRA=${3:-}
for c in $CFGS; do
  t=${c%%:*}; s=${c##*:}
  timeout -k 10 300 python tools/gemm_bench.py --tile $t --stages $s $EXTRA > gpurun_out/sweep/t${t}s${s}.log 2>&1 \
    || { echo "FAILED tile $t stages $s"; tail -20 gpurun_out/sweep/t${t}s${s}.log; exit 1; }
done
for c in $CFGS; do
  t=${c%%:*}; s=${c##*:}
  echo "== tile $t stages $s"
  grep -E "$PAT" gpurun_out/sweep/t${t}s${s}.log
done
