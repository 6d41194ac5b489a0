set -eu
mkdir -p gpurun_out
timeout -k 10 300 python tools/op_breakdown.py > gpurun_out/breakdown.log 2>&1 || { tail -30 gpurun_out/breakdown.log; exit 1; }
cat gpurun_out/breakdown.log
