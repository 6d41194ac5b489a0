# run GPU tests matching $1 (pytest -k expression; default all)
set -eu
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/t.log | tail -40
