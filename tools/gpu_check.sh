# full GPU check: gpu tests, smoke, default bench (with CPU baseline), kernel-trace profile summary
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/c_test.log 2>&1 || { tail -40 gpurun_out/c_test.log; exit 1; }
tail -1 gpurun_out/c_test.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c_smoke.log 2>&1 || { tail -20 gpurun_out/c_smoke.log; exit 1; }
tail -1 gpurun_out/c_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/c_bench.log 2>&1 || { tail -20 gpurun_out/c_bench.log; exit 1; }
tail -1 gpurun_out/c_bench.log | cut -c1-400
bash tools/gpu_prof.sh 2>&1 | tail -45
