# full GPU check: all gpu tests, bench (with CPU baseline), kernel profile of a short bench
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/full_test.log 2>&1 || { tail -30 gpurun_out/full_test.log; exit 1; }
tail -1 gpurun_out/full_test.log
timeout -k 10 900 python bench.py --no-cpu-baseline > gpurun_out/full_bench.log 2>&1
tail -1 gpurun_out/full_bench.log | cut -c1-300
bash tools/gpu_prof.sh
