# quick GPU check: kernel tests, microbench (auto tiles), bench without CPU baseline
set -eu
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q_test.log 2>&1 || { tail -30 gpurun_out/q_test.log; exit 1; }
tail -1 gpurun_out/q_test.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/q_bench.log 2>&1
tail -1 gpurun_out/q_bench.log | cut -c1-250
bash tools/gpu_prof.sh 2>&1 | grep -E "layernorm|gn_|total"
