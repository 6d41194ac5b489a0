set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/t7.log 2>&1; echo "pytest exit $?"; tail -8 gpurun_out/t7.log
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gb7.log 2>&1; echo "gemm_bench exit $?"; grep attn gpurun_out/gb7.log
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench7.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/bench7.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof7 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --inference-steps 10 --no-cpu-baseline --no-roofline > $GRAFT_REPO_ROOT/gpurun_out/bench7p.log 2>&1; echo "prof exit $?"
