mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "pytest exit $?"
tail -30 gpurun_out/t2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1; echo "smoke exit $?"; tail -5 gpurun_out/smoke2.log
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench2.log 2>&1; echo "bench exit $?"; tail -5 gpurun_out/bench2.log
