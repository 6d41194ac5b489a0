set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python bench.py > gpurun_out/bench8.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/bench8.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof8 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench8p.log 2>&1; echo "prof exit $?"; tail -1 $R/gpurun_out/bench8p.log | cut -c1-300
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc8f -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmc8f.log 2>&1; echo "pmc fetch exit $?"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc8w -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmc8w.log 2>&1; echo "pmc write exit $?"
ls $R/gpurun_out/pmc8f $R/gpurun_out/pmc8w
