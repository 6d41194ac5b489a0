# HBM traffic of the conv launches: separate FETCH_SIZE / WRITE_SIZE passes over a 2-step bench, then the
# per-launch summary (tools/pmc_traffic.py) -> gpurun_out/pmc_conv_traffic.json
set -eu
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcf -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmcf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcw -o run --output-format csv -- python3 $R/bench.py --inference-steps 2 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline > $R/gpurun_out/pmcw.log 2>&1
cd $R
python tools/pmc_traffic.py $(find gpurun_out/pmcf -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmcw -name '*counter_collection.csv' | head -1) --out gpurun_out/pmc_conv_traffic.json
