#!/bin/bash
# same-box: this build vs round-3 library (metric), halo on/off, SDXL (GELU table) and the GEGLU micro rows
set -u
mkdir -p gpurun_out/r04s
BA="--no-cpu-baseline --e2e-steps 0"
run() { local n=$1; shift; timeout -k 10 600 python bench.py "$@" $BA > gpurun_out/r04s/$n.log 2>&1 || { echo "FAILED $n"; tail -20 gpurun_out/r04s/$n.log; exit 1; }; echo "$n $(grep -a '^{' gpurun_out/r04s/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"] or {}; print(d["value"], d["ms_per_step"], r.get("achieved"), r.get("avg_launch_ms"))')"; }
run cur --steps 3 --warmup 1
SDMOE_LIB=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_r03.so run r03 --steps 3 --warmup 1
SDMOE_TUNE="16=0" run cur_nohalo --steps 3 --warmup 1
run cur2 --steps 3 --warmup 1
SDMOE_LIB=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_r03.so run r03_2 --steps 3 --warmup 1
SDMOE_TUNE="16=0" run cur_nohalo2 --steps 3 --warmup 1
run sdxl --model sdxl --steps 2 --warmup 1
SDMOE_LIB=$GRAFT_REPO_ROOT/diffusion-models-moe_amd/sdmoe/libsdmoe_hip_r03.so run sdxl_r03 --model sdxl --steps 2 --warmup 1
