#!/bin/bash
# LDS bank conflicts / instruction mix of the attention variants (one rocprofv3 --pmc pass per counter group and
# variant, each under its own limit) -> gpurun_out/attn_pmc.txt
set -eu
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for spec in ${ATTN_PMC_SPECS:-"40 4=0" "40 4=2" "64 4=0" "40 4=40"}; do
  set -- ${spec/:/ }
  d=$1; t=$2; tag=d${d}_${t/=/_}
  i=0
  for c in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/pma_${tag}_$i -o run --output-format csv -- python3 $R/tools/kernel_micro.py attn --iters 5 --d $d --tune $t > $R/gpurun_out/pma_${tag}_$i.log 2>&1
  done
done
cd $R
{
for spec in ${ATTN_PMC_SPECS:-"40 4=0" "40 4=2" "64 4=0" "40 4=40"}; do
  set -- ${spec/:/ }
  d=$1; t=$2; tag=d${d}_${t/=/_}
  echo "== attention d=$d N=4096 16 images x 8 heads, sdmoe_tune $t"; python tools/pmc_dump.py "gpurun_out/pma_${tag}_" attn
done
} > gpurun_out/attn_pmc.txt
cat gpurun_out/attn_pmc.txt
