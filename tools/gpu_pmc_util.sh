# MFMA / VALU / LDS utilisation counters for the two dominant kernels (64x64 conv 320->320, d=40 self-attention),
# one rocprofv3 --pmc pass per counter group, each under its own limit; the script stops at the first failure
set -eu
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for what in conv attn; do
  i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/pmu_${what}$i -o run --output-format csv -- python3 $R/tools/kernel_micro.py $what --iters 5 > $R/gpurun_out/pmu_${what}$i.log 2>&1
  done
done
cd $R
echo "== conv (gemm_kernel MODE 1)"; python tools/pmc_dump.py gpurun_out/pmu_conv gemm_kernel
echo "== attention d=40"; python tools/pmc_dump.py gpurun_out/pmu_attn attn_fwd
