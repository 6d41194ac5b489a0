# MFMA / VALU / LDS utilisation counters: the 64x64 conv 320->320 (full, and with its epilogue off: diag 4), the fused
# routed GEGLU projection and the d=40 self-attention; one rocprofv3 --pmc pass per counter group, each under its
# own limit; stops at the first failure. usage: bash tools/gpu_pmc_util.sh TAG [WHAT:DIAG ...]  -> gpurun_out/TAG_pmc_util.txt
# (WHAT = kernel_micro.py kernel, DIAG = GEMM diagnostics bits: 1 = no K-loop loads, 4 = no epilogue; default
#  conv:0 conv:4 geglu:0 attn:0)
set -eu
TAG=${1:-r02}
shift || true
SPECS=${@:-conv:0 conv:4 geglu:0 attn:0}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for spec in $SPECS; do
  what=${spec%%:*}; dg=${spec##*:}; i=0
  for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/pmu_${what}${dg}_$i -o run --output-format csv -- python3 $R/tools/kernel_micro.py $what --iters 5 --diag $dg > $R/gpurun_out/pmu_${what}${dg}_$i.log 2>&1
  done
done
cd $R
O=gpurun_out/${TAG}_pmc_util.txt
{
echo "# rocprofv3 --pmc (3 passes per kernel, tools/gpu_pmc_util.sh, build $(cat .build_rev 2>/dev/null || echo ?)): per-dispatch averages"
echo "# conv = 64x64 320->320 3x3 at batch 16 (halo-tiled gemm_kernel MODE 9); diag 1 = no K-loop loads, diag 4 = no"
echo "# epilogue; geglu = fused routed GEGLU projection M=65536 F=1280 K=320; attn = d=40 self-attention 4096x4096, 16x8"
echo "# effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH DVFS note)"
for spec in $SPECS; do
  what=${spec%%:*}; dg=${spec##*:}
  case $what in attn) k=attn_fwd ;; *) k=gemm_kernel ;; esac
  echo "== $what, diag $dg"; python tools/pmc_dump.py "gpurun_out/pmu_${what}${dg}_" $k
done
} > $O
cat $O
