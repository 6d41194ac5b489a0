// MFMA GEMM / implicit-GEMM 3x3 convolution for gfx950, fp16 in / fp32 accumulate / fp16 out.
//
// One kernel template covers every dense projection of the SD U-Net step:
//   * Linear layers (attention q/k/v/out, proj_in/proj_out 1x1 convs, GEGLU proj, FFN down-proj, time MLP):
//     activations [M, K] row-major (any row stride), weights [N, K] (nn.Linear layout);
//   * ResNet 3x3 convolutions (stride 1/2, fused nearest-2x upsample) on NHWC activations: weights
//     [Cout][Cin/64][3][3][64] so K = 9*Cin is contiguous per output channel, every 64-wide K-step is one tap of
//     one 64-channel slice, and the 9 taps of a slice are consecutive K-steps (L2 reuse of the activation rows).
// Main loop: 256 threads = 2x2 waves, BK = 64, 16x16x32 f16 MFMA. Both operand tiles go HBM -> LDS with
// global_load_lds_dwordx4 (LDS-DMA, no register staging), one 1-KiB wave-instruction per 8 rows; conv halo
// rows and M/N tails point at a zero line. A 3-stage LDS ring keeps two K-steps in flight behind a counted
// `s_waitcnt vmcnt` and one raw s_barrier per K-step. The LDS image is XOR-swizzled by pre-swizzling the
// per-lane SOURCE chunk (LDS-DMA writes lane-linearly), so 16 consecutive rows read conflict-free.
// BN = 160 divides every SD channel count (320*k), so N = 320/640/1280/2560/... tiles exactly.
// Small grids (8x8 / 16x16 latents, K up to 23040) split K over workgroups: fp32 partial slabs + a
// deterministic ordered reduce kernel that also runs the epilogue.
// Epilogue (fused): + bias[n] + coladd[image][n] (time embedding) -> activation -> + residual[m][n],
// staged through LDS so stores are 16 B per lane.
#include <type_traits>

#include "common.h"
#include "../../include/sdmoe.h"

namespace {

constexpr int BK = 64;

// tuning knobs (sdmoe_tune): 0 = LDS stages (0 = auto, 2 or 3); 1 = forced tile config (0 = auto)
int g_stages = 0;
int g_tile = 0;
int g_res16 = 1;  // knob 8: 1 = residual epilogues on the fp16 staging path (residual added in the copy-out), 0 = fp32
int g_ksplit = 0;  // knob 9: forced split-K factor (0 = auto; 1 = never split), for tile sweeps
int g_mfast = 1;   // knob 14: split-K conv grids ordered M-tile fastest (1) or split fastest (0)
// knob 23: fp16 epilogues storing 16-B row pieces straight from the fragments (no LDS staging): 1 (default) = when
// there is no residual (LN-folded projections 4-12 %, plain K = 320 linears ~3 % faster; with a residual its 16-B
// residual loads measured 3-7 % slower than the staged copy-out), 2 = always, 0 = never
int g_epi_direct = 1;
int g_cus = 256;  // compute units of the device (device_cus(): hipDeviceAttributeMultiprocessorCount, queried once)
bool g_cus_init = false;
int g_diag = 0;  // knob 6, diagnostics only (results garbage): bit 0 = no K-loop operand loads, bit 1 = no MFMAs,
                 // bit 4 = no A-operand pieces, bit 5 = no B-operand pieces,
                 // bit 2 = no epilogue (nothing stored), bit 3 = epilogue without its global stores

typedef __attribute__((address_space(3))) void lds_void_t;


struct GemmParams {
  const half_t* A; long lda;
  const half_t* W; long ldw;
  const half_t* bias;
  const half_t* coladd; long coladd_bstride;
  const half_t* R; long ldr;
  half_t* C; long ldc;
  float* part;  // split-K partial slabs [ksplit][M][N] fp32 (ld N), or null
  int M, N, K;
  int act;
  int rows_per_batch;
  int H, Wd, Cin, OH, OW, stride, upsample;
  int ksplit, kchunk;
  int kchunk2;  // halo conv: folded-shortcut K-steps (32 channels of A2 each) per split (kchunk = main slices per split)
  int mfast;  // tile order M-fastest (split-K grids, sdmoe_tune knob 14)
  int a_bytes, w_bytes;  // SRD num_records
  // routed-GEGLU epilogue (sdmoe_linear_geglu): W rows interleaved [value 2 | gate 2] per neuron pair, C is
  // the [M, N/2] product value * act(gate); score [M, ld_score] gets per-expert sums of act(gate) over
  // contiguous esize-neuron experts (neurons pre-permuted so every expert is contiguous)
  half_t* score; long ld_score;
  int esize;
  int res16;  // residual on the fp16 staging path (sdmoe_tune knob 8)
  int diag;  // diagnostic knob (sdmoe_tune 6): bit 0 skips the K-loop loads, bit 1 the MFMAs
  int epi_direct;  // fp16 epilogue: stores straight from the fragments instead of LDS staging (knob 23 policy)
  // expert keep mask of the A operand (MODE_KEEP / MODE_KEEPW): keep[(k / 64) * M * 8 + m * 8 + (k % 64) / 8] bit
  // (k % 8) = neuron k of token m survives the top-k; the A fragments are ANDed with it after their LDS read
  const uint8_t* keep;
  int keep_bytes;
  // Wanda weight mask of the W operand (MODE_WMASK / MODE_KEEPW), the same K-step-major layout over W's rows:
  // wmask[(k / 64) * N * 8 + n * 8 + (k % 64) / 8] bit (k % 8) SET = W[n, k] removed (zeroed on the B fragments)
  const uint8_t* wmask;
  int wmask_bytes;
  // LayerNorm folded into the GEMM (MODE_GEMM_LN / MODE_GEGLU_LN): C = rstd_m * (A W'^T - mean_m * wsum) + ln_bias
  // with W' = W diag(gamma) (fp16), wsum[n] = sum_k W'[n, k], ln_bias[n] = bias[n] + sum_k W[n, k] beta[k] (fp32,
  // sdmoe_ln_fold); mean_m / rstd_m over the K = C channels of row m, accumulated from the A tiles in LDS
  const float* ln_wsum;
  const float* ln_bias;
  float ln_eps;
  // MODE_CONV with a folded 1x1 shortcut (sdmoe_conv3x3_sc): K-steps past the 9 * Cin conv steps read A2 [M, K2]
  // (the block input at the output pixel, row stride lda2) against the shortcut weights appended to W's rows
  const half_t* A2; long lda2;
  int a2_bytes;
  // GroupNorm folded into the GEMM (sdmoe_linear_per_image): image i = m / rows_per_batch multiplies its own weights
  // W + i * w_bstride (0 = one weight set) and adds colf[i * colf_bstride + n] (fp32 per-image column add)
  long w_bstride;
  const float* colf; long colf_bstride;
  // routed GEGLU with act == GELU: the registered fp16 GELU table (gelu_tab_h), staged into LDS for the epilogue
  const half_t* gelu_tab;
  // halo conv: GroupNorm(+SiLU) of the main input applied to each staged halo slice (sdmoe_conv3x3_gn): per image
  // and channel fp32 scale / shift ([nimg][Cin]); null = the input is used as is
  const float* gn_scale; const float* gn_shift; int gn_silu;
};

SDMOE_DEV int swz(int row) { return (row >> 1) & 7; }
SDMOE_DEV bool g_res16_dev(const GemmParams& p) { return p.res16 != 0; }

constexpr unsigned OOB = 0x80000000u;  // > every num_records used here (tensors < 2 GiB)

SDMOE_DEV void bld16(__amdgpu_buffer_rsrc_t rs, char* lds_dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 16, voff, soff, 0, 0);
}

// shared epilogue for one 8-column chunk: v += bias, coladd; act; + residual; store fp16
SDMOE_DEV void epilogue8(const GemmParams& p, int m, int n, float (&v)[8]) {
  if (p.bias) {
    half8 bb = *reinterpret_cast<const half8*>(p.bias + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += (float)bb[j];
  }
  if (p.coladd) {
    const int b = m / p.rows_per_batch;
    half8 cc = *reinterpret_cast<const half8*>(p.coladd + (long)b * p.coladd_bstride + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += (float)cc[j];
  }
  if (p.colf) {
    const float* cf = p.colf + (long)(m / p.rows_per_batch) * p.colf_bstride + n;
    const float4v c0 = *reinterpret_cast<const float4v*>(cf), c1 = *reinterpret_cast<const float4v*>(cf + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += c0[j]; v[4 + j] += c1[j]; }
  }
  if (p.act != ACT_NONE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j], p.act);
  }
  if (p.R) {
    half8 rr = *reinterpret_cast<const half8*>(p.R + (long)m * p.ldr + n);
    if (p.res16 && p.act == ACT_NONE) {
      // the fp16 staging path's order (knob 8): output rounded to fp16, residual added, rounded again -- so split-K
      // launches (this reduce) and unsplit ones give the same residual semantics for every shape
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)(half_t)v[j] + (float)rr[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)rr[j];
    }
  }
  half8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (half_t)v[j];
  if (p.diag & 8) {  // diagnostics: everything but the global store
    asm volatile("" ::"v"(o));
    return;
  }
  *reinterpret_cast<half8*>(p.C + (long)m * p.ldc + n) = o;
}

// GEGLU: GEMM loads, routed-GEGLU epilogue; KEEP: GEMM whose A operand is masked per (row, neuron) by keep bits;
// WMASK: W operand masked per (row, k) by Wanda bits; KEEPW: both (the routed FFN down projection under a Wanda mask)
// GEMM_LN / GEGLU_LN: GEMM / GEGLU with the LayerNorm of the A rows folded in (row statistics from the A tiles)
enum { MODE_GEMM = 0, MODE_CONV = 1, MODE_CONV_UP = 2, MODE_GEGLU = 3, MODE_KEEP = 4, MODE_WMASK = 5, MODE_KEEPW = 6,
       MODE_GEMM_LN = 7, MODE_GEGLU_LN = 8, MODE_CONVH64 = 9, MODE_CONVH32 = 10, MODE_CONVH16 = 11,
       MODE_CONVHUP64 = 12, MODE_CONVHUP32 = 13, MODE_CONVHUP16 = 14, MODE_GEGLU_GT = 15 };
// MODE_GEGLU_GT: the routed GEGLU with act = GELU from the registered table (its own instantiation: a third epilogue
// variant inside MODE_GEGLU pushed the 256x320 kernel past 256 VGPRs into scratch, 115 -> 494 us)
// halo-tiled stride-1 3x3 conv (MODE_CONVH<W>, image width W): a tile is BM / W whole output rows of one image; per
// 32-channel slice the (BM / W + 2) x (W + 2) input halo is staged in LDS ONCE and read by all 9 taps at shifted
// rows, instead of 9 shifted A tiles (A pieces per K-step 27/9 instead of BM / 16)
// MODE_CONVHUP<OW>: the same for the fused nearest-2x upsample conv (output width OW): the halo is the
// (BM / OW / 2 + 2) x (OW / 2 + 2) LOW-resolution input patch; output pixel (oh, ow) at tap (kh, kw) reads input
// ((oh + kh - 1) >> 1, (ow + kw - 1) >> 1) -- two lanes of a fragment share each input row (an LDS broadcast)
constexpr bool mode_halo(int mode) { return mode >= MODE_CONVH64 && mode <= MODE_CONVHUP16; }
constexpr bool mode_halo_up(int mode) { return mode >= MODE_CONVHUP64 && mode <= MODE_CONVHUP16; }
constexpr int halo_w(int mode) {  // OUTPUT width
  return (mode == MODE_CONVH64 || mode == MODE_CONVHUP64) ? 64 : ((mode == MODE_CONVH32 || mode == MODE_CONVHUP32) ? 32 : 16);
}
constexpr bool mode_akeep(int mode) { return mode == MODE_KEEP || mode == MODE_KEEPW; }
constexpr bool mode_wmask(int mode) { return mode == MODE_WMASK || mode == MODE_KEEPW; }

// LDS bytes one ring stage holds besides the A/B tiles: the mask bytes of the tile's rows for one 64-deep K-step
// (A keep: BM rows x 8 bytes; W mask: BN rows x 8 bytes; each in whole 1-KiB LDS-DMA pieces)
template <int BM, int MODE>
constexpr int keep_a_bytes() { return mode_akeep(MODE) ? ((BM * 8 + 1023) / 1024) * 1024 : 0; }
template <int BN, int MODE>
constexpr int keep_w_bytes() { return mode_wmask(MODE) ? ((BN * 8 + 1023) / 1024) * 1024 : 0; }
template <int BM, int BN, int MODE>
constexpr int keep_stage_bytes() { return keep_a_bytes<BM, MODE>() + keep_w_bytes<BN, MODE>(); }
// MODE_KEEP: a keep byte (8 neurons) -> 4 x 32-bit masks of the 8 fp16 halves, one ds_read_b128 per A fragment
// (round 5: two dependent ds_read_b64 from a 16-entry nibble table: keep-masked down projections 1.5-3 % slower);
// the W-masked modes keep the nibble table (the byte table there cost the 128x160 KEEPW tile its second workgroup
// per CU: 173 -> 268 VGPRs)
template <int MODE>
constexpr int keep_lut_bytes() { return MODE == MODE_KEEP ? 256 * 16 : 16 * 8; }

// Routed-GEGLU expert scores over one staged pass of a wave's tile: the activated gates (fp16) of RG rows x NH
// neurons, experts = contiguous S-neuron slices (neurons pre-permuted expert-major). score = fp32 sum in neuron order,
// rounded to fp16 (as sdmoe_geglu_route). Row-fastest lane mapping (lane -> row id % RG).
// acc + (float)h for the low / high fp16 half of x in ONE v_fma_mix_f32 (fma(h, 1.0, acc): the f16 -> f32 conversion
// is exact and the fma rounds once, so the result is bit-identical to cvt + add; the compiler folds fma(h, 1, acc)
// back into the two-instruction cvt + add)
SDMOE_DEV float add_f16_lo(float acc, unsigned x) {
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x));
  return acc;
}
SDMOE_DEV float add_f16_hi(float acc, unsigned x) {
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x));
  return acc;
}

template <int S, int NH, int RG>
SDMOE_DEV void expert_sums(const GemmParams& p, const half_t* sg, int mrow0, int n0, int lane) {
  constexpr int NE = NH / S;
  for (int id = lane; id < RG * NE; id += 64) {
    const int r = id % RG, e = id / RG;
    const int m = mrow0 + r;
    const half_t* rp = sg + r * NH + e * S;
    float acc = 0.f;
    if constexpr (S % 4 == 0) {  // 8-B aligned quads, summed in neuron order by mixed-precision fmas
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const u2 x = *reinterpret_cast<const u2*>(rp + 4 * q);
        acc = add_f16_hi(add_f16_lo(acc, x[0]), x[0]);
        acc = add_f16_hi(add_f16_lo(acc, x[1]), x[1]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < S; ++t) acc += (float)rp[t];
    }
    if (p.diag & 8) asm volatile("" ::"v"(acc));
    else if (m < p.M) p.score[(long)m * p.ld_score + n0 / 2 / S + e] = (half_t)acc;
  }
}

template <int BM, int BN, int WMW, int WNW, int MODE, int NSTAGE, int BKT>
__global__ __launch_bounds__(64 * WMW * WNW, (NSTAGE == 2 && (WMW * WNW == 4 || BM * BN <= 20480) ? 2 : 1)) void gemm_kernel(
    GemmParams p) {
  constexpr int BK = BKT;                        // K per stage: 64 (128-B rows) or 32 (64-B rows, deeper ring)
  constexpr int RB = BK * 2, CPRW = BK / 8;      // LDS row bytes, 16-B chunks per row
  constexpr int RPP = 1024 / RB;                 // rows per 1-KiB LDS-DMA piece
  auto swzk = [](int row) { return (row >> 1) & (CPRW - 1); };  // conflict-free b128 fragment reads
  constexpr bool CONV = MODE == MODE_CONV || MODE == MODE_CONV_UP;
  constexpr bool GEGLU = MODE == MODE_GEGLU || MODE == MODE_GEGLU_LN || MODE == MODE_GEGLU_GT;
  constexpr bool LN = MODE == MODE_GEMM_LN || MODE == MODE_GEGLU_LN;
  constexpr bool AKEEP = mode_akeep(MODE), WKEEP = mode_wmask(MODE);
  constexpr bool KEEP = AKEEP || WKEEP;
  static_assert(!KEEP || BKT == 64, "keep bytes are laid out per 64-deep K-step");
  constexpr int NW = WMW * WNW;                  // waves per workgroup
  constexpr int WM = BM / WMW, WN = BN / WNW;    // per-wave output tile
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16x16 fragments");
  constexpr int A_INS = BM / RPP, B_INS = BN / RPP;  // 1-KiB LDS-DMA wave-instructions per stage
  constexpr int A_PW = (A_INS + NW - 1) / NW, B_PW = (B_INS + NW - 1) / NW;
  constexpr int KA_INS = keep_a_bytes<BM, MODE>() / 1024;     // A keep pieces per stage
  constexpr int K_INS = keep_stage_bytes<BM, BN, MODE>() / 1024;  // A keep + W mask pieces per stage (<= NW)
  static_assert(K_INS <= NW, "one keep piece per wave at most");
  constexpr int K_PW = KEEP ? 1 : 0;             // every wave issues one (waves >= K_INS repeat piece 0)
  constexpr int PER_WAVE = A_PW + B_PW + K_PW;   // every wave issues exactly this many (surplus -> dummy slot)
  constexpr int STAGE_AB = (BM + BN) * BK * 2;
  constexpr bool PADDED = (A_PW * NW != A_INS) || (B_PW * NW != B_INS);
  constexpr int KEEP_OFF = STAGE_AB + (PADDED ? 1024 : 0);
  constexpr int WKEEP_OFF = KEEP_OFF + keep_a_bytes<BM, MODE>();
  constexpr int STAGE = KEEP_OFF + keep_stage_bytes<BM, BN, MODE>();
  // epilogue staging: fp16 final values (row stride RS16 halves: 16-B aligned rows, conflict-free b64 stores of the
  // swapped fragments) in NPASS16 passes; the fp32 path (activation, residual) in NPASS passes; GEGLU: its own passes
  // halo conv (MODE_CONVH*): two halo buffers of H_INS pieces (input rows BM / HW_ + 2 at a pitch of HW_ + 8 pixels: a
  // multiple of 8 rows, so a fragment's swizzle depends only on its lane and tap column) + an NSTAGE ring of B tiles
  constexpr bool HALO = mode_halo(MODE);
  constexpr bool HUP = mode_halo_up(MODE);
  constexpr int HW_ = halo_w(MODE), HWIN = HUP ? HW_ / 2 : HW_, HP = HWIN + 8, HR = BM / HW_;
  constexpr int HROWS_IN = HUP ? HR / 2 + 2 : HR + 2;  // input rows of the halo
  constexpr int H_INS = HALO ? (HROWS_IN * HP + RPP - 1) / RPP : 0;
  // a halo buffer also holds two A2 ring slots (BM rows x 32 channels) of the folded-shortcut K-steps
  constexpr int A2BYTES = BM * RB;
  constexpr int HBYTES = H_INS * 1024 > 2 * A2BYTES ? H_INS * 1024 : 2 * A2BYTES, BSTAGE = BN * RB;
  constexpr int RING = HALO ? 2 * HBYTES + NSTAGE * BSTAGE : NSTAGE * STAGE;  // main-loop LDS
  constexpr int GN_MAXC = 1280;                                   // halo conv GroupNorm: fp32 scale + shift per channel
  constexpr int RINGX = RING + (HALO && !HUP ? GN_MAXC * 8 : 0);
  constexpr int RS16 = WN + 8;
  constexpr int NPASS16 = (NW * WM * RS16 * 2 <= RING) ? 1 : (NW * (WM / 2) * RS16 * 2 <= RING) ? 2
                          : ((NW * (WM / 4) * RS16 * 2 <= RING) ? 4 : 8);
  constexpr int WN_PAD = WN + 4;
  constexpr int NPASS = (NW * (WM / 2) * WN_PAD * 4 <= RING) ? 2 : ((NW * (WM / 4) * WN_PAD * 4 <= RING) ? 4 : 8);
  static_assert(FM % NPASS == 0 && FM % NPASS16 == 0, "epilogue passes must split the wave's fragment rows");
  constexpr int EPI = NW * (WM / NPASS) * WN_PAD * 4;
  constexpr int EPI16 = NW * (WM / NPASS16) * RS16 * 2;
  constexpr int SMEM0 = (RINGX > EPI) ? (RINGX > EPI16 ? RINGX : EPI16) : (EPI > EPI16 ? EPI : EPI16);
  constexpr int LUT_OFF = SMEM0;                 // MODE_KEEP: 256-entry byte -> lane-mask table behind everything
  constexpr int SMEM1 = SMEM0 + (KEEP ? keep_lut_bytes<MODE>() : 0);
  // LN: per tile row (rstd, -mean*rstd), then the tile's BN columns of wsum and ln_bias (fp32), behind everything
  constexpr int LN_ROW_OFF = SMEM1, LN_COL_OFF = SMEM1 + BM * 8;
  constexpr int SMEM = SMEM1 + (LN ? BM * 8 + BN * 8 : 0);
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  constexpr int NT = 64 * NW;
  // LN row statistics: lane tid reads 16-B chunk (tid % 8) of tile rows tid / 8 + (NT / 8) t, t < LN_IPL, every
  // K-step (8 lanes cover one 128-B row: conflict-free), summing x and x^2 with v_dot2_f32_f16
  constexpr int LN_IPL = LN ? (BM * 8) / NT : 1;
  static_assert(!LN || ((BM * 8) % NT == 0 && BK == 64), "LN statistics: whole 16-B chunks per lane");
  float ln_s1[LN_IPL], ln_s2[LN_IPL];
#pragma unroll
  for (int t = 0; t < LN_IPL; ++t) ln_s1[t] = ln_s2[t] = 0.f;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WNW, wc = wave % WNW;
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, ntn * ntm * p.ksplit);
  // tile order: (split, N-tile, M-tile) with the split fastest, or -- split-K grids under mfast -- the M-tile
  // fastest, so the workgroups xcd_remap puts on one XCD share (N-tile, split) weight slices in that XCD's L2
  int split, tn, tm;
  if (p.mfast) {
    tm = bid % ntm;
    const int r = bid / ntm;
    tn = r % ntn;
    split = r / ntn;
  } else {
    split = bid % p.ksplit;
    const int tile = bid / p.ksplit;
    tn = tile % ntn;
    tm = tile / ntn;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_total = p.K / BK;
  const int ks0 = split * p.kchunk;
  const int ks1 = min(nk_total, ks0 + p.kchunk);
  const int nk = ks1 - ks0;

  // ---- LDS-DMA sources: buffer loads through two SRDs (A, W); an out-of-range offset (OOB) is dropped by the
  // hardware range check and lands as zeros, which gives conv halo rows and M/N tails for free.
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
  // per-image weights (sdmoe_linear_per_image): a tile never straddles two images (host check rows_per_batch % BM)
  const half_t* Wimg = p.w_bstride ? p.W + (long)(m0 / p.rows_per_batch) * p.w_bstride : p.W;
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)Wimg, (short)0, p.w_bytes, 0x00020000);
  const int lrow = lane / CPRW, lch = lane % CPRW;
  // A rows: wave w stages rows [8*(w*A_PW + j), +8); B rows likewise with B_PW
  unsigned avoff[A_PW];  // GEMM: byte offset of (row, pre-swizzled chunk); conv: of the centre-tap pixel
  unsigned amask[A_PW];  // conv: bit t = tap t in bounds (0 = M-tail row)
  int aoh[A_PW], aow[A_PW], ab_[A_PW];  // conv-upsample rows
  unsigned avoff2[A_PW];  // conv + shortcut: byte offset of (output pixel row, pre-swizzled chunk) in A2
  unsigned bvoff[B_PW];
#pragma unroll
  for (int j = 0; j < A_PW; ++j) {
    const int r = RPP * (j * NW + wave) + lrow;
    const unsigned chb = (unsigned)((lch ^ swzk(r)) * 16);
    const int m = m0 + r;
    avoff[j] = OOB; amask[j] = 0; aoh[j] = 0; aow[j] = 0; ab_[j] = 0; avoff2[j] = OOB;
    if (MODE == MODE_CONV && p.A2 && j * NW + wave < A_INS && m < p.M) avoff2[j] = (unsigned)((long)m * p.lda2 * 2) + chb;
    if (j * NW + wave < A_INS && m < p.M) {
      if (!CONV) {
        avoff[j] = (unsigned)((long)m * p.lda * 2) + chb;
      } else {
        const int hw = p.OH * p.OW;
        const int b = m / hw, rr = m - b * hw;
        const int oh = rr / p.OW, ow = rr - oh * p.OW;
        if (MODE == MODE_CONV) {
          const int ih = oh * p.stride, iw = ow * p.stride;  // centre tap (kh = kw = 1)
          avoff[j] = (unsigned)(((long)(b * p.H + ih) * p.Wd + iw) * p.lda * 2) + chb;
          unsigned msk = 0;
#pragma unroll
          for (int t = 0; t < 9; ++t) {
            const int y = ih + t / 3 - 1, x = iw + t % 3 - 1;
            msk |= (y >= 0 && y < p.H && x >= 0 && x < p.Wd) ? (1u << t) : 0u;
          }
          amask[j] = msk;
        } else {
          amask[j] = 1; avoff[j] = chb; aoh[j] = oh; aow[j] = ow; ab_[j] = b;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < B_PW; ++j) {
    const int r = RPP * (j * NW + wave) + lrow;
    const int n = n0 + r;
    bvoff[j] = (j * NW + wave < B_INS && n < p.N) ? (unsigned)((long)n * p.ldw * 2) + (unsigned)((lch ^ swzk(r)) * 16)
                                                  : OOB;
  }
  // mask pieces: wave w < KA_INS stages the A keep bytes of tile rows [128 w, 128 w + 128) (16 B = two rows per
  // lane), waves KA_INS .. K_INS-1 the W mask bytes of tile columns [128 (w - KA_INS), +128); the other waves
  // repeat piece 0 -- the same bytes to the same LDS place -- so every wave issues PER_WAVE instructions per stage
  // and the counted vmcnt waits stay uniform
  const int kpiece = KEEP && wave < K_INS ? wave : 0;
  const bool kpa = AKEEP && kpiece < KA_INS;  // wave-uniform: this wave's piece is A keep bytes (else W mask bytes)
  const __amdgpu_buffer_rsrc_t rsK = __builtin_amdgcn_make_buffer_rsrc(
      kpa ? (void*)p.keep : (void*)p.wmask, (short)0, KEEP ? (kpa ? p.keep_bytes : p.wmask_bytes) : 0, 0x00020000);
  const unsigned kstride = kpa ? (unsigned)p.M * 8u : (unsigned)p.N * 8u;  // bytes per K-step of the mask layout
  unsigned kvoff = OOB;
  int kdst = KEEP_OFF;
  if constexpr (KEEP) {
    kvoff = kpa ? (unsigned)((m0 + 128 * kpiece) * 8 + lane * 16)
                : (unsigned)((n0 + 128 * (kpiece - KA_INS)) * 8 + lane * 16);
    kdst = kpa ? KEEP_OFF + kpiece * 1024 : WKEEP_OFF + (kpiece - KA_INS) * 1024;
    // byte -> four 32-bit masks: entry e masks fp16 halves 0..7 by bits 0..7 of e (one ds_read_b128 per fragment;
    // round 5's 16-entry nibble table took two dependent ds_read_b64)
    if constexpr (MODE == MODE_KEEP) {
      for (int e = tid; e < 256; e += NT) {
        uint4v m;
#pragma unroll
        for (int d = 0; d < 4; ++d)
          m[d] = (((e >> (2 * d)) & 1) ? 0xFFFFu : 0u) | (((e >> (2 * d + 1)) & 1) ? 0xFFFF0000u : 0u);
        *reinterpret_cast<uint4v*>(smem + LUT_OFF + e * 16) = m;
      }
    } else if (tid < 16) {  // nibble -> two 32-bit masks
      const unsigned lo = ((tid & 1) ? 0xFFFFu : 0u) | ((tid & 2) ? 0xFFFF0000u : 0u);
      const unsigned hi = ((tid & 4) ? 0xFFFFu : 0u) | ((tid & 8) ? 0xFFFF0000u : 0u);
      *reinterpret_cast<uint2v*>(smem + LUT_OFF + tid * 8) = (uint2v){lo, hi};
    }
    __syncthreads();  // no LDS-DMA in flight yet
  }
  // LDS destination of wave-instruction j (surplus instructions of a padded tile land in a dummy 1-KiB slot)
  auto a_dst = [&](int j) { return (j * NW + wave < A_INS) ? (j * NW + wave) * 1024 : STAGE_AB; };
  auto b_dst = [&](int j) { return (j * NW + wave < B_INS) ? BM * BK * 2 + (j * NW + wave) * 1024 : STAGE_AB; };

  // conv K walk: (64-channel step, tap) advanced incrementally in scalar registers. Channel-step-major: the 9
  // consecutive K-steps of one 64-channel slice re-read the same activation rows (shifted by a tap), so a
  // workgroup's A working set is ~(BM + halo) x 128 B and stays in the XCD's L2 across the taps.
  // Folded shortcut (MODE_CONV, p.A2): channel steps st_c >= csl (= Cin / 64) are single K-steps of A2.
  const int csl = CONV ? p.Cin / BK : 0;
  const __amdgpu_buffer_rsrc_t rsA2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A2, (short)0, p.A2 ? p.a2_bytes : 0, 0x00020000);
  int st_c = CONV ? ks0 / 9 : 0, st_tap = CONV ? ks0 - st_c * 9 : 0;
  if (MODE == MODE_CONV && ks0 >= 9 * csl) { st_c = csl + (ks0 - 9 * csl); st_tap = 0; }

  auto issue_stage = [&](int ks, int buf) {
    char* sa = smem + buf * STAGE;
    const unsigned kb = (unsigned)(ks * BK * 2);
    if (p.diag & 16) {  // diagnostics: no A pieces (B only)
    } else if (!CONV) {
#pragma unroll
      for (int j = 0; j < A_PW; ++j) bld16(rsA, sa + a_dst(j), avoff[j], kb);
    } else if (MODE == MODE_CONV && st_c >= csl) {  // folded shortcut K-step (wave-uniform)
      const unsigned c2b = (unsigned)((st_c - csl) * BK * 2);
      ++st_c;
#pragma unroll
      for (int j = 0; j < A_PW; ++j) bld16(rsA2, sa + a_dst(j), avoff2[j] == OOB ? OOB : avoff2[j] + c2b, 0);
    } else {
      const int tap = st_tap;
      const int kh = tap >= 6 ? 2 : (tap >= 3 ? 1 : 0);
      const int kw = tap - 3 * kh;
      const int c0b = st_c * BK * 2;
      if (++st_tap == 9) { st_tap = 0; ++st_c; }
      if (MODE == MODE_CONV) {
        const unsigned tapoff = (unsigned)(((kh - 1) * p.Wd + (kw - 1)) * (int)p.lda * 2 + c0b);
#pragma unroll
        for (int j = 0; j < A_PW; ++j) {
          const unsigned vo = ((amask[j] >> tap) & 1u) ? avoff[j] + tapoff : OOB;
          bld16(rsA, sa + a_dst(j), vo, 0);
        }
      } else {
#pragma unroll
        for (int j = 0; j < A_PW; ++j) {
          const int uh = aoh[j] + kh - 1, uw = aow[j] + kw - 1;
          const bool ok = amask[j] && uh >= 0 && uh < 2 * p.H && uw >= 0 && uw < 2 * p.Wd;
          const unsigned vo =
              ok ? (unsigned)(((long)(ab_[j] * p.H + (uh >> 1)) * p.Wd + (uw >> 1)) * p.lda * 2) + avoff[j] + c0b
                 : OOB;
          bld16(rsA, sa + a_dst(j), vo, 0);
        }
      }
    }
    if (!(p.diag & 32)) {  // diagnostics: bit 5 = no B pieces (A only)
#pragma unroll
      for (int j = 0; j < B_PW; ++j) bld16(rsW, sa + b_dst(j), bvoff[j], kb);
    }
    if constexpr (KEEP) bld16(rsK, sa + kdst, kvoff, (unsigned)ks * kstride);
  };

  // routed GEGLU under GELU: the 32-KiB activation table goes to LDS by LDS-DMA (GELU_TAB_N / 512 pieces over the
  // waves) -- during the last K-step into the top of the ring stage nothing reads then (stage nk % NSTAGE: consumed
  // at step nk - NSTAGE, or never), when a stage holds it; otherwise after the main loop, behind the staging area
  constexpr int TAB_BYTES = GELU_TAB_N * 2;
  constexpr int G_STAGING = NW * 2 * (16 * (FM % 2 == 0 ? 2 : 1)) * (WN / 2) * 2 + NW * WN * 4;  // GEGLU epilogue
  constexpr bool TAB_PREFETCH = MODE == MODE_GEGLU_GT && STAGE >= TAB_BYTES && G_STAGING <= STAGE;
  constexpr int TAB_LATE_OFF = ((G_STAGING + 1023) / 1024) * 1024;
  constexpr bool TAB_OK = MODE == MODE_GEGLU_GT && (TAB_PREFETCH || TAB_LATE_OFF + TAB_BYTES <= SMEM1);
  static_assert(MODE != MODE_GEGLU_GT || TAB_OK, "GELU table must fit this tile's LDS");
  auto issue_gelu_tab = [&](char* dst) {
    const __amdgpu_buffer_rsrc_t rsT = __builtin_amdgcn_make_buffer_rsrc((void*)p.gelu_tab, (short)0, TAB_BYTES, 0x00020000);
#pragma unroll
    for (int j = 0; j < (TAB_BYTES / 1024 + NW - 1) / NW; ++j) {
      const int piece = j * NW + wave;
      if (piece < TAB_BYTES / 1024) bld16(rsT, dst + piece * 1024, (unsigned)(piece * 1024 + lane * 16), 0);
    }
  };

  // SWAP: C^T fragments (the MFMA's operands swapped): acc[i][j][r] = C[row wr*WM + 16 i + fr][col wc*WN + 16 j +
  // 4 fg + r], 4 consecutive output columns of one row per lane, so the epilogue works on half4 / float4 row pieces
  // (and the routed GEGLU pairs value / gate columns with one lane swap).
  constexpr bool SWAP = true;
  float4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  if constexpr (HALO) {
    // ---- halo-tiled 3x3 conv main loop. Local K-steps: 9 per main 32-channel slice (tap t; the 9 taps unrolled: kh,
    // kw compile-time), then the folded shortcut's K-steps (32 channels of A2 at the output pixel each). Per step: a
    // counted wait for the NEXT step's B tile (older pieces -- this step's A2 tile, the halos -- with it), one barrier,
    // the MFMAs on the fragments read ahead at the end of the previous step (the DMA issue of the step after its first
    // MFMA group: A2(ks + 2), B(ks + 3), at t = 0 the next slice's halo into the other buffer), then the next step's B
    // fragments and first A pair. Round 5 read every step's fragments right behind its barrier: PMC of the 64x64
    // 320 -> 320 conv with the K-loop loads and the epilogue off (profiles/r06b_pmc_conv.txt) put the MFMA pipe at 61 %
    // busy with 32 % of the wave cycles in s_waitcnt / s_barrier -- ~800 idle cycles per 1280-cycle K-step.
    // A2 ring slots: slot s = k2 % 3 lives in halo buffer (nsl + (s == 2)) % 2 at offset (s == 1) * A2BYTES: slots 0 / 1
    // are in the buffer the last main slice does not read (their loads are issued during its taps 7 / 8), slot 2 in the
    // other one (issued after the first shortcut step's barrier).
    static_assert(BK == 32 && NSTAGE == 4 && BM % HW_ == 0 && WM % HW_ == 0 && HW_ % 16 == 0 && FM % 2 == 0 &&
                      (!HUP || ((WM / HW_) % 2 == 0 && HR % 2 == 0)),
                  "halo conv tile");
    constexpr int HB_INS = BN / RPP, H_PW = (H_INS + NW - 1) / NW, BH_PW = (HB_INS + NW - 1) / NW;
    constexpr int A2_INS = BM / RPP, A2_PW = (A2_INS + NW - 1) / NW;
    const int h_cnt = H_INS / NW + (wave < H_INS % NW ? 1 : 0);
    const int b_cnt = HB_INS / NW + (wave < HB_INS % NW ? 1 : 0);
    const int a2_cnt = p.A2 ? A2_INS / NW + (wave < A2_INS % NW ? 1 : 0) : 0;
    const int pix = (HUP ? 2 * p.H : p.H) * HW_;  // output pixels per image
    const int bimg = m0 / pix, oh0 = (m0 - bimg * pix) / HW_;
    // B / A2 pieces j > 0 sit whole 128-row rounds below piece 0 (same swizzle): their offsets go to the scalar
    // offset (j x bstep / a2step), one VGPR per operand instead of one per piece -- the 256x320 tile has none spare
    unsigned hvo[H_PW], bvo0, a2vo0;
    const unsigned bstep = (unsigned)(NW * RPP * p.ldw * 2), a2step = (unsigned)(NW * RPP * p.lda2 * 2);
#pragma unroll
    for (int j = 0; j < H_PW; ++j) {
      const int row = (j * NW + wave) * RPP + lane / CPRW;
      const int r = row / HP, c = row - r * HP;
      const int ih = (HUP ? oh0 / 2 : oh0) - 1 + r, iw = c - 1;
      const bool ok = j * NW + wave < H_INS && ih >= 0 && ih < p.H && iw >= 0 && iw < HWIN;
      hvo[j] = ok ? (unsigned)(((long)(bimg * p.H + ih) * HWIN + iw) * p.lda * 2) + (unsigned)(((lane % CPRW) ^ swzk(row)) << 4)
                  : OOB;
    }
    static_assert(NW * RPP % 8 == 0, "a piece round keeps the row swizzle");
    {  // (N is a multiple of 320 and M of BM on the halo path: every issued piece is in range)
      const int row = wave * RPP + lane / CPRW;
      bvo0 = (unsigned)((long)(n0 + row) * p.ldw * 2) + (unsigned)(((lane % CPRW) ^ swzk(row)) << 4);
      a2vo0 = p.A2 ? (unsigned)((long)(m0 + row) * p.lda2 * 2) + (unsigned)(((lane % CPRW) ^ swzk(row)) << 4) : OOB;
    }
    char* const hbase = smem;
    char* const bbase = smem + 2 * HBYTES;
    // this split's main slices [c_first, c_first + nsl) and shortcut steps [k2_first, k2_first + n2)
    const int nsl_all = p.Cin / 32, n2_all = p.A2 ? (p.K - 9 * p.Cin) / 32 : 0;
    const int c_first = min(nsl_all, split * p.kchunk), nsl = min(nsl_all, c_first + p.kchunk) - c_first;
    const int k2_first = min(n2_all, split * p.kchunk2), n2 = min(n2_all, k2_first + p.kchunk2) - k2_first;
    const int nkl = 9 * nsl + n2;
    auto issue_halo = [&](int c32, int hb) {  // input channels 32 c32 .. +31 of the halo, into buffer hb
#pragma unroll
      for (int j = 0; j < H_PW; ++j)  // (whole rounds of pieces need no per-wave test)
        if ((j + 1) * NW <= H_INS || j * NW + wave < H_INS)
          bld16(rsA, hbase + hb * HBYTES + (j * NW + wave) * 1024, hvo[j], (unsigned)(c32 * 64));
    };
    // B tiles: a 4-slot ring (slot ks % 4), issued three local K-steps ahead; A2 tiles (folded shortcut): three slots
    // in the halo buffers (slot ks % 3), issued two steps ahead, ahead of the B tile issued at the same point
    auto issue_b_kb = [&](int ks, unsigned kb) {
#pragma unroll
      for (int j = 0; j < BH_PW; ++j)
        if ((j + 1) * NW <= HB_INS || j * NW + wave < HB_INS)
          bld16(rsW, bbase + (ks & 3) * BSTAGE + (j * NW + wave) * 1024, bvo0, kb + j * bstep);
    };
    // W columns of main slice c32 (global 32-channel slice) at tap: ((c32 / 2) * 9 + tap) * 64 + (c32 % 2) * 32; of
    // shortcut step k2 (local): 9 Cin + 32 (k2_first + k2)
    auto kb_main = [&](int c32, int tap) { return (unsigned)(((c32 >> 1) * 9 + tap) * 128 + (c32 & 1) * 64); };
    auto kb_sc = [&](int k2) { return (unsigned)(18 * p.Cin + 64 * (k2_first + k2)); };
    auto a2_slot = [&](int ks) -> char* {
      const int slot = ks % 3;
      return hbase + ((nsl + (slot == 2 ? 1 : 0)) & 1) * HBYTES + (slot == 1 ? A2BYTES : 0);
    };
    auto issue_a2 = [&](int ks) {
      char* const a2s = a2_slot(ks);
      const int k2 = k2_first + ks - 9 * nsl;
#pragma unroll
      for (int j = 0; j < A2_PW; ++j)
        if ((j + 1) * NW <= A2_INS || j * NW + wave < A2_INS)
          bld16(rsA2, a2s + (j * NW + wave) * 1024, a2vo0, (unsigned)(64 * k2) + j * a2step);
    };
    auto vm_wait = [&](int n) {  // s_waitcnt vmcnt(n) for the wave-uniform n (immediates only; smaller = safe)
      if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (n == 11) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
      else if (n == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (n == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      else if (n == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (n == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
      else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    // per-lane LDS byte offsets: A row fr of a halo fragment at tap column kw (swizzle of row fr + kw: the fragment's
    // first halo row is a multiple of 8), row fr of an aligned B / A2 fragment
    unsigned aoff[3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {  // upsample: lane fr reads input column offset (fr + kw + 1) >> 1
      const int rr = HUP ? (fr + kw + 1) >> 1 : fr + kw;
      aoff[kw] = (unsigned)((HUP ? rr : fr) * RB + ((fg ^ swzk(rr)) << 4));
    }
    const unsigned boff = (unsigned)(fr * RB + ((fg ^ swzk(fr)) << 4));
    const int orow_w = (wr * WM) / HW_;  // the wave's first output row within the tile
    // GroupNorm(+SiLU) of the main input (sdmoe_conv3x3_gn): this image's per-channel scale / shift go to LDS first;
    // every staged halo slice is then normalised in place -- slice c + 1 at tap 5 of slice c (its pieces are older
    // than that step's group, so landed; nobody reads its buffer before slice c + 1), the first one before its taps.
    // Thread tid always holds 16-B chunk position tid % 4 of halo rows tid / 4 + 128 k, i.e. data chunk
    // (tid % 4) ^ swzk(row) = (tid % 4) ^ ((tid >> 3) & 3): eight fixed channels. Out-of-image pixels stay zero (the
    // conv pads the NORMALISED tensor). Same arithmetic as gn_apply_kernel: the conv input is bit-identical.
    const bool gn = !HUP && p.gn_scale != nullptr;
    float* const gsc = reinterpret_cast<float*>(smem + RING);
    float* const gsh = gsc + GN_MAXC;
    if constexpr (!HUP) {
      if (gn) {
        for (int i = tid; i < p.Cin; i += NT) {
          gsc[i] = p.gn_scale[(long)bimg * p.Cin + i];
          gsh[i] = p.gn_shift[(long)bimg * p.Cin + i];
        }
        __syncthreads();
      }
    }
    auto transform = [&](int c32, int hb) {
      if constexpr (!HUP) {
        static_assert(NT == 512 && RB == 64, "transform mapping: 128 halo rows of 4 chunks per pass");
        const int q = tid & 3, ch0 = c32 * 32 + ((q ^ ((tid >> 3) & 3)) << 3);
        const float4v s0 = *reinterpret_cast<const float4v*>(gsc + ch0), s1 = *reinterpret_cast<const float4v*>(gsc + ch0 + 4);
        const float4v h0 = *reinterpret_cast<const float4v*>(gsh + ch0), h1 = *reinterpret_cast<const float4v*>(gsh + ch0 + 4);
        const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        const float sh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        char* const buf = hbase + hb * HBYTES + q * 16;
#pragma unroll
        for (int k = 0; k < (HROWS_IN * HP + 127) / 128; ++k) {
          const int row = (tid >> 2) + 128 * k;
          const int r = row / HP, c = row - r * HP;
          const int ih = oh0 - 1 + r, iw = c - 1;
          if (row < HROWS_IN * HP && ih >= 0 && ih < p.H && iw >= 0 && iw < HW_) {
            half8 v = *reinterpret_cast<const half8*>(buf + row * RB);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float f = (float)v[j] * sc[j] + sh[j];
              if (p.gn_silu) f = silu_f(f);
              v[j] = (half_t)f;
            }
            *reinterpret_cast<half8*>(buf + row * RB) = v;
          }
        }
      }
    };
    // Issue points: j = -3, -2, -1 in the prologue, j = s after step s's barrier; point j issues A2(j + 2) (a shortcut
    // step), then B(j + 3), then -- at tap 0 of a slice with a successor -- that successor's halo. Step s's B fragments
    // and first A pair are read AHEAD, at the end of step s - 1 (so step s's MFMAs start right behind its barrier instead
    // of behind a burst of LDS reads): the barrier at the start of step s therefore waits for B(s + 1) (and with it
    // every older piece: A2(s), the halos), issued at point s - 2. Main-slice steps keep the tap compile-time.
    auto is_sc = [&](int ks) { return ks >= 9 * nsl && ks < nkl; };
    auto issue_b_any = [&](int ks) {  // (prologue / shortcut steps: runtime tap)
      if (ks < 9 * nsl) issue_b_kb(ks, kb_main(c_first + ks / 9, ks % 9));
      else issue_b_kb(ks, kb_sc(ks - 9 * nsl));
    };
    half8 bcur[FN], a0, a1;
    auto read_b = [&](int ks) {  // B fragments of step ks (slot ks % 4)
      const char* sb = bbase + (ks & 3) * BSTAGE + wc * WN * RB;
#pragma unroll
      for (int j = 0; j < FN; ++j) bcur[j] = *reinterpret_cast<const half8*>(sb + boff + 16 * j * RB);
    };
    auto a_frag = [&](const char* hbuf, auto tc, int i) -> half8 {  // A fragment i at compile-time tap, halo buffer hbuf
      constexpr int t = decltype(tc)::value, kh = t / 3, kw = t % 3;
      const int i16 = 16 * i;
      if constexpr (HUP)  // input row ((orow + kh - 1) >> 1) - (oh0 / 2 - 1), column (ocol0 / 2) + lane part
        return *reinterpret_cast<const half8*>(hbuf + aoff[kw] + (((((i16 / HW_) + kh - 1) >> 1) + 1) * HP + (i16 % HW_) / 2) * RB);
      else
        return *reinterpret_cast<const half8*>(hbuf + aoff[kw] + ((i16 / HW_ + kh) * HP + (i16 % HW_) + kw) * RB);
    };
    const int hrow = (HUP ? orow_w / 2 : orow_w) * HP * RB;  // the wave's first halo row
    // the step's MFMAs on bcur / a0 a1 (already in registers); the rest of the A pairs read one group ahead; mid()
    // (the step's DMA issue) after the first group, so both waves of a SIMD have matrix work queued while it issues
    auto mfma_groups = [&](auto&& a_at, auto&& mid) {
#pragma unroll
      for (int g = 0; g < FM / 2; ++g) {
        half8 n0 = a0, n1 = a1;
        if (g + 1 < FM / 2) {
          n0 = a_at(2 * g + 2);
          n1 = a_at(2 * g + 3);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[2 * g][j] = mfma16x16x32(bcur[j], a0, acc[2 * g][j]);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[2 * g + 1][j] = mfma16x16x32(bcur[j], a1, acc[2 * g + 1][j]);
        __builtin_amdgcn_sched_barrier(0);
        if (g == 0) {
          asm volatile("" ::: "memory");
          mid();
          __builtin_amdgcn_sched_barrier(0);
        }
        a0 = n0;
        a1 = n1;
      }
    };
    // Every main slice but the last has a successor (MORE), so its taps' waits are compile-time counts; the last slice
    // and the shortcut steps count at run time. (The diagnostics knob stays a run-time test: a copy of the loop with it
    // compile-time off pushed the 256x320 tiles to 256 VGPRs + 188 B of scratch.) The compile-time waits
    // use the smallest per-wave piece counts (b_lo, h_lo): a wave holding one more piece waits for that piece too --
    // issued a full K-step earlier -- instead of walking a compare-and-branch chain for its exact count every step.
    constexpr int b_lo = HB_INS / NW, h_lo = H_INS / NW;
    auto main_loop = [&]() {
      const int diag = p.diag;
      if (nkl > 0) {
        if (nsl > 0) issue_halo(c_first, 0);
        if (!(diag & 1)) {  // points -3, -2, -1: B(0); A2(0), B(1); A2(1), B(2)
          issue_b_any(0);
          if (is_sc(0)) issue_a2(0);
          if (nkl > 1) issue_b_any(1);
          if (is_sc(1)) issue_a2(1);
          if (nkl > 2) issue_b_any(2);
        }
        // younger than B(0): A2(0), B(1), A2(1), B(2)
        const int w0 = (is_sc(0) ? a2_cnt : 0) + (nkl > 1 ? b_cnt : 0) + (is_sc(1) ? a2_cnt : 0) + (nkl > 2 ? b_cnt : 0);
        if (gn && nsl > 0) {  // the first slice's halo (the oldest load) landed, visible to all, normalised
          vm_wait(w0 + b_cnt);
          __syncthreads();
          transform(c_first, 0);
        }
        vm_wait(w0);
        __syncthreads();
        read_b(0);
        if (nsl > 0) {
          a0 = a_frag(hbase + hrow, std::integral_constant<int, 0>(), 0);
          a1 = a_frag(hbase + hrow, std::integral_constant<int, 0>(), 1);
        }
      }
      auto slice = [&](int cs, auto more_tag) {
        constexpr bool MORE = decltype(more_tag)::value;
        const char* const hcur = hbase + (cs & 1) * HBYTES + hrow;
        const char* const hnxt = hbase + ((cs & 1) ^ 1) * HBYTES + hrow;
        const int c32 = c_first + cs;
        auto tap_step = [&](auto tc) {
          constexpr int t = decltype(tc)::value;
          const int ks = cs * 9 + t;
          // younger than B(ks + 1): the halo issued at point ks - 2 (t == 2) and ks - 1 (t == 1), A2(ks + 1) (the
          // first shortcut step, t == 8 of the last slice), B(ks + 2)
          if constexpr (MORE) {
            vm_wait(b_lo + ((t == 1 || t == 2) ? h_lo : 0));
          } else if constexpr (t <= 6) {  // last slice: B(ks + 2) is a main-slice tile up to tap 6, nothing else younger
            vm_wait(b_lo);
          } else {
            int nwait = ks + 2 < nkl ? b_cnt : 0;
            if (t == 8 && n2 > 0) nwait += a2_cnt;
            vm_wait(ks + 1 < nkl ? nwait : 0);
          }
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          if constexpr (MORE && t == 5) {
            if (gn) transform(c32 + 1, (cs & 1) ^ 1);
          }
          auto mid = [&]() {
            if (diag & 1) return;
            if constexpr (!MORE) {
              if (t >= 7 && n2 > t - 7) issue_a2(ks + 2);  // A2 of shortcut step t - 7
            }
            if constexpr (t + 3 < 9) {
              issue_b_kb(ks + 3, kb_main(c32, t + 3));
            } else if constexpr (MORE) {
              issue_b_kb(ks + 3, kb_main(c32 + 1, t - 6));
            } else {
              if (n2 > t - 6) issue_b_kb(ks + 3, kb_sc(t - 6));
            }
            if constexpr (MORE && t == 0) issue_halo(c32 + 1, (cs & 1) ^ 1);
          };
          if (!(diag & 2)) mfma_groups([&](int i) -> half8 { return a_frag(hcur, tc, i); }, mid);
          else mid();
          // read-ahead of step ks + 1: tap t + 1, or tap 0 of the next slice, or (B only) the first shortcut step
          if constexpr (t < 8) {
            read_b(ks + 1);
            a0 = a_frag(hcur, std::integral_constant<int, t + 1>(), 0);
            a1 = a_frag(hcur, std::integral_constant<int, t + 1>(), 1);
          } else if constexpr (MORE) {
            read_b(ks + 1);
            a0 = a_frag(hnxt, std::integral_constant<int, 0>(), 0);
            a1 = a_frag(hnxt, std::integral_constant<int, 0>(), 1);
          } else {
            if (ks + 1 < nkl) read_b(ks + 1);
          }
        };
        tap_step(std::integral_constant<int, 0>());
        tap_step(std::integral_constant<int, 1>());
        tap_step(std::integral_constant<int, 2>());
        tap_step(std::integral_constant<int, 3>());
        tap_step(std::integral_constant<int, 4>());
        tap_step(std::integral_constant<int, 5>());
        tap_step(std::integral_constant<int, 6>());
        tap_step(std::integral_constant<int, 7>());
        tap_step(std::integral_constant<int, 8>());
      };
      for (int cs = 0; cs + 1 < nsl; ++cs) slice(cs, std::true_type());
      if (nsl > 0) slice(nsl - 1, std::false_type());
      for (int k2l = 0; k2l < n2; ++k2l) {  // folded shortcut K-steps: B read ahead, the A2 pair right behind the barrier
        const int ks = 9 * nsl + k2l;
        // younger than B(ks + 1): A2(ks + 1), B(ks + 2) -- compile-time counts but for the last two steps
        if (ks + 2 < nkl) vm_wait(A2_INS / NW + b_lo);
        else vm_wait(ks + 1 < nkl ? (is_sc(ks + 1) ? a2_cnt : 0) + (ks + 2 < nkl ? b_cnt : 0) : 0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        auto mid = [&]() {
          if (diag & 1) return;
          if (is_sc(ks + 2)) issue_a2(ks + 2);
          if (ks + 3 < nkl) issue_b_kb(ks + 3, kb_sc(k2l + 3));
        };
        const char* a2s = a2_slot(ks) + wr * WM * RB;
        auto a2_at = [&](int i) -> half8 { return *reinterpret_cast<const half8*>(a2s + boff + 16 * i * RB); };
        if (!(diag & 2)) {
          a0 = a2_at(0);
          a1 = a2_at(1);
          mfma_groups(a2_at, mid);
        } else {
          mid();
        }
        if (ks + 1 < nkl) read_b(ks + 1);
      }
    };
    main_loop();
  } else {
  // prologue: stages 0 .. NSTAGE-2
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) issue_stage(ks0 + s, s);

  for (int it = 0; it < nk; ++it) {
    // wait for this K-step's tile (leave the later ones in flight), then make every wave's DMA visible
    {
      const int ahead = min(NSTAGE - 2, nk - 1 - it);  // stages issued after this one (wave-uniform)
      if (NSTAGE >= 4 && ahead >= 2) {
        if (NSTAGE >= 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER_WAVE) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_WAVE) : "memory");
      } else if (NSTAGE >= 3 && ahead >= 1) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // the next stage's LDS-DMA (into the slot read in step it - 1, which every wave finished before the barrier).
    // 3-stage rings: issued after this step's first fragment reads, so its ~60 issue cycles per piece overlap their
    // LDS latency instead of delaying the first MFMA behind the barrier. 2-stage rings keep it right behind the
    // barrier: their stage has one K-step to land, and the later issue measured 2-5 % slower there (routed GEGLU,
    // 128x160 convs, K = 5120 projections; r05f)
    auto issue_next = [&]() {
      if (it + NSTAGE - 1 < nk && !(p.diag & 1)) issue_stage(ks0 + it + NSTAGE - 1, (it + NSTAGE - 1) % NSTAGE);
      else if (TAB_PREFETCH && it == nk - 1) issue_gelu_tab(smem + (nk % NSTAGE) * STAGE + STAGE - TAB_BYTES);
    };
    constexpr bool PIPE = !(KEEP && FN > 5);
    constexpr bool LATE_DMA = PIPE && NSTAGE >= 3;
    if (!LATE_DMA || (p.diag & 2)) issue_next();

    const char* sa = smem + (it % NSTAGE) * STAGE;
    const char* sbm = sa + BM * BK * 2;
    if (p.diag & 2) continue;
    // fragment reads (A masked by MoE keep bits, B by Wanda bits where the mode says so)
    // MODE_KEEP on the software-pipelined tiles: every A fragment's lane mask of the K-step looked up up front, right
    // behind the barrier (one ds_read_b64 of a fragment row's 8 keep bytes, then one ds_read_b128 per fragment), so the
    // fragment reads of the loop carry no dependent keep-byte -> table chain (it was exposed behind the 10-MFMA groups
    // of the 64x160 / 128x160 tiles: keep-masked 16x16-level down projection 49.9 vs 32.5 us plain, loads and epilogue
    // off)
    constexpr bool KPRE = MODE == MODE_KEEP && !(KEEP && FN > 5) && BK == 64 && FM <= 4;  // (FM = 8: +64 VGPRs, spills)
    uint4v kmask[KPRE ? 2 : 1][KPRE ? FM : 1];
    if constexpr (KPRE) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const uint2v kq = *reinterpret_cast<const uint2v*>(sa + KEEP_OFF + (wr * WM + i * 16 + fr) * 8);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          kmask[kk][i] = *reinterpret_cast<const uint4v*>(smem + LUT_OFF + ((kq[kk] >> (8 * fg)) & 255u) * 16);
      }
    }
    auto read_a = [&](int kk, int i) -> half8 {
      const int row = wr * WM + i * 16 + fr;
      half8 a = *reinterpret_cast<const half8*>(sa + row * RB + (((kk * 4 + fg) ^ swzk(row)) << 4));
      if constexpr (KPRE) {
        uint4v u = __builtin_bit_cast(uint4v, a);
        const uint4v mk = kmask[kk][i];
        u[0] &= mk[0]; u[1] &= mk[1]; u[2] &= mk[2]; u[3] &= mk[3];
        a = __builtin_bit_cast(half8, u);
      } else if constexpr (AKEEP) {  // zero the neurons of this row's dropped experts (8 neurons = chunk kk*4+fg)
        const unsigned kbyte = *reinterpret_cast<const unsigned char*>(sa + KEEP_OFF + row * 8 + kk * 4 + fg);
        uint4v u = __builtin_bit_cast(uint4v, a);
        if constexpr (MODE == MODE_KEEP) {  // byte table: one ds_read_b128 behind the keep byte
          const uint4v mk = *reinterpret_cast<const uint4v*>(smem + LUT_OFF + kbyte * 16);
          u[0] &= mk[0]; u[1] &= mk[1]; u[2] &= mk[2]; u[3] &= mk[3];
        } else {  // KEEPW: the nibble table (its wider reads cost the 128x160 tile its second workgroup per CU)
          const uint2v lo = *reinterpret_cast<const uint2v*>(smem + LUT_OFF + (kbyte & 15u) * 8);
          const uint2v hi = *reinterpret_cast<const uint2v*>(smem + LUT_OFF + (kbyte >> 4) * 8);
          u[0] &= lo[0]; u[1] &= lo[1]; u[2] &= hi[0]; u[3] &= hi[1];
        }
        a = __builtin_bit_cast(half8, u);
      }
      return a;
    };
    auto read_b = [&](int kk, int j) -> half8 {
      const int row = wc * WN + j * 16 + fr;
      half8 b = *reinterpret_cast<const half8*>(sbm + row * RB + (((kk * 4 + fg) ^ swzk(row)) << 4));
      if constexpr (WKEEP) {  // zero this W row's Wanda-masked weights (8 k = chunk kk*4+fg); mask bit SET = removed
        const unsigned mbyte = ~*reinterpret_cast<const unsigned char*>(sa + WKEEP_OFF + row * 8 + kk * 4 + fg);
        const uint2v lo = *reinterpret_cast<const uint2v*>(smem + LUT_OFF + (mbyte & 15u) * 8);
        const uint2v hi = *reinterpret_cast<const uint2v*>(smem + LUT_OFF + ((mbyte >> 4) & 15u) * 8);
        uint4v u = __builtin_bit_cast(uint4v, b);
        u[0] &= lo[0]; u[1] &= lo[1]; u[2] &= hi[0]; u[3] &= hi[1];
        b = __builtin_bit_cast(half8, u);
      }
      return b;
    };
    if constexpr (PIPE) {  // (wide masked tiles: no registers to spare)
      // software-pipelined: A fragments in pairs, the next pair's LDS reads issued before the current pair's
      // 2*FN MFMAs (one group of latency cover); the next kk's B fragments read during the last group when they
      // fit a second register set. sched_barrier pins the read / MFMA order so hipcc cannot sink the reads to
      // their first use (which exposes the LDS latency every group).
      constexpr int NKK = BK / 32, NG = FM / 2;
      static_assert(FM % 2 == 0, "the pipelined loop reads fragment rows in pairs");
      constexpr bool BDB = FN <= 5 && !KEEP;  // second B set: +4*FN VGPRs (the masked modes need those registers)
      half8 bcur[FN], bnxt[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bcur[j] = read_b(0, j);
      half8 a0 = read_a(0, 0), a1 = read_a(0, 1);
      if constexpr (LATE_DMA) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
        issue_next();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          half8 n0 = a0, n1 = a1;
          if (g + 1 < NG) {
            n0 = read_a(kk, 2 * g + 2);
            n1 = read_a(kk, 2 * g + 3);
          } else if (kk + 1 < NKK) {
            if constexpr (BDB) {
#pragma unroll
              for (int j = 0; j < FN; ++j) bnxt[j] = read_b(kk + 1, j);
            }
            n0 = read_a(kk + 1, 0);
            n1 = read_a(kk + 1, 1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[2 * g][j] = SWAP ? mfma16x16x32(bcur[j], a0, acc[2 * g][j]) : mfma16x16x32(a0, bcur[j], acc[2 * g][j]);
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[2 * g + 1][j] = SWAP ? mfma16x16x32(bcur[j], a1, acc[2 * g + 1][j])
                                     : mfma16x16x32(a1, bcur[j], acc[2 * g + 1][j]);
          __builtin_amdgcn_sched_barrier(0);
          a0 = n0;
          a1 = n1;
        }
        if (kk + 1 < NKK) {
#pragma unroll
          for (int j = 0; j < FN; ++j) bcur[j] = BDB ? bnxt[j] : read_b(kk + 1, j);
        }
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        half8 af[FM], bf[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = read_a(kk, i);
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[j] = read_b(kk, j);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = SWAP ? mfma16x16x32(bf[j], af[i], acc[i][j]) : mfma16x16x32(af[i], bf[j], acc[i][j]);
      }
    }
    if constexpr (LN) {
      typedef _Float16 h2 __attribute__((ext_vector_type(2)));
      const h2 one2 = {(half_t)1.f, (half_t)1.f};
#pragma unroll
      for (int t = 0; t < LN_IPL; ++t) {
        const int row = tid / 8 + (NT / 8) * t, ch = tid & 7;
        const half8 x = *reinterpret_cast<const half8*>(sa + row * RB + ((ch ^ swzk(row)) << 4));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const h2 x2 = {x[2 * q], x[2 * q + 1]};
          ln_s1[t] = __builtin_amdgcn_fdot2(x2, one2, ln_s1[t], false);
          ln_s2[t] = __builtin_amdgcn_fdot2(x2, x2, ln_s2[t], false);
        }
      }
    }
  }
  }  // !HALO

  // ---- epilogue
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (p.diag & 4) {  // diagnostics: keep the accumulators live, store nothing
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  const int mw = m0 + wr * WM, nw = n0 + wc * WN;  // this wave's output tile origin
  if (SWAP && p.part) {  // split-K: fp32 partial slab [split][M][N], 16-B stores straight from the accumulators
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int m = mw + 16 * i + fr, n = nw + 16 * j + 4 * fg;
        if (m < p.M && n < p.N) *reinterpret_cast<float4v*>(p.part + ((long)split * p.M + m) * p.N + n) = acc[i][j];
      }
    return;
  }
  float* ln_row = reinterpret_cast<float*>(smem + LN_ROW_OFF);  // [BM][2]: rstd, -mean * rstd
  float* ln_col = reinterpret_cast<float*>(smem + LN_COL_OFF);  // [BN] wsum, then [BN] ln_bias
  if constexpr (LN) {
#pragma unroll
    for (int t = 0; t < LN_IPL; ++t) {
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) {
        ln_s1[t] += __shfl_xor(ln_s1[t], o, 64);
        ln_s2[t] += __shfl_xor(ln_s2[t], o, 64);
      }
      if ((tid & 7) == 0) {
        const int row = tid / 8 + (NT / 8) * t;
        const float mean = ln_s1[t] / (float)p.K;
        const float var = fmaxf(ln_s2[t] / (float)p.K - mean * mean, 0.f);
        const float rstd = rsqrtf(var + p.ln_eps);
        ln_row[2 * row] = rstd;
        ln_row[2 * row + 1] = -mean * rstd;
      }
    }
    for (int c = tid; c < BN; c += NT) {
      const bool ok = n0 + c < p.N;
      ln_col[c] = ok ? p.ln_wsum[n0 + c] : 0.f;
      ln_col[BN + c] = ok ? p.ln_bias[n0 + c] : 0.f;
    }
  }
  __syncthreads();
  constexpr int CPR = WN / 8;
  if (!GEGLU && p.act == ACT_NONE && (!p.R || g_res16_dev(p))) {
    // fp16 path: bias and per-image column add in registers on each lane's 4-column row piece (one rounding, as
    // epilogue8), staged as fp16 (one ds_write_b64 per fragment: 1/2.5 of the LDS time of staging fp32 with 4
    // ds_write_b32), then copied out in 16-B row chunks: 175 -> 166 us for the M = 65536, N = 2560, K = 320 linear,
    // 1-3 % on the convs. Measured slower and therefore not used: residual loads in registers (8-B pieces of 16
    // rows: 29 -> 33 us for linear+res at 64x64) and the GEGLU epilogue on fp16 staging (170 -> 179 us); an
    // activation's code keeps the unrolled fragment loop from unrolling (acc then lives in scratch).
    half4 b4[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nw + 16 * j + 4 * fg;
      b4[j] = (!LN && p.bias && n < p.N) ? *reinterpret_cast<const half4*>(p.bias + n) : (half4){0, 0, 0, 0};
    }
    if (!WKEEP && p.epi_direct) {  // (the Wanda-masked tiles: no registers to spare for it)
      // Direct fp16 stores, no LDS staging (sdmoe_tune knob 23): per fragment row and pair of fragments (j, j + 1)
      // two v_permlane16_swap per lane leave each lane 8 consecutive output columns of its row -- lane group g:
      // fragment j + (g & 1), columns 8 (g >> 1) .. +7 -- stored as one 16-B piece (the T21 widening on the 16x16
      // fragment layout); an unpaired last fragment stores 8 B per lane. Residual: loaded in the same layout and added
      // to the fp16-rounded output in fp16 arithmetic, as the staged path.
      const bool res = p.R != nullptr;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        const int m = mw + 16 * i + fr;
        const half_t* cap = (p.coladd && m < p.M) ? p.coladd + (long)(m / p.rows_per_batch) * p.coladd_bstride : nullptr;
        const float* cfp = (p.colf && m < p.M) ? p.colf + (long)(m / p.rows_per_batch) * p.colf_bstride : nullptr;
        float a = 0.f, c = 0.f;
        if constexpr (LN) {
          const int rl = wr * WM + 16 * i + fr;
          a = ln_row[2 * rl];
          c = ln_row[2 * rl + 1];
        }
        auto frag16 = [&](int j) -> uint2v {  // fragment j of row block i: + bias / column adds (/ LN), rounded
          const int n = nw + 16 * j + 4 * fg;
          float4v v = acc[i][j];
          if constexpr (LN) {
            const int cl = wc * WN + 16 * j + 4 * fg;
            const float4v ws = *reinterpret_cast<const float4v*>(ln_col + cl);
            const float4v lb = *reinterpret_cast<const float4v*>(ln_col + BN + cl);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(a, v[r], __builtin_fmaf(c, ws[r], lb[r]));
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)b4[j][r];
          if (cap && n < p.N) {
            const half4 cc = *reinterpret_cast<const half4*>(cap + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (float)cc[r];
          }
          if (cfp && n < p.N) {
            const float4v cc = *reinterpret_cast<const float4v*>(cfp + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += cc[r];
          }
          half4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = (half_t)v[r];
          return __builtin_bit_cast(uint2v, y);
        };
#pragma unroll
        for (int j = 0; j + 1 < FN; j += 2) {
          const uint2v ya = frag16(j), yb = frag16(j + 1);
          const auto s0 = __builtin_amdgcn_permlane16_swap(ya[0], yb[0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(ya[1], yb[1], false, false);
          const int n = nw + 16 * (j + (fg & 1)) + 8 * (fg >> 1);
          half8 o = __builtin_bit_cast(half8, (uint4v){s0[0], s1[0], s0[1], s1[1]});
          if (m < p.M && n < p.N) {
            if (res) {
              const half8 rr = *reinterpret_cast<const half8*>(p.R + (long)m * p.ldr + n);
#pragma unroll
              for (int r = 0; r < 8; ++r) o[r] = (half_t)((float)o[r] + (float)rr[r]);
            }
            if (p.diag & 8) asm volatile("" ::"v"(o));
            else *reinterpret_cast<half8*>(p.C + (long)m * p.ldc + n) = o;
          }
        }
        if constexpr (FN % 2) {
          const int n = nw + 16 * (FN - 1) + 4 * fg;
          half4 o = __builtin_bit_cast(half4, frag16(FN - 1));
          if (m < p.M && n < p.N) {
            if (res) {
              const half4 rr = *reinterpret_cast<const half4*>(p.R + (long)m * p.ldr + n);
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] = (half_t)((float)o[r] + (float)rr[r]);
            }
            if (p.diag & 8) asm volatile("" ::"v"(o));
            else *reinterpret_cast<half4*>(p.C + (long)m * p.ldc + n) = o;
          }
        }
      }
      return;
    }
    half_t* st = reinterpret_cast<half_t*>(smem) + wave * (WM / NPASS16) * RS16;
    // residual (fp16, 16-B row chunks): this pass's chunks are loaded before its accumulators are staged, so their
    // latency hides behind the staging; added to the staged fp16 output in the copy-out (the output is rounded to
    // fp16 and the residual added in fp16 arithmetic -- diffusers' fp16 `to_out(x) + hidden_states`)
    constexpr int NCH16 = (WM / NPASS16) * CPR, NIT16 = (NCH16 + 63) / 64;
    const bool res = p.R != nullptr;
#pragma unroll
    for (int h = 0; h < NPASS16; ++h) {
      half8 rr[NIT16];
      if (res) {
#pragma unroll
        for (int it = 0; it < NIT16; ++it) {
          const int id = lane + 64 * it;
          const int r = id / CPR, c8 = id - r * CPR;
          const int m = mw + h * (WM / NPASS16) + r, n = nw + c8 * 8;
          rr[it] = (id < NCH16 && m < p.M && n < p.N) ? *reinterpret_cast<const half8*>(p.R + (long)m * p.ldr + n)
                                                      : (half8){0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int i = 0; i < FM / NPASS16; ++i) {
        // one fragment row at a time: keeps the hoisted bias / column-add / residual loads to FN pieces (the 8-wave
        // 256x320 tiles hold 160 accumulator VGPRs here and spilled when the compiler hoisted all of them)
        __builtin_amdgcn_sched_barrier(0);
        const int m = mw + 16 * (h * (FM / NPASS16) + i) + fr;
        const half_t* cap = (p.coladd && m < p.M) ? p.coladd + (long)(m / p.rows_per_batch) * p.coladd_bstride : nullptr;
        const float* cfp = (p.colf && m < p.M) ? p.colf + (long)(m / p.rows_per_batch) * p.colf_bstride : nullptr;
        float a = 0.f, c = 0.f;  // LN: this lane's row (rstd, -mean * rstd), read once per fragment row
        if constexpr (LN) {
          const int rl = wr * WM + 16 * (h * (FM / NPASS16) + i) + fr;
          a = ln_row[2 * rl];
          c = ln_row[2 * rl + 1];
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = nw + 16 * j + 4 * fg;
          float4v v = acc[h * (FM / NPASS16) + i][j];
          if constexpr (LN) {  // rstd * (acc - mean * wsum) + ln_bias
            const int cl = wc * WN + 16 * j + 4 * fg;
            const float4v ws = *reinterpret_cast<const float4v*>(ln_col + cl);
            const float4v lb = *reinterpret_cast<const float4v*>(ln_col + BN + cl);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(a, v[r], __builtin_fmaf(c, ws[r], lb[r]));
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)b4[j][r];
          if (cap && n < p.N) {
            const half4 c = *reinterpret_cast<const half4*>(cap + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += (float)c[r];
          }
          if (cfp && n < p.N) {
            const float4v c = *reinterpret_cast<const float4v*>(cfp + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += c[r];
          }
          half4 y;
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = (half_t)v[r];
          *reinterpret_cast<half4*>(st + (16 * i + fr) * RS16 + 16 * j + 4 * fg) = y;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int it = 0; it < NIT16; ++it) {
        const int id = lane + 64 * it;
        const int r = id / CPR, c8 = id - r * CPR;
        const int m = mw + h * (WM / NPASS16) + r, n = nw + c8 * 8;
        if (id >= NCH16 || m >= p.M || n >= p.N) continue;
        half8 o = *reinterpret_cast<const half8*>(st + r * RS16 + c8 * 8);
        if (res) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (half_t)((float)o[j] + (float)rr[it][j]);
        }
        if (p.diag & 8) asm volatile("" ::"v"(o));
        else *reinterpret_cast<half8*>(p.C + (long)m * p.ldc + n) = o;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    return;
  }
  if constexpr (GEGLU) {
    // lane-derived epilogue values from an opaque copy of the lane id: nothing of this epilogue can be hoisted
    // above the main loop (hoisted addresses kept the table-GELU variant's K loop in scratch)
    int lane_o = lane;
    asm volatile("" : "+v"(lane_o));
    const int fr_e = lane_o & 15, fg_e = lane_o >> 4;
    // Routed GEGLU on the swapped fragments, value and gate paired in registers by the weight layout: lane
    // (fr, fg) holds columns 16 j + 4 fg .. +3 of row 16 i + fr, i.e. [value, value, gate, gate] of neurons
    // 8 j + 2 fg, +1 (W rows interleaved [v 2 | g 2] per neuron pair: no cross-lane move; the [v 8 | g 8] layout
    // of rounds 1-3 needed two v_permlane32_swap per fragment, 2 of its 11 epilogue instructions). The fp16
    // product and the activated gate (both exact fp16 values) are staged in LDS per wave ([RG rows][NH neurons]
    // each; the 16 rows x 4 lanes of a 4-B store phase hit 64 distinct banks at NH = 40), then copied out as 16-B
    // row chunks, and every (row, expert) lane sums its expert's gates in neuron order in fp32 -- the rounding
    // points of sdmoe_linear + sdmoe_geglu_route (bit-identical). LDS traffic per wave tile: 4 x WM x NH x 2 B.
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    constexpr int NH = WN / 2;                    // neurons of this wave's tile
    constexpr int FPP = FM % 2 == 0 ? 2 : 1;      // fragment rows per staging pass
    constexpr int RG = 16 * FPP;                  // rows per staging pass
    constexpr int GST = NW * 2 * RG * NH * 2;     // staging bytes of all waves
    static_assert(NH % 8 == 0, "whole 16-B product chunks per row");
    static_assert(GST + NW * WN * 4 <= SMEM1, "GEGLU staging and bias must fit in the kernel's LDS");
    // staging base: with the GELU table prefetched into ring stage nk % NSTAGE, the stage of the last K-step (free
    // since the barrier above) holds the staging; otherwise offset 0 and a late-loaded table behind the staging
    static_assert(GST + NW * WN * 4 == G_STAGING, "GEGLU staging size");
    constexpr bool gtab = TAB_OK;  // MODE_GEGLU_GT: launched only with a registered table and act = GELU
    char* const sbase = (TAB_PREFETCH && gtab) ? smem + ((nk - 1) % NSTAGE) * STAGE : smem;
    const half_t* const tab = reinterpret_cast<const half_t*>(
        TAB_PREFETCH ? smem + (nk % NSTAGE) * STAGE + STAGE - TAB_BYTES : smem + TAB_LATE_OFF);
    if (!TAB_PREFETCH && gtab) {  // no stage holds the table: load it now (the ring is idle)
      issue_gelu_tab(smem + TAB_LATE_OFF);
    }
    if (gtab) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every wave's table pieces visible
    }
    half_t* sp = reinterpret_cast<half_t*>(sbase) + wave * 2 * RG * NH;  // products [RG][NH]
    half_t* sg = sp + RG * NH;                                           // activated gates [RG][NH]
    float* gbias = reinterpret_cast<float*>(sbase + GST) + wave * WN;    // this wave's WN bias values (fp32)
    for (int c = lane_o; c < WN; c += 64) gbias[c] = LN ? p.ln_bias[nw + c] : (float)p.bias[nw + c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nsel = 2 * fg_e;  // this lane's neuron pair in every fragment: 8 j + nsel, +1
    constexpr int CPO = NH / 8, RPI = 64 / CPO;  // copy-out: 16-B chunks per staged row, rows per 64-lane round
    const int lr = lane_o / CPO, lc = lane_o - (lane_o / CPO) * CPO;
    half_t* const cout = p.C + (long)(mw + lr) * p.ldc + nw / 2 + 8 * lc;
    // this lane's bias quads in every fragment (columns 16 j + 4 fg .. +3: value, value, gate, gate), hoisted out
    // of the rows (the table GELU's epilogue reads them from LDS per fragment instead: its temporaries need those
    // 20 VGPRs)
    float4v bq[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bq[j] = gtab ? (float4v){0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const float4v*>(gbias + 16 * j + 4 * fg_e);
    auto stage_pass = [&](int h, auto act_tag) {
      constexpr int ACTK = decltype(act_tag)::value;  // 0: ReLU, 1: GELU from the LDS table, 2: apply_act
      constexpr bool RELU = ACTK == 0;
#pragma unroll
      for (int ii = 0; ii < FPP; ++ii) {
        const int i = h * FPP + ii;
        float la = 0.f, lc = 0.f;
        if constexpr (LN) {
          const int rl = wr * WM + 16 * i + fr_e;
          la = ln_row[2 * rl];
          lc = ln_row[2 * rl + 1];
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float4v v = acc[i][j];
          if constexpr (LN) {  // rstd * (acc - mean * wsum); ln_bias is the bias below
            const float4v ws = *reinterpret_cast<const float4v*>(ln_col + wc * WN + 16 * j + 4 * fg_e);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(la, v[r], lc * ws[r]);
          }
          const float4v b = ACTK == 1 ? *reinterpret_cast<const float4v*>(gbias + 16 * j + 4 * fg_e) : bq[j];
          const h2 yv = {(half_t)(v[0] + b[0]), (half_t)(v[1] + b[1])};
          const h2 yg = {(half_t)(v[2] + b[2]), (half_t)(v[3] + b[3])};
          h2 ga;
          if constexpr (RELU) ga = __builtin_elementwise_max(yg, (h2){(half_t)0.f, (half_t)0.f});
          else if constexpr (ACTK == 1) ga = (h2){gelu_tab_h(yg[0], tab), gelu_tab_h(yg[1], tab)};
          else ga = (h2){(half_t)apply_act((float)yg[0], p.act), (half_t)apply_act((float)yg[1], p.act)};
          const int off = (16 * ii + fr_e) * NH + 8 * j + nsel;
          *reinterpret_cast<h2*>(sp + off) = yv * ga;  // fp16 x fp16 is exact in fp32: rounds like the unfused path
          *reinterpret_cast<h2*>(sg + off) = ga;
          // the table GELU's temporaries: one fragment at a time (interleaving all FN pushed 256x320 into scratch)
          if constexpr (ACTK == 1) __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
#pragma unroll
    for (int h = 0; h < FM / FPP; ++h) {
      if constexpr (gtab) stage_pass(h, std::integral_constant<int, 1>());
      else if (p.act == ACT_RELU) stage_pass(h, std::integral_constant<int, 0>());
      else stage_pass(h, std::integral_constant<int, 2>());
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int mr0 = mw + h * RG;
      // copy-out: lane -> (row lr + RPI it, 16-B chunk lc) with a fixed per-lane chunk, so the global address is the
      // hoisted per-lane pointer plus a uniform row offset (no per-chunk 64-bit index arithmetic)
#pragma unroll
      for (int it = 0; it < (RG + RPI - 1) / RPI; ++it) {
        const int r = it * RPI + lr;
        if (lr < RPI && r < RG) {
          const half8 o = *reinterpret_cast<const half8*>(sp + r * NH + 8 * lc);
          if (p.diag & 8) asm volatile("" ::"v"(o));
          else if (mr0 + r < p.M) *reinterpret_cast<half8*>(cout + (long)(h * RG + it * RPI) * p.ldc) = o;
        }
      }
      if (p.score) {
        switch (p.esize) {
          case 20: expert_sums<20, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 10: expert_sums<10, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 40: expert_sums<40, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 8: expert_sums<8, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 5: expert_sums<5, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 4: expert_sums<4, NH, RG>(p, sg, mr0, nw, lane_o); break;
          case 2: expert_sums<2, NH, RG>(p, sg, mr0, nw, lane_o); break;
          default: expert_sums<1, NH, RG>(p, sg, mr0, nw, lane_o); break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    return;
  }
  // fp32 path (activation, residual): stage the raw accumulators (one b128 per fragment), then epilogue8 on
  // 8-column row chunks
  float* st = reinterpret_cast<float*>(smem) + wave * (WM / NPASS) * WN_PAD;
#pragma unroll
  for (int h = 0; h < NPASS; ++h) {
#pragma unroll
    for (int i = 0; i < FM / NPASS; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        *reinterpret_cast<float4v*>(st + (16 * i + fr) * WN_PAD + 16 * j + 4 * fg) = acc[h * (FM / NPASS) + i][j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int id = lane; id < (WM / NPASS) * CPR; id += 64) {
      const int r = id / CPR, c8 = id - r * CPR;
      const int m = mw + h * (WM / NPASS) + r, n = nw + c8 * 8;
      if (m >= p.M || n >= p.N) continue;
      const float* sp = st + r * WN_PAD + c8 * 8;
      const float4v v0 = *reinterpret_cast<const float4v*>(sp), v1 = *reinterpret_cast<const float4v*>(sp + 4);
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      epilogue8(p, m, n, v);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// split-K combine: ordered (deterministic) sum of the fp32 slabs + the fused epilogue
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  const long nchunk = (long)p.M * (p.N / 8);
  for (long id = blockIdx.x * 256L + threadIdx.x; id < nchunk; id += (long)gridDim.x * 256) {
    const int m = (int)(id / (p.N / 8)), n = (int)(id % (p.N / 8)) * 8;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int s = 0; s < p.ksplit; ++s) {
      const float* sp = p.part + ((long)s * p.M + m) * p.N + n;
      float4v a = *reinterpret_cast<const float4v*>(sp), b = *reinterpret_cast<const float4v*>(sp + 4);
      v[0] += a[0]; v[1] += a[1]; v[2] += a[2]; v[3] += a[3];
      v[4] += b[0]; v[5] += b[1]; v[6] += b[2]; v[7] += b[3];
    }
    epilogue8(p, m, n, v);
  }
}

// ---- launch planning (host only) ----------------------------------------------------------------------------
// A launch = a tile instantiation + a split-K factor. The split (with the 64-deep K walk every tile shares) is the
// only thing that decides each output's fp32 summation order -- tile shape and wave arrangement do not -- so it is
// computed by ONE function (plan_split) from the chosen tile, and the masked modes (MODE_KEEP / WMASK / KEEPW) take
// the plain GEMM's plan for their shape (dispatch below): a keep- or Wanda-masked product is bit-identical to masking
// the operand first and running sdmoe_linear by construction, not by a restated copy of the plain rules.
enum TileId { T128x160, T64x160, T256x320, T256x160_42, T256x320_42, T128x320, T128x160_42, T64x320, T128x32, T128x64,
              T128x128, T64x128, NTILE };
struct TileShape { int bm, bn, wmw, wnw; };
constexpr TileShape kTile[NTILE] = {{128, 160, 2, 2}, {64, 160, 2, 2}, {256, 320, 2, 4}, {256, 160, 4, 2},
                                    {256, 320, 4, 2}, {128, 320, 2, 4}, {128, 160, 4, 2}, {64, 320, 2, 4},
                                    {128, 32, 2, 2},  {128, 64, 2, 2},  {128, 128, 2, 2}, {64, 128, 2, 2}};
struct Plan {
  int tile;
  int ks_want;      // split-K wish of the tile rule (0 = the policy in plan_split)
  int stages_want;  // LDS ring depth wish (0 = launch_tile's policy)
};

// compute units of the current device, queried once (both split policies size their grids by it; 256 on MI355X, and
// the fallback when no device answers, e.g. sdmoe_gemm_plan on a CPU host). Splits -- hence the fp32 summation order
// of split-K outputs -- are per-device-SKU by design.
int device_cus() {
  if (g_cus_init) return g_cus;
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
      hipSuccess && n > 0)
    g_cus = n;
  g_cus_init = true;
  return g_cus;
}

// split-K factor of a launch on tile t (mode: the tile rule's MODE; ws: whether a slab workspace was handed in)
int plan_split(const TileShape& t, int mode, const GemmParams& p, const float* ws, long ws_floats, int ks_want) {
  const int ntiles = ((p.M + t.bm - 1) / t.bm) * ((p.N + t.bn - 1) / t.bn);
  const int nk = p.K / 64;
  const int cus = device_cus();
  int ksplit = 1;
  // fill the chip: split K when the tile grid covers well under one wave of CUs
  if (ws && (g_ksplit > 0 || ks_want > 0)) {
    ksplit = g_ksplit > 0 ? g_ksplit : ks_want;
    if (ksplit > nk) ksplit = nk;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
  } else if (ws && (mode == MODE_CONV || mode == MODE_CONV_UP) && ntiles <= 16 && nk >= 64) {
    // latency regime (one prompt per call, base_receiver.py:73: 8x8 / 16x16 / 32x32 convs at batch 2): up to two
    // workgroups per CU, >= 11 K-steps per split, <= 64 MB of fp32 slabs -- B = 1 sweep (profiles/r05_b1_split_sweep.txt):
    // 8x8 1280 -> 1280 28.1 -> 23.5 us, 2560 -> 1280 44.3 -> 29.6, 16x16 stride 2 39.9 -> 22.0, 32x32 1280 -> 640
    // 64.2 -> 55.2 (at most 8 splits before)
    ksplit = (2 * cus + ntiles - 1) / ntiles;
    if (ksplit > 24) ksplit = 24;
    if (ksplit > nk / 11) ksplit = nk / 11;
    while (ksplit > 1 && (long)ksplit * p.M * p.N * 4 > (64L << 20)) --ksplit;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
  } else if (ws && ntiles < 3 * cus / 4 && nk >= 16) {
    ksplit = (cus + ntiles - 1) / ntiles;
    if (ksplit > 8) ksplit = 8;
    if (ksplit > nk / 4) ksplit = nk / 4;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
  }
  if (ksplit < 1) ksplit = 1;
  // no empty trailing split: ceil(nk / ksplit) K-steps per split, as many splits as that takes (e.g. nk = 180 at 16
  // wanted: 12 per split -> 15 splits, not a 16th that writes a zero slab the reduce then reads)
  const int kchunk = (nk + ksplit - 1) / ksplit;
  return (nk + kchunk - 1) / kchunk;
}

template <int BM, int BN, int WMW, int WNW, int MODE>
int launch_tile(GemmParams p, float* ws, hipStream_t s, int ksplit, int stages_want = 0) {
  const int ntiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int nk = p.K / 64;
  if (p.w_bstride && p.rows_per_batch % BM) return SDMOE_EUNSUP;  // a tile would straddle two images' weights
  if (ksplit > 1 && !ws) return SDMOE_EARG;
  p.ksplit = ksplit > 1 ? ksplit : 1;
  constexpr int NTH = 64 * WMW * WNW;
  p.kchunk = (nk + p.ksplit - 1) / p.ksplit;
  p.part = p.ksplit > 1 ? ws : nullptr;
  // M-fastest order for split-K convs only: their weight slices (up to 29 MB at the 16x16 level) were re-fetched by
  // every XCD (PMC FETCH_SIZE of the split-K conv launches 140 -> 46 MB, time neutral); the M = 1024 split-K linears
  // measured 2 us slower with it
  p.mfast = (p.ksplit > 1 && g_mfast && (MODE == MODE_CONV || MODE == MODE_CONV_UP)) ? 1 : 0;
  p.diag = g_diag;
  p.epi_direct = g_epi_direct == 2 || (g_epi_direct == 1 && p.R == nullptr);  // host-side: a device test of R spilled
  p.res16 = g_res16;
  const dim3 grid(ntiles * p.ksplit);
  {
    // 64-deep K-steps (a 32-deep 4/5-stage ring measured slower on every shape; the kernel is generic in BK).
    // 4-wave tiles: 2-stage ring (2 workgroups/CU) when the grid has >= ~300 workgroups, else 3-stage; 8-wave
    // tiles: 3-stage where it fits in LDS -- measured crossovers on MI355X.
    const int stages = g_stages ? g_stages
                                : (stages_want ? stages_want : ((WMW * WNW == 4 && ntiles * p.ksplit >= 300) ? 2 : 3));
    constexpr bool FITS3 = 3 * ((BM + BN) * 64 * 2 + 1024 + keep_stage_bytes<BM, BN, MODE>()) +
                               (keep_stage_bytes<BM, BN, MODE>() ? keep_lut_bytes<MODE>() : 0) +
                               ((MODE == MODE_GEMM_LN || MODE == MODE_GEGLU_LN) ? BM * 8 + BN * 8 : 0) <= 160 * 1024;
    if constexpr (FITS3) {
      if (stages == 2) gemm_kernel<BM, BN, WMW, WNW, MODE, 2, 64><<<grid, NTH, 0, s>>>(p);
      else gemm_kernel<BM, BN, WMW, WNW, MODE, 3, 64><<<grid, NTH, 0, s>>>(p);
    } else {
      (void)stages;
      gemm_kernel<BM, BN, WMW, WNW, MODE, 2, 64><<<grid, NTH, 0, s>>>(p);
    }
  }
  SDMOE_CHECK_LAUNCH();
  if (p.ksplit > 1) {
    long nchunk = (long)p.M * (p.N / 8);
    int g = (int)((nchunk + 255) / 256);
    if (g > 2048) g = 2048;
    splitk_reduce_kernel<<<g, 256, 0, s>>>(p);
    SDMOE_CHECK_LAUNCH();
  }
  return SDMOE_OK;
}

// knob 16: halo-tiled stride-1 3x3 convs: 1 (default) = where they measured faster than the shifted-tile kernel:
// 64-wide outputs (256-row tiles), 16-wide ones on 256-row tiles (a whole image), the 32 -> 64, 16 -> 32 (256-row
// tiles) and 8 -> 16 upsample convs, 32-wide outputs with Cin >= 1280 (256-row tiles); 2 = every 128-row tile instead
// (32- / 16-wide outputs: 5-17 % slower, their 32-deep K-steps carry half the MFMAs per barrier); 3 = the default plus
// every 32-wide output on 256-row tiles (135.1 vs 118.0 us at 640 -> 640); 0 = off
int g_halo = 1;

// halo conv launch: BM x 320 tiles (8 waves 2 x 4, BK 32, 3-stage B ring), K split over whole 32-channel slices when
// the tile grid is under ~one wave of CUs
template <int BM, int MODE>
int launch_halo(GemmParams p, float* ws, long ws_floats, hipStream_t s) {
  const int cus = device_cus();
  constexpr int HW_ = halo_w(MODE);
  const int ntiles = (p.M / BM) * (p.N / 320);
  const int nsl = p.Cin / 32;
  int ksplit = 1;
  if (ws && g_ksplit > 0) {  // forced (knob 9, sweeps): at most one 32-channel slice per split
    ksplit = g_ksplit < nsl ? g_ksplit : nsl;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
  } else if (ws && ntiles <= 32) {
    // latency regime (batch 2: whole 16x16 images, the 8 -> 16 upsample, 64x64 at 32 tiles): up to two workgroups
    // per CU, >= 2 slices per split, <= 96 MB of fp32 slabs -- B = 1 sweep: 16x16 1280 -> 1280 56.1 -> 40.9 us
    // (20 splits), 2560 -> 1280 91.7 -> 55.3, 8 -> 16 upsample 38.0 -> 31.7 (at most 8 splits before)
    ksplit = (2 * cus + ntiles - 1) / ntiles;
    if (ksplit > 32) ksplit = 32;
    if (ksplit > nsl / 2) ksplit = nsl / 2;
    // whole rounds of one 8-wave workgroup per CU: 16 tiles x 20 splits left 64 workgroups alone in a second
    // round (8 -> 16 upsample at one prompt: 43.2 vs 30.9 us with 16 splits, profiles/r05_b1_conv_split_sweep.txt)
    if (ntiles * ksplit > cus && ntiles <= cus) ksplit = (cus / ntiles) * ((ksplit * ntiles) / cus);
    while (ksplit > 1 && (long)ksplit * p.M * p.N * 4 > (96L << 20)) --ksplit;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
    if (ksplit < 1) ksplit = 1;
  } else if (ws && ntiles < 200) {
    ksplit = (cus + ntiles - 1) / ntiles;  // 6 / 8 splits: 172 vs 128 us at 16x16 x 1280 (r04)
    if (ksplit > 8) ksplit = 8;
    if (ksplit > nsl / 2) ksplit = nsl / 2;
    while (ksplit > 1 && (long)ksplit * p.M * p.N > ws_floats) --ksplit;
    if (ksplit < 1) ksplit = 1;
  }
  const int slc = (nsl + ksplit - 1) / ksplit;   // main slices per split
  p.ksplit = (nsl + slc - 1) / slc;
  p.kchunk = slc;
  p.kchunk2 = p.A2 ? ((p.K - 9 * p.Cin) / 32 + p.ksplit - 1) / p.ksplit : 0;  // shortcut steps per split
  p.part = p.ksplit > 1 ? ws : nullptr;
  p.mfast = p.ksplit > 1 ? g_mfast : 0;
  p.diag = g_diag;
  p.epi_direct = g_epi_direct == 2 || (g_epi_direct == 1 && p.R == nullptr);  // host-side: a device test of R spilled
  p.res16 = g_res16;
  (void)HW_;
  gemm_kernel<BM, 320, 2, 4, MODE, 4, 32><<<dim3(ntiles * p.ksplit), 512, 0, s>>>(p);
  SDMOE_CHECK_LAUNCH();
  if (p.ksplit > 1) {
    long nchunk = (long)p.M * (p.N / 8);
    int g = (int)((nchunk + 255) / 256);
    if (g > 2048) g = 2048;
    splitk_reduce_kernel<<<g, 256, 0, s>>>(p);
    SDMOE_CHECK_LAUNCH();
  }
  return SDMOE_OK;
}

// stride-1, non-upsampling 3x3 conv (+ folded shortcut) on a halo tile: image widths 64 (256-row tiles = 4
// output rows), 32 and 16 (128-row tiles), N a multiple of 320; otherwise -1 (the shifted-tile path)
int try_halo(const GemmParams& p, float* ws, long ws_floats, hipStream_t s) {
  if (!g_halo || g_tile || p.stride != 1 || p.N % 320 || p.Cin % 32 || (p.K - 9 * p.Cin) % 32) return -1;
  if (p.upsample) {  // output width 2 W, output rows per image 2 H
    if (p.A2) return -1;
    const int ohw = 4 * p.H * p.Wd;
    if (p.Wd == 32 && ohw % 256 == 0) return launch_halo<256, MODE_CONVHUP64>(p, ws, ws_floats, s);
    if (p.Wd == 8 && ohw % 128 == 0) return launch_halo<128, MODE_CONVHUP16>(p, ws, ws_floats, s);  // 125.6 vs 137.0
    // one prompt per call (<= 32 tiles of 256 output rows): 128-row tiles, 68.8 vs 72.5 us at 2 images
    if (g_halo == 1 && p.Wd == 16 && ohw % 128 == 0 && (p.M / 256) * (p.N / 320) <= 32)
      return launch_halo<128, MODE_CONVHUP32>(p, ws, ws_floats, s);
    // 16 -> 32 upsample on 256-row tiles (8 output rows, K split over slices): 360.3 vs 383.1-395.8 us
    if (g_halo != 2 && p.Wd == 16 && ohw % 256 == 0) return launch_halo<256, MODE_CONVHUP32>(p, ws, ws_floats, s);
    if (g_halo < 2) return -1;
    if (p.Wd == 16 && ohw % 128 == 0) return launch_halo<128, MODE_CONVHUP32>(p, ws, ws_floats, s);  // 449 vs 383 us
    return -1;
  }
  const int hw = p.H * p.Wd;
  // 64-wide outputs at one prompt (<= 32 tiles of 256 rows): 128-row tiles (two output rows), twice the workgroups
  // for the split to fill the chip with: 33.6 vs 41.0 us (320 -> 320) and 43.5 vs 51.1 (640 -> 320) at 2 images,
  // --batch 1 +0.8 % (profiles/r05_halo64_b1.txt)
  if (g_halo == 1 && p.Wd == 64 && hw % 128 == 0 && (p.M / 256) * (p.N / 320) <= 32)
    return launch_halo<128, MODE_CONVH64>(p, ws, ws_floats, s);
  if (p.Wd == 64 && hw % 256 == 0) return launch_halo<256, MODE_CONVH64>(p, ws, ws_floats, s);
  // one prompt per call (<= 32 tiles of 256 rows): 128-row tiles for the 16-wide and the narrow-input 32-wide convs,
  // twice the workgroups for the split -- 31.9 vs 39.9 us (16x16 1280 -> 1280), 32.3 vs 35.2 (32x32 640 -> 640), 38.9
  // vs 41.3 (960 -> 640) at 2 images; the Cin >= 1280 32-wide convs keep 256-row tiles (57.8 vs 52.0 us)
  // (profiles/r05_halo128_b1.txt)
  const bool small = (p.M / 256) * (p.N / 320) <= 32;
  if (g_halo == 1 && small && p.Wd == 16 && hw % 128 == 0) return launch_halo<128, MODE_CONVH16>(p, ws, ws_floats, s);
  if (g_halo == 1 && small && p.Wd == 32 && hw % 128 == 0 && p.Cin < 1280)
    return launch_halo<128, MODE_CONVH32>(p, ws, ws_floats, s);
  // 16-wide outputs: a whole 16x16 image per 256-row tile, K split over slices (1280 -> 1280: 127.6 vs 133.0 us)
  if (g_halo != 2 && p.Wd == 16 && hw % 256 == 0) return launch_halo<256, MODE_CONVH16>(p, ws, ws_floats, s);
  // 32-wide outputs: halo tiles (8 output rows) for the wide-input convs only (up-block conv1, Cin 1920 / 1280): 292 vs
  // 307 us and 206 vs 208 at 16 images, 62 vs 66 and 52 vs 54 at 2; at Cin 640 / 960 they ran 10-14 % slower
  // (profiles/r05_halo32_geglu_diag.txt)
  if (g_halo == 1 && p.Wd == 32 && hw % 256 == 0 && p.Cin >= 1280) return launch_halo<256, MODE_CONVH32>(p, ws, ws_floats, s);
  if (g_halo == 3 && p.Wd == 32 && hw % 256 == 0) return launch_halo<256, MODE_CONVH32>(p, ws, ws_floats, s);
  if (g_halo < 2) return -1;
  if (p.Wd == 32 && hw % 128 == 0) return launch_halo<128, MODE_CONVH32>(p, ws, ws_floats, s);
  if (p.Wd == 16 && hw % 128 == 0) return launch_halo<128, MODE_CONVH16>(p, ws, ws_floats, s);
  return -1;
}

// knob 20: 1 (default) = the table-GELU GEGLU on the 256x320 2x4-wave tiles like the ReLU one (no scratch since the
// [v 2 | g 2] layout: 150.9-154.3 vs 178.2-186.2 us at M = 16384, C = 640; SDXL pipeline +4.0 %, same box);
// 0 = 256x160 4x2 tiles (rounds 3-4 until the layout change: 364 B/lane of scratch on 256x320)
int g_gt320 = 1;
int g_narrow = 1;  // knob 21: 1 (default) = N <= 32 conv outputs (conv_out's 8 padded channels) on 128x32 tiles
                   // (31.9 vs 34.8-35.1 us at 64x64 x 320 -> 8, same box), 0 = 128x64

// routed-GEGLU linear: BN in {160, 320} tiles only (wave tile width 80 = 40 neurons = whole experts), no split-K
template <int MODE>
int dispatch_geglu(const GemmParams& p, hipStream_t s) {
  const int nt320 = ((p.M + 255) / 256) * (p.N / 320);
  const int nt160_128 = ((p.M + 127) / 128) * (p.N / 160);
  if (g_tile == 1) return launch_tile<128, 160, 2, 2, MODE>(p, nullptr, s, 1);
  if (g_tile == 4) return launch_tile<256, 160, 4, 2, MODE>(p, nullptr, s, 1);
  if constexpr (MODE != MODE_GEGLU_GT)  // (no room for the GELU table behind that tile's staging)
    if (g_tile == 7) return launch_tile<128, 160, 4, 2, MODE>(p, nullptr, s, 1);  // sweep: two workgroups per CU
  if (MODE == MODE_GEGLU_GT && g_tile == 0 && !g_gt320 && p.N % 320 == 0 && nt320 >= 240)
    // knob 20 = 0: the same rows on 256x160 tiles, 8 waves 4 x 2 (wave tile 64 x 80)
    return launch_tile<256, 160, 4, 2, MODE>(p, nullptr, s, 1);
  if (p.N % 320 == 0 && nt320 >= 240) {
    // 2x4 waves (wave tile 128 rows x 40 neurons): with the row-fastest epilogue its 32-row staging passes are
    // conflict-free (4x2's 16-row passes are not: two 16-lane b128 groups mix column pairs); 174.6 vs 181.2 us at
    // M = 65536, 129.8 vs 132.9 at 16384, 103.4 vs 106.4 at 4096 (same box)
    if (g_tile == 5) return launch_tile<256, 320, 4, 2, MODE>(p, nullptr, s, 1);
    return launch_tile<256, 320, 2, 4, MODE>(p, nullptr, s, 1);
  }
  // one prompt per call at the 16x16 level (M = 512, N = 10240): 8-wave 128x160 tiles, 20.5 vs 27.3 us on the 4-wave
  // ones (the 32x32 level's M = 2048 measured 24.3 vs 19.0 with them; profiles/r05_b1_geglu_keep_tiles.txt)
  if constexpr (MODE != MODE_GEGLU_GT)
    if (p.M <= 1024 && nt160_128 >= 128) return launch_tile<128, 160, 4, 2, MODE>(p, nullptr, s, 1);
  if (nt160_128 >= 200 || p.M > 2048) return launch_tile<128, 160, 2, 2, MODE>(p, nullptr, s, 1);
  return launch_tile<64, 160, 2, 2, MODE>(p, nullptr, s, 1);
}

// Tile rule of the dense modes (GEMM, CONV, CONV_UP, GEMM_LN); the masked modes plan as MODE_GEMM (dispatch).
template <int MODE>
Plan choose_tile(const GemmParams& p) {
  static_assert(!mode_akeep(MODE) && !mode_wmask(MODE), "masked modes take the plain GEMM's plan");
  const int tm256 = (p.M + 255) / 256;
  // forced tile (sdmoe_tune knob 1): 1 = 128x160, 2 = 64x160, 3 = 256x320 (8 waves), 4 = 256x160 (8 waves)
  if (g_tile == 1) return {T128x160, 0, 0};
  if (g_tile == 2) return {T64x160, 0, 0};
  if (g_tile == 3 && p.N % 320 == 0) return {T256x320, 0, 0};
  if (g_tile == 4 && p.N % 160 == 0) return {T256x160_42, 0, 0};
  if (g_tile == 5 && p.N % 320 == 0) return {T256x320_42, 0, 0};
  if (g_tile == 6 && p.N % 320 == 0) return {T128x320, 0, 0};
  // sweep-only 8-wave tiles with a 32x80 wave tile (two workgroups per CU on a 2-stage ring)
  if (MODE != MODE_CONV_UP && g_tile == 7 && p.N % 160 == 0) return {T128x160_42, 0, 0};
  if (MODE != MODE_CONV_UP && g_tile == 8 && p.N % 320 == 0) return {T64x320, 0, 0};
  // 8-wave 256x320 tile (wave tile 128x80: 2.5x the MFMA work per LDS byte of 64x80) whenever it alone fills
  // the chip; 256x160 8-wave + split-K for long-K problems whose 128x160 grid is under ~1.2 waves of CUs.
  // Measured on MI355X with tools/gemm_bench.py --tile.
  const int nt320 = tm256 * (p.N / 320);
  const int nt160_128 = ((p.M + 127) / 128) * ((p.N + 159) / 160);
  // (180: the 16x16-level fused QKV, M = 4096 x N = 3840 x K = 1280 -- also SDXL's 32x32 level -- 43.8 vs 49.9 us on
  // 128x160; every other U-Net shape is outside 180..240)
  // 32x32-level projections (M = 16384): the LayerNorm-folded QKV / Q and the plain (no residual) N = 640 GEMM on
  // 128x320 8-wave tiles (wave tile 64x80, one workgroup per CU): 58.8 vs 62.7 us (QKV, N = 1920), 19.5 vs 22.1 us
  // (N = 640) in a same-box tools/gpu_tile_sweep.sh run; the residual / conv shapes measured neutral or slower there
  if ((MODE == MODE_GEMM_LN && p.M >= 8192 && p.M <= 16384 && p.N % 320 == 0) ||
      (MODE == MODE_GEMM && !p.R && p.act == ACT_NONE && p.M >= 8192 && p.M <= 16384 && p.N == 640 && p.K == 640))
    return {T128x320, 0, 0};
  if (p.N % 320 == 0 && nt320 >= 180) return {T256x320, 0, 0};
  // 1-1.25 waves of 128x160 tiles (M = 4096 x N = 1280 projections at the 16x16 level): 64x160 tiles double
  // the grid to two workgroups per CU — 15-18 % faster in isolation (tools/gpu_tiles_all.sh). Convs keep their
  // tiles: with the convs included the same-box pipeline A/B measured 0.5 % slower.
  if ((MODE == MODE_GEMM || MODE == MODE_GEMM_LN) && p.N % 160 == 0 && nt160_128 >= 200 && nt160_128 < 320 &&
      p.K <= 5120)
    return {T64x160, 0, 0};
  // convs (tools/gemm_bench.py --tile/--stages sweep, same box): the 16x16-level 3x3 convs (M = 4096, N = 1280,
  // K = 9 x 1280 / 9 x 2560) on the 8-wave 256x320 tile with a 4-way split-K: 120 / 205 us vs 135 / 237 us on
  // 256x160 with a 2-way split (the 32x32 level's 1280 -> 640 conv stays on 128x160: 207 vs 221 us); the
  // 64x64 -> 32x32 stride-2 conv (M = 16384, N = 320) on 64x160 tiles at two workgroups per CU: 38 vs 57 us on
  // 128x160 with a 3-stage ring
  if constexpr (MODE == MODE_CONV) {
    // 8x8-level 3x3 convs (M = 1024, K = 9 x 1280 / 9 x 2560): 8-wave 128x160 tiles (wave tile 32x80), 2-stage ring
    // (two workgroups per CU), 8-way split-K: 44.6 / 68.2 us vs 51.2 / 72.8 on 256x160 4x2 waves (tile_sweep.py)
    // At one prompt per call (M = 128: 8 tiles) the fixed 8-way split left 64 workgroups streaming ~23 K-steps each
    // behind a 2-stage ring; such grids (<= 16 tiles) take plan_split's latency-regime split instead (16-24 ways)
    if (p.stride == 1 && p.N % 160 == 0 && p.M <= 1024 && p.K >= 9 * 1280)
      return {T128x160_42, nt160_128 <= 16 ? 0 : 8, 2};
    if (p.stride == 1 && p.N % 320 == 0 && nt320 < 240 && p.K >= 9 * 1280 && p.M >= 2048 && p.M <= 4096)
      return {T256x320, 0, 0};
    if (p.stride == 2 && p.N % 160 == 0 && p.M >= 8192) return {T64x160, 0, 0};
    // the 32x32 -> 16x16 and 16x16 -> 8x8 downsamplers (M = 4096 / 1024): a 4-way split-K, two workgroups per CU
    // (their strided-tap A loads want the extra waves in flight): 46.1-46.7 vs 65.7-66.3 us and 46.4-46.9 vs
    // 78.4-80.1 us with the auto ~one-per-CU split of 2, on every tile shape (same box)
    if (p.stride == 2 && p.N % 160 == 0 && p.M < 8192) {
      if (p.M > 2048) return {T128x160, 4, 0};
      // (<= 16 tiles, the 16x16 -> 8x8 downsampler at one prompt: plan_split's latency-regime split)
      const int nt64 = ((p.M + 63) / 64) * (p.N / 160);
      return {T64x160, nt64 <= 16 ? 0 : 4, 0};
    }
  }
  // (the keep-masked down projection at one prompt, <= 128 tiles of 128x160, runs on 64x160 tiles through the plain
  // rule below: 22.3 vs 29.5 us at the 64x64 level, profiles/r05_b1_geglu_keep_tiles.txt)
  if (p.N % 160 == 0 && p.K >= 2560 && nt160_128 < 300 && !(MODE == MODE_CONV && p.stride == 2))
    return {T256x160_42, 0, 0};
  if (MODE == MODE_CONV_UP) return {p.N % 160 == 0 ? T128x160 : T128x128, 0, 0};
  if constexpr (MODE == MODE_CONV)  // conv_out (N = 8 padded channels): a quarter of 128x64's MFMA padding
    if (p.N <= 32 && g_narrow) return {T128x32, 0, 0};
  if (p.N <= 64) return {T128x64, 0, 0};
  if (p.N % 160 == 0) {
    // plain GEMMs under ~one wave of 128x160 tiles take 64x160 at any M: the 64x64 level's K = 320 projections at one
    // prompt (M = 8192, N = 320: 128 tiles) 7.8 vs 10.6 us, 8.4 vs 11.8 with the residual (r05_b1_linear_tiles.txt)
    if (nt160_128 >= 200 || (p.M > 2048 && MODE != MODE_GEMM)) return {T128x160, 0, 0};
    return {T64x160, 0, 0};
  }
  const int nt128 = ((p.M + 127) / 128) * ((p.N + 127) / 128);
  if (nt128 >= 200 || p.M > 2048) return {T128x128, 0, 0};
  return {T64x128, 0, 0};
}

// the tile a masked mode runs the plain GEMM's plan on: the same one where it is instantiated for the mode, with the
// keep-masked A operand on the 4x2-wave arrangement of 256x320 (wave tile 64x160: half the A fragments to mask per
// wave, 61 vs 69 us at M = 65536, N = 320, K = 1280); the split stays the plain GEMM's, so the bits do too
template <int MODE>
int masked_tile(int t, const GemmParams& p) {
  if (mode_akeep(MODE) && t == T256x320) return T256x320_42;
  if (t == T128x320 || t == T128x160_42 || t == T64x320 || t == T128x32) return p.N % 160 == 0 ? T128x160 : T128x128;
  return t;
}

template <int MODE>
int launch_plan(int tile, int ksplit, int stages_want, const GemmParams& p, float* ws, hipStream_t s) {
  switch (tile) {
    case T128x160: return launch_tile<128, 160, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T64x160: return launch_tile<64, 160, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T256x320: return launch_tile<256, 320, 2, 4, MODE>(p, ws, s, ksplit, stages_want);
    case T256x160_42: return launch_tile<256, 160, 4, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T256x320_42: return launch_tile<256, 320, 4, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T128x320: return launch_tile<128, 320, 2, 4, MODE>(p, ws, s, ksplit, stages_want);
    case T128x64: return launch_tile<128, 64, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T128x128: return launch_tile<128, 128, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
    case T64x128: return launch_tile<64, 128, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
    default: break;
  }
  if constexpr (MODE == MODE_GEMM || MODE == MODE_CONV || MODE == MODE_GEMM_LN) {
    if (tile == T128x160_42) return launch_tile<128, 160, 4, 2, MODE>(p, ws, s, ksplit, stages_want);
    if (tile == T64x320) return launch_tile<64, 320, 2, 4, MODE>(p, ws, s, ksplit, stages_want);
  }
  if constexpr (MODE == MODE_CONV)
    if (tile == T128x32) return launch_tile<128, 32, 2, 2, MODE>(p, ws, s, ksplit, stages_want);
  return SDMOE_EUNSUP;
}

// plan of a dense or masked launch: {tile, split, stages wish}; masked modes plan as the plain GEMM of the shape
template <int MODE>
Plan plan_launch(const GemmParams& p, const float* ws, long ws_floats, int* ksplit) {
  constexpr bool MASKED = mode_akeep(MODE) || mode_wmask(MODE);
  constexpr int PM = MASKED ? MODE_GEMM : MODE;
  Plan pl = choose_tile<PM>(p);
  *ksplit = plan_split(kTile[pl.tile], PM, p, ws, ws_floats, pl.ks_want);
  if constexpr (MASKED) pl.tile = masked_tile<MODE>(pl.tile, p);
  return pl;
}

template <int MODE>
int dispatch(const GemmParams& p, float* ws, long ws_floats, hipStream_t s) {
  int ksplit = 1;
  const Plan pl = plan_launch<MODE>(p, ws, ws_floats, &ksplit);
  return launch_plan<MODE>(pl.tile, ksplit, pl.stages_want, p, ws, s);
}

// ---- elementwise helpers for the GEMM operands ------------------------------------------------------

// GroupNorm apply (+SiLU): Y = act(X * scale[img, c] + shift[img, c]) on [nimg*HW, C] (16 B per thread)
__global__ __launch_bounds__(256) void gn_apply_kernel(const half_t* __restrict__ X, long ldx, int HW, int C,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       int silu, half_t* __restrict__ Y, long ldy, long rows) {
  const int cpr = C / 8;
  const long n = rows * cpr;
  for (long id = blockIdx.x * 256L + threadIdx.x; id < n; id += (long)gridDim.x * 256) {
    const long r = id / cpr;
    const int c = (int)(id - r * cpr) * 8;
    const int img = (int)(r / HW);
    half8 x = *reinterpret_cast<const half8*>(X + r * ldx + c);
    const float* sc = scale + (long)img * C + c;
    const float* sh = shift + (long)img * C + c;
    float4v s0 = *reinterpret_cast<const float4v*>(sc), s1 = *reinterpret_cast<const float4v*>(sc + 4);
    float4v h0 = *reinterpret_cast<const float4v*>(sh), h1 = *reinterpret_cast<const float4v*>(sh + 4);
    float s[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    float h[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)x[j] * s[j] + h[j];
      if (silu) f = silu_f(f);
      o[j] = (half_t)f;
    }
    *reinterpret_cast<half8*>(Y + r * ldy + c) = o;
  }
}

// Wanda weight mask: Wm[n, k] = bit(n, k) ? 0 : W[n, k]   (bits [N][K/8], little-endian within a byte)
__global__ __launch_bounds__(256) void mask_weight_kernel(const half_t* __restrict__ W, const uint8_t* __restrict__ bits,
                                                          half_t* __restrict__ Wm, long n8) {
  for (long id = blockIdx.x * 256L + threadIdx.x; id < n8; id += (long)gridDim.x * 256) {
    half8 w = reinterpret_cast<const half8*>(W)[id];
    const unsigned b = bits[id];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((b >> j) & 1u) w[j] = (half_t)0.f;
    reinterpret_cast<half8*>(Wm)[id] = w;
  }
}

// Wanda bits [N][K/8] (bit k%8 of byte (n, k/8) = W[n, k] removed) -> the GEMM's K-step-major layout
// out[s][n] (uint64) bit j = mask(n, k = perm ? perm[64 s + j] : 64 s + j): one thread per output word. perm maps a
// permuted column position to the original column (the routed FFN down projection's expert-major neuron order).
__global__ __launch_bounds__(256) void wmask_kmajor_kernel(const uint8_t* __restrict__ bits, long ldb, int N, int K,
                                                           const int* __restrict__ perm, unsigned long long* __restrict__ out) {
  const long nwords = (long)(K / 64) * N;
  for (long id = blockIdx.x * 256L + threadIdx.x; id < nwords; id += (long)gridDim.x * 256) {
    const int s = (int)(id / N), n = (int)(id - (long)s * N);
    const uint8_t* row = bits + (long)n * ldb;
    unsigned long long w = 0;
    if (perm) {
      for (int j = 0; j < 64; ++j) {
        const int k = perm[64 * s + j];
        w |= (unsigned long long)((row[k >> 3] >> (k & 7)) & 1u) << j;
      }
    } else {
#pragma unroll
      for (int b = 0; b < 8; ++b) w |= (unsigned long long)row[8 * s + b] << (8 * b);
    }
    out[id] = w;
  }
}

// LayerNorm fold (sdmoe_ln_fold): one block per output row n of W [N, K]:
//   Wf[n, k] = fp16(W[n, k] * gamma[k]); wsum[n] = sum_k Wf[n, k]; bias_f[n] = bias[n] + sum_k W[n, k] * beta[k]
// (fp32; fixed-order block reduction, so the fold is deterministic)
__global__ __launch_bounds__(256) void ln_fold_kernel(const half_t* __restrict__ W, long ldw, int K,
                                                      const half_t* __restrict__ gamma, const half_t* __restrict__ beta,
                                                      const half_t* __restrict__ bias, half_t* __restrict__ Wf, long ldf,
                                                      float* __restrict__ bias_f, float* __restrict__ wsum) {
  __shared__ float red[2][256];
  const int n = blockIdx.x, tid = threadIdx.x;
  float sw = 0.f, sb = 0.f;
  for (int k = tid; k < K; k += 256) {
    const float w = (float)W[(long)n * ldw + k];
    const half_t wf = (half_t)(w * (float)gamma[k]);
    Wf[(long)n * ldf + k] = wf;
    sw += (float)wf;
    sb = __builtin_fmaf(w, (float)beta[k], sb);
  }
  red[0][tid] = sw;
  red[1][tid] = sb;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) { red[0][tid] += red[0][tid + o]; red[1][tid] += red[1][tid + o]; }
    __syncthreads();
  }
  if (tid == 0) {
    wsum[n] = red[0][0];
    bias_f[n] = red[1][0] + (bias ? (float)bias[n] : 0.f);
  }
}

// GroupNorm fold (sdmoe_gn_fold): one wave per (image, output row n): Wf[i][n, k] = fp16(W[n, k] * scale[i, k]) and
// colbias[i][n] = bias[n] + sum_k W[n, k] * shift[i, k] (fp32, fixed-order lane sums + xor tree: deterministic)
__global__ __launch_bounds__(256) void gn_fold_kernel(const half_t* __restrict__ W, long ldw, int N, int K,
                                                      const half_t* __restrict__ bias, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, half_t* __restrict__ Wf,
                                                      float* __restrict__ colbias) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6), img = blockIdx.y;
  if (n >= N) return;
  const float* sc = scale + (long)img * K;
  const float* sh = shift + (long)img * K;
  half_t* wo = Wf + ((long)img * N + n) * K;
  float acc = 0.f;
  for (int k = lane * 8; k < K; k += 512) {
    const half8 w = *reinterpret_cast<const half8*>(W + (long)n * ldw + k);
    const float4v s0 = *reinterpret_cast<const float4v*>(sc + k), s1 = *reinterpret_cast<const float4v*>(sc + k + 4);
    const float4v h0 = *reinterpret_cast<const float4v*>(sh + k), h1 = *reinterpret_cast<const float4v*>(sh + k + 4);
    const float s[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
    const float h[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = (half_t)((float)w[j] * s[j]);
      acc = __builtin_fmaf((float)w[j], h[j], acc);
    }
    *reinterpret_cast<half8*>(wo + k) = o;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) colbias[(long)img * N + n] = acc + (bias ? (float)bias[n] : 0.f);
}

// fp16 GELU tables registered per device (sdmoe_set_gelu_table)
constexpr int MAX_DEV = 64;
const void* g_gelu_tab[MAX_DEV] = {};

int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

const half_t* sdmoe_gelu_tab_current() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return nullptr;
  return (const half_t*)g_gelu_tab[dev];
}

extern "C" int sdmoe_set_gelu_table(const void* table) {
  int dev = 0;
  const hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  if (dev < 0 || dev >= MAX_DEV) return SDMOE_EARG;
  if (table && (reinterpret_cast<uintptr_t>(table) & 15)) return SDMOE_ESHAPE;
  g_gelu_tab[dev] = table;
  return SDMOE_OK;
}

extern "C" int sdmoe_linear(const void* A, long lda, const void* W, long ldw, const void* bias,
                            const void* coladd, long coladd_bstride, int rows_per_batch,
                            const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act,
                            float* workspace, long workspace_floats, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !W || !C || M < 0 || N <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || N % 8 || lda % 8 || ldw % 8 || ldc % 8 || (R && ldr % 8)) return SDMOE_ESHAPE;
  if (coladd && rows_per_batch <= 0) return SDMOE_EARG;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = act;
  p.rows_per_batch = rows_per_batch > 0 ? rows_per_batch : 1;
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(N - 1) * ldw + K) * 2;
  if (ab >= (long)OOB || wb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  return dispatch<MODE_GEMM>(p, workspace, workspace_floats, (hipStream_t)stream);
}

extern "C" int sdmoe_gn_fold(const void* W, long ldw, int N, int K, const void* bias, const float* scale,
                             const float* shift, int nimg, void* Wf, float* colbias, void* stream) {
  if (N == 0 || nimg == 0) return SDMOE_OK;
  if (!W || !scale || !shift || !Wf || !colbias || N < 0 || K <= 0 || nimg < 0) return SDMOE_EARG;
  if (K % 8 || ldw % 8 || ldw < K) return SDMOE_ESHAPE;
  gn_fold_kernel<<<dim3((N + 3) / 4, nimg), 256, 0, (hipStream_t)stream>>>(
      (const half_t*)W, ldw, N, K, (const half_t*)bias, scale, shift, (half_t*)Wf, colbias);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_linear_per_image(const void* A, long lda, const void* Wf, long ldw, long w_bstride,
                                      const float* colbias, long colbias_bstride, int rows_per_batch, const void* R,
                                      long ldr, void* C, long ldc, int M, int N, int K, float* workspace,
                                      long workspace_floats, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !Wf || !C || M < 0 || N <= 0 || K <= 0 || rows_per_batch <= 0 || w_bstride <= 0) return SDMOE_EARG;
  if (K % 64 || N % 8 || lda % 8 || ldw % 8 || ldc % 8 || (R && ldr % 8) || rows_per_batch % 256 ||
      M % rows_per_batch || w_bstride % 8 || (colbias && colbias_bstride % 4))
    return SDMOE_ESHAPE;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)Wf; p.ldw = ldw; p.w_bstride = w_bstride;
  p.colf = colbias; p.colf_bstride = colbias_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = ACT_NONE; p.rows_per_batch = rows_per_batch;
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(N - 1) * ldw + K) * 2;
  if (ab >= (long)OOB || wb >= (long)OOB || (long)(M / rows_per_batch) * w_bstride * 2 >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  return dispatch<MODE_GEMM>(p, workspace, workspace_floats, (hipStream_t)stream);
}

extern "C" int sdmoe_linear_masked(const void* A, long lda, const void* keep, const void* W, long ldw,
                                   const void* wmask, const void* bias, const void* R, long ldr, void* C, long ldc,
                                   int M, int N, int K, float* workspace, long workspace_floats, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !W || !C || M < 0 || N <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || N % 8 || lda % 8 || ldw % 8 || ldc % 8 || (R && ldr % 8)) return SDMOE_ESHAPE;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw;
  p.bias = (const half_t*)bias; p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = ACT_NONE; p.rows_per_batch = 1;
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(N - 1) * ldw + K) * 2;
  const long kb = (long)(K / 64) * M * 8, mb = (long)(K / 64) * N * 8;
  if (ab >= (long)OOB || wb >= (long)OOB || kb >= (long)OOB || mb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  p.keep = (const uint8_t*)keep; p.keep_bytes = keep ? (int)kb : 0;
  p.wmask = (const uint8_t*)wmask; p.wmask_bytes = wmask ? (int)mb : 0;
  hipStream_t s = (hipStream_t)stream;
  if (keep && wmask) return dispatch<MODE_KEEPW>(p, workspace, workspace_floats, s);
  if (keep) return dispatch<MODE_KEEP>(p, workspace, workspace_floats, s);
  if (wmask) return dispatch<MODE_WMASK>(p, workspace, workspace_floats, s);
  return dispatch<MODE_GEMM>(p, workspace, workspace_floats, s);
}

extern "C" int sdmoe_gemm_plan(int mode, int M, int N, int K, int has_residual, int act, long workspace_floats,
                               int* out) {
  if (!out || M <= 0 || N <= 0 || K <= 0 || workspace_floats < 0) return SDMOE_EARG;
  if (K % 64 || N % 8) return SDMOE_ESHAPE;
  GemmParams p{};
  p.M = M; p.N = N; p.K = K; p.act = act; p.rows_per_batch = 1;
  static const half_t dummy[8] = {};
  p.R = has_residual ? dummy : nullptr;  // (only its presence enters the plan)
  // a non-null stand-in for the workspace pointer: only its presence and size enter the plan
  float* ws = workspace_floats > 0 ? reinterpret_cast<float*>(out) : nullptr;
  int ksplit = 1;
  Plan pl;
  switch (mode) {
    case MODE_GEMM: pl = plan_launch<MODE_GEMM>(p, ws, workspace_floats, &ksplit); break;
    case MODE_KEEP: pl = plan_launch<MODE_KEEP>(p, ws, workspace_floats, &ksplit); break;
    case MODE_WMASK: pl = plan_launch<MODE_WMASK>(p, ws, workspace_floats, &ksplit); break;
    case MODE_KEEPW: pl = plan_launch<MODE_KEEPW>(p, ws, workspace_floats, &ksplit); break;
    case MODE_GEMM_LN: pl = plan_launch<MODE_GEMM_LN>(p, nullptr, 0, &ksplit); break;  // (as sdmoe_linear_ln)
    default: return SDMOE_EUNSUP;
  }
  const TileShape& t = kTile[pl.tile];
  out[0] = t.bm; out[1] = t.bn; out[2] = t.wmw; out[3] = t.wnw; out[4] = ksplit;
  return SDMOE_OK;
}

extern "C" int sdmoe_linear_keep(const void* A, long lda, const void* keep, const void* W, long ldw, const void* bias,
                                 const void* R, long ldr, void* C, long ldc, int M, int N, int K, float* workspace,
                                 long workspace_floats, void* stream) {
  if (M != 0 && !keep) return SDMOE_EARG;
  return sdmoe_linear_masked(A, lda, keep, W, ldw, nullptr, bias, R, ldr, C, ldc, M, N, K, workspace,
                             workspace_floats, stream);
}

extern "C" int sdmoe_linear_geglu(const void* A, long lda, const void* W, long ldw, const void* bias, void* P,
                                  long ldp, int M, int F, int K, int act, void* score, long ld_score, int esize,
                                  void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !W || !bias || !P || M < 0 || F <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || F % 80 || lda % 8 || ldw % 8 || ldp % 8) return SDMOE_ESHAPE;
  if (score && (esize <= 0 || 40 % esize || ld_score < F / esize)) return SDMOE_ESHAPE;
  if (!(act == ACT_GELU || act == ACT_RELU || act == ACT_NONE || act == ACT_SILU)) return SDMOE_EUNSUP;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw;
  p.bias = (const half_t*)bias; p.C = (half_t*)P; p.ldc = ldp;
  p.M = M; p.N = 2 * F; p.K = K; p.act = act; p.rows_per_batch = 1;
  p.score = (half_t*)score; p.ld_score = ld_score; p.esize = esize;
  if (act == ACT_GELU) p.gelu_tab = sdmoe_gelu_tab_current();
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(2 * F - 1) * ldw + K) * 2;
  if (ab >= (long)OOB || wb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  if (p.gelu_tab) return dispatch_geglu<MODE_GEGLU_GT>(p, (hipStream_t)stream);
  return dispatch_geglu<MODE_GEGLU>(p, (hipStream_t)stream);
}

extern "C" int sdmoe_ln_fold(const void* W, long ldw, int N, int K, const void* gamma, const void* beta,
                             const void* bias, void* Wf, long ldf, float* bias_f, float* wsum, void* stream) {
  if (N == 0) return SDMOE_OK;
  if (!W || !gamma || !beta || !Wf || !bias_f || !wsum || N < 0 || K <= 0 || ldw < K || ldf < K) return SDMOE_EARG;
  ln_fold_kernel<<<N, 256, 0, (hipStream_t)stream>>>((const half_t*)W, ldw, K, (const half_t*)gamma,
                                                     (const half_t*)beta, (const half_t*)bias, (half_t*)Wf, ldf,
                                                     bias_f, wsum);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_linear_ln(const void* A, long lda, const void* Wf, long ldw, const float* bias_f,
                               const float* wsum, float eps, void* C, long ldc, int M, int N, int K, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !Wf || !bias_f || !wsum || !C || M < 0 || N <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || N % 8 || lda % 8 || ldw % 8 || ldc % 8) return SDMOE_ESHAPE;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)Wf; p.ldw = ldw;
  p.C = (half_t*)C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = ACT_NONE; p.rows_per_batch = 1;
  p.ln_wsum = wsum; p.ln_bias = bias_f; p.ln_eps = eps;
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(N - 1) * ldw + K) * 2;
  if (ab >= (long)OOB || wb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  return dispatch<MODE_GEMM_LN>(p, nullptr, 0, (hipStream_t)stream);  // no split-K: a tile's K loop sees whole rows
}

extern "C" int sdmoe_linear_geglu_ln(const void* A, long lda, const void* W, long ldw, const float* bias_f,
                                     const float* wsum, float eps, void* P, long ldp, int M, int F, int K, int act,
                                     void* score, long ld_score, int esize, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!A || !W || !bias_f || !wsum || !P || M < 0 || F <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || F % 80 || lda % 8 || ldw % 8 || ldp % 8) return SDMOE_ESHAPE;
  if (score && (esize <= 0 || 40 % esize || ld_score < F / esize)) return SDMOE_ESHAPE;
  if (!(act == ACT_GELU || act == ACT_RELU || act == ACT_NONE || act == ACT_SILU)) return SDMOE_EUNSUP;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw;
  p.C = (half_t*)P; p.ldc = ldp;
  p.M = M; p.N = 2 * F; p.K = K; p.act = act; p.rows_per_batch = 1;
  p.score = (half_t*)score; p.ld_score = ld_score; p.esize = esize;
  p.ln_wsum = wsum; p.ln_bias = bias_f; p.ln_eps = eps;  // (GELU from erfc here: the LN variant has no table form)
  const long ab = ((long)(M - 1) * lda + K) * 2, wb = ((long)(2 * F - 1) * ldw + K) * 2;
  if (ab >= (long)OOB || wb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  return dispatch_geglu<MODE_GEGLU_LN>(p, (hipStream_t)stream);
}

extern "C" int sdmoe_conv3x3(const void* X, long ldx, int nimg, int H, int W, int Cin,
                             const void* Wt, const void* bias, const void* coladd, long coladd_bstride,
                             const void* R, long ldr, void* Y, long ldy, int Cout, int stride, int upsample,
                             int act, float* workspace, long workspace_floats, void* stream) {
  if (nimg == 0) return SDMOE_OK;
  if (!X || !Wt || !Y || nimg < 0 || H <= 0 || W <= 0 || Cout <= 0) return SDMOE_EARG;
  if (Cin % 64 || Cout % 8 || ldx % 8 || ldy % 8 || (R && ldr % 8)) return SDMOE_ESHAPE;
  if (!(stride == 1 || stride == 2) || (upsample && stride != 1)) return SDMOE_EUNSUP;
  GemmParams p{};
  int OH, OW;
  if (upsample) { OH = 2 * H; OW = 2 * W; }
  else { OH = (H - 1) / stride + 1; OW = (W - 1) / stride + 1; }
  p.A = (const half_t*)X; p.lda = ldx; p.W = (const half_t*)Wt; p.ldw = 9L * Cin;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)Y; p.ldc = ldy;
  p.M = nimg * OH * OW; p.N = Cout; p.K = 9 * Cin; p.act = act;
  p.rows_per_batch = OH * OW;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = OH; p.OW = OW; p.stride = stride; p.upsample = upsample;
  const long ab = ((long)nimg * H * W - 1) * ldx * 2 + (long)Cin * 2, wb = (long)Cout * 9 * Cin * 2;
  if (ab >= (long)OOB || wb >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb;
  const int hs = try_halo(p, workspace, workspace_floats, (hipStream_t)stream);
  if (hs >= 0) return hs;
  if (upsample) return dispatch<MODE_CONV_UP>(p, workspace, workspace_floats, (hipStream_t)stream);
  return dispatch<MODE_CONV>(p, workspace, workspace_floats, (hipStream_t)stream);
}

extern "C" int sdmoe_conv3x3_sc(const void* X, long ldx, int nimg, int H, int W, int Cin, const void* Wt,
                                const void* bias, const void* coladd, long coladd_bstride, const void* X2, long ldx2,
                                int Cin2, void* Y, long ldy, int Cout, int act, float* workspace,
                                long workspace_floats, void* stream) {
  if (nimg == 0) return SDMOE_OK;
  if (!X || !Wt || !X2 || !Y || nimg < 0 || H <= 0 || W <= 0 || Cout <= 0 || Cin2 <= 0) return SDMOE_EARG;
  if (Cin % 64 || Cin2 % 64 || Cout % 8 || ldx % 8 || ldx2 % 8 || ldy % 8) return SDMOE_ESHAPE;
  GemmParams p{};
  p.A = (const half_t*)X; p.lda = ldx; p.W = (const half_t*)Wt; p.ldw = 9L * Cin + Cin2;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.C = (half_t*)Y; p.ldc = ldy;
  p.M = nimg * H * W; p.N = Cout; p.K = 9 * Cin + Cin2; p.act = act;
  p.rows_per_batch = H * W;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = H; p.OW = W; p.stride = 1; p.upsample = 0;
  p.A2 = (const half_t*)X2; p.lda2 = ldx2;
  const long ab = ((long)nimg * H * W - 1) * ldx * 2 + (long)Cin * 2, wb = (long)Cout * p.ldw * 2;
  const long a2b = ((long)nimg * H * W - 1) * ldx2 * 2 + (long)Cin2 * 2;
  if (ab >= (long)OOB || wb >= (long)OOB || a2b >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb; p.a2_bytes = (int)a2b;
  const int hs = try_halo(p, workspace, workspace_floats, (hipStream_t)stream);
  if (hs >= 0) return hs;
  return dispatch<MODE_CONV>(p, workspace, workspace_floats, (hipStream_t)stream);
}

extern "C" int sdmoe_conv3x3_gn(const void* X, long ldx, int nimg, int H, int W, int Cin, const float* gn_scale,
                                const float* gn_shift, int silu, const void* Wt, const void* bias, const void* coladd,
                                long coladd_bstride, const void* R, long ldr, const void* X2, long ldx2, int Cin2,
                                void* Y, long ldy, int Cout, float* workspace, long workspace_floats, void* stream) {
  if (nimg == 0) return SDMOE_OK;
  if (!X || !gn_scale || !gn_shift || !Wt || !Y || nimg < 0 || H <= 0 || W <= 0 || Cout <= 0 || Cin2 < 0) return SDMOE_EARG;
  if (Cin % 64 || Cin2 % 64 || Cout % 8 || ldx % 8 || ldy % 8 || (R && ldr % 8) || (X2 && ldx2 % 8)) return SDMOE_ESHAPE;
  if ((X2 != nullptr) != (Cin2 > 0) || (X2 && R)) return SDMOE_EARG;
  // only the halo tiles apply the GroupNorm in the kernel: the caller falls back to apply + conv on EUNSUP
  if (!g_halo || g_tile || Cin > 1280 || Cout % 320 || W != 64 || (H * W) % 256) return SDMOE_EUNSUP;
  GemmParams p{};
  p.A = (const half_t*)X; p.lda = ldx; p.W = (const half_t*)Wt; p.ldw = 9L * Cin + Cin2;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)Y; p.ldc = ldy;
  p.M = nimg * H * W; p.N = Cout; p.K = 9 * Cin + Cin2; p.act = ACT_NONE;
  p.rows_per_batch = H * W;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = H; p.OW = W; p.stride = 1; p.upsample = 0;
  p.A2 = (const half_t*)X2; p.lda2 = ldx2;
  p.gn_scale = gn_scale; p.gn_shift = gn_shift; p.gn_silu = silu;
  const long ab = ((long)nimg * H * W - 1) * ldx * 2 + (long)Cin * 2, wb = (long)Cout * p.ldw * 2;
  const long a2b = X2 ? ((long)nimg * H * W - 1) * ldx2 * 2 + (long)Cin2 * 2 : 0;
  if (ab >= (long)OOB || wb >= (long)OOB || a2b >= (long)OOB) return SDMOE_ESHAPE;
  p.a_bytes = (int)ab; p.w_bytes = (int)wb; p.a2_bytes = (int)a2b;
  const int hs = try_halo(p, workspace, workspace_floats, (hipStream_t)stream);
  return hs >= 0 ? hs : SDMOE_EUNSUP;
}

extern "C" int sdmoe_groupnorm_apply(const void* X, long ldx, int nimg, int HW, int C, const float* scale,
                                     const float* shift, int silu, void* Y, long ldy, void* stream) {
  if (!X || !Y || !scale || !shift || nimg <= 0 || HW <= 0 || C <= 0) return SDMOE_EARG;
  if (C % 8 || ldx % 8 || ldy % 8) return SDMOE_ESHAPE;
  const long rows = (long)nimg * HW;
  gn_apply_kernel<<<grid_for(rows * (C / 8)), 256, 0, (hipStream_t)stream>>>(
      (const half_t*)X, ldx, HW, C, scale, shift, silu, (half_t*)Y, ldy, rows);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_wmask_kmajor(const void* bits, long ldb, int N, int K, const int* perm, void* out, void* stream) {
  if (N == 0) return SDMOE_OK;
  if (!bits || !out || N < 0 || K <= 0) return SDMOE_EARG;
  if (K % 64 || ldb < K / 8) return SDMOE_ESHAPE;
  wmask_kmajor_kernel<<<grid_for((long)(K / 64) * N), 256, 0, (hipStream_t)stream>>>(
      (const uint8_t*)bits, ldb, N, K, perm, (unsigned long long*)out);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_mask_weight(const void* W, const void* bits, long N, long K, void* Wm, void* stream) {
  if (!W || !bits || !Wm || N <= 0 || K <= 0) return SDMOE_EARG;
  if (K % 8) return SDMOE_ESHAPE;
  const long n8 = N * K / 8;
  mask_weight_kernel<<<grid_for(n8), 256, 0, (hipStream_t)stream>>>((const half_t*)W, (const uint8_t*)bits,
                                                                   (half_t*)Wm, n8);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

int sdmoe_attn_set_nqf(int v);  // attention.hip
int sdmoe_gn_set_fused(int v);  // norm.hip
extern int g_topk_tpw;          // moe.hip

extern "C" int sdmoe_tune(int knob, int value) {
  if (knob == 4) return sdmoe_attn_set_nqf(value);
  if (knob == 7) return sdmoe_gn_set_fused(value);
  if (knob == 0 && (value == 0 || value == 2 || value == 3)) { g_stages = value; return SDMOE_OK; }
  if (knob == 1 && value >= 0 && value <= 8) { g_tile = value; return SDMOE_OK; }
  if (knob == 9 && value >= 0 && value <= 32) { g_ksplit = value; return SDMOE_OK; }
  if (knob == 14 && (value == 0 || value == 1)) { g_mfast = value; return SDMOE_OK; }
  if (knob == 6 && value >= 0 && value <= 63) { g_diag = value; return SDMOE_OK; }
  if (knob == 8 && (value == 0 || value == 1)) { g_res16 = value; return SDMOE_OK; }
  if (knob == 15 && (value == 0 || value == 1 || value == 4)) { g_topk_tpw = value; return SDMOE_OK; }
  if (knob == 16 && value >= 0 && value <= 3) { g_halo = value; return SDMOE_OK; }
  if (knob == 20 && (value == 0 || value == 1)) { g_gt320 = value; return SDMOE_OK; }
  if (knob == 21 && (value == 0 || value == 1)) { g_narrow = value; return SDMOE_OK; }
  if (knob == 23 && value >= 0 && value <= 2) { g_epi_direct = value; return SDMOE_OK; }
  return SDMOE_EARG;
}
