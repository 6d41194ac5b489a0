// Flash-style attention forward for the SD U-Net (self-attention N<=4096 and cross-attention, 77 keys),
// fp16 in/out, fp32 softmax/accumulate, head_dim D in {32, 40, 64, 80, 160}.
//
// Replaces diffusers Attention + AttnProcessor (softmax(QK^T/sqrt(d))V) on the hot path.
// Layout: Q/K/V/O are read straight out of the projection GEMM outputs ([tokens, heads*D] rows with an
// arbitrary row stride, so a fused QKV or KV projection needs no split/transposes).
//
// Structure (one 256-thread workgroup = 4 waves x 16*NQF queries of one (image, head); NQF = 2 by default, 4 on
// request -- it amortises every K/V LDS read and LDS-DMA piece over 64 queries per wave, but measured no faster):
//   * "swapped" product S^T = K Q^T with v_mfma_f32_16x16x32_f16: the query sits on the MFMA lane, so the
//     running max / sum / output rescale of the online softmax are lane-local (two shuffles per tile for
//     the max only; the row sum is kept as lane partials and combined once at the end);
//   * the S^T accumulator, converted to fp16, is directly the B operand of O^T = V^T P^T with a key
//     permutation inside each 32-key slot; V^T comes out of LDS with ds_read_b64_tr_b16 (gfx950 transpose
//     read), with the same permutation, so no LDS round trip for P;
//   * K/V tiles of 64 keys arrive by LDS-DMA (buffer_load ... lds, out-of-range keys and padding slots read
//     as zeros) into a double-buffered ring: tile kt+1 is issued before tile kt's MFMAs, one barrier per tile.
#include <type_traits>

#include "common.h"
#include "../../include/sdmoe.h"

namespace {

struct AttnParams {
  const half_t* Q; long ldq;
  const half_t* K; long ldk;
  const half_t* V; long ldv;
  half_t* O; long ldo;
  int Nq, Nk, heads;
  float scale_log2;
};

SDMOE_DEV half4 ds_read_tr(const half_t* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4 __attribute__((address_space(3)))*)(p));
  return __builtin_bit_cast(half4, v);
}

// This file is compiled with -fno-honor-nans (csrc/Makefile): fmaxf chains on MFMA results then lower to
// v_max3_f32 without a canonicalising v_max in front of each operand. (Inline-asm v_max3 is not an option:
// the hazard recognizer does not pad an asm VALU read of a just-written MFMA result.)
SDMOE_DEV float max3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
SDMOE_DEV float max2(float a, float b) { return fmaxf(a, b); }
// max over the 4 lanes {l, l^16, l^32, l^48} with the gfx950 cross-row swaps (no LDS round trip)
SDMOE_DEV float max_xrows(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = max2(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return max2(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

typedef __attribute__((address_space(3))) void lds_void_t;
SDMOE_DEV void bld16(__amdgpu_buffer_rsrc_t rs, const half_t* lds_dst, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 16, voff, 0, 0, 0);
}

template <int D, int NQF, int NW = 4>
__global__ __launch_bounds__(NW * 64, (D >= 160 || NW >= 8 ? 1 : 2)) void attn_fwd_kernel(AttnParams p) {
  constexpr int DK = ((D + 31) / 32) * 32;   // contraction dim padded for 16x16x32
  constexpr int DV = ((D + 15) / 16) * 16;   // output dim padded to 16-row fragments
  constexpr int KB = 64;                      // keys per tile
  // K and V row stride (halves) in LDS: the smallest odd multiple of 16 >= D (48, 80, 176 for D = 40, 80, 160)
  // makes both the ds_read_b128 K-fragment reads and the ds_read_b64_tr_b16 V^T reads bank-conflict-free. A K
  // row may be shorter than DK: the fragment read of columns D..DK-1 then runs into the next row (or the
  // zeroed tail), harmless because the matching Q columns are zero.
  constexpr int RS = ((D + 15) / 16) % 2 ? ((D + 15) / 16) * 16 : ((D + 15) / 16) * 16 + 16;
  constexpr int NDC = DK / 32, NDF = DV / 16;
  constexpr int CH = D / 8;                   // real 16-B chunks per row
  constexpr int SL = RS / 8;                  // 16-B LDS slots per row (SL - CH padding slots, loaded as zeros)
  constexpr int TILE = KB * RS;               // halves per K (or V) tile image
  constexpr int NPIECE = TILE * 2 / 1024;     // 1-KiB LDS-DMA wave-instructions per K (or V) tile
  constexpr int NPW = (2 * NPIECE + NW - 1) / NW;  // per wave, K and V together (the last round may be partial)
  constexpr int KBUF = TILE + 64;             // + zeroed tail for the over-read of the last K row
  constexpr bool SUM_BY_MFMA = DV > D;        // O^T row D accumulates sum_k P[k][q] (V column D := 1.0)
  static_assert(!SUM_BY_MFMA || D % 16 == 8, "ones column sits at the start of a 4-column tr-read group");
  constexpr float RESCALE_THR = 8.0f;
  constexpr unsigned OOB = 0x80000000u;

  // separate arrays per ring slot: with the slot a compile-time constant the compiler can tell the DMA into
  // one slot from the ds_reads of the other and does not drain vmcnt in front of every LDS read
  // slot layout: [K tile | zero tail | V tile]
  constexpr int SLOT = KBUF + TILE;
  __shared__ __attribute__((aligned(1024))) half_t S0[SLOT];
  __shared__ __attribute__((aligned(1024))) half_t S1[SLOT];
  // the ones column's V^T operand: 16 rows of [1 0 0 0] at a 32-B row stride, offset 16 B into each row, so the 16
  // lanes that read it take banks 4-5 (mod 8) of distinct 8-bank groups, beside the V-tile lanes' banks 0-3 and 6-7
  // of the same read (a single shared [1 0 0 0] block read by all 16 lanes cost 2 conflict cycles per read)
  __shared__ __attribute__((aligned(1024))) half_t ONES[SUM_BY_MFMA ? 16 * 16 : 1];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, w = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * (NW * 16 * NQF) + wave * (16 * NQF);

  const half_t* Qb = p.Q + (long)b * p.Nq * p.ldq + h * D;
  const half_t* Kb = p.K + (long)b * p.Nk * p.ldk + h * D;
  const half_t* Vb = p.V + (long)b * p.Nk * p.ldv + h * D;
  // buffer resources end at the last key's row: keys >= Nk (ragged last tile) read as zeros
  const __amdgpu_buffer_rsrc_t rsK =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kb, (short)0, (int)(((long)p.Nk - 1) * p.ldk * 2 + D * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsV =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vb, (short)0, (int)(((long)p.Nk - 1) * p.ldv * 2 + D * 2), 0x00020000);

  // per-wave LDS-DMA pieces: global piece gp = wave + NW j (K pieces first, then V); lane = one 16-B slot
  unsigned voff[NPW], vstep[NPW];
  int ldsoff[NPW];
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int gp = wave + NW * j;
    const bool isk = gp < NPIECE;
    const int pc = isk ? gp : gp - NPIECE;
    const int slot = pc * 64 + lane, r = slot / SL, c = slot - (slot / SL) * SL;
    const long ld = isk ? p.ldk : p.ldv;
    voff[j] = c < CH ? (unsigned)(r * ld * 2 + c * 16) : OOB;
    vstep[j] = (unsigned)(KB * ld * 2);
    ldsoff[j] = (isk ? 0 : KBUF) + pc * 512;
  }
  auto issue_tile = [&](half_t* Sd) {  // DMA the tile at the current voff into ring slot Sd, advance voff
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      if ((2 * NPIECE) % NW == 0 || wave + NW * j < 2 * NPIECE)  // wave-uniform
        bld16(wave + NW * j < NPIECE ? rsK : rsV, Sd + ldsoff[j], voff[j]);
      voff[j] += vstep[j];
    }
  };

  // zeroed over-read tails, the constant [1 0 0 0 | 0 0 0 0] block the V^T reads of the ones column use
  for (int i = tid; i < KBUF - TILE; i += NW * 64) S0[TILE + i] = S1[TILE + i] = 0;
  if constexpr (SUM_BY_MFMA)
    for (int i = tid; i < 16 * 16; i += NW * 64) ONES[i] = (half_t)(i % 16 == 8 ? 1.f : 0.f);

  const int nkt = (p.Nk + KB - 1) / KB;
  issue_tile(S0);

  // Q fragments (B operand of S^T = K Q^T), pre-multiplied by scale*log2(e) so that the score accumulator is
  // already the exp2 argument: lane holds Q[q = w][d = 32c + 8g + j]
  half8 qf[NQF][NDC];
#pragma unroll
  for (int f = 0; f < NQF; ++f)
#pragma unroll
    for (int c = 0; c < NDC; ++c) {
      const int q = q0 + f * 16 + w, d = 32 * c + 8 * g;
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q < p.Nq && d < D) v = *reinterpret_cast<const half8*>(Qb + (long)q * p.ldq + d);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] * p.scale_log2);
      qf[f][c] = v;
    }

  float4v oacc[NQF][NDF];
#pragma unroll
  for (int f = 0; f < NQF; ++f)
#pragma unroll
    for (int d = 0; d < NDF; ++d) oacc[f][d] = (float4v){0.f, 0.f, 0.f, 0.f};
  float mrun[NQF], lrun[NQF];
#pragma unroll
  for (int f = 0; f < NQF; ++f) mrun[f] = lrun[f] = 0.f;

  // V^T fragment addresses (tr reads, key slots permuted to match P); the lanes of the ones column read the ONES
  // rows instead, the lanes past it the V tile's zero-loaded padding columns
  const int tq = w >> 2, tp = w & 3;
  auto vaddr = [&](const half_t* Vt, int c2, int hi, int df) -> const half_t* {
    const int normal = (32 * c2 + 16 * hi + 4 * g + tq) * RS + 16 * df + 4 * tp;
    if (SUM_BY_MFMA && df == D / 16 && 4 * tp == D % 16) return ONES + (4 * g + tq) * 16 + 8;
    return Vt + normal;
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto tile = [&](int kt, auto ragged_tag, auto buf_tag) {
    constexpr bool RAGGED = decltype(ragged_tag)::value;
    constexpr int BUF = decltype(buf_tag)::value;
    const half_t* Kt = BUF ? S1 : S0;
    const half_t* Vt = Kt + KBUF;
    // the other slot was last read in tile kt-1, which every wave finished before the previous barrier
    if (kt + 1 < nkt) issue_tile(BUF ? S0 : S1);

    // ---- S'^T = K Q~^T - m: the accumulator starts at -m (running max, log2 units), so after the MFMAs it
    //      holds exp2's argument directly (tile 0 starts at 0 and sets m from its own max)
    float4v s[NQF][4];
#pragma unroll
    for (int f = 0; f < NQF; ++f) {
      const float nm = -mrun[f];
#pragma unroll
      for (int kf = 0; kf < 4; ++kf) s[f][kf] = (float4v){nm, nm, nm, nm};
    }
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int c = 0; c < NDC; ++c) {
        half8 a = *reinterpret_cast<const half8*>(Kt + (kf * 16 + w) * RS + 32 * c + 8 * g);
#pragma unroll
        for (int f = 0; f < NQF; ++f) s[f][kf] = mfma16x16x32(a, qf[f][c], s[f][kf]);
      }

    // ---- online softmax (query on the lane), VALU-lean: per score one exp2, a third of a max3 and half a
    //      cvt_pk; deferred rescale (m moves only when a tile max exceeds it by > RESCALE_THR, log2 units, so
    //      p <= 2^8 stays well inside fp16); masking only in the peeled ragged last tile
    half8 pb[NQF][2];
#pragma unroll
    for (int f = 0; f < NQF; ++f) {
      if constexpr (RAGGED) {
#pragma unroll
        for (int kf = 0; kf < 4; ++kf)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (kt * KB + kf * 16 + 4 * g + i >= p.Nk) s[f][kf][i] = -INFINITY;
      }
      float m0 = max3(s[f][0][0], s[f][0][1], s[f][0][2]);
      float m1 = max3(s[f][0][3], s[f][1][0], s[f][1][1]);
      float m2 = max3(s[f][1][2], s[f][1][3], s[f][2][0]);
      float m3 = max3(s[f][2][1], s[f][2][2], s[f][2][3]);
      float m4 = max3(s[f][3][0], s[f][3][1], s[f][3][2]);
      m0 = max3(m0, m1, s[f][3][3]);
      m2 = max3(m2, m3, m4);
      // lane-local max: the wave-uniform rescale test needs no cross-lane step (all lane maxima <= THR iff all row
      // maxima are); the row max over the 4 lanes of a query (l, l^16, l^32, l^48) only where m moves
      const float ml = max2(m0, m2);
      if (kt == 0) {  // first tile: m = its max (O and l are still zero)
        const float mx = max_xrows(ml);
        mrun[f] = mx;
#pragma unroll
        for (int kf = 0; kf < 4; ++kf) s[f][kf] -= mx;
      } else if (!__all(ml <= RESCALE_THR)) {  // wave-uniform decision
        const float delta = fmaxf(max_xrows(ml), 0.f);
        mrun[f] += delta;
        const float alpha = __builtin_amdgcn_exp2f(-delta);
        if (!SUM_BY_MFMA) lrun[f] *= alpha;
#pragma unroll
        for (int d = 0; d < NDF; ++d) oacc[f][d] *= alpha;
#pragma unroll
        for (int kf = 0; kf < 4; ++kf) s[f][kf] -= delta;
      }
      float ls = 0.f;
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(s[f][kf][i]);
          s[f][kf][i] = e;
          if (!SUM_BY_MFMA) ls += e;
        }
      if (!SUM_BY_MFMA) lrun[f] += ls;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        half8 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = (half_t)s[f][2 * c2][i];
          v[4 + i] = (half_t)s[f][2 * c2 + 1][i];
        }
        pb[f][c2] = v;
      }
    }

    // ---- O^T += V^T P^T
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
      for (int df = 0; df < NDF; ++df) {
        half4 lo = ds_read_tr(vaddr(Vt, c2, 0, df));
        half4 hi = ds_read_tr(vaddr(Vt, c2, 1, df));
        half8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int f = 0; f < NQF; ++f) oacc[f][df] = mfma16x16x32(a, pb[f][c2], oacc[f][df]);
      }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile kt+1 have landed
    __syncthreads();
  };

  using F_ = std::integral_constant<bool, false>;
  using T_ = std::integral_constant<bool, true>;
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  const int nfull = p.Nk / KB;
  int kt = 0;
  for (; kt + 1 < nfull; kt += 2) {  // unrolled by the two ring slots
    tile(kt, F_(), B0());
    tile(kt + 1, F_(), B1());
  }
  if (kt < nfull) { tile(kt, F_(), B0()); ++kt; }
  if (kt < nkt) {
    if (kt & 1) tile(kt, T_(), B1());
    else tile(kt, T_(), B0());
  }

  // ---- normalise and store O[q][d] (lane: query w, rows d = 16df + 4g + i)
  half_t* Ob = p.O + (long)b * p.Nq * p.ldo + h * D;
#pragma unroll
  for (int f = 0; f < NQF; ++f) {
    float l;
    if (SUM_BY_MFMA) {
      // O^T row D (df = D/16, lane group g = (D%16)/4, register D%4) holds sum_k P[k][q]; broadcast to all g
      l = __shfl(oacc[f][D / 16][D % 4], ((D % 16) / 4) * 16 + w, 64);
    } else {
      l = lrun[f];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
    }
    const float inv = 1.0f / l;
    const int q = q0 + f * 16 + w;
    if (q >= p.Nq) continue;
#pragma unroll
    for (int df = 0; df < NDF; ++df) {
      const int d = 16 * df + 4 * g;
      if (d < D) {
        half4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (half_t)(oacc[f][df][i] * inv);
        *reinterpret_cast<half4*>(Ob + (long)q * p.ldo + d) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// attn32_kernel: the same flash-style forward on v_mfma_f32_32x32x16_f16, both products with the QUERY ON THE LANE:
//   S^T (32 keys x 32 queries per MFMA block) = K Q^T   -- A = K rows from LDS (ds_read_b128), B = Q^T in registers;
//   O^T (32 d x 32 queries)                   = V^T P^T -- A = V^T by ds_read_b64_tr_b16, B = P^T straight from the
//     S^T accumulator registers (registers 8s..8s+7 of a block = k-step s; the V^T reads use the same permuted keys).
// So the online-softmax state (running max m, sum l, the rescale of O) stays lane-local. Against the 16x16x32 kernel:
// half the MFMA instructions per tile (14 vs 28 at d = 40: each issue slot an MFMA holds is VALU time lost), the QK
// contraction padded only to 16 (40 -> 48, not 64), the exp2 argument -m kept as a persistent C operand (reloaded
// only when the deferred rescale moves m), one cross-lane max per tile.
// Row sums: by MFMA through a ones column at d = D where D % 32 leaves room in the last O^T block (d = 40, 80; the
// lanes that would read V column D read a constant [1 0 0 0] block instead), else as VALU partial sums.
// 4 waves x 32 queries per workgroup, 64-key K/V tiles in a double-buffered LDS-DMA ring, one barrier per tile.
typedef float float16v __attribute__((ext_vector_type(16)));

SDMOE_DEV float16v mfma32x32x16(half8 a, half8 b, float16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int D, int NW = 4>
__global__ __launch_bounds__(NW * 64, (D >= 160 || NW >= 8 ? 1 : 2)) void attn32_kernel(AttnParams p) {
  constexpr int NQC = (D + 15) / 16;                  // 16-deep QK contraction steps (d zero-padded to 16 NQC)
  constexpr int DQ = 16 * NQC;
  constexpr bool SUM_MFMA = (D % 32) != 0 && (D % 4) == 0;  // ones column at d = D inside the last O^T block
  // -m through the QK contraction when it has a spare column (d = 40 -> 48): K[:, D] := 1 (one ds_write per lane per
  // tile into the row's pad slot) and Q~[:, D] := -m (fp16), so S' = K Q~^T - m needs no C operand at all; else the
  // score MFMAs start from a 16-register -m vector
  constexpr bool ONES_K = (D % 16) == 8;
  constexpr int NDB = (D + (SUM_MFMA ? 1 : 0) + 31) / 32;   // 32-row blocks of O^T
  constexpr int KB = 64;                              // keys per tile
  constexpr int RS = DQ + 8;                          // K row stride (halves): RS/8 odd -> conflict-free K reads
  static_assert((RS / 8) % 2 == 1, "row stride must be an odd number of 16-B slots");
  constexpr int CH = D / 8;                           // real 16-B chunks per row (the rest load as zeros)
  constexpr int SL = RS / 8;
  // V row stride: SLV 16-B slots with SLV = 4 (mod 8), >= the 32 NDB columns the O^T blocks read, so the 8 rows x
  // 64 B of one V^T transposed read cover all 128 banks once (the K stride, 11 slots at d = 80, gave 3-way
  // conflicts); the columns past D load as zeros
  constexpr int SLV = ((4 * NDB + 3) / 8) * 8 + 4;
  constexpr int RSV = SLV * 8;
  constexpr int TILE = KB * RS, TILEV = KB * RSV;
  constexpr int NPK = TILE * 2 / 1024, NPV = TILEV * 2 / 1024;  // 1-KiB LDS-DMA wave-instructions per K / V tile
  static_assert(NPK * 1024 == TILE * 2 && NPV * 1024 == TILEV * 2, "tiles must be whole 1-KiB pieces");
  constexpr int NPW = (NPK + NPV + NW - 1) / NW;       // per wave (the last round partly empty)
  constexpr int TAIL = 64;                            // zeroed tail behind the K tile
  constexpr int VOFF = TILE + TAIL, SLOT = VOFF + TILEV;
  static_assert(SLV >= 4 * NDB, "V rows hold every column the O^T blocks read");
  constexpr float RESCALE_THR = 8.0f;
  constexpr unsigned OOB = 0x80000000u;
  __shared__ __attribute__((aligned(1024))) half_t S0[SLOT];
  __shared__ __attribute__((aligned(1024))) half_t S1[SLOT];
  // the ones column's V^T operand: one [1 0 0 0 | 0 0 0 0] slot per row class r = row mod 8, placed on the banks row r's
  // slot of column D would occupy in the V tile, so its 8 reader lanes neither share a slot nor collide with the others
  constexpr int ONES_AT = (VOFF / 8 + D / 8) % 32;    // 16-B unit of row 0's column-D slot, modulo the 512-B bank cycle
  __shared__ __attribute__((aligned(1024))) half_t ONES[SUM_MFMA ? 256 : 1];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ln = lane & 31, hf = lane >> 5;           // query column of the MFMA blocks, lane half
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * (32 * NW) + wave * 32;

  const half_t* Qb = p.Q + (long)b * p.Nq * p.ldq + h * D;
  const half_t* Kb = p.K + (long)b * p.Nk * p.ldk + h * D;
  const half_t* Vb = p.V + (long)b * p.Nk * p.ldv + h * D;
  const __amdgpu_buffer_rsrc_t rsK =
      __builtin_amdgcn_make_buffer_rsrc((void*)Kb, (short)0, (int)(((long)p.Nk - 1) * p.ldk * 2 + D * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsV =
      __builtin_amdgcn_make_buffer_rsrc((void*)Vb, (short)0, (int)(((long)p.Nk - 1) * p.ldv * 2 + D * 2), 0x00020000);

  unsigned voff[NPW], vstep[NPW];
  int ldsoff[NPW];
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int gp = wave + NW * j;
    const bool isk = gp < NPK;
    const int pc = isk ? gp : gp - NPK;
    const int sl = isk ? SL : SLV;
    const int slot = pc * 64 + lane, r = slot / sl, c = slot - (slot / sl) * sl;
    const long ld = isk ? p.ldk : p.ldv;
    voff[j] = c < CH ? (unsigned)(r * ld * 2 + c * 16) : OOB;
    vstep[j] = (unsigned)(KB * ld * 2);
    ldsoff[j] = (isk ? 0 : VOFF) + pc * 512;
  }
  auto issue_tile = [&](half_t* Sd) {
#pragma unroll
    for (int j = 0; j < NPW; ++j) {
      if ((NPK + NPV) % NW == 0 || wave + NW * j < NPK + NPV) bld16(wave + NW * j < NPK ? rsK : rsV, Sd + ldsoff[j], voff[j]);
      voff[j] += vstep[j];
    }
  };

  for (int i = tid; i < TAIL; i += NW * 64) S0[TILE + i] = S1[TILE + i] = 0;
  if constexpr (SUM_MFMA) {
    for (int i = tid; i < 256; i += NW * 64) {
      const int u = i / 8;  // 16-B unit; row class r sits at unit (ONES_AT + SLV r) mod 32
      bool one = false;
#pragma unroll
      for (int r = 0; r < 8; ++r) one |= (i % 8 == 0) && u == (ONES_AT + SLV * r) % 32;
      ONES[i] = (half_t)(one ? 1.f : 0.f);
    }
  }

  const int nkt = (p.Nk + KB - 1) / KB;
  issue_tile(S0);

  // Q^T fragments (B operand): lane holds Q[q0 + ln][16c + 8hf .. +8], prescaled by scale*log2(e) so the score
  // accumulator is already exp2's argument; zero past D and past Nq
  half8 qf[NQC];
#pragma unroll
  for (int c = 0; c < NQC; ++c) {
    const int q = q0 + ln, d = 16 * c + 8 * hf;
    half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q < p.Nq && d < D) v = *reinterpret_cast<const half8*>(Qb + (long)q * p.ldq + d);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] * p.scale_log2);
    qf[c] = v;
  }

  float16v oacc[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) oacc[db] = (float16v)(0.f);
  float16v negm = (float16v)(0.f);  // -m in every register: the initial accumulator of the score MFMAs (!ONES_K)
  float mrun = 0.f, lrun = 0.f;      // ONES_K: mrun is the fp16-representable shift actually in Q~[:, D]
  auto set_shift = [&](float m) {    // lanes of the upper half hold d = 16 (NQC-1) + 8 = D in element 0
    if constexpr (ONES_K) {
      if (hf) qf[NQC - 1][0] = (half_t)(-m);
    } else {
      negm = (float16v)(-m);
    }
  };

  // V^T operand addresses: lane (group g16 = lane / 16, index 4 tq + tp in it) supplies row 4 hf + tq (+ 8 for the
  // second read) and columns 16 (g16 & 1) + 4 tp of its 4 x 16 transposed-read block
  const int gi = lane & 15, g16 = lane >> 4, tq = gi >> 2, tp = gi & 3;
  const int vbase = VOFF + (4 * hf + tq) * RSV + 16 * (g16 & 1) + 4 * tp;
  const half_t* ones_at = ONES + 8 * ((ONES_AT + SLV * (4 * hf + tq)) % 32);  // rows 4 hf + tq (+ 8): same class
  const bool onecol = SUM_MFMA && (g16 & 1) == (D % 32) / 16 && tp == (D % 16) / 4;

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto tile = [&](int kt, auto ragged_tag, auto buf_tag, auto first_tag) {
    constexpr bool RAGGED = decltype(ragged_tag)::value;
    constexpr int BUF = decltype(buf_tag)::value;
    constexpr bool FIRST = decltype(first_tag)::value;  // the first tile sets m (peeled: no runtime merge of states)
    const half_t* St = BUF ? S1 : S0;
    if (kt + 1 < nkt) issue_tile(BUF ? S0 : S1);
    if constexpr (ONES_K) const_cast<half_t*>(St)[lane * RS + D] = (half_t)1.f;  // K[key][D] = 1 for this tile

    // ---- S^T = K Q~^T - m (two 32-key blocks)
    float16v s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = (FIRST || ONES_K) ? (float16v)(0.f) : negm;
#pragma unroll
      for (int c = 0; c < NQC; ++c) {
        const half8 a = *reinterpret_cast<const half8*>(St + (32 * kb + ln) * RS + 16 * c + 8 * hf);
        s[kb] = mfma32x32x16(a, qf[c], s[kb]);
      }
    }
    if constexpr (RAGGED) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * KB + 32 * kb + (r & 3) + 8 * (r >> 2) + 4 * hf >= p.Nk) s[kb][r] = -INFINITY;
    }
    // ---- online softmax, query on the lane: 32 scores here, the other 32 keys in lane ^ 32
    // lane-local max of the 32 scores: a balanced v_max3 tree (16 instructions); the row max over the lane pair
    // (l, l ^ 32) only where m is set or moves -- the wave-uniform rescale test needs none (every lane's maximum is
    // <= THR iff every row's is)
    auto sv = [&](int i) { return s[i >> 4][i & 15]; };
    float a1[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) a1[i] = max3(sv(3 * i), sv(3 * i + 1), sv(3 * i + 2));
    const float b0 = max3(a1[0], a1[1], a1[2]), b1 = max3(a1[3], a1[4], a1[5]), b2 = max3(a1[6], a1[7], a1[8]);
    const float b3 = max3(a1[9], sv(30), sv(31));
    const float ml = max2(max3(b0, b1, b2), b3);
    auto xmax = [](float v) {
      auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
      return max2(__uint_as_float(r[0]), __uint_as_float(r[1]));
    };
    if constexpr (FIRST) {  // first tile: m = its max (O and l are still zero)
      const float mx = xmax(ml);
      mrun = ONES_K ? (float)(half_t)mx : mx;
      set_shift(mrun);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) s[kb] -= mrun;
    } else if (!__all(ml <= RESCALE_THR)) {  // wave-uniform: deferred rescale (p <= 2^8 keeps fp16 safe)
      const float mx = xmax(ml);
      const float mnew = ONES_K ? (float)(half_t)(mrun + fmaxf(mx, 0.f)) : mrun + fmaxf(mx, 0.f);
      const float delta = mnew - mrun;  // exact: the shifts old and new are both in use as given
      mrun = mnew;
      set_shift(mrun);
      const float alpha = __builtin_amdgcn_exp2f(-delta);
      if (!SUM_MFMA) lrun *= alpha;
#pragma unroll
      for (int db = 0; db < NDB; ++db) oacc[db] *= alpha;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) s[kb] -= delta;
    }
    // ---- P = exp2(S'), packed to fp16 k-step fragments: registers 8cs..8cs+7 of block kb = keys 16cs + ...
    half8 pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[kb][r]);
        if (!SUM_MFMA) ls += e;
        pb[kb][r >> 3][r & 7] = (half_t)e;
      }
      if (!SUM_MFMA) lrun += ls;
    }
    // ---- O^T += V^T P^T over the four 16-key steps
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int cs = 0; cs < 2; ++cs)
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const half_t* a1 = St + vbase + (32 * kb + 16 * cs) * RSV + 32 * db;
          const half_t* a2 = a1 + 8 * RSV;
          if (SUM_MFMA && db == NDB - 1 && onecol) a1 = a2 = ones_at;
          const half4 lo = ds_read_tr(a1), hi = ds_read_tr(a2);
          const half8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          oacc[db] = mfma32x32x16(a, pb[kb][cs], oacc[db]);
        }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile kt+1 have landed
    __syncthreads();
  };

  using F_ = std::integral_constant<bool, false>;
  using T_ = std::integral_constant<bool, true>;
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  const int nfull = p.Nk / KB;
  int kt = 0;
  if (nfull == 0) {  // a single ragged tile (Nk < 64)
    tile(0, T_(), B0(), T_());
    kt = 1;
  } else {
    tile(0, F_(), B0(), T_());
    kt = 1;
    for (; kt + 1 < nfull; kt += 2) {
      tile(kt, F_(), B1(), F_());
      tile(kt + 1, F_(), B0(), F_());
    }
    if (kt < nfull) { tile(kt, F_(), B1(), F_()); ++kt; }
    if (kt < nkt) {
      if (kt & 1) tile(kt, T_(), B1(), F_());
      else tile(kt, T_(), B0(), F_());
    }
  }

  // ---- normalise and store: lane (query q0 + ln) holds O^T rows d = 32 db + 8 t + 4 hf + 0..3 in registers 4t..4t+3
  float l;
  if constexpr (SUM_MFMA) {
    constexpr int HD = ((D % 32) >> 2) & 1, TD = (D % 32) >> 3;
    l = __shfl(oacc[D / 32][4 * TD], HD * 32 + ln, 64);
  } else {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lrun), __float_as_uint(lrun), false, false);
    l = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const float inv = 1.0f / l;
  const int q = q0 + ln;
  if (q >= p.Nq) return;
  half_t* Orow = p.O + (long)b * p.Nq * p.ldo + h * D + (long)q * p.ldo;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int d = 32 * db + 8 * t + 4 * hf;
      if (d < D) {
        half4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (half_t)(oacc[db][4 * t + i] * inv);
        *reinterpret_cast<half4*>(Orow + d) = o;
      }
    }
}

// sdmoe_tune knob 4: 0 = by shape (default): attn32_kernel for d = 80 self-attention (Nk > 128), the 16x16x32 kernel
// in 8-wave workgroups for d = 40 / 64 self-attention (Nk > 128), the 4-wave 16x16x32 kernel (NQF = 2) everywhere
// else; 1 = attn32_kernel; 2 or 4 = the 4-wave 16x16x32 kernel with NQF = 2 / 4; 8 = the 16x16x32 kernel in
// 8-wave workgroups (d <= 80); 9 = attn32_kernel in 8-wave workgroups (d <= 80)
int g_attn_nqf = 0;

template <int D>
int launch(const AttnParams& p, int nimg, hipStream_t s) {
  // 64 queries per wave (NQF = 4) only on request (knob 4): at d = 40, N = 4096 it measured equal to NQF = 2
  // (500 us both; 232 vs 128 VGPRs halves the waves per SIMD) and 12 % slower on the 77-key cross-attention;
  // head dims above 40 would spill at NQF = 4 (64: 16 VGPRs, 80: 130)
  constexpr bool WIDE_OK = D <= 40;
  const bool wide = g_attn_nqf == 4;
  // same-box timings, 16 images x 8 heads, 16x16x32 vs 32x32x16 (us): d = 40 N = 4096 self 499 vs 524, 77-key cross
  // 34.1 vs 41.0; d = 64 N = 4096 630 vs 645, cross 43.4 vs 50.8; d = 80 N = 1024 self 66.9 vs 64.0 (the contraction
  // 80 -> 80 instead of 96), cross 21.4 vs 22.2; d = 160 19.2 vs 19.5. The 32x32x16 loop issues fewer instructions
  // (14 MFMAs and ~100 VALU per 64-key tile vs 28 and ~110 at d = 40) but runs slower: lower clock under DVFS for
  // the 32x32 MFMA (MI355X_MICROARCH.md) and 2-way LDS bank conflicts on its V^T transpose reads (row stride 56)
  const bool use32 = g_attn_nqf == 1 || (g_attn_nqf == 0 && D == 80 && p.Nk > 128);
  // 8-wave workgroups (256 queries share each K/V tile: half the LDS-DMA pieces per wave and tile) for the long
  // self-attentions at d = 40 / 64: d = 40 N = 4096 448 vs 464-475 us, pipeline +0.5 % (same box); slower on the
  // 77-key cross-attention (34.4 vs 31.1 us: fewer workgroups) and at d = 80 (65.4 vs 62.4 us with attn32)
  const bool use8 = g_attn_nqf == 8 || (g_attn_nqf == 0 && (D == 40 || D == 64) && p.Nk > 128);
  if (g_attn_nqf == 9 && D <= 80) {  // 32x32x16 kernel in 8-wave workgroups
    dim3 grid((p.Nq + 255) / 256, p.heads, nimg);
    attn32_kernel<D, (D <= 80 ? 8 : 4)><<<grid, (D <= 80 ? 512 : 256), 0, s>>>(p);
  } else if (use32) {
    dim3 grid((p.Nq + 127) / 128, p.heads, nimg);
    attn32_kernel<D><<<grid, 256, 0, s>>>(p);
  } else if (WIDE_OK && wide) {
    dim3 grid((p.Nq + 255) / 256, p.heads, nimg);
    attn_fwd_kernel<D, (WIDE_OK ? 4 : 2)><<<grid, 256, 0, s>>>(p);
  } else if (use8 && D <= 80) {
    dim3 grid((p.Nq + 255) / 256, p.heads, nimg);
    attn_fwd_kernel<D, 2, (D <= 80 ? 8 : 4)><<<grid, (D <= 80 ? 512 : 256), 0, s>>>(p);
  } else {
    dim3 grid((p.Nq + 127) / 128, p.heads, nimg);
    attn_fwd_kernel<D, 2><<<grid, 256, 0, s>>>(p);
  }
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

}  // namespace

int sdmoe_attn_set_nqf(int v) {
  if (v != 0 && v != 1 && v != 2 && v != 4 && v != 8 && v != 9) return SDMOE_EARG;
  g_attn_nqf = v;
  return SDMOE_OK;
}

extern "C" int sdmoe_attention(const void* Q, long ldq, const void* K, long ldk, const void* V, long ldv,
                               void* O, long ldo, int nimg, int Nq, int Nk, int heads, int head_dim,
                               float scale, void* stream) {
  if (nimg == 0 || Nq == 0) return SDMOE_OK;  // empty batch / no queries: nothing to write
  if (!Q || !K || !V || !O || nimg < 0 || Nq < 0 || Nk <= 0 || heads <= 0) return SDMOE_EARG;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4) return SDMOE_ESHAPE;
  AttnParams p{(const half_t*)Q, ldq, (const half_t*)K, ldk, (const half_t*)V, ldv, (half_t*)O, ldo,
               Nq, Nk, heads, scale * 1.4426950408889634f};
  hipStream_t s = (hipStream_t)stream;
  switch (head_dim) {
    case 32: return launch<32>(p, nimg, s);
    case 40: return launch<40>(p, nimg, s);
    case 64: return launch<64>(p, nimg, s);
    case 80: return launch<80>(p, nimg, s);
    case 160: return launch<160>(p, nimg, s);
    default: return SDMOE_EUNSUP;
  }
}
