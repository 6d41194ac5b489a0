// Flash-style attention forward for the SD U-Net (self-attention N<=4096 and cross-attention, 77 keys),
// fp16 in/out, fp32 softmax/accumulate, head_dim D in {32, 40, 64, 80, 160}.
//
// Replaces diffusers Attention + AttnProcessor (softmax(QK^T/sqrt(d))V) on the hot path.
// Layout: Q/K/V/O are read straight out of the projection GEMM outputs ([tokens, heads*D] rows with an
// arbitrary row stride, so a fused QKV or KV projection needs no split/transposes).
//
// Structure (one 256-thread workgroup = 4 waves = 128 queries of one (image, head)):
//   * "swapped" product S^T = K Q^T with v_mfma_f32_16x16x32_f16: the query sits on the MFMA lane, so the
//     running max / sum / output rescale of the online softmax are lane-local (two shuffles per tile for
//     the max only; the row sum is kept as lane partials and combined once at the end);
//   * the S^T accumulator, converted to fp16, is directly the B operand of O^T = V^T P^T with a key
//     permutation inside each 32-key slot; V^T comes out of LDS with ds_read_b64_tr_b16 (gfx950 transpose
//     read), with the same permutation, so no LDS round trip for P;
//   * K/V tiles of 64 keys are register-prefetched (issue before the tile's MFMAs, LDS write after).
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

template <int D>
__global__ __launch_bounds__(256, (D >= 160 ? 1 : 2)) void attn_fwd_kernel(AttnParams p) {
  constexpr int DK = ((D + 31) / 32) * 32;   // contraction dim padded for 16x16x32
  constexpr int DV = ((D + 15) / 16) * 16;   // output dim padded to 16-row fragments
  constexpr int KB = 64;                      // keys per tile
  constexpr int KS = DK + 8;                  // K row stride (halves): +16 B pad -> conflict-free b128
  constexpr int VS = DV + 4;                  // V row stride (halves): 8-B aligned rows for tr reads
  constexpr int NDC = DK / 32, NDF = DV / 16;
  constexpr int CH = D / 8;                   // 16-B chunks per row
  constexpr int TOT = KB * CH;
  constexpr int PER = (TOT + 255) / 256;
  constexpr bool SUM_BY_MFMA = DV > D;     // V column D = 1.0 -> O^T row D accumulates sum_k P[k][q]
  constexpr float RESCALE_THR = 8.0f;

  __shared__ __attribute__((aligned(16))) half_t Ks[KB * KS];
  __shared__ __attribute__((aligned(16))) half_t Vs[KB * VS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, w = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 128 + wave * 32;

  const half_t* Qb = p.Q + (long)b * p.Nq * p.ldq + h * D;
  const half_t* Kb = p.K + (long)b * p.Nk * p.ldk + h * D;
  const half_t* Vb = p.V + (long)b * p.Nk * p.ldv + h * D;

  // zero the padding columns once (tiles never write them)
  for (int i = tid; i < KB * (KS - D); i += 256) {
    int r = i / (KS - D), c = D + i % (KS - D);
    Ks[r * KS + c] = (half_t)0.f;
  }
  for (int i = tid; i < KB * (VS - D); i += 256) {
    int r = i / (VS - D), c = D + i % (VS - D);
    Vs[r * VS + c] = (half_t)((SUM_BY_MFMA && c == D) ? 1.f : 0.f);
  }

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[q = w][d = 32c + 8g + j]
  half8 qf[2][NDC];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int c = 0; c < NDC; ++c) {
      const int q = q0 + f * 16 + w, d = 32 * c + 8 * g;
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q < p.Nq && d < D) v = *reinterpret_cast<const half8*>(Qb + (long)q * p.ldq + d);
      qf[f][c] = v;
    }

  float4v oacc[2][NDF];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int d = 0; d < NDF; ++d) oacc[f][d] = (float4v){0.f, 0.f, 0.f, 0.f};
  float mrun[2] = {-1e30f, -1e30f}, lrun[2] = {0.f, 0.f};

  uint4v rk[PER], rv[PER];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + 256 * i;
      uint4v a = {0u, 0u, 0u, 0u}, c = {0u, 0u, 0u, 0u};
      if (id < TOT) {
        const int r = id / CH, ch = id - r * CH;
        const int key = kt * KB + r;
        if (key < p.Nk) {
          a = *reinterpret_cast<const uint4v*>(Kb + (long)key * p.ldk + ch * 8);
          c = *reinterpret_cast<const uint4v*>(Vb + (long)key * p.ldv + ch * 8);
        }
      }
      rk[i] = a; rv[i] = c;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + 256 * i;
      if (id < TOT) {
        const int r = id / CH, ch = id - r * CH;
        *reinterpret_cast<uint4v*>(Ks + r * KS + ch * 8) = rk[i];
        // V rows are only 8-B aligned (VS*2 bytes): store as two 8-B halves
        uint2* vd = reinterpret_cast<uint2*>(Vs + r * VS + ch * 8);
        vd[0] = (uint2){rv[i][0], rv[i][1]};
        vd[1] = (uint2){rv[i][2], rv[i][3]};
      }
    }
  };

  const int nkt = (p.Nk + KB - 1) / KB;
  load_tile(0);
  __syncthreads();
  store_tile();
  __syncthreads();

  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt) load_tile(kt + 1);

    // ---- S^T = K Q^T for the 4 key fragments of this tile
    float4v s[2][4];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int kf = 0; kf < 4; ++kf) s[f][kf] = (float4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int c = 0; c < NDC; ++c) {
        half8 a = *reinterpret_cast<const half8*>(Ks + (kf * 16 + w) * KS + 32 * c + 8 * g);
#pragma unroll
        for (int f = 0; f < 2; ++f) s[f][kf] = mfma16x16x32(a, qf[f][c], s[f][kf]);
      }

    // ---- online softmax (query on the lane), VALU-lean:
    //  * raw-score max (scale > 0 commutes with max), scale folded into the exp2 argument: p = 2^(s*c - m);
    //  * key masking only on the ragged last tile (uniform branch);
    //  * deferred rescale: the running max moves only when some query's tile max exceeds it by > RESCALE_THR
    //    (log2 units), so most tiles skip the O/l rescale; p <= 2^RESCALE_THR stays well inside fp16;
    //  * for D with a pad column (D = 40) the row sum comes out of the PV MFMA (V pad column = 1.0).
    const int kbase = kt * KB;
    const bool ragged = kbase + KB > p.Nk;
    half8 pb[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (ragged) {
#pragma unroll
        for (int kf = 0; kf < 4; ++kf)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (kbase + kf * 16 + 4 * g + i >= p.Nk) s[f][kf][i] = -INFINITY;
      }
      float mx = fmaxf(fmaxf(s[f][0][0], s[f][0][1]), fmaxf(s[f][0][2], s[f][0][3]));
#pragma unroll
      for (int kf = 1; kf < 4; ++kf)
        mx = fmaxf(mx, fmaxf(fmaxf(s[f][kf][0], s[f][kf][1]), fmaxf(s[f][kf][2], s[f][kf][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mxs = mx * p.scale_log2;
      if (!__all(mxs - mrun[f] <= RESCALE_THR)) {  // wave-uniform decision
        const float mnew = fmaxf(mrun[f], mxs);
        const float alpha = __builtin_amdgcn_exp2f(mrun[f] - mnew);
        mrun[f] = mnew;
        if (!SUM_BY_MFMA) lrun[f] *= alpha;
#pragma unroll
        for (int d = 0; d < NDF; ++d) oacc[f][d] *= alpha;
      }
      const float nm = -mrun[f];
      float ls = 0.f;
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[f][kf][i], p.scale_log2, nm));
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

    // ---- O^T += V^T P^T (V^T via transpose reads, key slots permuted to match P)
    const int tq = w >> 2, tp = w & 3;
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
      for (int df = 0; df < NDF; ++df) {
        half4 lo = ds_read_tr(Vs + (32 * c2 + 4 * g + tq) * VS + 16 * df + 4 * tp);
        half4 hi = ds_read_tr(Vs + (32 * c2 + 16 + 4 * g + tq) * VS + 16 * df + 4 * tp);
        half8 a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int f = 0; f < 2; ++f) oacc[f][df] = mfma16x16x32(a, pb[f][c2], oacc[f][df]);
      }

    __syncthreads();
    if (kt + 1 < nkt) store_tile();
    __syncthreads();
  }

  // ---- normalise and store O[q][d] (lane: query w, rows d = 16df + 4g + i)
  half_t* Ob = p.O + (long)b * p.Nq * p.ldo + h * D;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
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

template <int D>
int launch(const AttnParams& p, int nimg, hipStream_t s) {
  dim3 grid((p.Nq + 127) / 128, p.heads, nimg);
  attn_fwd_kernel<D><<<grid, 256, 0, s>>>(p);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

}  // namespace

extern "C" int sdmoe_attention(const void* Q, long ldq, const void* K, long ldk, const void* V, long ldv,
                               void* O, long ldo, int nimg, int Nq, int Nk, int heads, int head_dim,
                               float scale, void* stream) {
  if (!Q || !K || !V || !O || nimg <= 0 || Nq <= 0 || Nk <= 0 || heads <= 0) return SDMOE_EARG;
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
