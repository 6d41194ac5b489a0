// CLIP text encoder helpers for gfx950 (the prompt encoder in front of the denoising loop,
// and the reference's hook_module='text' seam, base_receiver.py:59-65 / remove_wanda_neurons_fast.py:114-120).
// Everything GEMM-shaped in the encoder (fused QKV, out_proj, fc1 + quick_gelu, fc2 + residual) runs on
// sdmoe_linear; these kernels cover the rest:
//   * sdmoe_gather_rows: out[r] = table[idx[r]] (+ add[r % period]) — token + position embedding
//     (CLIPTextEmbeddings) and the end-of-text pooling row gather (CLIPTextTransformer pooled_output);
//   * sdmoe_attention_short: causal (or full) softmax(Q K^T * scale) V for short sequences (N <= 128, CLIP's 77
//     tokens), one workgroup per (sequence, head) with K and V resident in LDS — the 77-token, 64-wide heads are
//     far below the flash kernel's 128-key tiles, and this path is < 0.1 % of a 50-step pipeline call.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

// one thread per 16-B chunk of an output row
__global__ __launch_bounds__(256) void gather_rows_kernel(const half_t* __restrict__ T, long ldt,
                                                          const int* __restrict__ idx, int R, int C,
                                                          const half_t* __restrict__ A, long lda, int period,
                                                          half_t* __restrict__ Y, long ldy) {
  const int cpr = C / 8;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= (long)R * cpr) return;
  const int r = (int)(t / cpr), c = (int)(t % cpr) * 8;
  half8 v = *reinterpret_cast<const half8*>(T + (long)idx[r] * ldt + c);
  if (A) {
    const half8 a = *reinterpret_cast<const half8*>(A + (long)(r % period) * lda + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (half_t)((float)v[j] + (float)a[j]);
  }
  *reinterpret_cast<half8*>(Y + (long)r * ldy + c) = v;
}

constexpr int SHORT_MAXN = 128;
constexpr int SHORT_MAXD = 128;

// Block = 4 waves for one (sequence b, head h). K/V rows in LDS with an odd dword stride (D/2 + 1) so the 64
// lanes of a wave reading 64 different key rows at the same column hit 64 different banks. One wave per query
// row: lanes own keys (lane, lane + 64), exact fp32 softmax with wave reductions, then lanes own output columns.
__global__ __launch_bounds__(256) void attention_short_kernel(const half_t* __restrict__ Q, long ldq,
                                                              const half_t* __restrict__ K, long ldk,
                                                              const half_t* __restrict__ V, long ldv,
                                                              half_t* __restrict__ O, long ldo, int N, int heads,
                                                              int D, float scale, int causal) {
  __shared__ uint32_t ks[SHORT_MAXN * (SHORT_MAXD / 2 + 1)];
  __shared__ half_t vs[SHORT_MAXN * SHORT_MAXD];
  __shared__ float qs[4][SHORT_MAXD];
  __shared__ float ps[4][SHORT_MAXN];
  const int b = blockIdx.x / heads, h = blockIdx.x % heads;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kst = D / 2 + 1;  // K row stride in dwords
  const long row0 = (long)b * N;
  const int col0 = h * D;
  // stage K (as dword pairs, padded stride) and V (dense) for this head
  for (int i = threadIdx.x; i < N * (D / 2); i += 256) {
    const int r = i / (D / 2), c = i % (D / 2);
    ks[r * kst + c] = *reinterpret_cast<const uint32_t*>(K + (row0 + r) * ldk + col0 + 2 * c);
  }
  for (int i = threadIdx.x; i < N * (D / 8); i += 256) {
    const int r = i / (D / 8), c = (i % (D / 8)) * 8;
    *reinterpret_cast<half8*>(vs + r * D + c) = *reinterpret_cast<const half8*>(V + (row0 + r) * ldv + col0 + c);
  }
  __syncthreads();
  for (int i = wave; i < N; i += 4) {
    for (int c = lane; c < D; c += 64) qs[wave][c] = (float)Q[(row0 + i) * ldq + col0 + c] * scale;
    __builtin_amdgcn_wave_barrier();
    const int nk = causal ? i + 1 : N;
    float s[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = lane + 64 * u;
      s[u] = -INFINITY;
      if (j < nk) {
        float acc = 0.f;
        const uint32_t* kr = ks + j * kst;
        for (int c = 0; c < D / 2; ++c) {
          const uint32_t w = kr[c];
          const half2_t kv = __builtin_bit_cast(half2_t, w);
          acc += qs[wave][2 * c] * (float)kv[0] + qs[wave][2 * c + 1] * (float)kv[1];
        }
        s[u] = acc;
      }
    }
    const float m = wave_max(fmaxf(s[0], s[1]));
    float p0 = lane < nk ? __expf(s[0] - m) : 0.f;
    float p1 = lane + 64 < nk ? __expf(s[1] - m) : 0.f;
    const float inv = 1.0f / wave_sum(p0 + p1);
    ps[wave][lane] = p0;
    ps[wave][lane + 64] = p1;
    __builtin_amdgcn_wave_barrier();
    for (int c = lane; c < D; c += 64) {
      float acc = 0.f;
      for (int j = 0; j < nk; ++j) acc += ps[wave][j] * (float)vs[j * D + c];
      O[(row0 + i) * ldo + col0 + c] = (half_t)(acc * inv);
    }
    __builtin_amdgcn_wave_barrier();  // qs / ps of this wave are rewritten by its next row
  }
}

}  // namespace

extern "C" int sdmoe_gather_rows(const void* table, long ld_table, const int* idx, int R, int C, const void* add,
                                 long ld_add, int period, void* out, long ld_out, void* stream) {
  if (R == 0) return SDMOE_OK;
  if (!table || !idx || !out || R < 0 || C <= 0) return SDMOE_EARG;
  if (C % 8 || ld_table % 8 || ld_out % 8 || (add && (ld_add % 8 || period <= 0))) return SDMOE_ESHAPE;
  const long work = (long)R * (C / 8);
  gather_rows_kernel<<<(unsigned)((work + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      (const half_t*)table, ld_table, idx, R, C, (const half_t*)add, ld_add, period, (half_t*)out, ld_out);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_attention_short(const void* Q, long ldq, const void* K, long ldk, const void* V, long ldv,
                                     void* O, long ldo, int nseq, int N, int heads, int head_dim, float scale,
                                     int causal, void* stream) {
  if (nseq == 0) return SDMOE_OK;
  if (!Q || !K || !V || !O || nseq < 0 || N <= 0 || heads <= 0 || head_dim <= 0) return SDMOE_EARG;
  if (N > SHORT_MAXN || head_dim > SHORT_MAXD || head_dim % 8 || ldq % 2 || ldk % 2 || ldv % 8)
    return SDMOE_ESHAPE;
  attention_short_kernel<<<nseq * heads, 256, 0, (hipStream_t)stream>>>(
      (const half_t*)Q, ldq, (const half_t*)K, ldk, (const half_t*)V, ldv, (half_t*)O, ldo, N, heads, head_dim,
      scale, causal);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
