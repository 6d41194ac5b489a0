// Skill-discovery statistics on the same hook seam as the routing kernels, gfx950:
//   sdmoe_expert_mean_topk  GetExperts.hook_fn (neuron_receivers/get_experts.py:50-83): expert scores averaged
//                           over every token (or the bounding-box tokens of each image), then top-k experts
//   sdmoe_colnorm_accum     Wanda.hook_fn (neuron_receivers/wanda_receiver.py:37-57) + utils.ColumnNormCalculator
//                           (utils.py:321-341): L2-normalise each token row of the GEGLU output, accumulate the
//                           squared column norms (the running sqrt(c^2 + n^2) of the reference, kept squared)
//   sdmoe_wanda_mask        modularity/wanda.py:140-160: per down-projection row, metric = |W| * act_norm; the top
//                           `kprune` adjusted-prompt metrics that also beat the base-prompt metric -> mask bits
// All three are HBM-streaming reductions (no MFMA): coalesced 16-B row reads, fp32 accumulation, fixed slab
// partitions and ordered combines so every result is deterministic run to run.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

constexpr int SLAB_ROWS = 256;  // rows per partial-sum slab (fixed: results do not depend on the grid)

// ---- expert score mean + top-k ------------------------------------------------------------------------------
// selected row r -> physical row: all rows (row_idx == null) or image r / n_idx, position row_idx[r % n_idx]
__global__ __launch_bounds__(256) void score_colsum_kernel(const half_t* __restrict__ S, long lds, int nsel, int E,
                                                           int rows_per_img, const int* __restrict__ row_idx,
                                                           int n_idx, float* __restrict__ part) {
  const int slab = blockIdx.x;
  const int r0 = slab * SLAB_ROWS, r1 = min(nsel, r0 + SLAB_ROWS);
  for (int e = threadIdx.x; e < E; e += 256) {
    float acc = 0.f;
    for (int r = r0; r < r1; ++r) {
      const long m = row_idx ? (long)(r / n_idx) * rows_per_img + row_idx[r % n_idx] : r;
      acc += (float)S[m * lds + e];
    }
    part[(long)slab * E + e] = acc;
  }
}

// one block: ordered slab combine, mean = fp16(sum * (1/n)) (torch's fp16 mean: fp32 accumulate, one rounding),
// then rank = #{j : v_j > v_e or (v_j == v_e and j < e)}; rank < k -> topk[rank] = e (descending, ties -> low id)
__global__ __launch_bounds__(1024) void score_mean_topk_kernel(const float* __restrict__ part, int nslab, int E,
                                                               float inv_n, int k, half_t* __restrict__ mean_out,
                                                               int* __restrict__ topk) {
  __shared__ float v[1024];
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < nslab; ++i) s += part[(long)i * E + e];
    const half_t h = (half_t)(s * inv_n);
    v[e] = (float)h;
    if (mean_out) mean_out[e] = h;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    const float ve = v[e];
    int rank = 0;
    for (int j = 0; j < E; ++j) {
      const float vj = v[j];
      rank += (vj > ve) || (vj == ve && j < e);
    }
    if (rank < k) topk[rank] = e;
  }
}

// ---- Wanda activation column norms --------------------------------------------------------------------------
// inv[m] = 1 / max(||P[m, :]||_2, 1e-12)   (F.normalize(p=2, dim=1)); one wave per row
__global__ __launch_bounds__(256) void row_invnorm_kernel(const half_t* __restrict__ P, long ldp, int M, int F,
                                                          float* __restrict__ inv) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (m >= M) return;
  const half_t* row = P + (long)m * ldp;
  float s = 0.f;
  for (int c = lane; c < F / 8; c += 64) {
    half8 v = *reinterpret_cast<const half8*>(row + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (float)v[j] * (float)v[j];
  }
  s = wave_sum(s);
  if (lane == 0) inv[m] = 1.0f / fmaxf(sqrtf(s), 1e-12f);
}

// part[slab][f] = sum over the slab's rows of (P[m, f] * inv[m])^2; block = 64 chunk-columns x 4 row lanes
__global__ __launch_bounds__(256) void colsq_partial_kernel(const half_t* __restrict__ P, long ldp, int M, int F,
                                                            const float* __restrict__ inv, float* __restrict__ part) {
  __shared__ float red[3][64][9];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk = blockIdx.x * 64 + lane;  // 8-column chunk
  const int slab = blockIdx.y;
  const int r0 = slab * SLAB_ROWS, r1 = min(M, r0 + SLAB_ROWS);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (chunk < F / 8) {
    for (int m = r0 + wave; m < r1; m += 4) {
      half8 v = *reinterpret_cast<const half8*>(P + (long)m * ldp + 8 * chunk);
      const float s = inv[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = (float)v[j] * s;
        acc[j] += x * x;
      }
    }
  }
  if (wave > 0)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave - 1][lane][j] = acc[j];
  __syncthreads();
  if (wave == 0 && chunk < F / 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = ((acc[j] + red[0][lane][j]) + red[1][lane][j]) + red[2][lane][j];
      part[(long)slab * F + 8 * chunk + j] = t;
    }
  }
}

__global__ __launch_bounds__(256) void colsq_combine_kernel(const float* __restrict__ part, int nslab, int F,
                                                            float* __restrict__ sumsq) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= F) return;
  float s = 0.f;
  for (int i = 0; i < nslab; ++i) s += part[(long)i * F + f];
  sumsq[f] += s;
}

// ---- Wanda mask: per row, top-kprune of metric_adj (ties -> lowest column) AND metric_adj > metric_base ----
SDMOE_DEV unsigned key16(half_t h) {  // metrics are >= 0: the raw fp16 bits order them (-0 -> 0)
  unsigned short u = __builtin_bit_cast(unsigned short, h);
  return (u & 0x8000) ? 0u : (unsigned)u;
}

SDMOE_DEV int block_sum(int v, int* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// one 256-thread block per row; F <= 8192, F % 8 == 0. Thread t owns 8-column chunks t, t+256, ... (round r =
// chunks [256r, 256r+256)), so "lower column" == (round, thread, j) lexicographic.
__global__ __launch_bounds__(256) void wanda_mask_kernel(const half_t* __restrict__ W, long ldw, int F,
                                                         const half_t* __restrict__ nb, const half_t* __restrict__ na,
                                                         int kprune, uint8_t* __restrict__ bits) {
  __shared__ unsigned short kadj[8192];
  __shared__ int red[4];
  __shared__ int scan[256];
  const int row = blockIdx.x, tid = threadIdx.x;
  const half_t* w = W + (long)row * ldw;
  const int nch = F / 8;
  // metric_adj = fp16(|W| * n_adj) as the reference's fp16 tensor product
  for (int c = tid; c < nch; c += 256) {
    half8 wv = *reinterpret_cast<const half8*>(w + 8 * c);
    half8 av = *reinterpret_cast<const half8*>(na + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const half_t m = (half_t)((float)__builtin_fabsf16(wv[j]) * (float)av[j]);
      kadj[8 * c + j] = (unsigned short)key16(m);
    }
  }
  __syncthreads();
  // MSB-first radix select of the kprune-th largest key
  unsigned prefix = 0;
  int need = kprune;
  for (int b = 15; b >= 0; --b) {
    const unsigned hi_mask = 0xffffu << (b + 1) & 0xffffu;
    int cnt = 0;
    for (int c = tid; c < nch; c += 256)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned k = kadj[8 * c + j];
        cnt += ((k & hi_mask) == prefix) && ((k >> b) & 1u);
      }
    cnt = block_sum(cnt, red);
    if (cnt >= need) prefix |= 1u << b;
    else need -= cnt;
  }
  // prefix = threshold key; `need` of the keys equal to it are selected, lowest columns first
  const unsigned thr = prefix;
  int tie_base = 0;
  for (int r = 0; r * 256 < nch; ++r) {
    const int c = r * 256 + tid;
    int ties = 0;
    if (c < nch)
#pragma unroll
      for (int j = 0; j < 8; ++j) ties += kadj[8 * c + j] == thr;
    scan[tid] = ties;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan
      const int add = tid >= o ? scan[tid - o] : 0;
      __syncthreads();
      scan[tid] += add;
      __syncthreads();
    }
    int before = tie_base + scan[tid] - ties;
    const int round_total = scan[255];
    if (c < nch) {
      half8 wv = *reinterpret_cast<const half8*>(w + 8 * c);
      half8 bv = *reinterpret_cast<const half8*>(nb + 8 * c);
      unsigned byte = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned k = kadj[8 * c + j];
        bool sel = k > thr;
        if (k == thr && kprune > 0) { sel = before < need; ++before; }
        const half_t mb = (half_t)((float)__builtin_fabsf16(wv[j]) * (float)bv[j]);
        const bool beats = k > key16(mb);  // metric_adj > metric_base (both >= 0: key order == value order)
        byte |= (sel && beats) ? (1u << j) : 0u;
      }
      bits[(long)row * nch + c] = (uint8_t)byte;
    }
    tie_base += round_total;
    __syncthreads();
  }
}

int nblocks(long n, int per) { return (int)((n + per - 1) / per); }

}  // namespace

extern "C" int sdmoe_expert_mean_topk(const void* score, long ld_score, int M, int E, int rows_per_img,
                                      const int* row_idx, int n_idx, int k, void* mean_out, int* topk_out,
                                      float* workspace, long workspace_floats, void* stream) {
  if (!score || !topk_out || !workspace || M <= 0 || E <= 0 || k < 0) return SDMOE_EARG;
  if (E > 1024 || k > E) return SDMOE_ESHAPE;
  if (row_idx && (n_idx <= 0 || rows_per_img <= 0 || M % rows_per_img)) return SDMOE_EARG;
  const int nsel = row_idx ? (M / rows_per_img) * n_idx : M;
  const int nslab = nblocks(nsel, SLAB_ROWS);
  if ((long)nslab * E > workspace_floats) return SDMOE_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  score_colsum_kernel<<<nslab, 256, 0, s>>>((const half_t*)score, ld_score, nsel, E, rows_per_img, row_idx, n_idx,
                                            workspace);
  SDMOE_CHECK_LAUNCH();
  score_mean_topk_kernel<<<1, 1024, 0, s>>>(workspace, nslab, E, 1.0f / (float)nsel, k, (half_t*)mean_out,
                                            topk_out);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_colnorm_accum(const void* P, long ldp, int M, int F, float* sumsq, float* workspace,
                                   long workspace_floats, void* stream) {
  if (!P || !sumsq || !workspace || M <= 0 || F <= 0) return SDMOE_EARG;
  if (F % 8 || ldp % 8) return SDMOE_ESHAPE;
  const int nslab = nblocks(M, SLAB_ROWS);
  if ((long)M + (long)nslab * F > workspace_floats) return SDMOE_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  float* inv = workspace;
  float* part = workspace + M;
  row_invnorm_kernel<<<nblocks(M, 4), 256, 0, s>>>((const half_t*)P, ldp, M, F, inv);
  SDMOE_CHECK_LAUNCH();
  colsq_partial_kernel<<<dim3(nblocks(F / 8, 64), nslab), 256, 0, s>>>((const half_t*)P, ldp, M, F, inv, part);
  SDMOE_CHECK_LAUNCH();
  colsq_combine_kernel<<<nblocks(F, 256), 256, 0, s>>>(part, nslab, F, sumsq);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_wanda_mask(const void* W, long ldw, int C, int F, const void* norm_base, const void* norm_adj,
                                int kprune, void* bits, void* stream) {
  if (!W || !norm_base || !norm_adj || !bits || C <= 0 || F <= 0 || kprune < 0) return SDMOE_EARG;
  if (F % 8 || ldw % 8 || F > 8192 || kprune > F) return SDMOE_ESHAPE;
  wanda_mask_kernel<<<C, 256, 0, (hipStream_t)stream>>>((const half_t*)W, ldw, F, (const half_t*)norm_base,
                                                        (const half_t*)norm_adj, kprune, (uint8_t*)bits);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

// ---- static "union-timesteps" mask (benchmarks/save_union_over_time.py:189-207) ----------------------------------
// out bit = (number of the T per-timestep masks with the bit set) > threshold (select_ratio * timesteps), over T
// bit-packed masks [T][nbytes] (t-th mask at bits + t * t_stride). One thread per 32-bit word: 32 counters in
// registers, one coalesced 4-B load per mask.
namespace {
__global__ __launch_bounds__(256) void union_over_time_kernel(const uint32_t* __restrict__ bits, long t_stride_words,
                                                              int T, long nwords, float thr,
                                                              uint32_t* __restrict__ out) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nwords; i += (long)gridDim.x * 256) {
    unsigned cnt[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) cnt[j] = 0;
    for (int t = 0; t < T; ++t) {
      const uint32_t w = bits[(long)t * t_stride_words + i];
#pragma unroll
      for (int j = 0; j < 32; ++j) cnt[j] += (w >> j) & 1u;
    }
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) o |= ((float)cnt[j] > thr ? 1u : 0u) << j;
    out[i] = o;
  }
}
}  // namespace

extern "C" int sdmoe_union_over_time(const void* bits, long t_stride_bytes, int T, long nbytes, float threshold,
                                     void* out, void* stream) {
  if (!bits || !out || T <= 0 || nbytes <= 0) return SDMOE_EARG;
  if (nbytes % 4 || t_stride_bytes % 4 || t_stride_bytes < nbytes) return SDMOE_ESHAPE;
  const long nw = nbytes / 4;
  long g = (nw + 255) / 256;
  if (g > 4096) g = 4096;
  union_over_time_kernel<<<(int)g, 256, 0, (hipStream_t)stream>>>((const uint32_t*)bits, t_stride_bytes / 4, T, nw,
                                                                   threshold, (uint32_t*)out);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
