// MFMA GEMM / implicit-GEMM 3x3 convolution for gfx950, fp16 in / fp32 accumulate / fp16 out.
//
// One kernel template covers every dense projection of the SD U-Net step:
//   * Linear layers (attention q/k/v/out, proj_in/proj_out 1x1 convs, GEGLU proj, FFN down-proj,
//     time-embedding MLP)  -- MODE_GEMM, activations [M, K] row-major, weights [N, K] (nn.Linear layout);
//   * ResNet 3x3 convolutions (stride 1/2, fused nearest-2x upsample) on NHWC activations -- MODE_CONV,
//     weights [Cout][3][3][Cin] so K = 9*Cin is contiguous per output channel.
// Fusions (all optional, chosen per launch):
//   A-load : GroupNorm apply (per (image, channel) fp32 scale/shift) + SiLU, done in registers while the
//            tile is staged to LDS (zero padding stays zero, as in F.conv2d on the normalised tensor);
//   B-load : Wanda weight bitmask (bit = 1 -> weight zeroed), replacing the reference's per-call
//            W.clone()*(1-M) (remove_wanda_neurons_fast.py:69-83);
//   epilogue: + bias[n] + coladd[image][n] (time embedding) -> activation -> + residual[m][n].
// Tiles: BMxBNx64, 256 threads = 2x2 waves, 16x16x32 f16 MFMA, register-staged double-buffered LDS with an
// XOR chunk swizzle (conflict-free ds_read_b128 for 16 consecutive rows), fp32 epilogue staged through LDS
// so global stores are 16 B per lane.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

constexpr int BK = 64;

struct GemmParams {
  const half_t* A; long lda;
  const half_t* W; long ldw;
  const half_t* bias;
  const half_t* coladd; long coladd_bstride;
  const half_t* R; long ldr;
  half_t* C; long ldc;
  int M, N, K;
  int act;
  const float* a_scale; const float* a_shift; int a_silu; int a_chan;  // a_chan: channels per image row
  int rows_per_batch;
  int H, Wd, Cin, OH, OW, stride, upsample;
  const uint8_t* wmask;  // [N][K/8] bytes
};

SDMOE_DEV int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int BM, int BN, bool CONV, bool ATRANS, bool WMASK>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmParams p) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int A_PER = BM / 32, B_PER = BN / 32;
  constexpr int STAGE_BYTES = 2 * (BM + BN) * BK * 2;
  constexpr int WN_PAD = WN + 4;
  constexpr int EPI_BYTES = 4 * WM * WN_PAD * 4;
  constexpr int SMEM = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  half_t* sA = reinterpret_cast<half_t*>(smem);
  half_t* sB = sA + 2 * BM * BK;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, ntn * ntm);
  const int tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = p.K / BK;

  // per-thread staging rows (fixed for the whole K loop)
  int a_row[A_PER], a_kc[A_PER];
  int a_b[A_PER], a_oh[A_PER], a_ow[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    int id = tid + 256 * i;
    a_row[i] = id >> 3; a_kc[i] = id & 7;
    int m = m0 + a_row[i];
    a_ok[i] = m < p.M;
    int mm = a_ok[i] ? m : 0;
    if (CONV) {
      int hw = p.OH * p.OW;
      a_b[i] = mm / hw; int r = mm - a_b[i] * hw;
      a_oh[i] = r / p.OW; a_ow[i] = r - a_oh[i] * p.OW;
    } else {
      a_b[i] = ATRANS ? mm / p.rows_per_batch : 0; a_oh[i] = 0; a_ow[i] = 0;
    }
  }
  int b_row[B_PER], b_kc[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    int id = tid + 256 * i;
    b_row[i] = id >> 3; b_kc[i] = id & 7;
    b_ok[i] = (n0 + b_row[i]) < p.N;
  }

  uint4v ra[A_PER], rb[B_PER];

  auto load_stage = [&](int ks) {
    const int k0 = ks * BK;
    int tap = 0, c0 = k0;
    if (CONV) { tap = k0 / p.Cin; c0 = k0 - tap * p.Cin; }
    const int kh = tap / 3, kw = tap - (tap / 3) * 3;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      uint4v v = {0u, 0u, 0u, 0u};
      bool ok = a_ok[i];
      const half_t* src = nullptr;
      if (CONV) {
        int ih, iw;
        if (p.upsample) {
          int uh = a_oh[i] + kh - 1, uw = a_ow[i] + kw - 1;
          ok = ok && uh >= 0 && uh < 2 * p.H && uw >= 0 && uw < 2 * p.Wd;
          ih = uh >> 1; iw = uw >> 1;
        } else {
          ih = a_oh[i] * p.stride + kh - 1; iw = a_ow[i] * p.stride + kw - 1;
          ok = ok && ih >= 0 && ih < p.H && iw >= 0 && iw < p.Wd;
        }
        if (ok) src = p.A + ((long)(a_b[i] * p.H + ih) * p.Wd + iw) * p.lda + c0 + a_kc[i] * 8;
      } else {
        if (ok) src = p.A + (long)(m0 + a_row[i]) * p.lda + k0 + a_kc[i] * 8;
      }
      if (ok) {
        v = *reinterpret_cast<const uint4v*>(src);
        if (ATRANS) {
          const int c = c0 + a_kc[i] * 8;
          const float* sc = p.a_scale + (long)a_b[i] * p.a_chan + c;
          const float* sh = p.a_shift + (long)a_b[i] * p.a_chan + c;
          float4v s0 = *reinterpret_cast<const float4v*>(sc), s1 = *reinterpret_cast<const float4v*>(sc + 4);
          float4v h0 = *reinterpret_cast<const float4v*>(sh), h1 = *reinterpret_cast<const float4v*>(sh + 4);
          half8 x = __builtin_bit_cast(half8, v);
          float s[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
          float h[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float f = (float)x[j] * s[j] + h[j];
            if (p.a_silu) f = silu_f(f);
            x[j] = (half_t)f;
          }
          v = __builtin_bit_cast(uint4v, x);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      uint4v v = {0u, 0u, 0u, 0u};
      if (b_ok[i]) {
        const long n = n0 + b_row[i];
        const int k = k0 + b_kc[i] * 8;
        v = *reinterpret_cast<const uint4v*>(p.W + n * p.ldw + k);
        if (WMASK) {
          unsigned bits = p.wmask[n * (p.K >> 3) + (k >> 3)];
          if (bits) {
            half8 x = __builtin_bit_cast(half8, v);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if ((bits >> j) & 1u) x[j] = (half_t)0.0f;
            v = __builtin_bit_cast(uint4v, x);
          }
        }
      }
      rb[i] = v;
    }
  };

  auto store_stage = [&](int buf) {
    half_t* a = sA + buf * BM * BK;
    half_t* b = sB + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
      *reinterpret_cast<uint4v*>(a + a_row[i] * BK + swz(a_row[i], a_kc[i]) * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      *reinterpret_cast<uint4v*>(b + b_row[i] * BK + swz(b_row[i], b_kc[i]) * 8) = rb[i];
  };

  float4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};

  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) load_stage(ks + 1);
    const half_t* a = sA + cur * BM * BK;
    const half_t* b = sB + cur * BN * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      half8 af[FM], bf[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        int row = wr * WM + i * 16 + fr;
        af[i] = *reinterpret_cast<const half8*>(a + row * BK + swz(row, kk * 4 + fg) * 8);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        int row = wc * WN + j * 16 + fr;
        bf[j] = *reinterpret_cast<const half8*>(b + row * BK + swz(row, kk * 4 + fg) * 8);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32(af[i], bf[j], acc[i][j]);
    }
    if (ks + 1 < nk) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: stage fp32 tile per wave, then 16-B vector stores with fused bias/coladd/act/residual
  float* st = reinterpret_cast<float*>(smem) + wave * WM * WN_PAD;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) st[(i * 16 + fg * 4 + r) * WN_PAD + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int CPR = WN / 8;  // 8-column chunks per row
  for (int id = lane; id < WM * CPR; id += 64) {
    const int r = id / CPR, c8 = id - r * CPR;
    const int m = m0 + wr * WM + r, n = n0 + wc * WN + c8 * 8;
    if (m >= p.M || n >= p.N) continue;
    const float* sp = st + r * WN_PAD + c8 * 8;
    float4v v0 = *reinterpret_cast<const float4v*>(sp), v1 = *reinterpret_cast<const float4v*>(sp + 4);
    float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
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
    if (p.act != ACT_NONE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = apply_act(v[j], p.act);
    }
    if (p.R) {
      half8 rr = *reinterpret_cast<const half8*>(p.R + (long)m * p.ldr + n);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += (float)rr[j];
    }
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (half_t)v[j];
    *reinterpret_cast<half8*>(p.C + (long)m * p.ldc + n) = o;
  }
}

template <int BM, int BN, bool CONV>
int launch_tile(const GemmParams& p, hipStream_t s) {
  const int blocks = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const bool at = p.a_scale != nullptr, wm = p.wmask != nullptr;
  if (at && wm) gemm_kernel<BM, BN, CONV, true, true><<<blocks, 256, 0, s>>>(p);
  else if (at) gemm_kernel<BM, BN, CONV, true, false><<<blocks, 256, 0, s>>>(p);
  else if (wm) gemm_kernel<BM, BN, CONV, false, true><<<blocks, 256, 0, s>>>(p);
  else gemm_kernel<BM, BN, CONV, false, false><<<blocks, 256, 0, s>>>(p);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

template <bool CONV>
int dispatch(const GemmParams& p, hipStream_t s) {
  // Pick the largest tile that still gives >= ~1 wave of blocks per CU (256 CUs).
  const long t128 = (long)((p.M + 127) / 128) * ((p.N + 127) / 128);
  const long t64x128 = (long)((p.M + 63) / 64) * ((p.N + 127) / 128);
  if (p.N <= 64) return launch_tile<64, 64, CONV>(p, s);
  if (t128 >= 240) return launch_tile<128, 128, CONV>(p, s);
  if (t64x128 >= 240 || p.N < 128) return launch_tile<64, 128, CONV>(p, s);
  return launch_tile<64, 64, CONV>(p, s);
}

}  // namespace

extern "C" int sdmoe_linear(const void* A, long lda, const void* W, long ldw, const void* bias,
                            const void* coladd, long coladd_bstride, int rows_per_batch,
                            const void* R, long ldr, void* C, long ldc, int M, int N, int K, int act,
                            const float* a_scale, const float* a_shift, int a_silu,
                            const void* wmask_bits, void* stream) {
  if (!A || !W || !C || M < 0 || N <= 0 || K <= 0) return SDMOE_EARG;
  if (M == 0) return SDMOE_OK;
  if (K % 64 || N % 8 || lda % 8 || ldw % 8 || ldc % 8 || (R && ldr % 8)) return SDMOE_ESHAPE;
  if ((a_scale || coladd) && rows_per_batch <= 0) return SDMOE_EARG;
  GemmParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.act = act;
  p.a_scale = a_scale; p.a_shift = a_shift; p.a_silu = a_silu; p.a_chan = K;
  p.rows_per_batch = rows_per_batch > 0 ? rows_per_batch : 1;
  p.wmask = (const uint8_t*)wmask_bits;
  return dispatch<false>(p, (hipStream_t)stream);
}

extern "C" int sdmoe_conv3x3(const void* X, long ldx, int nimg, int H, int W, int Cin,
                             const void* Wt, const void* bias, const void* coladd, long coladd_bstride,
                             const void* R, long ldr, void* Y, long ldy, int Cout, int stride, int upsample,
                             int act, const float* a_scale, const float* a_shift, int a_silu, void* stream) {
  if (!X || !Wt || !Y || nimg <= 0 || H <= 0 || W <= 0 || Cout <= 0) return SDMOE_EARG;
  if (Cin % 64 || Cout % 8 || ldx % 8 || ldy % 8 || (R && ldr % 8)) return SDMOE_ESHAPE;
  if (!(stride == 1 || stride == 2) || (upsample && stride != 1)) return SDMOE_EUNSUP;
  GemmParams p{};
  int OH, OW;
  if (upsample) { OH = 2 * H; OW = 2 * W; }
  else { OH = (H + 2 - 3) / stride + 1; OW = (W + 2 - 3) / stride + 1; }
  p.A = (const half_t*)X; p.lda = ldx; p.W = (const half_t*)Wt; p.ldw = 9L * Cin;
  p.bias = (const half_t*)bias; p.coladd = (const half_t*)coladd; p.coladd_bstride = coladd_bstride;
  p.R = (const half_t*)R; p.ldr = ldr; p.C = (half_t*)Y; p.ldc = ldy;
  p.M = nimg * OH * OW; p.N = Cout; p.K = 9 * Cin; p.act = act;
  p.a_scale = a_scale; p.a_shift = a_shift; p.a_silu = a_silu; p.a_chan = Cin;
  p.rows_per_batch = OH * OW;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = OH; p.OW = OW; p.stride = stride; p.upsample = upsample;
  return dispatch<true>(p, (hipStream_t)stream);
}
