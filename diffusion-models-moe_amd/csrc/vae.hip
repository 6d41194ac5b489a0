// VAE decoder helpers for gfx950 (AutoencoderKL.decode after the denoising loop).
// The decoder's mid-block attention is ONE head of width 512 over the 64x64 latent grid (4096 tokens); it runs as
// two MFMA GEMMs (sdmoe_linear) around these kernels:
//   * sdmoe_softmax_rows: P = softmax(S) per row, fp16 in/out, fp32 max/sum (the scale is folded into Q);
//   * sdmoe_transpose: V [tokens, 512] -> V^T [512, tokens], the nn.Linear-layout operand of O = P V.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

// one wave per row, 8 halves per lane per step; two passes over the row in registers when it fits (N <= 8192),
// re-reading it otherwise
template <int CHUNKS>  // 16-B chunks per lane held in registers (N = 512 * CHUNKS)
__global__ __launch_bounds__(256) void softmax_rows_kernel(const half_t* __restrict__ X, long ldx, half_t* __restrict__ Y,
                                                           long ldy, int R, int N) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;  // wave-uniform
  const half_t* xr = X + (long)row * ldx;
  half8 v[CHUNKS];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int col = (c * 64 + lane) * 8;
    v[c] = col < N ? *reinterpret_cast<const half8*>(xr + col) : (half8){0, 0, 0, 0, 0, 0, 0, 0};
    if (col < N) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, (float)v[c][j]);
    }
  }
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf((float)v[c][j] - mx);
    }
  }
  const float inv = 1.0f / wave_sum(s);
  half_t* yr = Y + (long)row * ldy;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < N) {
      half8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)(__expf((float)v[c][j] - mx) * inv);
      *reinterpret_cast<half8*>(yr + col) = o;
    }
  }
}

// 64 x 64 tile through LDS (padded rows: conflict-free column reads)
__global__ __launch_bounds__(256) void transpose_kernel(const half_t* __restrict__ X, long ldx, half_t* __restrict__ Y,
                                                        long ldy, int R, int C) {
  __shared__ half_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i / 64, c = i % 64;
    tile[r][c] = (r0 + r < R && c0 + c < C) ? X[(long)(r0 + r) * ldx + c0 + c] : (half_t)0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int c = i / 64, r = i % 64;
    if (c0 + c < C && r0 + r < R) Y[(long)(c0 + c) * ldy + r0 + r] = tile[r][c];
  }
}

}  // namespace

extern "C" int sdmoe_softmax_rows(const void* X, long ldx, void* Y, long ldy, int R, int N, void* stream) {
  if (R == 0) return SDMOE_OK;
  if (!X || !Y || R < 0 || N <= 0) return SDMOE_EARG;
  if (N % 8 || ldx % 8 || ldy % 8 || N > 8192) return SDMOE_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (R + 3) / 4;
  const half_t* x = (const half_t*)X;
  half_t* y = (half_t*)Y;
  if (N <= 512) softmax_rows_kernel<1><<<blocks, 256, 0, s>>>(x, ldx, y, ldy, R, N);
  else if (N <= 1024) softmax_rows_kernel<2><<<blocks, 256, 0, s>>>(x, ldx, y, ldy, R, N);
  else if (N <= 4096) softmax_rows_kernel<8><<<blocks, 256, 0, s>>>(x, ldx, y, ldy, R, N);
  else softmax_rows_kernel<16><<<blocks, 256, 0, s>>>(x, ldx, y, ldy, R, N);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_transpose(const void* X, long ldx, void* Y, long ldy, int R, int C, void* stream) {
  if (R == 0 || C == 0) return SDMOE_OK;
  if (!X || !Y || R < 0 || C < 0) return SDMOE_EARG;
  const dim3 grid((C + 63) / 64, (R + 63) / 64);
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const half_t*)X, ldx, (half_t*)Y, ldy, R, C);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
