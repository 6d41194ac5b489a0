// Normalisation kernels for the SD U-Net step (gfx950).
//
// GroupNorm is split into a statistics pass and an APPLY that is fused into the consumer's A-operand load
// (gemm.hip): the stats pass reads the activation once and emits per-(image, channel) fp32 scale/shift,
// so GN(+SiLU) never writes a normalised copy of the activation to HBM.
//   diffusers ResnetBlock2D norm1/norm2 (GroupNorm(32, C, eps=1e-5)), Transformer2DModel.norm
//   (GroupNorm(32, C, eps=1e-6)), conv_norm_out.
// LayerNorm (BasicTransformerBlock norm1/2/3, eps=1e-5) is one wave per token row, two-pass in registers.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

// Partial sums of (x - ref) and (x - ref)^2 over a slice of rows for one (image, group).
// ref = first element of the group in the image's row 0 (shifted sums keep the variance well conditioned).
__global__ __launch_bounds__(256) void gn_partial_kernel(const half_t* __restrict__ X, long ldx, int HW, int C,
                                                         int G, int S, float2* __restrict__ part) {
  const int s = blockIdx.x, g = blockIdx.y, img = blockIdx.z;
  const int cpg = C / G, hp = cpg / 2;
  const int r0 = (int)((long)HW * s / S), r1 = (int)((long)HW * (s + 1) / S);
  const half_t* base = X + (long)img * HW * ldx + g * cpg;
  const float ref = (float)base[0];
  float s1 = 0.f, s2 = 0.f;
  const int n = (r1 - r0) * hp;
  for (int e = threadIdx.x; e < n; e += 256) {
    const int r = r0 + e / hp, pr = e % hp;
    half2_t v = *reinterpret_cast<const half2_t*>(base + (long)r * ldx + 2 * pr);
    const float a = (float)v[0] - ref, b = (float)v[1] - ref;
    s1 += a + b;
    s2 += a * a + b * b;
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  __shared__ float r[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { r[0][wave] = s1; r[1][wave] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((long)img * G + g) * S + s] = make_float2(r[0][0] + r[0][1] + r[0][2] + r[0][3],
                                                    r[1][0] + r[1][1] + r[1][2] + r[1][3]);
  }
}

// One wave per (image, group): combine slices in fp64, emit scale = rstd*gamma, shift = beta - mean*scale.
__global__ __launch_bounds__(64) void gn_finalize_kernel(const half_t* __restrict__ X, long ldx, int HW, int C,
                                                         int G, int S, const float2* __restrict__ part,
                                                         const half_t* __restrict__ gamma,
                                                         const half_t* __restrict__ beta, float eps,
                                                         float* __restrict__ scale, float* __restrict__ shift) {
  const int g = blockIdx.x, img = blockIdx.y, lane = threadIdx.x;
  const int cpg = C / G;
  double a = 0.0, b = 0.0;
  for (int s = lane; s < S; s += 64) {
    float2 v = part[((long)img * G + g) * S + s];
    a += v.x; b += v.y;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
  const double n = (double)HW * cpg;
  const double ref = (double)(float)X[(long)img * HW * ldx + g * cpg];
  const double m1 = a / n;
  double var = b / n - m1 * m1;
  if (var < 0) var = 0;
  const float mean = (float)(ref + m1);
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int c = lane; c < cpg; c += 64) {
    const int ch = g * cpg + c;
    const float sc = rstd * (float)gamma[ch];
    scale[(long)img * C + ch] = sc;
    shift[(long)img * C + ch] = (float)beta[ch] - mean * sc;
  }
}

// LayerNorm over the last dim (C <= 2048, C % 8 == 0), one wave per row, values kept in registers.
template <int MAXCH>
__global__ __launch_bounds__(256) void layernorm_kernel(const half_t* __restrict__ X, long ldx, half_t* __restrict__ Y,
                                                        long ldy, int M, int C, const half_t* __restrict__ gamma,
                                                        const half_t* __restrict__ beta, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = C / 8;
  half8 v[MAXCH];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      v[i] = *reinterpret_cast<const half8*>(X + (long)row * ldx + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (float)v[i][j];
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = (float)v[i][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < MAXCH; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      half8 gm = *reinterpret_cast<const half8*>(gamma + c * 8);
      half8 bt = *reinterpret_cast<const half8*>(beta + c * 8);
      half8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)(((float)v[i][j] - mean) * rstd * (float)gm[j] + (float)bt[j]);
      *reinterpret_cast<half8*>(Y + (long)row * ldy + c * 8) = o;
    }
  }
}

}  // namespace

extern "C" int sdmoe_groupnorm_stats(const void* X, long ldx, int nimg, int HW, int C, int groups,
                                     const void* gamma, const void* beta, float eps, float* scale, float* shift,
                                     float* workspace, long workspace_floats, void* stream) {
  if (!X || !gamma || !beta || !scale || !shift || !workspace || nimg <= 0 || HW <= 0 || groups <= 0)
    return SDMOE_EARG;
  if (C % groups || (C / groups) % 2 || ldx % 2) return SDMOE_ESHAPE;
  const long elems = (long)HW * (C / groups);
  int S = (int)(elems / 8192);
  S = S < 1 ? 1 : (S > 64 ? 64 : S);
  if (S > HW) S = HW;
  if ((long)nimg * groups * S * 2 > workspace_floats) return SDMOE_EARG;
  hipStream_t s = (hipStream_t)stream;
  float2* part = reinterpret_cast<float2*>(workspace);
  gn_partial_kernel<<<dim3(S, groups, nimg), 256, 0, s>>>((const half_t*)X, ldx, HW, C, groups, S, part);
  SDMOE_CHECK_LAUNCH();
  gn_finalize_kernel<<<dim3(groups, nimg), 64, 0, s>>>((const half_t*)X, ldx, HW, C, groups, S, part,
                                                       (const half_t*)gamma, (const half_t*)beta, eps, scale, shift);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_layernorm(const void* X, long ldx, void* Y, long ldy, int M, int C, const void* gamma,
                               const void* beta, float eps, void* stream) {
  if (!X || !Y || !gamma || !beta || M < 0 || C <= 0) return SDMOE_EARG;
  if (M == 0) return SDMOE_OK;
  if (C % 8 || ldx % 8 || ldy % 8 || C > 2048) return SDMOE_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (M + 3) / 4;
  if (C <= 512)
    layernorm_kernel<1><<<blocks, 256, 0, s>>>((const half_t*)X, ldx, (half_t*)Y, ldy, M, C, (const half_t*)gamma,
                                               (const half_t*)beta, eps);
  else if (C <= 1024)
    layernorm_kernel<2><<<blocks, 256, 0, s>>>((const half_t*)X, ldx, (half_t*)Y, ldy, M, C, (const half_t*)gamma,
                                               (const half_t*)beta, eps);
  else
    layernorm_kernel<4><<<blocks, 256, 0, s>>>((const half_t*)X, ldx, (half_t*)Y, ldy, M, C, (const half_t*)gamma,
                                               (const half_t*)beta, eps);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
