// Back-to-back MFMA issue rate on one wave per SIMD: v_mfma_f32_16x16x32_f16 vs v_mfma_f32_16x16x16_f16 (the d = 40
// attention's QK^T could take its last 8 head dims as a K = 16 MFMA instead of a half-empty K = 32 one).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/mfma_rate tools/micro/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float float4v __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ __launch_bounds__(64) void k(float* out, int iters) {
  float4v c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  half8 a8, b8;
  half4 a4, b4;
  for (int i = 0; i < 8; ++i) { a8[i] = (_Float16)(threadIdx.x * 1e-3f + i); b8[i] = (_Float16)(i * 1e-3f); }
  for (int i = 0; i < 4; ++i) { a4[i] = a8[i]; b4[i] = b8[i]; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (KIND == 0) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c3, 0, 0, 0);
      } else {
        c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c3, 0, 0, 0);
      }
    }
  }
  float4v s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 64 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <int KIND>
double run(float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<KIND><<<1024, 64>>>(out, 10);
  hipEventRecord(e0);
  k<KIND><<<1024, 64>>>(out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  hipMalloc(&out, 1024 * 64 * 4);
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    double m32 = run<0>(out, iters), m16 = run<1>(out, iters);
    const double n = 16.0 * iters;  // MFMAs per wave
    printf("16x16x32 f16: %.3f ms  %.2f ns/MFMA/wave | 16x16x16 f16: %.3f ms  %.2f ns/MFMA/wave | ratio %.3f\n", m32,
           m32 * 1e6 / n, m16, m16 * 1e6 / n, m16 / m32);
  }
  hipFree(out);
  return 0;
}
