// Issue cost of the softmax VALU candidates on gfx950, one and two waves per SIMD: v_exp_f32 vs v_exp_f16 (low half,
// and high half through SDWA) vs v_fma_f32 (the 4-cycle reference), and the packed fp16 max. Eight independent
// registers per instruction kind, so the stream is issue-bound, not latency-bound.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/valu_rate tools/micro/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(64) void k(float* out, int iters) {
  float f[8];
  unsigned h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f[i] = -0.001f * (threadIdx.x + i);
    _Float16 a = (_Float16)(-0.01f * i), b = (_Float16)(-0.02f * i);
    h[i] = (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(f[i]));
      if constexpr (KIND == 1) asm volatile("v_exp_f16 %0, %0" : "+v"(h[i]));
      if constexpr (KIND == 2) asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(h[i]));
      if constexpr (KIND == 3) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(f[i]));
      if constexpr (KIND == 4) asm volatile("v_pk_max_f16 %0, %0, %0" : "+v"(h[i]));
      if constexpr (KIND == 5) asm volatile("v_max3_f32 %0, %0, %0, %0" : "+v"(f[i]));
      if constexpr (KIND == 6) asm volatile("v_cvt_pk_f16_f32 %0, %0, %0" : "+v"(h[i]));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += f[i] + (float)h[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int KIND>
double run(float* out, int iters, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<KIND><<<blocks, 64>>>(out, 100);
  hipEventRecord(e0);
  k<KIND><<<blocks, 64>>>(out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * 64 * 4);
  const int iters = 20000;
  const char* names[] = {"v_exp_f32", "v_exp_f16", "v_exp_f16_sdwa(hi)", "v_fma_f32", "v_pk_max_f16", "v_max3_f32",
                         "v_cvt_pk_f16_f32"};
  for (int blocks : {1024, 2048}) {
    for (int rep = 0; rep < 2; ++rep) {
      double ms[7] = {run<0>(out, iters, blocks), run<1>(out, iters, blocks), run<2>(out, iters, blocks),
                      run<3>(out, iters, blocks), run<4>(out, iters, blocks), run<5>(out, iters, blocks),
                      run<6>(out, iters, blocks)};
      printf("waves/SIMD %d:", blocks / 1024);
      for (int i = 0; i < 7; ++i) printf("  %s %.3f (x%.2f fma)", names[i], ms[i], ms[i] / ms[3]);
      printf("\n");
    }
  }
  hipFree(out);
  return 0;
}
