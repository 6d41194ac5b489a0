// Shared device helpers for the sdmoe gfx950 (CDNA4) kernels.
// All kernels are written for wave64 and the gfx950 MFMA set; nothing here is portable on purpose.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 half_t;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float4v __attribute__((ext_vector_type(4)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef unsigned int uint4v __attribute__((ext_vector_type(4)));
typedef unsigned int uint2v __attribute__((ext_vector_type(2)));

#define SDMOE_DEV __device__ __forceinline__

// Status codes returned by every C-ABI entry point (0 = ok, >0 = hipError_t, <0 = argument error).
enum {
  SDMOE_OK = 0,
  SDMOE_EARG = -1,     // null pointer / bad size
  SDMOE_ESHAPE = -2,   // unsupported shape (alignment / divisibility)
  SDMOE_EUNSUP = -3,   // unsupported mode
};

#define SDMOE_CHECK_LAUNCH()                          \
  do {                                                \
    hipError_t _e = hipGetLastError();                \
    if (_e != hipSuccess) return (int)_e;             \
  } while (0)

SDMOE_DEV float4v mfma16x16x32(half8 a, half8 b, float4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

SDMOE_DEV float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// exact-erf GELU written through erfc so the negative tail keeps full relative precision (1 + erf(x/sqrt2)
// cancels in fp32 below x ~ -3); within 1 fp16 ulp of the correctly rounded value.
SDMOE_DEV float gelu_erf_f(float x) { return 0.5f * x * erfcf(-x * 0.70710678118654752f); }

// GELU of the reference's GEGLU (module.gelu = F.gelu on an fp16 tensor) over fp16 inputs, bit for bit: the
// values for 2^-5 <= |x| < 8 come from a 16384-entry fp16 table -- the module's own activation evaluated on every
// such input, registered per device by sdmoe_set_gelu_table -- at index (|x| bits - 0x2800) | sign << 13; below 2^-5
// x * Phi(x) = 0.5 x + x^2 (1/sqrt(2 pi) - x^2 / (6 sqrt(2 pi))) in fp32 (next term 0.02 x^5 relative: < 1e-9);
// x >= 8 -> x, x <= -8 -> -0 (fp32 erf saturates: the reference returns exactly these). One LDS (or L1) read and
// ~10 VALU instead of erfcf's branchy polynomial + exp; also exact where the fp32 1 + erf form the reference
// computes is not correctly rounded (0.9 % of fp16 inputs, mostly the negative tail).
constexpr int GELU_TAB_N = 16384;
SDMOE_DEV half_t gelu_tab_h(half_t x, const half_t* tab) {
  const unsigned u = __builtin_bit_cast(unsigned short, x), a = u & 0x7fffu;
  const float f = (float)x, x2 = f * f;
  float sf = __builtin_fmaf(x2, __builtin_fmaf(x2, -0.0664903745f, 0.3989422804f), 0.5f * f);
  asm volatile("" : "+v"(sf));  // round to fp32 first (as the reference): no fused fma -> f16 (v_fma_mix) rounding
  const half_t small = (half_t)sf;
  int idx = (int)a - 0x2800;
  idx = idx < 0 ? 0 : (idx > 8191 ? 8191 : idx);
  const half_t t = tab[idx | (int)((u >> 15) << 13)];
  const half_t big = (u & 0x8000u) ? (half_t)(-0.0f) : x;
  return a < 0x2800u ? small : (a >= 0x4800u ? big : t);
}
// the table registered for the calling thread's current device (gemm.hip), or null
const half_t* sdmoe_gelu_tab_current();

SDMOE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SDMOE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Activation kinds shared by the host ABI (include/sdmoe.h).
enum { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_RELU = 3, ACT_QUICK_GELU = 4 };

SDMOE_DEV float apply_act(float v, int act) {
  if (act == ACT_SILU) return silu_f(v);
  if (act == ACT_GELU) return gelu_erf_f(v);
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_QUICK_GELU) return v / (1.0f + __expf(-1.702f * v));  // CLIP quick_gelu: x*sigmoid(1.702x)
  return v;
}

// XCD-aware bijective remap of a 1-D block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2.
SDMOE_DEV int xcd_remap(int bid, int nblocks) {
  const int nx = 8;
  if (nblocks < nx) return bid;
  int q = nblocks / nx, r = nblocks % nx;
  int xcd = bid % nx, idx = bid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
