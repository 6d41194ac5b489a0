// Small step-loop kernels for the SD denoising step (gfx950): timestep embedding, CFG+DDIM update,
// U-Net input preparation. All device-side so the 50-step loop never touches host memory.
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

// diffusers get_timestep_embedding(t, dim, flip_sin_to_cos, downscale_freq_shift, max_period=10000)
__global__ void timestep_embedding_kernel(half_t* out, const float* tptr, float tval, int dim, int flip,
                                          float freq_shift) {
  const int half = dim / 2;
  const float t = tptr ? *tptr : tval;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float expo = -logf(10000.0f) * (float)i / ((float)half - freq_shift);
    const float a = t * expf(expo);
    const float sv = sinf(a), cv = cosf(a);
    if (flip) { out[i] = (half_t)cv; out[half + i] = (half_t)sv; }
    else { out[i] = (half_t)sv; out[half + i] = (half_t)cv; }
  }
}

// n timesteps t_dev[0..n) -> rows; row r lands at out + (r / group) * ldo + (r % group) * dim (SDXL text_time:
// the 6 time-id sinusoids of an image sit side by side in its add-embedding input row)
__global__ void timestep_embedding_rows_kernel(half_t* out, long ldo, const float* t_dev, int group, int dim,
                                               int flip, float freq_shift) {
  const int r = blockIdx.x;
  half_t* o = out + (long)(r / group) * ldo + (long)(r % group) * dim;
  const int half = dim / 2;
  const float t = t_dev[r];
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float expo = -logf(10000.0f) * (float)i / ((float)half - freq_shift);
    const float a = t * expf(expo);
    const float sv = sinf(a), cv = cosf(a);
    if (flip) { o[i] = (half_t)cv; o[half + i] = (half_t)sv; }
    else { o[i] = (half_t)sv; o[half + i] = (half_t)cv; }
  }
}

// latents fp32 NCHW [B,4,H,W] -> U-Net input fp16 NHWC [ncopy*B, H*W, ldo] (channels 0..3; CFG copies)
__global__ void prepare_input_kernel(const float* __restrict__ lat, half_t* __restrict__ out, int B, int HW,
                                     long ldo, int ncopy) {
  const long n = (long)ncopy * B * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int p = (int)(i % HW);
    const int bb = (int)(i / HW);
    const int b = bb % B;
    half4 v;
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = (half_t)lat[((long)b * 4 + c) * HW + p];
    *reinterpret_cast<half4*>(out + i * ldo) = v;
  }
}

// eps fp16 [ncopy*B, HW, lde] (uncond images first, as diffusers' torch.cat([uncond, cond])),
// guidance: eps = eu + g*(ec - eu); DDIM (eta=0): x0 = (x - sqrt(1-a_t) eps)/sqrt(a_t);
// x_prev = sqrt(a_prev) x0 + sqrt(1-a_prev) eps.  Optionally writes the next U-Net input.
__global__ void cfg_ddim_kernel(const half_t* __restrict__ eps, long lde, float* __restrict__ lat, int B, int HW,
                                int do_cfg, float guidance, float a_t, float a_prev, half_t* __restrict__ next_in,
                                long ldn) {
  const long n = (long)B * HW;
  const float sa = sqrtf(a_t), sb = sqrtf(1.f - a_t), sp = sqrtf(a_prev), sq = sqrtf(1.f - a_prev);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / HW), p = (int)(i % HW);
    half4 eu = *reinterpret_cast<const half4*>(eps + ((long)b * HW + p) * lde);
    half4 ec = eu;
    if (do_cfg) ec = *reinterpret_cast<const half4*>(eps + ((long)(B + b) * HW + p) * lde);
    half4 nx;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float e = do_cfg ? (float)eu[c] + guidance * ((float)ec[c] - (float)eu[c]) : (float)eu[c];
      const long li = ((long)b * 4 + c) * HW + p;
      const float x = lat[li];
      const float x0 = (x - sb * e) / sa;
      const float xp = sp * x0 + sq * e;
      lat[li] = xp;
      nx[c] = (half_t)xp;
    }
    if (next_in) {
      *reinterpret_cast<half4*>(next_in + ((long)b * HW + p) * ldn) = nx;
      if (do_cfg) *reinterpret_cast<half4*>(next_in + ((long)(B + b) * HW + p) * ldn) = nx;
    }
  }
}

// CFG + one linear multistep update (PNDMScheduler.step_plms, prediction_type "epsilon"):
//   e   = CFG(eps)                               (stored into history slot `store` when store >= 0)
//   mo  = c_new * e + sum_j c[j] * hist[j]       (the PLMS combination of the current and past eps)
//   src = use_cur ? cur : lat ;  if save_cur: cur = lat (before the update)
//   lat = a * src - b * mo                       (_get_prev_sample: a = sqrt(ap/at), b = (ap - at)/denom)
// hist: [4][B*4*HW] fp32 NCHW like lat; cur: [B*4*HW] fp32.
struct MultistepCoef {
  float c_new, c[4], a, b;
  int store, use_cur, save_cur;
};

__global__ void cfg_multistep_kernel(const half_t* __restrict__ eps, long lde, float* __restrict__ lat, int B, int HW,
                                     int do_cfg, float guidance, float* __restrict__ hist, float* __restrict__ cur,
                                     MultistepCoef k, half_t* __restrict__ next_in, long ldn) {
  const long n = (long)B * HW;
  const long plane = (long)B * 4 * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / HW), p = (int)(i % HW);
    half4 eu = *reinterpret_cast<const half4*>(eps + ((long)b * HW + p) * lde);
    half4 ec = eu;
    if (do_cfg) ec = *reinterpret_cast<const half4*>(eps + ((long)(B + b) * HW + p) * lde);
    half4 nx;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float e = do_cfg ? (float)eu[c] + guidance * ((float)ec[c] - (float)eu[c]) : (float)eu[c];
      const long li = ((long)b * 4 + c) * HW + p;
      float mo = k.c_new * e;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (k.c[j] != 0.f) mo += k.c[j] * hist[j * plane + li];
      if (k.store >= 0) hist[k.store * plane + li] = e;
      const float x = lat[li];
      const float src = k.use_cur ? cur[li] : x;
      if (k.save_cur) cur[li] = x;
      const float xp = k.a * src - k.b * mo;
      lat[li] = xp;
      nx[c] = (half_t)xp;
    }
    if (next_in) {
      *reinterpret_cast<half4*>(next_in + ((long)b * HW + p) * ldn) = nx;
      if (do_cfg) *reinterpret_cast<half4*>(next_in + ((long)(B + b) * HW + p) * ldn) = nx;
    }
  }
}

__global__ void add_kernel(const half_t* a, const half_t* b, half_t* o, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    half8 x = reinterpret_cast<const half8*>(a)[i], y = reinterpret_cast<const half8*>(b)[i], z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (half_t)((float)x[j] + (float)y[j]);
    reinterpret_cast<half8*>(o)[i] = z;
  }
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int sdmoe_timestep_embedding(void* out, const float* t_dev, float t, int dim, int flip_sin_to_cos,
                                        float freq_shift, void* stream) {
  if (!out || dim <= 0 || dim % 2) return SDMOE_EARG;
  timestep_embedding_kernel<<<1, 256, 0, (hipStream_t)stream>>>((half_t*)out, t_dev, t, dim, flip_sin_to_cos,
                                                                freq_shift);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_timestep_embedding_rows(void* out, long ldo, const float* t_dev, int n, int group, int dim,
                                             int flip_sin_to_cos, float freq_shift, void* stream) {
  if (!out || !t_dev || n <= 0 || group <= 0 || dim <= 0 || dim % 2) return SDMOE_EARG;
  if (ldo < (long)group * dim) return SDMOE_ESHAPE;
  timestep_embedding_rows_kernel<<<n, 128, 0, (hipStream_t)stream>>>((half_t*)out, ldo, t_dev, group, dim,
                                                                     flip_sin_to_cos, freq_shift);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_prepare_input(const float* lat, void* out, int B, int HW, long ldo, int ncopy, void* stream) {
  if (!lat || !out || B <= 0 || HW <= 0 || ncopy <= 0) return SDMOE_EARG;
  if (ldo % 4) return SDMOE_ESHAPE;
  const long n = (long)ncopy * B * HW;
  prepare_input_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>(lat, (half_t*)out, B, HW, ldo, ncopy);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_cfg_ddim_step(const void* eps, long lde, float* lat, int B, int HW, int do_cfg, float guidance,
                                   float alpha_t, float alpha_prev, void* next_in, long ldn, void* stream) {
  if (!eps || !lat || B <= 0 || HW <= 0) return SDMOE_EARG;
  if (lde % 4 || (next_in && ldn % 4)) return SDMOE_ESHAPE;
  const long n = (long)B * HW;
  cfg_ddim_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>((const half_t*)eps, lde, lat, B, HW, do_cfg, guidance,
                                                               alpha_t, alpha_prev, (half_t*)next_in, ldn);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_cfg_multistep_step(const void* eps, long lde, float* lat, int B, int HW, int do_cfg,
                                        float guidance, float* hist, float* cur, const float* coef, const int* flags,
                                        void* next_in, long ldn, void* stream) {
  if (!eps || !lat || !hist || !cur || !coef || !flags || B <= 0 || HW <= 0) return SDMOE_EARG;
  if (lde % 4 || (next_in && ldn % 4)) return SDMOE_ESHAPE;
  if (flags[0] < -1 || flags[0] > 3) return SDMOE_EARG;
  MultistepCoef k;
  k.c_new = coef[0];
  for (int j = 0; j < 4; ++j) k.c[j] = coef[1 + j];
  k.a = coef[5];
  k.b = coef[6];
  k.store = flags[0];
  k.use_cur = flags[1];
  k.save_cur = flags[2];
  cfg_multistep_kernel<<<grid_for((long)B * HW), 256, 0, (hipStream_t)stream>>>(
      (const half_t*)eps, lde, lat, B, HW, do_cfg, guidance, hist, cur, k, (half_t*)next_in, ldn);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_add(const void* a, const void* b, void* out, long n, void* stream) {
  if (!a || !b || !out || n < 0) return SDMOE_EARG;
  if (n % 8) return SDMOE_ESHAPE;
  if (n == 0) return SDMOE_OK;
  add_kernel<<<grid_for(n / 8), 256, 0, (hipStream_t)stream>>>((const half_t*)a, (const half_t*)b, (half_t*)out,
                                                               n / 8);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" const char* sdmoe_version(void) { return "sdmoe-hip 0.1 gfx950"; }
