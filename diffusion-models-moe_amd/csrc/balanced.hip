// Offline MoE-fication: the balanced ("size-constrained") k-means that
// moefication/moe_utils.py:97-107 (ParamSplit.split) runs through k_means_constrained.KMeansConstrained with
// size_min = size_max = expert_size on the L2-normalised gate rows of every GEGLU projection.
//   sdmoe_sqdist_f32      GPU: D[i][c] = max(|x_i|^2 + |c_c|^2 - 2 x_i.c_c, 0) in exact fp32 (v_mfma_f32_16x16x4_f32:
//                         a k-ordered fmaf chain), the euclidean_distances expansion k-means uses
//   sdmoe_balanced_assign host: the assignment step — minimum-cost assignment of n points to k clusters holding
//                         exactly n/k points each (the min-cost-flow the reference solves with OR-tools), here an
//                         epsilon-scaling auction over integer costs with per-cluster slot prices; optimal for the
//                         integer costs once eps < 1/n. Prices can be carried across k-means iterations (warm
//                         start: the centres move little, so later assignments need few bids).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <vector>

#include "common.h"
#include "../../include/sdmoe.h"

namespace {

// 64 points x 64 centres per 256-thread block; wave w owns points [16w, 16w+16) against all 64 centres
// (4 accumulators of 16x16). d staged through LDS in 32-wide slabs (row stride 33: conflict-free column reads).
__global__ __launch_bounds__(256) void sqdist_kernel(const float* __restrict__ X, long ldx, const float* __restrict__ Cc,
                                                     long ldc, int n, int k, int d, float* __restrict__ D, long ldd) {
  __shared__ float xs[64][33];
  __shared__ float cs[64][33];
  __shared__ float xn[64], cn[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  float4v acc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) acc[f] = (float4v){0.f, 0.f, 0.f, 0.f};
  float xsq = 0.f, csq = 0.f;  // thread tid < 64: row tid of the X tile; 64 <= tid < 128: row tid-64 of C
  for (int k0 = 0; k0 < d; k0 += 32) {
    for (int e = tid; e < 64 * 32; e += 256) {
      const int r = e >> 5, c = e & 31;
      const int gi = i0 + r, gc = c0 + r, kk = k0 + c;
      xs[r][c] = (gi < n && kk < d) ? X[(long)gi * ldx + kk] : 0.f;
      cs[r][c] = (gc < k && kk < d) ? Cc[(long)gc * ldc + kk] : 0.f;
    }
    __syncthreads();
    if (tid < 64) {
      for (int c = 0; c < 32; ++c) xsq = fmaf(xs[tid][c], xs[tid][c], xsq);
    } else if (tid < 128) {
      for (int c = 0; c < 32; ++c) csq = fmaf(cs[tid - 64][c], cs[tid - 64][c], csq);
    }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const float a = xs[16 * wave + (lane & 15)][4 * ks + (lane >> 4)];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float b = cs[16 * f + (lane & 15)][4 * ks + (lane >> 4)];
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[f], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  if (tid < 64) xn[tid] = xsq;
  else if (tid < 128) cn[tid - 64] = csq;
  __syncthreads();
  // C/D layout: col (centre) = lane & 15, row (point) = (lane >> 4) * 4 + reg
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pi = 16 * wave + (lane >> 4) * 4 + r, cc = 16 * f + (lane & 15);
      const int gi = i0 + pi, gc = c0 + cc;
      if (gi < n && gc < k) D[(long)gi * ldd + gc] = fmaxf(xn[pi] + cn[cc] - 2.f * acc[f][r], 0.f);
    }
}

// ---- epsilon-scaling auction for the balanced assignment (maximise -cost) ----------------------------------
struct Auction {
  int n, k, s;
  const int64_t* cost;          // [n][k]
  std::vector<int64_t> price;   // [k][s]
  std::vector<int> owner;       // [k][s] point holding the slot, -1 free
  std::vector<int> slot_of;     // [n] global slot id (c * s + j) or -1
  std::vector<int> min1, min2;  // per cluster: index of the cheapest / second-cheapest slot

  void refresh(int c) {
    const int64_t* p = &price[(size_t)c * s];
    int a = 0, b = -1;
    for (int j = 1; j < s; ++j) {
      if (p[j] < p[a]) { b = a; a = j; }
      else if (b < 0 || p[j] < p[b]) b = j;
    }
    min1[c] = a;
    min2[c] = b;
  }

  // one phase at eps: every point ends up assigned (prices only rise)
  void phase(int64_t eps) {
    std::fill(owner.begin(), owner.end(), -1);
    std::fill(slot_of.begin(), slot_of.end(), -1);
    std::vector<int> queue(n);
    for (int i = 0; i < n; ++i) queue[i] = n - 1 - i;
    const int64_t NEG = std::numeric_limits<int64_t>::min() / 4;
    while (!queue.empty()) {
      const int i = queue.back();
      queue.pop_back();
      const int64_t* ci = cost + (size_t)i * k;
      int64_t best = NEG, second = NEG;
      int bc = -1;
      for (int c = 0; c < k; ++c) {
        const int64_t v = -ci[c] - price[(size_t)c * s + min1[c]];
        if (v > best) { second = best; best = v; bc = c; }
        else if (v > second) second = v;
      }
      if (min2[bc] >= 0) second = std::max(second, -ci[bc] - price[(size_t)bc * s + min2[bc]]);
      if (second == NEG) second = best;  // k == 1 and s == 1
      const int j = min1[bc];
      const size_t slot = (size_t)bc * s + j;
      price[slot] += best - second + eps;
      const int prev = owner[slot];
      owner[slot] = i;
      slot_of[i] = (int)slot;
      if (prev >= 0) {
        slot_of[prev] = -1;
        queue.push_back(prev);
      }
      refresh(bc);
    }
  }
};

}  // namespace

extern "C" int sdmoe_sqdist_f32(const float* X, long ldx, const float* C, long ldc, int n, int k, int d, float* D,
                                long ldd, void* stream) {
  if (!X || !C || !D || n <= 0 || k <= 0 || d <= 0) return SDMOE_EARG;
  if (ldx < d || ldc < d || ldd < k) return SDMOE_ESHAPE;
  dim3 grid((n + 63) / 64, (k + 63) / 64);
  sqdist_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(X, ldx, C, ldc, n, k, d, D, ldd);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_balanced_assign(const double* cost, int n, int k, double scale, int64_t* prices, int warm,
                                     int* labels) {
  if (!cost || !labels || n <= 0 || k <= 0 || !(scale >= 0)) return SDMOE_EARG;
  if (n % k) return SDMOE_ESHAPE;
  const int s = n / k;
  double cmax = 0.0;
  for (long i = 0; i < (long)n * k; ++i) {
    if (!std::isfinite(cost[i]) || cost[i] < 0) return SDMOE_EARG;
    cmax = std::max(cmax, cost[i]);
  }
  // integer costs: `scale` units per cost unit (auto: the largest cost -> 2^40). Every cost is then multiplied
  // by (n + 1), so that the final eps = 1 is below 1/n of the integer cost unit: the eps-complementary-slackness
  // assignment the auction ends with is then an exact optimum for the integer costs.
  if (scale == 0) scale = cmax > 0 ? std::ldexp(1.0, 40) / cmax : 1.0;
  if (cmax * scale > std::ldexp(1.0, 42)) return SDMOE_ESHAPE;
  const int64_t unit = (int64_t)n + 1;
  std::vector<int64_t> ic((size_t)n * k);
  int64_t imax = 0;
  for (long i = 0; i < (long)n * k; ++i) {
    ic[i] = (int64_t)std::llround(cost[i] * scale) * unit;
    imax = std::max(imax, ic[i]);
  }
  Auction a;
  a.n = n; a.k = k; a.s = s; a.cost = ic.data();
  a.price.assign((size_t)k * s, 0);
  if (warm && prices)
    for (size_t i = 0; i < a.price.size(); ++i) a.price[i] = prices[i];
  a.owner.assign((size_t)k * s, -1);
  a.slot_of.assign(n, -1);
  a.min1.assign(k, 0);
  a.min2.assign(k, -1);
  for (int c = 0; c < k; ++c) a.refresh(c);
  // eps scaling: cold from range/8, warm (prices near equilibrium) from range/4096, /8 per phase down to 1
  int64_t eps = std::max<int64_t>(1, warm ? imax / 4096 : imax / 8);
  for (;;) {
    a.phase(eps);
    if (eps == 1) break;
    eps = std::max<int64_t>(1, eps / 8);
  }
  for (int i = 0; i < n; ++i) labels[i] = a.slot_of[i] / s;
  if (prices) {  // prices are relative: store them shifted to min 0 so warm starts never drift toward overflow
    const int64_t pmin = *std::min_element(a.price.begin(), a.price.end());
    for (size_t i = 0; i < a.price.size(); ++i) prices[i] = a.price[i] - pmin;
  }
  return SDMOE_OK;
}
