// Routed GEGLU projection as a persistent ping-pong kernel (gfx950): the epilogue of one tile runs under the MFMAs of
// the next.
//
// Same operation and rounding points as gemm.hip's MODE_GEGLU (sdmoe_linear_geglu): C = A W^T + bias over W rows
// interleaved [value 2 | gate 2] per neuron pair (ops.geglu_rows), output P[m, n] = value * act(gate) in fp16 and the
// per-(row, expert) fp32 sums of act(gate) in neuron order rounded to fp16 -- bit-identical to that kernel (test).
// Replaces the hook body of neuron_receivers/moefy.py:12-23 / remove_skilled_experts.py:26-49 fused into the GEGLU
// projection, like MODE_GEGLU.
//
// Why: MODE_GEGLU at the 64x64 level runs one 8-wave 256x320 workgroup per CU (208-238 VGPRs), so a tile's epilogue
// (58 of its 124-158 us: LDS staging, copy-out, expert sums) overlaps nothing (profiles/r05_halo32_geglu_diag.txt).
// Here one persistent 8-wave workgroup per CU holds TWO 4-wave groups of 2x2 waves, each owning its own accumulators
// of a 256x160 tile (wave tile 128x80, the same per-wave epilogue as MODE_GEGLU). Phase k: group k % 2 runs the main
// loop of the workgroup's k-th tile while the other group runs the epilogue of tile k - 1, one staging pass per K-step;
// the roles swap every phase. Every K-step ends in one workgroup barrier that both groups take (the ring's hand-off);
// the epilogue uses only wave barriers in between.
// LDS: a 2-stage ring of 64-deep K-steps (A 256 rows + W 160 rows, 52 KiB a stage, LDS-DMA with pre-swizzled chunks)
// + one 21.8 KiB staging area (only one group is in its epilogue at a time) = 128 KiB. The main group issues every
// stage -- including step 0 of its successor's tile during its own last K-step -- and drains it (vmcnt) before the
// next barrier, so the epilogue group never waits on memory it did not issue.
#include <type_traits>

#include "common.h"
#include "../../include/sdmoe.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void_pp;

struct GppParams {
  const half_t* A; long lda;
  const half_t* W; long ldw;
  const half_t* bias;
  half_t* C; long ldc;
  half_t* score; long ld_score;
  int esize;
  int M, N, K, act;
  int a_bytes, w_bytes;
  int ntiles, ntn;
};

constexpr unsigned PP_OOB = 0x80000000u;
constexpr int PBM = 256, PBN = 160, PBK = 64;
constexpr int PWM = 128, PWN = 80, PFM = PWM / 16, PFN = PWN / 16;   // 2x2 waves per group
constexpr int PRB = PBK * 2;                                       // LDS row bytes
constexpr int PSTAGE = (PBM + PBN) * PRB;                          // 53248
constexpr int PA_INS = PBM / 8, PB_INS = PBN / 8;                  // 1-KiB pieces (8 rows) per stage: 32 + 20
constexpr int PA_PW = PA_INS / 4, PB_PW = PB_INS / 4;              // per main-group wave: 8 + 5
constexpr int PNH = PWN / 2;                                       // neurons per wave tile: 40
constexpr int PRG = 32;                                            // rows per staging pass (2 fragment rows)
constexpr int PGST = 4 * 2 * PRG * PNH * 2;                        // staging of the 4 epilogue waves: 20480
constexpr int PSTG_OFF = 2 * PSTAGE;                               // staging behind the ring
constexpr int PBIAS_OFF = PSTG_OFF + PGST;                         // 4 waves x 80 fp32 bias values
constexpr int PSMEM = PBIAS_OFF + 4 * PWN * 4;                     // 129536
static_assert(PSMEM <= 160 * 1024, "ping-pong GEGLU LDS");
static_assert(PA_INS % 4 == 0 && PB_INS % 4 == 0, "whole pieces per main-group wave");

SDMOE_DEV int pswz(int row) { return (row >> 1) & 7; }

SDMOE_DEV float pp_add_lo(float acc, unsigned x) {
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x));
  return acc;
}
SDMOE_DEV float pp_add_hi(float acc, unsigned x) {
  asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(x));
  return acc;
}

// per-(row, expert) sums of one staged pass, in neuron order (gemm.hip expert_sums)
template <int S>
SDMOE_DEV void pp_expert_sums(const GppParams& p, const half_t* sg, int mrow0, int n0, int lane) {
  constexpr int NE = PNH / S;
  for (int id = lane; id < PRG * NE; id += 64) {
    const int r = id % PRG, e = id / PRG;
    const int m = mrow0 + r;
    const half_t* rp = sg + r * PNH + e * S;
    float acc = 0.f;
    if constexpr (S % 4 == 0) {
#pragma unroll
      for (int q = 0; q < S / 4; ++q) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        const u2 x = *reinterpret_cast<const u2*>(rp + 4 * q);
        acc = pp_add_hi(pp_add_lo(acc, x[0]), x[0]);
        acc = pp_add_hi(pp_add_lo(acc, x[1]), x[1]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < S; ++t) acc += (float)rp[t];
    }
    if (m < p.M) p.score[(long)m * p.ld_score + n0 / 2 / S + e] = (half_t)acc;
  }
}

template <bool RELU>  // ReLU specialised at compile time (a runtime act test branches inside every fragment)
__global__ __launch_bounds__(512, 1) void geglu_pp_kernel(GppParams p) {
  __shared__ __attribute__((aligned(1024))) char smem[PSMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3, wr = wq >> 1, wc = wq & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int ntile_wg = L < p.ntiles ? (p.ntiles - L + G - 1) / G : 0;
  const int NK = p.K / PBK;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, (short)0, p.w_bytes, 0x00020000);
  const int lch = lane & 7;

  // LDS-DMA of K-step ks of tile t into ring slot `slot`: main-group wave wq issues pieces j * 4 + wq (8 rows each);
  // the row offsets are recomputed per issue (keeping 13 of them live across the loop cost registers the
  // accumulators need)
  auto issue = [&](int t, int ks, int slot) {
    const int m0 = (t / p.ntn) * PBM, n0 = (t % p.ntn) * PBN;
    int lrow = lane >> 3;
    asm volatile("" : "+v"(lrow));  // opaque: the per-row products are not hoisted out of the loop (and spilled)
    char* sa = smem + slot * PSTAGE;
    const unsigned kb = (unsigned)(ks * PBK * 2);
#pragma unroll
    for (int j = 0; j < PA_PW; ++j) {
      const int r = 8 * (j * 4 + wq) + lrow, m = m0 + r;
      const unsigned vo = m < p.M ? (unsigned)((long)m * p.lda * 2) + (unsigned)((lch ^ pswz(r)) << 4) : PP_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void_pp*)(sa + (j * 4 + wq) * 1024), 16, vo, kb, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < PB_PW; ++j) {
      const int r = 8 * (j * 4 + wq) + lrow, n = n0 + r;
      const unsigned vo = n < p.N ? (unsigned)((long)n * p.ldw * 2) + (unsigned)((lch ^ pswz(r)) << 4) : PP_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lds_void_pp*)(sa + PBM * PRB + (j * 4 + wq) * 1024), 16, vo, kb,
                                               0, 0);
    }
  };

  float4v acc[PFM][PFN];
  bool issued = false;  // this wave issued LDS-DMA since its last drain
  if (ntile_wg > 0 && grp == 0) {
    issue(L, 0, 0);
    issued = true;
  }
  int gs = 0;  // global K-step (ring slot gs & 1)
  for (int k = 0; k <= ntile_wg; ++k) {
    const bool is_main = grp == (k & 1) && k < ntile_wg;  // wave-uniform
    const bool is_epi = grp != (k & 1) && k >= 1;
    const int tcur = L + k * G;
    if (is_main) {
#pragma unroll
      for (int i = 0; i < PFM; ++i)
#pragma unroll
        for (int j = 0; j < PFN; ++j) acc[i][j] = (float4v){0.f, 0.f, 0.f, 0.f};
    }
    // epilogue geometry (tile k - 1 of this workgroup)
    const int tprev = L + (k - 1) * G;
    const int mw = (tprev / p.ntn) * PBM + wr * PWM, nw = (tprev % p.ntn) * PBN + wc * PWN;
    // every wave takes NK workgroup barriers per phase, whatever its role; a wave that issued LDS-DMA drains it first
    auto step_sync = [&]() {
      if (issued) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        issued = false;
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    // the two roles as separate loops: each holds only its own temporaries beside the accumulators
    if (is_main) {
      for (int s = 0; s < NK; ++s, ++gs) {
        step_sync();
        // next stage into the other slot (read in step gs - 1, finished before the barrier): this tile's step s + 1,
        // or step 0 of the workgroup's next tile, which the other group computes in the next phase
        if (s + 1 < NK) {
          issue(tcur, s + 1, (gs + 1) & 1);
          issued = true;
        } else if (k + 1 < ntile_wg) {
          issue(tcur + G, 0, (gs + 1) & 1);
          issued = true;
        }
        const char* sa = smem + (gs & 1) * PSTAGE;
        const char* sbm = sa + PBM * PRB;
        auto read_a = [&](int kk, int i) -> half8 {
          const int row = wr * PWM + i * 16 + fr;
          return *reinterpret_cast<const half8*>(sa + row * PRB + (((kk * 4 + fg) ^ pswz(row)) << 4));
        };
        auto read_b = [&](int kk, int j) -> half8 {
          const int row = wc * PWN + j * 16 + fr;
          return *reinterpret_cast<const half8*>(sbm + row * PRB + (((kk * 4 + fg) ^ pswz(row)) << 4));
        };
        // gemm.hip's software-pipelined order: A fragments in pairs, the next pair read before the current MFMAs
        constexpr int NG = PFM / 2;
        half8 bcur[PFN];
#pragma unroll
        for (int j = 0; j < PFN; ++j) bcur[j] = read_b(0, j);
        half8 a0 = read_a(0, 0), a1 = read_a(0, 1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
          for (int g = 0; g < NG; ++g) {
            half8 n0 = a0, n1 = a1;
            if (g + 1 < NG) {
              n0 = read_a(kk, 2 * g + 2);
              n1 = read_a(kk, 2 * g + 3);
            } else if (kk == 0) {
              n0 = read_a(1, 0);
              n1 = read_a(1, 1);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < PFN; ++j) acc[2 * g][j] = mfma16x16x32(bcur[j], a0, acc[2 * g][j]);
#pragma unroll
            for (int j = 0; j < PFN; ++j) acc[2 * g + 1][j] = mfma16x16x32(bcur[j], a1, acc[2 * g + 1][j]);
            __builtin_amdgcn_sched_barrier(0);
            a0 = n0;
            a1 = n1;
          }
          if (kk == 0) {
#pragma unroll
            for (int j = 0; j < PFN; ++j) bcur[j] = read_b(1, j);
          }
        }
      }
    } else {
      // ---- one staging pass (fragment rows 2H, 2H + 1) of the previous tile: MODE_GEGLU's epilogue per wave. The
      // pass index must be a compile-time constant (a runtime index into acc[][] sends the array to scratch)
      auto epi_pass = [&](auto htag) {
        constexpr int H = decltype(htag)::value;
        int lane_o = lane;
        asm volatile("" : "+v"(lane_o));
        const int fr_e = lane_o & 15, fg_e = lane_o >> 4;
        half_t* sp = reinterpret_cast<half_t*>(smem + PSTG_OFF) + wq * 2 * PRG * PNH;
        half_t* sg = sp + PRG * PNH;
        float* gbias = reinterpret_cast<float*>(smem + PBIAS_OFF) + wq * PWN;
        if (H == 0) {
          for (int c = lane_o; c < PWN; c += 64) gbias[c] = (float)p.bias[nw + c];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const int nsel = 2 * fg_e;
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = 2 * H + ii;
#pragma unroll
          for (int j = 0; j < PFN; ++j) {
            const float4v v = acc[i][j];
            const float4v b = *reinterpret_cast<const float4v*>(gbias + 16 * j + 4 * fg_e);
            const h2 yv = {(half_t)(v[0] + b[0]), (half_t)(v[1] + b[1])};
            const h2 yg = {(half_t)(v[2] + b[2]), (half_t)(v[3] + b[3])};
            h2 ga;
            if constexpr (RELU) ga = __builtin_elementwise_max(yg, (h2){(half_t)0.f, (half_t)0.f});
            else ga = (h2){(half_t)apply_act((float)yg[0], p.act), (half_t)apply_act((float)yg[1], p.act)};
            const int off = (16 * ii + fr_e) * PNH + 8 * j + nsel;
            *reinterpret_cast<h2*>(sp + off) = yv * ga;
            *reinterpret_cast<h2*>(sg + off) = ga;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int mr0 = mw + H * PRG;
        constexpr int CPO = PNH / 8, RPI = 64 / CPO;  // 5 chunks per staged row, 12 rows per round
        const int lr = lane_o / CPO, lc = lane_o - lr * CPO;
        half_t* const cout = p.C + (long)(mr0 + lr) * p.ldc + nw / 2 + 8 * lc;
#pragma unroll
        for (int it = 0; it < (PRG + RPI - 1) / RPI; ++it) {
          const int r = it * RPI + lr;
          if (lr < RPI && r < PRG) {
            const half8 o = *reinterpret_cast<const half8*>(sp + r * PNH + 8 * lc);
            if (mr0 + r < p.M) *reinterpret_cast<half8*>(cout + (long)(it * RPI) * p.ldc) = o;
          }
        }
        if (p.score) {
          switch (p.esize) {
            case 20: pp_expert_sums<20>(p, sg, mr0, nw, lane_o); break;
            case 10: pp_expert_sums<10>(p, sg, mr0, nw, lane_o); break;
            case 40: pp_expert_sums<40>(p, sg, mr0, nw, lane_o); break;
            case 8: pp_expert_sums<8>(p, sg, mr0, nw, lane_o); break;
            case 5: pp_expert_sums<5>(p, sg, mr0, nw, lane_o); break;
            case 4: pp_expert_sums<4>(p, sg, mr0, nw, lane_o); break;
            case 2: pp_expert_sums<2>(p, sg, mr0, nw, lane_o); break;
            default: pp_expert_sums<1>(p, sg, mr0, nw, lane_o); break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      };
      static_assert(PFM / 2 == 4, "four staging passes");
      step_sync();
      if (is_epi) epi_pass(std::integral_constant<int, 0>());
      step_sync();
      if (is_epi) epi_pass(std::integral_constant<int, 1>());
      step_sync();
      if (is_epi) epi_pass(std::integral_constant<int, 2>());
      step_sync();
      if (is_epi) epi_pass(std::integral_constant<int, 3>());
      for (int s = 4; s < NK; ++s) step_sync();
      gs += NK;
    }
  }
}

int g_pp_cus = 0;

}  // namespace

// Launch the ping-pong routed GEGLU; SDMOE_EUNSUP when the shape is not one it takes (the caller falls back to
// MODE_GEGLU). Called by sdmoe_linear_geglu (gemm.hip) with its validated arguments.
int geglu_pp_launch(const void* A, long lda, const void* W, long ldw, const void* bias, void* P, long ldp, int M,
                    int F, int K, int act, void* score, long ld_score, int esize, int a_bytes, int w_bytes,
                    hipStream_t s) {
  if (K < 4 * PBK || K % PBK || (2 * F) % PBN || act == ACT_GELU) return SDMOE_EUNSUP;
  if (!g_pp_cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess || n <= 0)
      n = 256;
    g_pp_cus = n;
  }
  GppParams p{};
  p.A = (const half_t*)A; p.lda = lda; p.W = (const half_t*)W; p.ldw = ldw; p.bias = (const half_t*)bias;
  p.C = (half_t*)P; p.ldc = ldp; p.score = (half_t*)score; p.ld_score = ld_score; p.esize = esize;
  p.M = M; p.N = 2 * F; p.K = K; p.act = act; p.a_bytes = a_bytes; p.w_bytes = w_bytes;
  p.ntn = p.N / PBN;
  p.ntiles = ((M + PBM - 1) / PBM) * p.ntn;
  const int grid = p.ntiles < g_pp_cus ? p.ntiles : g_pp_cus;
  if (act == ACT_RELU) geglu_pp_kernel<true><<<grid, 512, 0, s>>>(p);
  else geglu_pp_kernel<false><<<grid, 512, 0, s>>>(p);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
