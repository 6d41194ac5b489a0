// MoE-fied GEGLU routing for gfx950: the hot arithmetic of the reference receivers
//   MOEFy.hook_fn            (neuron_receivers/moefy.py:10-27)
//   RemoveExperts.hook_fn    (neuron_receivers/remove_skilled_experts.py:24-55)
// restated as ONE kernel over the GEGLU projection output Y = proj(x) = [value | gate] (diffusers GEGLU:
// first half value, second half gate, moe_utils.py:68-72):
//   g      = act(gate)                   (exact-erf GELU, or ReLU for the relufied U-Net), rounded to fp16
//   score  = g @ patterns^T              per-expert fp32 sum over its neurons in neuron order, rounded to fp16
//                                        (removed experts: patterns row zeroed -> score exactly 0)
//   sel    = top-k(score)                wave-wide 16-bit radix select on order-preserving fp16 keys,
//                                        ties at the k-th value broken toward the LOWEST expert id
//   keep_n = sel[label[n]] && !removed[label[n]]   (embedding(labels, patterns').sum(-2) != 0)
//   out    = keep ? fp16(value * g) : 0             (gate[mask == 0] = 0; hidden_states * gate)
// One wave per token, no [tokens, k, 4C] temporaries (reference K5), no host sync (reference K8 is an optional
// gate_out capture written on device).
#include "common.h"
#include "../../include/sdmoe.h"

namespace {

struct RouteParams {
  const half_t* Y; long ldy;
  int M, F, E, k, act;
  const int* labels;        // [F] expert id of each inner neuron
  const int* e_off;         // [E+1] CSR offsets into e_nid
  const int* e_nid;         // [F] neuron ids grouped by expert, ascending within an expert
  const uint32_t* removed;  // [ceil(E/32)] or null
  half_t* out; long ldo;
  half_t* gate_out; long ldg;
  uint32_t* sel_out;        // [M][ceil(E/32)] or null (top-k result, before the removal mask)
  half_t* score_out;        // [M][E] or null
  const half_t* gelu_tab;   // act == GELU: the registered fp16 GELU table (gelu_tab_h), or null (erfc form)
};

SDMOE_DEV uint32_t order_key(half_t s) {
  unsigned short u = __builtin_bit_cast(unsigned short, s);
  if ((u & 0x7fff) == 0) u = 0;  // -0 == +0 for topk
  return (u & 0x8000) ? (uint32_t)(~u & 0xffff) : (uint32_t)(u | 0x8000);
}

template <int SLOTS>
__global__ __launch_bounds__(256) void geglu_route_kernel(RouteParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int F = p.F;
  half_t* gact = reinterpret_cast<half_t*>(smem) + wave * F;
  uint32_t* selw = reinterpret_cast<uint32_t*>(reinterpret_cast<half_t*>(smem) + 4 * F) + wave * 8;
  const int m = blockIdx.x * 4 + wave;
  const bool live = m < p.M;
  const int mm = live ? m : 0;
  const half_t* yrow = p.Y + (long)mm * p.ldy;
  const int nch = F >> 3;

  // 1) activated gate -> LDS (fp16, as the reference's module.gelu(gate) on an fp16 tensor)
  for (int c = lane; c < nch; c += 64) {
    half8 v = *reinterpret_cast<const half8*>(yrow + F + 8 * c);
    half8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = p.gelu_tab ? gelu_tab_h(v[j], p.gelu_tab) : (half_t)apply_act((float)v[j], p.act);
    *reinterpret_cast<half8*>(gact + 8 * c) = o;
  }
  __syncthreads();

  const int nw = (p.E + 31) >> 5;
  if (p.E > 0) {
    // 2) expert scores
    uint32_t key[SLOTS];
    bool valid[SLOTS];
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int e = lane + 64 * i;
      valid[i] = e < p.E;
      half_t sc = (half_t)0.f;
      if (valid[i]) {
        float acc = 0.f;
        const int j0 = p.e_off[e], j1 = p.e_off[e + 1];
        for (int j = j0; j < j1; ++j) acc += (float)gact[p.e_nid[j]];
        sc = (half_t)acc;
        if (p.removed && ((p.removed[e >> 5] >> (e & 31)) & 1u)) sc = (half_t)0.f;
        if (p.score_out && live) p.score_out[(long)m * p.E + e] = sc;
      }
      key[i] = valid[i] ? order_key(sc) : 0u;
    }
    // 3) radix select of the k-th largest key
    uint32_t T = 0;
    for (int bit = 15; bit >= 0; --bit) {
      const uint32_t cand = T | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < SLOTS; ++i) cnt += __popcll(__ballot(valid[i] && key[i] >= cand));
      if (cnt >= p.k) T = cand;
    }
    int gt = 0;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) gt += __popcll(__ballot(valid[i] && key[i] > T));
    const int need = p.k - gt;
    const unsigned long long below = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
    int rank_base = 0;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const bool tie = valid[i] && key[i] == T;
      const unsigned long long tm = __ballot(tie);
      const bool sel = p.k > 0 && valid[i] && (key[i] > T || (tie && rank_base + __popcll(tm & below) < need));
      rank_base += __popcll(tm);
      const unsigned long long sm = __ballot(sel);
      if (lane == 0) {
        if (2 * i < 8) selw[2 * i] = (uint32_t)sm;
        if (2 * i + 1 < 8) selw[2 * i + 1] = (uint32_t)(sm >> 32);
      }
    }
    __syncthreads();
    if (p.sel_out && live && lane < nw) p.sel_out[(long)m * nw + lane] = selw[lane];
    if (p.removed && lane < nw) selw[lane] &= ~p.removed[lane];
    __syncthreads();
  } else {
    __syncthreads();
    __syncthreads();
  }

  // 4) gated output
  if (!live) return;
  for (int c = lane; c < nch; c += 64) {
    half8 hv = *reinterpret_cast<const half8*>(yrow + 8 * c);
    half8 ga = *reinterpret_cast<const half8*>(gact + 8 * c);
    half8 o, go;
    if (p.E > 0) {
      const int4* lp = reinterpret_cast<const int4*>(p.labels + 8 * c);
      int4 l0 = lp[0], l1 = lp[1];
      int lab[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool keep = (selw[lab[j] >> 5] >> (lab[j] & 31)) & 1u;
        go[j] = keep ? ga[j] : (half_t)0.f;
        o[j] = keep ? (half_t)((float)hv[j] * (float)ga[j]) : (half_t)0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { go[j] = ga[j]; o[j] = (half_t)((float)hv[j] * (float)ga[j]); }
    }
    *reinterpret_cast<half8*>(p.out + (long)m * p.ldo + 8 * c) = o;
    if (p.gate_out) *reinterpret_cast<half8*>(p.gate_out + (long)m * p.ldg + 8 * c) = go;
  }
}

// Top-k expert mask over a routed-GEGLU product computed by sdmoe_linear_geglu (experts contiguous, esize
// neurons each): per token, scores (fp16, removed experts -> 0) -> the same radix top-k as above -> zero the
// neurons of every expert that is not selected (or is removed). One wave per TPW tokens: the TPW score rows are
// loaded up front (one 128-B row per token and wave left the kernel latency-bound: ~30 us for 65536 tokens), then
// selected one after the other; only zeros are written.
// KEEPOUT: P is left alone; the kept neurons are written as keep bits for the down projection to apply to its
// A operand (sdmoe_linear_keep): keep[(n / 64) * M + m] bit n % 64, one 64-bit word per token and 64-neuron
// K-step, staged in LDS so each K-step's 16 words of the workgroup's tokens leave as one whole 128-B line.
struct Slots64 {  // per-slot 64-bit expert masks (slot i = experts 64 i .. 64 i + 63)
  unsigned long long a = 0, b = 0, c = 0, d = 0;
  SDMOE_DEV void set(int i, unsigned long long v) {
    if (i == 0) a = v; else if (i == 1) b = v; else if (i == 2) c = v; else d = v;
  }
  SDMOE_DEV unsigned long long get(int i) const { return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d)); }
};

// TPW tokens per wave (4, or 1 for M <= 16384: the per-token radix search is a serial ballot / popcount chain, and
// with 4 tokens per wave the 4096-token launches ran 256 workgroups -- one wave per SIMD, 18.7 us at E = 256);
// always 16 tokens per workgroup (4 or 16 waves)
template <int SLOTS, int SC, bool KEEPOUT, int TPW>  // SC: compile-time expert size (0 = runtime S)
__global__ __launch_bounds__(64 * 16 / TPW) void moe_topk_mask_kernel(
    half_t* __restrict__ P, long ldp, int M, int F, int E, int S_, int k, const half_t* __restrict__ score, long lds,
    const uint32_t* __restrict__ removed, uint32_t* __restrict__ sel_out, unsigned long long* __restrict__ keep) {
  constexpr int WPB = 16 / TPW;                 // waves per workgroup
  constexpr int TPB = TPW * WPB;                // tokens per workgroup
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int S = SC ? SC : S_;
  const int mw = blockIdx.x * TPB + wave * TPW;  // first token of this wave
  if (!KEEPOUT && mw >= M) return;  // wave-uniform; the mask form has no block-level barrier below
  const int nw = (E + 31) >> 5;
  // the TPW score rows first, all loads in flight before anything waits on them (unconditional loads at clamped
  // indices: a per-lane validity branch around each load made the compiler wait for each separately), then the
  // removed bits; separate row arrays keep every index constant
  half_t sc0[SLOTS], sc1[SLOTS], sc2[SLOTS], sc3[SLOTS];
  static_assert(TPW == 4 || TPW == 1, "one or four score rows per wave");
  auto load_row = [&](half_t (&dst)[SLOTS], int t) {
    const half_t* srow = score + (long)min(mw + t, M - 1) * lds;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) dst[i] = srow[min(lane + 64 * i, E - 1)];
  };
  load_row(sc0, 0);
  if constexpr (TPW == 4) {
    load_row(sc1, 1);
    load_row(sc2, 2);
    load_row(sc3, 3);
  }
  uint32_t rmw[SLOTS];  // removed bits of this lane's experts
  bool valid[SLOTS];
#pragma unroll
  for (int i = 0; i < SLOTS; ++i) {
    const int e = lane + 64 * i;
    valid[i] = e < E;
    const uint32_t r = removed ? (removed[min(e, E - 1) >> 5] >> (e & 31)) & 1u : 0u;
    rmw[i] = valid[i] ? r : 0u;
  }
  const unsigned long long below = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  // KEEPOUT: [TPB][F/64 + 1] words in dynamic LDS (16 tokens x 8 B = one whole 128-B line per K-step)
  extern __shared__ unsigned long long kw_dyn[];
  const int kws = (F >> 6) + 1;

  auto process = [&](const half_t (&scr)[SLOTS], int t) {
    const int m = mw + t;
    const bool live = m < M;
    uint32_t key[SLOTS];
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) key[i] = valid[i] ? order_key(rmw[i] ? (half_t)0.f : scr[i]) : 0u;
    uint32_t T = 0;
    for (int bit = 15; bit >= 0; --bit) {
      const uint32_t cand = T | (1u << bit);
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < SLOTS; ++i) cnt += __popcll(__ballot(valid[i] && key[i] >= cand));
      if (cnt >= k) T = cand;
    }
    int gt = 0;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) gt += __popcll(__ballot(valid[i] && key[i] > T));
    const int need = k - gt;
    // selection and kept experts (selected, not removed) as wave-uniform ballots: bit e & 63 of slot e >> 6. They
    // stay in registers -- no lane reads a word another lane wrote to LDS
    // (four named scalars, not an array: a select chain over array elements is folded back into a dynamically
    //  indexed private array, i.e. scratch)
    int rank_base = 0;
    Slots64 sel_sl, keep_sl;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const bool tie = valid[i] && key[i] == T;
      const unsigned long long tm = __ballot(tie);
      const bool sel = k > 0 && valid[i] && (key[i] > T || (tie && rank_base + __popcll(tm & below) < need));
      rank_base += __popcll(tm);
      sel_sl.set(i, __ballot(sel));
      keep_sl.set(i, __ballot(sel && !rmw[i]));
    }
    auto slot_of = [&](const Slots64& v, int sidx) { return v.get(sidx); };
    if (sel_out && live && lane < nw)
      sel_out[(long)m * nw + lane] = (uint32_t)(slot_of(sel_sl, lane >> 1) >> (32 * (lane & 1)));
    if constexpr (KEEPOUT) {
      // one lane per 64-neuron K-step ORs in the neuron ranges of the (at most 64 / S + 2) experts it overlaps
      for (int ks = lane; ks < (F >> 6); ks += 64) {
        const int n0 = 64 * ks;
        const int e0 = n0 / S, e1 = (n0 + 63) / S;
        unsigned long long w = 0;
        for (int e = e0; e <= e1 && e < E; ++e) {
          if ((slot_of(keep_sl, e >> 6) >> (e & 63)) & 1ull) {
            const int lo = max(e * S, n0) - n0, hi = min((e + 1) * S, n0 + 64) - n0;
            w |= (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo;
          }
        }
        kw_dyn[(wave * TPW + t) * kws + ks] = w;
      }
    } else {
      if (!live) return;  // wave-uniform
      half_t* row = P + (long)m * ldp;
      for (int c = lane; c < (F >> 3); c += 64) {
        unsigned kb = 0;  // keep bit per neuron of this 8-neuron chunk
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int e = (8 * c + j) / S;
          kb |= (unsigned)((slot_of(keep_sl, e >> 6) >> (e & 63)) & 1ull) << j;
        }
        if (kb == 0xffu) continue;
        half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (kb) {
          v = *reinterpret_cast<const half8*>(row + 8 * c);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!((kb >> j) & 1u)) v[j] = (half_t)0.f;
        }
        *reinterpret_cast<half8*>(row + 8 * c) = v;
      }
    }
  };
  process(sc0, 0);
  if constexpr (TPW == 4) {
    process(sc1, 1);
    process(sc2, 2);
    process(sc3, 3);
  }
  if constexpr (KEEPOUT) {
    __syncthreads();
    const int m0 = blockIdx.x * TPB, nks = F >> 6;
    for (int idx = threadIdx.x; idx < nks * TPB; idx += WPB * 64) {
      const int ks = idx / TPB, t = idx - ks * TPB;
      if (m0 + t < M) keep[(long)ks * M + m0 + t] = kw_dyn[t * kws + ks];
    }
  }
}

// DPP moves inside a quad of lanes (quad_perm): lane q reads lane SEL(q)
template <int CTRL>
SDMOE_DEV uint32_t quad_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
constexpr int QP_XOR1 = 0xB1, QP_XOR2 = 0x4E, QP_B0 = 0x00, QP_B1 = 0x55, QP_B2 = 0xAA, QP_B3 = 0xFF;

// Top-k keep bits for E <= 64 experts with ONE QUAD OF LANES PER TOKEN (16 tokens per wave): lane q of a quad holds
// the order keys of experts 16 q .. 16 q + 15 in registers and runs the same 16-bit radix search as above on them,
// its counts summed over the quad with two DPP adds per bit -- no ballots, no SALU chain, 4096 independent waves at
// M = 65536 (the ballot kernel's serial per-token chain left it at ~28 us there). Same selection rule: the k
// largest keys, ties at the k-th key toward the lowest expert id. Each lane then writes every 4th 64-neuron keep
// word of its token (16 tokens x 8 B per word and quad lane: whole 128-B lines).
// FULL (E = 64 experts of 20 neurons, 16-B aligned score rows -- every 64x64-level FFN of SD-1.4): no validity
// masks, and lane q's 16 experts are exactly neurons 320 q .. 320 q + 319, i.e. keep words 5 q .. 5 q + 4, whose
// expert -> bit-range pattern is then a compile-time constant (only the lane's own keep bits enter them).
template <bool FULL, int SC>  // compile-time expert size (0 = runtime S)
__global__ __launch_bounds__(256) void moe_topk_keep_quad_kernel(
    int M, int F, int E, int S_, int k, const half_t* __restrict__ score, long lds,
    const uint32_t* __restrict__ removed, uint32_t* __restrict__ sel_out, unsigned long long* __restrict__ keep) {
  static_assert(!FULL || SC == 20, "FULL: 64 experts of 20 neurons");
  const int S = SC ? SC : S_;
  const int lane = threadIdx.x & 63, q = lane & 3;
  const int m = blockIdx.x * 64 + (threadIdx.x >> 2);
  const int mc = min(m, M - 1);
  const half_t* srow = score + (long)mc * lds + 16 * q;
  half_t s[16];
  if constexpr (FULL) {  // E == 64, 16-B aligned rows
    const half8 a = *reinterpret_cast<const half8*>(srow), b = *reinterpret_cast<const half8*>(srow + 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] = a[i]; s[8 + i] = b[i]; }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = srow[min(16 * q + i, E - 1) - 16 * q];
  }
  const uint64_t rm64 = removed ? ((uint64_t)removed[0] | (E > 32 ? (uint64_t)removed[1] << 32 : 0ull)) : 0ull;
  const uint32_t rm16 = (uint32_t)(rm64 >> (16 * q)) & 0xffffu;
  const int nval = min(max(E - 16 * q, 0), 16);  // valid experts of this lane
  const uint32_t vmask = FULL || nval >= 16 ? 0xffffu : ((1u << nval) - 1u);
  uint32_t key[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) key[i] = order_key(((rm16 >> i) & 1u) ? (half_t)0.f : s[i]);
  auto quad_sum = [](uint32_t c) {
    c += quad_mov<QP_XOR1>(c);
    return c + quad_mov<QP_XOR2>(c);
  };
  uint32_t T = 0;
  for (int bit = 15; bit >= 0; --bit) {
    const uint32_t cand = T | (1u << bit);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) c += (((vmask >> i) & 1u) && key[i] >= cand) ? 1u : 0u;
    if ((int)quad_sum(c) >= k) T = cand;
  }
  uint32_t gt = 0, ties = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool v = (vmask >> i) & 1u;
    gt += (v && key[i] > T) ? 1u : 0u;
    ties += (v && key[i] == T) ? 1u : 0u;
  }
  const int need = k - (int)quad_sum(gt);
  // ties of the quad's lower lanes (lower expert ids) come first
  const uint32_t t0 = quad_mov<QP_B0>(ties), t1 = quad_mov<QP_B1>(ties), t2 = quad_mov<QP_B2>(ties);
  int r = (q > 0 ? (int)t0 : 0) + (q > 1 ? (int)t1 : 0) + (q > 2 ? (int)t2 : 0);
  uint32_t sel16 = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool v = (vmask >> i) & 1u;
    const bool tie = v && key[i] == T;
    const bool sel = k > 0 && v && (key[i] > T || (tie && r < need));
    r += tie ? 1 : 0;
    sel16 |= (sel ? 1u : 0u) << i;
  }
  const uint32_t keep16 = sel16 & ~rm16;
  // the token's 64 selection / keep bits in every lane of the quad
  const uint32_t slo = quad_mov<QP_B0>(sel16) | (quad_mov<QP_B1>(sel16) << 16);
  const uint32_t shi = quad_mov<QP_B2>(sel16) | (quad_mov<QP_B3>(sel16) << 16);
  const uint64_t keep64 = (uint64_t)(quad_mov<QP_B0>(keep16) | (quad_mov<QP_B1>(keep16) << 16)) |
                          ((uint64_t)(quad_mov<QP_B2>(keep16) | (quad_mov<QP_B3>(keep16) << 16)) << 32);
  if (m >= M) return;
  if (sel_out && q < ((E + 31) >> 5)) sel_out[(long)m * ((E + 31) >> 5) + q] = q ? shi : slo;
  if constexpr (FULL) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      unsigned long long w = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int lo = max(20 * i, 64 * j) - 64 * j, hi = min(20 * i + 20, 64 * j + 64) - 64 * j;
        if (hi > lo) w |= ((keep16 >> i) & 1u) ? ((1ull << (hi - lo)) - 1ull) << lo : 0ull;
      }
      keep[(long)(5 * q + j) * M + m] = w;
    }
    (void)keep64;
    return;
  }
  const int nks = F >> 6;
  for (int ks = q; ks < nks; ks += 4) {
    const int n0 = 64 * ks, e0 = n0 / S, e1 = min((n0 + 63) / S, E - 1);
    unsigned long long w = 0;
    auto add = [&](int e) {
      if ((keep64 >> e) & 1ull) {
        const int lo = max(e * S, n0) - n0, hi = min((e + 1) * S, n0 + 64) - n0;
        w |= (hi - lo >= 64 ? ~0ull : ((1ull << (hi - lo)) - 1ull)) << lo;
      }
    };
    if constexpr (SC > 0) {
      constexpr int SPAN = 64 / (SC > 0 ? SC : 1) + 2;  // experts one 64-neuron word can overlap
#pragma unroll
      for (int d = 0; d < SPAN; ++d)
        if (e0 + d <= e1) add(e0 + d);
    } else {
      for (int e = e0; e <= e1; ++e) add(e);
    }
    keep[(long)ks * M + m] = w;
  }
}

// The FULL quad kernel's scheme for E = 16 L experts of 20 neurons with a GROUP of L = 8 / 16 lanes per token (E = 128:
// the 32x32-level FFNs of SD-1.x and SDXL's 64x64 level; E = 256: the 16x16 / 8x8 levels; 8 / 4 tokens per wave):
// lane r of a group holds experts 16 r .. 16 r + 15 (= neurons 320 r .. 320 r + 319 = keep words 5 r .. 5 r + 4, a
// compile-time bit pattern), the 16-bit radix counts are summed over the group with DPP (quad xor 1 / 2, then
// row_half_mirror, row_mirror: no ballots, no SALU chain, no LDS), ties at the k-th key go to the lowest expert id via
// a group prefix of the tie counts. Same selection rule and outputs as moe_topk_mask_kernel's keep form, which it
// replaces for these E (that kernel's one token per wave walked a serial ballot / popcount chain: 13.0 us at M =
// 16384, E = 128 and 8.5 us at M = 4096, E = 256 in the metric's profile, latency-bound on a few MB).
template <int L>
__global__ __launch_bounds__(256) void moe_topk_keep_group_kernel(
    int M, int F, int E, int k, const half_t* __restrict__ score, long lds, const uint32_t* __restrict__ removed,
    uint32_t* __restrict__ sel_out, unsigned long long* __restrict__ keep) {
  static_assert(L == 8 || L == 16, "8 or 16 lanes per token");
  const int lane = threadIdx.x & 63, r = lane & (L - 1);
  const int m = blockIdx.x * (256 / L) + (int)(threadIdx.x / L);
  const int mc = min(m, M - 1);
  const half_t* srow = score + (long)mc * lds + 16 * r;
  const half8 a = *reinterpret_cast<const half8*>(srow), b = *reinterpret_cast<const half8*>(srow + 8);
  const uint32_t rm16 = removed ? (removed[(16 * r) >> 5] >> ((16 * r) & 31)) & 0xffffu : 0u;
  uint32_t key[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    key[i] = order_key(((rm16 >> i) & 1u) ? (half_t)0.f : a[i]);
    key[8 + i] = order_key(((rm16 >> (8 + i)) & 1u) ? (half_t)0.f : b[i]);
  }
  auto group_sum = [](uint32_t c) {
    c += quad_mov<QP_XOR1>(c);
    c += quad_mov<QP_XOR2>(c);
    c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x141, 0xf, 0xf, false);  // row_half_mirror
    if constexpr (L == 16) c += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)c, 0x140, 0xf, 0xf, false);  // row_mirror
    return c;
  };
  uint32_t T = 0;
  for (int bit = 15; bit >= 0; --bit) {
    const uint32_t cand = T | (1u << bit);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) c += key[i] >= cand ? 1u : 0u;
    if ((int)group_sum(c) >= k) T = cand;
  }
  uint32_t gt = 0, ties = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    gt += key[i] > T ? 1u : 0u;
    ties += key[i] == T ? 1u : 0u;
  }
  const int need = k - (int)group_sum(gt);
  // exclusive prefix of the group's tie counts (lower lanes = lower expert ids first): Hillis-Steele inside the group
  uint32_t inc = ties;
#pragma unroll
  for (int d = 1; d < L; d <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)inc, d, 64);
    if (r >= d) inc += v;
  }
  int rk = (int)(inc - ties);
  uint32_t sel16 = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const bool tie = key[i] == T;
    const bool sel = k > 0 && (key[i] > T || (tie && rk < need));
    rk += tie ? 1 : 0;
    sel16 |= (sel ? 1u : 0u) << i;
  }
  const uint32_t keep16 = sel16 & ~rm16;
  const uint32_t sel_hi = quad_mov<QP_XOR1>(sel16);  // the odd neighbour's experts (32-expert selection words)
  if (m >= M) return;
  if (sel_out && (r & 1) == 0) sel_out[(long)m * (E >> 5) + (r >> 1)] = sel16 | (sel_hi << 16);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    unsigned long long w = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int lo = max(20 * i, 64 * j) - 64 * j, hi = min(20 * i + 20, 64 * j + 64) - 64 * j;
      if (hi > lo) w |= ((keep16 >> i) & 1u) ? ((1ull << (hi - lo)) - 1ull) << lo : 0ull;
    }
    keep[(long)(5 * r + j) * M + m] = w;
  }
  (void)F;
}

}  // namespace

int g_topk_tpw = 0;  // sdmoe_tune knob 15: 0 = by M (default; keep bits at E <= 64: one quad per token), 1 / 4 =
                     // always the ballot kernel at 1 / 4 tokens per wave

template <bool KEEPOUT>
int launch_topk(half_t* P, long ldp, int M, int F, int E, int esize, int k, const half_t* sc, long ld_score,
                const uint32_t* rm, uint32_t* sel_out, unsigned long long* keep, hipStream_t s) {
  const int blocks = (M + 15) / 16;  // 16 tokens per workgroup: 4 waves x 4 tokens, or 16 waves x 1 (M <= 16384)
  const size_t lds = KEEPOUT ? (size_t)16 * ((F >> 6) + 1) * 8 : 0;
  const bool one = g_topk_tpw == 1 || (M <= 16384 && g_topk_tpw != 4);
#define SDMOE_TOPK_MASK(SL, SC)                                                                                 \
  if (one)                                                                                                      \
    moe_topk_mask_kernel<SL, SC, KEEPOUT, 1><<<blocks, 1024, lds, s>>>(P, ldp, M, F, E, esize, k, sc, ld_score, \
                                                                       rm, sel_out, keep);                      \
  else                                                                                                          \
    moe_topk_mask_kernel<SL, SC, KEEPOUT, 4><<<blocks, 256, lds, s>>>(P, ldp, M, F, E, esize, k, sc, ld_score,  \
                                                                      rm, sel_out, keep)
  if (esize == 20) {  // the reference's expert size (KMeansConstrained, 20 neurons): divisions by a constant
    if (E <= 64) SDMOE_TOPK_MASK(1, 20);
    else if (E <= 128) SDMOE_TOPK_MASK(2, 20);
    else SDMOE_TOPK_MASK(4, 20);
  } else {
    if (E <= 64) SDMOE_TOPK_MASK(1, 0);
    else if (E <= 128) SDMOE_TOPK_MASK(2, 0);
    else SDMOE_TOPK_MASK(4, 0);
  }
#undef SDMOE_TOPK_MASK
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}

extern "C" int sdmoe_moe_topk_mask(void* P, long ldp, int M, int F, int E, int esize, int k, const void* score,
                                   long ld_score, const unsigned* removed_bits, unsigned* sel_out, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!P || !score || M < 0 || F <= 0 || E <= 0 || esize <= 0) return SDMOE_EARG;
  if (F % 8 || ldp % 8 || E * esize != F || ld_score < E) return SDMOE_ESHAPE;
  if (E > 256) return SDMOE_EUNSUP;
  if (k < 0 || k > E) return SDMOE_EARG;
  return launch_topk<false>((half_t*)P, ldp, M, F, E, esize, k, (const half_t*)score, ld_score,
                            (const uint32_t*)removed_bits, sel_out, nullptr, (hipStream_t)stream);
}

extern "C" int sdmoe_moe_topk_keep(int M, int F, int E, int esize, int k, const void* score, long ld_score,
                                   const unsigned* removed_bits, void* keep, unsigned* sel_out, void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!keep || !score || M < 0 || F <= 0 || E <= 0 || esize <= 0) return SDMOE_EARG;
  if (F % 64 || E * esize != F || ld_score < E) return SDMOE_ESHAPE;
  if (E > 256 || esize > 40) return SDMOE_EUNSUP;
  if (k < 0 || k > E) return SDMOE_EARG;
  if (E <= 64 && g_topk_tpw == 0) {
    const bool full = E == 64 && esize == 20 && ld_score % 8 == 0 && ((uintptr_t)score & 15) == 0;
    hipStream_t s = (hipStream_t)stream;
    const int g = (M + 63) / 64;
    const half_t* sc = (const half_t*)score;
    const uint32_t* rm = (const uint32_t*)removed_bits;
    unsigned long long* kp = (unsigned long long*)keep;
    if (full)
      moe_topk_keep_quad_kernel<true, 20><<<g, 256, 0, s>>>(M, F, E, esize, k, sc, ld_score, rm, sel_out, kp);
    else if (esize == 20)
      moe_topk_keep_quad_kernel<false, 20><<<g, 256, 0, s>>>(M, F, E, esize, k, sc, ld_score, rm, sel_out, kp);
    else
      moe_topk_keep_quad_kernel<false, 0><<<g, 256, 0, s>>>(M, F, E, esize, k, sc, ld_score, rm, sel_out, kp);
    SDMOE_CHECK_LAUNCH();
    return SDMOE_OK;
  }
  if ((E == 128 || E == 256) && esize == 20 && g_topk_tpw == 0 && ld_score % 8 == 0 && ((uintptr_t)score & 15) == 0) {
    hipStream_t s = (hipStream_t)stream;
    const half_t* sc = (const half_t*)score;
    const uint32_t* rm = (const uint32_t*)removed_bits;
    unsigned long long* kp = (unsigned long long*)keep;
    if (E == 128)
      moe_topk_keep_group_kernel<8><<<(M + 31) / 32, 256, 0, s>>>(M, F, E, k, sc, ld_score, rm, sel_out, kp);
    else
      moe_topk_keep_group_kernel<16><<<(M + 15) / 16, 256, 0, s>>>(M, F, E, k, sc, ld_score, rm, sel_out, kp);
    SDMOE_CHECK_LAUNCH();
    return SDMOE_OK;
  }
  return launch_topk<true>(nullptr, 0, M, F, E, esize, k, (const half_t*)score, ld_score, (const uint32_t*)removed_bits,
                           sel_out, (unsigned long long*)keep, (hipStream_t)stream);
}

extern "C" int sdmoe_geglu_route(const void* Y, long ldy, int M, int F, int E, int k, int act, const int* labels,
                                 const int* e_off, const int* e_nid, const unsigned* removed_bits, void* out,
                                 long ldo, void* gate_out, long ldg, unsigned* sel_out, void* score_out,
                                 void* stream) {
  if (M == 0) return SDMOE_OK;
  if (!Y || !out || M < 0 || F <= 0 || E < 0) return SDMOE_EARG;
  if (F % 8 || ldy % 8 || ldo % 8 || (gate_out && ldg % 8)) return SDMOE_ESHAPE;
  if (E > 256) return SDMOE_EUNSUP;
  if (E > 0 && (!labels || !e_off || !e_nid || k < 0 || k > E)) return SDMOE_EARG;
  if (!(act == ACT_GELU || act == ACT_RELU || act == ACT_NONE || act == ACT_SILU)) return SDMOE_EUNSUP;
  RouteParams p{(const half_t*)Y, ldy, M, F, E, k, act, labels, e_off, e_nid, removed_bits,
                (half_t*)out, ldo, (half_t*)gate_out, ldg, sel_out, (half_t*)score_out,
                act == ACT_GELU ? sdmoe_gelu_tab_current() : nullptr};
  const size_t smem = (size_t)4 * F * sizeof(half_t) + 4 * 8 * sizeof(uint32_t);
  if (smem > 160 * 1024) return SDMOE_ESHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (M + 3) / 4;
  if (E <= 64) geglu_route_kernel<1><<<blocks, 256, smem, s>>>(p);
  else if (E <= 128) geglu_route_kernel<2><<<blocks, 256, smem, s>>>(p);
  else geglu_route_kernel<4><<<blocks, 256, smem, s>>>(p);
  SDMOE_CHECK_LAUNCH();
  return SDMOE_OK;
}
