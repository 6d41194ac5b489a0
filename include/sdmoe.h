/*
 * sdmoe.h — C ABI of libsdmoe_hip.so, the MI355X (gfx950) kernels behind the MoE-fied Stable-Diffusion
 * denoising step of ruchikachavhan/diffusion-models-moe.
 *
 * Conventions (every entry point):
 *   - plain device pointers (fp16 = IEEE binary16, fp32, int32) and sizes; no framework types;
 *   - activations are row-major [rows, channels] with an explicit row stride `ld*` in ELEMENTS, so a
 *     channel slice of a wider buffer (zero-copy skip concatenation, fused QKV) is passed as (ptr, ld);
 *     spatial tensors are NHWC, i.e. [images * H * W, C];
 *   - `stream` is a hipStream_t (pass torch.cuda.current_stream().cuda_stream); every call is asynchronous,
 *     allocates nothing, never synchronises and is safe under hipGraph stream capture;
 *   - return 0 on success, >0 a hipError_t from the launch, <0 an argument error:
 *     -1 bad pointer/size, -2 unsupported shape/alignment, -3 unsupported mode;
 *   - an empty problem (zero rows / images / sequences) is a no-op that returns 0 before any pointer is checked
 *     (an empty framework tensor may carry a NULL data pointer).
 *   The library neither frees nor retains caller buffers.
 */
#ifndef SDMOE_H
#define SDMOE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Activation codes for `act` arguments. */
#define SDMOE_ACT_NONE 0
#define SDMOE_ACT_SILU 1
#define SDMOE_ACT_GELU 2 /* exact erf GELU, diffusers GEGLU.gelu / F.gelu */
#define SDMOE_ACT_RELU 3 /* relufied U-Net, sparsity/relufy_model.py:8-15 */
#define SDMOE_ACT_QUICK_GELU 4 /* x*sigmoid(1.702x), CLIP ViT-L text encoder MLP (transformers ACT2FN['quick_gelu']) */

const char* sdmoe_version(void);

/*
 * C[m, n] = act( sum_k A[m, k] * W[n, k] + bias[n] + coladd[m / rows_per_batch][n] ) + R[m, n]
 * W is nn.Linear layout [N, K]. workspace (optional, fp32, workspace_floats elements) enables split-K for
 * small tile grids; pass NULL/0 to disable.
 * Replaces: torch.nn.Linear / LoRACompatibleLinear.forward on the U-Net hot path (diffusers, external), the
 * GEGLU projection recomputed by MOEFy.hook_fn (neuron_receivers/moefy.py:12) and RemoveExperts.hook_fn
 * (neuron_receivers/remove_skilled_experts.py:26), and F.linear(x, W*(1-M), b) of
 * WandaRemoveNeuronsFast.linear_hook_fn (neuron_receivers/remove_wanda_neurons_fast.py:76, with
 * sdmoe_mask_weight). Requires K % 64 == 0, N % 8 == 0, strides % 8 == 0.
 */
int sdmoe_linear(const void* A, long lda, const void* W, long ldw, const void* bias, const void* coladd,
                 long coladd_bstride, int rows_per_batch, const void* R, long ldr, void* C, long ldc, int M, int N,
                 int K, int act, float* workspace, long workspace_floats, void* stream);

/*
 * 3x3 convolution, padding 1, on NHWC X [nimg, H, W, Cin] (pixel stride ldx): stride 1 or 2, or a fused
 * nearest-neighbour 2x upsample in front (upsample=1, output 2H x 2W). Weights [Cout][Cin/64][3][3][64]
 * (torch [Cout, Cin, 3, 3] -> permute(0, 2, 3, 1) -> [Cout, 9, Cin/64, 64] -> [Cout, Cin/64, 9, 64]).
 * Same fused epilogue as sdmoe_linear (bias, per-image coladd = time embedding, activation, residual R).
 * Replaces: diffusers ResnetBlock2D conv1/conv2 (+temb add/residual), Downsample2D, Upsample2D,
 * conv_in/conv_out of UNet2DConditionModel (external). Requires Cin % 64 == 0, Cout % 8 == 0.
 */
int sdmoe_conv3x3(const void* X, long ldx, int nimg, int H, int W, int Cin, const void* Wt, const void* bias,
                  const void* coladd, long coladd_bstride, const void* R, long ldr, void* Y, long ldy, int Cout,
                  int stride, int upsample, int act, float* workspace, long workspace_floats, void* stream);

/*
 * sdmoe_conv3x3 (stride 1) with a 1x1 projection shortcut folded in as extra K-steps:
 *   Y = conv3x3(X; Wt[:, :9 Cin]) + X2 Wt[:, 9 Cin:]^T + bias + coladd, X2 [nimg*H*W, Cin2] (row stride ldx2).
 * Wt [Cout][9 Cin + Cin2]: the conv weights in the sdmoe_conv3x3 layout followed by the shortcut's [Cout, Cin2]
 * columns; bias = conv2.bias + conv_shortcut.bias. Cin2 % 64 == 0.
 * Replaces: diffusers ResnetBlock2D conv2 + conv_shortcut + the residual add (`output_tensor = input_tensor +
 * hidden_states` with input_tensor = conv_shortcut(input_tensor); external) — no shortcut output is written or re-read.
 */
int sdmoe_conv3x3_sc(const void* X, long ldx, int nimg, int H, int W, int Cin, const void* Wt, const void* bias,
                     const void* coladd, long coladd_bstride, const void* X2, long ldx2, int Cin2, void* Y, long ldy,
                     int Cout, int act, float* workspace, long workspace_floats, void* stream);

/*
 * Y = conv3x3(act(GroupNorm(X))) [+ X2 W_sc^T] (+ bias + coladd + R): the ResNet conv with the GroupNorm(+SiLU)
 * in front of it applied INSIDE the conv (diffusers ResnetBlock2D: conv1(silu(norm1(x))), conv2(silu(norm2(h)))):
 * gn_scale / gn_shift are the per-image, per-channel fp32 affine of sdmoe_groupnorm_stats ([nimg][Cin]); the
 * normalised tensor is never written. Each 32-channel slice of the staged input halo is normalised once in LDS
 * (zero padding stays zero), with sdmoe_groupnorm_apply's arithmetic, so Y equals sdmoe_groupnorm_apply followed by
 * sdmoe_conv3x3 / sdmoe_conv3x3_sc bit for bit. X2 / Cin2: the optional folded 1x1 shortcut (raw input, not
 * normalised; then R must be NULL). Only the halo-tiled shapes take it (W = 64, Cout % 320 == 0, Cin <= 1280):
 * -3 (unsupported) otherwise -- the caller then applies the GroupNorm and calls sdmoe_conv3x3.
 */
int sdmoe_conv3x3_gn(const void* X, long ldx, int nimg, int H, int W, int Cin, const float* gn_scale,
                     const float* gn_shift, int silu, const void* Wt, const void* bias, const void* coladd,
                     long coladd_bstride, const void* R, long ldr, const void* X2, long ldx2, int Cin2, void* Y,
                     long ldy, int Cout, float* workspace, long workspace_floats, void* stream);
/* Y = (SiLU?)(X * scale[img, c] + shift[img, c]) on [nimg*HW, C] (the GroupNorm apply; scale/shift from
 * sdmoe_groupnorm_stats). C % 8 == 0. */
int sdmoe_groupnorm_apply(const void* X, long ldx, int nimg, int HW, int C, const float* scale, const float* shift,
                          int silu, void* Y, long ldy, void* stream);

/* Wm = W with every weight whose bit is set in bits [N][K/8] (little-endian bit order) zeroed: the device form
 * of W * (1 - M) (remove_wanda_neurons_fast.py:75, 80). */
int sdmoe_mask_weight(const void* W, const void* bits, long N, long K, void* Wm, void* stream);

/*
 * GroupNorm statistics of X [nimg, HW, C] (row stride ldx) with `groups` groups: writes per (image, channel)
 * scale = rstd*gamma and shift = beta - mean*scale (fp32 [nimg, C]) consumed by sdmoe_groupnorm_apply.
 * workspace: >= nimg*groups*64*2 floats.
 * Replaces: torch.nn.GroupNorm in ResnetBlock2D / Transformer2DModel / conv_norm_out (external).
 */
int sdmoe_groupnorm_stats(const void* X, long ldx, int nimg, int HW, int C, int groups, const void* gamma,
                          const void* beta, float eps, float* scale, float* shift, float* workspace,
                          long workspace_floats, void* stream);

/*
 * GroupNorm (+SiLU) in one call: Y = act(X * scale + shift) with the statistics of sdmoe_groupnorm_stats (scale /
 * shift are written too), i.e. sdmoe_groupnorm_stats followed by sdmoe_groupnorm_apply. Y must not alias X. Same
 * workspace as _stats.
 * Replaces: GroupNorm(+SiLU) in front of ResnetBlock2D conv1/conv2, Transformer2DModel.proj_in, conv_norm_out.
 */
int sdmoe_groupnorm(const void* X, long ldx, int nimg, int HW, int C, int groups, const void* gamma, const void* beta,
                    float eps, int silu, void* Y, long ldy, float* scale, float* shift, float* workspace,
                    long workspace_floats, void* stream);

/*
 * GroupNorm folded into the linear (1x1 conv) that consumes it — Transformer2DModel.norm -> proj_in (diffusers,
 * external): the normalised activation is never written or re-read.
 *  sdmoe_gn_fold (per call, after sdmoe_groupnorm_stats): for each image i, Wf[i][n, k] = fp16(W[n, k] * scale[i, k])
 *    (Wf [nimg][N][K], dense) and colbias[i][n] = bias[n] + sum_k W[n, k] * shift[i, k] (fp32 [nimg][N]; bias may
 *    be NULL), so proj_in(GN(x)) = x . Wf[i]^T + colbias[i] on the rows of image i. K % 8 == 0, ldw % 8 == 0.
 *  sdmoe_linear_per_image: C[m, n] = sum_k A[m, k] Wf[m / rows_per_batch][n, k] + colbias[m / rows_per_batch][n]
 *    + R[m, n] (weights of image i at Wf + i * w_bstride elements, row stride ldw; colbias row stride
 *    colbias_bstride). rows_per_batch % 256 == 0 (no GEMM tile straddles two images), K % 64 == 0, N % 8 == 0.
 * Replaces sdmoe_groupnorm + sdmoe_linear of Transformer2DModel (GroupNorm(32, C) -> proj_in).
 */
int sdmoe_gn_fold(const void* W, long ldw, int N, int K, const void* bias, const float* scale, const float* shift,
                  int nimg, void* Wf, float* colbias, void* stream);
int sdmoe_linear_per_image(const void* A, long lda, const void* Wf, long ldw, long w_bstride, const float* colbias,
                           long colbias_bstride, int rows_per_batch, const void* R, long ldr, void* C, long ldc, int M,
                           int N, int K, float* workspace, long workspace_floats, void* stream);

/* LayerNorm over the last dimension (C % 64 == 0, C <= 2048). Replaces BasicTransformerBlock norm1/2/3. */
int sdmoe_layernorm(const void* X, long ldx, void* Y, long ldy, int M, int C, const void* gamma, const void* beta,
                    float eps, void* stream);

/*
 * LayerNorm folded into the GEMM that consumes it (BasicTransformerBlock norm1 -> attn1 QKV, norm2 -> attn2 Q,
 * norm3 -> ff.net.0 GEGLU projection): no normalised activation is written or re-read.
 *  sdmoe_ln_fold (once per weight set): Wf[n, k] = fp16(W[n, k] * gamma[k]) (row stride ldf), wsum[n] = sum_k
 *    Wf[n, k] and bias_f[n] = bias[n] + sum_k W[n, k] * beta[k] (fp32; bias may be NULL).
 *  sdmoe_linear_ln: C[m, n] = rstd_m * (sum_k A[m, k] Wf[n, k] - mean_m * wsum[n]) + bias_f[n]
 *    = LayerNorm(A)[m] . W[n] + bias[n], mean_m / rstd_m = 1 / sqrt(var_m + eps) over the K channels of row m,
 *    accumulated (v_dot2_f32_f16 sums of x and x^2) from the A tiles the GEMM already stages in LDS.
 *  sdmoe_linear_geglu_ln: sdmoe_linear_geglu with the same fold (W / bias_f / wsum interleaved like W and bias).
 * K % 64 == 0 and K = the normalised dimension. Replaces sdmoe_layernorm + sdmoe_linear / sdmoe_linear_geglu
 * (diffusers BasicTransformerBlock.norm1/2/3 + to_q/k/v / GEGLU.proj).
 */
int sdmoe_ln_fold(const void* W, long ldw, int N, int K, const void* gamma, const void* beta, const void* bias,
                  void* Wf, long ldf, float* bias_f, float* wsum, void* stream);
int sdmoe_linear_ln(const void* A, long lda, const void* Wf, long ldw, const float* bias_f, const float* wsum,
                    float eps, void* C, long ldc, int M, int N, int K, void* stream);
int sdmoe_linear_geglu_ln(const void* A, long lda, const void* W, long ldw, const float* bias_f, const float* wsum,
                          float eps, void* P, long ldp, int M, int F, int K, int act, void* score, long ld_score,
                          int esize, void* stream);

/*
 * Scaled-dot-product attention, fp16: O[b, q, h*d:(h+1)*d] = softmax(Q K^T * scale) V per (image b, head h),
 * with Q [nimg*Nq, *] (stride ldq), K/V [nimg*Nk, *] (strides ldk/ldv), head h at column offset h*head_dim.
 * head_dim in {32, 40, 64, 80, 160}.
 * Replaces: diffusers Attention (attn1 self / attn2 cross) + AttnProcessor softmax(QK^T/sqrt(d))V (external;
 * SURVEY §2.3 K10).
 */
int sdmoe_attention(const void* Q, long ldq, const void* K, long ldk, const void* V, long ldv, void* O, long ldo,
                    int nimg, int Nq, int Nk, int heads, int head_dim, float scale, void* stream);

/*
 * MoE-fied GEGLU routing over Y = proj(x) [M, 2F] (value | gate halves, row stride ldy), F = 4C inner neurons:
 *   g = act(gate); score[e] = sum_{n: labels[n]==e} g[n]; removed experts score 0; sel = top-k(score) with
 *   ties toward the lowest expert id; keep[n] = sel[labels[n]] && !removed[labels[n]];
 *   out[m, n] = keep ? value*g : 0.
 * labels [F] int32 (0..E-1); e_off [E+1] / e_nid [F]: neurons grouped per expert (ascending neuron id);
 * removed_bits [ceil(E/32)] (bit e => expert e removed) or NULL; E == 0 => dense GEGLU (value * act(gate)).
 * Optional outputs: gate_out [M, F] (the masked gate the reference appends to self.gates), sel_out
 * [M, ceil(E/32)] uint32 top-k bitmask, score_out [M, E] fp16 scores. E <= 256, F % 8 == 0.
 * Replaces: MOEFy.hook_fn (neuron_receivers/moefy.py:10-27) and RemoveExperts.hook_fn
 * (neuron_receivers/remove_skilled_experts.py:24-55) after the projection: gelu, matmul(gate, patterns^T),
 * torch.topk, F.embedding(...).sum(-2), gate[mask==0]=0, hidden_states*gate, gate.cpu().
 */
int sdmoe_geglu_route(const void* Y, long ldy, int M, int F, int E, int k, int act, const int* labels,
                      const int* e_off, const int* e_nid, const unsigned* removed_bits, void* out, long ldo,
                      void* gate_out, long ldg, unsigned* sel_out, void* score_out, void* stream);

/*
 * Fused form of the same routing for balanced experts (the reference's KMeansConstrained split: every expert
 * has esize neurons, esize | 40), in two launches and without the [M, 2F] projection output:
 *  1. sdmoe_linear_geglu: P[m, n] = fp16(fp16(x W_v^T + b_v) * fp16(act(fp16(x W_g^T + b_g)))) for all F neurons
 *     and score[m, e] = fp16(sum over expert e's neurons of act(gate)) in the GEMM epilogue. W [2F, K] / bias
 *     [2F] hold the neurons permuted so every expert is contiguous (expert-major, ascending neuron id), value
 *     and gate rows interleaved in pairs ([v 2 | g 2] per neuron pair, sdmoe/ops.py geglu_rows). F % 80 == 0. score
 *     may be NULL
 *     (dense GEGLU). Same rounding points as sdmoe_linear + sdmoe_geglu_route.
 *  2. sdmoe_moe_topk_mask: per token, removed experts score 0, top-k (ties toward the lowest expert id) and
 *     zero every neuron of P whose expert is not selected or removed. sel_out as above (may be NULL).
 * The permuted P feeds the down projection with W_down's columns permuted the same way.
 * Replaces: the same reference hooks as sdmoe_geglu_route (moefy.py:10-27, remove_skilled_experts.py:24-55),
 * with SURVEY §3 K1+K2+K3 fused into the projection GEMM.
 */
int sdmoe_linear_geglu(const void* A, long lda, const void* W, long ldw, const void* bias, void* P, long ldp,
                       int M, int F, int K, int act, void* score, long ld_score, int esize, void* stream);
int sdmoe_moe_topk_mask(void* P, long ldp, int M, int F, int E, int esize, int k, const void* score,
                        long ld_score, const unsigned* removed_bits, unsigned* sel_out, void* stream);

/*
 * The same routing with the mask moved into the FFN down projection (ff.net.2) instead of a pass over P:
 *  sdmoe_moe_topk_keep: the selection of sdmoe_moe_topk_mask (removed experts score 0, top-k, ties toward the
 *    lowest id) written as keep bits of the expert-major permuted neurons: keep [F/64][M] 64-bit words, bit j of
 *    word (s, m) = neuron 64 s + j of token m is kept (selected and not removed). P is not touched. F % 64 == 0.
 *  sdmoe_linear_keep: C = (A with every dropped neuron zeroed) @ W^T + bias + R, the zeroing applied to the A
 *    fragments after their LDS read, so the result is bit-identical to sdmoe_moe_topk_mask followed by
 *    sdmoe_linear. A [M, K] (K = F), keep as above, W [N, K]. K % 64 == 0.
 * Replaces: gate[cur_mask == 0] = 0 and hidden_states * gate of MOEFy / RemoveExperts.hook_fn (moefy.py:23-26,
 * remove_skilled_experts.py:49-55) feeding ff.net.2 (diffusers FeedForward), without a pass over the product.
 */
int sdmoe_moe_topk_keep(int M, int F, int E, int esize, int k, const void* score, long ld_score,
                        const unsigned* removed_bits, void* keep, unsigned* sel_out, void* stream);
int sdmoe_linear_keep(const void* A, long lda, const void* keep, const void* W, long ldw, const void* bias,
                      const void* R, long ldr, void* C, long ldc, int M, int N, int K, float* workspace,
                      long workspace_floats, void* stream);

/*
 * sdmoe_linear_masked — SURVEY §8b's masked linear: C = (A ⊙ keep) @ (W ⊙ (1 - M))^T + bias + R with both masks
 * applied to the MFMA fragments after their LDS read (no masked copy of A or W is ever written):
 *   keep  (nullable): the A operand's per-(row, k) keep bits, layout of sdmoe_moe_topk_keep ([K/64][M] 64-bit words);
 *   wmask (nullable): the Wanda weight mask in the same K-step-major layout over W's rows ([K/64][N] 64-bit words,
 *     bit j of word (s, n) SET = W[n, 64 s + j] removed), made once per mask by sdmoe_wmask_kmajor.
 * Both NULL = sdmoe_linear without coladd/act. K % 64 == 0, N % 8 == 0, strides % 8 == 0.
 * Replaces: F.linear(input[0], W.clone() * (1 - M[t][l]), b) of WandaRemoveNeuronsFast.linear_hook_fn
 * (neuron_receivers/remove_wanda_neurons_fast.py:69-83) -- no W clone, no mask H2D copy, no second GEMM -- and,
 * with keep, that hook under MoE routing (the union remover of multi_concept_remover.py:43-53 on a MoE-fied U-Net,
 * BASELINE config 4).
 */
int sdmoe_linear_masked(const void* A, long lda, const void* keep, const void* W, long ldw, const void* wmask,
                        const void* bias, const void* R, long ldr, void* C, long ldc, int M, int N, int K,
                        float* workspace, long workspace_floats, void* stream);

/*
 * sdmoe_gemm_plan — host-only query (no device memory, no launch): the launch sdmoe_linear (mode 0),
 * sdmoe_linear_masked with keep (4), wmask (5) or both (6), or sdmoe_linear_ln (7) would make for an M x N x K
 * product with / without a residual and activation act, given workspace_floats of split-K workspace (0 = none):
 * out[0..4] = tile rows, tile columns, waves along M, waves along N, split-K factor. Masked modes take the plain
 * GEMM's plan (its split, hence each output's fp32 summation order), so sdmoe_linear_masked is bit-identical to
 * masking A / W first and calling sdmoe_linear; the tests check that over every U-Net shape. Splits depend on the
 * device's CU count (256 on MI355X, also the value without a device).
 */
int sdmoe_gemm_plan(int mode, int M, int N, int K, int has_residual, int act, long workspace_floats, int* out);

/*
 * sdmoe_wmask_kmajor — packed Wanda bits [N][K/8] (row stride ldb bytes; bit k%8 of byte (n, k/8) = W[n, k] removed;
 * the layout of the reference's [C, 4C] masks bit-packed, sdmoe/mask_io.py) -> out [K/64][N] 64-bit words for
 * sdmoe_linear_masked. perm (nullable, int32 [K]) permutes the columns: bit j of word (s, n) = mask(n, perm[64 s + j])
 * -- the FFN down projection's expert-major neuron order of the fused routed path. K % 64 == 0.
 */
int sdmoe_wmask_kmajor(const void* bits, long ldb, int N, int K, const int* perm, void* out, void* stream);

/*
 * Skill discovery on the same hook seam.
 * sdmoe_expert_mean_topk — GetExperts.hook_fn (neuron_receivers/get_experts.py:50-83): mean over tokens of the
 *   fp16 expert scores [M, E] (score_within_bb.mean(0): fp32 accumulate, one rounding to fp16), restricted to the
 *   bounding-box positions row_idx[0..n_idx) of every rows_per_img-row image when row_idx != NULL, then the k
 *   best experts (descending; ties toward the lowest id) into topk_out[k]; mean_out (fp16 [E]) optional.
 *   E <= 1024. workspace >= ceil(selected rows / 256) * E floats.
 * sdmoe_colnorm_accum — Wanda.hook_fn (neuron_receivers/wanda_receiver.py:37-57) + ColumnNormCalculator
 *   (utils.py:321-341): sumsq[f] += sum_m (P[m,f] / max(||P[m,:]||_2, 1e-12))^2 (the squared running column
 *   norm). workspace >= M + ceil(M / 256) * F floats.
 * sdmoe_wanda_mask — modularity/wanda.py:140-160: per row n of the down projection W [C, F], metric = fp16(|W| *
 *   norm) for the base and adjusted prompts (fp16 norms [F]); bit (n, f) = f among the kprune largest adjusted
 *   metrics of the row (ties toward the lowest column) AND metric_adj > metric_base. bits [C, F/8], the
 *   bit-packed layout WandaRemoveNeuronsFast consumes. F % 8 == 0, F <= 8192.
 */
int sdmoe_expert_mean_topk(const void* score, long ld_score, int M, int E, int rows_per_img, const int* row_idx,
                           int n_idx, int k, void* mean_out, int* topk_out, float* workspace, long workspace_floats,
                           void* stream);
int sdmoe_colnorm_accum(const void* P, long ldp, int M, int F, float* sumsq, float* workspace, long workspace_floats,
                        void* stream);
int sdmoe_wanda_mask(const void* W, long ldw, int C, int F, const void* norm_base, const void* norm_adj, int kprune,
                     void* bits, void* stream);

/*
 * Offline MoE-fication: ParamSplit.split (moefication/moe_utils.py:97-107) clusters the
 * L2-normalised gate rows of each GEGLU with KMeansConstrained(size_min = size_max = expert_size).
 * sdmoe_sqdist_f32 — D[i][c] = max(|x_i|^2 + |c_c|^2 - 2 x_i.c_c, 0), fp32 device arrays (exact fp32 MFMA
 *   dot products); X [n, d] (ld ldx), C [k, d] (ld ldc), D [n, k] (ld ldd).
 * sdmoe_balanced_assign — HOST function: labels[n] minimising sum cost[i][labels[i]] subject to every cluster
 *   holding exactly n/k points (the min-cost flow of k_means_constrained); cost [n, k] host doubles >= 0.
 *   Epsilon-scaling auction on integer costs (cost * scale; scale 0 = auto), exact for the integer costs.
 *   prices [n] (int64, optional) carries the slot prices across calls: warm = 1 starts from them.
 */
int sdmoe_sqdist_f32(const float* X, long ldx, const float* C, long ldc, int n, int k, int d, float* D, long ldd,
                     void* stream);
int sdmoe_balanced_assign(const double* cost, int n, int k, double scale, int64_t* prices, int warm, int* labels);

/*
 * Static "union-timesteps" mask (benchmarks/save_union_over_time.py:189-207): out bit =
 * (number of the T per-timestep Wanda masks with that bit set) > threshold, threshold = select_ratio * timesteps.
 * bits: T bit-packed masks of nbytes each (mask t at bits + t * t_stride_bytes, the [C, F/8] layout of
 * sdmoe_mask_weight); out: nbytes. Baking the result into ff.net.2 (W * (1 - M), :214-221) is sdmoe_mask_weight
 * with Wm = W. nbytes % 4 == 0.
 */
int sdmoe_union_over_time(const void* bits, long t_stride_bytes, int T, long nbytes, float threshold, void* out,
                          void* stream);

/*
 * VAE decoder helpers (diffusers AutoencoderKL.decode, external): the decoder mid-block's
 * single 512-wide attention head runs as sdmoe_linear (S = Q K^T) -> sdmoe_softmax_rows -> sdmoe_linear (O = P V,
 * with V^T from sdmoe_transpose).
 * sdmoe_softmax_rows — Y[r, :] = softmax(X[r, :]) for R rows of N (fp16, fp32 math; N % 8 == 0, N <= 8192).
 * sdmoe_transpose — Y [C, R] = X [R, C]^T, fp16, any leading dimensions.
 */
int sdmoe_softmax_rows(const void* X, long ldx, void* Y, long ldy, int R, int N, void* stream);
int sdmoe_transpose(const void* X, long ldx, void* Y, long ldy, int R, int C, void* stream);

/*
 * CLIP text encoder helpers (transformers CLIPTextModel, external — the pipelines' text_encoder
 * and the reference's hook_module='text' seam, base_receiver.py:59-65, remove_wanda_neurons_fast.py:114-120).
 * sdmoe_gather_rows — out[r, :C] = table[idx[r], :C] (+ add[r % period, :C] when add != NULL), fp16, C % 8 == 0.
 *   Replaces CLIPTextEmbeddings (token_embedding(ids) + position_embedding(arange)) and the pooled-output gather
 *   last_hidden_state[arange(B), eos_position].
 * sdmoe_attention_short — O = softmax(Q K^T * scale [+ causal mask]) V per (sequence, head) for N <= 128 tokens,
 *   head_dim <= 128 (% 8); same operand layout as sdmoe_attention. Replaces CLIPAttention with the causal mask of
 *   CLIPTextTransformer (_create_4d_causal_attention_mask).
 */
int sdmoe_gather_rows(const void* table, long ld_table, const int* idx, int R, int C, const void* add, long ld_add,
                      int period, void* out, long ld_out, void* stream);
int sdmoe_attention_short(const void* Q, long ldq, const void* K, long ldk, const void* V, long ldv, void* O,
                          long ldo, int nseq, int N, int heads, int head_dim, float scale, int causal, void* stream);

/* diffusers get_timestep_embedding for one timestep (t_dev if non-NULL, else t), fp16 [dim]. */
int sdmoe_timestep_embedding(void* out, const float* t_dev, float t, int dim, int flip_sin_to_cos, float freq_shift,
                             void* stream);
/* n timestep embeddings (t_dev[0..n)), row r written at out + (r/group)*ldo + (r%group)*dim: SDXL's add_time_proj
 * over the 6 micro-conditioning time ids per image (diffusers UNet2DConditionModel.get_aug_embed, "text_time";
 * the reference loads SDXL at utils.py:111-112). */
int sdmoe_timestep_embedding_rows(void* out, long ldo, const float* t_dev, int n, int group, int dim,
                                  int flip_sin_to_cos, float freq_shift, void* stream);

/* latents fp32 NCHW [B,4,H,W] -> U-Net input fp16 NHWC [ncopy*B, HW, ldo] channels 0..3 (CFG copies). */
int sdmoe_prepare_input(const float* lat, void* out, int B, int HW, long ldo, int ncopy, void* stream);

/*
 * Classifier-free guidance + DDIM (eta = 0) update of fp32 NCHW latents in place from eps fp16
 * [ncopy*B, HW, lde] (uncond first); optionally writes the next fp16 U-Net input (both CFG copies).
 * Replaces StableDiffusionPipeline's CFG combine + DDIMScheduler.step (external).
 */
int sdmoe_cfg_ddim_step(const void* eps, long lde, float* lat, int B, int HW, int do_cfg, float guidance,
                        float alpha_t, float alpha_prev, void* next_in, long ldn, void* stream);

/*
 * Classifier-free guidance + one linear multistep update of fp32 NCHW latents in place: the PLMS step of
 * diffusers' PNDMScheduler (skip_prk_steps, prediction_type "epsilon"; SD-1.x's default scheduler, 51 U-Net calls
 * for 50 steps — the reference's T = 51). Host-computed per step:
 *   coef[7] = {c_new, c_hist[0..3], a, b}, flags[3] = {store slot (-1 none), use cur, save cur}:
 *   e = CFG(eps); mo = c_new*e + sum c_hist[j]*hist[j]; hist[store] = e; src = use_cur ? cur : lat;
 *   if save_cur: cur = lat; lat = a*src - b*mo. hist [4][B*4*HW], cur [B*4*HW] fp32 device buffers.
 */
int sdmoe_cfg_multistep_step(const void* eps, long lde, float* lat, int B, int HW, int do_cfg, float guidance,
                             float* hist, float* cur, const float* coef, const int* flags, void* next_in, long ldn,
                             void* stream);

/* Tuning knobs for A/B experiments: knob 0 = GEMM LDS pipeline stages (0 auto, 2 or 3); knob 1 = forced GEMM tile
   (0 auto, 1 = 128x160, 2 = 64x160, 3 = 256x320 8-wave, 4 = 256x160 8-wave, 5 = 256x320 4x2-wave, 6 = 128x320 8-wave,
   7 = 128x160 8-wave, 8 = 64x320 8-wave; 7/8 plain GEMM / conv / LN-folded GEMM only); knob 9 = forced split-K
   factor (0 auto, 1 = never split, 2..32; halo convs: at most one 32-channel slice per split); knob 14 = split-K conv tile order: 1 (default) M-tile fastest (one XCD's
   workgroups share weight slices in its L2), 0 split fastest; knob 4 = attention kernel (0 auto by shape,
   1 = 32x32x16 MFMA kernel, 2 / 4 = 4-wave 16x16x32 kernel with 32 / 64 queries per wave, 64 for head_dim <= 40
   only; 8 = 16x16x32 kernel in 8-wave workgroups (head_dim <= 80));
   knob 6 = GEMM diagnostics bits (1 no K-loop loads, 2 no MFMA, 4 no epilogue, 8 no global stores);
   knob 7 = sdmoe_groupnorm at HW <= 256: 1 (default) statistics + apply in one launch with the rows held in
   registers, 2 the same launch re-reading the rows for the apply, 0 two launches;
   knob 8 = GEMM residual epilogue: 1 (default) output rounded to fp16 then the residual added in fp16 arithmetic
   (diffusers' fp16 `linear(x) + residual`), 0 = accumulator + residual rounded once (fp32 staging);
   knob 15 = top-k expert selection kernels: 0 (default) one token per wave at M <= 16384, four above, and the keep
   bits at E <= 64 with one quad of lanes per token; 1 / 4 = always the ballot kernel at one / four tokens per wave;
   knob 16 = halo-tiled 3x3 convs: 1 (default) where measured faster (64- and 16-wide outputs, the upsample convs,
   32-wide outputs with Cin >= 1280; grids of <= 32 256-row tiles -- one prompt per call -- on 128-row tiles for the
   64-, 16- and narrow-input 32-wide outputs and the 16 -> 32 upsample), 2 = every 128-row halo tile instead, 3 = the
   default plus every 32-wide output on 256-row tiles, 0 = off;
   knob 20 = table-GELU routed GEGLU tiles: 1 (default) 256x320 like the ReLU kernel, 0 = 256x160 (4x2 waves);
   knob 21 = convs with at most 32 output channels (conv_out): 1 (default) 128x32 tiles, 0 = 128x64;
   knob 23 = fp16 GEMM / conv epilogues: 1 (default) 16-B row pieces stored straight from the MFMA fragments (two
   v_permlane16_swap per fragment pair, no LDS staging) when there is no residual, 2 = always, 0 = staged in LDS. */
int sdmoe_tune(int knob, int value);

/*
 * Registers, for the calling thread's current HIP device, the fp16 GELU table the GEGLU kernels apply for
 * act == SDMOE_ACT_GELU (sdmoe_linear_geglu / _ln, sdmoe_geglu_route): table[i] = gelu(x) for the 16384 fp16 inputs
 * x with 2^-5 <= |x| < 8, i = ((bits(x) & 0x7fff) - 0x2800) | (sign(x) << 13), device memory, 16-B aligned, kept
 * alive by the caller while registered (NULL unregisters: the kernels then evaluate 0.5 x erfc(-x / sqrt 2) in
 * fp32, within 1 fp16 ulp). The host layer fills it with the reference module's own activation (GEGLU.gelu =
 * F.gelu on fp16 tensors, diffusers activations.py; the hook's module.gelu(gate), remove_skilled_experts.py:27,
 * moefy.py:13) evaluated on every such input, so the fused routed GEGLU reproduces the reference's fp16 gate
 * values bit for bit on all of them; |x| < 2^-5, |x| >= 8 are computed (see csrc/common.h gelu_tab_h).
 * No GPU call; not stream-ordered: register before launching work that reads it.
 */
int sdmoe_set_gelu_table(const void* table);

/* out = a + b (fp16, n % 8 == 0). */
int sdmoe_add(const void* a, const void* b, void* out, long n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SDMOE_H */
