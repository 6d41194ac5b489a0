"""SD-1.x UNet2DConditionModel on the sdmoe HIP kernels (gfx950), with diffusers' module tree and names.

The module tree exists so the reference's receiver API works unchanged: `model.unet.named_modules()` yields
`down_blocks.0.attentions.0.transformer_blocks.0.ff.net.0` (a GEGLU) and `...ff.net.2` (a
LoRACompatibleLinear), forward hooks registered on them fire once per U-Net call in execution order, and
`module.patterns` / `module.k` / `module.gelu` / `module.proj` mean what they mean in the reference
(base_receiver.py:49-57, helper.py:48-62, relufy_model.py:28-40).

Everything else is MI355X-first:
  * activations live in HBM as NHWC fp16 [images*H*W, C] (the transformer's token layout, so no permutes);
  * skip concatenations are zero-copy: each up-block ResNet input is one [rows, C_prev + C_skip] buffer; the
    down path writes its skip outputs straight into the right-hand channel slice and reads them from there;
  * GroupNorm is one coalesced statistics pass + one vectorised apply(+SiLU) pass feeding the LDS-DMA
    conv/GEMM; the time-embedding add, bias, residual adds and activations are GEMM/conv epilogues;
  * attention projections are fused (QKV [3C, C], cross KV [2C, 768]) and attention reads the heads in place;
  * all 22 ResNet time-embedding projections run as ONE GEMM per step.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .config import UNetConfig

CTX_LEN = 77
FUSED_GEGLU = True  # fused projection+GEGLU(+expert scores) path where eligible (tests flip it for A/B parity)
FUSED_KEEP = True   # fused path: top-k mask applied inside the down projection (sdmoe_linear_keep) instead of a pass
# BasicTransformerBlock LayerNorms folded into the QKV / Q / GEGLU projection GEMMs (SDMOE_FUSED_LN=0: explicit, A/B)
FUSED_LN = os.environ.get("SDMOE_FUSED_LN", "1") != "0"
FUSED_LN_FFN = os.environ.get("SDMOE_FUSED_LN_FFN", "0") == "1"  # norm3 into the GEGLU GEMM too (slower, see run)
# ResnetBlock2D conv_shortcut (1x1) folded into conv2 as extra K-steps (sdmoe_conv3x3_sc; SDMOE_FUSED_SC=0: separate)
FUSED_SC = os.environ.get("SDMOE_FUSED_SC", "1") != "0"
# Transformer2DModel GroupNorm folded into proj_in (per-image weights, sdmoe_gn_fold + sdmoe_linear_per_image) at
# latents of >= 32x32 (SDMOE_FUSED_GN=0: GroupNorm apply pass + proj_in, A/B)
FUSED_GN = os.environ.get("SDMOE_FUSED_GN", "1") != "0"
GN_FOLD_MIN_HW = 1024
IN_PAD = 64    # conv_in input channels padded 4 -> 64 (K-step of the implicit GEMM)
OUT_PAD = 8    # conv_out output channels padded 4 -> 8 (16-B epilogue stores)


def _buf(t):
    return nn.Parameter(t, requires_grad=False)


class LoRACompatibleLinear(nn.Module):
    """nn.Linear stand-in (diffusers 0.27 LoRACompatibleLinear naming); weight [out, in] fp16."""

    def __init__(self, weight, bias=None):
        super().__init__()
        self.weight = _buf(weight)
        self.bias = None if bias is None else _buf(bias)
        self._sdmoe_deferred = 0

    @property
    def in_features(self):
        return self.weight.shape[1]

    @property
    def out_features(self):
        return self.weight.shape[0]

    def run(self, x2d, weight=None, **kw):
        """y = x2d @ W^T + b (W = self.weight unless a stand-in of the same shape is given, e.g. a baked masked copy)."""
        return ops.linear(x2d, self.weight if weight is None else weight, self.bias, **kw)

    def forward(self, x, scale=1.0):
        if self._sdmoe_deferred and self._forward_hooks:
            return None  # a sdmoe receiver hook computes this module's output (no double compute)
        shp = x.shape
        return self.run(x.reshape(-1, shp[-1])).view(*shp[:-1], self.out_features)


class Conv2d(nn.Module):
    """3x3 conv; weight stored [Cout, Cin/64, 3, 3, 64] fp16 (the implicit GEMM's K order, ops.conv_weight)."""

    def __init__(self, weight, bias, stride=1):
        super().__init__()
        self.weight = _buf(weight)
        self.bias = _buf(bias)
        self.stride = stride


class Norm(nn.Module):
    def __init__(self, weight, bias, eps, groups=None):
        super().__init__()
        self.weight = _buf(weight)
        self.bias = _buf(bias)
        self.eps = eps
        self.groups = groups

    def stats(self, x2d, nimg, HW):
        return ops.groupnorm_stats(x2d, nimg, HW, self.weight, self.bias, self.eps, self.groups)

    def normalize(self, x2d, nimg, HW, silu):
        """act(GroupNorm(x)) as a new tensor (sdmoe_groupnorm: statistics + apply in one ABI call)."""
        return ops.groupnorm(x2d, nimg, HW, self.weight, self.bias, self.eps, self.groups, silu)


def act_code(fn):
    """Map a GEGLU `.gelu` callable to the kernel's activation code (diffusers gelu or the relufied ReLU)."""
    from_name = getattr(fn, "_sdmoe_act", None)
    if from_name is not None:
        return ops.ACT_BY_NAME[from_name]
    if fn is F.gelu or fn is torch.nn.functional.gelu:
        return ops.ACT_GELU
    if fn is F.relu or fn is torch.relu:
        return ops.ACT_RELU
    raise NotImplementedError(f"GEGLU activation {fn!r} has no HIP kernel (supported: gelu, relu)")


def _gelu(x):
    return F.gelu(x)


_gelu._sdmoe_act = "gelu"


class GEGLU(nn.Module):
    """diffusers GEGLU: proj = Linear(C, 8C); out = value * gelu(gate) (value = first half).

    MoE-fication state (set by moefication.helper.modify_ffn): `patterns` [E, 4C] 0/1 and `k`."""

    def __init__(self, proj: LoRACompatibleLinear):
        super().__init__()
        self.proj = proj
        self.gelu = _gelu
        self.patterns = None
        self.k = None
        self.bounding_box = None
        self._routing = None
        self._routing_key = None
        self._sdmoe_deferred = 0
        # fused projection+GEGLU (+expert scores) path: interleaved/permuted proj weights, and what the last
        # routed() call produced (its output pointer and permutation) for the FeedForward down projection
        self._allow_permuted_out = False
        self._out_perm = None
        self._out_keep = None  # (keep bits, output pointer) when the top-k mask is left to the down projection
        self._il_key = None
        self._il = None
        # LayerNorm deferred into the projection GEMM (FeedForward.run, FUSED_LN): (the un-normalised input view
        # handed to this module's call, its Norm). routed()/scored()/dense() fold it into the GEMM on the fused
        # path and apply it explicitly on every other path, so a caller of those methods always gets LN(x) semantics
        self._ln_pending = None
        self._il_ln_key = None
        self._il_ln = None

    @property
    def inner_dim(self):
        return self.proj.out_features // 2

    def routing(self):
        """Device expert layout for the current (patterns, k); rebuilt only when either changes."""
        if self.patterns is None:
            return None
        key = (id(self.patterns), self.patterns.data_ptr(), int(self.k))
        if self._routing_key != key:
            if getattr(self, "labels", None) is not None and self.labels.numel() == self.inner_dim:
                self._routing = ops.Routing(self.labels, self.patterns.shape[0], int(self.k), self.proj.weight.device)
            else:
                self._routing = ops.Routing.from_patterns(self.patterns, int(self.k), self.proj.weight.device)
            self._routing_key = key
        return self._routing

    def _interleaved(self, routing):
        w = self.proj.weight
        key = (id(routing), w.data_ptr(), w._version,
               None if self.proj.bias is None else (self.proj.bias.data_ptr(), self.proj.bias._version))
        if self._il_key != key:
            perm = routing.perm if routing is not None else None
            self._il = ops.interleave_geglu(w.data, None if self.proj.bias is None else self.proj.bias.data, perm)
            self._il_key = key
        return self._il

    def _take_ln(self, x):
        """The Norm deferred into this call when x is the pending un-normalised input, else None."""
        pend = self._ln_pending
        return pend[1] if pend is not None and x is pend[0] else None

    def _interleaved_ln(self, routing, norm):
        w, b = self.proj.weight, self.proj.bias
        key = (id(routing), w.data_ptr(), w._version, None if b is None else (b.data_ptr(), b._version),
               norm.weight.data_ptr(), norm.weight._version, norm.bias.data_ptr(), norm.bias._version)
        if self._il_ln_key != key:
            fold = ops.LNFold(w.data, norm.weight.data, norm.bias.data, norm.eps, None if b is None else b.data)
            self._il_ln = ops.interleave_ln_fold(fold, routing.perm if routing is not None else None)
            self._il_ln_key = key
        return self._il_ln

    def routed(self, x, removed=None, want_gate=False, sel_out=None, score_out=None):
        """proj GEMM + routed GEGLU kernel. x: [..., C] fp16. Returns (out [..., 4C], masked gate or None).
        sel_out (optional int32 [tokens, ceil(E/32)]) receives the per-token top-k expert bitmask, score_out
        (optional fp16 [tokens, E]) the expert scores the top-k ranked (removed experts: 0 on the unfused path; their
        raw gate sums on the fused path, where the removal is applied inside the top-k kernel).

        When the caller (FeedForward) allows it and the experts are balanced, the fused path runs instead:
        the projection GEMM's epilogue computes value*act(gate) and the expert scores, a small kernel applies
        the top-k mask; `out` is then in the expert-major neuron order (self._out_perm records it)."""
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        norm = self._take_ln(x)
        routing = self.routing()
        act = act_code(self.gelu)
        self._out_perm = None
        self._out_keep = None
        if (FUSED_GEGLU and self._allow_permuted_out and not want_gate and self.inner_dim % 80 == 0 and x2.shape[1] % 64 == 0
                and (routing is None or routing.fusable)):
            if norm is not None:
                w_il = b_il = None
                lnf = self._interleaved_ln(routing, norm)
            else:
                w_il, b_il = self._interleaved(routing)
                lnf = None
            if routing is None:
                out = ops.linear_geglu(x2, w_il, b_il, act, ln=lnf)
            else:
                score = score_out if score_out is not None else \
                    torch.empty((x2.shape[0], routing.E), dtype=torch.float16, device=x.device)
                out = ops.linear_geglu(x2, w_il, b_il, act, score=score, esize=routing.esize, ln=lnf)
                if FUSED_KEEP and routing.F % 64 == 0:
                    # the dropped experts' neurons are zeroed by the down projection as it reads them
                    # (sdmoe_linear_keep); `out` is then the unmasked product, an operand only FeedForward consumes
                    keep = ops.moe_topk_keep(score, routing, x2.shape[0], removed=removed, sel_out=sel_out)
                    self._out_keep = (keep, out.data_ptr())
                else:
                    ops.moe_topk_mask(out, score, routing, removed=removed, sel_out=sel_out)
                self._out_perm = (routing, out.data_ptr())
            return out.view(*shp[:-1], self.inner_dim), None
        if norm is not None:
            x2 = ops.layernorm(x2, norm.weight, norm.bias, norm.eps)
        y = self.proj.run(x2)
        gate = torch.empty((x2.shape[0], self.inner_dim), dtype=torch.float16, device=x.device) if want_gate else None
        out = ops.geglu_route(y, self.routing(), act_code(self.gelu), removed=removed, gate_out=gate, sel_out=sel_out,
                              score_out=score_out)
        out = out.view(*shp[:-1], self.inner_dim)
        return out, (gate.view(*shp[:-1], self.inner_dim) if want_gate else None)

    def scored(self, x):
        """Dense GEGLU output (no top-k mask) plus per-token expert scores [tokens, E] fp16 — the arithmetic of
        GetExperts.hook_fn (neuron_receivers/get_experts.py:50-67). Fused path when eligible (out permuted
        expert-major, recorded in _out_perm for the down projection)."""
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        norm = self._take_ln(x)
        if norm is not None:
            x2 = ops.layernorm(x2, norm.weight, norm.bias, norm.eps)
        routing = self.routing()
        act = act_code(self.gelu)
        self._out_perm = None
        score = torch.empty((x2.shape[0], routing.E), dtype=torch.float16, device=x.device)
        if (FUSED_GEGLU and self._allow_permuted_out and self.inner_dim % 80 == 0 and x2.shape[1] % 64 == 0
                and routing.fusable):
            w_il, b_il = self._interleaved(routing)
            out = ops.linear_geglu(x2, w_il, b_il, act, score=score, esize=routing.esize)
            self._out_perm = (routing, out.data_ptr())
        else:
            out = ops.geglu_route(self.proj.run(x2), routing, act, score_out=score, k=routing.E)
        return out.view(*shp[:-1], self.inner_dim), score

    def dense(self, x):
        """value * act(gate) in the natural neuron order, ignoring any MoE routing (Wanda discovery,
        neuron_receivers/wanda_receiver.py:37-57)."""
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        norm = self._take_ln(x)
        if norm is not None:
            x2 = ops.layernorm(x2, norm.weight, norm.bias, norm.eps)
        act = act_code(self.gelu)
        self._out_perm = None
        if FUSED_GEGLU and self.inner_dim % 80 == 0 and x2.shape[1] % 64 == 0:
            w_il, b_il = self._interleaved(None)
            out = ops.linear_geglu(x2, w_il, b_il, act)
        else:
            out = ops.geglu_route(self.proj.run(x2), None, act)
        return out.view(*shp[:-1], self.inner_dim)

    def forward(self, x, scale=1.0):
        if self._sdmoe_deferred and self._forward_hooks:
            return None  # a sdmoe receiver hook computes the routed output (no double compute)
        return self.routed(x)[0]


def _sole_receiver(module, method):
    """The sdmoe receiver owning `module`'s only forward hook, if it has `method`; else None."""
    hooks = list(module._forward_hooks.values())
    if len(hooks) != 1:
        return None
    owner = getattr(hooks[0], "__self__", None)
    if owner is None or not getattr(owner, "_sdmoe_receiver", False) or not hasattr(owner, method):
        return None
    return owner


def _ln_safe_hook(module, owner):
    """True when `module`'s one forward hook is exactly the function its receiver class marks LN-safe
    (`_sdmoe_ln_safe_hook`: a hook_fn that only hands input[0] to GEGLU.routed(), which resolves a LayerNorm deferred
    into the call). Compares the REGISTERED hook's function with the marker looked up on the class, so a subclass that
    overrides hook_fn without re-marking it is not LN-safe."""
    if owner is None:
        return False
    hooks = list(module._forward_hooks.values())
    fn = getattr(hooks[0], "__func__", None) if len(hooks) == 1 else None
    return fn is not None and fn is getattr(type(owner), "_sdmoe_ln_safe_hook", None)


class FeedForward(nn.Module):
    def __init__(self, geglu, down):
        super().__init__()
        self.net = nn.ModuleList([geglu, nn.Dropout(0.0), down])
        self._wperm_key = None
        self._wperm = None

    def _down_weight_permuted(self, routing):
        w = self.net[2].weight
        key = (id(routing), w.data_ptr(), w._version)
        if self._wperm_key != key:
            self._wperm = w.data[:, routing.perm.to(w.device)].contiguous()
            self._wperm_key = key
        return self._wperm

    def run(self, x2d, nimg, residual, ln=None):
        """GEGLU -> down projection (+ the block's residual). The fused routed GEGLU (GEGLU.routed) hands over an
        expert-permuted product whose top-k mask is still pending (applied by the down projection as it reads it);
        that intermediate must stay private to this FeedForward, so the fused path runs only when
          * the GEGLU has no forward hook, or exactly one owned by an sdmoe receiver (whose hook_fn computes it), and
          * ff.net.2 has no hook, or exactly one owned by a receiver that can apply its weight mask in the fused form
            (WandaRemoveNeuronsFast.fused_linear: same (t, l) mask, columns permuted, counter advanced).
        Any other hook sees exactly the reference's tensors (natural neuron order, mask applied)."""
        geglu, down = self.net[0], self.net[2]
        dhooks = bool(down._forward_hooks)
        masker = _sole_receiver(down, "fused_linear") if dhooks else None
        owner = _sole_receiver(geglu, "hook_fn") if geglu._forward_hooks else None
        geglu._allow_permuted_out = (not dhooks or masker is not None) and (not geglu._forward_hooks or owner is not None)
        # ln (the block's norm3): deferred into the GEGLU projection when nothing but GEGLU's own methods can see
        # the module input (no hook, or one sdmoe receiver whose hook hands input[0] to routed()); else applied here
        if ln is not None and geglu._forward_hooks and not _ln_safe_hook(geglu, owner):
            x2d = ops.layernorm(x2d, ln.weight, ln.bias, ln.eps)
            ln = None
        xv = x2d.view(nimg, -1, x2d.shape[1])
        geglu._ln_pending = (xv, ln) if ln is not None else None
        try:
            h = geglu(xv)
        finally:
            geglu._allow_permuted_out = False
            geglu._ln_pending = None
        h2 = h.reshape(-1, h.shape[-1])
        perm = geglu._out_perm
        permuted = perm is not None and perm[1] == h2.data_ptr()
        if dhooks and not (permuted and masker is not None):
            o = down(h)  # the hook sees the natural neuron order
            return ops.add(o.reshape(residual.shape).contiguous(), residual)
        if permuted:
            wp = self._down_weight_permuted(perm[0])
            keep = geglu._out_keep
            keep = keep[0] if keep is not None and keep[1] == h2.data_ptr() else None
            if masker is not None:
                return masker.fused_linear(down, h2, keep, perm[0].perm_dev, wp, residual)
            if keep is not None:
                return ops.linear_keep(h2, keep, wp, down.bias, residual=residual)
            return ops.linear(h2, wp, down.bias, residual=residual)
        return down.run(h2, residual=residual)


class Attention(nn.Module):
    def __init__(self, wq, wk, wv, wo, bo, heads, self_attn):
        super().__init__()
        self.heads = heads
        self.self_attn = self_attn
        C = wq.shape[0]
        if self_attn:
            self.w_qkv = _buf(torch.cat([wq, wk, wv], 0).contiguous())
            self.to_q = LoRACompatibleLinear(self.w_qkv.data[:C])
            self.to_k = LoRACompatibleLinear(self.w_qkv.data[C:2 * C])
            self.to_v = LoRACompatibleLinear(self.w_qkv.data[2 * C:])
        else:
            self.w_kv = _buf(torch.cat([wk, wv], 0).contiguous())
            self.to_q = LoRACompatibleLinear(wq)
            self.to_k = LoRACompatibleLinear(self.w_kv.data[:C])
            self.to_v = LoRACompatibleLinear(self.w_kv.data[C:])
        self.to_out = nn.ModuleList([LoRACompatibleLinear(wo, bo), nn.Dropout(0.0)])
        self._kv_key = None
        self._kv = None
        self._ln_key = None
        self._ln_fold = None

    def _fold(self, norm):
        """LNFold of the query (cross) or fused QKV (self) projection with the block's norm in front."""
        w = self.w_qkv if self.self_attn else self.to_q.weight
        key = (w.data_ptr(), w._version, norm.weight.data_ptr(), norm.weight._version, norm.bias.data_ptr(),
               norm.bias._version)
        if self._ln_key != key:
            self._ln_fold = ops.LNFold(w.data, norm.weight.data, norm.bias.data, norm.eps)
            self._ln_key = key
        return self._ln_fold

    def cross_kv(self, ctx2d):
        """K|V projection of the text context. The context is the same tensor for every denoising step of one
        pipeline call, so the projection is computed at its first U-Net evaluation and reused by the others
        (loop-invariant: bit-identical to recomputing it; keyed on the context object, its version and the
        weights' version, so a new prompt batch or an in-place edit recomputes)."""
        key = (ctx2d, ctx2d._version, self.w_kv.data_ptr(), self.w_kv._version)
        k = self._kv_key
        if k is None or k[0] is not ctx2d or k[1:] != key[1:]:
            self._kv = ops.linear(ctx2d, self.w_kv)
            self._kv_key = key
        return self._kv

    def run(self, x2d, nimg, N, residual, ctx2d=None, ln=None):
        """ln (the block's norm1/norm2): x2d is un-normalised and the LayerNorm is folded into the projection."""
        C = x2d.shape[1]
        if self.self_attn:
            qkv = ops.linear(x2d, self.w_qkv) if ln is None else ops.linear_ln(x2d, self._fold(ln))
            a = ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nimg, N, N, self.heads)
        else:
            q = ops.linear(x2d, self.to_q.weight) if ln is None else ops.linear_ln(x2d, self._fold(ln))
            kv = self.cross_kv(ctx2d)
            a = ops.attention(q, kv[:, :C], kv[:, C:], nimg, N, ctx2d.shape[0] // nimg, self.heads)
        return self.to_out[0].run(a, residual=residual)


class BasicTransformerBlock(nn.Module):
    def __init__(self, norm1, attn1, norm2, attn2, norm3, ff):
        super().__init__()
        self.norm1, self.attn1, self.norm2, self.attn2, self.norm3, self.ff = norm1, attn1, norm2, attn2, norm3, ff

    def run(self, hs, nimg, N, ctx2d):
        if FUSED_LN and hs.shape[1] % 64 == 0:
            # norm1 / norm2 folded into the QKV / Q projections (sdmoe_linear_ln). norm3 stays explicit unless
            # FUSED_LN_FFN: folding it into the routed-GEGLU GEMM (sdmoe_linear_geglu_ln) measured slower than
            # sdmoe_layernorm + the fused GEGLU (193 vs 172 + 15 us at 64x64, 144 vs 127 + 9 at 32x32): the LDS row
            # statistics cost the GEGLU main loop more than the LayerNorm pass they replace
            hs = self.attn1.run(hs, nimg, N, residual=hs, ln=self.norm1)
            hs = self.attn2.run(hs, nimg, N, residual=hs, ctx2d=ctx2d, ln=self.norm2)
            if FUSED_LN_FFN:
                return self.ff.run(hs, nimg, residual=hs, ln=self.norm3)
            n = ops.layernorm(hs, self.norm3.weight, self.norm3.bias, self.norm3.eps)
            return self.ff.run(n, nimg, residual=hs)
        n = ops.layernorm(hs, self.norm1.weight, self.norm1.bias, self.norm1.eps)
        hs = self.attn1.run(n, nimg, N, residual=hs)
        n = ops.layernorm(hs, self.norm2.weight, self.norm2.bias, self.norm2.eps)
        hs = self.attn2.run(n, nimg, N, residual=hs, ctx2d=ctx2d)
        n = ops.layernorm(hs, self.norm3.weight, self.norm3.bias, self.norm3.eps)
        return self.ff.run(n, nimg, residual=hs)


class Transformer2DModel(nn.Module):
    """GroupNorm -> proj_in -> transformer_blocks (1 for SD-1.x, up to 10 for SDXL) -> proj_out (+ input).
    proj_in/out are 1x1 convs (SD-1.x) or Linears (SDXL use_linear_projection): the same [C, C] GEMM on NHWC."""

    def __init__(self, norm, proj_in, blocks, proj_out):
        super().__init__()
        self.norm = norm
        self.proj_in = proj_in
        self.transformer_blocks = nn.ModuleList(blocks)
        self.proj_out = proj_out

    def run(self, x, nimg, HW, ctx2d, out):
        pi = self.proj_in
        if FUSED_GN and HW >= GN_FOLD_MIN_HW and HW % 256 == 0 and x.shape[1] % 64 == 0 and not pi._forward_hooks:
            # proj_in(GN(x)) = x . (W diag(scale_i))^T + (b + W shift_i) per image i: the normalised tensor (a full
            # read + write of the activation) is never materialised; below 32x32 the one-launch GroupNorm is cheaper
            scale, shift = self.norm.stats(x, nimg, HW)
            wf, cb = ops.gn_fold(pi.weight, pi.bias, scale, shift)
            hs = ops.linear_per_image(x, wf, cb, HW)
        else:
            hs = pi.run(self.norm.normalize(x, nimg, HW, False))
        for blk in self.transformer_blocks:
            hs = blk.run(hs, nimg, HW, ctx2d)
        return self.proj_out.run(hs, residual=x, out=out)


class ResnetBlock2D(nn.Module):
    def __init__(self, norm1, conv1, temb_proj, norm2, conv2, shortcut):
        super().__init__()
        self.norm1, self.conv1, self.time_emb_proj, self.norm2, self.conv2 = norm1, conv1, temb_proj, norm2, conv2
        self.conv_shortcut = shortcut
        self.temb_slice = None  # (offset, Cout) into the fused time-embedding projection output
        self._sc_key = None
        self._sc_w = None

    def _conv2_with_shortcut(self):
        """conv2's weight with conv_shortcut's columns appended and the two biases summed (fp32, rounded once)."""
        w2, b2, ws, bs = self.conv2.weight, self.conv2.bias, self.conv_shortcut.weight, self.conv_shortcut.bias
        key = tuple(None if t is None else (t.data_ptr(), t._version) for t in (w2, b2, ws, bs))
        if self._sc_key != key:
            b = sum(t.data.float() for t in (b2, bs) if t is not None)
            self._sc_w = (ops.conv_weight_with_shortcut(w2.data, ws.data),
                          None if isinstance(b, int) else b.half())
            self._sc_key = key
        return self._sc_w

    def run(self, x, nimg, H, W, temb_all, out):
        HW = H * W
        o, n = self.temb_slice
        # temb_all: [1, sum Cout] (SD-1.x, one timestep embedding for the batch) or [nimg, sum Cout] (SDXL:
        # per-image text_time conditioning) -> per-image column add in the conv epilogue
        bstride = temb_all.stride(0) if temb_all.shape[0] > 1 else 0
        cmid = self.conv1.weight.shape[0]
        # GroupNorm + SiLU inside the conv where the halo tiles take it (sdmoe_conv3x3_gn: statistics only, no
        # normalised copy of the activation written and re-read); elsewhere the one-call GroupNorm first
        if ops.conv_gn_fusable(H, W, x.shape[1], cmid):
            h = ops.conv3x3(x, nimg, H, W, self.conv1.weight, self.conv1.bias, coladd=temb_all[:, o:o + n],
                            coladd_bstride=bstride, gn=self.norm1.stats(x, nimg, HW) + (True,))
        else:
            xn = self.norm1.normalize(x, nimg, HW, True)
            h = ops.conv3x3(xn, nimg, H, W, self.conv1.weight, self.conv1.bias,
                            coladd=temb_all[:, o:o + n], coladd_bstride=bstride)
        gn2 = None
        hn = h
        if ops.conv_gn_fusable(H, W, cmid, self.conv2.weight.shape[0]):
            gn2 = self.norm2.stats(h, nimg, HW) + (True,)
        else:
            hn = self.norm2.normalize(h, nimg, HW, True)
        if self.conv_shortcut is not None and FUSED_SC and x.shape[1] % 64 == 0:
            # conv2(hn) + conv_shortcut(x) in one implicit GEMM: the shortcut is K-steps over x at the output pixel
            w, b = self._conv2_with_shortcut()
            return ops.conv3x3(hn, nimg, H, W, w, b, shortcut=x, out=out, gn=gn2)
        res = x if self.conv_shortcut is None else self.conv_shortcut.run(x)
        return ops.conv3x3(hn, nimg, H, W, self.conv2.weight, self.conv2.bias, residual=res, out=out, gn=gn2)


class Sampler(nn.Module):
    def __init__(self, conv):
        super().__init__()
        self.conv = conv


class Block(nn.Module):
    """Down/mid/up block container with diffusers' child names (resnets / attentions / down|upsamplers)."""

    def __init__(self, resnets, attentions=None, downsamplers=None, upsamplers=None):
        super().__init__()
        self.resnets = nn.ModuleList(resnets)
        if attentions:
            self.attentions = nn.ModuleList(attentions)
        else:
            self.attentions = None
        if downsamplers:
            self.downsamplers = nn.ModuleList(downsamplers)
        if upsamplers:
            self.upsamplers = nn.ModuleList(upsamplers)


class TimestepEmbedding(nn.Module):
    def __init__(self, l1, l2):
        super().__init__()
        self.linear_1, self.linear_2 = l1, l2


class UNet2DConditionModel(nn.Module):
    def __init__(self, cfg: UNetConfig):
        super().__init__()
        self.config = cfg

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_state_dict(cls, sd, cfg: UNetConfig, device="cuda"):
        """Build from a diffusers-layout state dict (fp32/fp16 CPU tensors), converting layouts once."""
        m = cls(cfg)
        dev = torch.device(device)

        def t(name):
            return sd[name].to(dev, torch.float16).contiguous()

        def lin(p, bias=True):
            return LoRACompatibleLinear(t(p + ".weight"), t(p + ".bias") if bias else None)

        def conv(p, stride=1):
            w = ops.conv_weight_from_torch(sd[p + ".weight"].to(dev, torch.float16))
            return Conv2d(w, t(p + ".bias"), stride)

        def conv1x1(p):
            w = sd[p + ".weight"]
            return LoRACompatibleLinear(w.reshape(w.shape[0], w.shape[1]).to(dev, torch.float16).contiguous(),
                                        t(p + ".bias"))

        def gn(p, eps):
            return Norm(t(p + ".weight"), t(p + ".bias"), eps, cfg.norm_num_groups)

        def ln(p):
            return Norm(t(p + ".weight"), t(p + ".bias"), cfg.layer_norm_eps)

        def resnet(p):
            sc = conv1x1(p + ".conv_shortcut") if (p + ".conv_shortcut.weight") in sd else None
            return ResnetBlock2D(gn(p + ".norm1", cfg.norm_eps), conv(p + ".conv1"), lin(p + ".time_emb_proj"),
                                 gn(p + ".norm2", cfg.norm_eps), conv(p + ".conv2"), sc)

        def block(b):
            heads = cfg.heads_for(sd[b + ".attn1.to_q.weight"].shape[0])
            a1 = Attention(t(b + ".attn1.to_q.weight"), t(b + ".attn1.to_k.weight"), t(b + ".attn1.to_v.weight"),
                           t(b + ".attn1.to_out.0.weight"), t(b + ".attn1.to_out.0.bias"), heads, True)
            a2 = Attention(t(b + ".attn2.to_q.weight"), t(b + ".attn2.to_k.weight"), t(b + ".attn2.to_v.weight"),
                           t(b + ".attn2.to_out.0.weight"), t(b + ".attn2.to_out.0.bias"), heads, False)
            ff = FeedForward(GEGLU(lin(b + ".ff.net.0.proj")), lin(b + ".ff.net.2"))
            return BasicTransformerBlock(ln(b + ".norm1"), a1, ln(b + ".norm2"), a2, ln(b + ".norm3"), ff)

        def transformer(p):
            blocks = []
            while f"{p}.transformer_blocks.{len(blocks)}.norm1.weight" in sd:
                blocks.append(block(f"{p}.transformer_blocks.{len(blocks)}"))
            return Transformer2DModel(gn(p + ".norm", cfg.transformer_norm_eps), conv1x1(p + ".proj_in"), blocks,
                                      conv1x1(p + ".proj_out"))

        w_in = sd["conv_in.weight"].to(dev, torch.float16)
        w_in = ops.conv_weight_from_torch(F.pad(w_in, (0, 0, 0, 0, 0, IN_PAD - w_in.shape[1])))
        m.conv_in = Conv2d(w_in, t("conv_in.bias"))
        m.time_embedding = TimestepEmbedding(lin("time_embedding.linear_1"), lin("time_embedding.linear_2"))
        if cfg.addition_embed_type == "text_time":
            a1 = lin("add_embedding.linear_1")
            k_real = a1.weight.shape[1]
            kp = (k_real + 63) // 64 * 64  # K padded to the GEMM's 64-wide K-step (zero columns)
            a1.weight = _buf(F.pad(a1.weight.data, (0, kp - k_real)).contiguous())
            m.add_embedding = TimestepEmbedding(a1, lin("add_embedding.linear_2"))
            m.add_in_features = k_real
        nblk = len(cfg.block_out_channels)
        L = cfg.layers_per_block
        downs = []
        for i, typ in enumerate(cfg.down_block_types):
            res = [resnet(f"down_blocks.{i}.resnets.{j}") for j in range(L)]
            att = [transformer(f"down_blocks.{i}.attentions.{j}") for j in range(L)] if typ.startswith("CrossAttn") \
                else None
            ds = [Sampler(conv(f"down_blocks.{i}.downsamplers.0.conv", 2))] if i < nblk - 1 else None
            downs.append(Block(res, att, downsamplers=ds))
        m.down_blocks = nn.ModuleList(downs)
        m.mid_block = Block([resnet("mid_block.resnets.0"), resnet("mid_block.resnets.1")],
                            [transformer("mid_block.attentions.0")])
        ups = []
        for i, typ in enumerate(cfg.up_block_types):
            res = [resnet(f"up_blocks.{i}.resnets.{j}") for j in range(L + 1)]
            att = [transformer(f"up_blocks.{i}.attentions.{j}") for j in range(L + 1)] \
                if typ.startswith("CrossAttn") else None
            us = [Sampler(conv(f"up_blocks.{i}.upsamplers.0.conv"))] if i < nblk - 1 else None
            ups.append(Block(res, att, upsamplers=us))
        m.up_blocks = nn.ModuleList(ups)
        m.conv_norm_out = gn("conv_norm_out", cfg.norm_eps)
        w_out = sd["conv_out.weight"].to(dev, torch.float16)
        w_out = ops.conv_weight_from_torch(F.pad(w_out, (0, 0, 0, 0, 0, 0, 0, OUT_PAD - w_out.shape[0])))
        b_out = F.pad(sd["conv_out.bias"].to(dev, torch.float16), (0, OUT_PAD - cfg.out_channels)).contiguous()
        m.conv_out = Conv2d(w_out, b_out)

        # fuse every ResNet's time_emb_proj into one [sum Cout, temb] GEMM; modules keep views
        resnets = [r for _, r in m.named_modules() if isinstance(r, ResnetBlock2D)]
        ws = torch.cat([r.time_emb_proj.weight.data for r in resnets], 0).contiguous()
        bs = torch.cat([r.time_emb_proj.bias.data for r in resnets], 0).contiguous()
        m.temb_w, m.temb_b = _buf(ws), _buf(bs)
        off = 0
        for r in resnets:
            n = r.time_emb_proj.weight.shape[0]
            r.time_emb_proj.weight = _buf(ws[off:off + n])
            r.time_emb_proj.bias = _buf(bs[off:off + n])
            r.temb_slice = (off, n)
            off += n
        return m

    # ------------------------------------------------------------------ forward
    def add_embed_hidden(self, text_embeds, time_ids):
        """SDXL text_time conditioning, step-invariant half: SiLU(add_embedding.linear_1([text_embeds ;
        sinusoid(time_ids)])) [nimg, temb] fp16 (UNet2DConditionModel.get_aug_embed). Computed once per
        pipeline call; the per-step half is in time_embed()."""
        cfg = self.config
        dev = self.conv_in.weight.device
        n = time_ids.shape[0]
        d = cfg.addition_time_embed_dim
        kp = self.add_embedding.linear_1.weight.shape[1]
        add = torch.zeros((n, kp), dtype=torch.float16, device=dev)
        add[:, :text_embeds.shape[1]] = text_embeds.to(dev, torch.float16)
        tid = time_ids.to(dev, torch.float32).reshape(-1).contiguous()
        p = text_embeds.shape[1]
        ops.timestep_embedding_rows(tid, d, add[:, p:p + 6 * d], group=6, flip_sin_to_cos=cfg.flip_sin_to_cos,
                                    freq_shift=cfg.freq_shift)
        return self.add_embedding.linear_1.run(add, act=ops.ACT_SILU)

    def time_embed(self, t, t_dev=None, add_hidden=None):
        cfg = self.config
        dev = self.conv_in.weight.device
        e = ops.timestep_embedding(t, cfg.block_out_channels[0], dev, cfg.flip_sin_to_cos, cfg.freq_shift, t_dev=t_dev)
        e = self.time_embedding.linear_1.run(e, act=ops.ACT_SILU)
        if cfg.addition_embed_type == "text_time":
            # emb = linear_2(...) + add_embedding(...); every consumer applies SiLU(emb) first:
            # SiLU(add_hidden @ W2a^T + b2a + e_t) with e_t broadcast to every image by the column-add epilogue
            e = self.time_embedding.linear_2.run(e)
            e = self.add_embedding.linear_2.run(add_hidden, act=ops.ACT_SILU, coladd=e, coladd_bstride=0,
                                                rows_per_batch=add_hidden.shape[0])
        else:
            e = self.time_embedding.linear_2.run(e, act=ops.ACT_SILU)  # every consumer applies SiLU(temb) first
        return ops.linear(e, self.temb_w, self.temb_b)

    def time_embed_table(self, ts):
        """SD-1.x: the projected time embeddings of a whole schedule at once — [len(ts), sum Cout] fp16, row s =
        time_embed(ts[s]) — as three M = len(ts) GEMMs instead of len(ts) GEMV chains (the 20160 x 1280 fused
        ResNet projection is read once per pipeline call, not once per step). None for SDXL (its per-step half
        depends on the per-image micro-conditioning)."""
        cfg = self.config
        if cfg.addition_embed_type == "text_time":
            return None
        dev = self.conv_in.weight.device
        t_dev = torch.tensor([float(t) for t in ts], dtype=torch.float32, device=dev)
        d = cfg.block_out_channels[0]
        e = torch.empty((len(ts), d), dtype=torch.float16, device=dev)
        ops.timestep_embedding_rows(t_dev, d, e, flip_sin_to_cos=cfg.flip_sin_to_cos, freq_shift=cfg.freq_shift)
        e = self.time_embedding.linear_1.run(e, act=ops.ACT_SILU)
        e = self.time_embedding.linear_2.run(e, act=ops.ACT_SILU)
        return ops.linear(e, self.temb_w, self.temb_b)

    def forward_nhwc(self, x_in, t, ctx2d, out=None, t_dev=None, add_hidden=None, temb=None):
        """One U-Net evaluation. x_in: [nimg*H*W, 64] fp16 (channels 0..3 = latent), ctx2d: [nimg*77, ctx dim].
        add_hidden (SDXL): add_embed_hidden(text_embeds, time_ids). Returns eps as [nimg*H*W, 8] fp16
        (channels 0..3 valid)."""
        cfg = self.config
        dev = x_in.device
        nimg = ctx2d.shape[0] // CTX_LEN
        H = W = cfg.sample_size
        ch = cfg.block_out_channels
        nblk = len(ch)
        L = cfg.layers_per_block
        # temb: this step's row of time_embed_table (precomputed for the pipeline call's schedule), else per step
        temb_all = temb if temb is not None else self.time_embed(t, t_dev, add_hidden)

        # ---- plan the up-path concat buffers [rows, C_prev + C_skip] (consumption order)
        rev = list(reversed(ch))
        sizes = [H >> i for i in range(nblk)]
        up_in = []
        prev = rev[0]
        for i in range(nblk):
            cout = rev[i]
            skip_in = rev[min(i + 1, nblk - 1)]
            hh = sizes[nblk - 1 - i]
            for j in range(L + 1):
                cp = prev if j == 0 else cout
                cs = skip_in if j == L else cout
                buf = torch.empty((nimg * hh * hh, cp + cs), dtype=torch.float16, device=dev)
                up_in.append((buf, cp, hh))
            prev = cout
        nskip = len(up_in)

        def skip_slot(k):  # k-th produced skip -> right-hand slice of its consumer's concat buffer
            buf, cp, _ = up_in[nskip - 1 - k]
            return buf[:, cp:]

        def new(rows, c):
            return torch.empty((rows, c), dtype=torch.float16, device=dev)

        # ---- down path
        k = 0
        h = ops.conv3x3(x_in, nimg, H, W, self.conv_in.weight, self.conv_in.bias, out=skip_slot(k))
        k += 1
        hh = H
        for i, blk in enumerate(self.down_blocks):
            rows = nimg * hh * hh
            for j in range(L):
                if blk.attentions is not None:
                    r = blk.resnets[j].run(h, nimg, hh, hh, temb_all, out=new(rows, ch[i]))
                    h = blk.attentions[j].run(r, nimg, hh * hh, ctx2d, out=skip_slot(k))
                else:
                    h = blk.resnets[j].run(h, nimg, hh, hh, temb_all, out=skip_slot(k))
                k += 1
            if hasattr(blk, "downsamplers"):
                c = blk.downsamplers[0].conv
                h = ops.conv3x3(h, nimg, hh, hh, c.weight, c.bias, stride=2, out=skip_slot(k))
                k += 1
                hh //= 2

        # ---- mid
        rows = nimg * hh * hh
        mb = self.mid_block
        r = mb.resnets[0].run(h, nimg, hh, hh, temb_all, out=new(rows, ch[-1]))
        a = mb.attentions[0].run(r, nimg, hh * hh, ctx2d, out=new(rows, ch[-1]))
        buf0, cp0, _ = up_in[0]
        mb.resnets[1].run(a, nimg, hh, hh, temb_all, out=buf0[:, :cp0])

        # ---- up path
        idx = 0
        final = None
        for i, blk in enumerate(self.up_blocks):
            cout = rev[i]
            for j in range(L + 1):
                inp, cp, hh = up_in[idx]
                rows = nimg * hh * hh
                last_in_block = j == L
                has_up = hasattr(blk, "upsamplers")
                if not last_in_block:
                    nb, ncp, _ = up_in[idx + 1]
                    dest = nb[:, :ncp]
                elif has_up or i == nblk - 1:
                    dest = new(rows, cout)
                if blk.attentions is not None:
                    r = blk.resnets[j].run(inp, nimg, hh, hh, temb_all, out=new(rows, cout))
                    o = blk.attentions[j].run(r, nimg, hh * hh, ctx2d, out=dest)
                else:
                    o = blk.resnets[j].run(inp, nimg, hh, hh, temb_all, out=dest)
                idx += 1
                if last_in_block:
                    if has_up:
                        nb, ncp, _ = up_in[idx]
                        c = blk.upsamplers[0].conv
                        ops.conv3x3(o, nimg, hh, hh, c.weight, c.bias, upsample=True, out=nb[:, :ncp])
                    else:
                        final = o

        # ---- out
        fn = self.conv_norm_out.normalize(final, nimg, H * W, True)
        if out is None:
            out = new(nimg * H * W, OUT_PAD)
        return ops.conv3x3(fn, nimg, H, W, self.conv_out.weight, self.conv_out.bias, out=out)

    def forward(self, sample, timestep, encoder_hidden_states, added_cond_kwargs=None):
        """diffusers-style call: sample [n, 4, H, W], encoder_hidden_states [n, 77, ctx]; returns eps [n,4,H,W].
        added_cond_kwargs (SDXL): {"text_embeds": [n, pooled], "time_ids": [n, 6]}, as diffusers."""
        n, c, H, W = sample.shape
        x = torch.zeros((n * H * W, IN_PAD), dtype=torch.float16, device=sample.device)
        x[:, :c] = sample.permute(0, 2, 3, 1).reshape(n * H * W, c).to(torch.float16)
        ctx = encoder_hidden_states.reshape(-1, encoder_hidden_states.shape[-1]).to(torch.float16).contiguous()
        add_hidden = None
        if self.config.addition_embed_type == "text_time":
            add_hidden = self.add_embed_hidden(added_cond_kwargs["text_embeds"], added_cond_kwargs["time_ids"])
        eps = self.forward_nhwc(x, float(timestep), ctx, add_hidden=add_hidden)
        return eps[:, :c].reshape(n, H, W, c).permute(0, 3, 1, 2).contiguous()
