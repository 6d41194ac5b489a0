"""Synthetic, seeded SD U-Net weights in the diffusers state-dict layout (no checkpoints exist offline).

Every tensor is drawn from its own CPU torch.Generator seeded by (seed, crc32(name)), so any subset can be
regenerated independently and identically on any host. Scales are chosen so 50 fp16 DDIM steps stay tame:
unit-variance-preserving fan-in init for convs/linears, small biases, GN/LN affine near identity, and a
damped cross-attention output (so the CFG difference eps_c - eps_u is small, as in a trained model).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import torch

from .config import UNetConfig


def _resnet(prefix, cin, cout, temb):
    p = [(f"{prefix}.norm1.weight", (cin,), "gn_w"), (f"{prefix}.norm1.bias", (cin,), "gn_b"),
         (f"{prefix}.conv1.weight", (cout, cin, 3, 3), "conv"), (f"{prefix}.conv1.bias", (cout,), "bias"),
         (f"{prefix}.time_emb_proj.weight", (cout, temb), "linear"), (f"{prefix}.time_emb_proj.bias", (cout,), "bias"),
         (f"{prefix}.norm2.weight", (cout,), "gn_w"), (f"{prefix}.norm2.bias", (cout,), "gn_b"),
         (f"{prefix}.conv2.weight", (cout, cout, 3, 3), "conv_res"), (f"{prefix}.conv2.bias", (cout,), "bias")]
    if cin != cout:
        p += [(f"{prefix}.conv_shortcut.weight", (cout, cin, 1, 1), "conv"),
              (f"{prefix}.conv_shortcut.bias", (cout,), "bias")]
    return p


def _block(b, C, ctx):
    """BasicTransformerBlock `b` (self-attn, cross-attn, GEGLU FFN)."""
    return [
        (f"{b}.norm1.weight", (C,), "gn_w"), (f"{b}.norm1.bias", (C,), "gn_b"),
        (f"{b}.attn1.to_q.weight", (C, C), "linear"), (f"{b}.attn1.to_k.weight", (C, C), "linear"),
        (f"{b}.attn1.to_v.weight", (C, C), "linear"),
        (f"{b}.attn1.to_out.0.weight", (C, C), "linear_res"), (f"{b}.attn1.to_out.0.bias", (C,), "bias"),
        (f"{b}.norm2.weight", (C,), "gn_w"), (f"{b}.norm2.bias", (C,), "gn_b"),
        (f"{b}.attn2.to_q.weight", (C, C), "linear"), (f"{b}.attn2.to_k.weight", (C, ctx), "linear"),
        (f"{b}.attn2.to_v.weight", (C, ctx), "linear"),
        (f"{b}.attn2.to_out.0.weight", (C, C), "linear_xattn"), (f"{b}.attn2.to_out.0.bias", (C,), "bias"),
        (f"{b}.norm3.weight", (C,), "gn_w"), (f"{b}.norm3.bias", (C,), "gn_b"),
        (f"{b}.ff.net.0.proj.weight", (8 * C, C), "linear"), (f"{b}.ff.net.0.proj.bias", (8 * C,), "bias"),
        (f"{b}.ff.net.2.weight", (C, 4 * C), "linear_res"), (f"{b}.ff.net.2.bias", (C,), "bias"),
    ]


def _transformer(prefix, C, ctx, depth=1, linear_proj=False):
    """Transformer2DModel: GroupNorm, proj_in (1x1 conv, or Linear for use_linear_projection), `depth`
    BasicTransformerBlocks, proj_out."""
    pshape = (C, C) if linear_proj else (C, C, 1, 1)
    p = [(f"{prefix}.norm.weight", (C,), "gn_w"), (f"{prefix}.norm.bias", (C,), "gn_b"),
         (f"{prefix}.proj_in.weight", pshape, "conv"), (f"{prefix}.proj_in.bias", (C,), "bias")]
    for d in range(depth):
        p += _block(f"{prefix}.transformer_blocks.{d}", C, ctx)
    p += [(f"{prefix}.proj_out.weight", pshape, "conv_res"), (f"{prefix}.proj_out.bias", (C,), "bias")]
    return p


def param_specs(cfg: UNetConfig):
    """[(name, shape, kind)] of UNet2DConditionModel (diffusers naming), in construction order."""
    ch = cfg.block_out_channels
    temb = cfg.time_embed_dim
    ctx = cfg.cross_attention_dim
    L = cfg.layers_per_block
    specs = [("conv_in.weight", (ch[0], cfg.in_channels, 3, 3), "conv"), ("conv_in.bias", (ch[0],), "bias"),
             ("time_embedding.linear_1.weight", (temb, ch[0]), "linear"),
             ("time_embedding.linear_1.bias", (temb,), "bias"),
             ("time_embedding.linear_2.weight", (temb, temb), "linear"),
             ("time_embedding.linear_2.bias", (temb,), "bias")]
    if cfg.addition_embed_type == "text_time":
        specs += [("add_embedding.linear_1.weight", (temb, cfg.projection_class_embeddings_input_dim), "linear"),
                  ("add_embedding.linear_1.bias", (temb,), "bias"),
                  ("add_embedding.linear_2.weight", (temb, temb), "linear"),
                  ("add_embedding.linear_2.bias", (temb,), "bias")]
    lp = cfg.use_linear_projection
    cout = ch[0]
    for i, t in enumerate(cfg.down_block_types):
        cin, cout = cout, ch[i]
        for j in range(L):
            specs += _resnet(f"down_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout, temb)
            if t.startswith("CrossAttn"):
                specs += _transformer(f"down_blocks.{i}.attentions.{j}", cout, ctx, cfg.depth_of("down", i), lp)
        if i < len(ch) - 1:
            specs += [(f"down_blocks.{i}.downsamplers.0.conv.weight", (cout, cout, 3, 3), "conv"),
                      (f"down_blocks.{i}.downsamplers.0.conv.bias", (cout,), "bias")]
    C = ch[-1]
    specs += _resnet("mid_block.resnets.0", C, C, temb)
    specs += _transformer("mid_block.attentions.0", C, ctx, cfg.depth_of("mid", 0), lp)
    specs += _resnet("mid_block.resnets.1", C, C, temb)
    rev = list(reversed(ch))
    prev = rev[0]
    for i, t in enumerate(cfg.up_block_types):
        cout = rev[i]
        skip_in = rev[min(i + 1, len(ch) - 1)]
        for j in range(L + 1):
            res_skip = skip_in if j == L else cout
            res_in = prev if j == 0 else cout
            specs += _resnet(f"up_blocks.{i}.resnets.{j}", res_in + res_skip, cout, temb)
            if t.startswith("CrossAttn"):
                specs += _transformer(f"up_blocks.{i}.attentions.{j}", cout, ctx, cfg.depth_of("up", i), lp)
        if i < len(ch) - 1:
            specs += [(f"up_blocks.{i}.upsamplers.0.conv.weight", (cout, cout, 3, 3), "conv"),
                      (f"up_blocks.{i}.upsamplers.0.conv.bias", (cout,), "bias")]
        prev = cout
    specs += [("conv_norm_out.weight", (ch[0],), "gn_w"), ("conv_norm_out.bias", (ch[0],), "gn_b"),
              ("conv_out.weight", (cfg.out_channels, ch[0], 3, 3), "conv"), ("conv_out.bias", (cfg.out_channels,),
                                                                             "bias")]
    return specs


def _init(name, shape, kind, seed):
    g = torch.Generator().manual_seed((seed * 1000003 + zlib.crc32(name.encode())) & 0x7FFFFFFFFFFF)
    if kind == "gn_w":
        return 1.0 + 0.05 * torch.randn(shape, generator=g)
    if kind == "gn_b":
        return 0.05 * torch.randn(shape, generator=g)
    if kind == "bias":
        return 0.02 * torch.randn(shape, generator=g)
    fan_in = 1
    for s in shape[1:]:
        fan_in *= s
    std = fan_in ** -0.5
    if kind in ("conv_res", "linear_res"):
        std *= 0.5        # residual-branch outputs: keep the residual stream growth modest over 25 blocks
    elif kind == "linear_xattn":
        std *= 0.1        # cross-attention output: small cond/uncond gap, like a trained SD U-Net
    return std * torch.randn(shape, generator=g)


def make_state_dict(cfg: UNetConfig, seed: int = 0, names=None):
    """OrderedDict name -> fp32 CPU tensor (diffusers layout), optionally only for `names`."""
    sd = OrderedDict()
    for name, shape, kind in param_specs(cfg):
        if names is None or name in names:
            sd[name] = _init(name, shape, kind, seed)
    return sd
