"""CPU fp32 restatement of diffusers' AutoencoderKL.decode for SD-1.x (post_quant_conv + Decoder), the oracle of
sdmoe.vae. TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.

diffusers is not vendored or pinned by the reference and is absent here, so this restatement is
parity-unpinned against diffusers itself; it follows the 0.27-era modules the reference's pipelines load
(utils.py:64-84 -> StableDiffusionPipeline.__call__ -> vae.decode): Decoder(conv_in, UNetMidBlock2D(resnet,
Attention(heads=1, dim_head=C, GroupNorm, residual), resnet), UpDecoderBlock2D x4 (nearest 2x + conv
upsamplers), conv_norm_out, SiLU, conv_out); ResnetBlock2D without time embedding, GroupNorm eps 1e-6.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _gn(x, sd, p, groups=32, eps=1e-6):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def _conv(x, sd, p, padding=1):
    return F.conv2d(x, sd[p + ".weight"], sd[p + ".bias"], padding=padding)


def _resnet(x, sd, p):
    h = _conv(F.silu(_gn(x, sd, p + ".norm1")), sd, p + ".conv1")
    h = _conv(F.silu(_gn(h, sd, p + ".norm2")), sd, p + ".conv2")
    if p + ".conv_shortcut.weight" in sd:
        x = _conv(x, sd, p + ".conv_shortcut", padding=0)
    return x + h


def _attention(x, sd, p):
    B, C, H, W = x.shape
    r = x
    t = _gn(x, sd, p + ".group_norm").reshape(B, C, H * W).transpose(1, 2)
    q = F.linear(t, sd[p + ".to_q.weight"], sd[p + ".to_q.bias"])
    k = F.linear(t, sd[p + ".to_k.weight"], sd[p + ".to_k.bias"])
    v = F.linear(t, sd[p + ".to_v.weight"], sd[p + ".to_v.bias"])
    a = torch.softmax(q @ k.transpose(1, 2) / C ** 0.5, dim=-1) @ v
    o = F.linear(a, sd[p + ".to_out.0.weight"], sd[p + ".to_out.0.bias"])
    return o.transpose(1, 2).reshape(B, C, H, W) + r


def decode(sd, cfg, latents):
    """latents fp32 [B, 4, h, w] -> decoder sample fp32 [B, 3, 8h, 8w] (vae.decode(latents / scaling_factor))."""
    z = _conv(latents / cfg.scaling_factor, sd, "post_quant_conv", padding=0)
    h = _conv(z, sd, "decoder.conv_in")
    h = _resnet(h, sd, "decoder.mid_block.resnets.0")
    h = _attention(h, sd, "decoder.mid_block.attentions.0")
    h = _resnet(h, sd, "decoder.mid_block.resnets.1")
    n = len(cfg.block_out_channels)
    for i in range(n):
        for j in range(cfg.layers_per_block + 1):
            h = _resnet(h, sd, f"decoder.up_blocks.{i}.resnets.{j}")
        if i < n - 1:
            h = _conv(F.interpolate(h, scale_factor=2.0, mode="nearest"), sd, f"decoder.up_blocks.{i}.upsamplers.0.conv")
    h = F.silu(_gn(h, sd, "decoder.conv_norm_out"))
    return _conv(h, sd, "decoder.conv_out")
