"""AutoencoderKL decoder (SD-1.x VAE) on the sdmoe HIP kernels — SURVEY §8f rank 4, the step after the denoising
loop: `StableDiffusionPipeline.__call__` ends with `vae.decode(latents / scaling_factor)` (diffusers, external;
the reference reaches it through `model(prompt).images`, base_receiver.py:73).

Structure (diffusers Decoder, SD-1.x config): post_quant_conv (1x1, 4->4) -> conv_in (3x3, 4->512) -> mid block
(ResNet, one 512-wide self-attention head over the latent grid, ResNet) -> 4 up blocks of 3 ResNets (512, 512,
256, 128 channels; nearest-2x + 3x3 conv upsamplers after the first three) -> GroupNorm + SiLU -> conv_out
(128->3). ResNets: GN(32, eps 1e-6) + SiLU + conv3x3, twice, plus the (1x1) shortcut.

MI355X layout as the U-Net: NHWC fp16 [images*H*W, C]; GN statistics + a fused apply(+SiLU) pass feed the
LDS-DMA implicit-GEMM convs; the residual add is the conv epilogue. The mid-block attention runs as MFMA GEMMs
(S = Q K^T, O = P V) around sdmoe_softmax_rows / sdmoe_transpose (head width 512 is beyond the flash kernel's
register tiles); 1/sqrt(512) is folded into W_q, b_q and 1/scaling_factor into post_quant_conv.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import ops
from .unet import IN_PAD, OUT_PAD


@dataclass
class VAEConfig:
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    latent_channels: int = 4
    out_channels: int = 3
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    scaling_factor: float = 0.18215

    @staticmethod
    def sd14():
        return VAEConfig()

    @staticmethod
    def tiny():
        return VAEConfig(block_out_channels=(64, 64), layers_per_block=1)


def _resnet_specs(p, cin, cout):
    s = [(f"{p}.norm1.weight", (cin,), "gn_w"), (f"{p}.norm1.bias", (cin,), "gn_b"),
         (f"{p}.conv1.weight", (cout, cin, 3, 3), "conv"), (f"{p}.conv1.bias", (cout,), "bias"),
         (f"{p}.norm2.weight", (cout,), "gn_w"), (f"{p}.norm2.bias", (cout,), "gn_b"),
         (f"{p}.conv2.weight", (cout, cout, 3, 3), "conv_res"), (f"{p}.conv2.bias", (cout,), "bias")]
    if cin != cout:
        s += [(f"{p}.conv_shortcut.weight", (cout, cin, 1, 1), "conv"), (f"{p}.conv_shortcut.bias", (cout,), "bias")]
    return s


def vae_param_specs(cfg: VAEConfig):
    """[(name, shape, kind)] of AutoencoderKL's post_quant_conv + decoder (diffusers naming)."""
    ch = cfg.block_out_channels
    top = ch[-1]
    L = cfg.latent_channels
    s = [("post_quant_conv.weight", (L, L, 1, 1), "conv"), ("post_quant_conv.bias", (L,), "bias"),
         ("decoder.conv_in.weight", (top, L, 3, 3), "conv"), ("decoder.conv_in.bias", (top,), "bias")]
    s += _resnet_specs("decoder.mid_block.resnets.0", top, top)
    a = "decoder.mid_block.attentions.0"
    s += [(f"{a}.group_norm.weight", (top,), "gn_w"), (f"{a}.group_norm.bias", (top,), "gn_b")]
    for n in ("to_q", "to_k", "to_v"):
        s += [(f"{a}.{n}.weight", (top, top), "linear"), (f"{a}.{n}.bias", (top,), "bias")]
    s += [(f"{a}.to_out.0.weight", (top, top), "linear_res"), (f"{a}.to_out.0.bias", (top,), "bias")]
    s += _resnet_specs("decoder.mid_block.resnets.1", top, top)
    rev = list(reversed(ch))
    prev = rev[0]
    for i, cout in enumerate(rev):
        for j in range(cfg.layers_per_block + 1):
            s += _resnet_specs(f"decoder.up_blocks.{i}.resnets.{j}", prev if j == 0 else cout, cout)
        if i < len(rev) - 1:
            s += [(f"decoder.up_blocks.{i}.upsamplers.0.conv.weight", (cout, cout, 3, 3), "conv"),
                  (f"decoder.up_blocks.{i}.upsamplers.0.conv.bias", (cout,), "bias")]
        prev = cout
    s += [("decoder.conv_norm_out.weight", (ch[0],), "gn_w"), ("decoder.conv_norm_out.bias", (ch[0],), "gn_b"),
          ("decoder.conv_out.weight", (cfg.out_channels, ch[0], 3, 3), "conv"),
          ("decoder.conv_out.bias", (cfg.out_channels,), "bias")]
    return s


def make_vae_state_dict(cfg: VAEConfig, seed: int = 0):
    """Seeded synthetic decoder weights (no checkpoint offline), same init recipe as sdmoe.weights."""
    from .weights import _init
    sd = OrderedDict()
    for name, shape, kind in vae_param_specs(cfg):
        sd[name] = _init("vae." + name, shape, kind, seed)
    return sd


class AutoencoderKLDecoder:
    """post_quant_conv + Decoder of diffusers' AutoencoderKL, weights converted once to the kernels' layouts."""

    def __init__(self, sd, cfg: VAEConfig, device="cuda"):
        self.config = cfg
        dev = torch.device(device)
        self.device = dev
        h = lambda n: sd[n].to(dev, torch.float16).contiguous()  # noqa: E731

        def conv(n, cin_pad=None, cout_pad=None):
            w = sd[n + ".weight"].to(dev, torch.float32)
            b = sd[n + ".bias"].to(dev, torch.float32)
            if cin_pad:
                w = F.pad(w, (0, 0, 0, 0, 0, cin_pad - w.shape[1]))
            if cout_pad:
                w = F.pad(w, (0, 0, 0, 0, 0, 0, 0, cout_pad - w.shape[0]))
                b = F.pad(b, (0, cout_pad - b.shape[0]))
            return ops.conv_weight_from_torch(w.half()), b.half().contiguous()

        def resnet(p):
            r = {"n1": (h(p + ".norm1.weight"), h(p + ".norm1.bias")), "c1": conv(p + ".conv1"),
                 "n2": (h(p + ".norm2.weight"), h(p + ".norm2.bias")), "c2": conv(p + ".conv2"), "sc": None}
            if p + ".conv_shortcut.weight" in sd:
                w = sd[p + ".conv_shortcut.weight"]
                r["sc"] = (w.reshape(w.shape[0], w.shape[1]).to(dev, torch.float16).contiguous(),
                           h(p + ".conv_shortcut.bias"))
            return r

        L = cfg.latent_channels
        wq = sd["post_quant_conv.weight"].reshape(L, L).to(dev, torch.float32) / cfg.scaling_factor
        self.pq_w = F.pad(wq, (0, IN_PAD - L, 0, IN_PAD - L)).half().contiguous()
        self.pq_b = F.pad(sd["post_quant_conv.bias"].to(dev, torch.float32), (0, IN_PAD - L)).half().contiguous()
        self.conv_in = conv("decoder.conv_in", cin_pad=IN_PAD)
        self.mid0 = resnet("decoder.mid_block.resnets.0")
        self.mid1 = resnet("decoder.mid_block.resnets.1")
        a = "decoder.mid_block.attentions.0"
        C = cfg.block_out_channels[-1]
        sc = C ** -0.5
        self.attn_norm = (h(a + ".group_norm.weight"), h(a + ".group_norm.bias"))
        self.wq = (sd[a + ".to_q.weight"] * sc).to(dev, torch.float16).contiguous()
        self.bq = (sd[a + ".to_q.bias"] * sc).to(dev, torch.float16).contiguous()
        self.wk, self.bk = h(a + ".to_k.weight"), h(a + ".to_k.bias")
        self.wv, self.bv = h(a + ".to_v.weight"), h(a + ".to_v.bias")
        self.wo, self.bo = h(a + ".to_out.0.weight"), h(a + ".to_out.0.bias")
        rev = list(reversed(cfg.block_out_channels))
        self.up = []
        for i in range(len(rev)):
            res = [resnet(f"decoder.up_blocks.{i}.resnets.{j}") for j in range(cfg.layers_per_block + 1)]
            ups = conv(f"decoder.up_blocks.{i}.upsamplers.0.conv") if i < len(rev) - 1 else None
            self.up.append((res, ups))
        self.norm_out = (h("decoder.conv_norm_out.weight"), h("decoder.conv_norm_out.bias"))
        self.conv_out = conv("decoder.conv_out", cout_pad=OUT_PAD)

    # ------------------------------------------------------------------ forward
    def _stats(self, x, nimg, HW, norm):
        return ops.groupnorm_stats(x, nimg, HW, norm[0], norm[1], self.config.norm_eps, self.config.norm_num_groups)

    def _resnet(self, x, nimg, H, W, r):
        sc1, sh1 = self._stats(x, nimg, H * W, r["n1"])
        hdn = ops.conv3x3(x, nimg, H, W, r["c1"][0], r["c1"][1], gn=(sc1, sh1, True))
        sc2, sh2 = self._stats(hdn, nimg, H * W, r["n2"])
        res = x if r["sc"] is None else ops.linear(x, r["sc"][0], r["sc"][1])
        return ops.conv3x3(hdn, nimg, H, W, r["c2"][0], r["c2"][1], gn=(sc2, sh2, True), residual=res)

    def _attention(self, x, nimg, HW):
        sc, sh = self._stats(x, nimg, HW, self.attn_norm)
        xn = ops.groupnorm_apply(x, nimg, HW, sc, sh, False)
        q = ops.linear(xn, self.wq, self.bq)  # already scaled by 1/sqrt(C)
        k = ops.linear(xn, self.wk, self.bk)
        v = ops.linear(xn, self.wv, self.bv)
        o = torch.empty_like(q)
        s = torch.empty((HW, HW), dtype=torch.float16, device=x.device)
        for i in range(nimg):
            rows = slice(i * HW, (i + 1) * HW)
            ops.linear(q[rows], k[rows], out=s)          # S = Q K^T / sqrt(C)
            ops.softmax_rows(s, out=s)
            ops.linear(s, ops.transpose(v[rows]), out=o[rows])  # O = P V
        return ops.linear(o, self.wo, self.bo, residual=x)

    def decode_nhwc(self, lat):
        """lat: fp32 [B, 4, h, w] (denoised latents, before 1/scaling_factor). Returns the decoder sample as NHWC
        fp16 [B*8h*8w, 8] (channels 0..2 valid, in [-1, 1] for a trained VAE)."""
        B, _, h0, w0 = lat.shape
        x = torch.zeros((B * h0 * w0, IN_PAD), dtype=torch.float16, device=self.device)
        ops.prepare_input(lat.to(self.device, torch.float32).contiguous(), x, 1)
        z = ops.linear(x, self.pq_w, self.pq_b)          # post_quant_conv (1x1) with 1/scaling_factor folded in
        H, W = h0, w0
        hdn = ops.conv3x3(z, B, H, W, self.conv_in[0], self.conv_in[1])
        hdn = self._resnet(hdn, B, H, W, self.mid0)
        hdn = self._attention(hdn, B, H * W)
        hdn = self._resnet(hdn, B, H, W, self.mid1)
        for res, ups in self.up:
            for r in res:
                hdn = self._resnet(hdn, B, H, W, r)
            if ups is not None:
                hdn = ops.conv3x3(hdn, B, H, W, ups[0], ups[1], upsample=True)
                H, W = 2 * H, 2 * W
        sc, sh = self._stats(hdn, B, H * W, self.norm_out)
        return ops.conv3x3(hdn, B, H, W, self.conv_out[0], self.conv_out[1], gn=(sc, sh, True)), H, W

    def decode(self, lat):
        """diffusers `vae.decode(lat / scaling_factor).sample`: fp32 NCHW [B, 3, 8h, 8w]."""
        y, H, W = self.decode_nhwc(lat)
        B = lat.shape[0]
        c = self.config.out_channels
        return y[:, :c].float().reshape(B, H, W, c).permute(0, 3, 1, 2).contiguous()


def postprocess(sample):
    """diffusers VaeImageProcessor.postprocess(output_type='pt'/'np' denormalisation): (x / 2 + 0.5).clamp(0, 1)."""
    return (sample / 2 + 0.5).clamp(0, 1)
