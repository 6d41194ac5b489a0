"""ORACLE (test infrastructure only) — fp32 CPU restatement of the diffusers SD-1.x / SDXL UNet2DConditionModel
forward, DDIM scheduler and classifier-free-guidance loop that the reference's hooks run inside
(utils.py:64-84 builds it; base_receiver.py:73 runs it). diffusers is not vendored in the reference and is
absent here, so this U-Net body is PARITY-UNPINNED against diffusers itself: it restates diffusers 0.27's
published module semantics (ResnetBlock2D, Transformer2DModel/BasicTransformerBlock, Attention, GEGLU,
Downsample2D/Upsample2D, get_timestep_embedding, DDIMScheduler; for SDXL also use_linear_projection,
transformer_layers_per_block and the "text_time" add_embedding of UNet2DConditionModel.get_aug_embed — the
reference loads SDXL at utils.py:111-112) and is checked by unit identities in
tests/test_oracle_unet.py. The hook points reproduce where the reference's receivers attach:
  ff_hook(layer, x, proj_w, proj_b)  <- forward hook on every `ff.net.0` GEGLU (base_receiver.py:49-53)
  down_hook(layer, x, w, b)          <- forward hook on every `ff.net.2` Linear (remove_wanda_neurons_fast.py:107-112)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.nn.functional as F


def timestep_embedding(t, dim, flip_sin_to_cos=True, freq_shift=0.0, max_period=10000):
    """diffusers.models.embeddings.get_timestep_embedding."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32) / (half - freq_shift)
    emb = torch.tensor([float(t)], dtype=torch.float32)[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


# conv operands in channels_last (NHWC): the CPU (oneDNN) conv runs several times faster on NHWC operands than on NCHW
# ones at these widths; the layout changes only the fp32 summation order. SDMOE_ORACLE_NHWC=0: plain NCHW.
NHWC = os.environ.get("SDMOE_ORACLE_NHWC", "1") != "0"


class UNetRef:
    def __init__(self, sd, cfg):
        self.sd = {k: (v.float().contiguous(memory_format=torch.channels_last) if v.dim() == 4 and NHWC else v.float())
                   for k, v in sd.items()}
        self.cfg = cfg
        self.layer = 0

    # -- primitives
    def lin(self, x, name, bias=True):
        return F.linear(x, self.sd[name + ".weight"], self.sd.get(name + ".bias") if bias else None)

    def conv(self, x, name, stride=1, padding=1):
        if not NHWC:
            return F.conv2d(x, self.sd[name + ".weight"], self.sd[name + ".bias"], stride=stride, padding=padding)
        return F.conv2d(x.contiguous(memory_format=torch.channels_last), self.sd[name + ".weight"],
                        self.sd[name + ".bias"], stride=stride, padding=padding).contiguous()

    def gn(self, x, name, eps):
        return F.group_norm(x, self.cfg.norm_num_groups, self.sd[name + ".weight"], self.sd[name + ".bias"], eps)

    def ln(self, x, name):
        return F.layer_norm(x, (x.shape[-1],), self.sd[name + ".weight"], self.sd[name + ".bias"],
                            self.cfg.layer_norm_eps)

    # -- blocks
    def resnet(self, x, temb, p):
        h = F.silu(self.gn(x, p + ".norm1", self.cfg.norm_eps))
        h = self.conv(h, p + ".conv1")
        h = h + self.lin(F.silu(temb), p + ".time_emb_proj")[:, :, None, None]
        h = F.silu(self.gn(h, p + ".norm2", self.cfg.norm_eps))
        h = self.conv(h, p + ".conv2")
        sc = self.conv(x, p + ".conv_shortcut", padding=0) if (p + ".conv_shortcut.weight") in self.sd else x
        return sc + h

    def attention(self, x, ctx, p):
        heads = self.cfg.heads_for(x.shape[-1])
        q = self.lin(x, p + ".to_q", bias=False)
        src = x if ctx is None else ctx
        k = self.lin(src, p + ".to_k", bias=False)
        v = self.lin(src, p + ".to_v", bias=False)
        B, N, C = q.shape
        d = C // heads
        q = q.view(B, N, heads, d).transpose(1, 2)
        k = k.view(B, -1, heads, d).transpose(1, 2)
        v = v.view(B, -1, heads, d).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v)
        o = o.transpose(1, 2).reshape(B, N, C)
        return self.lin(o, p + ".to_out.0")

    def feedforward(self, x, p):
        layer = self.layer
        self.layer += 1
        w0, b0 = self.sd[p + ".net.0.proj.weight"], self.sd[p + ".net.0.proj.bias"]
        if self.ff_hook is not None:
            h = self.ff_hook(layer, x, w0, b0)
        else:
            hv, g = F.linear(x, w0, b0).chunk(2, dim=-1)
            h = hv * F.gelu(g)
        w2, b2 = self.sd[p + ".net.2.weight"], self.sd[p + ".net.2.bias"]
        if self.down_hook is not None:
            return self.down_hook(layer, h, w2, b2)
        return F.linear(h, w2, b2)

    def transformer(self, x, ctx, p):
        B, C, H, W = x.shape
        res = x
        h = self.gn(x, p + ".norm", self.cfg.transformer_norm_eps)
        if self.cfg.use_linear_projection:
            h = self.lin(h.permute(0, 2, 3, 1).reshape(B, H * W, C), p + ".proj_in")
        else:
            h = self.conv(h, p + ".proj_in", padding=0)
            h = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
        d = 0
        while (b := f"{p}.transformer_blocks.{d}") + ".norm1.weight" in self.sd:
            h = self.attention(self.ln(h, b + ".norm1"), None, b + ".attn1") + h
            h = self.attention(self.ln(h, b + ".norm2"), ctx, b + ".attn2") + h
            h = self.feedforward(self.ln(h, b + ".norm3"), b + ".ff") + h
            d += 1
        if self.cfg.use_linear_projection:
            h = self.lin(h, p + ".proj_out")
            return h.reshape(B, H, W, C).permute(0, 3, 1, 2) + res
        h = h.reshape(B, H, W, C).permute(0, 3, 1, 2)
        return self.conv(h, p + ".proj_out", padding=0) + res

    def aug_embed(self, text_embeds, time_ids):
        """UNet2DConditionModel.get_aug_embed, addition_embed_type "text_time": add_time_proj (Timesteps over
        each of the 6 time ids) flattened, concatenated after the pooled text embedding, add_embedding MLP."""
        cfg = self.cfg
        n = time_ids.shape[0]
        tp = torch.cat([timestep_embedding(float(v), cfg.addition_time_embed_dim, True, 0.0)
                        for v in time_ids.reshape(-1).tolist()]).reshape(n, -1)
        add = torch.cat([text_embeds.float(), tp], dim=-1)
        return self.lin(F.silu(self.lin(add, "add_embedding.linear_1")), "add_embedding.linear_2")

    def __call__(self, sample, t, ctx, ff_hook=None, down_hook=None, added_cond=None):
        """added_cond (SDXL): {"text_embeds": [n, pooled], "time_ids": [n, 6]}."""
        cfg = self.cfg
        self.ff_hook, self.down_hook, self.layer = ff_hook, down_hook, 0
        temb = timestep_embedding(t, cfg.block_out_channels[0], cfg.flip_sin_to_cos, cfg.freq_shift)
        temb = self.lin(F.silu(self.lin(temb, "time_embedding.linear_1")), "time_embedding.linear_2")
        if cfg.addition_embed_type == "text_time":
            temb = temb + self.aug_embed(added_cond["text_embeds"], added_cond["time_ids"])
        h = self.conv(sample, "conv_in")
        skips = [h]
        L = cfg.layers_per_block
        nblk = len(cfg.block_out_channels)
        for i, typ in enumerate(cfg.down_block_types):
            for j in range(L):
                h = self.resnet(h, temb, f"down_blocks.{i}.resnets.{j}")
                if typ.startswith("CrossAttn"):
                    h = self.transformer(h, ctx, f"down_blocks.{i}.attentions.{j}")
                skips.append(h)
            if i < nblk - 1:
                h = self.conv(h, f"down_blocks.{i}.downsamplers.0.conv", stride=2)
                skips.append(h)
        h = self.resnet(h, temb, "mid_block.resnets.0")
        h = self.transformer(h, ctx, "mid_block.attentions.0")
        h = self.resnet(h, temb, "mid_block.resnets.1")
        for i, typ in enumerate(cfg.up_block_types):
            for j in range(L + 1):
                h = torch.cat([h, skips.pop()], dim=1)
                h = self.resnet(h, temb, f"up_blocks.{i}.resnets.{j}")
                if typ.startswith("CrossAttn"):
                    h = self.transformer(h, ctx, f"up_blocks.{i}.attentions.{j}")
            if i < nblk - 1:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
                h = self.conv(h, f"up_blocks.{i}.upsamplers.0.conv")
        h = F.silu(self.gn(h, "conv_norm_out", cfg.norm_eps))
        return self.conv(h, "conv_out")


def ddim_schedule(num_inference_steps=50, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                  steps_offset=1, set_alpha_to_one=False):
    """DDIMScheduler(beta_schedule='scaled_linear', timestep_spacing='leading') as configured by SD-1.x."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
    alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
    final = torch.tensor(1.0) if set_alpha_to_one else alphas_cumprod[0]
    ratio = num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64) + steps_offset
    a_t = [float(alphas_cumprod[t]) for t in ts]
    a_prev = [float(alphas_cumprod[t - ratio]) if t - ratio >= 0 else float(final) for t in ts]
    return ts, a_t, a_prev


class PNDMRef:
    """diffusers PNDMScheduler with skip_prk_steps=True (SD-1.x's scheduler config: scaled_linear betas
    0.00085..0.012, steps_offset 1, set_alpha_to_one False, prediction_type epsilon): set_timesteps + step_plms +
    _get_prev_sample, restated on tensors (the reference pipelines' default scheduler, utils.py:64-84)."""

    def __init__(self, num_inference_steps=50, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                 steps_offset=1, set_alpha_to_one=False):
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        self.ac = torch.cumprod(1.0 - betas, dim=0).double()
        self.final = 1.0 if set_alpha_to_one else float(self.ac[0])
        self.n, self.T = num_inference_steps, num_train_timesteps
        ts = (np.arange(0, num_inference_steps) * (num_train_timesteps // num_inference_steps)).round()
        ts = ts + steps_offset
        self.timesteps = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1].copy().astype(np.int64)
        self.ets, self.counter, self.cur_sample = [], 0, None

    def prev_sample(self, sample, t, prev_t, mo):
        at = float(self.ac[t])
        ap = float(self.ac[prev_t]) if prev_t >= 0 else self.final
        bt, bp = 1 - at, 1 - ap
        denom = at * bp ** 0.5 + (at * bt * ap) ** 0.5
        return (ap / at) ** 0.5 * sample - (ap - at) * mo / denom

    def step(self, mo, timestep, sample):
        ratio = self.T // self.n
        prev_t = timestep - ratio
        if self.counter != 1:
            self.ets = self.ets[-3:]
            self.ets.append(mo)
        else:
            prev_t = timestep
            timestep = timestep + ratio
        if len(self.ets) == 1 and self.counter == 0:
            mo = mo
            self.cur_sample = sample
        elif len(self.ets) == 1 and self.counter == 1:
            mo = (mo + self.ets[-1]) / 2
            sample = self.cur_sample
            self.cur_sample = None
        elif len(self.ets) == 2:
            mo = (3 * self.ets[-1] - self.ets[-2]) / 2
        elif len(self.ets) == 3:
            mo = (23 * self.ets[-1] - 16 * self.ets[-2] + 5 * self.ets[-3]) / 12
        else:
            mo = (1 / 24) * (55 * self.ets[-1] - 59 * self.ets[-2] + 37 * self.ets[-3] - 9 * self.ets[-4])
        out = self.prev_sample(sample, int(timestep), int(prev_t), mo)
        self.counter += 1
        return out


def denoise(unet: UNetRef, latents, ctx_uncond, ctx_cond, num_inference_steps=50, guidance_scale=7.5,
            ff_hook_factory=None, down_hook_factory=None, steps=None, added_cond=None, scheduler="ddim"):
    """StableDiffusionPipeline.__call__'s loop with DDIM + CFG (uncond first). Hook factories take the step
    index and return the (layer, ...) hook for that U-Net call — the reference's (t, l) counter.
    added_cond (SDXL): {"text_embeds": [2B, pooled], "time_ids": [2B, 6]} rows in the [uncond; cond] order."""
    x = latents.float().clone()
    B = x.shape[0]
    ctx = torch.cat([ctx_uncond, ctx_cond]).float()
    if scheduler == "pndm":
        sch = PNDMRef(num_inference_steps)
        nsteps = len(sch.timesteps) if steps is None else steps
        for s in range(nsteps):
            t = int(sch.timesteps[s])
            ffh = ff_hook_factory(s) if ff_hook_factory else None
            dh = down_hook_factory(s) if down_hook_factory else None
            eps = unet(torch.cat([x, x]), float(t), ctx, ff_hook=ffh, down_hook=dh, added_cond=added_cond)
            eu, ec = eps[:B], eps[B:]
            x = sch.step(eu + guidance_scale * (ec - eu), t, x).float()
        return x
    ts, a_t, a_prev = ddim_schedule(num_inference_steps)
    nsteps = len(ts) if steps is None else steps
    for s in range(nsteps):
        inp = torch.cat([x, x])
        ffh = ff_hook_factory(s) if ff_hook_factory else None
        dh = down_hook_factory(s) if down_hook_factory else None
        eps = unet(inp, float(ts[s]), ctx, ff_hook=ffh, down_hook=dh, added_cond=added_cond)
        eu, ec = eps[:B], eps[B:]
        e = eu + guidance_scale * (ec - eu)
        x0 = (x - math.sqrt(1 - a_t[s]) * e) / math.sqrt(a_t[s])
        x = math.sqrt(a_prev[s]) * x0 + math.sqrt(1 - a_prev[s]) * e
    return x
