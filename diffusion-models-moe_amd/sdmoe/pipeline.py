"""StableDiffusionPipeline stand-in: synthetic text conditioning + DDIM + classifier-free guidance, with the
denoising loop entirely on the GPU (U-Net on the sdmoe kernels, CFG + DDIM update in one HIP kernel).

Call shape kept from diffusers / the reference's callers: `pipe(prompt_or_list, safety_checker=...)` returns
an object with `.images` (base_receiver.py:73, remove_wanda_neurons_fast.py:127-130, eval_coco.py:266-272).
Without `text_encoder` / `vae` attached (the metric's workload) prompts map to seeded synthetic
[77, 768] embeddings and `.images` holds the final latents ([4, H, W] fp32 per prompt); with them attached
(sdmoe.clip, sdmoe.vae) prompts are encoded by the HIP CLIP encoder and `output_type` "pt" / "np" decodes to RGB.
Loop invariants are hoisted per call: the cross-attention K/V of the context (unet.Attention.cross_kv) and the
projected time embeddings of every step of the schedule (UNet2DConditionModel.time_embed_table).
"""
from __future__ import annotations

import os
import zlib
from dataclasses import dataclass

import numpy as np
import torch

from . import ops
from .config import UNetConfig
from .unet import CTX_LEN, IN_PAD, OUT_PAD, UNet2DConditionModel
from .weights import make_state_dict

# all steps' time embeddings in one batched pass per call (0: per step, the A/B reference)
PRECOMPUTE_TEMB = os.environ.get("SDMOE_TEMB_TABLE", "1") != "0"


def ddim_schedule(num_inference_steps=50, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                  steps_offset=1, set_alpha_to_one=False):
    """DDIMScheduler as SD-1.x configures it (scaled_linear betas, 'leading' spacing, steps_offset=1):
    returns (timesteps, alpha_cumprod[t], alpha_cumprod[prev t]) as host lists (scheduler constants)."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
    ac = torch.cumprod(1.0 - betas, dim=0)
    final = 1.0 if set_alpha_to_one else float(ac[0])
    ratio = num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].astype(np.int64) + steps_offset
    a_t = [float(ac[t]) for t in ts]
    a_prev = [float(ac[t - ratio]) if t - ratio >= 0 else final for t in ts]
    return [int(t) for t in ts], a_t, a_prev


def pndm_schedule(num_inference_steps=50, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                  steps_offset=1, set_alpha_to_one=False):
    """PNDMScheduler(skip_prk_steps=True) as SD-1.x configures it — the reference pipelines' default scheduler
    (51 U-Net calls for 50 steps, hence the reference's T = 51). Returns, per U-Net call, (timestep, coef[7],
    flags[3]) for sdmoe_cfg_multistep_step: the PLMS combination of step_plms (diffusers
    schedulers/scheduling_pndm.py) over a 4-slot eps history ring and _get_prev_sample's a, b."""
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
    ac = torch.cumprod(1.0 - betas, dim=0).double().numpy()
    final = 1.0 if set_alpha_to_one else float(ac[0])
    ratio = num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round() + steps_offset
    plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1].astype(np.int64)
    plan, ets, counter = [], [], 0
    for t_call in plms:
        timestep, prev_t = int(t_call), int(t_call) - ratio
        c_hist = [0.0, 0.0, 0.0, 0.0]
        store, use_cur, save_cur = -1, 0, 0
        if counter != 1:
            ets = ets[-3:]
            store = next(s for s in range(4) if s not in ets)
            new_ets = ets + [store]
        else:
            prev_t, timestep = timestep, timestep + ratio
            new_ets = ets
        n = len(new_ets)
        if n == 1 and counter == 0:
            c_new, save_cur = 1.0, 1
        elif n == 1 and counter == 1:
            c_new, use_cur = 0.5, 1
            c_hist[new_ets[-1]] = 0.5
        elif n == 2:
            c_new = 1.5
            c_hist[new_ets[-2]] = -0.5
        elif n == 3:
            c_new = 23.0 / 12
            c_hist[new_ets[-2]], c_hist[new_ets[-3]] = -16.0 / 12, 5.0 / 12
        else:
            c_new = 55.0 / 24
            c_hist[new_ets[-2]], c_hist[new_ets[-3]], c_hist[new_ets[-4]] = -59.0 / 24, 37.0 / 24, -9.0 / 24
        at = float(ac[timestep])
        ap = float(ac[prev_t]) if prev_t >= 0 else final
        a = (ap / at) ** 0.5
        denom = at * (1 - ap) ** 0.5 + (at * (1 - at) * ap) ** 0.5
        plan.append((int(t_call), [c_new] + c_hist + [a, (ap - at) / denom], [store, use_cur, save_cur]))
        ets = new_ets
        counter += 1
    return plan


def prompt_embedding(prompt: str, dim: int = 768) -> torch.Tensor:
    """Seeded synthetic text conditioning [77, dim] fp32 (CPU) standing in for the CLIP text encoder."""
    rng = np.random.default_rng(zlib.crc32(prompt.encode("utf-8")))
    return torch.from_numpy((rng.standard_normal((CTX_LEN, dim)) * 0.5).astype(np.float32))


def pooled_embedding(prompt: str, dim: int = 1280) -> torch.Tensor:
    """Seeded synthetic pooled text embedding [dim] (SDXL text_embeds; CLIP-G pooled output stand-in)."""
    rng = np.random.default_rng(zlib.crc32(("pooled:" + prompt).encode("utf-8")))
    return torch.from_numpy((rng.standard_normal(dim) * 0.5).astype(np.float32))


def sdxl_time_ids(height: int, width: int) -> list:
    """SDXL micro-conditioning (original_size, crops_coords_top_left, target_size) for an uncropped image."""
    return [float(height), float(width), 0.0, 0.0, float(height), float(width)]


def initial_latents(seed: int, index: int, cfg: UNetConfig) -> torch.Tensor:
    """Per-prompt latents from a CPU generator seeded by (seed, global prompt index): identical for any
    world size / sharding."""
    # masked to 63 bits: torch.initial_seed() of an unseeded process is a random 64-bit value
    g = torch.Generator().manual_seed((int(seed) * 1_000_003 + int(index)) & 0x7FFF_FFFF_FFFF_FFFF)
    return torch.randn((1, cfg.in_channels, cfg.sample_size, cfg.sample_size), generator=g)


@dataclass
class PipelineOutput:
    images: list


class StableDiffusionPipeline:
    def __init__(self, unet: UNet2DConditionModel, device="cuda", num_inference_steps=50, guidance_scale=7.5,
                 scheduler="ddim", vae=None, text_encoder=None, tokenizer=None, text_encoder_2=None,
                 tokenizer_2=None):
        if scheduler not in ("ddim", "pndm"):
            raise ValueError(f"scheduler must be 'ddim' or 'pndm', got {scheduler!r}")
        self.scheduler = scheduler  # "pndm": the reference's default (51 U-Net calls per 50 steps)
        self.unet = unet
        self.config = unet.config
        self.device = torch.device(device)
        self.num_inference_steps = num_inference_steps
        self.guidance_scale = guidance_scale
        self.prompt_offset = 0  # global index of the first prompt (data-parallel shards set this per rank)
        self.vae = vae  # sdmoe.vae.AutoencoderKLDecoder or None (output_type "pt"/"np" then decodes the latents)
        self.output_type = "latent"  # default of __call__'s output_type (the receivers call pipe(prompt) bare)
        # sdmoe.clip.CLIPTextModel(s) or None (None: seeded synthetic [77, dim] conditioning, prompt_embedding)
        self.text_encoder = text_encoder
        self.tokenizer = tokenizer
        self.text_encoder_2 = text_encoder_2
        self.tokenizer_2 = tokenizer_2

    @classmethod
    def synthetic(cls, cfg: UNetConfig | None = None, seed: int = 0, device="cuda", **kw):
        cfg = cfg or UNetConfig.sd14()
        unet = UNet2DConditionModel.from_state_dict(make_state_dict(cfg, seed), cfg, device)
        return cls(unet, device, **kw)

    @property
    def is_sdxl(self):
        return self.config.addition_embed_type == "text_time"

    def _ids(self, tok, texts):
        return tok(texts, padding="max_length", max_length=CTX_LEN, truncation=True, return_tensors="pt").input_ids

    def encode_prompt(self, prompts, return_pooled=False):
        """[uncond x B ; cond x B] context rows [2B*77, dim] fp16 on device (uncond first, as diffusers).
        SDXL base sets force_zeros_for_empty_prompt: the unconditional embeddings are zeros.
        With text encoders: SD-1.x runs text_encoder on [""] * B + prompts (last_hidden_state); SDXL writes the
        two encoders' penultimate hidden states straight into the two column halves of the context and takes
        text_encoder_2's projected pooled output (diffusers StableDiffusionXLPipeline.encode_prompt)."""
        dim = self.config.cross_attention_dim
        B = len(prompts)
        if self.text_encoder is not None:
            ctx = torch.empty((2 * B * CTX_LEN, dim), dtype=torch.float16, device=self.device)
            pooled = None
            if not self.is_sdxl:
                self.text_encoder.encode(self._ids(self.tokenizer, [""] * B + list(prompts)), out=ctx)
            else:
                d1 = self.text_encoder.config.hidden_size
                ctx[:B * CTX_LEN].zero_()
                cond = ctx[B * CTX_LEN:]
                self.text_encoder.encode(self._ids(self.tokenizer, prompts), hidden_layer=-2, out=cond[:, :d1])
                r = self.text_encoder_2.encode(self._ids(self.tokenizer_2 or self.tokenizer, prompts),
                                               hidden_layer=-2, out=cond[:, d1:], pooled=True)
                pooled = torch.zeros((2 * B, r["text_embeds"].shape[1]), dtype=torch.float16, device=self.device)
                pooled[B:] = r["text_embeds"]
            return (ctx, pooled) if return_pooled else ctx
        unc = torch.zeros(CTX_LEN, dim) if self.is_sdxl else prompt_embedding("", dim)
        embs = [unc] * len(prompts) + [prompt_embedding(p, dim) for p in prompts]
        ctx = torch.cat(embs, 0).to(self.device, torch.float16).contiguous()
        return (ctx, None) if return_pooled else ctx

    def added_cond(self, prompts, pooled=None):
        """SDXL added_cond_kwargs rows [uncond x B ; cond x B]: pooled text_embeds [2B, pooled] and time_ids
        [2B, 6] (1024^2 uncropped at sample_size 128)."""
        cfg = self.config
        d = cfg.pooled_dim
        if pooled is None:
            pooled = torch.stack([torch.zeros(d)] * len(prompts) + [pooled_embedding(p, d) for p in prompts])
        px = 8 * cfg.sample_size
        tids = torch.tensor([sdxl_time_ids(px, px)] * (2 * len(prompts)), dtype=torch.float32)
        return {"text_embeds": pooled, "time_ids": tids}

    def __call__(self, prompt, num_inference_steps=None, guidance_scale=None, latents=None, seed=None,
                 prompt_offset=None, safety_checker=None, output_type=None, **unused):
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        B = len(prompts)
        cfg = self.config
        steps = num_inference_steps or self.num_inference_steps
        g = self.guidance_scale if guidance_scale is None else guidance_scale
        do_cfg = g > 1.0
        if seed is None:
            seed = torch.initial_seed()  # receivers call torch.manual_seed(self.seed) first (base_receiver.py:70)
        if prompt_offset is None:
            prompt_offset = self.prompt_offset
        if latents is None:
            latents = torch.cat([initial_latents(seed, prompt_offset + i, cfg) for i in range(B)])
        lat = latents.to(self.device, torch.float32).contiguous()
        ncopy = 2 if do_cfg else 1
        ctx, pooled = self.encode_prompt(prompts, return_pooled=True)
        add_hidden = None
        if self.is_sdxl:
            ac = self.added_cond(prompts, pooled)
            add_hidden = self.unet.add_embed_hidden(ac["text_embeds"], ac["time_ids"])  # once per call
            if not do_cfg:
                add_hidden = add_hidden[B:]
        if not do_cfg:
            ctx = ctx[B * CTX_LEN:]
        HW = cfg.sample_size * cfg.sample_size
        x_in = torch.zeros((ncopy * B * HW, IN_PAD), dtype=torch.float16, device=self.device)
        eps = torch.empty((ncopy * B * HW, OUT_PAD), dtype=torch.float16, device=self.device)
        ops.prepare_input(lat, x_in, ncopy)
        bufs = dict(lat=lat, x_in=x_in, eps=eps, ctx=ctx, add_hidden=add_hidden)
        self._denoise(bufs, steps, g, do_cfg)
        out = PipelineOutput(images=self._finish(lat, output_type or self.output_type))
        return out

    def _denoise(self, bufs, steps, g, do_cfg):
        """The denoising loop over bufs (lat, x_in, eps, ctx, add_hidden)."""
        lat, x_in, eps, ctx, add_hidden = (bufs[k] for k in ("lat", "x_in", "eps", "ctx", "add_hidden"))

        def temb_row(table, i):
            return None if table is None else table[i:i + 1]

        time_table = self.unet.time_embed_table if PRECOMPUTE_TEMB else (lambda ts: None)
        if self.scheduler == "pndm":
            hist = bufs.setdefault("hist", torch.zeros((4,) + tuple(lat.shape), dtype=torch.float32, device=self.device))
            cur = bufs.setdefault("cur", torch.zeros_like(lat))
            plan = pndm_schedule(steps)
            if "table" not in bufs:
                bufs["table"] = time_table([t for t, _, _ in plan])  # loop-invariant: all steps at once
            table = bufs["table"]
            for i, (t, coef, flags) in enumerate(plan):
                def body(i=i, t=t, coef=coef, flags=flags):
                    self.unet.forward_nhwc(x_in, float(t), ctx, out=eps, add_hidden=add_hidden, temb=temb_row(table, i))
                    ops.cfg_multistep_step(eps, lat, do_cfg, g, hist, cur, coef, flags, next_in=x_in)
                body()
        else:
            ts, a_t, a_prev = ddim_schedule(steps)
            if "table" not in bufs:
                bufs["table"] = time_table(list(ts))  # loop-invariant: all steps at once
            table = bufs["table"]
            for s, t in enumerate(ts):
                def body(s=s, t=t):
                    self.unet.forward_nhwc(x_in, float(t), ctx, out=eps, add_hidden=add_hidden, temb=temb_row(table, s))
                    ops.cfg_ddim_step(eps, lat, do_cfg, g, a_t[s], a_prev[s], next_in=x_in)
                body()

    def _finish(self, lat, output_type):
        """output_type "latent": the denoised latents; "pt" / "np": vae.decode(latents / scaling_factor) then
        (x / 2 + 0.5).clamp(0, 1) as diffusers' VaeImageProcessor does (images [3, H, W] / [H, W, 3])."""
        B = lat.shape[0]
        if output_type == "latent":
            return [lat[i] for i in range(B)]
        if self.vae is None:
            raise ValueError(f"output_type {output_type!r} needs a VAE decoder (pipe.vae = AutoencoderKLDecoder(...))")
        from .vae import postprocess
        img = postprocess(self.vae.decode(lat))
        if output_type == "np":
            return [img[i].permute(1, 2, 0).cpu().numpy() for i in range(B)]
        return [img[i] for i in range(B)]

    def to(self, device):
        """Weights are placed at construction; kept for the reference's `model.to(args.gpu)` call shape."""
        return self
