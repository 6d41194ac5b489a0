"""CLIP text encoder and the reference's hook_module='text' seam on the GPU.

Oracle: oracle/clip_ref.py, pinned against transformers' CLIPTextModel on CPU (tests/test_clip_oracle.py). The HIP
encoder runs fp16 storage / fp32 accumulation; it is compared with the oracle on the same fp16-rounded weights:
hidden states within rel-L2 1e-2 (12 and 32 fp16 layers), pooled / projected outputs within 2e-2; the helper kernels
are exact (gather) or within 2e-3 of torch fp32 (short attention)."""
import pytest
import torch

from oracle import clip_ref as CR
from sdmoe import ops
from sdmoe.clip import (CLIPTextConfig, CLIPTextModel, SyntheticCLIPTokenizer, attach_text_encoders,
                        make_clip_state_dict)

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PROMPTS = ["a photo of a cat", "", "The Starry Night, a painting by Vincent van Gogh", "a dog " * 40]


def rel_l2(a, b):
    return ((a.float().cpu() - b.float().cpu()).norm() / b.float().cpu().norm()).item()


def h16(sd):
    return {k: v.half().float() for k, v in sd.items()}


def test_gather_rows_exact():
    table = torch.randn(1000, 136).half().to(DEV)
    pos = torch.randn(77, 136).half().to(DEV)
    idx = torch.randint(0, 1000, (3 * 77,), dtype=torch.int32).to(DEV)
    y = ops.gather_rows(table, idx, add=pos, period=77)
    exp = (table[idx.long()].float() + pos.float().repeat(3, 1)).half()
    assert torch.equal(y, exp)
    out = torch.zeros(5, 200, dtype=torch.float16, device=DEV)
    ops.gather_rows(table, idx[:5], out=out[:, 8:144])
    assert torch.equal(out[:, 8:144], table[idx[:5].long()]) and not out[:, :8].any()


@pytest.mark.parametrize("nseq,N,heads,D,causal", [(4, 77, 12, 64, True), (2, 77, 20, 64, True),
                                                   (3, 128, 1, 128, False), (2, 5, 3, 8, True),
                                                   (1, 77, 2, 64, False)])
def test_attention_short(nseq, N, heads, D, causal):
    C = heads * D
    qkv = torch.randn(nseq * N, 3 * C + 8).half().to(DEV)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:3 * C]
    o = ops.attention_short(q, k, v, nseq, N, heads, causal=causal)

    def split(t):
        return t.float().view(nseq, N, heads, D).transpose(1, 2)
    s = split(q) @ split(k).transpose(-1, -2) * D ** -0.5
    if causal:
        s = s + torch.full((N, N), float("-inf"), device=DEV).triu(1)
    ref = (s.softmax(-1) @ split(v)).transpose(1, 2).reshape(nseq * N, C)
    assert (o.float() - ref).abs().max().item() <= 2e-3 * max(1.0, ref.abs().max().item())


def test_linear_quick_gelu():
    x = torch.randn(300, 128).half().to(DEV)
    w = (torch.randn(512, 128) / 11).half().to(DEV)
    b = torch.randn(512).half().to(DEV)
    y = ops.linear(x, w, b, act=ops.ACT_QUICK_GELU)
    z = x.float() @ w.float().t() + b.float()
    ref = z * torch.sigmoid(1.702 * z)
    assert (y.float() - ref).abs().max().item() <= 1e-2 * max(1.0, ref.abs().max().item())


ENC = [("tiny_quick_gelu", CLIPTextConfig.tiny(128, 2, 2)),
       ("tiny_gelu_proj", CLIPTextConfig(hidden_size=128, intermediate_size=512, num_hidden_layers=3,
                                         num_attention_heads=2, hidden_act="gelu", projection_dim=64,
                                         eos_token_id=49407, pad_token_id=0)),
       ("sd14", CLIPTextConfig.sd14()),
       ("sdxl_g", CLIPTextConfig.sdxl_g())]


@pytest.mark.parametrize("name,cfg", ENC, ids=[e[0] for e in ENC])
def test_encoder_vs_oracle(name, cfg):
    sd = make_clip_state_dict(cfg, 5)
    enc = CLIPTextModel.from_state_dict(sd, cfg, DEV)
    ids = SyntheticCLIPTokenizer(pad_token_id=cfg.pad_token_id)(PROMPTS).input_ids
    hs, last, pooled, te = CR.encode_ref(ids, h16(sd), cfg)
    r = enc.encode(ids, pooled=True)
    torch.cuda.synchronize()
    B, L, C = last.shape
    assert rel_l2(r["hidden"], last.reshape(B * L, C)) <= 1e-2
    assert rel_l2(r["pooled"], pooled) <= 2e-2
    if cfg.projection_dim:
        assert rel_l2(r["text_embeds"], te) <= 2e-2
    pen = enc.encode(ids, hidden_layer=-2)["hidden"]
    assert rel_l2(pen, hs[-2].reshape(B * L, C)) <= 1e-2
    # transformers-shaped call
    o = enc(ids, output_hidden_states=True)
    assert torch.equal(o.last_hidden_state.reshape(B * L, C), r["hidden"])
    assert torch.equal(o.hidden_states[-2].reshape(B * L, C), pen)


def test_penultimate_into_column_slices_and_pooled():
    """SDXL layout: both encoders write their penultimate states straight into column halves of one buffer; the
    bigG-style encoder still runs its last layer for the pooled projection."""
    c1 = CLIPTextConfig.tiny(64, 2, 1)
    c2 = CLIPTextConfig(hidden_size=128, intermediate_size=512, num_hidden_layers=3, num_attention_heads=2,
                        hidden_act="gelu", projection_dim=96, pad_token_id=0)
    sd1, sd2 = make_clip_state_dict(c1, 1), make_clip_state_dict(c2, 2)
    e1, e2 = CLIPTextModel.from_state_dict(sd1, c1, DEV), CLIPTextModel.from_state_dict(sd2, c2, DEV)
    ids1 = SyntheticCLIPTokenizer()(PROMPTS[:2]).input_ids
    ids2 = SyntheticCLIPTokenizer(pad_token_id=0)(PROMPTS[:2]).input_ids
    buf = torch.zeros(2 * 77, 192, dtype=torch.float16, device=DEV)
    e1.encode(ids1, hidden_layer=-2, out=buf[:, :64])
    r = e2.encode(ids2, hidden_layer=-2, out=buf[:, 64:], pooled=True)
    h1 = CR.encode_ref(ids1, h16(sd1), c1)[0][-2].reshape(-1, 64)
    hs2, _, _, te2 = CR.encode_ref(ids2, h16(sd2), c2)
    assert rel_l2(buf[:, :64], h1) <= 1e-2
    assert rel_l2(buf[:, 64:], hs2[-2].reshape(-1, 128)) <= 1e-2
    assert rel_l2(r["text_embeds"], te2) <= 2e-2


def test_pipeline_encode_prompt_sd_and_denoise_vs_oracle():
    from oracle.unet_ref import UNetRef, denoise
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline, initial_latents
    from sdmoe.weights import make_state_dict
    cfg = UNetConfig.tiny(8)
    sd = make_state_dict(cfg, 0)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device=DEV, num_inference_steps=2)
    (sdt,) = attach_text_encoders(pipe, seed=3)
    prompts = ["a cat", "a painting by van gogh"]
    ctx = pipe.encode_prompt(prompts)
    tcfg = pipe.text_encoder.config
    ids = pipe.tokenizer([""] * 2 + prompts).input_ids
    exp_ctx = CR.encode_ref(ids, h16(sdt), tcfg)[1]
    assert rel_l2(ctx, exp_ctx.reshape(-1, tcfg.hidden_size)) <= 1e-2
    out = pipe(prompts, seed=0).images
    ref = UNetRef({k: v.half().float() for k, v in sd.items()}, cfg)
    lat = torch.cat([initial_latents(0, i, cfg) for i in range(2)])
    exp = denoise(ref, lat, exp_ctx[:2], exp_ctx[2:], num_inference_steps=2)
    assert rel_l2(torch.stack(out), exp) <= 3e-2


def test_pipeline_sdxl_text_encoders_tiny():
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    cfg = UNetConfig.tiny_xl(8)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device=DEV, num_inference_steps=1)
    sd1, sd2 = attach_text_encoders(pipe, seed=4)
    prompts = ["a cat", "a dog"]
    ctx, pooled = pipe.encode_prompt(prompts, return_pooled=True)
    c1, c2 = pipe.text_encoder.config, pipe.text_encoder_2.config
    h1 = CR.encode_ref(pipe.tokenizer(prompts).input_ids, h16(sd1), c1)[0][-2]
    hs2, _, _, te = CR.encode_ref(pipe.tokenizer_2(prompts).input_ids, h16(sd2), c2)
    d1 = c1.hidden_size
    assert not ctx[:2 * 77].any() and not pooled[:2].any()  # force_zeros_for_empty_prompt
    assert rel_l2(ctx[2 * 77:, :d1], h1.reshape(-1, d1)) <= 1e-2
    assert rel_l2(ctx[2 * 77:, d1:], hs2[-2].reshape(-1, c2.hidden_size)) <= 1e-2
    assert rel_l2(pooled[2:], te) <= 2e-2
    imgs = pipe(prompts, seed=0).images
    assert all(torch.isfinite(i).all() for i in imgs)


def _tiny_sd_pipe():
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    pipe = StableDiffusionPipeline.synthetic(UNetConfig.tiny(8), seed=0, device=DEV, num_inference_steps=1)
    (sdt,) = attach_text_encoders(pipe, seed=6)
    return pipe, sdt


def test_text_hook_wanda_remove_vs_oracle():
    """WandaRemoveNeuronsFast(hook_module='text'): fc2 weights masked by M[0][layer] in every CLIP layer
    (remove_wanda_neurons_fast.py:85-101), through the receiver's registered hooks."""
    from neuron_receivers import WandaRemoveNeuronsFast
    pipe, sdt = _tiny_sd_pipe()
    tcfg = pipe.text_encoder.config
    C, F, L = tcfg.hidden_size, tcfg.intermediate_size, tcfg.num_hidden_layers
    g = torch.Generator().manual_seed(9)
    masks = {0: {l: (torch.rand(C, F, generator=g) < 0.3).to(torch.int64) for l in range(L)}}
    rec = WandaRemoveNeuronsFast(0, None, 1, L, hook_module='text', masks=masks, store_gates=False)
    prompts = ["a cat", "a dog"]
    rec.prepare(pipe)
    hooks = rec.register_hooks(pipe)
    try:
        ctx = pipe.encode_prompt(prompts)
    finally:
        rec.remove_hooks(hooks)
    assert rec.layer == 0 and rec.timestep == 1  # one hooked call per layer, counter wrapped once
    ids = pipe.tokenizer([""] * 2 + prompts).input_ids
    sd16 = h16(sdt)
    exp = CR.encode_ref(ids, sd16, tcfg, mlp_hook=lambda i, h: CR.wanda_remove_text_hook(
        h, sd16, f"text_model.encoder.layers.{i}.mlp", tcfg.hidden_act, masks[0][i].float()))[1]
    base = CR.encode_ref(ids, sd16, tcfg)[1]
    assert rel_l2(ctx, exp.reshape(-1, C)) <= 1e-2
    assert rel_l2(exp, base) > 5e-2  # the masks matter at this tolerance
    # hooks removed: the plain encoder path is back
    assert rel_l2(pipe.encode_prompt(prompts), base.reshape(-1, C)) <= 1e-2
    # and the full receiver flow runs end to end
    out, _ = rec.observe_activation(pipe, prompts)
    assert len(out) == 2 and all(torch.isfinite(o).all() for o in out)


def test_text_hook_wanda_stats_vs_oracle():
    """Wanda(hook_module='text'): per-layer column norms of the row-normalised act(fc1 x) (wanda_receiver.py:59-71)."""
    from neuron_receivers import Wanda
    pipe, sdt = _tiny_sd_pipe()
    tcfg = pipe.text_encoder.config
    L = tcfg.num_hidden_layers
    rec = Wanda(0, 1, L, hook_module='text')
    prompts = ["a cat", "a dog"]
    hooks = rec.register_hooks(pipe)
    try:
        ctx = pipe.encode_prompt(prompts)
    finally:
        rec.remove_hooks(hooks)
    ids = pipe.tokenizer([""] * 2 + prompts).input_ids
    sd16 = h16(sdt)
    rows = {}

    def hook(i, h):
        r, out = CR.wanda_text_stats(h, sd16, f"text_model.encoder.layers.{i}.mlp", tcfg.hidden_act)
        rows[i] = r
        return out
    last = CR.encode_ref(ids, sd16, tcfg, mlp_hook=hook)[1]
    assert rel_l2(ctx, last.reshape(-1, tcfg.hidden_size)) <= 1e-2
    for l in range(L):
        got = rec.predictivity[l].get_column_norms().float()
        exp = rows[l].norm(dim=0)
        assert rel_l2(got, exp) <= 1e-2, l


@pytest.mark.parametrize("name", ["clip_quick_gelu_legacy", "clip_gelu_proj"])
def test_text_hooks_vs_reference_goldens(name, golden_dir):
    """Our HIP receivers' text_hook_fn vs the REFERENCE's own text_hook_fn outputs (tests/golden/make_clip_golden.py,
    computed in fp32 on transformers' CLIPMLP): fp16 storage, rel-L2 <= 1e-2; the encoder vs transformers' outputs."""
    import os
    import numpy as np
    from neuron_receivers import Wanda, WandaRemoveNeuronsFast
    from test_clip_oracle import GOLDEN
    g = np.load(os.path.join(golden_dir, f"{name}.npz"))
    cfg = GOLDEN[name]
    sd = make_clip_state_dict(cfg, int(g["seed"]))
    enc = CLIPTextModel.from_state_dict(sd, cfg, DEV)
    ids = torch.from_numpy(g["ids"])
    r = enc.encode(ids, pooled=True)
    B, L_, C = g["last"].shape
    assert rel_l2(r["hidden"], torch.from_numpy(g["last"]).reshape(B * L_, C)) <= 1e-2
    key = "text_embeds" if cfg.projection_dim else "pooled"
    assert rel_l2(r[key], torch.from_numpy(g[key])) <= 2e-2
    L = cfg.num_hidden_layers
    mlps = [enc.text_model.encoder.layers[l].mlp for l in range(L)]
    h = torch.from_numpy(g["hook_h"]).half().to(DEV)
    rm = WandaRemoveNeuronsFast.from_packed(0, {0: {l: g["hook_mask_bits"][l] for l in range(L)}}, 1, L,
                                            hook_module='text')
    for l in range(L):
        out = rm.text_hook_fn(mlps[l], (h,), None)
        assert rel_l2(out, torch.from_numpy(g["remove_out"][l])) <= 1e-2, l
    assert [rm.timestep, rm.layer] == list(g["remove_counter"])
    w = Wanda(0, 1, L, hook_module='text')
    for rep in range(2):
        for l in range(L):
            out = w.text_hook_fn(mlps[l], (h * (1.0 + rep),), None)
            assert rel_l2(out, torch.from_numpy(g["wanda_out"][rep * L + l])) <= 1e-2
    for l in range(L):
        assert rel_l2(w.predictivity[l].get_column_norms(), torch.from_numpy(g["wanda_norms"][l])) <= 1e-2
