"""CPU tests of the CLIP text-encoder oracle and host logic (no GPU).

The oracle (oracle/clip_ref.py) is pinned against transformers' own CLIPTextModel / CLIPTextModelWithProjection
(transformers 5.15.0, importable in this image; the reference imports its CLIPMLP, base_receiver.py:5) on the
same random weights: last_hidden_state, every hidden state, the pooled output and text_embeds agree to fp32
rounding (atol 2e-5), for quick_gelu (SD-1.x) and gelu + projection (SDXL text_encoder_2) configs, with the
legacy (argmax) and the first-eos pooling rules."""
import pytest
import torch

from oracle import clip_ref as CR
from sdmoe.clip import CLIPTextConfig, SyntheticCLIPTokenizer, clip_param_specs, make_clip_state_dict

transformers = pytest.importorskip("transformers")


def _hf_model(cfg, sd):
    from transformers import CLIPTextConfig as HFConfig, CLIPTextModel, CLIPTextModelWithProjection
    hc = HFConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                  num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                  max_position_embeddings=cfg.max_position_embeddings, hidden_act=cfg.hidden_act,
                  layer_norm_eps=cfg.layer_norm_eps, projection_dim=cfg.projection_dim or 512,
                  bos_token_id=cfg.bos_token_id, eos_token_id=cfg.eos_token_id, pad_token_id=cfg.pad_token_id,
                  attn_implementation="eager")
    m = (CLIPTextModelWithProjection if cfg.projection_dim else CLIPTextModel)(hc).eval()
    own = m.state_dict()
    mapped = {}
    for k in own:
        src = k if k in sd else "text_model." + k
        if src not in sd and k.startswith("text_model."):
            src = k
        mapped[k] = sd[src]
    m.load_state_dict(mapped, strict=True)
    return m


CASES = [
    ("quick_gelu_legacy_eos", CLIPTextConfig.tiny(64, 3, 2), 0),
    ("gelu_proj_first_eos", CLIPTextConfig(hidden_size=128, intermediate_size=512, num_hidden_layers=2,
                                           num_attention_heads=2, hidden_act="gelu", projection_dim=96,
                                           eos_token_id=49407, pad_token_id=0), 1),
]


@pytest.mark.parametrize("name,cfg,seed", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_transformers(name, cfg, seed):
    sd = make_clip_state_dict(cfg, seed)
    tok = SyntheticCLIPTokenizer(pad_token_id=cfg.pad_token_id)
    ids = tok(["a photo of a cat", "", "the starry night, by Vincent van Gogh", "x" * 3 + " y"]).input_ids
    m = _hf_model(cfg, sd)
    with torch.no_grad():
        o = m(ids, output_hidden_states=True)
    hs, last, pooled, te = CR.encode_ref(ids, sd, cfg)
    torch.testing.assert_close(last, o.last_hidden_state, atol=2e-5, rtol=1e-5)
    assert len(hs) == len(o.hidden_states)
    for a, b in zip(hs, o.hidden_states):
        torch.testing.assert_close(a, b, atol=2e-5, rtol=1e-5)
    if cfg.projection_dim:
        torch.testing.assert_close(te, o.text_embeds, atol=2e-5, rtol=1e-5)
    else:
        torch.testing.assert_close(pooled, o.pooler_output, atol=2e-5, rtol=1e-5)


def test_oracle_mlp_hook_seam_is_identity_with_reference_body():
    cfg = CLIPTextConfig.tiny(64, 2, 2)
    sd = make_clip_state_dict(cfg, 3)
    ids = SyntheticCLIPTokenizer()(["a dog"]).input_ids
    base = CR.encode_ref(ids, sd, cfg)[1]
    hooked = CR.encode_ref(ids, sd, cfg, mlp_hook=lambda i, h: CR.mlp_ref(
        h, sd, f"text_model.encoder.layers.{i}.mlp", cfg.hidden_act))[1]
    torch.testing.assert_close(base, hooked)
    # zero mask: WandaRemoveNeuronsFast.text_hook_fn == plain MLP
    F = cfg.intermediate_size
    zero = torch.zeros(cfg.hidden_size, F)
    h = torch.randn(1, 5, cfg.hidden_size)
    p = "text_model.encoder.layers.0.mlp"
    torch.testing.assert_close(CR.wanda_remove_text_hook(h, sd, p, cfg.hidden_act, zero),
                               CR.mlp_ref(h, sd, p, cfg.hidden_act))
    rows, out = CR.wanda_text_stats(h, sd, p, cfg.hidden_act)
    torch.testing.assert_close(rows.norm(dim=1), torch.ones(5))
    torch.testing.assert_close(out, CR.mlp_ref(h, sd, p, cfg.hidden_act))


def test_tokenizer_layout():
    tok = SyntheticCLIPTokenizer()
    e = tok(["a cat", "word " * 100])
    ids = e.input_ids
    assert ids.shape == (2, 77)
    assert ids[0, 0] == 49406 and ids[0, 3] == 49407 and bool((ids[0, 3:] == 49407).all())
    assert ids[1, 0] == 49406 and ids[1, 76] == 49407  # truncated to 75 words + bos + eos
    assert bool((ids[:, 1:] < 49406).sum(1).ge(2).all())
    assert e.attention_mask[0].sum() == 4
    assert tok("A Cat").input_ids.equal(tok("a cat").input_ids[:1])
    t2 = SyntheticCLIPTokenizer(pad_token_id=0)
    assert t2("a").input_ids[0, 3:].eq(0).all()


def test_param_specs_sd14_and_sdxl_g():
    n14 = sum(torch.Size(s).numel() for _, s in clip_param_specs(CLIPTextConfig.sd14()))
    assert n14 == 123_060_480  # openai/clip-vit-large-patch14 text tower
    ng = sum(torch.Size(s).numel() for _, s in clip_param_specs(CLIPTextConfig.sdxl_g()))
    assert ng == 694_659_840  # SDXL text_encoder_2 (OpenCLIP bigG text tower + projection)


def test_text_hook_seam_module_names_cpu():
    """hook_module='text' finds the 12 CLIPMLP modules by the reference's filter (base_receiver.py:62-63) and the
    text receivers register text_hook_fn on them (no GPU compute: weights stay on the CPU)."""
    from neuron_receivers import Wanda, WandaRemoveNeuronsFast
    from neuron_receivers.base_receiver import text_mlp_modules
    from sdmoe.clip import CLIPTextModel
    cfg = CLIPTextConfig.sd14()
    enc = CLIPTextModel.from_state_dict({n: torch.zeros(s) for n, s in clip_param_specs(cfg)}, cfg, "cpu")

    class P:
        text_encoder = enc
    mods = text_mlp_modules(P)
    assert [n for n, _ in mods] == [f"text_model.encoder.layers.{i}.mlp" for i in range(12)]
    assert type(mods[0][1]).__name__ == "CLIPMLP" and mods[0][1].fc2.weight.shape == (768, 3072)
    rec = Wanda(0, 1, 12, hook_module='text')
    hooks = rec.register_hooks(P)
    assert len(hooks) == 12 and all(m._sdmoe_deferred == 1 for _, m in mods)
    rec.remove_hooks(hooks)
    assert all(m._sdmoe_deferred == 0 and not m._forward_hooks for _, m in mods)
    masks = {0: {l: torch.zeros(768, 3072, dtype=torch.int64) for l in range(12)}}
    r2 = WandaRemoveNeuronsFast(0, None, 1, 12, hook_module='text', masks=masks)
    assert r2.mask_bits[0][11].shape == (768, 384)
    hooks = r2.register_hooks(P)
    assert all(h is not None for h in hooks) and len(hooks) == 12
    r2.remove_hooks(hooks)


GOLDEN = {"clip_quick_gelu_legacy": CLIPTextConfig.tiny(64, 2, 2),
          "clip_gelu_proj": CLIPTextConfig(hidden_size=64, intermediate_size=256, num_hidden_layers=2,
                                           num_attention_heads=2, hidden_act="gelu", projection_dim=32,
                                           eos_token_id=49407, pad_token_id=0)}


@pytest.mark.parametrize("name", sorted(GOLDEN))
def test_oracle_vs_reference_text_goldens(name, golden_dir):
    """Committed fixtures (tests/golden/make_clip_golden.py): transformers' CLIPTextModel outputs and the
    REFERENCE's own text_hook_fn bodies (remove_wanda_neurons_fast.py:85-101, wanda_receiver.py:59-71) run on
    transformers' CLIPMLP — the oracle reproduces all of them without transformers or the reference present."""
    import os
    import numpy as np
    from oracle import hooks_ref  # noqa: F401  (oracle package import check)
    from sdmoe import mask_io
    g = np.load(os.path.join(golden_dir, f"{name}.npz"))
    cfg = GOLDEN[name]
    sd = make_clip_state_dict(cfg, int(g["seed"]))
    ids = torch.from_numpy(g["ids"])
    assert torch.equal(ids, SyntheticCLIPTokenizer(pad_token_id=cfg.pad_token_id)(
        ["a photo of a cat", "", "The Starry Night, a painting by Vincent van Gogh",
         "nude figure, oil on canvas"]).input_ids)
    hs, last, pooled, te = CR.encode_ref(ids, sd, cfg)
    torch.testing.assert_close(last, torch.from_numpy(g["last"]), atol=2e-5, rtol=1e-5)
    torch.testing.assert_close(torch.stack(hs), torch.from_numpy(g["hidden"]), atol=2e-5, rtol=1e-5)
    if cfg.projection_dim:
        torch.testing.assert_close(te, torch.from_numpy(g["text_embeds"]), atol=2e-5, rtol=1e-5)
    else:
        torch.testing.assert_close(pooled, torch.from_numpy(g["pooled"]), atol=2e-5, rtol=1e-5)
    h = torch.from_numpy(g["hook_h"])
    L, F = cfg.num_hidden_layers, cfg.intermediate_size
    for l in range(L):
        p = f"text_model.encoder.layers.{l}.mlp"
        mask = torch.from_numpy(mask_io.unpack_mask(g["hook_mask_bits"][l], F).astype(np.float32))
        torch.testing.assert_close(CR.wanda_remove_text_hook(h, sd, p, cfg.hidden_act, mask),
                                   torch.from_numpy(g["remove_out"][l]), atol=1e-5, rtol=1e-5)
        rows = []
        for rep in range(2):
            r, out = CR.wanda_text_stats(h * (1.0 + rep), sd, p, cfg.hidden_act)
            rows.append(r)
            torch.testing.assert_close(out, torch.from_numpy(g["wanda_out"][rep * L + l]), atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(torch.cat(rows).norm(dim=0), torch.from_numpy(g["wanda_norms"][l]),
                                   atol=1e-5, rtol=1e-5)
    assert list(g["remove_counter"]) == [1, 0]  # one hooked call per layer wraps the (t, l) counter once
