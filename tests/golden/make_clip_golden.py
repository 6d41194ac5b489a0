"""Golden vectors for the CLIP text encoder and the reference's hook_module='text' hook bodies.

Runs only in the build container (needs /root/reference and transformers): the encoder outputs come from
transformers' own CLIPTextModel / CLIPTextModelWithProjection (the reference's text_encoder class, unpinned
external dependency) on seeded random weights (sdmoe.clip.make_clip_state_dict, regenerated bit-exactly from the
seed by the tests); the hook outputs come from the REFERENCE's own functions, imported through the same diffusers
stub as make_golden.py and called on transformers' real CLIPMLP modules:
  * WandaRemoveNeuronsFast.text_hook_fn   neuron_receivers/remove_wanda_neurons_fast.py:85-101
  * Wanda.text_hook_fn + ColumnNormCalculator   neuron_receivers/wanda_receiver.py:59-71, utils.py:321-340
Only data (inputs and outputs) is written.

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_clip_golden.py
"""
from __future__ import annotations

import os
import pickle
import sys
import tempfile

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(OUT))
sys.path[:0] = [OUT, os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
import make_golden as MG  # noqa: E402
from sdmoe.clip import CLIPTextConfig, SyntheticCLIPTokenizer, make_clip_state_dict  # noqa: E402

PROMPTS = ["a photo of a cat", "", "The Starry Night, a painting by Vincent van Gogh", "nude figure, oil on canvas"]
CASES = {
    "clip_quick_gelu_legacy": (CLIPTextConfig.tiny(64, 2, 2), 11),
    "clip_gelu_proj": (CLIPTextConfig(hidden_size=64, intermediate_size=256, num_hidden_layers=2,
                                      num_attention_heads=2, hidden_act="gelu", projection_dim=32,
                                      eos_token_id=49407, pad_token_id=0), 12),
}


def hf_model(cfg, sd):
    from transformers import CLIPTextConfig as HC, CLIPTextModel, CLIPTextModelWithProjection
    hc = HC(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
            max_position_embeddings=cfg.max_position_embeddings, hidden_act=cfg.hidden_act,
            layer_norm_eps=cfg.layer_norm_eps, projection_dim=cfg.projection_dim or 512,
            bos_token_id=cfg.bos_token_id, eos_token_id=cfg.eos_token_id, pad_token_id=cfg.pad_token_id,
            attn_implementation="eager")
    m = (CLIPTextModelWithProjection if cfg.projection_dim else CLIPTextModel)(hc).eval()
    own = m.state_dict()
    m.load_state_dict({k: sd[k] if k in sd else sd["text_model." + k] for k in own}, strict=True)
    return m


def mlp_of(m, i):
    tm = m.text_model if hasattr(m, "text_model") else m
    return tm.encoder.layers[i].mlp


def main():
    import transformers
    MG.install_stubs()
    MG.load_ref("neuron_receivers.base_receiver", "neuron_receivers/base_receiver.py")
    MG.load_ref("neuron_receivers.predictivity", "neuron_receivers/predictivity.py")
    MG.load_ref("utils", "utils.py")
    wanda_rm = MG.load_ref("neuron_receivers.remove_wanda_neurons_fast", "neuron_receivers/remove_wanda_neurons_fast.py")
    wanda_rx = MG.load_ref("neuron_receivers.wanda_receiver", "neuron_receivers/wanda_receiver.py")
    import scipy.sparse
    for name, (cfg, seed) in CASES.items():
        sd = make_clip_state_dict(cfg, seed)
        ids = SyntheticCLIPTokenizer(pad_token_id=cfg.pad_token_id)(PROMPTS).input_ids
        m = hf_model(cfg, sd)
        with torch.no_grad():
            o = m(ids, output_hidden_states=True)
        rec = dict(kind=np.array("clip_text"), dtype=np.array("float32"), ids=ids.numpy(), seed=np.array(seed),
                   transformers_version=np.array(transformers.__version__), last=o.last_hidden_state.numpy(), hidden=np.stack([h.numpy() for h in o.hidden_states]))
        if cfg.projection_dim:
            rec["text_embeds"] = o.text_embeds.numpy()
        else:
            rec["pooled"] = o.pooler_output.numpy()
        # reference hook bodies on transformers' CLIPMLP modules
        L, C, F = cfg.num_hidden_layers, cfg.hidden_size, cfg.intermediate_size
        g = torch.Generator().manual_seed(seed + 100)
        h = torch.randn(2, 7, C, generator=g)
        masks = (torch.rand(L, C, F, generator=g) < 0.3).to(torch.int64)
        with tempfile.TemporaryDirectory() as d:
            for l in range(L):
                with open(os.path.join(d, f"timestep_0_layer_{l}.pkl"), "wb") as f:
                    pickle.dump(scipy.sparse.csr_matrix(masks[l].numpy()), f)
            r = MG.quiet(wanda_rm.WandaRemoveNeuronsFast, 0, d, 1, L, hook_module='text')
            with torch.no_grad():
                rm_out = [r.text_hook_fn(mlp_of(m, l), (h,), mlp_of(m, l)(h)).numpy() for l in range(L)]
        w = MG.quiet(wanda_rx.Wanda, 0, 1, L, hook_module='text')
        with torch.no_grad():
            w_out = []
            for rep in range(2):  # two calls per layer: the running column norm combines them
                for l in range(L):
                    x = h * (1.0 + rep)
                    w_out.append(w.text_hook_fn(mlp_of(m, l), (x,), mlp_of(m, l)(x)).numpy())
        rec.update(hook_h=h.numpy(), hook_mask_bits=np.packbits(masks.numpy().astype(np.uint8), axis=-1,
                                                                bitorder="little"),
                   remove_out=np.stack(rm_out), wanda_out=np.stack(w_out),
                   wanda_norms=np.stack([w.predictivity[l].get_column_norms().numpy() for l in range(L)]),
                   remove_counter=np.array([r.timestep, r.layer]))
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **rec)
        print("wrote", name)


if __name__ == "__main__":
    main()
