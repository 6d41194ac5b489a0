"""CPU fp32 restatement of the CLIP text encoder (transformers CLIPTextModel / CLIPTextModelWithProjection), the
oracle of sdmoe.clip, plus the reference's two text-encoder hook bodies. TEST INFRASTRUCTURE: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.

transformers is an unpinned external dependency of the reference (base_receiver.py:5 and
remove_wanda_neurons_fast.py:9 import `transformers.models.clip.modeling_clip.CLIPMLP`; the pipelines'
text_encoder is transformers' CLIPTextModel). transformers 5.15.0 is importable in this image, so this
restatement is PINNED against transformers' own CLIPTextModel(WithProjection) on the same random weights
(tests/test_clip_oracle.py). It follows modeling_clip.py: CLIPTextEmbeddings (token + position embedding),
CLIPEncoderLayer (pre-LN causal self-attention, pre-LN MLP fc1 -> act -> fc2, residuals), final_layer_norm,
pooled output at argmax(ids) for the legacy eos_token_id == 2 configs (else the first eos position), optional
text_projection.

Hook bodies (hook_module='text'):
  * remove_wanda_neurons_fast.py:85-101 (WandaRemoveNeuronsFast.text_hook_fn): fc2 with W * (1 - M[0][layer]);
  * wanda_receiver.py:59-71 (Wanda.text_hook_fn): act(fc1 x) rows, L2-normalised, column norms accumulated.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _act(x, name):
    if name == "quick_gelu":
        return x * torch.sigmoid(1.702 * x)
    if name == "gelu":
        return F.gelu(x)
    raise ValueError(name)


def _lin(x, sd, p, wmask=None):
    w = sd[p + ".weight"]
    if wmask is not None:
        w = w * (1 - wmask)
    return F.linear(x, w, sd.get(p + ".bias"))


def _ln(x, sd, p, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def mlp_ref(h, sd, p, act):
    """CLIPMLP.forward (modeling_clip.py CLIPMLP): fc2(act(fc1(h)))."""
    return _lin(_act(_lin(h, sd, p + ".fc1"), act), sd, p + ".fc2")


def encode_ref(ids, sd, cfg, mlp_hook=None):
    """Returns (hidden_states tuple [emb, layer0, ..., layerN-1] (pre final LN), last_hidden_state, pooled,
    text_embeds or None). ids: int64 [B, L]. mlp_hook(layer_index, h [B, L, C]) -> MLP output replaces CLIPMLP
    (the forward hook seam, base_receiver.py:59-65)."""
    B, L = ids.shape
    C, H = cfg.hidden_size, cfg.num_attention_heads
    d = C // H
    x = sd["text_model.embeddings.token_embedding.weight"][ids] + \
        sd["text_model.embeddings.position_embedding.weight"][:L][None]
    hs = [x]
    causal = torch.full((L, L), float("-inf")).triu(1)
    for i in range(cfg.num_hidden_layers):
        p = f"text_model.encoder.layers.{i}"
        h = _ln(x, sd, p + ".layer_norm1", cfg.layer_norm_eps)
        q = _lin(h, sd, p + ".self_attn.q_proj").view(B, L, H, d).transpose(1, 2)
        k = _lin(h, sd, p + ".self_attn.k_proj").view(B, L, H, d).transpose(1, 2)
        v = _lin(h, sd, p + ".self_attn.v_proj").view(B, L, H, d).transpose(1, 2)
        s = q @ k.transpose(-1, -2) * d ** -0.5 + causal
        a = (s.softmax(-1) @ v).transpose(1, 2).reshape(B, L, C)
        x = x + _lin(a, sd, p + ".self_attn.out_proj")
        h = _ln(x, sd, p + ".layer_norm2", cfg.layer_norm_eps)
        x = x + (mlp_hook(i, h) if mlp_hook is not None else mlp_ref(h, sd, p + ".mlp", cfg.hidden_act))
        hs.append(x)
    last = _ln(x, sd, "text_model.final_layer_norm", cfg.layer_norm_eps)
    if cfg.eos_token_id == 2:
        pos = ids.argmax(-1)
    else:
        pos = (ids == cfg.eos_token_id).int().argmax(-1)
    pooled = last[torch.arange(B), pos]
    te = F.linear(pooled, sd["text_projection.weight"]) if cfg.projection_dim else None
    return tuple(hs), last, pooled, te


def wanda_remove_text_hook(h, sd, p, act, mask):
    """WandaRemoveNeuronsFast.text_hook_fn (remove_wanda_neurons_fast.py:85-101): fc1 -> act ->
    F.linear(., fc2.weight * (1 - mask), fc2.bias)."""
    return _lin(_act(_lin(h, sd, p + ".fc1"), act), sd, p + ".fc2", wmask=mask)


def wanda_text_stats(h, sd, p, act):
    """Wanda.text_hook_fn (wanda_receiver.py:59-71): the rows the ColumnNormCalculator receives
    (act(fc1 h) flattened, L2-normalised per row) and the unchanged MLP output."""
    a = _act(_lin(h, sd, p + ".fc1"), act)
    rows = F.normalize(a.reshape(-1, a.shape[-1]), p=2, dim=1)
    return rows, _lin(a, sd, p + ".fc2")
