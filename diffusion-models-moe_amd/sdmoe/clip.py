"""CLIP text encoder on the sdmoe HIP kernels — SURVEY §8f rank 4, the prompt encoder in front of the denoising
loop (`StableDiffusionPipeline.encode_prompt` -> `text_encoder(input_ids)[0]`, diffusers/transformers, external;
the reference reaches it through `model(prompt)`, base_receiver.py:73) and the reference's second hook seam:
`hook_module='text'` registers `text_hook_fn` on every `CLIPMLP` named `...encoder.layers.{i}.mlp`
(base_receiver.py:59-65, remove_wanda_neurons_fast.py:114-120, wanda_receiver.py:59-71).

Module tree and state-dict names follow transformers' CLIPTextModel (`text_model.embeddings.token_embedding`,
`text_model.encoder.layers.{i}.{self_attn.{q,k,v,out}_proj, layer_norm1, mlp.{fc1,fc2}, layer_norm2}`,
`text_model.final_layer_norm`, `text_projection` for CLIPTextModelWithProjection), so `named_modules()` filters
and checkpoint keys mean what they mean in the reference. Configs: SD-1.x ViT-L/14 text tower (12 x 768,
quick_gelu), and SDXL's pair (ViT-L penultimate layer + OpenCLIP bigG, 32 x 1280, gelu, 1280-d projection).

MI355X layout: the residual stream is one fp16 [sequences*77, C] row view (it may be a column slice of a wider
buffer: SDXL's two encoders write their penultimate hidden states straight into the two halves of the [.., 2048]
U-Net context, no concatenation copy). Per layer: sdmoe_layernorm -> fused QKV sdmoe_linear [3C, C] ->
sdmoe_attention_short (causal, K/V in LDS) -> out_proj with the residual add in its epilogue -> sdmoe_layernorm ->
fc1 with quick_gelu/gelu in the epilogue -> fc2 with the residual add in its epilogue. Two ping-pong stream
buffers, no in-place epilogues. A hooked CLIPMLP is deferred (skips its own forward) and the receiver's
text_hook_fn computes it; the residual is then added by sdmoe_add.

Tokenizer: the CLIP BPE vocabulary (vocab.json / merges.txt) is not available offline, so `SyntheticCLIPTokenizer`
maps words to stable ids (crc32) with CLIP's BOS/EOS/padding and the 77-token truncation; any tokenizer with the
transformers call signature (e.g. transformers.CLIPTokenizer on a local checkpoint directory) can replace it.
"""
from __future__ import annotations

import re
import zlib
from dataclasses import dataclass

import torch
import torch.nn as nn

from . import ops
from .unet import LoRACompatibleLinear, _buf


@dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: int = 0      # > 0: CLIPTextModelWithProjection (SDXL text_encoder_2)
    bos_token_id: int = 49406
    eos_token_id: int = 2        # the SD checkpoints' text configs carry the legacy value 2 (pool at argmax(ids))
    pad_token_id: int = 49407

    @staticmethod
    def sd14():
        """openai/clip-vit-large-patch14 text tower (SD-1.x text_encoder)."""
        return CLIPTextConfig()

    @staticmethod
    def sdxl_l():
        """SDXL-base text_encoder (ViT-L, penultimate hidden states)."""
        return CLIPTextConfig()

    @staticmethod
    def sdxl_g():
        """SDXL-base text_encoder_2 (OpenCLIP ViT-bigG text tower with projection; its tokenizer pads with '!')."""
        return CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=20,
                              hidden_act="gelu", projection_dim=1280, pad_token_id=0)

    @staticmethod
    def tiny(width=64, layers=2, heads=2, act="quick_gelu", projection_dim=0):
        return CLIPTextConfig(hidden_size=width, intermediate_size=4 * width, num_hidden_layers=layers,
                              num_attention_heads=heads, hidden_act=act, projection_dim=projection_dim)


def clip_param_specs(cfg: CLIPTextConfig):
    """[(name, shape)] of CLIPTextModel(WithProjection) in transformers' checkpoint naming."""
    C, F = cfg.hidden_size, cfg.intermediate_size
    s = [("text_model.embeddings.token_embedding.weight", (cfg.vocab_size, C)),
         ("text_model.embeddings.position_embedding.weight", (cfg.max_position_embeddings, C))]
    for i in range(cfg.num_hidden_layers):
        p = f"text_model.encoder.layers.{i}"
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s += [(f"{p}.self_attn.{n}.weight", (C, C)), (f"{p}.self_attn.{n}.bias", (C,))]
        s += [(f"{p}.layer_norm1.weight", (C,)), (f"{p}.layer_norm1.bias", (C,)),
              (f"{p}.mlp.fc1.weight", (F, C)), (f"{p}.mlp.fc1.bias", (F,)),
              (f"{p}.mlp.fc2.weight", (C, F)), (f"{p}.mlp.fc2.bias", (C,)),
              (f"{p}.layer_norm2.weight", (C,)), (f"{p}.layer_norm2.bias", (C,))]
    s += [("text_model.final_layer_norm.weight", (C,)), ("text_model.final_layer_norm.bias", (C,))]
    if cfg.projection_dim:
        s += [("text_projection.weight", (cfg.projection_dim, C))]
    return s


def make_clip_state_dict(cfg: CLIPTextConfig, seed: int = 0):
    """Random-init fp32 weights of the architecture (no checkpoints offline), seeded; CLIP-like scales
    (embeddings 0.02 / 0.01, linear std 1/sqrt(fan_in), LayerNorm affine near identity)."""
    g = torch.Generator().manual_seed(int(seed) + 7919)
    sd = {}
    for name, shape in clip_param_specs(cfg):
        if name.endswith("token_embedding.weight"):
            t = torch.randn(shape, generator=g) * 0.02
        elif name.endswith("position_embedding.weight"):
            t = torch.randn(shape, generator=g) * 0.01
        elif "layer_norm" in name and name.endswith("weight"):
            t = 1.0 + 0.05 * torch.randn(shape, generator=g)
        elif name.endswith("bias"):
            t = 0.02 * torch.randn(shape, generator=g)
        else:
            t = torch.randn(shape, generator=g) / shape[1] ** 0.5
        sd[name] = t
    return sd


class _ActFn:
    """transformers ACT2FN stand-in carrying the kernel activation code."""

    def __init__(self, name):
        self.name = name
        self.code = ops.ACT_BY_NAME[name]

    def __call__(self, x):
        if self.name == "quick_gelu":
            return x * torch.sigmoid(1.702 * x)
        return torch.nn.functional.gelu(x)

    def __repr__(self):
        return f"ACT2FN[{self.name!r}]"


class CLIPMLP(nn.Module):
    """transformers CLIPMLP: fc2(act(fc1(x))). Its forward runs only when no sdmoe receiver defers it."""

    def __init__(self, fc1, fc2, act):
        super().__init__()
        self.fc1 = fc1
        self.fc2 = fc2
        self.activation_fn = _ActFn(act)
        self._sdmoe_deferred = 0

    def hidden(self, x2d):
        """act(fc1(x)) [rows, F] (one GEMM, activation in the epilogue)."""
        return self.fc1.run(x2d, act=self.activation_fn.code)

    def run(self, x2d, residual=None, out=None, wmask=None):
        return self.fc2.run(self.hidden(x2d), residual=residual, out=out, wmask=wmask)

    def forward(self, hidden_states):
        if self._sdmoe_deferred and self._forward_hooks:
            return None  # a sdmoe receiver's text_hook_fn computes this module's output
        shp = hidden_states.shape
        return self.run(hidden_states.reshape(-1, shp[-1])).view(*shp)


class CLIPAttention(nn.Module):
    def __init__(self, q, k, v, o, heads):
        super().__init__()
        self.q_proj, self.k_proj, self.v_proj, self.out_proj = q, k, v, o
        self.num_heads = heads
        self._qkv_key = None
        self._qkv = None

    def fused_qkv(self):
        """[3C, C] weight / [3C] bias views built once (rebuilt if a projection's weights change)."""
        ps = (self.q_proj, self.k_proj, self.v_proj)
        key = tuple((p.weight.data_ptr(), p.weight._version, p.bias._version) for p in ps)
        if self._qkv_key != key:
            w = torch.cat([p.weight.data for p in ps], 0).contiguous()
            b = torch.cat([p.bias.data for p in ps], 0).contiguous()
            self._qkv = (w, b)
            self._qkv_key = key
        return self._qkv

    def run(self, h, nseq, L, residual, out):
        C = h.shape[1]
        w, b = self.fused_qkv()
        qkv = ops.linear(h, w, b)
        a = ops.attention_short(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], nseq, L, self.num_heads, causal=True)
        return self.out_proj.run(a, residual=residual, out=out)


class _LayerNorm(nn.Module):
    def __init__(self, w, b, eps):
        super().__init__()
        self.weight = _buf(w)
        self.bias = _buf(b)
        self.eps = eps

    def run(self, x, out=None):
        return ops.layernorm(x, self.weight, self.bias, self.eps, out=out)


class CLIPEncoderLayer(nn.Module):
    def __init__(self, self_attn, ln1, mlp, ln2):
        super().__init__()
        self.self_attn = self_attn
        self.layer_norm1 = ln1
        self.mlp = mlp
        self.layer_norm2 = ln2

    def run(self, x, scratch, out, nseq, L):
        """x -> out (out may be x; scratch must alias neither): x + attn(ln1 x) -> scratch; scratch + mlp(ln2 .)."""
        self.self_attn.run(self.layer_norm1.run(x), nseq, L, residual=x, out=scratch)
        h = self.layer_norm2.run(scratch)
        if self.mlp._forward_hooks:
            # reference hook seam: module(input) fires the registered text_hook_fn, whose return value replaces
            # the MLP output (the module itself is deferred by sdmoe receivers)
            C = h.shape[1]
            m = self.mlp(h.view(nseq, L, C)).reshape(-1, C)
            return _add_rows(scratch, m, out)
        return self.mlp.run(h, residual=scratch, out=out)


def _add_rows(a, b, out):
    """out = a + b on 2-D row views (contiguous temporaries when a view is strided)."""
    if a.is_contiguous() and b.is_contiguous() and out.is_contiguous():
        return ops.add(a, b, out=out)
    r = ops.add(a.contiguous(), b.contiguous())
    out.copy_(r)
    return out


class CLIPEncoder(nn.Module):
    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)


class CLIPTextEmbeddings(nn.Module):
    def __init__(self, tok, pos):
        super().__init__()
        self.token_embedding = nn.Module()
        self.token_embedding.weight = _buf(tok)
        self.position_embedding = nn.Module()
        self.position_embedding.weight = _buf(pos)


class CLIPTextTransformer(nn.Module):
    def __init__(self, embeddings, encoder, final_ln):
        super().__init__()
        self.embeddings = embeddings
        self.encoder = encoder
        self.final_layer_norm = final_ln


@dataclass
class CLIPTextOutput:
    last_hidden_state: torch.Tensor | None
    pooler_output: torch.Tensor | None = None
    text_embeds: torch.Tensor | None = None
    hidden_states: tuple | None = None

    def __getitem__(self, i):
        first = self.text_embeds if self.text_embeds is not None else self.last_hidden_state
        vals = (first, self.pooler_output if self.text_embeds is None else self.last_hidden_state)
        return vals[i]


class CLIPTextModel(nn.Module):
    """CLIPTextModel / CLIPTextModelWithProjection on the HIP kernels (weights fp16 on `device`)."""

    def __init__(self, cfg: CLIPTextConfig, transformer: CLIPTextTransformer, text_projection=None):
        super().__init__()
        self.config = cfg
        self.text_model = transformer
        if text_projection is not None:
            self.text_projection = text_projection

    @classmethod
    def from_state_dict(cls, sd, cfg: CLIPTextConfig, device="cuda"):
        def T(n):
            return sd[n].to(device=device, dtype=torch.float16).contiguous()

        def lin(p, bias=True):
            return LoRACompatibleLinear(T(p + ".weight"), T(p + ".bias") if bias else None)

        emb = CLIPTextEmbeddings(T("text_model.embeddings.token_embedding.weight"),
                                 T("text_model.embeddings.position_embedding.weight"))
        layers = []
        for i in range(cfg.num_hidden_layers):
            p = f"text_model.encoder.layers.{i}"
            a = CLIPAttention(*(lin(f"{p}.self_attn.{n}") for n in ("q_proj", "k_proj", "v_proj", "out_proj")),
                              cfg.num_attention_heads)
            ln1 = _LayerNorm(T(f"{p}.layer_norm1.weight"), T(f"{p}.layer_norm1.bias"), cfg.layer_norm_eps)
            ln2 = _LayerNorm(T(f"{p}.layer_norm2.weight"), T(f"{p}.layer_norm2.bias"), cfg.layer_norm_eps)
            mlp = CLIPMLP(lin(f"{p}.mlp.fc1"), lin(f"{p}.mlp.fc2"), cfg.hidden_act)
            layers.append(CLIPEncoderLayer(a, ln1, mlp, ln2))
        fln = _LayerNorm(T("text_model.final_layer_norm.weight"), T("text_model.final_layer_norm.bias"),
                         cfg.layer_norm_eps)
        proj = lin("text_projection", bias=False) if cfg.projection_dim else None
        return cls(cfg, CLIPTextTransformer(emb, CLIPEncoder(layers), fln), proj)

    @property
    def device(self):
        return self.text_model.embeddings.token_embedding.weight.device

    def eos_positions(self, ids: torch.Tensor) -> torch.Tensor:
        """Pooling position per sequence, as transformers' CLIPTextTransformer: argmax(ids) for the legacy
        eos_token_id == 2 configs, else the first position holding eos_token_id."""
        ids = ids.to("cpu", torch.int64)
        if self.config.eos_token_id == 2:
            return ids.argmax(-1)
        return (ids == self.config.eos_token_id).int().argmax(-1)

    def encode(self, input_ids, *, hidden_layer=-1, out=None, pooled=False):
        """Run the encoder on input_ids [nseq, L] (host or device ints).
        hidden_layer=-1: last_hidden_state (after final_layer_norm) -> out [nseq*L, C];
        hidden_layer=-2: hidden_states[-2] (penultimate layer output, no final LN; SDXL) -> out.
        pooled=True also returns pooler_output [nseq, C] (final-LN rows at the eos position) and, with a
        projection, text_embeds [nseq, projection_dim]. `out` may be a strided column slice of a wider buffer."""
        cfg = self.config
        tm = self.text_model
        ids = torch.as_tensor(input_ids)
        nseq, L = ids.shape
        if L > cfg.max_position_embeddings:
            raise ValueError(f"sequence length {L} exceeds max_position_embeddings {cfg.max_position_embeddings}")
        if hidden_layer not in (-1, -2):
            raise ValueError("hidden_layer must be -1 (last_hidden_state) or -2 (penultimate hidden states)")
        dev = self.device
        C = cfg.hidden_size
        M = nseq * L
        if out is None:
            out = torch.empty((M, C), dtype=torch.float16, device=dev)
        if out.shape != (M, C):
            raise ValueError(f"out: expected [{M}, {C}], got {tuple(out.shape)}")
        idx = ids.reshape(-1).to(dev, torch.int32).contiguous()
        pos = tm.embeddings.position_embedding.weight[:L]
        nl = cfg.num_hidden_layers
        # the stream lives in `out` itself when it is the penultimate state that is returned
        x = out if hidden_layer == -2 else torch.empty((M, C), dtype=torch.float16, device=dev)
        ops.gather_rows(tm.embeddings.token_embedding.weight, idx, add=pos, period=L, out=x)
        scratch = torch.empty((M, C), dtype=torch.float16, device=dev)
        run_last = hidden_layer == -1 or pooled
        for i, layer in enumerate(tm.encoder.layers):
            if i == nl - 1 and hidden_layer == -2:
                if not run_last:
                    break
                x2 = torch.empty((M, C), dtype=torch.float16, device=dev)
                layer.run(x, scratch, x2, nseq, L)
                x = x2
                continue
            layer.run(x, scratch, x, nseq, L)
        res = {"hidden": out}
        if hidden_layer == -1:
            tm.final_layer_norm.run(x, out=out)
        if pooled:
            rows = (torch.arange(nseq) * L + self.eos_positions(ids)).to(dev, torch.int32)
            g = ops.gather_rows(x, rows)
            pool = tm.final_layer_norm.run(g)
            res["pooled"] = pool
            if cfg.projection_dim:
                res["text_embeds"] = self.text_projection.run(pool)
        return res

    def forward(self, input_ids, attention_mask=None, output_hidden_states=False, **unused):
        """transformers-shaped call: [0] is last_hidden_state [nseq, L, C] (CLIPTextModel) or text_embeds
        (WithProjection); output_hidden_states=True returns hidden_states[-2] as the only materialised entry
        (hidden_states[-2] is what SDXL reads)."""
        if attention_mask is not None and not bool(torch.all(torch.as_tensor(attention_mask) != 0)):
            raise NotImplementedError("padding attention masks are not used by the SD text encoders")
        ids = torch.as_tensor(input_ids)
        nseq, L = ids.shape
        C = self.config.hidden_size
        r = self.encode(ids, hidden_layer=-1, pooled=True)
        hs = None
        if output_hidden_states:
            pen = self.encode(ids, hidden_layer=-2)["hidden"].view(nseq, L, C)
            hs = (None,) * (self.config.num_hidden_layers - 1) + (pen, r["hidden"].view(nseq, L, C))
        return CLIPTextOutput(r["hidden"].view(nseq, L, C), r["pooled"], r.get("text_embeds"), hs)


class SyntheticCLIPTokenizer:
    """Offline stand-in for transformers.CLIPTokenizer (no vocab.json / merges.txt here): lower-cased words and
    punctuation map to stable ids in [1, bos) by crc32; [bos] + tokens + [eos], truncated to model_max_length,
    padded with pad_token_id (49407 = eos for SD-1.x's tokenizer, 0 = '!' for SDXL's tokenizer_2)."""

    _pat = re.compile(r"[a-z]+|[0-9]|[^\sa-z0-9]+")

    def __init__(self, model_max_length=77, bos_token_id=49406, eos_token_id=49407, pad_token_id=49407):
        self.model_max_length = model_max_length
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        self.pad_token_id = pad_token_id

    def tokenize_ids(self, text):
        return [1 + zlib.crc32(w.encode("utf-8")) % (self.bos_token_id - 1)
                for w in self._pat.findall(text.lower())]

    def __call__(self, text, padding="max_length", max_length=None, truncation=True, return_tensors="pt"):
        texts = [text] if isinstance(text, str) else list(text)
        n = max_length or self.model_max_length
        rows = []
        for t in texts:
            ids = self.tokenize_ids(t)
            if truncation:
                ids = ids[:n - 2]
            ids = [self.bos_token_id] + ids + [self.eos_token_id]
            if padding == "max_length":
                ids = ids + [self.pad_token_id] * (n - len(ids))
            rows.append(ids)

        class _Enc:
            pass

        enc = _Enc()
        enc.input_ids = torch.tensor(rows, dtype=torch.int64)
        enc.attention_mask = (torch.arange(n)[None, :] < torch.tensor([[len(self.tokenize_ids(t)) + 2]
                                                                      for t in texts])).long()
        return enc


def text_encoder_configs(unet_cfg):
    """The text-encoder config(s) that feed a U-Net config: SD-1.x ViT-L (768), SDXL ViT-L + bigG (768 + 1280,
    pooled projection = the U-Net's pooled_dim); small U-Net test configs get narrow encoders of the same shape."""
    d = unet_cfg.cross_attention_dim
    if unet_cfg.addition_embed_type == "text_time":
        if d == 2048:
            return CLIPTextConfig.sdxl_l(), CLIPTextConfig.sdxl_g()
        h = d // 2
        return (CLIPTextConfig.tiny(h, 2, 1),
                CLIPTextConfig(hidden_size=d - h, intermediate_size=4 * (d - h), num_hidden_layers=3,
                               num_attention_heads=1, hidden_act="gelu", projection_dim=unet_cfg.pooled_dim,
                               pad_token_id=0))
    return (CLIPTextConfig.sd14() if d == 768 else CLIPTextConfig.tiny(d, 2, 2)), None


def attach_text_encoders(pipe, seed: int = 0):
    """Random-init text encoder(s) + synthetic tokenizer(s) on the pipeline's device (no checkpoints offline);
    returns the fp32 state dicts (the oracle's weights)."""
    c1, c2 = text_encoder_configs(pipe.config)
    sd1 = make_clip_state_dict(c1, seed)
    pipe.text_encoder = CLIPTextModel.from_state_dict(sd1, c1, pipe.device)
    pipe.tokenizer = SyntheticCLIPTokenizer(pad_token_id=c1.pad_token_id)
    sds = [sd1]
    if c2 is not None:
        sd2 = make_clip_state_dict(c2, seed + 1)
        pipe.text_encoder_2 = CLIPTextModel.from_state_dict(sd2, c2, pipe.device)
        pipe.tokenizer_2 = SyntheticCLIPTokenizer(pad_token_id=c2.pad_token_id)
        sds.append(sd2)
    return sds
