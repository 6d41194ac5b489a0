"""Generate golden vectors for the hot-path hooks by running the REFERENCE's own hook functions.

Runs only in the build container (the reference tree is not present on the GPU box): it imports the
reference receivers from /root/reference through a minimal stub of the absent `diffusers` package
(SURVEY §8c), calls them on seeded inputs, and writes small .npz fixtures next to this script.
Only data (inputs and outputs) is written; nothing of the reference's source is copied.

Covered reference functions:
  * MOEFy.hook_fn                        neuron_receivers/moefy.py:10-27
  * RemoveExperts.hook_fn (+ counter)    neuron_receivers/remove_skilled_experts.py:24-55, predictivity.py:25-39
  * WandaRemoveNeuronsFast.linear_hook_fn neuron_receivers/remove_wanda_neurons_fast.py:69-83, with the real
    Wanda masks of weights_320_1280.csv (the reference's only mask fixture)
  * helper.modify_ffn                    moefication/helper.py:48-62 (labels -> patterns, k)
  * GetExperts.hook_fn                   neuron_receivers/get_experts.py:50-83 (token-mean expert top-k, bboxes)
  * Wanda.hook_fn + TimeLayerColumnNorm  neuron_receivers/wanda_receiver.py:37-57, utils.py:321-370

usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [name-prefix ...]
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import pickle
import sys
import tempfile
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

REF = os.environ.get("SDMOE_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)
import synth  # noqa: E402
from synth import balanced_labels  # noqa: E402


# --------------------------------------------------------------------------------------------- stubs
class LoRACompatibleLinear(nn.Linear):
    """Stand-in with the diffusers-0.27 call signature forward(x, scale=1.0) used by the hooks."""

    def forward(self, x, scale=1.0):  # noqa: D401
        return F.linear(x, self.weight, self.bias)


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = LoRACompatibleLinear(dim_in, dim_out * 2)

    def gelu(self, gate):
        return F.gelu(gate)

    def forward(self, x, scale=1.0):
        h, g = self.proj(x).chunk(2, dim=-1)
        return h * self.gelu(g)


class GELU(nn.Module):
    pass


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Anything:
        def __init__(self, *a, **k):
            pass

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise RuntimeError("no checkpoints offline")

    names = ["AutoPipelineForText2Image", "StableDiffusionPipeline", "UNet2DConditionModel", "PixArtAlphaPipeline",
             "DiffusionPipeline", "LCMScheduler", "EulerDiscreteScheduler", "DPMSolverMultistepScheduler"]
    mod("diffusers", **{n: _Anything for n in names})
    mod("diffusers.models")
    mod("diffusers.models.activations", GEGLU=GEGLU, GELU=GELU, LoRACompatibleLinear=LoRACompatibleLinear)
    mod("diffusers.pipelines")
    sc = types.SimpleNamespace(StableDiffusionSafetyChecker=type("StableDiffusionSafetyChecker", (), {}))
    mod("diffusers.pipelines.stable_diffusion", safety_checker=sc)
    mod("diffusers.pipelines.stable_diffusion_safe", SafetyConfig=_Anything)
    mod("sld", SLDPipeline=_Anything)
    mod("cv2")
    # load the receiver modules from their files without running neuron_receivers/__init__.py
    pkg = types.ModuleType("neuron_receivers")
    pkg.__path__ = [os.path.join(REF, "neuron_receivers")]
    sys.modules["neuron_receivers"] = pkg
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "sparsity"))


def load_ref(modname, relpath):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
    m = importlib.util.module_from_spec(spec)
    sys.modules[modname] = m
    spec.loader.exec_module(m)
    return m


# --------------------------------------------------------------------------------------------- helpers
def make_geglu(C, seed, dtype, gate_bias=0.0):
    m = GEGLU(C, 4 * C)
    w, b = synth.geglu_weights(C, seed, gate_bias)
    with torch.no_grad():
        m.proj.weight.copy_(torch.from_numpy(w))
        m.proj.bias.copy_(torch.from_numpy(b))
    return m.to(dtype)


def sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().float().numpy()).tobytes()).hexdigest()[:16]


def topk_tie_flags(score, k):
    """True where the k-th and (k+1)-th largest fp scores are equal (tie at the selection boundary)."""
    s = score.float()
    if k >= s.shape[-1] or k == 0:
        return torch.zeros(s.shape[0], dtype=torch.bool)
    v = torch.sort(s, dim=-1, descending=True).values
    return v[:, k - 1] == v[:, k]


def quiet(fn, *a, **k):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


# --------------------------------------------------------------------------------------------- cases
def gen_moefy(helper, moefy_mod):
    cases = []
    spec = [  # (C, rows_per_image, topk, act, dtype)
        (320, 32, 0.2, "gelu", torch.float32),
        (320, 32, 0.2, "gelu", torch.float16),
        (320, 32, 0.2, "relu", torch.float16),
        (320, 32, 1.0, "gelu", torch.float16),
        (640, 16, 0.2, "gelu", torch.float16),
        (640, 16, 0.2, "relu", torch.float32),
        (1280, 8, 0.2, "gelu", torch.float16),
        (1280, 8, 0.2, "relu", torch.float16),
    ]
    for i, (C, N, topk, act, dtype) in enumerate(spec):
        seed = 1000 + i
        E = 4 * C // 20
        labels = balanced_labels(4 * C, E, seed)
        m = make_geglu(C, seed, dtype)
        if act == "relu":
            m.gelu = F.relu  # sparsity/relufy_model.py:8-15,35
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "labels")
            torch.save(list(map(int, labels)), path)
            quiet(helper.modify_ffn, m, path, topk)  # reference helper: patterns [E,4C], k = int(E*topk)
        x = torch.from_numpy(synth.tokens((2, N, C), seed + 1)).to(dtype)
        rec = moefy_mod.MOEFy(seed=0)
        with torch.no_grad():
            out = rec.hook_fn(m, (x,), None)
            gate = rec.gates[-1]
            y = m.proj(x)
            gact = m.gelu(y.chunk(2, -1)[1])
            score = torch.matmul(gact.reshape(-1, 4 * C), m.patterns.t())
            sel = torch.topk(score, k=m.k, dim=-1)[1]
        cases.append(dict(
            name=f"moefy_C{C}_N{N}_k{topk}_{act}_{str(dtype).split('.')[-1]}", kind="moefy", C=C, act=act,
            dtype=str(dtype).split(".")[-1], topk=topk, k=m.k, E=E, labels=labels, x=x.numpy(),
            seed=seed, w_sha=sha(m.proj.weight), y=y.numpy(), out=out.numpy(),
            gate=gate.numpy(), score=score.numpy(), sel=sel.numpy(), tie=topk_tie_flags(score, m.k).numpy(),
            patterns_sha=sha(m.patterns)))
    return cases


def gen_remove_experts(helper, rem_mod):
    cases = []
    spec = [  # (C, N, act, gate_bias, dtype)
        (320, 32, "gelu", 0.0, torch.float16),
        (320, 32, "gelu", -1.5, torch.float16),  # mostly negative expert scores: removed experts (score 0) win slots
        (640, 16, "relu", 0.0, torch.float16),
        (320, 32, "gelu", -1.5, torch.float32),
        (1280, 8, "relu", 0.0, torch.float16),   # E = 256, k = 51 (the 16x16 / 8x8 levels)
        (1280, 8, "gelu", -1.0, torch.float16),
    ]
    for i, (C, N, act, gb, dtype) in enumerate(spec):
        seed = 2000 + i
        E = 4 * C // 20
        labels = balanced_labels(4 * C, E, seed)
        m = make_geglu(C, seed, dtype, gate_bias=gb)
        if act == "relu":
            m.gelu = F.relu
        rng = np.random.default_rng(seed)
        T, L = 22, 2
        lists = {(t, l): sorted(rng.choice(E, size=max(1, E // 10), replace=False).tolist()) for t in range(T)
                 for l in range(L)}
        lists[(1, 0)] = []  # empty list -> patterns unchanged
        x = torch.from_numpy(synth.tokens((2, N, C), seed + 1)).to(dtype)
        with tempfile.TemporaryDirectory() as d:
            lp = os.path.join(d, "labels")
            torch.save(list(map(int, labels)), lp)
            quiet(helper.modify_ffn, m, lp, 0.2)
            for (t, l), ids in lists.items():
                with open(os.path.join(d, f"timestep_{t}_layer_{l}.json"), "w") as f:
                    json.dump(ids, f)
            rec = quiet(rem_mod.RemoveExperts, 0, d, T, L)
        outs, gates, tl = [], [], []
        with torch.no_grad():
            y = m.proj(x)
            for call in range(T * L):
                tl.append((rec.timestep, rec.layer))
                outs.append(rec.hook_fn(m, (x,), None).numpy())
                gates.append(rec.gates[-1].numpy())
        keep_calls = [0, 1, 2, 3, 38, 39, 40, 41, 42, 43]  # t=0,1 (removal), t=19 (last removal), t=20,21 (none)
        cases.append(dict(
            name=f"remove_C{C}_{act}_gb{gb}_{str(dtype).split('.')[-1]}", kind="remove", C=C, act=act,
            dtype=str(dtype).split(".")[-1], k=m.k, E=E, T=T, L=L, labels=labels, x=x.numpy(),
            seed=seed, gate_bias=gb, w_sha=sha(m.proj.weight), y=y.numpy(),
            lists=json.dumps({f"{t},{l}": v for (t, l), v in lists.items()}),
            calls=np.array(keep_calls), call_tl=np.array([tl[c] for c in keep_calls]),
            out=np.stack([outs[c] for c in keep_calls]), gate=np.stack([gates[c] for c in keep_calls])))
    return cases


def gen_wanda(wanda_mod):
    import scipy.sparse
    csv = np.loadtxt(os.path.join(REF, "weights_320_1280.csv"), delimiter=",", skiprows=1, dtype=np.int64)
    with open(os.path.join(REF, "weights_320_1280.csv")) as f:
        header = f.readline().strip().split(",")
    masks = csv.T.reshape(len(header), 320, 1280)  # flattened row-major [320, 1280] per column
    cases = []
    with tempfile.TemporaryDirectory() as d:
        for l in range(len(header)):
            with open(os.path.join(d, f"timestep_0_layer_{l}.pkl"), "wb") as f:
                pickle.dump(scipy.sparse.csr_matrix(masks[l]), f)
        rec = quiet(wanda_mod.WandaRemoveNeuronsFast, 0, d, 1, len(header))
        for dtype in (torch.float32, torch.float16):
            rec.reset_time_layer()
            lin = LoRACompatibleLinear(1280, 320)
            w, b = synth.down_weights(320, 3000)
            with torch.no_grad():
                lin.weight.copy_(torch.from_numpy(w))
                lin.bias.copy_(torch.from_numpy(b))
            lin = lin.to(dtype)
            x = torch.from_numpy(synth.tokens((2, 16, 1280), 3001)).to(dtype)
            outs = []
            with torch.no_grad():
                for l in range(len(header)):
                    y = lin(x)
                    outs.append(rec.linear_hook_fn(lin, (x,), y).numpy())
            cases.append(dict(
                name=f"wanda_320x1280_{str(dtype).split('.')[-1]}", kind="wanda", dtype=str(dtype).split(".")[-1],
                header=json.dumps(header), mask_bits=np.packbits(masks.astype(np.uint8), axis=-1, bitorder="little"),
                x=x.numpy(), w_seed=3000, w_sha=sha(lin.weight), out=np.stack(outs),
                density=masks.reshape(len(header), -1).mean(1)))
    return cases


def gen_counter(pred_mod):
    rec = quiet(pred_mod.NeuronPredictivity, 0, 51, 16)
    seq = []
    for _ in range(16 * 51):
        seq.append((rec.timestep, rec.layer))
        rec.update_time_layer()
    seq.append((rec.timestep, rec.layer))
    rec.reset_time_layer()
    return [dict(name="counter_T51_L16", kind="counter", seq=np.array(seq), after_reset=np.array([rec.timestep,
                                                                                                rec.layer]))]


def gen_get_experts(helper, ge_mod):
    cases = []
    spec = [  # (C, N, topk, act, dtype, bbox)
        (320, 32, 0.2, "gelu", torch.float32, None),
        (320, 32, 0.2, "gelu", torch.float16, None),
        (640, 16, 0.2, "relu", torch.float16, None),
        (320, 32, 0.2, "gelu", torch.float16, [0, 3, 5, 17, 31]),
        (1280, 8, 0.2, "gelu", torch.float32, [1, 2, 6]),
    ]
    for i, (C, N, topk, act, dtype, bb) in enumerate(spec):
        seed = 4000 + i
        E = 4 * C // 20
        labels = balanced_labels(4 * C, E, seed)
        m = make_geglu(C, seed, dtype)
        if act == "relu":
            m.gelu = F.relu
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "labels")
            torch.save(list(map(int, labels)), path)
            quiet(helper.modify_ffn, m, path, topk)
        m.bounding_box = bb
        x = torch.from_numpy(synth.tokens((2, N, C), seed + 1)).to(dtype)
        name = "ffn0"
        rec = quiet(ge_mod.GetExperts, 0, 1, 16, {name: E}, [name] * 16)
        with torch.no_grad():
            out = rec.hook_fn(m, (x,), None)
            h, g = m.proj(x).chunk(2, -1)
            g = m.gelu(g)
            gb = g if bb is None else g[:, bb, :]
            mean = torch.matmul(gb.reshape(-1, 4 * C), m.patterns.t()).mean(0)
        sel = rec.label_counter[0][0]
        s = torch.sort(mean.float(), descending=True).values
        tie = bool(m.k < E and s[m.k - 1] == s[m.k])
        cases.append(dict(
            name=f"getexperts_C{C}_N{N}_{act}_{str(dtype).split('.')[-1]}{'_bb' if bb else ''}", kind="getexperts",
            C=C, act=act, dtype=str(dtype).split(".")[-1], k=m.k, E=E, labels=labels, x=x.numpy(), seed=seed,
            bb=np.array(bb if bb else [], dtype=np.int64), out=out.numpy(), sel=np.array(sel, dtype=np.int64),
            mean=mean.numpy(), tie=tie, counter_after=np.array([rec.timestep, rec.layer])))
    return cases


def gen_wanda_receiver(w_mod):
    cases = []
    for dtype in (torch.float32, torch.float16):
        C, N, T, L = 320, 16, 2, 2
        rec = quiet(w_mod.Wanda, 0, T, L)
        mods = [make_geglu(C, 5000 + l, dtype) for l in range(L)]
        xs = []
        with torch.no_grad():
            for call in range(T * L * 2):  # two "prompts": the statistic accumulates across them
                if call == T * L:
                    rec.reset_time_layer()
                x = torch.from_numpy(synth.tokens((2, N, C), 5100 + call)).to(dtype)
                xs.append(x.numpy())
                rec.hook_fn(mods[call % L], (x,), None)
        norms = rec.predictivity.get_column_norms()
        cases.append(dict(
            name=f"wanda_colnorm_C{C}_{str(dtype).split('.')[-1]}", kind="wanda_colnorm", C=C, T=T, L=L,
            dtype=str(dtype).split(".")[-1], x=np.stack(xs), w_seeds=np.array([5000 + l for l in range(L)]),
            norms=np.stack([np.stack([norms[t][l].float().numpy() for l in range(L)]) for t in range(T)])))
    return cases


def save(cases, only=None):
    """Write the cases (only those whose name starts with one of `only`, if given) and merge index.json."""
    index = []
    ipath = os.path.join(OUT, "index.json")
    if only and os.path.exists(ipath):
        with open(ipath) as f:
            index = list(json.load(f)["cases"])
    for c in cases:
        if only and not any(c["name"].startswith(o) for o in only):
            continue
        name = c.pop("name")
        arrays = {}
        for k, v in c.items():
            if isinstance(v, np.ndarray):
                arrays[k] = v
            else:
                arrays[k] = np.array(v)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
        if name not in index:
            index.append(name)
    with open(os.path.join(OUT, "index.json"), "w") as f:
        json.dump({"cases": index, "generator": "tests/golden/make_golden.py", "reference": "ruchikachavhan/"
                   "diffusion-models-moe @ 2024-10-08", "torch": torch.__version__}, f, indent=1)


def main():
    install_stubs()
    helper = load_ref("moefication_helper_ref", "moefication/helper.py")
    load_ref("neuron_receivers.base_receiver", "neuron_receivers/base_receiver.py")
    pred = load_ref("neuron_receivers.predictivity", "neuron_receivers/predictivity.py")
    moefy = load_ref("neuron_receivers.moefy", "neuron_receivers/moefy.py")
    rem = load_ref("neuron_receivers.remove_skilled_experts", "neuron_receivers/remove_skilled_experts.py")
    wanda = load_ref("neuron_receivers.remove_wanda_neurons_fast", "neuron_receivers/remove_wanda_neurons_fast.py")
    ge = load_ref("neuron_receivers.get_experts", "neuron_receivers/get_experts.py")
    load_ref("utils", "utils.py")
    wr = load_ref("neuron_receivers.wanda_receiver", "neuron_receivers/wanda_receiver.py")
    cases = gen_moefy(helper, moefy) + gen_remove_experts(helper, rem) + gen_wanda(wanda) + gen_counter(pred)
    cases += gen_get_experts(helper, ge) + gen_wanda_receiver(wr)
    only = sys.argv[1:] or None  # optional name prefixes: regenerate just those fixtures
    save(cases, only)
    print(f"wrote {'all' if only is None else only} golden cases to {OUT}")


if __name__ == "__main__":
    main()
