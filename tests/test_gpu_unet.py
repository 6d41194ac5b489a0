"""U-Net / pipeline / receiver parity on the MI355X vs the fp32 CPU oracle (oracle/unet_ref.py).

The oracle gets the same fp16-rounded weights, so differences come only from fp16 activations and fp32
accumulation order. Tolerances:
  * one U-Net evaluation, no routing: max|eps - ref| <= 3e-2 * max(1, max|ref|);
  * multi-step denoising with MoE routing: relative L2 of the final latents <= 3e-2 (an fp16 near-tie can
    flip one token's expert choice vs the fp32 oracle, which max-abs would over-weight).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe.config import UNetConfig  # noqa: E402
from sdmoe.unet import UNet2DConditionModel  # noqa: E402
from sdmoe.weights import make_state_dict  # noqa: E402
from sdmoe.pipeline import StableDiffusionPipeline, prompt_embedding, initial_latents  # noqa: E402
from oracle.unet_ref import UNetRef, denoise  # noqa: E402
from oracle import hooks_ref as H  # noqa: E402

DEV = "cuda"


def rel_l2(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


def max_rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return (a - b).abs().max().item() / max(1.0, b.abs().max().item())


def build(cfg, seed=0):
    sd = make_state_dict(cfg, seed)
    sd16 = {k: v.half().float() for k, v in sd.items()}
    return UNet2DConditionModel.from_state_dict(sd, cfg, DEV), UNetRef(sd16, cfg)


@pytest.fixture(scope="module")
def tiny():
    cfg = UNetConfig.tiny(16)
    return (cfg,) + build(cfg)


def ctx_for(cfg, prompts):
    d = cfg.cross_attention_dim
    return torch.stack([prompt_embedding("", d)] * len(prompts) + [prompt_embedding(p, d) for p in prompts])


def test_unet_forward_tiny(tiny):
    cfg, unet, ref = tiny
    moefy_tiny(StableDiffusionPipeline(unet, DEV), topk=None)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 16, 16, generator=g)
    ctx = ctx_for(cfg, ["a photo of a cat"])
    for t in (981.0, 501.0, 1.0):
        eps = unet(x.to(DEV), t, ctx.to(DEV))
        r = ref(x, t, ctx)
        assert max_rel(eps, r) <= 3e-2, t


def test_unet_forward_sd14_32x32():
    cfg = UNetConfig.sd14(32)
    unet, ref = build(cfg, seed=3)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 4, 32, 32, generator=g)
    ctx = ctx_for(cfg, ["Starry night by Van Gogh"])
    eps = unet(x.to(DEV), 741.0, ctx.to(DEV))
    r = ref(x, 741.0, ctx)
    assert max_rel(eps, r) <= 3e-2
    assert 0.1 < r.std().item() < 10  # synthetic weights stay numerically tame
    del unet


def moefy_tiny(pipe, topk=0.25, expert_size=16, relu=True):
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from sdmoe.unet import GEGLU, _gelu
    if topk is not None:
        moefy_synthetic(pipe, topk, expert_size, seed=5)
    for _, m in pipe.unet.named_modules():
        if isinstance(m, GEGLU):
            m.gelu = _gelu
            if topk is None:
                m.patterns = None
    if topk is None:
        return None
    if relu:
        find_and_change_geglu(pipe.unet)
    mods = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    return [(m.labels.numpy(), m.patterns.shape[0], m.k) for m in mods]


def oracle_ff_hook_factory(layers, act, removed=None):
    """The reference hook as it runs inside an fp16 pipeline (moefy.py:10-27 on fp16 tensors): projection,
    activation, expert scores and top-k in fp16, so routing decisions are made at fp16 resolution like the
    GPU's; the oracle's U-Net trunk stays fp32."""
    def factory(step):
        def hook(layer, x, w, b):
            labels, E, k = layers[layer]
            P = H.patterns_from_labels(labels, torch.float16)
            ids = removed[step][layer] if removed is not None else None
            out, *_ = H.geglu_hook(x.half(), w.half(), b.half(), P, k, act, removed=ids, apply_removal=step < 20)
            return out.float()
        return hook
    return factory


def sel_bits_to_bool(bits, E):
    import numpy as np
    b = bits.cpu().numpy().view(np.uint32)
    e = np.arange(E)
    return torch.from_numpy(((b[:, e >> 5] >> (e & 31)) & 1).astype(bool))


def recording(cls):
    """Receiver subclass that records every hooked call's device top-k selection (sdmoe_geglu_route sel_out)."""
    class Rec(cls):
        def hook_fn(self, module, input, output):
            x = input[0]
            E = module.patterns.shape[0]
            sel = torch.zeros((x.numel() // x.shape[-1], (E + 31) // 32), dtype=torch.int32, device=x.device)
            removed = None
            if hasattr(self, "removed_for"):
                removed = self.removed_for(module, self.timestep, self.layer)
                self.update_time_layer()
            out, gate = module.routed(x, removed=removed, want_gate=self.store_gates, sel_out=sel)
            if self.store_gates:
                self.gates.append(gate.cpu())
            self.sels.append(sel_bits_to_bool(sel, E))
            return out
        _sdmoe_ln_safe_hook = hook_fn  # only hands input[0] to routed(): the folded norm3 path stays on
    return Rec


def forced_factory(layers, act, sels, removed=None, stats=None, margin=16):
    """Oracle hook (fp16 arithmetic, as in the reference's fp16 pipeline) that checks its own top-k against
    the device's on every row clear of an fp16 near-tie, then uses the device's selection (teacher forcing).
    A row is clear when its k-th/(k+1)-th score gap exceeds `margin` fp16 ulps: the hook's INPUT comes from the
    oracle's fp32 trunk while the device's comes from its fp16 trunk, so the margin has to cover the trunk's
    propagated rounding noise (deeper stacks need more); stats["max_mismatch_gap_ulps"] records the largest gap of
    any row whose selections differ."""
    import numpy as np

    def factory(step):
        def hook(layer, x, w, b):
            labels, E, k = layers[layer]
            P = H.patterns_from_labels(labels, torch.float16)
            ids = removed[step][layer] if removed is not None else None
            y = torch.nn.functional.linear(x.half(), w.half(), b.half())
            _, _, sel_o, score = H.routed_geglu(y, P, k, act, ids, step < 20)
            dev_sel = sels[step * len(layers) + layer]
            s = np.sort(score.float().numpy(), axis=1)[:, ::-1]
            gap = s[:, k - 1] - s[:, k] if k < E else np.full(s.shape[0], np.inf)
            ulp = np.spacing(np.abs(s[:, min(k, E - 1)]).astype(np.float16)).astype(np.float32)
            clear = gap > margin * ulp
            mism = (sel_o.numpy() != dev_sel.numpy()).any(1)
            if stats is not None:
                if mism.any():
                    g = float(np.max(gap[mism] / ulp[mism]))
                    stats["max_mismatch_gap_ulps"] = max(stats.get("max_mismatch_gap_ulps", 0.0), g)
                stats["rows"] += clear.size
                stats["clear"] += int(clear.sum())
                stats["clear_mismatch"] += int((mism & clear).sum())
                stats["forced"] += int(mism.sum())
            return H.routed_geglu_given_selection(y, P, dev_sel, act, ids, step < 20).float()
        return hook
    return factory


def run_oracle(ref, cfg, prompts, steps, seed=0, **kw):
    lat = torch.cat([initial_latents(seed, i, cfg) for i in range(len(prompts))])
    d = cfg.cross_attention_dim
    cu = torch.stack([prompt_embedding("", d)] * len(prompts))
    cc = torch.stack([prompt_embedding(p, d) for p in prompts])
    return denoise(ref, lat, cu, cc, num_inference_steps=steps, **kw)


def test_pipeline_moefy_receiver_tiny(tiny):
    """MOEFy through observe_activation, batch of 2 prompts, 3 DDIM steps with CFG, vs the oracle pipeline:
    the device's expert selection equals the oracle's on every row clear of an fp16 near-tie, and with the
    near-tie rows teacher-forced the final latents agree to rel L2 <= 1e-2 (dense pipeline: ~4e-3)."""
    from neuron_receivers import MOEFy
    cfg, unet, ref = tiny
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=3)
    layers = moefy_tiny(pipe, relu=False)
    rec = recording(MOEFy)(seed=0)
    rec.sels = []
    prompts = ["a dog", "a painting of a river"]
    out, gates = rec.observe_activation(pipe, prompts)
    assert len(gates) == 3 * 16 and tuple(gates[0].shape) == (4, 256, 256)
    stats = dict(rows=0, clear=0, clear_mismatch=0, forced=0)
    exp = run_oracle(ref, cfg, prompts, 3, ff_hook_factory=forced_factory(layers, "gelu", rec.sels, stats=stats))
    assert stats["clear_mismatch"] == 0, stats
    assert stats["clear"] > 0.5 * stats["rows"], stats
    assert rel_l2(torch.stack(out), exp) <= 1e-2


class _Recorder:
    """MOEFy subclass factory that records every hook call's input and returned output."""

    @staticmethod
    def make():
        from neuron_receivers import MOEFy

        class Rec(MOEFy):
            def __init__(self):
                super().__init__(seed=0, store_gates=True)
                self.calls = []

            def hook_fn(self, module, input, output):
                out = super().hook_fn(module, input, output)
                self.calls.append((module, input[0].detach().float().cpu(), out.detach().float().cpu(),
                                   self.gates[-1]))
                return out
        return Rec()


def test_hook_level_parity_relu_tiny(tiny):
    """Every hooked GEGLU call of a relufied MoE pipeline step, re-run by the oracle's fp16 hook on the SAME
    input: gates >= 0, top-k count respected, and expert selection identical on rows clear of fp16 near-ties."""
    import numpy as np
    cfg, unet, ref = tiny
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=1)
    layers = moefy_tiny(pipe, relu=True)
    rec = _Recorder.make()
    rec.observe_activation(pipe, ["a dog", "a cat"])
    assert len(rec.calls) == 16
    n_clear = n_rows = 0
    for li, (module, x, out, gate) in enumerate(rec.calls):
        labels, E, k = layers[li]
        assert bool(torch.all(gate >= 0)), li
        w, b = module.proj.weight.detach().cpu(), module.proj.bias.detach().cpu()
        P = H.patterns_from_labels(labels, torch.float16)
        o_ref, g_ref, sel_ref, score = H.geglu_hook(x.half(), w, b, P, k, "relu")
        s = np.sort(score.float().numpy(), axis=1)[:, ::-1]
        gap = s[:, k - 1] - s[:, k]
        clear = gap > 8 * np.spacing(np.abs(s[:, k - 1]).astype(np.float16)).astype(np.float32) + 1e-3
        g2 = gate.reshape(-1, gate.shape[-1]).float()
        lab = torch.from_numpy(labels)
        active = torch.zeros(g2.shape[0], E).index_add_(1, lab, (g2 != 0).float()) > 0
        assert int(active.sum(1).max()) <= k
        sel_ref_np = sel_ref.numpy()
        # experts active on our side must be selected by the reference on clear rows
        assert np.all(~active.numpy()[clear] | sel_ref_np[clear])
        err = (out.reshape(-1, out.shape[-1]) - o_ref.float().reshape(-1, out.shape[-1])).abs()
        scale = max(1.0, o_ref.float().abs().max().item())
        assert err[torch.from_numpy(clear)].max().item() <= 3e-2 * scale
        n_clear += int(clear.sum())
        n_rows += clear.size
    assert n_clear > 0.5 * n_rows


def test_pipeline_remove_experts_receiver_tiny(tiny):
    """RemoveExperts (lists for every (t, l), removal active at t < 20) through observe_activation vs the oracle,
    same selection/teacher-forcing contract as the MOEFy test."""
    from neuron_receivers import GEGLU, RemoveExperts
    cfg, unet, ref = tiny
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=3)
    layers = moefy_tiny(pipe, relu=False)
    g = torch.Generator().manual_seed(9)
    T, L = 3, 16
    lists = {t: {l: sorted(torch.randperm(layers[l][1], generator=g)[:max(1, layers[l][1] // 4)].tolist())
                 for l in range(L)} for t in range(T)}
    rec = recording(RemoveExperts)(0, None, T, L, replace_fn=GEGLU, expert_indices=lists, store_gates=False)
    rec.sels = []
    out, gates = rec.observe_activation(pipe, ["a church"])
    assert gates == [] and (rec.timestep, rec.layer) == (3, 0)
    # removed experts may be selected (score 0) but never unmask: checked inside the oracle contract below
    stats = dict(rows=0, clear=0, clear_mismatch=0, forced=0)
    exp = run_oracle(ref, cfg, ["a church"], 3, ff_hook_factory=forced_factory(layers, "gelu", rec.sels, lists, stats))
    assert stats["clear_mismatch"] == 0, stats
    assert rel_l2(out[0], exp[0]) <= 1e-2


def test_pipeline_wanda_union_receiver_tiny(tiny):
    import numpy as np
    from neuron_receivers import WandaRemoveNeuronsFast, MultiConceptRemoverWanda
    cfg, unet, ref = tiny
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    moefy_tiny(pipe, topk=None)
    downs = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.2")]
    T, L = 2, 16
    rng = np.random.default_rng(0)
    concepts = {}
    for c in ("church", "parachute"):
        concepts[c] = {t: {l: (rng.random(tuple(downs[l].weight.shape)) < 0.03).astype(np.int64) for l in range(L)}
                       for t in range(T)}
    removers = {c: WandaRemoveNeuronsFast(0, None, T, L, masks=m, store_gates=False) for c, m in concepts.items()}
    mc = MultiConceptRemoverWanda(None, 0, T, L, concepts_to_remove=list(concepts), removers=removers)
    mc.handle_multiple_concepts(list(concepts))
    union = {t: {l: H.union_masks([concepts[c][t][l] for c in concepts]) for l in range(L)} for t in range(T)}
    for t in range(T):
        for l in range(L):
            assert np.array_equal(mc.union_neuron_remover.dense_mask(t, l), union[t][l])
    u = mc.union_neuron_remover
    u.reset_time_layer()
    out, _ = u.observe_activation(pipe, "a parachute over a church")

    def down_factory(step):
        def hook(layer, x, w, b):
            return H.wanda_linear(x, w, b, union[step][layer])
        return hook
    exp = run_oracle(ref, cfg, ["a parachute over a church"], 2, down_hook_factory=down_factory)
    assert rel_l2(out, exp[0]) <= 3e-2


@pytest.mark.parametrize("receiver", ["moefy", "remove"])
def test_pipeline_fused_geglu_sd14(receiver):
    """SD-1.4 widths (F = 1280/2560/5120, balanced 20-neuron experts): fused projection+GEGLU+score path vs
    the unfused proj GEMM + route kernel. Per call the two are bit-identical (test_gpu_route_parity); the down
    projection then sums the permuted neurons in another fp32 order, so with top-k = all experts (no
    near-tie can flip a choice) one U-Net evaluation agrees to rel L2 <= 2e-3 and a 2-step CFG 7.5 pipeline
    (which amplifies fp16 noise ~7.5x per step) to <= 2e-2. The removal variant zeroes fixed experts,
    exercising the removed-bit path through the permutation."""
    from moefication.helper import moefy_synthetic
    from neuron_receivers import MOEFy, RemoveExperts
    import sdmoe.unet as U
    cfg = UNetConfig.sd14(16)
    unet = UNet2DConditionModel.from_state_dict(make_state_dict(cfg, 4), cfg, DEV)
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    moefy_synthetic(pipe, 1.0, 20, seed=1)
    if receiver == "moefy":
        make = lambda: MOEFy(seed=0, store_gates=False)  # noqa: E731
    else:
        lists = {t: {l: list(range(l % 5, 64, 7)) for l in range(16)} for t in range(51)}
        make = lambda: RemoveExperts(0, None, T=51, n_layers=16, store_gates=False,  # noqa: E731
                                     expert_indices=lists)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 4, 16, 16, generator=g).to(DEV)
    ctx = ctx_for(cfg, ["Starry night by Van Gogh"]).to(DEV)
    evals, outs = [], []
    for fused in (True, False):
        U.FUSED_GEGLU = fused
        try:
            rec = make()
            if hasattr(rec, "prepare"):
                rec.prepare(pipe)
            hooks = rec.register_hooks(pipe)
            try:
                evals.append(unet(x, 741.0, ctx))
            finally:
                rec.remove_hooks(hooks)
            out, _ = make().observe_activation(pipe, ["a cat", "Starry night by Van Gogh"])
        finally:
            U.FUSED_GEGLU = True
        outs.append(torch.stack(out))
    assert torch.isfinite(outs[0]).all()
    assert rel_l2(evals[0], evals[1]) <= 2e-3
    assert rel_l2(outs[0], outs[1]) <= 2e-2
    ffs = [m for n, m in unet.named_modules() if n.endswith(".ff")]
    assert ffs and all(f._wperm is not None for f in ffs)  # the fused path actually ran


def test_pipeline_keep_mask_bit_identical_sd14():
    """Fused path with the top-k mask applied inside the down projection (sdmoe_linear_keep) vs the mask pass over
    the product (sdmoe_moe_topk_mask): the down projection sees identical operands, so a U-Net evaluation and a
    2-step RemoveExperts pipeline (top-k 0.2, removals active) are bit-identical."""
    from moefication.helper import moefy_synthetic
    from neuron_receivers import RemoveExperts
    import sdmoe.unet as U
    cfg = UNetConfig.sd14(16)
    unet = UNet2DConditionModel.from_state_dict(make_state_dict(cfg, 5), cfg, DEV)
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    moefy_synthetic(pipe, 0.2, 20, seed=3)
    lists = {t: {l: list(range(l % 5, 64, 7)) for l in range(16)} for t in range(51)}
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 4, 16, 16, generator=g).to(DEV)
    ctx = ctx_for(cfg, ["Starry night by Van Gogh"]).to(DEV)
    geglus = [m for n, m in unet.named_modules() if n.endswith("ff.net.0")]
    evals, outs, ran = [], [], []
    for keep in (True, False):
        U.FUSED_KEEP = keep
        try:
            rec = RemoveExperts(0, None, T=51, n_layers=16, store_gates=False, expert_indices=lists)
            rec.prepare(pipe)
            hooks = rec.register_hooks(pipe)
            try:
                evals.append(unet(x, 741.0, ctx))
            finally:
                rec.remove_hooks(hooks)
            ran.append(all(m._out_keep is not None for m in geglus))
            out, _ = RemoveExperts(0, None, T=51, n_layers=16, store_gates=False,
                                   expert_indices=lists).observe_activation(pipe, ["a cat", "Starry night"])
        finally:
            U.FUSED_KEEP = True
        outs.append(torch.stack(out))
    assert ran == [True, False]
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(evals[0], evals[1])
    assert torch.equal(outs[0], outs[1])


def test_pipeline_pndm_remove_experts_tiny(tiny):
    """The reference's default scheduler: PNDM (skip_prk_steps) = num_inference_steps + 1 U-Net calls, the
    receiver's (t, l) counter advancing once per call (T = 6 for 5 steps, as T = 51 for 50). RemoveExperts with
    removal at every call (t < 20) vs the oracle's PNDM restatement, near-tie rows teacher-forced."""
    from neuron_receivers import GEGLU, RemoveExperts
    cfg, unet, ref = tiny
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=5, scheduler="pndm")
    layers = moefy_tiny(pipe, relu=False)
    g = torch.Generator().manual_seed(21)
    T, L = 6, 16
    lists = {t: {l: sorted(torch.randperm(layers[l][1], generator=g)[:max(1, layers[l][1] // 4)].tolist())
                 for l in range(L)} for t in range(T)}
    rec = recording(RemoveExperts)(0, None, T, L, replace_fn=GEGLU, expert_indices=lists, store_gates=False)
    rec.sels = []
    out, _ = rec.observe_activation(pipe, ["a harbour at night"])
    assert (rec.timestep, rec.layer) == (6, 0) and len(rec.sels) == T * L
    stats = dict(rows=0, clear=0, clear_mismatch=0, forced=0)
    exp = run_oracle(ref, cfg, ["a harbour at night"], 5, scheduler="pndm",
                     ff_hook_factory=forced_factory(layers, "gelu", rec.sels, lists, stats))
    assert stats["clear_mismatch"] == 0, stats
    assert rel_l2(out[0], exp[0]) <= 1e-2


def test_pipeline_metric_workload_sd14_64x64(parity_report):
    """The bench's workload at 2 DDIM steps: SD-1.4 at 64x64 latents (512^2), 2 prompts (U-Net batch 4 with CFG),
    relufied, MoE-fied (expert 20, top-k 0.2), RemoveExperts with removal active (t < 20) through
    observe_activation on the fused + keep path (sdmoe_linear_geglu -> sdmoe_moe_topk_keep -> sdmoe_linear_keep),
    against the fp32 oracle with the reference hook in fp16 (remove_skilled_experts.py:24-55).
    Contract: the device's top-k selection equals the oracle's on every row whose k-th/(k+1)-th fp16 score gap is
    clear of near-tie noise (16 ulps: the two trunks' fp16 vs fp32 activations feed the hook); near-tie rows are
    teacher-forced and counted; final latents rel L2 <= 1e-2."""
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import GEGLU, RemoveExperts
    import sdmoe.unet as U
    assert U.FUSED_GEGLU and U.FUSED_KEEP
    cfg = UNetConfig.sd14(64)
    sd = make_state_dict(cfg, 11)
    unet = UNet2DConditionModel.from_state_dict(sd, cfg, DEV)
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    find_and_change_geglu(pipe.unet)
    moefy_synthetic(pipe, 0.2, 20, seed=12)
    mods = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    layers = [(m.labels.numpy(), m.patterns.shape[0], m.k) for m in mods]
    assert [k for _, _, k in layers] == [12, 12, 25, 25, 51, 51, 51, 51, 51, 51, 25, 25, 25, 12, 12, 12]
    g = torch.Generator().manual_seed(13)
    T, L = 2, 16
    lists = {t: {l: sorted(torch.randperm(layers[l][1], generator=g)[:layers[l][1] // 10].tolist())
                 for l in range(L)} for t in range(T)}
    rec = recording(RemoveExperts)(0, None, T, L, replace_fn=GEGLU, expert_indices=lists, store_gates=False)
    rec.sels = []
    prompts = ["Starry night by Van Gogh", "a wheat field with cypresses"]
    out, _ = rec.observe_activation(pipe, prompts)
    torch.cuda.synchronize()
    assert (rec.timestep, rec.layer) == (2, 0) and len(rec.sels) == T * L
    assert all(m._out_keep is not None for m in mods), "fused + keep path did not run"
    got = torch.stack(out).float().cpu()
    del unet, pipe
    torch.cuda.empty_cache()
    ref = UNetRef({k: v.half().float() for k, v in sd.items()}, cfg)
    stats = dict(rows=0, clear=0, clear_mismatch=0, forced=0)
    exp = run_oracle(ref, cfg, prompts, 2, ff_hook_factory=forced_factory(layers, "relu", rec.sels, lists, stats))
    parity_report("pipeline_sd14_64x64_remove_relu_topk0.2", rows=stats["rows"], clear=stats["clear"],
                  near_tie=stats["rows"] - stats["clear"], flips=stats["forced"], rel_l2=rel_l2(got, exp))
    assert stats["clear_mismatch"] == 0, stats
    assert torch.isfinite(got).all()
    assert rel_l2(got, exp) <= 1e-2
