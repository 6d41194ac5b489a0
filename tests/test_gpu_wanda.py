"""Wanda weight masks on the MI355X (BASELINE configs 4-5): the masked GEMM, the HIP Wanda hook on the reference's
own mask fixture, and union-Wanda + MoE routing through the pipeline against the oracle.

* sdmoe_linear_masked applies the mask to the W fragments after their LDS read: bit-identical to masking the
  weights first (sdmoe_mask_weight, the device form of W * (1 - M)) and running the same GEMM, in every mode
  (W mask; W mask + MoE keep bits) and on the tiles / split-K paths the U-Net's shapes take;
* WandaRemoveNeuronsFast.linear_hook_fn (remove_wanda_neurons_fast.py:69-83) on the masks of the reference's
  weights_320_1280.csv (tests/golden/wanda_320x1280_*.npz, produced by the reference's own hook): within 2 fp16 ulps
  of the reference's fp16 output (our GEMM accumulates in fp32 in its own order; the CPU's fp16 linear in another);
* config 4's per-GPU path at SD-1.4 widths: RemoveExperts routing (top-k 0.2, relufied) and a two-concept union
  Wanda mask on ff.net.2 together, fused routed FFN kept (the mask's columns permuted with the experts), against
  the oracle with the reference hooks (multi_concept_remover.py:43-53 -> remove_wanda_neurons_fast.py:69-83).
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe import ops  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
import synth  # noqa: E402

DEV = "cuda"


def packed(mask):
    return torch.from_numpy(np.packbits(mask.astype(np.uint8), axis=-1, bitorder="little")).to(DEV)


def fp16_spacing(a):
    return np.spacing(np.abs(a).astype(np.float16)).astype(np.float32)


@pytest.mark.parametrize("M,N,K,density", [(256, 320, 1280, 0.03), (65536, 320, 1280, 0.025),
                                           (16384, 640, 2560, 0.025), (4096, 1280, 5120, 0.025),
                                           (777, 1280, 5120, 0.3), (64, 1280, 5120, 0.025), (1000, 168, 640, 0.5)])
def test_linear_masked_equals_masked_weight_gemm(M, N, K, density):
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).half().to(DEV)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(DEV)
    b = (torch.randn(N, generator=g) * 0.1).half().to(DEV)
    r = torch.randn(M, N, generator=g).half().to(DEV)
    mask = (torch.rand(N, K, generator=g) < density).numpy()
    bits = packed(mask)
    wm = ops.wmask_kmajor(bits)
    y = ops.linear_masked(x, w, b, wmask=wm, residual=r)
    w_masked = ops.mask_weight(w, bits)
    assert torch.equal(w_masked.cpu(), torch.where(torch.from_numpy(mask), torch.zeros_like(w.cpu()), w.cpu()))
    assert torch.equal(y, ops.linear(x, w_masked, b, residual=r))
    assert torch.equal(ops.linear(x, w, b, residual=r, wmask=wm), y)
    # with MoE keep bits on the A operand as well (the routed FFN down projection under a Wanda mask)
    keep = torch.randint(-2 ** 62, 2 ** 62, (K // 64, M), generator=g, dtype=torch.int64).to(DEV)
    y2 = ops.linear_masked(x, w, b, keep=keep, wmask=wm, residual=r)
    assert torch.equal(y2, ops.linear_keep(x, keep, w_masked, b, residual=r))
    ref = x.float() @ (w.float() * torch.from_numpy(~mask).to(DEV).float()).t() + b.float() + r.float()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * max(1.0, ref.abs().max().item())


def test_wmask_kmajor_layout_and_permutation():
    N, K = 48, 320
    rng = np.random.default_rng(1)
    mask = rng.random((N, K)) < 0.2
    perm = rng.permutation(K).astype(np.int32)
    for p in (None, perm):
        out = ops.wmask_kmajor(packed(mask), None if p is None else torch.from_numpy(p).to(DEV)).cpu().numpy()
        words = out.view(np.uint64)  # [K/64, N]
        bits = ((words[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)  # [K/64, N, 64]
        got = bits.transpose(1, 0, 2).reshape(N, K)
        exp = mask if p is None else mask[:, p]
        assert np.array_equal(got, exp)


@pytest.mark.parametrize("dtype", ["float16"])
@pytest.mark.parametrize("bake", [True, False], ids=["baked", "in_gemm"])
def test_wanda_hook_on_reference_fixture(dtype, bake, parity_report):
    """The HIP Wanda hook, driven like the reference (counter over the 5 layers of t = 0), on the masks of the
    reference's weights_320_1280.csv, vs the reference hook's own outputs -- with the baked masked weights (default)
    and with the mask applied inside the GEMM (bake_budget_bytes = 0)."""
    from neuron_receivers import WandaRemoveNeuronsFast
    from sdmoe.unet import LoRACompatibleLinear
    with np.load(os.path.join(GOLD, f"wanda_320x1280_{dtype}.npz"), allow_pickle=False) as z:
        c = {k: z[k] for k in z.files}
    bits = c["mask_bits"]  # [L, 320, 160]
    L = bits.shape[0]
    rec = WandaRemoveNeuronsFast.from_packed(0, {0: {l: bits[l] for l in range(L)}}, 1, L, store_gates=False)
    if not bake:
        rec.bake_budget_bytes = 0
    w, b = synth.down_weights(320, int(c["w_seed"]))
    lin = LoRACompatibleLinear(torch.from_numpy(w).half().to(DEV), torch.from_numpy(b).half().to(DEV))
    x = torch.from_numpy(c["x"]).to(DEV)
    worst = 0.0
    for l in range(L):
        assert (rec.timestep, rec.layer) == (0, l)
        y = rec.linear_hook_fn(lin, (x,), None).float().cpu().numpy()
        ref = c["out"][l].astype(np.float32)
        # 2 ulps of the element, floored at 1 ulp of a quarter of the output's range: cancellation in a K = 1280
        # fp32 dot product leaves a small output whose own ulp is far below the accumulation order noise
        unit = np.maximum(fp16_spacing(ref), fp16_spacing(np.full_like(ref, 0.25 * np.abs(ref).max())) / 2)
        ulps = np.abs(y - ref) / unit
        worst = max(worst, float(ulps.max()))
        assert ulps.max() <= 2.0, f"layer {l}: {ulps.max()} ulps"
        # the mask matters on this data: the unmasked product differs
        y0 = ops.linear(x.reshape(-1, 1280), lin.weight, lin.bias).float().cpu().numpy().reshape(y.shape)
        assert np.abs(y0 - ref).max() > 10 * np.abs(y - ref).max()
    assert (rec.timestep, rec.layer) == (1, 0)
    assert any(isinstance(k[0], str) and k[0] == ("baked" if bake else "kmajor") for k in rec._dev)
    parity_report(f"wanda_hook_fixture[{dtype},{'baked' if bake else 'in_gemm'}]", layers=L, max_ulps=worst)


def test_wanda_baked_weight_follows_in_place_update():
    """An in-place update of ff.net.2's weight (load_state_dict / copy_ / a LoRA merge keeps the address) must
    re-bake W * (1 - M): the cache is keyed by the Parameter's own version counter, not by `.data`'s."""
    from neuron_receivers import WandaRemoveNeuronsFast
    from sdmoe.unet import LoRACompatibleLinear
    g = torch.Generator().manual_seed(5)
    mask = (torch.rand(64, 256, generator=g) < 0.1).numpy()
    rec = WandaRemoveNeuronsFast.from_packed(0, {0: {0: np.packbits(mask, axis=-1, bitorder="little")}}, 1, 1,
                                             store_gates=False)
    lin = LoRACompatibleLinear((torch.randn(64, 256, generator=g) * 0.05).half().to(DEV),
                               torch.zeros(64, dtype=torch.float16, device=DEV))
    x = torch.randn(128, 256, generator=g).half().to(DEV)
    keep = torch.from_numpy(~mask).to(DEV)
    y1 = rec.linear_hook_fn(lin, (x,), None)
    assert torch.equal(y1, ops.linear(x, torch.where(keep, lin.weight, torch.zeros_like(lin.weight)), lin.bias))
    ptr = lin.weight.data_ptr()
    with torch.no_grad():
        lin.weight.copy_(lin.weight * 2)  # in place: same address, new version
    assert lin.weight.data_ptr() == ptr
    rec.reset_time_layer()
    y2 = rec.linear_hook_fn(lin, (x,), None)
    assert any(isinstance(k[0], str) and k[0] == "baked" for k in rec._dev)
    assert torch.equal(y2, ops.linear(x, torch.where(keep, lin.weight, torch.zeros_like(lin.weight)), lin.bias))
    assert not torch.equal(y1, y2)


@pytest.mark.parametrize("bake", [True, False], ids=["baked", "in_gemm"])
def test_union_wanda_moe_pipeline_sd14(bake, parity_report):
    """Config 4's per-GPU path at SD-1.4 widths (32x32 latents, 2 prompts, 2 DDIM steps): a two-concept union Wanda
    mask on every ff.net.2 together with RemoveExperts routing (relufied, top-k 0.2, removal for t < 20). The
    FeedForward keeps the fused routed path (union mask permuted with the experts, one sdmoe_linear_masked launch
    with the top-k keep bits); the oracle runs the reference hooks (fp16 routing, teacher-forced on near-ties) with
    the union mask in the natural neuron order. Final latents rel L2 <= 1e-2; selection identical on clear rows."""
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import GEGLU, RemoveExperts, WandaRemoveNeuronsFast, MultiConceptRemoverWanda
    from sdmoe.config import UNetConfig
    from sdmoe.unet import UNet2DConditionModel
    from sdmoe.weights import make_state_dict
    from sdmoe.pipeline import StableDiffusionPipeline
    from oracle.unet_ref import UNetRef
    from oracle import hooks_ref as H
    from test_gpu_unet import recording, forced_factory, run_oracle, rel_l2

    cfg = UNetConfig.sd14(32)
    sd = make_state_dict(cfg, 21)
    unet = UNet2DConditionModel.from_state_dict(sd, cfg, DEV)
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    find_and_change_geglu(pipe.unet)
    moefy_synthetic(pipe, 0.2, 20, seed=22)
    mods = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    downs = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.2")]
    layers = [(m.labels.numpy(), m.patterns.shape[0], m.k) for m in mods]
    T, L = 2, 16
    rng = np.random.default_rng(23)
    concepts = {c: {t: {l: (rng.random(tuple(downs[l].weight.shape)) < 0.025).astype(np.int64) for l in range(L)}
                    for t in range(T)} for c in ("van gogh", "monet")}
    removers = {c: WandaRemoveNeuronsFast(0, None, T, L, masks=m, store_gates=False) for c, m in concepts.items()}
    mc = MultiConceptRemoverWanda(None, 0, T, L, concepts_to_remove=list(concepts), removers=removers)
    mc.reset_union_remover()
    mc.handle_multiple_concepts(list(concepts))
    union = {t: {l: H.union_masks([concepts[c][t][l] for c in concepts]) for l in range(L)} for t in range(T)}
    wanda = mc.union_neuron_remover
    if not bake:
        wanda.bake_budget_bytes = 0
    g = torch.Generator().manual_seed(24)
    lists = {t: {l: sorted(torch.randperm(layers[l][1], generator=g)[:layers[l][1] // 10].tolist())
                 for l in range(L)} for t in range(T)}
    rec = recording(RemoveExperts)(0, None, T, L, replace_fn=GEGLU, expert_indices=lists, store_gates=False)
    rec.sels = []
    prompts = ["a church in the style of van gogh", "water lilies"]
    wanda.reset_time_layer()
    wanda.prepare(pipe)
    hooks = wanda.register_hooks(pipe)
    try:
        out, _ = rec.observe_activation(pipe, prompts)
    finally:
        wanda.remove_hooks(hooks)
    torch.cuda.synchronize()
    assert (wanda.timestep, wanda.layer) == (2, 0) and (rec.timestep, rec.layer) == (2, 0)
    assert all(m._out_keep is not None for m in mods), "fused routed path did not run under the Wanda hook"
    if bake:  # the masked weight baked once per (t, l) in the experts' column order
        assert any(k[0] == "baked" and k[3] is False for k in wanda._dev if isinstance(k[0], str))
    else:     # the mask's permuted K-major form applied inside the GEMM
        assert any(k[0] == "kmajor" and k[3] is False for k in wanda._dev if isinstance(k[0], str))
    got = torch.stack(out).float().cpu()
    ref = UNetRef({k: v.half().float() for k, v in sd.items()}, cfg)

    def down_factory(step):
        def hook(layer, x, w, b):
            return H.wanda_linear(x, w, b, union[step][layer])
        return hook
    stats = dict(rows=0, clear=0, clear_mismatch=0, forced=0)
    exp = run_oracle(ref, cfg, prompts, 2, ff_hook_factory=forced_factory(layers, "relu", rec.sels, lists, stats),
                     down_hook_factory=down_factory)
    parity_report(f"pipeline_sd14_32x32_union_wanda_moe[{'baked' if bake else 'in_gemm'}]", rows=stats["rows"], clear=stats["clear"],
                  near_tie=stats["rows"] - stats["clear"], flips=stats["forced"], rel_l2=rel_l2(got, exp))
    assert stats["clear_mismatch"] == 0, stats
    assert rel_l2(got, exp) <= 1e-2
    # the union mask actually changes the result (vs routing alone)
    rec2 = RemoveExperts(0, None, T, L, replace_fn=GEGLU, expert_indices=lists, store_gates=False)
    out2, _ = rec2.observe_activation(pipe, prompts)
    assert rel_l2(torch.stack(out2).float().cpu(), got) > 1e-3


@pytest.mark.parametrize("bake", [True, False], ids=["baked", "in_gemm"])
def test_union_wanda_receiver_survives_remoefication(bake):
    """One Wanda receiver reused across a re-MoE-fication with NEW expert labels (so a new Routing and a new neuron
    permutation, possibly at a recycled device address): its cached permuted masks / baked weights must follow the
    new permutation. The second run equals a fresh receiver's run bit for bit, and differs from the first run."""
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import MOEFy, WandaRemoveNeuronsFast
    from neuron_receivers import remove_wanda_neurons_fast as W
    from sdmoe.config import UNetConfig
    from sdmoe.unet import UNet2DConditionModel
    from sdmoe.weights import make_state_dict
    from sdmoe.pipeline import StableDiffusionPipeline

    cfg = UNetConfig.sd14(16)
    pipe = StableDiffusionPipeline(UNet2DConditionModel.from_state_dict(make_state_dict(cfg, 31), cfg, DEV), DEV,
                                   num_inference_steps=2)
    find_and_change_geglu(pipe.unet)
    downs = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.2")]
    T, L = 2, 16
    rng = np.random.default_rng(32)
    masks = {t: {l: (rng.random(tuple(downs[l].weight.shape)) < 0.05).astype(np.int64) for l in range(L)}
             for t in range(T)}

    def make():
        w = WandaRemoveNeuronsFast(0, None, T, L, masks=masks, store_gates=False)
        if not bake:
            w.bake_budget_bytes = 0
        return w

    def run(wanda):
        wanda.reset_time_layer()
        wanda.prepare(pipe)
        hooks = wanda.register_hooks(pipe)
        try:
            out, _ = MOEFy(seed=0, store_gates=False).observe_activation(pipe, ["a lighthouse"])
        finally:
            wanda.remove_hooks(hooks)
        return out[0].clone()

    reused = make()
    moefy_synthetic(pipe, 0.2, 20, seed=1)
    first = run(reused)
    baked0 = W._BAKED_BYTES.get(str(downs[0].weight.device), 0)
    moefy_synthetic(pipe, 0.2, 20, seed=2)  # new labels -> new Routing / perm for every layer
    torch.cuda.empty_cache()
    second = run(reused)
    fresh = run(make())
    assert torch.equal(second, fresh)
    assert not torch.equal(first, second)
    # stale permuted entries were replaced, not accumulated: one entry per (t, l) and form
    forms = [k for k in reused._dev if isinstance(k[0], str)]
    assert len(forms) == len(set(forms)) == T * L
    if bake:
        del reused, fresh
        import gc
        gc.collect()
        assert W._BAKED_BYTES.get(str(downs[0].weight.device), 0) <= baked0
