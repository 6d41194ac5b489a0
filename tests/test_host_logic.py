"""CPU-only tests of the host side: C-ABI library load + exported symbols, mask formats, receiver bookkeeping,
scheduler constants, synthetic weights, routing layout. No GPU compute is launched here."""
import ctypes
import io
import json
import os
import pickle
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "sdmoe.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sdmoe_\w+)\(", txt, re.M)))


def test_library_loads_and_exports_every_header_symbol():
    from sdmoe import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/sdmoe.h but not exported"
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(syms)
    assert lib.sdmoe_version().decode().startswith("sdmoe-hip")


def test_abi_argument_validation_without_gpu():
    """Argument errors are reported as negative codes before anything is launched."""
    from sdmoe import _lib
    lib = _lib.load()
    assert lib.sdmoe_linear(None, 0, None, 0, None, None, 0, 0, None, 0, None, 0, 1, 8, 64, 0, None, 0, None) == -1
    assert lib.sdmoe_linear(1, 64, 1, 64, None, None, 0, 0, None, 0, 1, 8, 4, 8, 60, 0, None, 0, None) == -2
    assert lib.sdmoe_conv3x3(1, 64, 1, 8, 8, 64, 1, None, None, 0, None, 0, 1, 8, 8, 3, 0, 0, None, 0, None) == -3
    assert lib.sdmoe_attention(1, 8, 1, 8, 1, 8, 1, 8, 1, 4, 4, 1, 48, 1.0, None) == -3
    assert lib.sdmoe_geglu_route(1, 8, 4, 16, 300, 4, 2, 1, 1, 1, None, 1, 16, None, 0, None, None, None) == -3
    assert lib.sdmoe_geglu_route(1, 8, 4, 16, 8, 9, 2, 1, 1, 1, None, 1, 16, None, 0, None, None, None) == -1
    assert lib.sdmoe_tune(0, 5) == -1 and lib.sdmoe_tune(0, 0) == 0


def test_ops_refuse_cpu_tensors():
    from sdmoe import ops, _lib
    x = torch.zeros(4, 64, dtype=torch.float16)
    with pytest.raises(_lib.SdmoeError):
        ops.linear(x, torch.zeros(8, 64, dtype=torch.float16))


def test_mask_pack_roundtrip_and_bit_order():
    from sdmoe import mask_io
    rng = np.random.default_rng(0)
    m = (rng.random((320, 1280)) < 0.025).astype(np.int64)
    bits = mask_io.pack_mask(m)
    assert bits.shape == (320, 160) and bits.dtype == np.uint8
    assert np.array_equal(mask_io.unpack_mask(bits, 1280), m)
    # device contract: bit j of byte (n*K + k)/8 is element k = 8*byte + j (little bit order)
    n, k = 7, 1000
    m2 = np.zeros((320, 1280), dtype=np.int64)
    m2[n, k] = 1
    b2 = mask_io.pack_mask(m2).reshape(-1)
    idx = (n * 1280 + k) // 8
    assert b2[idx] == 1 << (k % 8) and b2.sum() == b2[idx]


def test_restricted_unpickler_accepts_reference_formats_and_refuses_code(tmp_path):
    import scipy.sparse
    from sdmoe import mask_io
    m = (np.random.default_rng(1).random((64, 256)) < 0.05).astype(np.int64)
    p = tmp_path / "timestep_0_layer_0.pkl"
    with open(p, "wb") as f:
        pickle.dump(scipy.sparse.csr_matrix(m), f)  # modularity/wanda.py:169-173 format
    assert np.array_equal(mask_io.load_mask_pickle(p), m)
    p2 = tmp_path / "timestep_0_layer_1.pkl"
    with open(p2, "wb") as f:
        pickle.dump(np.asmatrix(m), f)  # benchmarks/save_union_experts.py:123-126 format
    assert np.array_equal(mask_io.load_mask_pickle(p2), m)
    p3 = tmp_path / "evil.pkl"
    with open(p3, "wb") as f:
        pickle.dump(os.system, f)
    with pytest.raises(pickle.UnpicklingError):
        mask_io.load_mask_pickle(p3)


def test_wanda_masks_load_from_all_formats(tmp_path):
    import scipy.sparse
    from sdmoe import mask_io
    from neuron_receivers import WandaRemoveNeuronsFast
    rng = np.random.default_rng(2)
    masks = [(rng.random((64, 256)) < 0.03).astype(np.int64) for _ in range(3)]
    with open(tmp_path / "timestep_0_layer_0.pkl", "wb") as f:
        pickle.dump(scipy.sparse.csr_matrix(masks[0]), f)
    mask_io.save_wanda_mask(tmp_path, 0, 1, masks[1])
    idx = np.argwhere(masks[2]).tolist()
    json.dump(idx, open(tmp_path / "timestep_0_layer_2.json", "w"))
    rec = WandaRemoveNeuronsFast(0, str(tmp_path), 1, 3, weights_shape=[(64, 256)] * 3)
    for l in range(3):
        assert np.array_equal(rec.dense_mask(0, l), masks[l])


def test_union_of_packed_masks_equals_oracle_or():
    from oracle import hooks_ref as H
    from sdmoe import mask_io
    from neuron_receivers import WandaRemoveNeuronsFast, MultiConceptRemoverWanda
    rng = np.random.default_rng(3)
    T, L = 2, 2
    concepts = {c: {t: {l: (rng.random((32, 128)) < 0.05).astype(np.int64) for l in range(L)} for t in range(T)}
                for c in ("a", "b", "c")}
    removers = {c: WandaRemoveNeuronsFast(0, None, T, L, masks=m) for c, m in concepts.items()}
    mc = MultiConceptRemoverWanda(None, 0, T, L, concepts_to_remove=list(concepts), removers=removers)
    mc.handle_multiple_concepts(["a", "c"])
    for t in range(T):
        for l in range(L):
            exp = H.union_masks([concepts["a"][t][l], concepts["c"][t][l]])
            assert np.array_equal(mc.union_neuron_remover.dense_mask(t, l), exp)
    mc.reset_union_remover()
    assert mc.union_neuron_remover.dense_mask(0, 0).sum() == 0


def test_union_starts_from_last_concept_and_accumulates():
    """multi_concept_remover.py:24-33: the union remover is built from the last configured concept's masks, and
    handle_multiple_concepts ORs into it (:43-53) until reset_union_remover (:35-41)."""
    from oracle import hooks_ref as H
    from neuron_receivers import WandaRemoveNeuronsFast, MultiConceptRemoverWanda
    rng = np.random.default_rng(5)
    T, L = 1, 2
    concepts = {c: {t: {l: (rng.random((16, 64)) < 0.1).astype(np.int64) for l in range(L)} for t in range(T)}
                for c in ("a", "b", "c")}
    removers = {c: WandaRemoveNeuronsFast(0, None, T, L, masks=m) for c, m in concepts.items()}
    mc = MultiConceptRemoverWanda(None, 0, T, L, concepts_to_remove=list(concepts), removers=removers)
    assert np.array_equal(mc.union_neuron_remover.dense_mask(0, 1), concepts["c"][0][1])
    mc.handle_multiple_concepts(["a", "b"])
    exp = H.union_masks([concepts[c][0][1] for c in ("a", "b", "c")])
    assert np.array_equal(mc.union_neuron_remover.dense_mask(0, 1), exp)


def test_remove_concepts_two_value_contract():
    """unified_editing.py:126 unpacks `output, single_image_removal = remove_concepts(...)` for 0, 1 and several
    concepts; output is [original | removed] side by side (multi_concept_remover.py:83-99)."""
    from neuron_receivers import WandaRemoveNeuronsFast, MultiConceptRemoverWanda
    T, L = 1, 1
    removers = {c: WandaRemoveNeuronsFast(0, None, T, L, masks={0: {0: np.zeros((8, 16), np.int64)}})
                for c in ("x", "y")}
    mc = MultiConceptRemoverWanda(None, 0, T, L, concepts_to_remove=["x", "y"], removers=removers)
    calls = []

    class FakePipe:
        def __call__(self, prompt, **kw):
            calls.append(prompt)
            return type("O", (), {"images": [torch.full((4, 8, 8), float(len(calls)))]})()
    for r in removers.values():  # no GPU here: the receivers' pipeline call is the fake one
        r.observe_activation = lambda model, ann, bboxes=None: (model(ann).images[0], [])
    mc.union_neuron_remover.observe_activation = lambda model, ann, bboxes=None: (model(ann).images[0], [])
    out, singles = mc.remove_concepts(FakePipe(), "p", [])
    assert singles is None and tuple(out.shape) == (4, 8, 8)
    out, singles = mc.remove_concepts(FakePipe(), "p", ["x"])
    assert singles is None and tuple(out.shape) == (4, 8, 16)
    assert torch.equal(out[..., 8:], mc.last_outputs["removal"]) and torch.equal(out[..., :8],
                                                                                  mc.last_outputs["original"])
    out, singles = mc.remove_concepts(FakePipe(), "p", ["x", "y"])
    assert tuple(out.shape) == (4, 8, 16) and len(singles) == 2 and tuple(singles[0].shape) == (4, 8, 16)


def test_modify_ffn_reads_numpy_scalar_labels(tmp_path):
    """ParamSplit.save writes [x for x in kmeans.labels_] -- numpy int32 scalars (moe_utils.py:54-61): they load
    through the restricted weights_only path; a file with any other global is refused."""
    from moefication.helper import modify_ffn, balanced_random_labels
    from sdmoe import mask_io
    from sdmoe.unet import GEGLU, LoRACompatibleLinear
    lab = balanced_random_labels(1280, 20, 2)
    for dt in (np.int32, np.int64):
        g = GEGLU(LoRACompatibleLinear(torch.zeros(2 * 1280, 320, dtype=torch.float16)))
        torch.save([dt(v) for v in lab], tmp_path / "labels")
        modify_ffn(g, str(tmp_path / "labels"), 0.2)
        assert g.k == 12 and torch.equal(g.patterns.float().argmax(0), torch.from_numpy(lab))

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))
    torch.save([Evil()], tmp_path / "evil")
    with pytest.raises(Exception):
        mask_io.load_labels(str(tmp_path / "evil"))


def test_union_random_drop_is_seeded_and_subset():
    from oracle import hooks_ref as H
    rng = np.random.default_rng(4)
    ms = [(rng.random((40, 80)) < 0.1).astype(np.int64) for _ in range(4)]
    u1 = H.union_with_random_drop(ms, 0.95, seed=7)
    u2 = H.union_with_random_drop(ms, 0.95, seed=7)
    assert np.array_equal(u1, u2)
    full = H.union_masks(ms)
    assert np.all(u1 <= full) and u1.sum() < full.sum()


def test_counter_semantics_match_reference_receivers():
    from neuron_receivers import NeuronPredictivity
    from oracle.hooks_ref import TimeLayerCounter
    r = NeuronPredictivity(0, 51, 16)
    o = TimeLayerCounter(16)
    for _ in range(16 * 51 + 5):
        assert (r.timestep, r.layer) == (o.timestep, o.layer)
        r.update_time_layer()
        o.update()
    r.reset_time_layer()
    assert (r.timestep, r.layer) == (0, 0)


def test_remove_experts_constructor_fixes_snapshot_defects(tmp_path):
    """App. A #1/#2: replace_fn is accepted as a keyword; keep_nsfw does not land in replace_fn."""
    from neuron_receivers import GEGLU, RemoveExperts
    for t in range(2):
        for l in range(2):
            json.dump([t, l], open(tmp_path / f"timestep_{t}_layer_{l}.json", "w"))
    r = RemoveExperts(0, str(tmp_path), 2, 2, keep_nsfw=True, replace_fn=GEGLU)
    assert r.replace_fn is GEGLU and r.keep_nsfw is True
    assert r.expert_indices[1][0] == [1, 0]


def test_ddim_schedule_matches_oracle():
    from sdmoe.pipeline import ddim_schedule
    from oracle.unet_ref import ddim_schedule as ref
    ts, at, ap = ddim_schedule(50)
    rts, rat, rap = ref(50)
    assert list(ts) == list(rts) and ts[0] == 981 and ts[-1] == 1
    assert np.allclose(at, rat, rtol=0, atol=0) and np.allclose(ap, rap, rtol=0, atol=0)


def test_synthetic_weights_match_sd14_architecture():
    import math
    from sdmoe.config import UNetConfig
    from sdmoe.weights import param_specs, make_state_dict
    cfg = UNetConfig.sd14()
    specs = param_specs(cfg)
    assert sum(math.prod(s) for _, s, _ in specs) == 859_520_964  # SD-1.4 UNet2DConditionModel
    geglu = [n for n, _, _ in specs if n.endswith("ff.net.0.proj.weight")]
    assert len(geglu) == 16
    assert [n[:-len(".proj.weight")] for n in sorted(geglu)] == [n for n, _ in cfg.geglu_layers()]
    sd1 = make_state_dict(cfg, 0, names={"conv_in.weight", "mid_block.resnets.0.conv1.bias"})
    sd2 = make_state_dict(cfg, 0, names={"conv_in.weight"})
    assert torch.equal(sd1["conv_in.weight"], sd2["conv_in.weight"])


def test_routing_layout_from_patterns():
    from sdmoe.ops import Routing
    from oracle.hooks_ref import patterns_from_labels
    from moefication.helper import balanced_random_labels
    lab = balanced_random_labels(1280, 20, 0)
    P = patterns_from_labels(lab)
    r = Routing.from_patterns(P, 12, "cpu")
    assert r.E == 64 and r.k == 12 and r.F == 1280
    off = r.e_off.numpy()
    nid = r.e_nid.numpy()
    for e in (0, 17, 63):
        members = nid[off[e]:off[e + 1]]
        assert len(members) == 20 and np.all(lab[members] == e) and np.all(np.diff(members) > 0)
    with pytest.raises(ValueError):
        Routing.from_patterns(torch.ones(2, 4), 1, "cpu")


def test_removed_bits_packing():
    from sdmoe.ops import removed_bits
    b = removed_bits([0, 31, 32, 255], 256, "cpu").numpy().view(np.uint32)
    assert b.shape == (8,) and b[0] == (1 | (1 << 31)) and b[1] == 1 and b[7] == 1 << 31
    with pytest.raises(IndexError):
        removed_bits([256], 256, "cpu")


def test_modify_ffn_reads_reference_label_format(tmp_path):
    """moe_utils.py:54-61 writes torch.save(list[int]); helper.modify_ffn sets patterns [E, 4C] and k."""
    from moefication.helper import modify_ffn, balanced_random_labels
    from sdmoe.unet import GEGLU, LoRACompatibleLinear
    g = GEGLU(LoRACompatibleLinear(torch.zeros(2 * 1280, 320, dtype=torch.float16)))
    lab = balanced_random_labels(1280, 20, 1)
    torch.save([int(v) for v in lab], tmp_path / "labels")
    modify_ffn(g, str(tmp_path / "labels"), 0.2)
    assert tuple(g.patterns.shape) == (64, 1280) and g.k == 12 and g.patterns.dtype == torch.float16
    assert torch.equal(g.patterns.float().argmax(0), torch.from_numpy(lab))


def test_synthetic_weights_match_sdxl_architecture():
    """SDXL-base UNet2DConditionModel (BASELINE config 5): 2,567,463,684 params, 70 GEGLU FFNs whose sorted
    names (helper.py:77) equal the hook execution order; the module tree carries diffusers' names."""
    import math
    from sdmoe.config import UNetConfig
    from sdmoe.weights import param_specs, make_state_dict
    from sdmoe.unet import UNet2DConditionModel
    cfg = UNetConfig.sdxl()
    specs = param_specs(cfg)
    assert sum(math.prod(s) for _, s, _ in specs) == 2_567_463_684
    geglu = sorted(n[:-len(".proj.weight")] for n, _, _ in specs if n.endswith("ff.net.0.proj.weight"))
    assert len(geglu) == 70 and geglu == [n for n, _ in cfg.geglu_layers()]
    assert {C for _, C in cfg.geglu_layers()} == {640, 1280}
    assert cfg.heads_for(640) == 10 and cfg.heads_for(1280) == 20
    tiny = UNetConfig.tiny_xl(16)
    u = UNet2DConditionModel.from_state_dict(make_state_dict(tiny, 0), tiny, "cpu")  # construction only
    names = [n for n, _ in u.named_modules() if n.endswith("ff.net.0")]
    assert names == [n for n, _ in tiny.geglu_layers()] and len(names) == 28
    assert u.add_embedding.linear_1.weight.shape[1] % 64 == 0


def test_oracle_sdxl_micro_conditioning():
    """The oracle's text_time add_embedding reaches the output; linear proj_in/out are used."""
    from sdmoe.config import UNetConfig
    from sdmoe.weights import make_state_dict
    from oracle.unet_ref import UNetRef
    cfg = UNetConfig.tiny_xl(8)
    sd = make_state_dict(cfg, 1)
    assert sd["down_blocks.1.attentions.0.proj_in.weight"].dim() == 2
    ref = UNetRef(sd, cfg)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 4, 8, 8, generator=g)
    ctx = torch.randn(1, 77, 128, generator=g)
    ac = {"text_embeds": torch.randn(1, 64, generator=g), "time_ids": torch.tensor([[64., 64, 0, 0, 64, 64]])}
    e1 = ref(x, 301.0, ctx, added_cond=ac)
    e2 = ref(x, 301.0, ctx, added_cond={"text_embeds": ac["text_embeds"] * 0, "time_ids": ac["time_ids"]})
    assert torch.isfinite(e1).all() and (e1 - e2).abs().max() > 1e-4


def test_pndm_plan_matches_oracle_scheduler():
    """pipeline.pndm_schedule (the per-call coefficients sdmoe_cfg_multistep_step applies) reproduces the
    oracle's PNDMScheduler(skip_prk_steps) restatement over all 51 calls, including the duplicated 961 call and
    the warm-up averaging step; the kernel's update rule is emulated on the host here."""
    from sdmoe.pipeline import pndm_schedule
    from oracle.unet_ref import PNDMRef
    plan = pndm_schedule(50)
    ref = PNDMRef(50)
    assert len(plan) == 51 and [p[0] for p in plan] == ref.timesteps.tolist()
    assert ref.timesteps[:4].tolist() == [981, 961, 961, 941] and ref.timesteps[-1] == 1
    g = torch.Generator().manual_seed(0)
    x_ref = torch.randn(2, 4, 8, 8, generator=g, dtype=torch.float64)
    x = x_ref.clone()
    hist = torch.zeros((4,) + tuple(x.shape), dtype=torch.float64)
    cur = torch.zeros_like(x)
    for t, coef, flags in plan:
        e = torch.randn(x.shape, generator=g, dtype=torch.float64)
        x_ref = ref.step(e, t, x_ref)
        mo = coef[0] * e + sum(coef[1 + j] * hist[j] for j in range(4))
        if flags[0] >= 0:
            hist[flags[0]] = e
        src = cur if flags[1] else x
        if flags[2]:
            cur = x.clone()
        x = coef[5] * src - coef[6] * mo
    assert torch.allclose(x, x_ref, rtol=1e-10, atol=1e-10)


def test_balanced_assign_native_is_exact():
    """sdmoe_balanced_assign (host C++ auction; no GPU involved) reaches the exact optimum of the balanced
    assignment that k_means_constrained solves by min-cost flow: objective equal to scipy's
    linear_sum_assignment on the slot-expanded cost matrix, every cluster exactly n/k points."""
    from sdmoe.kmeans import balanced_assign
    from oracle.kmeans_ref import assign_exact
    rng = np.random.default_rng(0)
    for n, k in [(60, 6), (320, 16), (640, 32), (256, 256), (128, 1)]:
        X = rng.standard_normal((n, 8))
        C = rng.standard_normal((k, 8))
        cost = np.sqrt(((X[:, None] - C[None]) ** 2).sum(-1))
        lab = balanced_assign(cost, k)
        ref = assign_exact(cost, k)
        assert np.all(np.bincount(lab, minlength=k) == n // k)
        assert abs(cost[np.arange(n), lab].sum() - cost[np.arange(n), ref].sum()) <= 1e-9 * n
        assert np.array_equal(lab, ref)  # continuous random costs: the optimum is unique
    # integer costs with many ties: the objective is still optimal
    cost = rng.integers(0, 4, size=(120, 12)).astype(np.float64)
    lab = balanced_assign(cost, 12)
    assert cost[np.arange(120), lab].sum() == cost[np.arange(120), assign_exact(cost, 12)].sum()


def test_oracle_constrained_kmeans_properties():
    from oracle.kmeans_ref import constrained_kmeans
    rng = np.random.default_rng(1)
    centers = rng.standard_normal((8, 16)) * 4
    blob = np.repeat(np.arange(8), 10)
    X = centers[blob] + 0.1 * rng.standard_normal((80, 16))
    perm = rng.permutation(80)
    X, blob = X[perm], blob[perm]
    lab, C, inertia = constrained_kmeans(X, 8, 10, n_init=3)
    assert np.all(np.bincount(lab, minlength=8) == 10)
    # well-separated equal-size blobs are recovered exactly (up to cluster ids)
    for c in range(8):
        assert len(set(blob[lab == c].tolist())) == 1
    assert inertia < 80 * 16 * 0.1 ** 2 * 2


def test_union_over_time_oracle_and_layer_order():
    """Oracle of save_union_over_time.py:189-204 (strict > select_ratio * timesteps on the summed masks) and the
    sorted ff.net.2 layer order it indexes masks by (:163-169) = the hook-call order of the U-Net."""
    from oracle import hooks_ref as H
    from sdmoe import union_bake
    from sdmoe.config import UNetConfig
    from sdmoe.unet import UNet2DConditionModel
    from sdmoe.weights import make_state_dict
    m = [np.array([[1, 0, 1, 1]]), np.array([[1, 0, 0, 1]]), np.array([[1, 1, 0, 1]]), np.array([[0, 0, 0, 1]])]
    assert H.union_over_time(m, 0.5, 4).tolist() == [[1, 0, 0, 1]]   # counts 3,1,1,4 > 2
    assert H.union_over_time(m, 0.75, 4).tolist() == [[0, 0, 0, 1]]  # > 3
    assert H.union_over_time(m, 0.0, 4).tolist() == [[1, 1, 1, 1]]
    cfg = UNetConfig.sd14(8)
    unet = UNet2DConditionModel.from_state_dict(make_state_dict(cfg, 0), cfg, "cpu")
    names = [n for n, _ in union_bake.down_projection_layers(unet)]
    hooked = [n for n, _ in unet.named_modules() if n.endswith("ff.net.2")]
    assert len(names) == 16 and names == hooked
    assert [tuple(m.weight.shape) for _, m in union_bake.down_projection_layers(unet)][:2] == [(320, 1280)] * 2


def test_vae_decoder_architecture():
    """SD-1.x AutoencoderKL decoder layout (diffusers naming): mid block (2 ResNets + one attention), 4 up blocks of
    3 ResNets, shortcuts where the width changes (512->256, 256->128), 3 upsamplers, conv_out to RGB."""
    from sdmoe.vae import VAEConfig, vae_param_specs
    specs = {n: s for n, s, _ in vae_param_specs(VAEConfig.sd14())}
    assert specs["decoder.conv_in.weight"] == (512, 4, 3, 3)
    assert specs["decoder.mid_block.attentions.0.to_q.weight"] == (512, 512)
    assert sum(n.endswith("conv1.weight") for n in specs) == 2 + 4 * 3
    assert sorted(n for n in specs if "conv_shortcut.weight" in n) == [
        "decoder.up_blocks.2.resnets.0.conv_shortcut.weight", "decoder.up_blocks.3.resnets.0.conv_shortcut.weight"]
    assert sum("upsamplers" in n and n.endswith("weight") for n in specs) == 3
    assert specs["decoder.conv_out.weight"] == (3, 128, 3, 3)
    n = sum(int(torch.tensor(s).prod()) for s in specs.values())
    assert 49_000_000 < n < 50_000_000  # ~49.5M decoder parameters


def test_initial_latents_unseeded_process_seed():
    """An unseeded process's torch.initial_seed() is a random 64-bit value; the per-prompt latent seed must not
    overflow the generator (seeds below 2^63 / 1000003 keep their old streams)."""
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import initial_latents
    cfg = UNetConfig.tiny(8)
    a = initial_latents(2 ** 64 - 1, 3, cfg)
    assert a.shape == (1, 4, 8, 8) and torch.isfinite(a).all()
    g = torch.Generator().manual_seed(7 * 1_000_003 + 2)
    assert torch.equal(initial_latents(7, 2, cfg), torch.randn((1, 4, 8, 8), generator=g))


def test_interleave_ln_fold_matches_geglu_interleave():
    """The LayerNorm fold's rows (folded weight, fp32 bias, row sums) are reordered exactly like interleave_geglu
    reorders the projection's rows, so sdmoe_linear_geglu_ln sees the same [value 2 | gate 2] expert-major layout."""
    from sdmoe import ops
    F, K = 160, 64
    g = torch.Generator().manual_seed(3)
    w = torch.randn(2 * F, K, generator=g)
    b = torch.randn(2 * F, generator=g)
    perm = torch.randperm(F, generator=g)
    fold = ops.LNFold.__new__(ops.LNFold)
    fold.eps, fold.w, fold.bias, fold.wsum = 1e-5, w, b, w.sum(1)
    il = ops.interleave_ln_fold(fold, perm)
    w_il, b_il = ops.interleave_geglu(w, b, perm)
    assert torch.equal(il.w, w_il) and torch.equal(il.bias, b_il)
    assert torch.equal(il.wsum, w_il.sum(1))


def test_conv_weight_with_shortcut_layout():
    """[Cout, 9*Cin + Cin2]: conv2's implicit-GEMM K order first, then the 1x1 shortcut's input channels."""
    from sdmoe import ops
    Cout, Cin, Cin2 = 16, 64, 128
    w = torch.randn(Cout, Cin // 64, 3, 3, 64)
    ws = torch.randn(Cout, Cin2)
    cat = ops.conv_weight_with_shortcut(w, ws)
    assert cat.shape == (Cout, 9 * Cin + Cin2) and cat.is_contiguous()
    assert torch.equal(cat[:, :9 * Cin], w.reshape(Cout, -1)) and torch.equal(cat[:, 9 * Cin:], ws)


def test_sdmoe_tune_env_is_parsed_at_load(monkeypatch):
    """SDMOE_TUNE="knob=value,..." applies sdmoe_tune at library load; a bad knob raises."""
    from sdmoe import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setenv("SDMOE_TUNE", "1=0,0=0")
    assert _lib.load() is not None
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setenv("SDMOE_TUNE", "99=1")
    with pytest.raises(_lib.SdmoeError):
        _lib.load()
    for bad in ("7", "a=1", "1=b", "1=2=3", "=1"):  # malformed entries: SdmoeError, not a bare ValueError
        monkeypatch.setattr(_lib, "_lib", None)
        monkeypatch.setenv("SDMOE_TUNE", bad)
        with pytest.raises(_lib.SdmoeError, match="SDMOE_TUNE"):
            _lib.load()
    assert _lib.parse_tune(" 1=0, 16=2,,") == [(1, 0), (16, 2)]
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.delenv("SDMOE_TUNE")
    _lib.load()


def test_bench_roofline_timer_samples_whole_evaluations():
    """bench.KernelTimer times the conv launches of every N-th U-Net evaluation only (event markers idle the GPU
    between kernels): on_eval is set for evaluations 0, N, 2N, ... of the active region and nowhere else."""
    import bench

    seen = []

    class FakeUNet:
        def forward_nhwc(self, *a, **k):
            seen.append(timer.on_eval)

    timer = bench.KernelTimer("conv3x3_launch", sample_every=10)
    u = FakeUNet()
    timer.wrap_evals(u)
    u.forward_nhwc()  # inactive: not counted
    timer.active = True
    for _ in range(25):
        u.forward_nhwc()
    timer.active = False
    assert seen[0] is False
    assert [i for i, on in enumerate(seen[1:]) if on] == [0, 10, 20]
    assert timer.evals == 25 and timer.sampled_evals == 3 and timer.on_eval is False


def _gelu_tab_h_np(x16, tab):
    """numpy restatement of csrc/common.h gelu_tab_h over fp16 inputs (fmaf emulated in float64, exact here: the
    products of two float32 values are exact in float64 and the sums round once to float32 below)."""
    u = x16.view(np.uint16).astype(np.int64)
    a = u & 0x7FFF
    np.seterr(over="ignore")  # the series is evaluated (and discarded) for every input, huge ones included
    f = x16.astype(np.float32).astype(np.float64)
    x2 = np.float32(f * f).astype(np.float64)
    inner = np.float32(x2 * np.float64(np.float32(-0.0664903745)) + np.float64(np.float32(0.3989422804)))
    small = np.float32(x2 * inner.astype(np.float64) + np.float64(np.float32(0.5 * f))).astype(np.float16)
    idx = np.clip(a - 0x2800, 0, 8191) | ((u >> 15) << 13)
    t = tab[idx]
    big = np.where(u & 0x8000, np.float16(-0.0), x16)
    return np.where(a < 0x2800, small, np.where(a >= 0x4800, big, t))


def test_gelu_table_reproduces_reference_activation():
    """The GEGLU kernels' GELU (csrc/common.h gelu_tab_h + the table ops.ensure_gelu_table registers) against the
    reference's own fp16 activation (F.gelu on an fp16 tensor: diffusers GEGLU.gelu, the hook's module.gelu(gate)) on
    EVERY finite fp16 input: the table covers 2^-5 <= |x| < 8 by construction; the fp32 series below 2^-5 and the
    saturated ends must reproduce F.gelu too (bit for bit up to a documented handful of inputs)."""
    import torch.nn.functional as F
    from sdmoe import ops
    xs_tab = ops.gelu_table_values()
    assert xs_tab.dtype == torch.float16 and xs_tab.numel() == 16384
    a = xs_tab.view(torch.int16).numpy().astype(np.int64) & 0x7FFF
    assert a.min() == 0x2800 and a.max() == 0x47FF  # 2^-5 <= |x| < 8
    tab = F.gelu(xs_tab).numpy()
    allx = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16)
    allx = allx[np.isfinite(allx)]
    ref = F.gelu(torch.from_numpy(allx.copy())).numpy()
    got = _gelu_tab_h_np(allx, tab)
    same = (got.view(np.uint16) == ref.view(np.uint16)) | ((got == 0) & (ref == 0))
    bad = allx[~same]
    # everything bit-identical except inputs outside the table whose fp32 series rounds the other way (measured: 1,
    # x = 2^-24, whose gelu is an exact fp16 tie that torch's vectorised erf form rounds up)
    assert (~same).sum() <= 1, bad
    assert np.all(np.abs(bad.astype(np.float32)) < 2.0 ** -5)
    ulps = np.abs(got[~same].astype(np.float32) - ref[~same].astype(np.float32)) / np.spacing(np.abs(ref[~same]))
    assert np.all(ulps <= 1.0)




def test_geglu_rows_layout():
    """sdmoe_linear_geglu's weight layout (ops.geglu_rows, include/sdmoe.h): rows 4 q .. 4 q + 3 = value 2 q, value
    2 q + 1, gate 2 q, gate 2 q + 1 of the (permuted) neurons; a permutation of all 2F rows."""
    from sdmoe import ops
    F = 120
    rows = ops.geglu_rows(F, None, "cpu")
    assert sorted(rows.tolist()) == list(range(2 * F))
    for r in range(2 * F):
        q, e = divmod(r, 4)
        c = 2 * q + (e & 1)
        assert rows[r].item() == (c if e < 2 else F + c)
    perm = torch.randperm(F, generator=torch.Generator().manual_seed(5))
    rp = ops.geglu_rows(F, perm, "cpu")
    assert torch.equal(rp, torch.where(rows < F, perm[rows % F], F + perm[rows % F]))
    w = torch.randn(2 * F, 8)
    w_il, _ = ops.interleave_geglu(w, None, perm)
    assert torch.equal(w_il[0], w[perm[0]]) and torch.equal(w_il[2], w[F + perm[0]]) and torch.equal(w_il[5], w[perm[3]])


def test_masked_gemm_plans_take_the_plain_split():
    """Keep-/Wanda-masked down projections are bit-identical to mask-then-sdmoe_linear only if they split K the same
    way (the split fixes each output's fp32 summation order; tile and wave shape do not). sdmoe_gemm_plan derives the
    masked launch from the plain GEMM's plan; this checks it over every FFN down projection SD-1.4 and SDXL issue at
    1 / 2 / 8 / 16 prompts per call, with and without the residual, plus a sweep of other shapes (M tails, the
    768px one-image shape M = 9216 of ADVICE r05, K up to 10240)."""
    from unet_shapes import down_projection_shapes
    from sdmoe import ops
    shapes = down_projection_shapes("sd14") + down_projection_shapes("sdxl")
    assert (8192, 1280, 320) in shapes and (131072, 2560, 640) in shapes  # SD-1.4 B = 1 64x64, SDXL B = 16 64x64
    sweep = [(m, k, n) for m in (64, 128, 200, 512, 1000, 2048, 4096, 6000, 9216, 16384, 40000, 65536)
             for k in (320, 1280, 2560, 5120, 10240) for n in (320, 640, 1280)]
    for M, K, N in shapes + sweep:
        for res in (False, True):
            plain = ops.gemm_plan("plain", M, N, K, residual=res)
            for mode in ("keep", "wmask", "keepw"):
                got = ops.gemm_plan(mode, M, N, K, residual=res)
                assert got["ksplit"] == plain["ksplit"], (mode, M, K, N, res, got, plain)
    # the U-Net's own shapes keep the tiles they were tuned on: 4x2 waves on 256x320 for the keep-masked A operand
    assert ops.gemm_plan("keep", 65536, 320, 1280) == {"tile": (256, 320), "waves": (4, 2), "ksplit": 1}
    assert ops.gemm_plan("plain", 65536, 320, 1280)["waves"] == (2, 4)
    assert ops.gemm_plan("keep", 8192, 320, 1280)["tile"] == (64, 160)    # one prompt, 64x64 level
    assert ops.gemm_plan("keep", 1024, 1280, 5120)["tile"] == (256, 160)  # 8 prompts, mid block
    # no empty trailing split: every split gets >= 1 K-step
    for M, K, N in sweep:
        ks = ops.gemm_plan("plain", M, N, K)["ksplit"]
        nk = K // 64
        kchunk = -(-nk // ks)
        assert (ks - 1) * kchunk < nk, (M, K, N, ks)
    # without a workspace nothing splits; sdmoe_linear_ln never splits
    assert ops.gemm_plan("plain", 128, 1280, 5120, workspace_floats=0)["ksplit"] == 1
    assert ops.gemm_plan("ln", 128, 1280, 1280)["ksplit"] == 1
