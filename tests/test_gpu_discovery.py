"""Skill-discovery kernels and receivers on the MI355X vs the CPU oracle
(oracle/hooks_ref.py, itself pinned to the reference's GetExperts / Wanda hooks by tests/test_oracle_golden.py).

Bars: Wanda mask bits bit-exact (integer selection over identical fp16 metrics); token-mean expert scores
within 1 fp16 ulp of the oracle (fp32 summation order) and the top-k set identical wherever the k-th/(k+1)-th
mean scores are further apart than that; column norms rel 1e-4 (fp32); GetExperts dense outputs within the fp16
GEMM tolerance 1e-2 * max(1, |ref|).
"""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe import ops, discovery  # noqa: E402
from oracle import hooks_ref as H  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


def fp16_ulp(v):
    return np.spacing(np.abs(np.asarray(v, dtype=np.float16))).astype(np.float32)


def check_topk(dev_ids, mean_ref, k):
    """dev_ids must equal the oracle's top-k set unless the boundary gap is within 2 fp16 ulps."""
    m = mean_ref.float().numpy()
    order = np.argsort(-m, kind="stable")
    s = m[order]
    if k < len(m) and s[k - 1] - s[k] <= 2 * fp16_ulp(s[k - 1]):
        # near tie: the device set must still be a valid top-k up to that margin
        thr = s[k - 1] - 2 * fp16_ulp(s[k - 1])
        assert all(m[i] >= thr for i in dev_ids)
        return False
    assert set(dev_ids) == set(order[:k].tolist())
    return True


@pytest.mark.parametrize("M,E,k,bb", [(4096, 64, 12, None), (65536, 64, 12, None), (16384, 128, 25, [0, 5, 77, 1023]),
                                      (2048, 256, 51, None), (1000, 1024, 100, None), (8192, 256, 51, list(range(0, 512, 3)))])
def test_expert_mean_topk_kernel(M, E, k, bb):
    g = torch.Generator().manual_seed(M + E)
    score = (torch.randn(M, E, generator=g) * 3).half()
    rows_per_img = 1024 if bb else 0
    if bb:
        sel_rows = (torch.arange(M // 1024)[:, None] * 1024 + torch.tensor(bb)[None, :]).reshape(-1)
        ref = H.mean_scores(score[sel_rows])
        idx = torch.tensor(bb, dtype=torch.int32, device=DEV)
    else:
        ref = H.mean_scores(score)
        idx = None
    mean = torch.empty(E, dtype=torch.float16, device=DEV)
    ids = ops.expert_mean_topk(score.to(DEV), k, rows_per_img=rows_per_img, row_idx=idx, mean_out=mean)
    torch.cuda.synchronize()
    d = (mean.float().cpu() - ref.float()).abs().numpy()
    assert np.all(d <= fp16_ulp(ref.float().numpy()))
    ids = ids.cpu().tolist()
    assert len(set(ids)) == k
    # descending order of the device's own means
    mv = mean.float().cpu().numpy()
    assert all(mv[ids[i]] >= mv[ids[i + 1]] for i in range(k - 1))
    check_topk(ids, ref, k)


def test_expert_mean_topk_ties_lowest_id():
    score = torch.zeros(64, 32, dtype=torch.float16)
    score[:, 7] = 1.0
    ids = ops.expert_mean_topk(score.to(DEV), 5).cpu().tolist()
    assert ids == [7, 0, 1, 2, 3]


@pytest.mark.parametrize("M,F", [(8192, 1280), (2048, 2560), (512, 5120), (77, 320)])
def test_colnorm_accum_kernel(M, F):
    g = torch.Generator().manual_seed(F)
    P1 = (torch.randn(M, F, generator=g) * torch.rand(M, 1, generator=g) * 4).half()
    P2 = (torch.randn(M // 2 + 1, F, generator=g)).half()
    P2[0] = 0  # an all-zero row: normalize's eps clamp keeps it zero
    s = torch.zeros(F, dtype=torch.float32, device=DEV)
    ops.colnorm_accum(P1.to(DEV), s)
    ops.colnorm_accum(P2.to(DEV), s)
    ref = H.column_norm_sumsq(P2, H.column_norm_sumsq(P1))
    assert torch.allclose(s.cpu(), ref, rtol=1e-4, atol=1e-6)
    # strided view (a slice of a wider buffer)
    buf = torch.zeros(M, F + 64, dtype=torch.float16)
    buf[:, 32:32 + F] = P1
    s2 = torch.zeros(F, dtype=torch.float32, device=DEV)
    ops.colnorm_accum(buf.to(DEV)[:, 32:32 + F], s2)
    assert torch.allclose(s2.cpu(), H.column_norm_sumsq(P1), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("C,F,ratio,quant", [(320, 1280, 0.05, False), (640, 2560, 0.05, True), (1280, 5120, 0.1, False),
                                             (64, 320, 0.5, True), (16, 1280, 0.0, False), (8, 64, 1.0, True)])
def test_wanda_mask_kernel_bit_exact(C, F, ratio, quant):
    g = torch.Generator().manual_seed(C + F)
    W = torch.randn(C, F, generator=g) * 0.05
    nb = torch.rand(F, generator=g) * 30
    na = torch.rand(F, generator=g) * 30
    if quant:  # coarse values -> many exact ties at the top-k boundary and between base and adjusted metrics
        W = (W * 40).round() / 40
        nb, na = nb.round(), na.round()
    W, nb, na = W.half(), nb.half(), na.half()
    bits = ops.wanda_mask(W.to(DEV), nb.to(DEV), na.to(DEV), int(ratio * F)).cpu().numpy()
    ref = H.wanda_mask(W, nb, na, ratio).numpy()
    got = np.unpackbits(bits, axis=-1, count=F, bitorder="little").astype(np.int64)
    assert np.array_equal(got, ref)


# ------------------------------------------------------------------------------------------ receivers
def golden(kind):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "*.npz"))):
        with np.load(f, allow_pickle=False) as z:
            if str(z["kind"]) == kind:
                out.append((os.path.basename(f), {k: z[k] for k in z.files}))
    return out


def make_geglu_module(C, seed, labels, topk, act):
    import sys
    sys.path.insert(0, GOLD)
    import synth
    from sdmoe.unet import GEGLU, LoRACompatibleLinear, _gelu
    from moefication.helper import modify_ffn
    w, b = synth.geglu_weights(C, seed)
    m = GEGLU(LoRACompatibleLinear(torch.from_numpy(w).half().to(DEV), torch.from_numpy(b).half().to(DEV)))
    if act == "relu":
        m.gelu = torch.nn.functional.relu
    else:
        m.gelu = _gelu
    modify_ffn(m, None, topk, labels=labels)
    return m, torch.from_numpy(w).half(), torch.from_numpy(b).half()


@pytest.mark.parametrize("name,c", golden("getexperts"), ids=[n for n, _ in golden("getexperts")])
@pytest.mark.parametrize("fused", [True, False])
def test_get_experts_receiver_vs_golden(name, c, fused):
    """GetExperts.hook_fn on the device, on the reference golden inputs (fp16): dense output and the token-mean
    top-k vs the oracle (and through it the reference)."""
    from neuron_receivers import GetExperts
    C, E = int(c["C"]), int(c["E"])
    m, w, b = make_geglu_module(C, int(c["seed"]), c["labels"], 0.2, str(c["act"]))
    bb = c["bb"].tolist() or None
    m.bounding_box = bb
    m._allow_permuted_out = fused
    x = torch.from_numpy(c["x"]).half()
    rec = GetExperts(0, 1, 16, {"ffn0": E}, ["ffn0"] * 16)
    out = rec.hook_fn(m, (x.to(DEV),), None)
    rec.flush()
    if m._out_perm is not None:  # fused path: expert-major neuron order
        inv = torch.argsort(m._out_perm[0].perm)
        out = out[..., inv.to(DEV)]
    P = H.patterns_from_labels(c["labels"], torch.float16)
    o_ref, sel_ref, mean_ref = H.get_experts_hook(x, w, b, P, int(c["k"]), str(c["act"]), bb=bb)
    scale = max(1.0, o_ref.float().abs().max().item())
    assert (out.float().cpu() - o_ref.float()).abs().max().item() <= 1e-2 * scale
    ids = rec.label_counter[0][0]
    assert len(ids) == int(c["k"]) and (rec.timestep, rec.layer) == (0, 1)
    check_topk(ids, mean_ref, int(c["k"]))


def test_get_experts_and_wanda_pipeline_tiny():
    """End to end on the tiny U-Net: GetExperts fills label_counter[t][l] for every (t, l) with k distinct ids,
    leaves the images equal to the dense pipeline's; Wanda's column norms for base/adjusted prompts build masks
    (device kernel == oracle, bit-exact) that WandaRemoveNeuronsFast then consumes."""
    from test_gpu_unet import moefy_tiny
    from sdmoe.config import UNetConfig
    from sdmoe.unet import UNet2DConditionModel
    from sdmoe.weights import make_state_dict
    from sdmoe.pipeline import StableDiffusionPipeline
    from neuron_receivers import GetExperts, Wanda, WandaRemoveNeuronsFast
    cfg = UNetConfig.tiny(16)
    unet = UNet2DConditionModel.from_state_dict(make_state_dict(cfg, 2), cfg, DEV)
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    layers = moefy_tiny(pipe, topk=0.25, expert_size=16, relu=False)
    names = sorted(n + ".proj.weight" for n, _ in unet.named_modules() if n.endswith("ff.net.0"))
    nexp = {n: layers[i][1] for i, n in enumerate(names)}
    T, L = 2, 16
    ge = GetExperts(0, T, L, nexp, names)
    out_ge, _ = ge.observe_activation(pipe, "a photo of a dog")
    for t in range(T):
        for l in range(L):
            ids = ge.label_counter[t][l]
            assert len(ids) == layers[l][2] and len(set(ids)) == len(ids) and max(ids) < layers[l][1]
    # GetExperts does not mask: same latents as a pipeline without hooks on the MoE-fied model but dense FFN
    for _, mod in unet.named_modules():
        if hasattr(mod, "patterns"):
            mod._keep = mod.patterns
            mod.patterns = None
    dense = pipe("a photo of a dog").images[0]
    for _, mod in unet.named_modules():
        if hasattr(mod, "_keep"):
            mod.patterns = mod._keep
    assert ((out_ge - dense).norm() / dense.norm()).item() < 5e-3

    base, adj = Wanda(0, T, L), Wanda(0, T, L)
    base.observe_activation(pipe, "a church")
    adj.observe_activation(pipe, "a church in the style of Van Gogh")
    nb, na = base.predictivity.get_column_norms(), adj.predictivity.get_column_norms()
    assert nb[1][3].dtype == torch.float16 and nb[1][3].numel() == 4 * 128
    downs = {n: m.weight.detach().abs().cpu() for n, m in unet.named_modules() if n.endswith("ff.net.2")}
    masks = discovery.wanda_masks(downs, list(downs), nb, na, 0.05, T)
    dnames = sorted(downs)
    for t in range(T):
        for l in range(L):
            ref = H.wanda_mask(downs[dnames[l]].half(), nb[t][l], na[t][l], 0.05).numpy()
            got = np.unpackbits(masks[t][l], axis=-1, count=ref.shape[1], bitorder="little")
            assert np.array_equal(got.astype(np.int64), ref), (t, l)
    assert sum(int(masks[t][l].any()) for t in range(T) for l in range(L)) > 0
    rem = WandaRemoveNeuronsFast.from_packed(0, masks, T, L, store_gates=False)
    out_w, _ = rem.observe_activation(pipe, "a church in the style of Van Gogh")
    assert torch.isfinite(out_w).all()
