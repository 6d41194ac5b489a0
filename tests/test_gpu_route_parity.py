"""Parity of the HIP routing kernel and the receiver hooks against the REFERENCE's golden vectors (tests/golden).

* route kernel fed the reference's own projection output y (fp16 cases): expert selection bit-exact on every
  row whose scores are identical and on every row whose k-th/(k+1)-th gap exceeds 2 fp16 ulps; gated output
  bit-exact wherever the activated gate is. The activated gate itself may differ by a few fp16 ulps on a small
  fraction of elements: the reference's CPU fp16 GELU is not correctly rounded (45 of 81,920 elements of one
  fixture differ from the fp64-rounded value), and in the negative tail its fp32 1+erf(x/sqrt2) cancels
  (our erfc form does not) -- measured max 3 ulps, 2 % of elements, in the gate-bias -1.5 fixture;
* full hook (our proj GEMM + route) vs the reference hook: output within fp16 tolerance 2e-2 * max|ref|, and
  selection identical on rows whose k-th/(k+1)-th score gap exceeds the GEMM's fp16 rounding (near-ties counted).
"""
import glob
import json
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


def cases(kinds, dtype="float16"):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "*.npz"))):
        with np.load(f, allow_pickle=False) as z:
            if str(z["kind"]) in kinds and str(z["dtype"]) == dtype:
                out.append((os.path.basename(f), {k: z[k] for k in z.files}))
    return out


def act_code(name):
    return {"gelu": ops.ACT_GELU, "relu": ops.ACT_RELU}[str(name)]


def sel_bits_to_bool(bits, E):
    b = bits.cpu().numpy().view(np.uint32)
    out = np.zeros((b.shape[0], E), dtype=bool)
    for e in range(E):
        out[:, e] = (b[:, e >> 5] >> (e & 31)) & 1
    return out


def fp16_spacing(a):
    return np.spacing(np.abs(a).astype(np.float16)).astype(np.float32)


def near_tie_rows(score, k, slack_ulps=2):
    """Rows whose k-th/(k+1)-th score gap is within `slack_ulps` fp16 ulps (1-ulp GELU/sum-order noise can
    legitimately reorder them)."""
    s = np.sort(score.astype(np.float32), axis=1)[:, ::-1]
    if k == 0 or k >= s.shape[1]:
        return np.zeros(s.shape[0], dtype=bool)
    return (s[:, k - 1] - s[:, k]) <= slack_ulps * fp16_spacing(s[:, k - 1])


def check_out(o, ro, g, rg, h, rows):
    """On `rows`: the activated gate equals the reference's up to 3 fp16 ulps (see module docstring; < 3 % of
    elements differ at all), and the output is bit-identical wherever the gate is, otherwise within
    |value| * |gate diff| + ulp(out) (the product's exact propagation of that gate difference)."""
    if not np.any(rows):
        return
    o, ro, g, rg, h = (a[rows].astype(np.float32) for a in (o, ro, g, rg, h))
    gd = np.abs(g - rg)
    sp = fp16_spacing(np.maximum(np.abs(g), np.abs(rg)))
    assert np.all(gd <= 3.01 * sp), f"gate max ulps {(gd / sp).max()}"
    assert (gd > 0).mean() < 3e-2, (gd > 0).mean()
    same = gd == 0
    assert np.array_equal(o[same], ro[same])
    tol = np.abs(h) * gd + fp16_spacing(np.maximum(np.abs(o), np.abs(ro)))
    assert np.all(np.abs(o - ro)[~same] <= 1.01 * tol[~same])


@pytest.mark.parametrize("name,c", cases({"moefy"}), ids=[n for n, _ in cases({"moefy"})])
def test_route_kernel_vs_reference_moefy(name, c, parity_report):
    """Selection contract: identical to the reference on every row that is not an exact tie at the
    k-th score. ReLU: relu(y) is exact in fp16 and the reference's fp16 score matmul is an fp32 sum of the same
    20 fp16 values rounded once, so scores, selection and output must be bit-identical on every such row.
    GELU: the reference's CPU fp16 GELU is not correctly rounded (module docstring), so a score may move by an
    ulp; a selection may then differ only on a row whose k-th/(k+1)-th gap is within 2 fp16 ulps (a near-tie
    flip) -- counted and reported, never accepted on a clear row."""
    C, E, k = int(c["C"]), int(c["E"]), int(c["k"])
    y = torch.from_numpy(c["y"]).reshape(-1, 8 * C).to(DEV)
    routing = ops.Routing(torch.from_numpy(c["labels"]), E, k, DEV)
    sel = torch.zeros((y.shape[0], (E + 31) // 32), dtype=torch.int32, device=DEV)
    score = torch.empty((y.shape[0], E), dtype=torch.float16, device=DEV)
    gate = torch.empty((y.shape[0], 4 * C), dtype=torch.float16, device=DEV)
    out = ops.geglu_route(y, routing, act_code(c["act"]), gate_out=gate, sel_out=sel, score_out=score)
    torch.cuda.synchronize()
    tie = c["tie"].astype(bool)  # exact ties at the boundary: torch.topk's order there is implementation-defined
    ref_score = c["score"]
    sc = score.cpu().numpy()
    ref_sel = np.zeros((y.shape[0], E), dtype=bool)
    np.put_along_axis(ref_sel, c["sel"].reshape(y.shape[0], -1), True, axis=1)
    ours = sel_bits_to_bool(sel, E)
    assert (ours.sum(1) == k).all()
    h = c["y"].reshape(-1, 8 * C)[:, :4 * C]
    mism = (ours != ref_sel).any(1)
    if str(c["act"]) == "relu":
        assert np.array_equal(sc, ref_score), f"{(sc != ref_score).sum()} scores differ"
        assert not mism[~tie].any(), f"selection differs on {int(mism[~tie].sum())} non-tie rows"
        assert np.array_equal(gate.cpu().numpy()[~tie], c["gate"].reshape(-1, 4 * C)[~tie])
        assert np.array_equal(out.cpu().numpy()[~tie], c["out"].reshape(-1, 4 * C)[~tie])
        parity_report(f"route_moefy[{name}]", rows=mism.size, exact_tie=tie.sum(), near_tie=0,
                      flips=(mism & ~tie).sum(), tie_row_choices_differing=(mism & tie).sum())
        return
    exact_score_rows = (sc == ref_score).all(1)
    assert not mism[~tie & exact_score_rows].any()  # identical scores -> identical selection
    near = near_tie_rows(ref_score, k)
    assert not mism[~tie & ~near].any(), "selection differs on a row clear of the near-tie band"
    parity_report(f"route_moefy[{name}]", rows=mism.size, exact_tie=tie.sum(), near_tie=(near & ~tie).sum(),
                  flips=(mism & ~tie).sum(), score_ulp_diffs=(sc != ref_score).sum())
    check_out(out.cpu().numpy(), c["out"].reshape(-1, 4 * C), gate.cpu().numpy(), c["gate"].reshape(-1, 4 * C), h,
              ~mism)


@pytest.mark.parametrize("name,c", cases({"remove"}), ids=[n for n, _ in cases({"remove"})])
def test_route_kernel_vs_reference_remove(name, c, parity_report):
    """RemoveExperts calls (removal for t < 20, score-0 semantics) on the reference's projection output: ReLU
    selection and output bit-identical on every row that is not an exact boundary tie; GELU flips only inside
    the near-tie band (counted). The fused path is bit-identical to this kernel (test_fused_geglu_bit_exact_*)."""
    C, E, k = int(c["C"]), int(c["E"]), int(c["k"])
    y = torch.from_numpy(c["y"]).reshape(-1, 8 * C).to(DEV)
    routing = ops.Routing(torch.from_numpy(c["labels"]), E, k, DEV)
    lists = json.loads(str(c["lists"]))
    from oracle import hooks_ref as H
    P = H.patterns_from_labels(c["labels"], torch.float16)
    relu = str(c["act"]) == "relu"
    totals = dict(rows=0, exact_tie=0, near_tie=0, flips=0)
    for i, (t, l) in enumerate(c["call_tl"]):
        ids = lists[f"{t},{l}"]
        removed = ops.removed_bits(ids, E, DEV) if (ids and t < 20) else None
        gate = torch.empty((y.shape[0], 4 * C), dtype=torch.float16, device=DEV)
        sel = torch.zeros((y.shape[0], (E + 31) // 32), dtype=torch.int32, device=DEV)
        out = ops.geglu_route(y, routing, act_code(c["act"]), removed=removed, gate_out=gate,
                              sel_out=sel).cpu().numpy()
        # boundary ties from the reference-dtype scores (same arithmetic as the hook; removed experts score 0)
        _, _, sel_o, score = H.routed_geglu(torch.from_numpy(c["y"]), P, k, str(c["act"]), ids, t < 20)
        tie = H.tie_rows(score, k).numpy()
        near = near_tie_rows(score.numpy(), k)
        ro = c["out"][i].reshape(-1, 4 * C)
        mism = (sel_bits_to_bool(sel, E) != sel_o.numpy()).any(1)
        totals["rows"] += tie.size
        totals["exact_tie"] += int(tie.sum())
        totals["near_tie"] += int((near & ~tie).sum())
        totals["flips"] += int((mism & ~tie).sum())
        if relu:
            assert not mism[~tie].any(), f"call {i}: selection differs on a non-tie row"
            assert np.array_equal(out[~tie], ro[~tie]), f"call {i}"
        else:
            assert not mism[~tie & ~near].any(), f"call {i}: selection differs on a clear row"
            check_out(out, ro, gate.cpu().numpy(), c["gate"][i].reshape(-1, 4 * C),
                      c["y"].reshape(-1, 8 * C)[:, :4 * C], ~near & ~tie)
    parity_report(f"route_remove[{name}]", **totals)


@pytest.mark.parametrize("name,c", cases({"moefy"}), ids=[n for n, _ in cases({"moefy"})])
def test_full_hook_vs_reference(name, c, parity_report):
    """Our proj GEMM + route on the reference's inputs vs the reference hook output. The projection is our own
    fp32-accumulated GEMM (1-ulp differences in y vs the CPU's fp16 linear), so the selection must agree on every
    row whose k-th/(k+1)-th gap exceeds 8 fp16 ulps; flips inside that band are counted and reported."""
    C, E, k = int(c["C"]), int(c["E"]), int(c["k"])
    w, b = synth.geglu_weights(C, int(c["seed"]))
    x = torch.from_numpy(c["x"]).reshape(-1, C).to(DEV)
    y = ops.linear(x, torch.from_numpy(w).half().to(DEV), torch.from_numpy(b).half().to(DEV))
    routing = ops.Routing(torch.from_numpy(c["labels"]), E, k, DEV)
    score = torch.empty((x.shape[0], E), dtype=torch.float16, device=DEV)
    out = ops.geglu_route(y, routing, act_code(c["act"]), score_out=score).float().cpu()
    ref = torch.from_numpy(c["out"].reshape(-1, 4 * C)).float()
    yref = torch.from_numpy(c["y"].reshape(-1, 8 * C)).float()
    assert (y.float().cpu() - yref).abs().max() <= 2e-2 * max(1.0, yref.abs().max().item())
    # rows whose selection boundary is clear of fp16 GEMM rounding must match exactly in selection
    s = np.sort(c["score"].astype(np.float32), axis=1)[:, ::-1]
    gap = s[:, k - 1] - s[:, k] if k < E else np.full(s.shape[0], np.inf)
    clear = gap > 8 * fp16_spacing(s[:, min(k, E - 1)])
    o, r = out.numpy(), ref.numpy()
    err = np.abs(o[clear] - r[clear]).max() if clear.any() else 0.0
    assert err <= 2e-2 * max(1.0, np.abs(r).max())
    ref_sel = np.zeros((x.shape[0], E), dtype=bool)
    np.put_along_axis(ref_sel, c["sel"].reshape(x.shape[0], -1), True, axis=1)
    ours = np.zeros_like(ref_sel)
    sc = score.float().cpu().numpy()
    ours[np.arange(sc.shape[0])[:, None], np.argsort(-sc, axis=1, kind="stable")[:, :k]] = True
    assert (ours[clear] == ref_sel[clear]).all()
    tie = c["tie"].astype(bool)
    mism = (ours != ref_sel).any(1)
    parity_report(f"full_hook[{name}]", rows=mism.size, exact_tie=tie.sum(), near_tie=(~clear & ~tie).sum(),
                  flips=(mism & ~tie).sum())


# ---- fused path: proj GEMM epilogue (value*act(gate) + expert scores) + top-k mask kernel -----------------

def _fused(x, w, b, routing, act, removed=None):
    w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
    score = torch.empty((x.shape[0], routing.E), dtype=torch.float16, device=DEV)
    sel = torch.zeros((x.shape[0], (routing.E + 31) // 32), dtype=torch.int32, device=DEV)
    P = ops.linear_geglu(x, w_il, b_il, act, score=score, esize=routing.esize)
    ops.moe_topk_mask(P, score, routing, removed=removed, sel_out=sel)
    out = torch.empty_like(P)
    out[:, routing.perm.to(DEV)] = P  # back to the natural neuron order
    return out, score, sel


@pytest.mark.parametrize("M,C,E,k,act,nrem", [(4096, 320, 64, 12, ops.ACT_GELU, 0), (1000, 320, 64, 12, ops.ACT_RELU, 5),
                                              (2048, 640, 128, 25, ops.ACT_GELU, 9), (512, 1280, 256, 51, ops.ACT_GELU, 20),
                                              (333, 640, 128, 128, ops.ACT_RELU, 0), (256, 320, 64, 12, ops.ACT_GELU, 3),
                                              (8192, 640, 128, 25, ops.ACT_GELU, 9)])
def test_fused_geglu_bit_exact_vs_unfused(M, C, E, k, act, nrem):
    """Same rounding points and the same neuron-order fp32 score sums as proj GEMM + sdmoe_geglu_route:
    output, scores and top-k bits are bit-identical (no split-K at K = C, so the GEMM sums agree too)."""
    g = torch.Generator().manual_seed(M + C)
    F = 4 * C
    x = (torch.randn(M, C, generator=g)).half().to(DEV)
    w = (torch.randn(2 * F, C, generator=g) * C ** -0.5).half().to(DEV)
    b = (torch.randn(2 * F, generator=g) * 0.3).half().to(DEV)
    labels = torch.randperm(F, generator=g) % E  # balanced, scattered over the neurons
    routing = ops.Routing(labels, E, k, DEV)
    assert routing.fusable and routing.esize == F // E
    removed = ops.removed_bits(torch.randperm(E, generator=g)[:nrem].tolist(), E, DEV) if nrem else None
    out, score, sel = _fused(x, w, b, routing, act, removed)
    y = ops.linear(x, w, b)
    score_u = torch.empty_like(score)
    sel_u = torch.zeros_like(sel)
    out_u = ops.geglu_route(y, routing, act, removed=removed, sel_out=sel_u, score_out=score_u)
    if removed is not None:  # the unfused kernel reports removed experts' scores as 0; fused reports raw sums
        rm = sel_bits_to_bool(removed.view(1, -1).expand(M, -1).contiguous(), E)
        score = score.masked_fill(torch.from_numpy(rm).to(DEV), 0)
    assert torch.equal(score, score_u)
    assert torch.equal(sel, sel_u)
    assert torch.equal(out, out_u)


@pytest.mark.parametrize("M,C,E,k,nrem,N", [(4096, 320, 64, 12, 5, 320), (1000, 320, 64, 12, 0, 320),
                                            (2048, 640, 128, 25, 9, 640), (777, 1280, 256, 51, 20, 1280),
                                            (256, 1280, 256, 51, 0, 1280), (333, 640, 128, 128, 0, 640)])
def test_keep_mask_in_down_projection_bit_exact(M, C, E, k, nrem, N):
    """sdmoe_moe_topk_keep + sdmoe_linear_keep (the mask applied to the down projection's A fragments) vs
    sdmoe_moe_topk_mask + sdmoe_linear: same top-k bits, keep bits = the zero pattern of the masked product, and a
    bit-identical down projection (+bias +residual), across tile choices, M tails and split-K (M = 256, K = 5120)."""
    g = torch.Generator().manual_seed(3 * M + C)
    F = 4 * C
    x = torch.randn(M, C, generator=g).half().to(DEV)
    w = (torch.randn(2 * F, C, generator=g) * C ** -0.5).half().to(DEV)
    b = (torch.randn(2 * F, generator=g) * 0.3).half().to(DEV)
    wd = (torch.randn(N, F, generator=g) * F ** -0.5).half().to(DEV)
    bd = (torch.randn(N, generator=g) * 0.1).half().to(DEV)
    res = torch.randn(M, N, generator=g).half().to(DEV)
    routing = ops.Routing(torch.randperm(F, generator=g) % E, E, k, DEV)
    removed = ops.removed_bits(torch.randperm(E, generator=g)[:nrem].tolist(), E, DEV) if nrem else None
    w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
    score = torch.empty((M, E), dtype=torch.float16, device=DEV)
    P = ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=routing.esize)
    Pm = P.clone()
    sel_m = torch.zeros((M, (E + 31) // 32), dtype=torch.int32, device=DEV)
    sel_k = torch.zeros_like(sel_m)
    ops.moe_topk_mask(Pm, score, routing, removed=removed, sel_out=sel_m)
    keep = ops.moe_topk_keep(score, routing, M, removed=removed, sel_out=sel_k)
    assert torch.equal(sel_m, sel_k)
    kb = keep.cpu().numpy().view(np.uint64)  # [F/64, M]
    bits = ((kb[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)  # [F/64, M, 64]
    kmask = torch.from_numpy(np.ascontiguousarray(bits.transpose(1, 0, 2).reshape(M, F))).to(DEV)
    assert torch.equal(Pm, torch.where(kmask, P, torch.zeros_like(P)))
    y_ref = ops.linear(Pm, wd, bd, residual=res)
    y = ops.linear_keep(P, keep, wd, bd, residual=res)
    assert torch.equal(y, y_ref)


def _unet_down_shapes():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from unet_shapes import down_projection_shapes
    return [("sd14",) + s for s in down_projection_shapes("sd14")] + [("sdxl",) + s for s in down_projection_shapes("sdxl")]


@pytest.mark.parametrize("model,M,K,N", _unet_down_shapes())
def test_masked_down_projection_bit_exact_every_unet_shape(model, M, K, N):
    """Every FFN down projection SD-1.4 (512^2) and SDXL (1024^2) issue at 1 / 2 / 8 / 16 prompts per call
    (tests/unet_shapes.py): the keep-masked product (sdmoe_linear_keep) equals top-k-masking the GEGLU product first and
    running sdmoe_linear, and with a Wanda mask as well (sdmoe_linear_masked, keep + wmask) it equals the plain GEMM
    on the masked product and the masked weight -- bit for bit, +bias +residual. (Both hold because the masked launch
    takes the plain GEMM's split-K plan, sdmoe_gemm_plan; test_host_logic checks the plans over a wider sweep.)"""
    g = torch.Generator().manual_seed(M + K + N)
    C, F = N, K
    E = F // 20
    k = int(E * 0.2)
    act = ops.ACT_RELU if model == "sd14" else ops.ACT_GELU
    x = torch.randn(M, C, generator=g).half().to(DEV)
    w = (torch.randn(2 * F, C, generator=g) * C ** -0.5).half().to(DEV)
    b = (torch.randn(2 * F, generator=g) * 0.3).half().to(DEV)
    wd = (torch.randn(N, F, generator=g) * F ** -0.5).half().to(DEV)
    bd = (torch.randn(N, generator=g) * 0.1).half().to(DEV)
    res = torch.randn(M, N, generator=g).half().to(DEV)
    routing = ops.Routing(torch.randperm(F, generator=g) % E, E, k, DEV)
    removed = ops.removed_bits(torch.randperm(E, generator=g)[:E // 10].tolist(), E, DEV)
    w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
    score = torch.empty((M, E), dtype=torch.float16, device=DEV)
    P = ops.linear_geglu(x, w_il, b_il, act, score=score, esize=routing.esize)
    keep = ops.moe_topk_keep(score, routing, M, removed=removed)
    y = ops.linear_keep(P, keep, wd, bd, residual=res)
    ops.moe_topk_mask(P, score, routing, removed=removed)  # P -> the top-k-masked product, in place
    assert torch.equal(y, ops.linear(P, wd, bd, residual=res)), "keep-masked vs mask-then-plain"
    # + a Wanda mask on the down projection's weight (config 4's fused form): ~2.5 % of the weights removed
    bits = (torch.rand(N, F, generator=g) < 0.025)
    packed = torch.from_numpy(np.packbits(bits.numpy(), axis=1, bitorder="little")).to(DEV)
    yw = ops.linear_keep(P, keep, wd, bd, residual=res, wmask=ops.wmask_kmajor(packed))
    assert torch.equal(yw, ops.linear(P, ops.mask_weight(wd, packed), bd, residual=res)), "keep+wmask vs masked-then-plain"


@pytest.mark.parametrize("M,E,k,nrem", [(4096, 256, 51, 20), (1000, 64, 12, 5), (16384, 128, 25, 0), (16385, 128, 25, 3)])
def test_topk_one_token_per_wave_matches_four(M, E, k, nrem):
    """The top-k kernels at one token per wave (M <= 16384, default) and four per wave (sdmoe_tune knob 15 = 4):
    identical selection, masked product and keep bits, on scores quantised to force ties at the k-th place."""
    from sdmoe import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + E)
    esize = 20
    F = E * esize
    routing = ops.Routing(torch.arange(F) // esize, E, k, DEV)
    score = (torch.randint(0, 12, (M, E), generator=g).float() / 4).half().to(DEV)  # many exact ties
    P = torch.randn(M, F, generator=g).half().to(DEV)
    removed = ops.removed_bits(torch.randperm(E, generator=g)[:nrem].tolist(), E, DEV) if nrem else None
    res = {}
    for tpw in (0, 4):
        _lib.check(lib.sdmoe_tune(15, tpw), "tune")
        try:
            Pm = P.clone()
            sel_m = torch.zeros((M, (E + 31) // 32), dtype=torch.int32, device=DEV)
            sel_k = torch.zeros_like(sel_m)
            ops.moe_topk_mask(Pm, score, routing, removed=removed, sel_out=sel_m)
            keep = ops.moe_topk_keep(score, routing, M, removed=removed, sel_out=sel_k)
            res[tpw] = (Pm, sel_m, sel_k, keep)
        finally:
            _lib.check(lib.sdmoe_tune(15, 0), "tune")
    for a_, b_ in zip(res[0], res[4]):
        assert torch.equal(a_, b_)
    assert torch.equal(res[0][1], res[0][2])


@pytest.mark.parametrize("M,E,k,nrem,esize,ld", [(65536, 64, 12, 5, 20, 64), (4097, 64, 13, 0, 20, 64),
                                                  (1000, 64, 64, 3, 20, 72), (333, 48, 9, 2, 20, 48),
                                                  (70, 32, 6, 1, 20, 33), (129, 64, 0, 0, 20, 64),
                                                  (500, 64, 12, 4, 10, 64), (256, 16, 4, 0, 40, 16),
                                                  (16384, 128, 25, 12, 20, 128), (2049, 128, 25, 0, 20, 136),
                                                  (77, 128, 128, 5, 20, 128), (4096, 256, 51, 25, 20, 256),
                                                  (513, 256, 51, 3, 20, 264), (100, 256, 0, 0, 20, 256),
                                                  (300, 128, 25, 2, 20, 130)])
def test_topk_keep_quad_kernel(M, E, k, nrem, esize, ld):
    """sdmoe_moe_topk_keep at E <= 64 (one quad of lanes per token, the default there) and at E = 128 / 256 with the
    reference's 20-neuron experts (a group of 8 / 16 lanes per token) vs the ballot kernel (sdmoe_tune knob 15 = 4)
    and vs a numpy restatement of the selection rule (moefy.py:20-23 top-k; ties at the k-th score toward the lowest
    expert id; removed experts score 0 and are never kept): identical keep words and selection bits, on scores
    quantised to force ties, with M tails, strided / unaligned score rows (ld != E; ld % 8 != 0 takes the ballot
    kernel), k = 0 and k = E."""
    from sdmoe import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(M + 7 * E + k)
    F = E * esize
    routing = ops.Routing(torch.arange(F) // esize, E, k, DEV)
    full = (torch.randint(-3, 12, (M, ld), generator=g).float() / 4).half()
    score = full.to(DEV)[:, :E]
    rm_list = torch.randperm(E, generator=g)[:nrem].tolist()
    removed = ops.removed_bits(rm_list, E, DEV) if nrem else None
    res = {}
    for tpw in (0, 4):
        _lib.check(lib.sdmoe_tune(15, tpw), "tune")
        try:
            sel = torch.zeros((M, (E + 31) // 32), dtype=torch.int32, device=DEV)
            keep = ops.moe_topk_keep(score, routing, M, removed=removed, sel_out=sel)
            torch.cuda.synchronize()
            res[tpw] = (sel.cpu(), keep.cpu())
        finally:
            _lib.check(lib.sdmoe_tune(15, 0), "tune")
    assert torch.equal(res[0][0], res[4][0])
    assert torch.equal(res[0][1], res[4][1])
    # numpy: stable descending order of the fp16 scores (removed -> 0; -0 == +0), first k are selected
    s = full[:, :E].float().numpy().copy()
    s[:, rm_list] = 0.0
    order = np.argsort(-s, axis=1, kind="stable")[:, :k]
    selb = np.zeros((M, E), bool)
    np.put_along_axis(selb, order, True, axis=1)
    got = sel_bits_to_bool(res[0][0], E)
    assert np.array_equal(got, selb)
    keepb = selb.copy()
    keepb[:, rm_list] = False
    neur = np.repeat(keepb, esize, axis=1)  # [M, F]
    kb = res[0][1].numpy().view(np.uint64)  # [F/64, M]
    bits = ((kb[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
    assert np.array_equal(bits.transpose(1, 0, 2).reshape(M, F), neur)


# 64x160 (table loaded after the K loop), 128x160, 256x160 4x2 (knob 20 = 0) / 256x320 2x4 (default at M = 8192) tiles
@pytest.mark.parametrize("M,gt320", [(64, 0), (4096, 0), (8192, 0), (8192, 1)])
def test_gelu_every_fp16_input_matches_reference_activation(M, gt320):
    """The GEGLU kernels' GELU on EVERY finite fp16 gate value vs the reference's activation itself (F.gelu on an fp16
    tensor: diffusers GEGLU.gelu, the hook's module.gelu(gate), moefy.py:13): sdmoe_geglu_route (gate_out) and the
    fused routed-GEGLU epilogue (value 1.0, so P = gelu(gate)) are bit-identical to it on all but <= 2 inputs (the fp32
    series below 2^-5, tests/test_host_logic.py::test_gelu_table_reproduces_reference_activation), and to each other.
    The fused GEMM is driven so that its gate outputs are exact chosen fp16 values: x rows are unit vectors e_(m % 64)
    and W's gate rows hold the values (one fp16 product per fp32 sum)."""
    allx = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.float16)
    allx = allx[torch.isfinite(allx)]
    F = 1280
    vals = torch.zeros(64 * F, dtype=torch.float16)
    vals[:allx.numel()] = allx
    gate = vals.view(64, F)                                   # gate[j, n]: the value row j of x selects
    # the reference's fp16 GELU on the device (the hook runs module.gelu on the GPU gate, moefy.py:13)
    ref = torch.nn.functional.gelu(gate.to(DEV)).cpu()
    # unfused: y = [value 1.0 | gate]
    y = torch.cat([torch.ones(64, F, dtype=torch.float16), gate], 1).to(DEV)
    g_out = torch.empty((64, F), dtype=torch.float16, device=DEV)
    ops.geglu_route(y, None, ops.ACT_GELU, gate_out=g_out)
    got_u = g_out.cpu()
    # fused: x = e_(m % 64) (K = 64), W = [ones | gate^T] rows, bias 0
    x = torch.zeros(M, 64, dtype=torch.float16)
    x[torch.arange(M), torch.arange(M) % 64] = 1.0
    w = torch.cat([torch.ones(F, 64, dtype=torch.float16), gate.t().contiguous()], 0).to(DEV)
    w_il, b_il = ops.interleave_geglu(w, torch.zeros(2 * F, dtype=torch.float16, device=DEV), None)
    from sdmoe import _lib
    lib = _lib.load()
    _lib.check(lib.sdmoe_tune(20, gt320), "tune")
    try:
        P = ops.linear_geglu(x.to(DEV), w_il, b_il, ops.ACT_GELU).cpu()
    finally:
        _lib.check(lib.sdmoe_tune(20, 1), "tune")
    exp_rows = torch.arange(M) % 64
    assert torch.equal(P, got_u[exp_rows])                    # fused == unfused, bit for bit
    same = (got_u.view(torch.int16) == ref.view(torch.int16)) | ((got_u == 0) & (ref == 0))
    bad = gate[~same]
    # the fp32 series below 2^-5 sits within an fp32 ulp of an fp16 rounding midpoint for a handful of inputs (the
    # reference's own fp32 1 + erf form rounds those either way too): <= 4 inputs, each within 1 fp16 ulp
    assert (~same).sum().item() <= 4, bad
    assert bool((bad.float().abs() < 2.0 ** -5).all())
    d = (got_u[~same].float() - ref[~same].float()).abs()
    sp = torch.from_numpy(np.spacing(np.abs(ref[~same].numpy()).astype(np.float16)).astype(np.float32))
    assert bool((d <= sp).all()), (d, sp)


def test_fused_geglu_dense_matches_unfused():
    M, C = 1500, 320
    g = torch.Generator().manual_seed(7)
    x = torch.randn(M, C, generator=g).half().to(DEV)
    w = (torch.randn(8 * C, C, generator=g) * C ** -0.5).half().to(DEV)
    b = (torch.randn(8 * C, generator=g) * 0.3).half().to(DEV)
    w_il, b_il = ops.interleave_geglu(w, b, None)
    assert torch.equal(ops.linear_geglu(x, w_il, b_il, ops.ACT_GELU), ops.geglu_route(ops.linear(x, w, b), None))


@pytest.mark.parametrize("name,c", cases({"moefy"}), ids=[n for n, _ in cases({"moefy"})])
def test_fused_hook_vs_reference(name, c, parity_report):
    """The fused path on the reference's inputs vs the reference hook output (same bar as the unfused path)."""
    C, E, k = int(c["C"]), int(c["E"]), int(c["k"])
    w, b = synth.geglu_weights(C, int(c["seed"]))
    x = torch.from_numpy(c["x"]).reshape(-1, C).to(DEV)
    routing = ops.Routing(torch.from_numpy(c["labels"]), E, k, DEV)
    assert routing.fusable
    out, score, sel = _fused(x, torch.from_numpy(w).half().to(DEV), torch.from_numpy(b).half().to(DEV), routing,
                             act_code(c["act"]))
    ref = c["out"].reshape(-1, 4 * C).astype(np.float32)
    s = np.sort(c["score"].astype(np.float32), axis=1)[:, ::-1]
    gap = s[:, k - 1] - s[:, k] if k < E else np.full(s.shape[0], np.inf)
    clear = gap > 8 * fp16_spacing(s[:, min(k, E - 1)])
    o = out.float().cpu().numpy()
    err = np.abs(o[clear] - ref[clear]).max() if clear.any() else 0.0
    assert err <= 2e-2 * max(1.0, np.abs(ref).max())
    ref_sel = np.zeros((x.shape[0], E), dtype=bool)
    np.put_along_axis(ref_sel, c["sel"].reshape(x.shape[0], -1), True, axis=1)
    ours = sel_bits_to_bool(sel, E)
    assert (ours[clear] == ref_sel[clear]).all()
    tie = c["tie"].astype(bool)
    mism = (ours != ref_sel).any(1)
    parity_report(f"fused_hook[{name}]", rows=mism.size, exact_tie=tie.sum(), near_tie=(~clear & ~tie).sum(),
                  flips=(mism & ~tie).sum())
