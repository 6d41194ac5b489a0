"""Pin the CPU oracle (oracle/hooks_ref.py) against golden vectors produced by the REFERENCE's own hook functions
(tests/golden/make_golden.py: MOEFy.hook_fn, RemoveExperts.hook_fn, WandaRemoveNeuronsFast.linear_hook_fn,
helper.modify_ffn, NeuronPredictivity counter). CPU only.

Bar: bit-exact in the reference dtype on every row whose top-k boundary is not a tie; on tie rows (k-th and
(k+1)-th score equal) torch.topk's order is implementation-defined, so the oracle (lowest-index tie-break) must
produce a tie-consistent selection and the rows are counted separately.
"""
import glob
import json
import os
import sys

import numpy as np
import pytest
import torch

from oracle import hooks_ref as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
import synth  # noqa: E402


def cases(kind):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, "*.npz"))):
        with np.load(f, allow_pickle=False) as z:
            if str(z["kind"]) == kind:
                out.append((os.path.basename(f), {k: z[k] for k in z.files}))
    return out


def tdtype(name):
    return {"float16": torch.float16, "float32": torch.float32}[str(name)]


def sel_from_topk(idx, E):
    s = np.zeros((idx.shape[0], E), dtype=bool)
    np.put_along_axis(s, idx.reshape(idx.shape[0], -1), True, axis=1)
    return s


@pytest.mark.parametrize("name,c", cases("moefy"), ids=[n for n, _ in cases("moefy")])
def test_moefy_golden(name, c):
    dt = tdtype(c["dtype"])
    C = int(c["C"])
    w, b = synth.geglu_weights(C, int(c["seed"]))
    w, b = torch.from_numpy(w).to(dt), torch.from_numpy(b).to(dt)
    assert H.k_from_topk(int(c["E"]), float(c["topk"])) == int(c["k"])
    P = H.patterns_from_labels(c["labels"], dt)
    x = torch.from_numpy(c["x"])
    out, gate, sel, score = H.geglu_hook(x, w, b, P, int(c["k"]), str(c["act"]))
    # projection restatement is bit-exact vs the reference's module.proj
    y = torch.nn.functional.linear(x, w, b)
    assert torch.equal(y, torch.from_numpy(c["y"]))
    assert torch.equal(score, torch.from_numpy(c["score"]))
    tie = c["tie"].astype(bool)
    ref_sel = sel_from_topk(c["sel"], int(c["E"]))
    ours = sel.numpy()
    assert (ours[~tie] == ref_sel[~tie]).all(), "selection differs on a non-tie row"
    # tie rows: same set of strictly-above-threshold experts, same count
    sc = score.float().numpy()
    k = int(c["k"])
    for r in np.where(tie)[0]:
        thr = np.sort(sc[r])[::-1][k - 1]
        assert (ours[r] & (sc[r] > thr)).sum() == (sc[r] > thr).sum() and ours[r].sum() == k
    rows_nt = np.repeat(~tie, 1).reshape(-1)
    o = out.reshape(-1, out.shape[-1]).numpy()
    ro = c["out"].reshape(-1, c["out"].shape[-1])
    assert np.array_equal(o[rows_nt], ro[rows_nt])
    assert np.array_equal(gate.reshape(-1, gate.shape[-1]).numpy()[rows_nt],
                          c["gate"].reshape(-1, c["gate"].shape[-1])[rows_nt])


@pytest.mark.parametrize("name,c", cases("remove"), ids=[n for n, _ in cases("remove")])
def test_remove_experts_golden(name, c):
    dt = tdtype(c["dtype"])
    C = int(c["C"])
    w, b = synth.geglu_weights(C, int(c["seed"]), float(c["gate_bias"]))
    w, b = torch.from_numpy(w).to(dt), torch.from_numpy(b).to(dt)
    P = H.patterns_from_labels(c["labels"], dt)
    lists = json.loads(str(c["lists"]))
    x = torch.from_numpy(c["x"])
    k = int(c["k"])
    counter = H.TimeLayerCounter(int(c["L"]))
    calls = list(c["calls"])
    n_removed_slots = 0
    for call in range(int(c["T"]) * int(c["L"])):
        t, l = counter.timestep, counter.layer
        if call in calls:
            i = calls.index(call)
            assert (t, l) == tuple(c["call_tl"][i])
            ids = lists[f"{t},{l}"]
            out, gate, sel, score = H.geglu_hook(x, w, b, P, k, str(c["act"]), removed=ids, apply_removal=t < 20)
            tie = H.tie_rows(score, k).numpy()
            o = out.reshape(-1, out.shape[-1]).numpy()
            ro = c["out"][i].reshape(-1, o.shape[-1])
            assert np.array_equal(o[~tie], ro[~tie]), f"call {call} (t={t}, l={l})"
            if t < 20 and ids:
                n_removed_slots += int(sel.numpy()[:, ids].sum())
        counter.update()
    if float(c["gate_bias"]) < 0:
        # the negative-score case must exercise "removed experts (score 0) still occupy top-k slots"
        assert n_removed_slots > 0


@pytest.mark.parametrize("name,c", cases("wanda"), ids=[n for n, _ in cases("wanda")])
def test_wanda_golden(name, c):
    dt = tdtype(c["dtype"])
    w, b = synth.down_weights(320, int(c["w_seed"]))
    w, b = torch.from_numpy(w).to(dt), torch.from_numpy(b).to(dt)
    x = torch.from_numpy(c["x"])
    bits = c["mask_bits"]
    for l in range(bits.shape[0]):
        mask = np.unpackbits(bits[l], axis=-1, count=1280, bitorder="little").astype(np.int64)
        y = H.wanda_linear(x, w, b, mask)
        ref = torch.from_numpy(c["out"][l])
        if dt == torch.float32:
            torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
        else:
            assert torch.equal(y, ref)
    # the reference fixture's mask density (weights_320_1280.csv): 2.2-2.8 %
    assert np.all((c["density"] > 0.02) & (c["density"] < 0.03))


def test_counter_golden():
    (name, c), = cases("counter")
    ctr = H.TimeLayerCounter(16)
    for tl in c["seq"]:
        assert (ctr.timestep, ctr.layer) == tuple(tl)
        ctr.update()
    ctr.reset()
    assert (ctr.timestep, ctr.layer) == tuple(c["after_reset"])


@pytest.mark.parametrize("name,c", cases("getexperts"), ids=[n for n, _ in cases("getexperts")])
def test_get_experts_golden(name, c):
    """GetExperts.hook_fn: dense output bit-exact; top-k of the token-mean score equal as a set unless the
    reference's k-th/(k+1)-th mean scores tie; counter advanced once."""
    dt = tdtype(c["dtype"])
    C = int(c["C"])
    w, b = synth.geglu_weights(C, int(c["seed"]))
    w, b = torch.from_numpy(w).to(dt), torch.from_numpy(b).to(dt)
    P = H.patterns_from_labels(c["labels"], dt)
    x = torch.from_numpy(c["x"])
    bb = c["bb"].tolist() or None
    out, sel, mean = H.get_experts_hook(x, w, b, P, int(c["k"]), str(c["act"]), bb=bb)
    assert torch.equal(out, torch.from_numpy(c["out"]))
    ref_mean = torch.from_numpy(c["mean"])
    # the reference ran on CPU: fp16 mean = fp16(sum) / n (two roundings) vs the device's one rounding
    tol = 0 if dt == torch.float32 else 2 * float(torch.finfo(torch.float16).eps) * float(ref_mean.abs().max())
    assert (mean.float() - ref_mean.float()).abs().max().item() <= tol + 1e-6 * float(ref_mean.abs().max())
    if not bool(c["tie"]):
        assert set(sel) == set(c["sel"].tolist())
    assert len(sel) == int(c["k"])
    assert c["counter_after"].tolist() == [0, 1]


@pytest.mark.parametrize("name,c", cases("wanda_colnorm"), ids=[n for n, _ in cases("wanda_colnorm")])
def test_wanda_colnorm_golden(name, c):
    """Wanda.hook_fn + TimeLayerColumnNorm over 2 prompts x T x L calls: the oracle's fp32 column norms match
    the reference's (fp32 exactly up to summation order; fp16 within its rounding of each step)."""
    dt = tdtype(c["dtype"])
    C, T, L = int(c["C"]), int(c["T"]), int(c["L"])
    mods = [tuple(torch.from_numpy(a).to(dt) for a in synth.geglu_weights(C, int(s))) for s in c["w_seeds"]]
    sums = {}
    calls = c["x"].shape[0]
    ctr = H.TimeLayerCounter(L)
    for i in range(calls):
        if i == T * L:
            ctr.reset()
        x = torch.from_numpy(c["x"][i])
        w, b = mods[i % L]
        h, g = torch.nn.functional.linear(x, w, b).chunk(2, -1)
        out = h * torch.nn.functional.gelu(g)
        key = (ctr.timestep, ctr.layer)
        sums[key] = H.column_norm_sumsq(out, sums.get(key))
        ctr.update()
    for t in range(T):
        for l in range(L):
            ours = sums[(t, l)].sqrt()
            ref = torch.from_numpy(c["norms"][t][l])
            rtol = 1e-5 if dt == torch.float32 else 4e-3
            assert torch.allclose(ours, ref, rtol=rtol, atol=1e-6), (t, l, (ours - ref).abs().max())


def test_wanda_mask_restatement_properties():
    """modularity/wanda.py:140-160 restatement: at most kprune bits per row, every set bit is among the row's
    kprune largest adjusted metrics and beats the base metric; ties at the boundary go to the lowest column."""
    g = torch.Generator().manual_seed(0)
    W = torch.randn(64, 256, generator=g).half()
    nb = torch.rand(256, generator=g).half()
    na = torch.rand(256, generator=g).half()
    m = H.wanda_mask(W, nb, na, 0.05)
    kp = int(0.05 * 256)
    assert int(m.sum(1).max()) <= kp
    ma = (W.abs() * na).float()
    mb = (W.abs() * nb).float()
    thr = torch.sort(ma, dim=1, descending=True).values[:, kp - 1:kp]
    assert bool(((m == 0) | ((ma >= thr) & (ma > mb))).all())
    # all-equal metrics: the first kprune columns are the selected ones
    m2 = H.wanda_mask(torch.ones(2, 64).half(), torch.zeros(64).half(), torch.ones(64).half(), 0.25)
    assert m2[:, :16].all() and not m2[:, 16:].any()
