"""The RECEIVERS themselves driven through the reference's golden call sequences (tests/golden, written by
make_golden.py from the reference's own hook functions).

test_gpu_route_parity.py checks the routing kernel on the reference's projection output and decides the removal
(t < 20) itself. Here the drop-in objects do everything, as a reference driver would use them:
  * the label file is written with torch.save and read by moefication.helper.modify_ffn (helper.py:48-62);
  * the per-(t, l) expert lists are JSON files read by RemoveExperts' constructor (remove_skilled_experts.py:13-19);
  * RemoveExperts.hook_fn / MOEFy.hook_fn are called with (module, (x,), None) for the whole golden sequence --
    44 calls for T = 22, L = 2: removal at t = 0..19, none at t = 20, 21 (:32) -- and the receiver's own (t, l)
    counter (predictivity.py:25-30) decides which list applies.

The hook computes its projection with the sdmoe GEMM (fp32 accumulation in another order than the CPU's fp16
linear), so a y element can differ from the reference's by an fp16 ulp -- at C = 1280 almost every row has one such
element. The contract per call (compare_call) is therefore:
  (1) the restated reference hook (oracle/hooks_ref.py, pinned bit-exactly to these goldens on CPU) on the DEVICE's
      y: output and stored gate bit-identical on every row that is not an exact top-k boundary tie (ReLU), or within
      the GELU contract of test_gpu_route_parity.check_out;
  (2) the golden output itself: the same bar on rows whose device y equals the golden y bit for bit, fp16
      tolerance on the others wherever the k-th/(k+1)-th gap clears the 8-ulp near-tie band.
"""
import glob
import json
import os
import sys
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe import ops  # noqa: E402
from sdmoe.unet import GEGLU, LoRACompatibleLinear  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import synth  # noqa: E402
from test_gpu_route_parity import check_out, fp16_spacing, near_tie_rows  # noqa: E402

DEV = "cuda"


def cases(kind):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLD, f"{kind}_*.npz"))):
        with np.load(f, allow_pickle=False) as z:
            if str(z["dtype"]) == "float16":
                out.append((os.path.basename(f), {k: z[k] for k in z.files}))
    return out


def make_module(c, d):
    """Our GEGLU with the fixture's weights, MoE-fied from a label FILE through helper.modify_ffn."""
    from moefication.helper import modify_ffn
    C = int(c["C"])
    w, b = synth.geglu_weights(C, int(c["seed"]), float(c["gate_bias"]) if "gate_bias" in c else 0.0)
    m = GEGLU(LoRACompatibleLinear(torch.from_numpy(w).half().to(DEV), torch.from_numpy(b).half().to(DEV)))
    if str(c["act"]) == "relu":
        m.gelu = torch.nn.functional.relu  # sparsity/relufy_model.py:35
    lp = os.path.join(d, "labels")
    torch.save([np.int64(v) for v in c["labels"]], lp)  # ParamSplit.save's format (moe_utils.py:54-61)
    modify_ffn(m, lp, float(c["topk"]) if "topk" in c else 0.2)
    assert m.k == int(c["k"]) and m.patterns.shape == (int(c["E"]), 4 * C)
    return m, w, b


def compare_call(c, i, y_dev, out, gate, P, ids, apply_removal, k, relu, totals):
    """One hooked call, two contracts:
      (1) the reference hook arithmetic restated in oracle/hooks_ref.py (itself pinned bit-exactly to these
          goldens by tests/test_oracle_golden.py) applied to the DEVICE's projection y: the receiver's output and
          stored gate are bit-identical on every row that is not an exact k-th-score tie (ReLU; a tie at score 0
          selects no neuron either way, so those rows are compared too), or within the GELU contract of
          test_gpu_route_parity.check_out (GELU: the reference's CPU fp16 GELU is not correctly rounded);
      (2) the golden output itself: bit-identical on rows whose device y equals the golden y bit for bit, and within
          fp16 tolerance on the others wherever the k-th/(k+1)-th gap clears the 8-ulp near-tie band."""
    from oracle import hooks_ref as H
    C = int(c["C"])
    act = "relu" if relu else "gelu"
    yg = c["y"].reshape(-1, 8 * C)
    ro = (c["out"][i] if i is not None else c["out"]).reshape(-1, 4 * C)
    rg = (c["gate"][i] if i is not None else c["gate"]).reshape(-1, 4 * C)
    o, g = out.reshape(-1, 4 * C), gate.reshape(-1, 4 * C)
    # (1) the restated hook on the device's y
    o1, g1, _, s1 = H.routed_geglu(torch.from_numpy(y_dev), P, k, act, ids, apply_removal)
    o1, g1, s1 = o1.numpy(), g1.numpy(), s1.float().numpy()
    s = np.sort(s1, axis=1)[:, ::-1]
    tie = (s[:, k - 1] == s[:, k]) if k < s.shape[1] else np.zeros(s.shape[0], bool)
    if relu:
        rows = ~tie | (s[:, k - 1] == 0)
        assert np.array_equal(o[rows], o1[rows]), f"call {i}: output differs from the restated hook"
        assert np.array_equal(g[rows], g1[rows]), f"call {i}: stored gate differs from the restated hook"
    else:
        rows = ~tie & ~near_tie_rows(s1, k)
        check_out(o, o1, g, g1, y_dev[:, :4 * C], rows)
    # (2) the golden output
    exact_y = (y_dev == yg).all(1)
    if relu:
        assert np.array_equal(o[exact_y & rows], ro[exact_y & rows]), f"call {i}: differs from golden on exact-y rows"
    else:
        check_out(o, ro, g, rg, yg[:, :4 * C], exact_y & rows)
    _, _, _, sg = H.routed_geglu(torch.from_numpy(yg), P, k, act, ids, apply_removal)  # the reference's own scores
    other = ~exact_y & ~tie & ~near_tie_rows(sg.float().numpy(), k, slack_ulps=8)
    if other.any():
        err = np.abs(o[other].astype(np.float32) - ro[other].astype(np.float32)).max()
        assert err <= 2e-2 * max(1.0, np.abs(ro.astype(np.float32)).max()), f"call {i}: {err}"
    # exact-tie rows: the device's tie-break may differ from the restatement's lowest-index one; where the choice does
    # not change the output (tied experts removed, or their gates all zero) the row is compared bit for bit too
    tie_same = tie & ~rows & (o == o1).all(1) & (g == g1).all(1)
    totals["rows"] += rows.size
    totals["compared"] += int(rows.sum() + tie_same.sum())
    totals["tie_rows_same_output"] += int(tie_same.sum())
    totals["exact_tie"] += int(tie.sum())
    totals["exact_y_rows"] += int(exact_y.sum())
    totals["golden_tolerance_rows"] += int(other.sum())


@pytest.mark.parametrize("name,c", cases("remove"), ids=[n for n, _ in cases("remove")])
def test_remove_experts_receiver_golden_sequence(name, c, parity_report):
    from oracle import hooks_ref as H
    from neuron_receivers import RemoveExperts
    C, E, k, T, L = (int(c[n]) for n in ("C", "E", "k", "T", "L"))
    relu = str(c["act"]) == "relu"
    lists = {tuple(map(int, key.split(","))): v for key, v in json.loads(str(c["lists"])).items()}
    with tempfile.TemporaryDirectory() as d:
        m, w, b = make_module(c, d)
        for (t, l), ids in lists.items():
            with open(os.path.join(d, f"timestep_{t}_layer_{l}.json"), "w") as f:
                json.dump(ids, f)
        rec = RemoveExperts(0, d, T, L)  # reads the JSON files (remove_skilled_experts.py:13-19)
    x = torch.from_numpy(c["x"]).to(DEV)
    y_dev = ops.linear(x.reshape(-1, C), m.proj.weight, m.proj.bias).cpu().numpy()
    keep = {int(cl): j for j, cl in enumerate(c["calls"])}
    P = H.patterns_from_labels(c["labels"], torch.float16)
    totals = dict(rows=0, exact_y_rows=0, exact_tie=0, compared=0, golden_tolerance_rows=0, tie_rows_same_output=0)
    with torch.no_grad():
        for call in range(T * L):
            tl = (rec.timestep, rec.layer)
            out = rec.hook_fn(m, (x,), None)
            if call not in keep:
                continue
            j = keep[call]
            assert tl == tuple(int(v) for v in c["call_tl"][j]), (call, tl)
            t, l = tl
            compare_call(c, j, y_dev, out.cpu().numpy(), rec.gates[call].numpy(), P, lists[(t, l)], t < 20, k, relu,
                         totals)
    assert (rec.timestep, rec.layer) == (T, 0) and len(rec.gates) == T * L
    assert totals["compared"] >= 0.85 * totals["rows"], totals
    parity_report(f"receiver_remove_sequence[{name}]", **totals)


@pytest.mark.parametrize("name,c", cases("moefy"), ids=[n for n, _ in cases("moefy")])
def test_moefy_receiver_golden(name, c, parity_report):
    from neuron_receivers import MOEFy
    C, k = int(c["C"]), int(c["k"])
    with tempfile.TemporaryDirectory() as d:
        m, w, b = make_module(c, d)
    rec = MOEFy(seed=0)
    x = torch.from_numpy(c["x"]).to(DEV)
    y_dev = ops.linear(x.reshape(-1, C), m.proj.weight, m.proj.bias).cpu().numpy()
    with torch.no_grad():
        out = rec.hook_fn(m, (x,), None)
    from oracle import hooks_ref as H
    P = H.patterns_from_labels(c["labels"], torch.float16)
    totals = dict(rows=0, exact_y_rows=0, exact_tie=0, compared=0, golden_tolerance_rows=0, tie_rows_same_output=0)
    compare_call(c, None, y_dev, out.cpu().numpy(), rec.gates[-1].numpy(), P, None, False, k, str(c["act"]) == "relu",
                 totals)
    assert totals["compared"] >= totals["rows"] // 2, totals  # one call of 16-64 rows: no fraction bar
    parity_report(f"receiver_moefy[{name}]", **totals)
