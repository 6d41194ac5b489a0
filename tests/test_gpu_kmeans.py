"""Offline MoE-fication on the MI355X: fp32 MFMA distance kernel vs float64 numpy, the
native size-constrained k-means vs the float64 oracle (oracle/kmeans_ref.py, exact scipy assignment), and the
reference's ParamSplit flow (state dict -> labels file -> helper.modify_ffn -> routed GEGLU).
Parity of the clustering against k_means_constrained itself is UNPINNED (library absent offline).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe import kmeans  # noqa: E402
from oracle import kmeans_ref as KR  # noqa: E402

DEV = "cuda"


@pytest.mark.parametrize("n,k,d", [(5120, 256, 1280), (1280, 64, 320), (100, 7, 33), (64, 64, 4)])
def test_sqdist_f32_kernel(n, k, d):
    rng = np.random.default_rng(n + d)
    X = rng.standard_normal((n, d))
    C = rng.standard_normal((k, d))
    D = kmeans.sqdist(torch.from_numpy(X).float().to(DEV), torch.from_numpy(C).float().to(DEV)).cpu().numpy()
    ref = KR.sq_dists(X.astype(np.float32).astype(np.float64), C.astype(np.float32).astype(np.float64))
    assert np.allclose(D, ref, rtol=2e-5, atol=2e-5 * d)


@pytest.mark.parametrize("n,k,d", [(320, 16, 32), (640, 32, 64)])
def test_constrained_kmeans_native_matches_oracle(n, k, d):
    """Same init (sklearn k-means++ from the same seeds), fp32 device distances + native auction vs float64 +
    exact LSA: identical labels on tie-free data (L2-normalised Gaussian rows, like normalised gate weights)."""
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, d))
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    lab, C, inertia, _ = kmeans.constrained_kmeans(X, k, n // k, n_init=3, random_state=0, device=DEV)
    rl, rc, ri = KR.constrained_kmeans(X, k, n // k, n_init=3, random_state=0)
    assert np.all(np.bincount(lab, minlength=k) == n // k)
    assert np.array_equal(lab, rl)
    assert abs(inertia - ri) <= 1e-4 * ri
    assert np.allclose(C, rc, atol=1e-5)


def test_param_split_flow(tmp_path):
    """moefy_sd_model.py:28-45: torch.save(unet.state_dict()) -> ModelConfig/ParamSplit.split/save ->
    <res>/param_split/<template> -> helper.modify_ffn -> balanced experts the fused routing path accepts."""
    from moefication.moe_utils import ModelConfig, ParamSplit, RandomSplit
    from moefication.helper import modify_ffn
    from sdmoe.unet import GEGLU, LoRACompatibleLinear
    C = 320
    tmpl = "down_blocks.0.attentions.0.transformer_blocks.0.ff.net.0.proj.weight"
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(8 * C, C, generator=g) * C ** -0.5).half()
    torch.save({tmpl: w, "other.weight": torch.zeros(3)}, tmp_path / "model.pt")
    cfg = ModelConfig(str(tmp_path / "model.pt"), str(tmp_path / "res"), split_size=20)
    sp = ParamSplit(cfg, tmpl, n_init=2, max_iter=50)
    sp.split()
    sp.save()
    assert np.all(np.bincount(sp.labels, minlength=64) == 20)
    rnd = RandomSplit(cfg, tmpl)
    rnd.split()
    # clustering beats the trivial contiguous split on the objective it optimises
    x = w[4 * C:].double().numpy()
    x /= np.linalg.norm(x, axis=1, keepdims=True)

    def inertia(lab):
        lab = np.asarray(lab)
        return sum(((x[lab == c] - x[lab == c].mean(0)) ** 2).sum() for c in range(64))
    assert inertia(sp.labels) < inertia(rnd.labels)
    m = GEGLU(LoRACompatibleLinear(w.to(DEV), torch.zeros(8 * C, dtype=torch.float16, device=DEV)))
    modify_ffn(m, str(tmp_path / "res" / "param_split" / tmpl), 0.2)
    assert tuple(m.patterns.shape) == (64, 4 * C) and m.k == 12
    assert m.routing().fusable and m.routing().esize == 20
