"""Size-constrained k-means (every cluster exactly n/k points) for offline MoE-fication — the algorithm of
k_means_constrained.KMeansConstrained that moefication/moe_utils.py:97-107 (ParamSplit.split) calls with
size_min = size_max = expert_size, n_init = 10, max_iter = 300, tol = 1e-4, random_state = 0.

k_means_constrained (joshlk, PyPI) is not vendored in the reference and is absent here, so this restates its
published algorithm (parity UNPINNED against the library itself):
  * X is centred on its column mean; tolerance = tol * mean(per-column variance) (sklearn _tolerance);
  * per init: sklearn's greedy k-means++ (_k_init: 2 + int(log k) local trials, potentials in float64) from
    RandomState(seed), seeds drawn as random_state.randint(int32 max, size=n_init);
  * iterate: assignment = minimum-cost flow with costs = Euclidean (not squared) point-centre distances and
    every cluster holding exactly n/k points; centres = cluster means; stop when the squared centre shift
    <= tolerance or after max_iter;
  * keep the init with the lowest inertia (sum of squared distances to the assigned centres).
MI355X split: the n x k distance matrix is one fp32 MFMA kernel (sdmoe_sqdist_f32) per iteration, the
assignment is the native epsilon-scaling auction (sdmoe_balanced_assign, exact for its integer costs), the
k-means++ init and centre means are host numpy (O(n d) per step).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def sqdist(X: torch.Tensor, C: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 device [n, k] squared distances between the rows of X [n, d] and C [k, d] (fp32, device)."""
    lib = _lib.load()
    if X.dtype != torch.float32 or C.dtype != torch.float32 or not X.is_cuda or not C.is_cuda:
        raise _lib.SdmoeError("sqdist: fp32 device tensors expected (no CPU path)")
    n, d = X.shape
    k = C.shape[0]
    if out is None:
        out = torch.empty((n, k), dtype=torch.float32, device=X.device)
    st = lib.sdmoe_sqdist_f32(X.data_ptr(), X.stride(0), C.data_ptr(), C.stride(0), n, k, d, out.data_ptr(),
                              out.stride(0), torch.cuda.current_stream().cuda_stream)
    _lib.check(st, "sdmoe_sqdist_f32")
    return out


def balanced_assign(cost: np.ndarray, k: int, scale: float = 0.0) -> np.ndarray:
    """Labels [n] minimising sum cost[i, label_i] with every cluster holding n/k points (host, native)."""
    lib = _lib.load()
    c = np.ascontiguousarray(cost, dtype=np.float64)
    n = c.shape[0]
    labels = np.zeros(n, dtype=np.int32)
    st = lib.sdmoe_balanced_assign(c.ctypes.data_as(ctypes.c_void_p), n, int(k), float(scale), None, 0,
                                   labels.ctypes.data_as(ctypes.c_void_p))
    _lib.check(st, "sdmoe_balanced_assign")
    return labels.astype(np.int64)


def _stable_cumsum(a):
    return np.cumsum(a, dtype=np.float64)


def kmeans_plusplus(X: np.ndarray, n_clusters: int, rs: np.random.RandomState, x_sq: np.ndarray) -> np.ndarray:
    """sklearn's greedy k-means++ (_k_init) in float64."""
    n, d = X.shape
    centers = np.empty((n_clusters, d), dtype=X.dtype)
    trials = 2 + int(np.log(n_clusters))
    cid = rs.randint(n)
    centers[0] = X[cid]
    closest = np.maximum(x_sq[cid] + x_sq - 2.0 * (X @ X[cid]), 0.0)
    pot = closest.sum()
    for c in range(1, n_clusters):
        vals = rs.random_sample(trials) * pot
        cand = np.searchsorted(_stable_cumsum(closest), vals)
        np.clip(cand, None, closest.size - 1, out=cand)
        dc = np.maximum(x_sq[cand][:, None] + x_sq[None, :] - 2.0 * (X[cand] @ X.T), 0.0)
        np.minimum(closest, dc, out=dc)
        pots = dc.sum(axis=1)
        best = int(np.argmin(pots))
        pot, closest = pots[best], dc[best]
        centers[c] = X[cand[best]]
    return centers


def constrained_kmeans(X: np.ndarray, n_clusters: int, size: int, n_init: int = 10, max_iter: int = 300,
                       tol: float = 1e-4, random_state: int = 0, device="cuda"):
    """Returns (labels int64 [n], centers [k, d] float64, inertia, n_iter of the kept init)."""
    X = np.asarray(X, dtype=np.float64)
    n, d = X.shape
    if n != n_clusters * size:
        raise ValueError(f"{n} points cannot form {n_clusters} clusters of exactly {size}")
    mean = X.mean(axis=0)
    Xc = X - mean
    tol_abs = float(np.mean(np.var(Xc, axis=0)) * tol)
    x_sq = (Xc * Xc).sum(axis=1)
    Xd = torch.from_numpy(Xc.astype(np.float32)).to(device)
    rs = np.random.RandomState(random_state)
    seeds = rs.randint(np.iinfo(np.int32).max, size=n_init)
    best = None

    def e_step(centers):
        D = sqdist(Xd, torch.from_numpy(centers.astype(np.float32)).to(device)).double().cpu().numpy()
        labels = balanced_assign(np.sqrt(D), n_clusters)
        return labels, float(D[np.arange(n), labels].sum())

    for seed in seeds:
        centers = kmeans_plusplus(Xc, n_clusters, np.random.RandomState(seed), x_sq)
        b_lab = b_cen = b_in = None
        shift = 0.0
        for it in range(1, max_iter + 1):  # sklearn's lloyd loop as k_means_constrained restates it
            old = centers
            labels, inertia = e_step(old)
            centers = np.zeros_like(old)
            np.add.at(centers, labels, Xc)
            centers /= size
            if b_in is None or inertia < b_in:
                b_lab, b_cen, b_in = labels, centers, inertia
            shift = float(((old - centers) ** 2).sum())
            if shift <= tol_abs:
                break
        if shift > 0:  # re-run the E-step so the labels match the returned centres
            b_lab, b_in = e_step(b_cen)
        if best is None or b_in < best[2]:
            best = (b_lab, b_cen + mean, b_in, it)
    return best
