"""ORACLE (test infrastructure only) — float64 numpy restatement of size-constrained k-means as
k_means_constrained.KMeansConstrained (joshlk, not vendored in the reference, absent here: PARITY UNPINNED against
the library; restated from its published algorithm) runs it for moefication/moe_utils.py:97-107:
  X centred; tol = 1e-4 * mean column variance; n_init seeds = RandomState(random_state).randint(2^31-1, n_init);
  greedy k-means++ init (sklearn _k_init); Lloyd iterations whose E-step is the minimum-cost balanced assignment
  with Euclidean (not squared) costs — solved EXACTLY here with scipy.optimize.linear_sum_assignment on the cost
  matrix with every cluster column repeated n/k times (small problems only) — M-step = cluster means; best
  iterate kept, final E-step when not converged; best init by inertia.
Only tests/ may import this module.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linear_sum_assignment


def sq_dists(X, C):
    return np.maximum((X * X).sum(1)[:, None] + (C * C).sum(1)[None, :] - 2.0 * X @ C.T, 0.0)


def assign_exact(cost, k):
    n = cost.shape[0]
    s = n // k
    _, col = linear_sum_assignment(np.repeat(cost, s, axis=1))
    return (col // s).astype(np.int64)


def kpp(X, k, rs):
    n = X.shape[0]
    trials = 2 + int(np.log(k))
    C = np.empty((k, X.shape[1]))
    first = rs.randint(n)
    C[0] = X[first]
    closest = sq_dists(X[first:first + 1], X)[0]
    pot = closest.sum()
    for c in range(1, k):
        r = rs.random_sample(trials) * pot
        ids = np.minimum(np.searchsorted(np.cumsum(closest, dtype=np.float64), r), n - 1)
        d = np.minimum(closest[None, :], sq_dists(X[ids], X))
        p = d.sum(1)
        j = int(np.argmin(p))
        pot, closest = p[j], d[j]
        C[c] = X[ids[j]]
    return C


def constrained_kmeans(X, k, size, n_init=10, max_iter=300, tol=1e-4, random_state=0):
    X = np.asarray(X, dtype=np.float64)
    n = X.shape[0]
    assert n == k * size
    mu = X.mean(0)
    Xc = X - mu
    tol_abs = np.var(Xc, axis=0).mean() * tol
    seeds = np.random.RandomState(random_state).randint(np.iinfo(np.int32).max, size=n_init)

    def e_step(C):
        D = sq_dists(Xc, C)
        lab = assign_exact(np.sqrt(D), k)
        return lab, D[np.arange(n), lab].sum()

    best = None
    for seed in seeds:
        C = kpp(Xc, k, np.random.RandomState(seed))
        bl = bc = bi = None
        shift = 0.0
        for _ in range(max_iter):
            lab, inertia = e_step(C)
            newC = np.stack([Xc[lab == c].mean(0) for c in range(k)])
            if bi is None or inertia < bi:
                bl, bc, bi = lab, newC, inertia
            shift = ((C - newC) ** 2).sum()
            C = newC
            if shift <= tol_abs:
                break
        if shift > 0:
            bl, bi = e_step(bc)
        if best is None or bi < best[2]:
            best = (bl, bc + mu, bi)
    return best
