"""Deterministic synthetic tensors shared by make_golden.py (generation, build container) and the parity tests
(GPU box): numpy PCG64 streams are bit-reproducible across machines, so fixtures store seeds, not weights."""
import numpy as np


def geglu_weights(C, seed, gate_bias=0.0):
    """GEGLU proj weight [8C, C] and bias [8C] (fp32), gate half biased by gate_bias."""
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((8 * C, C)) * C ** -0.5).astype(np.float32)
    b = (rng.standard_normal(8 * C) * 0.1).astype(np.float32)
    b[4 * C:] += np.float32(gate_bias)
    return w, b


def down_weights(C, seed):
    """ff.net.2 weight [C, 4C] and bias [C] (fp32)."""
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((C, 4 * C)) * (4 * C) ** -0.5).astype(np.float32)
    b = (rng.standard_normal(C) * 0.1).astype(np.float32)
    return w, b


def tokens(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def balanced_labels(F_, E, seed):
    """A balanced expert partition (F_/E neurons per expert) standing in for KMeansConstrained labels."""
    g = np.random.default_rng(seed)
    lab = np.repeat(np.arange(E), F_ // E)
    g.shuffle(lab)
    return lab.astype(np.int64)
