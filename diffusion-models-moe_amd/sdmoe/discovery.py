"""Skill discovery on the HIP kernels: the statistics that PRODUCE the removal lists and Wanda
masks the hot-path receivers consume.

  * ColumnNormCalculator / TimeLayerColumnNorm — utils.py:321-370 of the reference. The running column norm
    sqrt(c^2 + n^2) is kept on the device as a squared fp32 sum per (t, l) (sdmoe_colnorm_accum), so a hooked
    call costs one streaming pass over the GEGLU output instead of a device->host copy of it (the reference's
    `.detach().cpu()` per call, wanda_receiver.py:50).
  * wanda_masks — modularity/wanda.py:140-173: metric = |W_down| * act_norm per (t, l), per row the top
    `sparsity_ratio` adjusted-prompt metrics that also beat the base-prompt metric -> bit-packed masks on device
    (sdmoe_wanda_mask), saved in the reference's pickle format or the native .npz.
  * update_set_diff / select_skilled_experts / save_expert_lists — the host bookkeeping of
    modularity/moefy_skilled_experts.py:97-124 and mod_utils.py:178-182 that turns GetExperts label lists into
    the timestep_{t}_layer_{l}.json files RemoveExperts reads.
"""
from __future__ import annotations

import json
import os
import pickle
from collections import Counter

import numpy as np
import torch

from . import mask_io, ops


class ColumnNormCalculator:
    """Column L2 norms of a growing stack of (row-normalised) fp16 rows, accumulated on the device."""

    def __init__(self, device=None):
        self.device = device
        self.sumsq = None
        self.rows = 0

    def add_rows(self, rows: torch.Tensor):
        """rows: [M, F] fp16 device view of the RAW activations; each row is L2-normalised in the kernel
        (F.normalize(p=2, dim=1), wanda_receiver.py:52) before its squares are added."""
        if self.sumsq is None:
            self.sumsq = torch.zeros(rows.shape[1], dtype=torch.float32, device=rows.device)
        ops.colnorm_accum(rows, self.sumsq)
        self.rows += rows.shape[0]

    def get_column_norms(self) -> torch.Tensor:
        """fp16 CPU tensor [F] (the reference's norms are fp16 CPU tensors); empty if nothing was added."""
        if self.sumsq is None:
            return torch.tensor([])
        return self.sumsq.sqrt().to(torch.float16).cpu()


class TimeLayerColumnNorm:
    def __init__(self, T, n_layers):
        self.T = T
        self.n_layers = n_layers
        self.column_norms = {t: {i: ColumnNormCalculator() for i in range(n_layers)} for t in range(T)}

    def update(self, rows, t, n_layer):
        self.column_norms[t][n_layer].add_rows(rows)

    def get_column_norms(self):
        return {t: {i: self.column_norms[t][i].get_column_norms() for i in range(self.n_layers)}
                for t in range(self.T)}

    def save(self, path):
        torch.save(self.get_column_norms(), path)


def wanda_masks(gate_weights, layer_names, act_norms_base, act_norms_adj, sparsity_ratio, timesteps, device="cuda"):
    """modularity/wanda.py:140-160 for every (t, l): returns {t: {l: np.uint8 [C, F/8]}} bit-packed masks.
    gate_weights[name] = |W_down| (or W_down: the kernel takes |.|) [C, F]; norms [F] (any float dtype, used
    as fp16 like the reference's); kprune = int(sparsity_ratio * F)."""
    names = sorted(layer_names)  # wanda.py:131 sorts the layer names
    out = {}
    wdev = {}
    for t in range(timesteps):
        out[t] = {}
        for l, name in enumerate(names):
            if name not in wdev:
                wdev[name] = gate_weights[name].to(device, torch.float16).contiguous()
            W = wdev[name]
            F = W.shape[1]
            nb = act_norms_base[t][l].to(device, torch.float16).contiguous()
            na = act_norms_adj[t][l].to(device, torch.float16).contiguous()
            bits = ops.wanda_mask(W, nb, na, int(sparsity_ratio * F))
            out[t][l] = bits
    torch.cuda.synchronize()
    return {t: {l: out[t][l].cpu().numpy() for l in out[t]} for t in out}


def save_wanda_masks(masks, path, fmt="pkl"):
    """Write timestep_{t}_layer_{l}.pkl (scipy csr_matrix int64, wanda.py:169-173) or .npz (bit-packed)."""
    os.makedirs(path, exist_ok=True)
    for t, layers in masks.items():
        for l, bits in layers.items():
            if fmt == "npz":
                np.savez_compressed(os.path.join(path, f"timestep_{t}_layer_{l}.npz"), bits=bits)
                continue
            import scipy.sparse
            dense = mask_io.unpack_mask(bits, bits.shape[-1] * 8)
            with open(os.path.join(path, f"timestep_{t}_layer_{l}.pkl"), "wb") as f:
                pickle.dump(scipy.sparse.csr_matrix(dense), f)


def update_set_diff(set1, set2, symm=False):
    """mod_utils.py:178-182."""
    return set1.symmetric_difference(set2) if symm else set1.difference(set2)


def select_skilled_experts(set_diff, n_prompts, skill_ratio):
    """moefy_skilled_experts.py:110-121: experts that appear in the per-prompt set differences of at least
    int(skill_ratio * n_prompts) prompts, most common first."""
    out = {}
    for t, layers in set_diff.items():
        out[t] = {}
        for l, diffs in layers.items():
            counter = Counter(diffs).most_common(len(Counter(diffs)))
            thr = int(skill_ratio * n_prompts)
            out[t][l] = [int(e) for e, c in counter if c >= thr]
    return out


def save_expert_lists(lists, path):
    """timestep_{t}_layer_{l}.json files (moefy_skilled_experts.py:106-124) for RemoveExperts."""
    os.makedirs(path, exist_ok=True)
    for t, layers in lists.items():
        for l, ids in layers.items():
            with open(os.path.join(path, f"timestep_{t}_layer_{l}.json"), "w") as f:
                json.dump([int(e) for e in ids], f)
