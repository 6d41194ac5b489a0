"""Static "union-timesteps" Wanda masks baked into the U-Net weights.

Restates benchmarks/save_union_over_time.py:160-246 of the reference: for every FFN down projection (`ff.net.2`,
layers in sorted-name order, :163-169 -- for SD-1.x that is also the hook-call order), count over the T
per-timestep masks M_t[l] (the `timestep_{t}_layer_{l}` files WandaRemoveNeuronsFast reads), keep the bits whose
count exceeds select_ratio * timesteps (:189-204), and bake W <- W * (1 - M) into the weights (:214-221), so the
removal costs nothing at run time (the "union-timesteps" checkpoint of `benchmarking results/union-timesteps`).
`binary_mask_iou` is iou_masks.py:8-14 on the bit-packed masks.

Device work: sdmoe_union_over_time (count + threshold over the packed masks) and sdmoe_mask_weight (the bake).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib, mask_io, ops


def down_projection_layers(unet):
    """(name, module) of every FFN down projection, sorted by name (save_union_over_time.py:163-169)."""
    mods = [(n, m) for n, m in unet.named_modules() if "ff.net" in n and "proj" not in n and n.endswith("ff.net.2")]
    return sorted(mods, key=lambda nm: nm[0])


def union_over_time(bits: torch.Tensor, select_ratio: float, timesteps: int | None = None) -> torch.Tensor:
    """bits: uint8 [T, C, F/8] device tensor of the T per-timestep masks of one layer. Returns the [C, F/8] mask
    of the bits set in more than select_ratio * timesteps of them (timesteps defaults to T)."""
    if bits.dim() != 3 or bits.dtype != torch.uint8 or not bits.is_cuda or not bits.is_contiguous():
        raise ValueError("bits must be a contiguous uint8 [T, C, F/8] device tensor")
    T = bits.shape[0]
    timesteps = T if timesteps is None else timesteps
    # count > select_ratio * timesteps for an integer count  <=>  count >= floor(.) + 1 (float64, as numpy does)
    thr = math.floor(select_ratio * timesteps) + 0.5
    out = torch.empty(bits.shape[1:], dtype=torch.uint8, device=bits.device)
    nbytes = out.numel()
    st = _lib.load().sdmoe_union_over_time(bits.data_ptr(), bits.stride(0), T, nbytes, float(thr), out.data_ptr(),
                                           ops._stream())
    _lib.check(st, "sdmoe_union_over_time")
    return out


def bake_masks(unet, masks: dict):
    """W <- W * (1 - M) on every down projection named in `masks` (bit-packed [C, F/8] device tensors). The weight
    gets new storage, so every cached derived copy (the FFN's permuted down weights) is rebuilt."""
    for name, mod in down_projection_layers(unet):
        if name in masks:
            w = mod.weight.data
            mod.weight.data = ops.mask_weight(w, masks[name].to(w.device).contiguous())
    return unet


def save_union_over_time(model, path, timesteps=51, select_ratio=0.0, n_layers=16, weights_shape=None,
                         device=None):
    """save_union_over_time.main (:150-246) on an sdmoe pipeline: loads the (t, l) masks from `path` (.npz bits,
    CSR / np.matrix .pkl, or JSON indices with weights_shape), unions them over time, bakes the result into
    model.unet and returns {layer name: dense int mask} as the reference's `masks` dict (:205-208)."""
    unet = model.unet
    layers = down_projection_layers(unet)[:n_layers]
    dev = device or layers[0][1].weight.device
    out_bits, dense = {}, {}
    for l, (name, mod) in enumerate(layers):
        per_t = np.stack([mask_io.load_wanda_mask(path, t, l, weights_shape) for t in range(timesteps)])
        bits = torch.from_numpy(np.ascontiguousarray(per_t)).to(dev)
        out_bits[name] = union_over_time(bits, select_ratio, timesteps)
        dense[name] = mask_io.unpack_mask(out_bits[name].cpu().numpy(), mod.weight.shape[1]).astype(np.int64)
    bake_masks(unet, out_bits)
    return dense


def binary_mask_iou(bits1, bits2):
    """iou_masks.binary_mask_iou (iou_masks.py:8-14) on bit-packed masks: (IoU, intersection, union) areas."""
    a = np.asarray(bits1, dtype=np.uint8)
    b = np.asarray(bits2, dtype=np.uint8)
    pc = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1)
    area1, area2 = int(pc[a].sum()), int(pc[b].sum())
    inter = int(pc[a & b].sum())
    union = area1 + area2 - inter
    return inter / union, inter, union
