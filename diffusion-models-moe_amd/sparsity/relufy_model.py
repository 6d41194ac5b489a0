"""Relufied U-Net — drop-in for sparsity/relufy_model.py:8-40 of the reference: swap every FFN GEGLU's
activation for ReLU. The routing kernel recognises this function (act code RELU)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from sdmoe.unet import GEGLU


def relu(gate: torch.Tensor) -> torch.Tensor:
    return F.relu(gate)


relu._sdmoe_act = "relu"


def test_relu(model):
    for name, module in model.named_modules():
        if isinstance(module, GEGLU) and 'ff.net' in name:
            y = module.gelu(torch.randn(1, 3, 8, 8))
            assert torch.all(y >= 0), f"Relu failed for {name}"
    return True


def find_and_change_geglu(model, blocks_to_change=('down_block', 'mid_block', 'up_block')):
    num_changed = 0
    for name, module in model.named_modules():
        if isinstance(module, GEGLU) and 'ff.net' in name and any(b in name for b in blocks_to_change):
            module.gelu = relu
            num_changed += 1
    test_relu(model)
    return model
