"""MoE-fication helpers — drop-in for moefication/helper.py:48-78 of the reference.

`modify_ffn` turns an expert-label file (moe_utils.ParamSplit output: torch.save(list[int]) of length 4C,
moe_utils.py:54-61) into `module.patterns` [E, 4C] (0/1, weight dtype/device) and `module.k = int(E * topk)`
(helper.py:48-62). `modify_ffn_to_experts` does it for every GEGLU FFN and returns the sorted layer names
(:65-78). The device routing layout (labels + per-expert neuron lists) is derived once from these attributes by
sdmoe.unet.GEGLU.routing(). The offline clustering itself (KMeansConstrained, moe_utils.py:97-107) is outside
this tier: `balanced_random_labels` is the seeded stand-in used for synthetic runs.
The template helpers of the offline driver (get_model_block_config / make_templates / test_template,
helper.py:6-46, used by moefy_sd_model.py) and the frequency counter (initialise_expert_counter, :80-96, used by
freq_expert_select.py) serve out-of-scope scripts and are not provided: GEGLU layers are found by walking the
module tree, as modify_ffn_to_experts does.
Label files hold whatever KMeansConstrained produced -- lists of numpy int32/int64 scalars in the reference's
own files -- and are read with mask_io.load_labels (torch.load weights_only=True plus the numpy scalar types).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from sdmoe import mask_io
from sdmoe.unet import GEGLU


def balanced_random_labels(num_neurons, expert_size, seed):
    """Seeded balanced partition (expert_size neurons per expert), standing in for KMeansConstrained labels."""
    if num_neurons % expert_size:
        raise ValueError("num_neurons must be a multiple of expert_size")
    rng = np.random.default_rng(seed)
    lab = np.repeat(np.arange(num_neurons // expert_size), expert_size)
    rng.shuffle(lab)
    return lab.astype(np.int64)


def modify_ffn(ffn, path, k, labels=None):
    """helper.py:48-62: labels -> ffn.patterns [E, 4C] (weight dtype/device), ffn.k = int(E * k)."""
    assert isinstance(ffn, GEGLU)
    if labels is None:
        labels = mask_io.load_labels(path)
    labels = np.asarray(labels, dtype=np.int64)
    cluster_num = int(labels.max()) + 1
    patterns = np.stack([labels == i for i in range(cluster_num)]).astype(np.float32)
    device, dtype = ffn.proj.weight.device, ffn.proj.weight.dtype
    ffn.patterns = torch.from_numpy(patterns).to(device).to(dtype)
    ffn.labels = torch.from_numpy(labels)
    ffn.k = int(cluster_num * k)


def modify_ffn_to_experts(model, args):
    """helper.py:65-78. args.res_path/param_split/<ffn>.proj.weight label files; args.moefication['topk_experts']."""
    num_experts_per_ffn = {}
    layer_names = []
    for name, module in model.unet.named_modules():
        if 'ff.net' in name and isinstance(module, GEGLU):
            ffn_name = name + '.proj.weight'
            path = os.path.join(args.res_path, 'param_split', ffn_name)
            modify_ffn(module, path, args.moefication['topk_experts'])
            layer_names.append(ffn_name)
            num_experts_per_ffn[ffn_name] = module.patterns.shape[0]
    layer_names.sort()
    return model, layer_names, num_experts_per_ffn


def moefy_synthetic(model, topk_experts=0.2, expert_size=20, seed=0):
    """modify_ffn on every GEGLU with seeded balanced labels (no param_split files offline)."""
    layer_names, nexp = [], {}
    for i, (name, module) in enumerate([(n, m) for n, m in model.unet.named_modules()
                                        if 'ff.net' in n and isinstance(m, GEGLU)]):
        labels = balanced_random_labels(module.inner_dim, expert_size, seed * 1000 + i)
        modify_ffn(module, None, topk_experts, labels=labels)
        layer_names.append(name + '.proj.weight')
        nexp[name + '.proj.weight'] = module.patterns.shape[0]
    layer_names.sort()
    return model, layer_names, nexp
