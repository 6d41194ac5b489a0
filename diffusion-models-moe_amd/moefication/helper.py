"""MoE-fication helpers — drop-in for moefication/helper.py:6-96 of the reference.

`modify_ffn` turns an expert-label file (moe_utils.ParamSplit output: torch.save(list[int]) of length 4C,
moe_utils.py:54-61) into `module.patterns` [E, 4C] (0/1, weight dtype/device) and `module.k = int(E * topk)`
(helper.py:48-62). `modify_ffn_to_experts` does it for every GEGLU FFN and returns the sorted layer names
(:65-78). The device routing layout (labels + per-expert neuron lists) is derived once from these attributes by
sdmoe.unet.GEGLU.routing(). The offline clustering itself (KMeansConstrained, moe_utils.py:97-107) is outside
this tier: `balanced_random_labels` is the seeded stand-in used for synthetic runs.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from sdmoe.unet import GEGLU


def get_model_block_config(model_id):
    config = {}
    if model_id in ('runwayml/stable-diffusion-v1-5', 'CompVis/stable-diffusion-v1-4', 'sd-1.4'):
        config['down_blocks'] = {'layer_idx': [0, 1, 2], 'attention_idx': [0, 1]}
        config['mid_block'] = {'layer_idx': [-1], 'attention_idx': [0]}
        config['up_blocks'] = {'layer_idx': [1, 2, 3], 'attention_idx': [0, 1, 2]}
    return config


def make_templates(template, config):
    templates = []
    for key in config.keys():
        for layer in config[key]['layer_idx']:
            if layer == -1:
                t_ = '{}.attentions.{}.transformer_blocks.0.ff.net.0.proj.weight'
                for att in config[key]['attention_idx']:
                    templates.append(t_.format(key, att))
            else:
                for att in config[key]['attention_idx']:
                    templates.append(template % (key, layer, att))
    return templates


def test_template(templates, model):
    model_ffns = [name + '.proj.weight' for name, m in model.unet.named_modules()
                  if 'ff.net' in name and isinstance(m, GEGLU)]
    assert all(ffn in templates for ffn in model_ffns)
    return True


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
        labels = torch.load(path, weights_only=True)
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


def initialise_expert_counter(model, timesteps=51):
    expert_counter = {t: {} for t in range(timesteps)}
    names = []
    for name, module in model.unet.named_modules():
        if 'ff.net' in name and isinstance(module, GEGLU):
            ffn_name = name + '.proj.weight'
            for t in range(timesteps):
                expert_counter[t][ffn_name] = np.zeros(module.patterns.shape[0])
            names.append(ffn_name)
    names.sort()
    return expert_counter, names
