"""moe_utils — drop-in for moefication/moe_utils.py:14-107 of the reference (offline MoE-fication, SURVEY §8f
rank 1): ModelConfig / LayerSplit / RandomSplit / ParamSplit with the same constructor arguments, `split()`,
`cnt()`, `save()` (torch.save(list[int]) at <folder>/<type>/<template>, the file helper.modify_ffn reads).

ParamSplit.split (:97-107): the gate half of the GEGLU projection (rows 4C..8C of proj.weight, :68-72), rows
L2-normalised (sklearn.preprocessing.normalize), clustered into 4C/expert_size experts of exactly expert_size
neurons by size-constrained k-means (KMeansConstrained(size_min = size_max = expert_size, random_state=0)):
here sdmoe.kmeans.constrained_kmeans (fp32 MFMA distances on the GPU + native balanced-assignment auction;
the k_means_constrained package is absent offline — parity unpinned against it).
The model file is read with torch.load(weights_only=True) (a state dict of tensors).
Fixed defect: RandomSplit.__init__ passed keyword arguments LayerSplit does not take (:79-81).
"""
from __future__ import annotations

import os
from collections import Counter

import numpy as np
import torch

from sdmoe.kmeans import constrained_kmeans


def load_ffn_weight(filename, template, layer=0):
    """moe_utils.py:27-31: the state-dict entry `template` as a float numpy array."""
    sd = torch.load(filename, map_location="cpu", weights_only=True)
    return sd[template].float().numpy()


class ModelConfig:
    def __init__(self, filename, folder, split_size):
        self.filename = filename
        self.folder = folder
        self.split_size = split_size


class LayerSplit:
    def __init__(self, config: ModelConfig, template, layer=0):
        self.config = config
        self.layer = layer
        self.template = template

    def split(self):
        pass

    def save(self):
        save_folder = os.path.join(self.config.folder, self.type)
        os.makedirs(save_folder, exist_ok=True)
        filename = os.path.join(save_folder, self.template.format(self.layer))
        torch.save([int(x) for x in self.labels], filename)

    def cnt(self):
        print(Counter(self.labels))

    def load_param(self):
        w = load_ffn_weight(self.config.filename, self.template, self.layer)
        self.neuron_num = w.shape[0] // 2
        self.ffn_weight = w[self.neuron_num:, :]  # the gate half (diffusers GEGLU: value first, gate second)
        self.split_size = self.config.split_size
        self.split_num = self.neuron_num // self.split_size
        assert self.split_num * self.config.split_size == self.neuron_num


class RandomSplit(LayerSplit):
    def __init__(self, config: ModelConfig, template="", layer=0):
        super().__init__(config, template=template, layer=layer)
        self.type = 'random_split'

    def split(self):
        self.load_param()
        self.labels = [i // self.split_size for i in range(self.neuron_num)]


class ParamSplit(LayerSplit):
    def __init__(self, config: ModelConfig, template, layer=0, n_init=10, max_iter=300, device="cuda"):
        super().__init__(config, template=template, layer=layer)
        self.type = 'param_split'
        self.n_init, self.max_iter, self.device = n_init, max_iter, device

    def split(self):
        self.load_param()
        w = self.ffn_weight.astype(np.float64)
        norm = np.linalg.norm(w, axis=1, keepdims=True)
        x = w / np.where(norm == 0, 1.0, norm)  # sklearn.preprocessing.normalize (zero rows stay zero)
        labels, centers, inertia, n_iter = constrained_kmeans(x, self.split_num, self.split_size, n_init=self.n_init,
                                                              max_iter=self.max_iter, random_state=0,
                                                              device=self.device)
        self.labels = [int(v) for v in labels]
        self.centers, self.inertia, self.n_iter = centers, inertia, n_iter
