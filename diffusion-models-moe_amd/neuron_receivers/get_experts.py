"""GetExperts — drop-in for neuron_receivers/get_experts.py:8-83 (skill discovery).

Per hooked GEGLU call with MoE-fied `patterns`: per-token expert scores of the activated gate, averaged over all
tokens of the CFG batch (or the bounding-box token positions, module.bounding_box), and the top-k experts of that
mean stored as label_counter[t][l] (a list of ints, :72-81); the module output is the dense, unmasked
value * act(gate) (:83-85). freq_counter is initialised (zeros) and left untouched, as in the reference.
MI355X path: the projection GEMM's epilogue produces the scores (sdmoe_linear_geglu), sdmoe_expert_mean_topk
reduces + selects on device; the label lists of a whole pipeline call are copied to the host once, when
observe_activation returns (the reference syncs per call through .tolist()).
Fixed defects: `keep_nsfw` is no longer passed into the `replace_fn` slot, and the counter
wraps at n_layers - 1 instead of the hard-coded 15 (identical for SD-1.x's 16 layers; SDXL has 70).
Bounding boxes: an empty or out-of-range position list falls back to all tokens (the reference's try/except
covers the out-of-range case).
"""
from __future__ import annotations

import numpy as np
import torch

from sdmoe import ops

from neuron_receivers.base_receiver import GEGLU, BaseNeuronReceiver


class GetExperts(BaseNeuronReceiver):
    def __init__(self, seed, T, n_layers, experts_per_layer, layer_names, keep_nsfw=False, replace_fn=GEGLU, **kw):
        super().__init__(seed, replace_fn, keep_nsfw, **kw)
        self.T = T
        self.n_layers = n_layers
        self.experts_per_layer = experts_per_layer
        self.layer_names = layer_names
        self.label_counter = {}
        self.freq_counter = {}
        self._pending = []
        self.reset()

    def update_time_layer(self):
        if self.layer == self.n_layers - 1:
            self.layer = 0
            self.timestep += 1
        else:
            self.layer += 1

    def reset_time_layer(self):
        self.timestep = 0
        self.layer = 0

    def reset(self):
        for t in range(self.T):
            self.label_counter[t] = {}
            self.freq_counter[t] = {}
            for i in range(self.n_layers):
                self.freq_counter[t][i] = np.zeros(self.experts_per_layer[self.layer_names[i]])
                self.label_counter[t][i] = []
        self._pending = []
        self.reset_time_layer()

    @staticmethod
    def _bb_rows(module, seq_len, device):
        bb = module.bounding_box
        if bb is None:
            return None
        idx = [int(i) for i in bb]
        if not idx or any(i < -seq_len or i >= seq_len for i in idx):
            return None  # reference: gate[:, bb, :] raises -> all tokens
        idx = [i % seq_len for i in idx]
        key = (tuple(idx), str(device))
        cache = getattr(module, "_sdmoe_bb_cache", None)
        if cache is None or cache[0] != key:
            module._sdmoe_bb_cache = (key, torch.tensor(idx, dtype=torch.int32, device=device))
        return module._sdmoe_bb_cache[1]

    def hook_fn(self, module, input, output):
        x = input[0]
        if module.patterns is not None:
            out, score = module.scored(x)
            seq_len = x.shape[1] if x.dim() == 3 else x.shape[0]
            rows = self._bb_rows(module, seq_len, x.device)
            topk = ops.expert_mean_topk(score, int(module.k), rows_per_img=seq_len if rows is not None else 0,
                                        row_idx=rows)
            self._pending.append((self.timestep, self.layer, topk))
        else:
            out = module.dense(x)
        self.update_time_layer()
        return out

    def flush(self):
        """Materialise the pending device top-k lists into label_counter (one device->host copy)."""
        if not self._pending:
            return
        flat = torch.cat([p[2] for p in self._pending]).cpu().tolist()
        o = 0
        for t, l, dev in self._pending:
            n = dev.numel()
            self.label_counter[t][l] = [int(v) for v in flat[o:o + n]]
            o += n
        self._pending = []

    def observe_activation(self, model, ann, bboxes=None):
        try:
            return super().observe_activation(model, ann, bboxes)
        finally:
            self.flush()
