"""Wanda — drop-in for neuron_receivers/wanda_receiver.py:9-57 (skill discovery).

hook_fn: out = value * act(gate) (dense GEGLU, natural neuron order); every token row of `out` is L2-normalised
and its squares are added to the (t, l) column statistic (utils.TimeLayerColumnNorm, utils.py:344-370); the (t, l)
counter wraps at n_layers - 1; the output is returned unchanged. MI355X path: sdmoe_linear_geglu +
sdmoe_colnorm_accum, the statistic stays on the device (no per-call `.cpu()` copy); get_column_norms() returns
fp16 CPU tensors like the reference's. hook_module='text' (:14-18, :59-71): one ColumnNormCalculator per CLIP
encoder layer over act(fc1 x) rows; fc1 + act run as one GEMM, the MLP output is fc2 of the same activations.
"""
from __future__ import annotations

from sdmoe.discovery import ColumnNormCalculator, TimeLayerColumnNorm

from neuron_receivers.base_receiver import GEGLU, BaseNeuronReceiver


class Wanda(BaseNeuronReceiver):
    def __init__(self, seed, T, n_layers, replace_fn=GEGLU, keep_nsfw=False, hook_module='unet', **kw):
        super().__init__(seed, replace_fn, keep_nsfw, hook_module, **kw)
        self.T = T
        self.n_layers = n_layers
        if hook_module == 'unet':
            self.predictivity = TimeLayerColumnNorm(T, n_layers)
        elif hook_module == 'text':
            self.predictivity = {l: ColumnNormCalculator() for l in range(n_layers)}
        else:
            raise ValueError(f"hook_module must be 'unet' or 'text', got {hook_module!r}")
        self.timestep = 0
        self.layer = 0

    def update_time_layer(self):
        if self.layer == self.n_layers - 1:
            self.layer = 0
            self.timestep += 1
        else:
            self.layer += 1

    def reset_time_layer(self):
        self.timestep = 0
        self.layer = 0

    def hook_fn(self, module, input, output):
        out = module.dense(input[0])
        self.predictivity.update(out.reshape(-1, out.shape[-1]), self.timestep, self.layer)
        self.update_time_layer()
        return out

    def text_hook_fn(self, module, input, output):
        x = input[0]
        a = module.hidden(x.reshape(-1, x.shape[-1]))
        if self.layer < self.n_layers:
            self.predictivity[self.layer].add_rows(a)
        out = module.fc2.run(a)
        self.update_time_layer()
        return out.view(*x.shape[:-1], out.shape[-1])
