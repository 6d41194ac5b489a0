"""NeuronPredictivity — the (timestep, layer) counter of neuron_receivers/predictivity.py:10-39.

Every masking receiver inherits it: one `update_time_layer()` per hooked call, wrapping `layer` at
n_layers-1 and advancing `timestep` (hook call order == U-Net execution order, one U-Net call per step).
The reference's own statistics hook (max-activation predictivity, :42-62) is skill DISCOVERY, outside this
tier; it raises here rather than silently running an unaccelerated path.
"""
from __future__ import annotations

from neuron_receivers.base_receiver import GEGLU, BaseNeuronReceiver


class NeuronPredictivity(BaseNeuronReceiver):
    def __init__(self, seed, T, n_layers, replace_fn=GEGLU, keep_nsfw=False, hook_module='unet', **kw):
        super().__init__(seed, replace_fn, keep_nsfw, hook_module, **kw)
        self.T = T
        self.n_layers = n_layers
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
        raise NotImplementedError("max-activation predictivity statistics are skill discovery (out of scope)")
