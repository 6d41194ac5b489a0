"""RemoveExperts — drop-in for neuron_receivers/remove_skilled_experts.py:9-86 (config 3: skilled-expert removal).

Semantics kept exactly: for timestep < 20 and a non-empty list, the listed experts'
pattern rows are zeroed, so they score exactly 0 (not -inf), may still occupy top-k slots, and never unmask
their neurons (:31-33, :45-49); the (t, l) counter advances once per hooked call (:51).
Constructor defects of the snapshot are fixed, not replicated (App. A #1, #2): `replace_fn` is accepted as a
keyword and `keep_nsfw` no longer lands in the `replace_fn` slot.
MI355X layout: each (t, l) list becomes a device bitmask [ceil(E/32)] once (at the first observe_activation),
consumed by the routing kernel; no per-call `patterns.clone()`.
"""
from __future__ import annotations

import os

from sdmoe import mask_io, ops

from neuron_receivers.base_receiver import GEGLU
from neuron_receivers.predictivity import NeuronPredictivity

REMOVE_BEFORE_TIMESTEP = 20  # remove_skilled_experts.py:32


class RemoveExperts(NeuronPredictivity):
    def __init__(self, seed, path_expert_indx, T, n_layers, keep_nsfw=False, replace_fn=GEGLU, expert_indices=None,
                 **kw):
        super().__init__(seed, T, n_layers, replace_fn=replace_fn, keep_nsfw=keep_nsfw, **kw)
        self.expert_indices = {}
        for i in range(T):
            self.expert_indices[i] = {}
            for j in range(n_layers):
                if expert_indices is not None:
                    self.expert_indices[i][j] = [int(e) for e in expert_indices[i][j]]
                else:
                    self.expert_indices[i][j] = mask_io.load_expert_list(
                        os.path.join(path_expert_indx, f'timestep_{i}_layer_{j}.json'))
        self.timestep = 0
        self.layer = 0
        self.gates = []
        self._bits = {}

    def prepare(self, model):
        """Upload every (t, l) removal list as a device bitmask (layer l = l-th hooked GEGLU)."""
        mods = [m for _, m in self.hook_modules(model)]
        for t in range(self.T):
            for l in range(self.n_layers):
                ids = self.expert_indices[t][l]
                if (t, l) in self._bits or len(ids) == 0 or t >= REMOVE_BEFORE_TIMESTEP:
                    continue
                m = mods[l % len(mods)]
                self._bits[(t, l)] = ops.removed_bits(ids, m.patterns.shape[0], m.proj.weight.device)

    def observe_activation(self, model, ann, bboxes=None):
        self.prepare(model)
        return super().observe_activation(model, ann, bboxes)

    def removed_for(self, module, t, l):
        ids = self.expert_indices[t][l]
        if len(ids) == 0 or t >= REMOVE_BEFORE_TIMESTEP:
            return None
        bits = self._bits.get((t, l))
        if bits is None:
            bits = self._bits[(t, l)] = ops.removed_bits(ids, module.patterns.shape[0], module.proj.weight.device)
        return bits

    def hook_fn(self, module, input, output):
        removed = self.removed_for(module, self.timestep, self.layer) if module.patterns is not None else None
        out, gate = module.routed(input[0], removed=removed, want_gate=self.store_gates)
        self.update_time_layer()
        if self.store_gates:
            self.gates.append(gate.detach().cpu())
        return out

    # this hook_fn only hands input[0] to module.routed(), which resolves a LayerNorm deferred into the GEGLU call:
    # the block's norm3 may then stay folded into the projection GEMM (sdmoe.unet.FeedForward.run). A subclass that
    # overrides hook_fn does not inherit this (the marker names this exact function).
    _sdmoe_ln_safe_hook = hook_fn
