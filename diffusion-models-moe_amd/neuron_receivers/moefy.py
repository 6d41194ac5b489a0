"""MOEFy — drop-in for neuron_receivers/moefy.py:7-54 (config 2: MoE-fied FFN, no mask).

hook_fn keeps the reference contract (module, input, output) -> gated hidden states [B, N, 4C]: the GEGLU
projection, activation, expert scores, per-token top-k, expert mask and value*gate product run as the
sdmoe proj GEMM + `sdmoe_geglu_route` kernel (include/sdmoe.h) on the module's own weights, patterns and k.
"""
from __future__ import annotations

from neuron_receivers.base_receiver import BaseNeuronReceiver


class MOEFy(BaseNeuronReceiver):
    def __init__(self, seed, **kw):
        super().__init__(seed, **kw)

    def hook_fn(self, module, input, output):
        out, gate = module.routed(input[0], removed=None, want_gate=self.store_gates)
        if self.store_gates:
            self.gates.append(gate.detach().cpu())
        return out

    # this hook_fn only hands input[0] to module.routed(), which resolves a LayerNorm deferred into the GEGLU call:
    # the block's norm3 may then stay folded into the projection GEMM (sdmoe.unet.FeedForward.run). A subclass that
    # overrides hook_fn does not inherit this (the marker names this exact function).
    _sdmoe_ln_safe_hook = hook_fn
