"""BaseNeuronReceiver — drop-in for neuron_receivers/base_receiver.py:10-82 of the reference.

Same constructor, same `observe_activation(model, ann, bboxes=None) -> (image(s), gates)` contract:
forward hooks are registered on every `replace_fn` module whose name contains 'ff.net' (:49-57), the torch and
numpy RNGs are seeded with `self.seed` (:70-71), the pipeline runs, the hooks are removed (:76).
MI355X difference: receivers built on this base compute the hooked module's output themselves on the HIP
kernels, so they mark the module "deferred" while hooked and the module skips its own forward (the reference
computes the GEGLU twice per call).
"""
from __future__ import annotations

import numpy as np
import torch

from sdmoe.unet import GEGLU, LoRACompatibleLinear  # noqa: F401  (re-exported for `replace_fn=GEGLU`)


def text_mlp_modules(model):
    """CLIPMLP modules of model.text_encoder with 'mlp' and 'encoder.layers' in the name (base_receiver.py:62-63)."""
    from sdmoe.clip import CLIPMLP
    te = getattr(model, "text_encoder", None)
    if te is None:
        raise ValueError("hook_module='text' needs a pipeline with a text_encoder (sdmoe.clip.CLIPTextModel)")
    return [(n, m) for n, m in te.named_modules() if isinstance(m, CLIPMLP) and 'mlp' in n and 'encoder.layers' in n]


class GELU(torch.nn.Module):
    """Placeholder for diffusers' GELU projection class (PixArt path, out of scope)."""


class BaseNeuronReceiver:
    '''Base class for hooking (and changing) the U-Net FFN activations.'''

    _sdmoe_receiver = True  # sdmoe.unet.FeedForward keeps its fused path only under hooks owned by these receivers

    def __init__(self, seed=0, replace_fn=GEGLU, keep_nsfw=False, hook_module='unet', store_gates=True):
        self.seed = seed
        self.gates = []
        self.hidden_states = []
        self.keep_nsfw = keep_nsfw
        self.safety_checker = None  # no safety checker in this tier (images are latents)
        self.replace_fn = replace_fn
        self.hook_module = hook_module
        # the reference copies every masked gate to host on every call (gate.detach().cpu(), moefy.py:25):
        # kept as an option; set False for timed runs.
        self.store_gates = store_gates
        self._deferred = []

    def hook_fn(self, module, input, output):
        raise NotImplementedError

    def text_hook_fn(self, module, input, output):
        raise NotImplementedError(f"{type(self).__name__} has no text-encoder hook body")

    def remove_hooks(self, hooks):
        for hook in hooks:
            hook.remove()
        for m in self._deferred:
            m._sdmoe_deferred = max(0, m._sdmoe_deferred - 1)
        self._deferred = []

    def _register(self, module, fn, defer=True):
        h = module.register_forward_hook(fn)
        if defer and hasattr(module, "_sdmoe_deferred"):
            module._sdmoe_deferred += 1
            self._deferred.append(module)
        return h

    def hook_modules(self, model):
        """(name, module) pairs this receiver hooks: replace_fn instances with 'ff.net' in the name (unet,
        :46-57), or the text encoder's CLIPMLP modules under 'encoder.layers' (hook_module='text', :59-65)."""
        if self.hook_module == 'text':
            return text_mlp_modules(model)
        if self.hook_module != 'unet':
            raise ValueError(f"hook_module must be 'unet' or 'text', got {self.hook_module!r}")
        return [(n, m) for n, m in model.unet.named_modules() if isinstance(m, self.replace_fn) and 'ff.net' in n]

    def register_hooks(self, model, bboxes=None):
        hooks = []
        if self.hook_module == 'text':
            return [self._register(m, self.text_hook_fn) for _, m in self.hook_modules(model)]
        for name, module in self.hook_modules(model):
            hooks.append(self._register(module, self.hook_fn))
            module.bounding_box = bboxes[name + '.proj.weight'] if bboxes is not None else None
        return hooks

    def run_model(self, model, ann):
        torch.manual_seed(self.seed)
        np.random.seed(self.seed)
        out = model(ann, safety_checker=self.safety_checker).images
        return out if isinstance(ann, list) else out[0]

    def observe_activation(self, model, ann, bboxes=None):
        self.gates = []
        hooks = self.register_hooks(model, bboxes)
        try:
            out = self.run_model(model, ann)
        finally:
            self.remove_hooks(hooks)
        return out, self.gates

    def test(self, model, ann='A brown dog in the snow', relu_condition=False):
        """moefy.py:29-54 / remove_skilled_experts.py:58-86: run with and without hooks; all stored gates must
        be >= 0 exactly when the U-Net is relufied. (No PNGs: the tier outputs latents.)"""
        keep = self.store_gates
        self.store_gates = True
        torch.manual_seed(self.seed)
        np.random.seed(self.seed)
        nochange = model(ann).images[0]
        out, gates = self.observe_activation(model, ann)
        for gate in gates:
            assert bool(torch.all(gate >= 0)) == relu_condition, "All gates should be positive"
        self.gates = []
        self.store_gates = keep
        return nochange, out
