"""MultiConceptRemoverWanda — drop-in for neuron_receivers/multi_concept_remover.py:13-99 (config 4 union).

One WandaRemoveNeuronsFast per concept plus a union remover whose (t, l) masks are the element-wise OR of the
selected concepts' masks (:43-53). The snapshot's union step crashes (App. A #6); this restates the intended
OR, done directly on the bit-packed masks (bitwise OR of packed bytes == element-wise OR of the masks).
As in the reference, the union remover starts from the masks of the LAST configured concept (its constructor
builds it from the loop's final `path_expert_indx`, :24-33) and keeps OR-ing across calls until
reset_union_remover() zeroes it (:35-41).
remove_concepts keeps the reference's two-value contract (:55-99; unified_editing.py:126 unpacks two values):
(stitched, singles) where `stitched` is [before | after] side by side along the width -- the tensor form of the
PIL paste at :83-99 (latents, or RGB when the pipeline decodes) -- and `singles` the same pair per concept (None for
one concept). The unstitched images of the last call are kept in `self.last_outputs`.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from neuron_receivers.base_receiver import GEGLU
from neuron_receivers.remove_wanda_neurons_fast import WandaRemoveNeuronsFast


class MultiConceptRemoverWanda:
    def __init__(self, root, seed, T, n_layers, replace_fn=GEGLU, keep_nsfw=False, remove_timesteps=None,
                 weights_shape=None, concepts_to_remove=None, wanda_thr=0.05, removers=None):
        self.concepts_to_remove = list(concepts_to_remove or [])
        self.seed, self.T, self.n_layers = seed, T, n_layers
        if removers is not None:
            self.removers = dict(removers)
        else:
            self.removers = {}
            for concept in self.concepts_to_remove:
                thr = wanda_thr[concept] if isinstance(wanda_thr, dict) else wanda_thr
                path = os.path.join(root % (seed, concept), f'skilled_neuron_wanda/{thr}')
                self.removers[concept] = WandaRemoveNeuronsFast(
                    seed=seed, path_expert_indx=path, T=T, n_layers=n_layers, replace_fn=replace_fn,
                    keep_nsfw=keep_nsfw, remove_timesteps=remove_timesteps, weights_shape=weights_shape)
        last = list(self.removers.values())[-1]  # the reference's union remover loads the last concept's masks
        start = {t: {l: np.array(last.mask_bits[t][l], copy=True) for l in range(n_layers)} for t in range(T)}
        self.union_neuron_remover = WandaRemoveNeuronsFast.from_packed(seed, start, T, n_layers, replace_fn=replace_fn,
                                                                       keep_nsfw=keep_nsfw)
        self.last_outputs = None

    def reset_union_remover(self):
        u = self.union_neuron_remover
        u.reset_time_layer()
        for t in range(self.T):
            for l in range(self.n_layers):
                u.set_mask_bits(t, l, np.zeros_like(u.mask_bits[t][l]))

    def handle_multiple_concepts(self, concepts):
        u = self.union_neuron_remover
        for c in concepts:
            self.removers[c].reset_time_layer()
            for t in range(self.T):
                for l in range(self.n_layers):
                    u.set_mask_bits(t, l, np.bitwise_or(u.mask_bits[t][l], self.removers[c].mask_bits[t][l]))

    @staticmethod
    def stitch(before, after):
        """[before | after] side by side along the WIDTH axis: the pair of multi_concept_remover.py:83-99.
        torch tensors are CHW (RGB, output_type 'pt') or latents [4, H, W]: width is the last axis. numpy arrays are
        the pipeline's HWC images (output_type 'np'): width is axis -2. Anything else is refused."""
        if isinstance(before, torch.Tensor) and isinstance(after, torch.Tensor):
            return torch.cat([before, after], dim=-1)
        if isinstance(before, np.ndarray) and isinstance(after, np.ndarray):
            if before.ndim != 3:
                raise ValueError(f"numpy images must be HWC, got shape {before.shape}")
            return np.concatenate([before, after], axis=-2)
        raise TypeError(f"cannot stitch {type(before).__name__} and {type(after).__name__}: expected two torch "
                        f"tensors (CHW / latents) or two numpy HWC arrays")

    def remove_concepts(self, model, prompt, concepts):
        """Returns (stitched [original | union removed], per-concept stitched pairs or None) -- two values, as the
        reference. self.last_outputs = {"removal", "original", "singles"} unstitched."""
        if len(concepts) == 0:
            out = model(prompt).images[0]
            self.last_outputs = {"removal": None, "original": out, "singles": None}
            return out, None
        singles = []
        if len(concepts) > 1:
            self.handle_multiple_concepts(concepts)
            self.union_neuron_remover.reset_time_layer()
            out_removal, _ = self.union_neuron_remover.observe_activation(model, prompt)
            for c in concepts:
                self.removers[c].reset_time_layer()
                singles.append(self.removers[c].observe_activation(model, prompt)[0])
        else:
            self.removers[concepts[0]].reset_time_layer()
            out_removal, _ = self.removers[concepts[0]].observe_activation(model, prompt)
        torch.manual_seed(self.seed)
        np.random.seed(self.seed)
        out_pre = model(prompt).images[0]
        self.last_outputs = {"removal": out_removal, "original": out_pre, "singles": singles or None}
        stitched_singles = [self.stitch(out_pre, s) for s in singles] if singles else None
        return self.stitch(out_pre, out_removal), stitched_singles
