"""WandaRemoveNeuronsFast — drop-in for neuron_receivers/remove_wanda_neurons_fast.py:12-167 (configs 4-5).

linear_hook_fn (:69-83) semantics kept: at every hooked `ff.net.2` call, y = F.linear(x, W * (1 - M[t][l]), b),
then the (t, l) counter advances. The mask applies at every step (App. A #8); `remove_timesteps` and
`weights_shape` are accepted (callers pass them, App. A #5) — weights_shape is used for JSON index masks,
remove_timesteps is stored but, as in the reference's Fast receiver, not consulted.
MI355X layout: masks are bit-packed [C, 4C/8] and uploaded once (all (t, l): 316 MB for SD-1.4 at T=51, vs
~20 GB as dense int64 in the reference), then converted once per (t, l) on the device into the masked GEMM's
K-step-major layout (sdmoe_wmask_kmajor); sdmoe_linear_masked zeroes the masked weights on the W fragments after
their LDS read, so there is no per-call host->device mask copy, no W.clone()/masked weight copy and no second GEMM
(reference K9).
Under MoE routing (config 4: union Wanda mask on a MoE-fied U-Net) the FeedForward keeps its fused routed path:
when this receiver is the only hook on ff.net.2 it calls fused_linear(), which applies the same (t, l) mask with
its columns permuted into the experts' neuron order (converted once per (t, l, layer routing)) together with the
top-k keep bits, in one sdmoe_linear_masked launch, and advances the counter exactly as linear_hook_fn does.
The GEGLU variant hook_fn (:31-61, mask over the gate half of proj.weight) uses the same bitmask path, and so does
the text-encoder variant text_hook_fn (:85-101, hook_module='text': mask M[0][l] over CLIPMLP.fc2).
Baked masked weights (the U-Net ff.net.2 hooks): the masks are the same for every prompt batch, so W * (1 - M[t][l])
is materialised ONCE per (t, l) (and routing order) into an HBM cache (bake_budget_bytes, default 24 GiB: all 50 x 16
masked SD-1.4 down projections are ~5 GB of the 288 GB) and the per-call GEMM is then the plain (or keep-masked)
one. In-GEMM masking re-applies the mask in every row tile -- 256 times per call at 64x64 -- and measured 156 us
against 86 us for the keep-only GEMM at M = 65536 (profiles/r02_rocprof_summary_union.txt); the two are
bit-identical (tests/test_gpu_wanda.py). Past the budget, or with bake_budget_bytes = 0, the in-GEMM path runs.
"""
from __future__ import annotations

import weakref

import numpy as np
import torch

from sdmoe import mask_io, ops
from sdmoe.unet import LoRACompatibleLinear

from neuron_receivers.base_receiver import GEGLU
from neuron_receivers.predictivity import NeuronPredictivity


# HBM held by baked masked weights, per device, over EVERY receiver of the process (a MultiConceptRemoverWanda holds
# one receiver per concept plus the union one: a per-instance count would let each bake its own budget's worth).
# Entries are released by a finalizer when the baked tensor is freed.
_BAKED_BYTES = {}


def _baked_release(dev, nbytes):
    _BAKED_BYTES[dev] = _BAKED_BYTES.get(dev, 0) - nbytes


class WandaRemoveNeuronsFast(NeuronPredictivity):
    def __init__(self, seed, path_expert_indx, T, n_layers, replace_fn=GEGLU, keep_nsfw=False, hook_module='unet',
                 remove_timesteps=None, weights_shape=None, masks=None, **kw):
        super().__init__(seed, T, n_layers, replace_fn, keep_nsfw, hook_module, **kw)
        self.remove_timesteps = remove_timesteps
        self.weights_shape = weights_shape
        # mask_bits[t][l]: np.uint8 [C, 4C/8] (host); device copies made once in prepare()
        self.mask_bits = {}
        for i in range(T):
            self.mask_bits[i] = {}
            for j in range(n_layers):
                if masks is not None:
                    bits = mask_io.pack_mask(masks[i][j])
                else:
                    bits = mask_io.load_wanda_mask(path_expert_indx, i, j, weights_shape)
                self.mask_bits[i][j] = bits
        self.timestep = 0
        self.layer = 0
        self.gates = []
        self._dev = {}

    @classmethod
    def from_packed(cls, seed, packed, T, n_layers, **kw):
        """Build from already bit-packed masks packed[t][l] (np.uint8 [C, 4C/8])."""
        obj = cls.__new__(cls)
        NeuronPredictivity.__init__(obj, seed, T, n_layers, kw.pop("replace_fn", GEGLU), kw.pop("keep_nsfw", False),
                                    kw.pop("hook_module", 'unet'), **kw)
        obj.remove_timesteps, obj.weights_shape = None, None
        obj.mask_bits = {t: {l: np.asarray(packed[t][l], dtype=np.uint8) for l in range(n_layers)} for t in range(T)}
        obj.timestep, obj.layer, obj.gates, obj._dev = 0, 0, [], {}
        return obj

    bake_budget_bytes = 24 << 30  # HBM for baked masked weights, per device and process (0 = always mask in the GEMM)

    def dense_mask(self, t, l):
        bits = self.mask_bits[t][l]
        return mask_io.unpack_mask(bits, bits.shape[-1] * 8)

    def set_mask_bits(self, t, l, bits):
        self.mask_bits[t][l] = np.asarray(bits, dtype=np.uint8)
        # drop the device copy and every layout derived from it (K-major, permuted, GEGLU gate-half forms)
        for key in [k for k in self._dev if k == (t, l) or (isinstance(k[0], str) and tuple(k[1:3]) == (t, l))]:
            del self._dev[key]  # a baked weight's HBM is returned to the budget by its finalizer

    def device_bits(self, t, l, device):
        d = self._dev.get((t, l))
        if d is None:
            d = self._dev[(t, l)] = torch.from_numpy(np.ascontiguousarray(self.mask_bits[t][l])).to(device)
        return d

    def device_kmajor(self, t, l, device, perm=None):
        """The (t, l) mask in sdmoe_linear_masked's layout (int64 [4C/64, C]); perm (int32 device [4C], the routed
        FFN's neuron order) permutes its columns. Converted once per (t, l, perm) on the device and cached. The cache
        entry holds the perm tensor itself and is matched by identity (an address could be reused by a later
        routing's perm after a re-MoE-fication); a new perm for the same (t, l) replaces the entry."""
        key = ("kmajor", t, l, perm is None)
        ent = self._dev.get(key)
        if ent is None or ent[0] is not perm:
            ent = self._dev[key] = (perm, ops.wmask_kmajor(self.device_bits(t, l, device), perm))
        return ent[1]

    def baked_weight(self, t, l, weight, perm=None):
        """W * (1 - M[t][l]) (columns reordered by perm, int32 device [4C], if given), made once per (t, l, weight
        version, perm) with sdmoe_mask_weight and kept in HBM; None when it would exceed bake_budget_bytes (shared by
        all receivers of the process on that device). The entry keeps references to the weight and perm it was made
        from (so neither address can be recycled while it lives) and is replaced -- its HBM released -- when either
        changes for the same (t, l).
        `weight` must share the module parameter's version counter (the Parameter itself or `.detach()`, never
        `.data`, whose counter is a fresh 0): an in-place update (load_state_dict / copy_ / a LoRA merge) keeps the
        address but bumps the version, and the stale bake is then replaced."""
        key = ("baked", t, l, perm is None)
        ent = self._dev.get(key)
        if ent is not None and ent[0].data_ptr() == weight.data_ptr() and ent[1] == weight._version \
                and ent[2] is perm:
            return ent[3]
        if ent is not None:
            del self._dev[key]  # stale: evict before accounting the replacement
        nbytes = weight.numel() * weight.element_size()
        dev = str(weight.device)
        if _BAKED_BYTES.get(dev, 0) + nbytes > self.bake_budget_bytes:
            return None
        w = ops.mask_weight(weight, self.device_bits(t, l, weight.device))
        if perm is not None:
            w = torch.index_select(w, 1, perm.long()).contiguous()
        _BAKED_BYTES[dev] = _BAKED_BYTES.get(dev, 0) + nbytes
        weakref.finalize(w, _baked_release, dev, nbytes)
        self._dev[key] = (weight, weight._version, perm, w)
        return w

    def _check_shape(self, bits, weight, what):
        if bits.shape[0] != weight.shape[0] or bits.shape[1] * 8 != weight.shape[1]:
            raise ValueError(f"{what} mask ({self.timestep},{self.layer}) shape {tuple(bits.shape)} does not match "
                             f"weight {tuple(weight.shape)}")

    def fused_linear(self, module, x2d, keep, perm, weight_perm, residual):
        """linear_hook_fn's arithmetic for the fused routed FFN (sdmoe.unet.FeedForward): x2d is the GEGLU product in
        the experts' neuron order perm (int32 device [4C]), keep its top-k keep bits (or None), weight_perm
        ff.net.2's weight with its columns in that order. Returns y + residual; advances the (t, l) counter."""
        bits = self.device_bits(self.timestep, self.layer, module.weight.device)
        self._check_shape(bits, module.weight, "ff.net.2")
        wb = self.baked_weight(self.timestep, self.layer, module.weight.detach(), perm)
        if wb is not None:
            y = ops.linear_masked(x2d, wb, module.bias, keep=keep, residual=residual)
        else:
            wm = self.device_kmajor(self.timestep, self.layer, module.weight.device, perm)
            y = ops.linear_masked(x2d, weight_perm, module.bias, keep=keep, wmask=wm, residual=residual)
        self.update_time_layer()
        return y

    def hook_modules(self, model):
        if self.hook_module == 'text':
            return super().hook_modules(model)  # CLIPMLP modules (:114-120)
        # remove_wanda_neurons_fast.py:107-112: LoRACompatibleLinear, 'ff.net' in name, not a '.proj'
        return [(n, m) for n, m in model.unet.named_modules()
                if isinstance(m, LoRACompatibleLinear) and 'ff.net' in n and 'proj' not in n]

    def prepare(self, model):
        mods = [m for _, m in self.hook_modules(model)]
        dev = (mods[0].fc2 if self.hook_module == 'text' else mods[0]).weight.device
        for t in range(self.T):
            for l in range(self.n_layers):
                self.device_bits(t, l, dev)

    def register_hooks(self, model, bboxes=None):
        fn = self.text_hook_fn if self.hook_module == 'text' else self.linear_hook_fn
        return [self._register(m, fn) for _, m in self.hook_modules(model)]

    def observe_activation(self, model, ann, bboxes=None):
        self.prepare(model)
        return super().observe_activation(model, ann, bboxes)

    def linear_hook_fn(self, module, input, output):
        x = input[0]
        bits = self.device_bits(self.timestep, self.layer, module.weight.device)
        self._check_shape(bits, module.weight, "ff.net.2")
        wb = self.baked_weight(self.timestep, self.layer, module.weight.detach())
        if wb is not None:
            y = module.run(x.reshape(-1, x.shape[-1]), weight=wb)
        else:
            y = module.run(x.reshape(-1, x.shape[-1]), wmask=self.device_kmajor(self.timestep, self.layer, bits.device))
        self.update_time_layer()
        return y.view(*x.shape[:-1], module.weight.shape[0])

    def text_hook_fn(self, module, input, output):
        """remove_wanda_neurons_fast.py:85-101: CLIPMLP with fc2.weight * (1 - M[0][layer]) — always timestep 0
        (text masks have T = 1); fc1 + act in one GEMM epilogue, the mask applied while fc2's W tiles stage."""
        x = input[0]
        fc2 = module.fc2
        bits = self.device_bits(0, self.layer, fc2.weight.device)
        self._check_shape(bits, fc2.weight, "text fc2")
        y = module.run(x.reshape(-1, x.shape[-1]), wmask=self.device_kmajor(0, self.layer, bits.device))
        self.update_time_layer()
        return y.view(*x.shape[:-1], fc2.weight.shape[0])

    def hook_fn(self, module, input, output):
        """GEGLU variant (:31-61): mask M [4C, C] over the gate half of proj.weight, dense value*act(gate)."""
        bits = self.device_bits(self.timestep, self.layer, module.proj.weight.device)
        key = ("gate_full", self.timestep, self.layer)
        full = self._dev.get(key)
        if full is None:  # [value rows unmasked ; gate rows masked] in the masked GEMM's layout, once per (t, l)
            F4, Kb = bits.shape
            full = torch.cat([torch.zeros((F4, Kb), dtype=torch.uint8, device=bits.device), bits], 0).contiguous()
            full = self._dev[key] = ops.wmask_kmajor(full)
        x = input[0]
        y = module.proj.run(x.reshape(-1, x.shape[-1]), wmask=full)
        gate = torch.empty((y.shape[0], module.inner_dim), dtype=torch.float16, device=y.device) \
            if self.store_gates else None
        from sdmoe.unet import act_code
        out = ops.geglu_route(y, None, act_code(module.gelu), gate_out=gate)
        if self.store_gates:
            self.gates.append(gate.view(*x.shape[:-1], -1).cpu())
        self.update_time_layer()
        return out.view(*x.shape[:-1], module.inner_dim)
