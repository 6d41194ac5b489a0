"""Static union-timesteps mask baking (benchmarks/save_union_over_time.py:150-246):
sdmoe_union_over_time vs the oracle restatement (bit-exact), the bake W*(1-M) (bit-exact), and the whole
save_union_over_time flow from reference-format mask files on a tiny U-Net."""
import os

import numpy as np
import pytest
import torch

from oracle import hooks_ref as H
from sdmoe import mask_io
from sdmoe import union_bake as U
from sdmoe.config import UNetConfig
from sdmoe.pipeline import StableDiffusionPipeline
from sdmoe.unet import UNet2DConditionModel
from sdmoe.weights import make_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("T,C,F,density,ratio", [(51, 320, 1280, 0.025, 0.0), (51, 320, 1280, 0.2, 0.1),
                                                  (51, 640, 2560, 0.5, 0.3), (7, 64, 96, 0.6, 0.5),
                                                  (10, 32, 64, 0.9, 1.0)])
def test_union_over_time_kernel_bit_exact(T, C, F, density, ratio):
    rng = np.random.default_rng(T * C + F)
    masks = [(rng.random((C, F)) < density).astype(np.int64) for _ in range(T)]
    bits = torch.from_numpy(np.stack([mask_io.pack_mask(m) for m in masks])).to(DEV)
    got = mask_io.unpack_mask(U.union_over_time(bits, ratio, T).cpu().numpy(), F)
    exp = H.union_over_time(masks, ratio, T)
    assert np.array_equal(got, exp)
    assert 0 < exp.sum() or ratio >= 1.0


def test_bake_bit_exact_and_iou():
    rng = np.random.default_rng(3)
    w = torch.from_numpy(rng.standard_normal((320, 1280)).astype(np.float16)).to(DEV)
    m = (rng.random((320, 1280)) < 0.3).astype(np.int64)
    from sdmoe import ops
    baked = ops.mask_weight(w, torch.from_numpy(mask_io.pack_mask(m)).to(DEV))
    assert torch.equal(baked.cpu(), H.bake_mask(w.cpu(), m))
    m2 = (rng.random((320, 1280)) < 0.3).astype(np.int64)
    got = U.binary_mask_iou(mask_io.pack_mask(m), mask_io.pack_mask(m2))
    exp = H.binary_mask_iou(m, m2)
    assert got[1:] == (int(exp[1]), int(exp[2])) and abs(got[0] - exp[0]) < 1e-12


def test_save_union_over_time_flow(tmp_path):
    """Reference-format (t, l) mask files (CSR pickles and .npz bits) -> union over time -> baked ff.net.2
    weights equal to the oracle's W*(1-M) for every layer; the other weights are untouched."""
    cfg = UNetConfig.tiny(16)
    sd = make_state_dict(cfg, 2)
    pipe = StableDiffusionPipeline(UNet2DConditionModel.from_state_dict(sd, cfg, DEV), DEV, num_inference_steps=1)
    layers = U.down_projection_layers(pipe.unet)
    T, ratio = 9, 0.25
    rng = np.random.default_rng(5)
    masks = {}
    for l, (name, mod) in enumerate(layers):
        C, F = mod.weight.shape
        masks[l] = [(rng.random((C, F)) < 0.4).astype(np.int64) for _ in range(T)]
        for t in range(T):
            if (t + l) % 2:
                mask_io.save_wanda_mask(str(tmp_path), t, l, masks[l][t])
            else:
                import pickle
                import scipy.sparse
                with open(os.path.join(tmp_path, f"timestep_{t}_layer_{l}.pkl"), "wb") as f:
                    pickle.dump(scipy.sparse.csr_matrix(masks[l][t]), f)
    before = {n: m.weight.detach().cpu().clone() for n, m in layers}
    other = pipe.unet.conv_in.weight.detach().clone()
    dense = U.save_union_over_time(pipe, str(tmp_path), timesteps=T, select_ratio=ratio, n_layers=len(layers))
    for l, (name, mod) in enumerate(layers):
        exp_m = H.union_over_time(masks[l], ratio, T)
        assert np.array_equal(dense[name], exp_m)
        assert torch.equal(mod.weight.detach().cpu(), H.bake_mask(before[name], exp_m))
    assert torch.equal(pipe.unet.conv_in.weight, other)
