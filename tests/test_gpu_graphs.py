"""HIP-graph replay of the denoising steps (StableDiffusionPipeline.graphs, sdmoe/pipeline.py StepGraphs).

A replayed call must be bit-identical to an eager call of the same inputs (the graphs hold the same kernels with the
same arguments), and must leave every receiver's (timestep, layer) counter where the eager hooks would
(predictivity.py:25-39): RemoveExperts (removal lists switch off at t = 20, remove_skilled_experts.py:32) across the
20-step boundary, RemoveExperts + the union Wanda receiver on ff.net.2 together (two hook owners), and PNDM.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from sdmoe.config import UNetConfig  # noqa: E402
from sdmoe.pipeline import StableDiffusionPipeline  # noqa: E402

from test_gpu_unet import DEV, build, moefy_tiny  # noqa: E402


@pytest.fixture(scope="module")
def tiny_unet():
    cfg = UNetConfig.tiny(16)
    return cfg, build(cfg)[0]


def lists_for(layers, T, seed):
    g = torch.Generator().manual_seed(seed)
    return {t: {l: sorted(torch.randperm(E, generator=g)[:max(1, E // 4)].tolist()) for l, (_, E, _) in
                enumerate(layers)} for t in range(T)}


@pytest.mark.parametrize("scheduler,steps", [("ddim", 22), ("pndm", 3)])
def test_graph_replay_bit_identical_remove_experts(tiny_unet, scheduler, steps):
    from neuron_receivers import GEGLU, RemoveExperts
    cfg, unet = tiny_unet
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=steps, scheduler=scheduler)
    layers = moefy_tiny(pipe, topk=0.25, relu=True)
    T = steps + (1 if scheduler == "pndm" else 0)
    rec = RemoveExperts(0, None, T, len(layers), replace_fn=GEGLU, expert_indices=lists_for(layers, T, 3),
                        store_gates=False)
    batches = [["a church", "a red car"], ["a lighthouse", "a cat"], ["a church", "a red car"]]
    eager = []
    for p in batches:
        rec.reset_time_layer()
        eager.append(torch.stack(rec.observe_activation(pipe, p)[0]).cpu())
        assert (rec.timestep, rec.layer) == (T, 0)
    assert not pipe._graph_states
    pipe.graphs = True
    try:
        for i, p in enumerate(batches):  # call 0: eager + capture; calls 1, 2: replay
            rec.reset_time_layer()
            got = torch.stack(rec.observe_activation(pipe, p)[0]).cpu()
            assert (rec.timestep, rec.layer) == (T, 0)
            assert len(pipe._graph_states) == 1
            assert torch.equal(got, eager[i]), f"call {i}"
        # a replay must start from the captured counter state: a stale counter raises instead of misrouting
        rec.timestep = 1
        with pytest.raises(RuntimeError, match="counter"):
            rec.observe_activation(pipe, batches[0])
    finally:
        pipe.graphs = False
        pipe.reset_graphs()


def test_graph_replay_two_hook_owners_union_wanda(tiny_unet):
    from neuron_receivers import GEGLU, RemoveExperts, WandaRemoveNeuronsFast
    cfg, unet = tiny_unet
    steps = 2
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=steps)
    layers = moefy_tiny(pipe, topk=0.25, relu=True)
    L = len(layers)
    downs = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.2")]
    rng = np.random.default_rng(4)
    masks = {t: {l: (rng.random(tuple(downs[l].weight.shape)) < 0.05).astype(np.int64) for l in range(L)}
             for t in range(steps)}
    wanda = WandaRemoveNeuronsFast(0, None, steps, L, masks=masks, store_gates=False)
    rec = RemoveExperts(0, None, steps, L, replace_fn=GEGLU, expert_indices=lists_for(layers, steps, 5),
                        store_gates=False)

    def run(p):
        wanda.reset_time_layer()
        rec.reset_time_layer()
        wanda.prepare(pipe)
        hooks = wanda.register_hooks(pipe)
        try:
            out = torch.stack(rec.observe_activation(pipe, p)[0]).cpu()
        finally:
            wanda.remove_hooks(hooks)
        assert (rec.timestep, rec.layer) == (steps, 0) and (wanda.timestep, wanda.layer) == (steps, 0)
        return out
    prompts = [["a church in the style of van gogh"], ["water lilies"]]
    eager = [run(p) for p in prompts]
    pipe.graphs = True
    try:
        got = [run(p) for p in prompts + prompts]
        assert len(pipe._graph_states) == 1
        for i, g in enumerate(got):
            assert torch.equal(g, eager[i % 2]), f"call {i}"
    finally:
        pipe.graphs = False
        pipe.reset_graphs()


def test_graphs_off_when_gates_are_captured(tiny_unet):
    """store_gates=True copies every gate to the host from inside the hook (moefy.py:25): not replayable, so the
    pipeline runs eagerly and captures nothing."""
    from neuron_receivers import MOEFy
    cfg, unet = tiny_unet
    pipe = StableDiffusionPipeline(unet, DEV, num_inference_steps=2)
    moefy_tiny(pipe, topk=0.25, relu=True)
    rec = MOEFy(0, store_gates=True)
    pipe.graphs = True
    try:
        out, gates = rec.observe_activation(pipe, "a church")
        assert len(gates) == 2 * 16 and not pipe._graph_states
    finally:
        pipe.graphs = False
