"""Multi-process (world_size 2, gloo, CPU) tests of the data-parallel host path: prompt sharding, one-time
broadcast of expert lists and bit-packed masks, max-over-ranks timing, world-size-independent seeds."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world_size, port, outq):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from sdmoe import distributed as D
        from sdmoe.config import UNetConfig
        from sdmoe.pipeline import initial_latents
        prompts = [f"p{i}" for i in range(10)]
        mine, off = D.shard(prompts, rank, world_size)
        lists = D.broadcast_object({t: {l: [t, l, 7] for l in range(3)} for t in range(4)} if rank == 0 else None)
        rng = np.random.default_rng(123)
        if rank == 0:
            masks = [torch.from_numpy(rng.integers(0, 256, size=(8, 16), dtype=np.uint8)) for _ in range(5)]
        else:
            masks = [torch.zeros((8, 16), dtype=torch.uint8) for _ in range(5)]
        D.broadcast_tensors(masks)
        mx = D.max_over_ranks(float(rank + 1), "cpu")
        cfg = UNetConfig.tiny(8)
        lat = [initial_latents(0, off + i, cfg) for i in range(len(mine))]
        outq.put((rank, mine, off, lists, [m.numpy().copy() for m in masks], mx, [x.numpy() for x in lat]))
    finally:
        dist.destroy_process_group()


def test_data_parallel_host_path_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, m0, o0, l0, k0, x0, lat0), (_, m1, o1, l1, k1, x1, lat1) = res
    assert m0 + m1 == [f"p{i}" for i in range(10)] and o0 == 0 and o1 == len(m0)
    assert l0 == l1 and l1[3][2] == [3, 2, 7]
    for a, b in zip(k0, k1):
        assert np.array_equal(a, b)
    assert x0 == x1 == 2.0
    # world-size independence: latents of global prompt i are the same as a 1-process run
    import sys
    sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import initial_latents
    cfg = UNetConfig.tiny(8)
    for i, x in enumerate(lat0 + lat1):
        assert np.array_equal(x, initial_latents(0, i, cfg).numpy())


class OraclePipe:
    """CPU stand-in for sdmoe.pipeline.StableDiffusionPipeline in the gloo test (the HIP path has no CPU backend):
    the same call contract -- a prompt list in, per-prompt latents out, latents seeded by prompt_offset + index --
    computed by the fp32 oracle. Its FFN hook is the reference hook arithmetic driven by the RemoveExperts
    receiver's own (t, l) lists and counter, so the receiver's per-call state machine runs exactly as in the
    product pipeline; the module tree (sdmoe.unet, CPU) only carries the hooked GEGLUs."""

    def __init__(self, cfg, sd, steps):
        from sdmoe.unet import UNet2DConditionModel
        from oracle.unet_ref import UNetRef
        self.cfg, self.steps = cfg, steps
        self.unet = UNet2DConditionModel.from_state_dict(sd, cfg, "cpu")
        self.ref = UNetRef({k: v.half().float() for k, v in sd.items()}, cfg)
        self.prompt_offset = 0
        self.receiver = None

    def __call__(self, prompts, safety_checker=None, **kw):
        from oracle import hooks_ref as H
        from oracle.unet_ref import denoise
        from sdmoe.pipeline import initial_latents, prompt_embedding, PipelineOutput
        rec = self.receiver
        mods = [m for n, m in self.unet.named_modules() if n.endswith("ff.net.0")]
        seed = torch.initial_seed()
        lat = torch.cat([initial_latents(seed, self.prompt_offset + i, self.cfg) for i in range(len(prompts))])
        d = self.cfg.cross_attention_dim

        def factory(step):
            def hook(layer, x, w, b):
                m = mods[layer]
                ids = rec.expert_indices[rec.timestep][rec.layer]
                out = H.geglu_hook(x, w, b, H.patterns_from_labels(m.labels.numpy()), m.k, "gelu", removed=ids,
                                   apply_removal=rec.timestep < 20)[0]
                rec.update_time_layer()
                return out
            return hook
        out = denoise(self.ref, lat, torch.stack([prompt_embedding("", d)] * len(prompts)),
                      torch.stack([prompt_embedding(p, d) for p in prompts]), num_inference_steps=self.steps,
                      ff_hook_factory=factory)
        return PipelineOutput(images=[out[i] for i in range(len(prompts))])


def _make_job(T=2):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
    from sdmoe.config import UNetConfig
    from sdmoe.weights import make_state_dict
    from moefication.helper import moefy_synthetic
    cfg = UNetConfig.tiny(8)
    pipe = OraclePipe(cfg, make_state_dict(cfg, 0), T)
    moefy_synthetic(pipe, 0.25, 16, seed=1)
    E = [m.patterns.shape[0] for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    return pipe, E


def _pipeline_worker(rank, world_size, port, outq):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        from sdmoe import distributed as D
        from neuron_receivers import RemoveExperts
        from test_distributed import _make_job
        pipe, E = _make_job()
        rng = np.random.default_rng(5)
        lists = {t: {l: sorted(rng.choice(E[l], size=2, replace=False).tolist()) for l in range(len(E))}
                 for t in range(2)} if rank == 0 else None
        lists = D.broadcast_object(lists)  # produced on rank 0, broadcast once
        rec = RemoveExperts(0, None, 2, len(E), expert_indices=lists, store_gates=False)
        pipe.receiver = rec
        prompts = [f"synthetic prompt {i}" for i in range(4)]
        out, off = D.run_shard(pipe, rec, prompts)
        mx = D.max_over_ranks(float(rank), "cpu")
        outq.put((rank, off, [o.numpy() for o in out], lists, (rec.timestep, rec.layer), mx))
    finally:
        dist.destroy_process_group()


def test_data_parallel_pipeline_world2():
    """bench.py's DP path end to end on CPU (gloo, 2 ranks): expert lists produced on rank 0 and broadcast once,
    contiguous prompt shards seeded by their global index, every rank's receiver driving its own pipeline call
    through observe_activation; each rank's images equal the single-process images of the same prompts."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_pipeline_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, o0, imgs0, l0, c0, mx), (_, o1, imgs1, l1, c1, _) = res
    assert (o0, o1) == (0, 2) and l0 == l1 and c0 == c1 == (2, 0) and mx == 1.0
    from neuron_receivers import RemoveExperts
    pipe, E = _make_job()
    rec = RemoveExperts(0, None, 2, len(E), expert_indices=l0, store_gates=False)
    pipe.receiver = rec
    from sdmoe import distributed as D
    prompts = [f"synthetic prompt {i}" for i in range(4)]
    full, off = D.run_shard(pipe, rec, prompts, rank=0, world_size=1)
    assert off == 0
    for a, b in zip(imgs0 + imgs1, full):
        np.testing.assert_allclose(a, b.numpy(), rtol=1e-4, atol=1e-4)


def test_bench_launcher_starts_n_ranks():
    """`bench.py --gpus 2` with no external launcher starts 2 ranks itself (torch.distributed.run as a child
    process); --launch-probe makes each rank join a gloo group instead of touching a GPU, and rank 0 reports the
    group's size."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-probe"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"probe": True, "n_gpus": 2, "rank_sum": 1}], r.stdout


def test_bench_refuses_world_size_mismatch():
    """--gpus N inside a process group of another size is an error, never a silent 1-rank measurement."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--launch-probe"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
