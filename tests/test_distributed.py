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
