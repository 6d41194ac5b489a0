"""Data parallelism for the denoising job: one process per GPU, prompts sharded contiguously,
masks produced once on rank 0 and broadcast (RCCL over xGMI on GPUs, gloo in CPU tests); no per-step
communication. Per-prompt latents are seeded by the GLOBAL prompt index, so every image is independent of the
world size (8-GPU output == 1-GPU output per prompt)."""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard(prompts, rank, world_size):
    """Contiguous shard of a global prompt list: (my prompts, global index of the first one)."""
    n = len(prompts)
    per = (n + world_size - 1) // world_size
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return list(prompts[lo:hi]), lo


def run_shard(pipe, receiver, prompts, rank=None, world_size=None):
    """This rank's part of a data-parallel batch: its contiguous shard of the GLOBAL prompt list, seeded at its
    global offset (pipe.prompt_offset), through the receiver's observe_activation (the reference call shape,
    base_receiver.py:40-77). Returns (outputs, offset)."""
    ws, rk = world()
    rank = rk if rank is None else rank
    world_size = ws if world_size is None else world_size
    mine, offset = shard(prompts, rank, world_size)
    pipe.prompt_offset = offset
    if hasattr(receiver, "reset_time_layer"):
        receiver.reset_time_layer()
    out, _ = receiver.observe_activation(pipe, mine)
    return out, offset


def broadcast_object(obj, src=0):
    """Python object (e.g. RemoveExperts lists {t: {l: [ids]}}) from `src` to every rank."""
    ws, rank = world()
    if ws == 1:
        return obj
    box = [obj if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def broadcast_tensors(tensors, src=0):
    """In-place broadcast of a list of same-shaped-on-every-rank tensors (bit-packed masks), coalesced into
    one flat buffer per dtype so the whole mask set moves in a single collective."""
    ws, _ = world()
    if ws == 1 or not tensors:
        return tensors
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dt, ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src=src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n
    return tensors


def max_over_ranks(value: float, device) -> float:
    ws, _ = world()
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
