"""Host-side issue cost of the bench's pipeline call: how long the Python/ctypes layer takes to ENQUEUE one step
(50 U-Net evaluations) against the GPU time of the same step, and a cProfile of the enqueue (top functions by own
time). When the enqueue time approaches the GPU time, the short-kernel phases (8x8 / 16x16 latents) leave the GPU
waiting on the host.

usage: python tools/host_issue_profile.py [bench.py args, e.g. --mask remove]"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:] + ["--no-cpu-baseline", "--e2e-steps", "0"]
    args = bench.parse()
    args.batch = args.batch or 8
    world, rank, local = bench.setup_dist(1)
    from sdmoe import _lib
    from sdmoe import ops as ops_mod
    from sdmoe import distributed as D
    _lib.load()
    cfg, pipe, rec, wanda, _ = bench.build(args, 1, 0, "cuda:0")
    prompts = [f"synthetic prompt {i}" for i in range(args.batch)]

    def step():
        return D.run_shard(pipe, rec, prompts, 0, 1)

    step()
    torch.cuda.synchronize()
    # GPU time of one step (host far ahead is not guaranteed, so this is wall with a sync at the end)
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # host cost per op: 200 tiny launches (well inside the hardware queue) of two representative wrappers
    x = torch.randn(256, 320, device="cuda").half()
    w = torch.randn(320, 320, device="cuda").half()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        ops_mod.linear(x, w)
    lin_us = (time.perf_counter() - t0) / 200 * 1e6
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        torch.cuda.current_stream().cuda_stream
    cs_us = (time.perf_counter() - t0) / 200 * 1e6
    prof = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prof.enable()
    step()
    prof.disable()
    torch.cuda.synchronize()
    pwall = time.perf_counter() - t0
    st = pstats.Stats(prof)
    ncalls = sum(v[1] for k, v in st.stats.items() if k[0].endswith(os.path.join("sdmoe", "ops.py"))
                 and not k[2].startswith("_"))
    print(f"step wall {wall * 1e3:.1f} ms; under cProfile {pwall * 1e3:.1f} ms; ops.* calls per step {ncalls} "
          f"({ncalls / args.inference_steps:.0f} per U-Net eval); host cost of ops.linear on a tiny shape "
          f"{lin_us:.1f} us per call, torch.cuda.current_stream().cuda_stream {cs_us:.1f} us", flush=True)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(45)
    pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
