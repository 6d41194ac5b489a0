"""Per-op / per-shape time breakdown of one CFG U-Net evaluation (bench workload) with HIP events.

usage: python tools/op_breakdown.py [--batch 8] [--evals 2]
Wraps every sdmoe.ops launch with events on the current stream, groups by (op, shape) and prints
time / count / achieved TFLOP/s (GEMM, conv, attention) or GB/s (norms, routing) per group."""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import ops  # noqa: E402

REC = defaultdict(lambda: [0, 0.0, 0.0, []])  # key -> [count, flops, bytes, event pairs]
ACTIVE = [False]


def key_flops(name, a, k, out):
    if name == "conv3x3_launch":
        nimg, H, W, Cin, w = a[2], a[3], a[4], a[5], a[6]
        Cout, stride, up = a[15], a[16], a[17]
        M = out.shape[0]
        return (f"conv {H}x{W} s{stride}{'u' if up else ''} {Cin}->{Cout} M={M}", 2.0 * M * Cout * 9 * Cin, 0)
    if name == "conv3x3_gn_launch":  # same leading arguments; GroupNorm(+SiLU) applied inside the halo conv
        if out is None:  # shape not normalised in the kernel: the caller falls back (apply + conv, timed there)
            return ("conv+gn declined", 0, 0)
        nimg, H, W, Cin, Cout = a[2], a[3], a[4], a[5], a[15]
        M = out.shape[0]
        return (f"conv+gn {H}x{W} s1 {Cin}->{Cout} M={M}", 2.0 * M * Cout * 9 * Cin, 0)
    if name == "linear":
        x, w = a[0], a[1]
        M, K = x.shape
        N = w.shape[0]
        return (f"linear M={M} N={N} K={K}", 2.0 * M * N * K, 0)
    if name == "linear_ln":
        x, f = a[0], a[1]
        M, K = x.shape
        N = f.w.shape[0]
        return (f"linear_ln M={M} N={N} K={K}", 2.0 * M * N * K, 0)
    if name == "linear_geglu":
        x, w = a[0], a[1]
        M, K = x.shape
        N = (w if w is not None else k["ln"].w).shape[0]
        return (f"geglu{'-ln' if k.get('ln') is not None else ''} M={M} N={N} K={K}", 2.0 * M * N * K, 0)
    if name == "attention":
        q = a[0]
        nimg, Nq, Nk, heads = a[3], a[4], a[5], a[6]
        d = q.shape[1] // heads
        return (f"attn Nq={Nq} Nk={Nk} d={d} n={nimg}", 4.0 * nimg * heads * Nq * Nk * d, 0)
    if name == "linear_keep":
        x, w = a[0], a[2]
        M, K = x.shape
        return (f"linear_keep M={M} N={w.shape[0]} K={K}", 2.0 * M * w.shape[0] * K, 0)
    if name == "groupnorm":
        x = a[0]
        return (f"groupnorm {tuple(x.shape)}", 0, x.numel() * 2 * 3)
    if name in ("groupnorm_stats", "groupnorm_apply", "layernorm"):
        x = a[0]
        return (f"{name} {tuple(x.shape)}", 0, x.numel() * 2 * (1 if name == "groupnorm_stats" else 2))
    if name == "moe_topk_mask":
        P = a[0]
        return (f"topk_mask {tuple(P.shape)}", 0, P.numel() * 4)
    if name == "add":
        return (f"add {tuple(a[0].shape)}", 0, a[0].numel() * 6)
    if name == "moe_topk_keep":
        sc, routing, M = a[0], a[1], a[2]
        return (f"topk_keep {tuple(sc.shape)}", 0, sc.numel() * 2 + M * routing.E * routing.esize // 8)
    if name == "linear_per_image":
        x, wf = a[0], a[1]
        M, K = x.shape
        N = wf.shape[1]
        return (f"linear_per_image (GN-folded proj_in) M={M} N={N} K={K}", 2.0 * M * N * K, 0)
    if name == "gn_fold":
        nimg, N, K = a[2].shape[0], a[0].shape[0], a[0].shape[1]
        return (f"gn_fold nimg={nimg} N={N} K={K}", 0, nimg * N * K * 2)
    return (name, 0, 0)


def wrap(name):
    orig = getattr(ops, name)

    def w(*a, **k):
        if not ACTIVE[0]:
            return orig(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(*a, **k)
        e.record()
        key, fl, by = key_flops(name, a, k, out)
        r = REC[key]
        r[0] += 1
        r[1] += fl
        r[2] += by
        r[3].append((s, e))
        return out
    setattr(ops, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--evals", type=int, default=2)
    a = ap.parse_args()
    for n in ("conv3x3_launch", "conv3x3_gn_launch", "linear", "linear_ln", "linear_geglu", "linear_keep", "groupnorm", "attention", "groupnorm_stats", "groupnorm_apply",
              "layernorm", "moe_topk_mask", "moe_topk_keep", "add", "mask_weight", "geglu_route", "gn_fold",
              "linear_per_image"):
        wrap(n)
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import RemoveExperts
    import bench
    cfg = UNetConfig.sd14(64)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device="cuda:0", num_inference_steps=a.evals)
    find_and_change_geglu(pipe.unet)
    moefy_synthetic(pipe, 0.2, 20, seed=0)
    geglus = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    lists = bench.synth_expert_lists([m.patterns.shape[0] for m in geglus], a.evals)
    rec = RemoveExperts(0, None, a.evals, len(geglus), expert_indices=lists, store_gates=False)
    prompts = [f"p{i}" for i in range(a.batch)]
    rec.observe_activation(pipe, prompts)
    torch.cuda.synchronize()
    rec.reset_time_layer()
    ACTIVE[0] = True
    # keep the GPU busy while Python enqueues the whole run, so no event pair brackets host launch latency
    torch.cuda._sleep(int(2.0e9 * 0.3 * a.evals))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    rec.observe_activation(pipe, prompts)
    e.record()
    torch.cuda.synchronize()
    ACTIVE[0] = False
    wall = s.elapsed_time(e) / a.evals
    rows = []
    for key, (n, fl, by, ev) in REC.items():
        ms = sum(x.elapsed_time(y) for x, y in ev) / a.evals
        rows.append((ms, key, n // a.evals, fl / a.evals, by / a.evals))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"per U-Net eval (batch {2 * a.batch}): wall {wall:.2f} ms, sum of op events {tot:.2f} ms")
    for ms, key, n, fl, by in rows:
        rate = f"{fl / (ms / 1e3) / 1e12:7.1f} TF/s" if fl else (f"{by / (ms / 1e3) / 1e9:7.0f} GB/s" if by else "")
        print(f"{ms:8.3f} ms {100 * ms / tot:5.1f}%  x{n:<3d} {rate:>13}  {key}")


if __name__ == "__main__":
    main()
