"""Expert-gather feasibility data (VERDICT r1 'decide expert-gather with data'): at the bench's routing (SD-1.4
64x64, 8 prompts -> U-Net batch 16, relufied, top-k 0.2, RemoveExperts removal for t < 20) record, for every hooked
GEGLU call of the first `--steps` DDIM steps, from the fused path's own top-k keep bits (sdmoe_moe_topk_keep):
  * union_T: the fraction of experts selected by at least one token of a T-row tile (T = 64/128/256: the down
    projection's row tiles) -- an expert-gather value/down GEMM can skip an expert's weights only outside the union;
  * skip_T: the fraction of (T-row tile, 64-neuron K-step) pairs whose keep bits are all zero -- the K-steps
    sdmoe_linear_keep could skip outright;
  * nz_act: nonzero fraction of value*relu(gate) before the top-k mask; nz_kept: after it.
With --model sdxl: SDXL-base 1024^2 (128x128 latents), its own GELU FFN (not relufied), U-Net batch 2 * --batch,
E = 128 / 256 experts (BASELINE config 5's routing).
usage: python tools/expert_union.py [--model sd14|sdxl] [--steps 2] [--out gpurun_out/expert_union.json]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="prompts (default 8 for sd14, 2 for sdxl: the bench's)")
    ap.add_argument("--model", choices=("sd14", "sdxl"), default="sd14")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "expert_union.json"))
    a = ap.parse_args()
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import RemoveExperts
    import bench

    dev = "cuda:0"
    sdxl = a.model == "sdxl"
    if a.batch is None:
        a.batch = 2 if sdxl else 8
    cfg = UNetConfig.sdxl(128) if sdxl else UNetConfig.sd14(64)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device=dev, num_inference_steps=50)
    if not sdxl:
        find_and_change_geglu(pipe.unet)  # relufied SD-1.4; SDXL keeps its GELU (utils.py:111-112)
    moefy_synthetic(pipe, 0.2, 20, seed=0)
    geglus = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    lists = bench.synth_expert_lists([m.patterns.shape[0] for m in geglus], 50)
    rows = []

    class Rec(RemoveExperts):
        def hook_fn(self, module, input, output):
            t, l = self.timestep, self.layer
            out = super().hook_fn(module, input, output)
            if t >= a.steps:
                raise StopIteration
            keep = module._out_keep[0]  # int64 [F/64, M] keep bits of the expert-major neurons
            F64, M = keep.shape
            E, es = module.patterns.shape[0], module._routing.esize
            first = torch.arange(E, device=keep.device) * es
            kb = ((keep[first // 64, :] >> (first % 64)[:, None]) & 1).bool()  # [E, M] expert kept per token
            r = {"t": t, "layer": l, "M": M, "E": E, "k": module.k, "removed": len(self.expert_indices[t][l]) if t < 20 else 0,
                 "sel_per_token": float(kb.float().sum(0).mean())}
            for T in (64, 128, 256):
                n = M // T
                r[f"union_{T}"] = float(kb[:, :n * T].view(E, n, T).any(-1).float().mean())
                r[f"skip_{T}"] = float(1.0 - (keep[:, :n * T].view(F64, n, T) != 0).any(-1).float().mean())
            P = out.reshape(M, -1)
            r["nz_act"] = float((P != 0).float().mean())
            bits = ((keep.t()[:, :, None] >> torch.arange(64, device=keep.device)) & 1).reshape(M, -1).bool()
            r["nz_kept"] = float(((P != 0) & bits).float().mean())
            rows.append(r)
            return out

    rec = Rec(0, None, 50, len(geglus), expert_indices=lists, store_gates=False)
    prompts = [f"synthetic prompt {i}" for i in range(a.batch)]
    try:
        rec.observe_activation(pipe, prompts)
    except StopIteration:
        pass
    torch.cuda.synchronize()
    summary = {}
    for key in ("union_64", "union_128", "union_256", "skip_64", "skip_128", "skip_256", "nz_act", "nz_kept",
                "sel_per_token"):
        summary[key] = {"mean": float(np.mean([r[key] for r in rows])), "min": float(np.min([r[key] for r in rows])),
                        "max": float(np.max([r[key] for r in rows]))}
    what = ("SDXL-base 128x128, U-Net batch %d, GELU" % (2 * a.batch) if sdxl else
            "SD-1.4 64x64, U-Net batch %d, relu" % (2 * a.batch))
    res = {"what": f"per hooked GEGLU call, bench routing ({what}, top-k 0.2, RemoveExperts t<20)",
           "calls": len(rows), "summary": summary, "per_call": rows}
    by_e = {}
    for r in rows:
        by_e.setdefault(r["E"], []).append(r)
    res["by_experts"] = {str(E): {key: float(np.mean([r[key] for r in rs])) for key in
                                  ("union_64", "union_128", "union_256", "skip_64", "skip_128", "skip_256")}
                         for E, rs in sorted(by_e.items())}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({"summary": summary, "by_experts": res["by_experts"]}, indent=1))


if __name__ == "__main__":
    main()
