#!/usr/bin/env python3
"""Headline benchmark: images/sec of the MoE-fied SD-1.4 denoising step on MI355X (BASELINE.json metric).

Workload (one bench "step" = one batch of B prompts per GPU denoised end to end):
  SD-1.4 U-Net (859.5M params, synthetic seeded weights), 512^2 -> 4x64x64 latents, 50 DDIM steps, CFG 7.5,
  relufied + MoE-fied FFNs (expert size 20, top-k 0.2), skilled-expert removal mask active
  (RemoveExperts: ~10 % of each layer's experts removed for t < 20) driven through the reference receiver API
  (observe_activation -> forward hooks on all 16 GEGLU FFNs). --mask union additionally applies a 10-concept
  union Wanda down-projection mask at every step (config 4).
Multi-GPU: one process per GPU (torchrun), prompts sharded data-parallel (weak scaling, B per GPU), masks
generated on rank 0 and broadcast once over RCCL; no per-step communication.

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the roofline and baseline definitions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

TFLOP_PER_IMAGE = {"sd14": 81.34,   # SD-1.x 512^2, 50 steps, CFG, MoE scoring on
                   "sdxl": 694.9}   # SDXL-base 1024^2, 50 steps, CFG, MoE scoring on
PEAK_FP16_TFLOPS = 2500.0     # MI355X dense FP16/BF16 MFMA (MI355X_MICROARCH.md, chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", choices=["sd14", "sdxl"], default="sd14",
                   help="sd14: SD-1.4 512^2 (the metric, configs 2-4); sdxl: SDXL-base 1024^2 (config 5)")
    p.add_argument("--batch", type=int, default=None,
                   help="prompts per GPU (default 8 = config 4's 64 prompts / 8 GPUs; 2 for sdxl)")
    p.add_argument("--inference-steps", type=int, default=50)
    p.add_argument("--scheduler", choices=["ddim", "pndm"], default="ddim",
                   help="ddim: the metric (50 U-Net calls); pndm: the reference's default (51 calls)")
    p.add_argument("--mask", choices=["remove", "union", "none"], default="remove")
    p.add_argument("--topk", type=float, default=0.2)
    p.add_argument("--act", choices=["relu", "gelu"], default=None,
                   help="FFN gate activation: relu = the relufied U-Net (find_and_change_geglu; default for sd14, the "
                        "reference's fine-tuned relufied SD, utils.py:66-74); gelu = the model's own GELU (default for "
                        "sdxl: the reference loads SDXL-base without relufying it, utils.py:111-112)")
    p.add_argument("--topk-mask", choices=["down", "pass"], default="down",
                   help="down: the top-k mask is applied by the down projection as it reads the GEGLU product "
                        "(sdmoe_linear_keep); pass: a separate masking pass over the product (A/B reference)")
    p.add_argument("--decode", action="store_true",
                   help="also run the CLIP text encoder and the VAE decoder inside the timed step (end-to-end "
                        "images; the metric excludes them, SURVEY §8d)")
    p.add_argument("--e2e-steps", type=int, default=1,
                   help="after the timed metric run, time this many end-to-end steps (text encoder + denoise + VAE "
                        "decode to RGB) and report them as 'end_to_end' (0: skip)")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--roofline-sample", type=int, default=25,
                   help="time the conv launches of every N-th U-Net evaluation (1 = every launch; event markers idle "
                        "the GPU ~5.7 us each)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-evals", type=int, default=2, help="CPU oracle U-Net evaluations to time")
    p.add_argument("--cpu-full-image", action="store_true",
                   help="cpu_baseline: time one whole image (all inference steps of the oracle's DDIM+CFG loop, "
                        "several minutes) instead of the bounded cpu-evals sample")
    p.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--traffic", type=str, default=None,
                   help="PMC summary json from tools/pmc_traffic.py (HBM bytes per conv launch); default "
                        "profiles/pmc_conv_traffic.json (8 prompts/GPU) or profiles/pmc_conv_traffic_b<B>.json; used "
                        "only when its recorded model / prompts per GPU / mask are this run's")
    return p.parse_args()


def launch_ranks(n, argv):
    """`bench.py --gpus N` without an external launcher: start N fresh worker processes (one per GPU) under
    torch.distributed.run as a CHILD process -- this process has made no GPU call, and it does not exec -- and exit
    with the workers' status. Rank 0's JSON line reaches stdout through the child's inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free port on the loopback interface for the rendezvous
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def setup_dist(n):
    """One process per GPU over RCCL ("nccl"). SDMOE_SAME_DEVICE_REHEARSAL=1 (rehearsal of the N > 1 code path on a
    one-GPU box, never used for a measurement): every rank on cuda:0, gloo collectives.
    The process group must have exactly n ranks (`--gpus n`): a mismatch is an error, not a silent 1-GPU run."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"bench.py: --gpus {n} but WORLD_SIZE={world}; launch with --nproc-per-node {n} (or run "
                         f"`bench.py --gpus {n}` with no launcher and it starts the ranks itself)")
    if world > 1 and os.environ.get("SDMOE_SAME_DEVICE_REHEARSAL") == "1":
        local = 0
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def synth_expert_lists(num_experts, T, seed=7):
    """RemoveExperts "Van Gogh" stand-in: ~10 % of E per (t, l) for t < 20 (no real lists offline)."""
    rng = np.random.default_rng(seed)
    out = {}
    for t in range(T):
        out[t] = {}
        for l, E in enumerate(num_experts):
            out[t][l] = sorted(rng.choice(E, size=max(1, E // 10), replace=False).tolist()) if t < 20 else []
    return out


def build(args, world, rank, dev):
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    from moefication.helper import moefy_synthetic
    from sparsity.relufy_model import find_and_change_geglu
    from neuron_receivers import RemoveExperts, MOEFy, WandaRemoveNeuronsFast
    from sdmoe import distributed as D

    cfg = UNetConfig.sdxl(128) if args.model == "sdxl" else UNetConfig.sd14(64)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device=dev, num_inference_steps=args.inference_steps,
                                             scheduler=args.scheduler)
    e2e = None
    if args.decode or (args.e2e_steps > 0 and args.model == "sd14"):
        from sdmoe.clip import attach_text_encoders
        from sdmoe.vae import AutoencoderKLDecoder, VAEConfig, make_vae_state_dict
        vae = AutoencoderKLDecoder(make_vae_state_dict(VAEConfig.sd14(), 0), VAEConfig.sd14(), dev)
        attach_text_encoders(pipe, seed=0)
        e2e = (pipe.text_encoder, vae)

    def set_e2e(on):
        """end-to-end mode: CLIP text encoder in front, VAE decode to RGB behind; off: the metric's workload
        (synthetic context, latents out)."""
        pipe.text_encoder = e2e[0] if on else None
        pipe.vae = e2e[1] if on else None
        pipe.output_type = "pt" if on else "latent"
    if e2e is not None:
        set_e2e(args.decode)
    if args.act == "relu":
        find_and_change_geglu(pipe.unet)              # relufied U-Net (configs 2-4); SDXL keeps its GELU (config 5)
    moefy_synthetic(pipe, args.topk, 20, seed=0)      # E = 4C/20 experts, k = int(E*topk)
    geglus = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.0")]
    T = args.inference_steps + (1 if args.scheduler == "pndm" else 0)  # U-Net calls = counter timesteps
    # masks are produced on rank 0 and broadcast once (RCCL); every rank then holds identical device copies
    if args.mask == "none":
        rec = MOEFy(seed=0, store_gates=False)
    else:
        lists = D.broadcast_object(synth_expert_lists([m.patterns.shape[0] for m in geglus], T) if rank == 0
                                   else None)
        rec = RemoveExperts(0, None, T, len(geglus), expert_indices=lists, store_gates=False)
    wanda = None
    if args.mask == "union":
        downs = [m for n, m in pipe.unet.named_modules() if n.endswith("ff.net.2")]
        # 10-concept union, each concept Bernoulli(0.0025) per weight (the union density of ten masks like
        # weights_320_1280.csv after save_union_experts' 95 % drop): drawn on device, bit-packed on device
        p_union = 1.0 - (1.0 - 0.0025) ** 10
        weights8 = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=dev)
        gen = torch.Generator(device=dev)
        bits = {}
        for t in range(T):
            bits[t] = {}
            for l, d in enumerate(downs):
                shape = tuple(d.weight.shape)
                if rank == 0:
                    gen.manual_seed(1000 * t + l)
                    m = torch.rand(shape, generator=gen, device=dev) < p_union
                    b = (m.view(shape[0], shape[1] // 8, 8).to(torch.uint8) * weights8).sum(-1, dtype=torch.uint8)
                else:
                    b = torch.empty((shape[0], shape[1] // 8), dtype=torch.uint8, device=dev)
                bits[t][l] = b.contiguous()
        D.broadcast_tensors([bits[t][l] for t in range(T) for l in range(len(downs))])  # once, over RCCL
        wanda = WandaRemoveNeuronsFast.from_packed(0, {t: {l: np.zeros((1, 1), np.uint8) for l in range(len(downs))}
                                                       for t in range(T)}, T, len(downs), store_gates=False)
        for t in range(T):
            for l in range(len(downs)):
                wanda._dev[(t, l)] = bits[t][l]
    return cfg, pipe, rec, wanda, (set_e2e if e2e is not None else None)


class KernelTimer:
    """HIP-event timing of the launches of one kernel family on the stream it is launched on, over the timed region.

    Sampled by U-Net evaluation: every `sample_every`-th evaluation of the timed steps has ALL its launches of the
    family bracketed by an event pair (2 of the 50 evaluations of a step: all 52 conv shapes each); the others run
    untouched. Each event record is a marker packet that idles the GPU for ~5.7 us between kernels (rocprofv3 kernel
    trace: a gap at every conv boundary, 0.6 ms per evaluation when all 104 records per evaluation were taken), so
    timing every launch slowed the very step it measures: 9.12 images/s timed at every launch vs 9.28 at every 10th
    evaluation vs 9.30 untimed (same box, same conv average 1.02-1.03 PFLOP/s)."""

    def __init__(self, family, sample_every=25):
        self.family = family
        self.pairs = []
        self.flops = 0.0
        self.bytes = 0.0
        self.active = False
        self.sample_every = max(1, int(sample_every))
        self.evals = 0
        self.sampled_evals = 0
        self.on_eval = False

    def wrap_evals(self, unet):
        """Count U-Net evaluations (forward_nhwc) while active; launches are timed only in sampled evaluations."""
        orig = unet.forward_nhwc
        timer = self

        def wrapped(*a, **k):
            if timer.active:
                timer.on_eval = timer.evals % timer.sample_every == 0
                timer.sampled_evals += int(timer.on_eval)
                timer.evals += 1
            try:
                return orig(*a, **k)
            finally:
                timer.on_eval = False
        unet.forward_nhwc = wrapped

    def wrap(self, ops_mod, family=None):
        """Time every launch of `family` (default self.family); several families (the conv with and without the
        in-kernel GroupNorm) can feed one timer."""
        family = family or self.family
        orig = getattr(ops_mod, family)
        timer = self

        def wrapped(*a, **k):
            if not (timer.active and timer.on_eval):
                return orig(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = orig(*a, **k)
            e.record()
            if out is not None:  # (sdmoe_conv3x3_gn declined the shape: nothing launched)
                timer.pairs.append((s, e))
                timer.account(a, k, out)
            return out
        setattr(ops_mod, family, wrapped)
        import sdmoe.unet as U
        if hasattr(U.ops, family):
            setattr(U.ops, family, wrapped)

    def account(self, a, k, out):
        # conv3x3_launch(xp, ldx, nimg, H, W, Cin, w, ...): algorithmic FLOPs = 2 * M * Cout * 9 * Cin (real
        # channel counts: conv_in has 4 of its 64 padded input channels, conv_out 4 of its 8 padded outputs)
        w = a[6]
        cin_real = 4 if getattr(w, "_sdmoe_conv_in", False) else a[5]
        M = out.shape[0]
        N = 4 if getattr(w, "_sdmoe_conv_out", False) else w.shape[0]
        self.flops += 2.0 * M * N * 9 * cin_real
        if k.get("sc") is not None:  # folded 1x1 shortcut (sdmoe_conv3x3_sc): + 2 * M * Cout * Cin2
            self.flops += 2.0 * M * N * k["sc"][2]

    def result(self):
        torch.cuda.synchronize()
        ms = sum(s.elapsed_time(e) for s, e in self.pairs)
        n = len(self.pairs)
        return n, ms, self.flops


def cpu_baseline(args):
    """The oracle (fp32 CPU restatement of the reference path, incl. the hook's projection recompute) timed on
    this host's cores for a bounded sample: `cpu_evals` CFG U-Net evaluations at B=1 (one denoising step each)."""
    from oracle.unet_ref import UNetRef
    from oracle import hooks_ref as H
    from sdmoe.config import UNetConfig
    from sdmoe.weights import make_state_dict
    from sdmoe.pipeline import prompt_embedding
    from moefication.helper import balanced_random_labels
    import torch.nn.functional as F

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    cfg = UNetConfig.sd14(64)
    ref = UNetRef(make_state_dict(cfg, 0), cfg)
    layers = []
    for i, (_, C) in enumerate(cfg.geglu_layers()):
        lab = balanced_random_labels(4 * C, 20, i)
        E = 4 * C // 20
        layers.append((H.patterns_from_labels(lab), int(E * args.topk)))
    rng = np.random.default_rng(7)

    def hook(layer, x, w, b):
        F.linear(x, w, b)  # the module's own GEGLU forward, which the reference hook then recomputes (K1)
        P, k = layers[layer]
        ids = rng.choice(P.shape[0], size=max(1, P.shape[0] // 10), replace=False).tolist()
        return H.geglu_hook(x, w, b, P, k, "relu", removed=ids)[0]

    x = torch.randn(2, 4, 64, 64)
    ctx = torch.stack([prompt_embedding("", 768), prompt_embedding("a painting", 768)])
    if args.cpu_full_image:  # one measured image: the oracle's whole DDIM + CFG loop
        from oracle.unet_ref import denoise

        def factory(step):
            print(f"[cpu_baseline] step {step}", file=sys.stderr, flush=True)
            return hook
        with torch.no_grad():
            ref(x, 981.0, ctx, ff_hook=hook)  # warm-up (allocator, threads)
            t0 = time.perf_counter()
            denoise(ref, x[:1], ctx[:1], ctx[1:], num_inference_steps=args.inference_steps, ff_hook_factory=factory)
            per_image = time.perf_counter() - t0
        return {"value": 1.0 / per_image, "unit": "images/s", "cores": threads, "kind": "port",
                "sample": f"one whole image measured: {args.inference_steps} DDIM steps x CFG U-Net eval (B=1, "
                          f"2x4x64x64, MoE routing + removal hooks) in {per_image:.1f} s"}
    with torch.no_grad():
        ref(x, 981.0, ctx, ff_hook=hook)  # warm-up (allocator, threads)
        t0 = time.perf_counter()
        for _ in range(args.cpu_evals):
            ref(x, 981.0, ctx, ff_hook=hook)
        dt = (time.perf_counter() - t0) / args.cpu_evals
    per_image = dt * args.inference_steps
    return {"value": 1.0 / per_image, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_evals} CFG U-Net evals (B=1, 2x4x64x64, MoE routing + removal hooks) at "
                      f"{dt:.2f} s each, x{args.inference_steps} steps per image"}


def metric_label(args):
    """BASELINE.json's metric string for the default run (SD-1.4, 50 DDIM steps); other runs say what they ran."""
    sched = f"{args.inference_steps}-step {args.scheduler.upper()}"
    if args.model == "sdxl":
        return f"images/sec SDXL-base 1024² {sched}, expert mask on (config 5)"
    mask = {"remove": "expert mask on", "union": "expert mask + union Wanda mask on", "none": "no mask"}[args.mask]
    return f"images/sec SD-1.4 512² {sched}, {mask}; 1→8 GPU scaling"


def launch_probe(args):
    """--launch-probe (CPU test of the launcher path, tests/test_distributed.py): each rank joins a gloo group, the
    ranks all-reduce their rank ids, rank 0 prints the line bench.py would print its n_gpus from. No GPU call."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    dist.init_process_group("gloo")
    t = torch.tensor([float(dist.get_rank())])
    dist.all_reduce(t)
    if dist.get_rank() == 0:
        print(json.dumps({"probe": True, "n_gpus": dist.get_world_size(), "rank_sum": int(t.item())}), flush=True)
    dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.launch_probe:
        return launch_probe(args)
    if args.batch is None:
        args.batch = 2 if args.model == "sdxl" else 8
    if args.traffic is None:
        args.traffic = os.path.join(ROOT, "profiles", "pmc_conv_traffic" + ("" if args.batch == 8 else
                                                                            f"_b{args.batch}") + ".json")
    if args.act is None:
        args.act = "gelu" if args.model == "sdxl" else "relu"
    world, rank, local = setup_dist(args.gpus)
    dev = f"cuda:{local}" if world > 1 else "cuda:0"
    from sdmoe import ops, _lib
    import sdmoe.unet as U
    _lib.load()
    U.FUSED_KEEP = args.topk_mask == "down"
    cfg, pipe, rec, wanda, set_e2e = build(args, world, rank, dev)
    # global prompt list: rank r takes its contiguous shard (per-prompt seeds use the global index)
    from sdmoe import distributed as D
    prompts = [f"synthetic prompt {i}" for i in range(world * args.batch)]

    timer = KernelTimer("conv3x3_launch", args.roofline_sample)
    if not args.no_roofline:
        timer.wrap(ops)
        timer.wrap(ops, "conv3x3_gn_launch")  # the 64x64-level ResNet convs with their GroupNorm applied in-kernel
        timer.wrap_evals(pipe.unet)
    pipe.unet.conv_in.weight._sdmoe_conv_in = True
    pipe.unet.conv_out.weight._sdmoe_conv_out = True

    def one_step():
        """One batch through the reference receiver API: this rank's shard of the global prompt list (seeded by
        global prompt index) through observe_activation(pipe, prompts) (sdmoe.distributed.run_shard)."""
        hooks = []
        if wanda is not None:
            wanda.reset_time_layer()
            hooks = wanda.register_hooks(pipe)
        try:
            out, _ = D.run_shard(pipe, rec, prompts, rank, world)
        finally:
            if wanda is not None:
                wanda.remove_hooks(hooks)
        return out

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        imgs = one_step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    timer.active = False
    if world > 1:
        dist.barrier()
    elapsed = D.max_over_ranks(t1 - t0, dev)
    finite = all(bool(torch.isfinite(x).all()) for x in imgs)
    images = world * args.batch * args.steps
    value = images / elapsed

    end_to_end = None
    if set_e2e is not None and not args.decode and args.e2e_steps > 0:
        set_e2e(True)
        one_step()  # warm the encoder / decoder shapes
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.e2e_steps):
            rgb = one_step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if world > 1:
            dist.barrier()
        el2 = D.max_over_ranks(t1 - t0, dev)
        set_e2e(False)
        end_to_end = {"value": round(world * args.batch * args.e2e_steps / el2, 4), "unit": "images/s",
                      "steps": args.e2e_steps, "ms_per_step": round(el2 / args.e2e_steps * 1e3, 2),
                      "what": "CLIP ViT-L text encoder (synthetic tokenizer) + the metric's denoise + VAE decode "
                              "to 512^2 RGB", "outputs_finite": all(bool(torch.isfinite(x).all()) for x in rgb)}

    roof = None
    if not args.no_roofline:
        n, ms, flops = timer.result()
        if n:
            achieved = flops / (ms / 1e3) / 1e12
            traffic, traffic_src = None, None
            pmc = json.load(open(args.traffic)) if args.traffic and os.path.exists(args.traffic) else {}
            # only a PMC run of THIS workload (model, prompts per GPU, mask) is evidence for this line's launches
            if pmc and (pmc.get("model"), pmc.get("batch"), pmc.get("mask")) == (args.model, args.batch, args.mask):
                traffic = pmc.get("bytes_per_launch")
                # not measured in this process: the committed rocprofv3 --pmc passes (FETCH_SIZE x2, WRITE_SIZE) of
                # this bench command on the build named in the file
                traffic_src = (f"{os.path.relpath(args.traffic, ROOT)} (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes"
                               f" of bench.py, build {pmc.get('build', '?')})")
            elif pmc:
                traffic_src = (f"null: {os.path.relpath(args.traffic, ROOT)} profiles model {pmc.get('model')}, "
                               f"{pmc.get('batch')} prompts/GPU, mask {pmc.get('mask')} -- not this run's launches")
            roof = {"bound": "mfma", "kernel": "sdmoe_conv3x3 / _sc / _gn: implicit-GEMM conv (gemm_kernel MODE 1/2 "
                                               "shifted tiles, MODE 9/11/12/14 halo tiles, + split-K reduce where used)",
                    "achieved": round(achieved, 1), "peak": PEAK_FP16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / PEAK_FP16_TFLOPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "launches": n, "avg_launch_ms": round(ms / n, 4),
                    "sampled": f"HIP events around every conv launch of every {timer.sample_every}th U-Net evaluation "
                               f"of the timed steps ({timer.sampled_evals} of {timer.evals})",
                    "algorithmic_flop_per_launch": round(flops / n)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "sd14":
        cpu = cpu_baseline(args)
    if rank == 0:
        line = {
            "metric": metric_label(args),
            "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp16", "data": "synthetic",
            "config": {"workload": f"{'SDXL-base' if args.model == 'sdxl' else 'SD-1.4'} MoE-fied ({args.act}, top-k {args.topk}, expert 20) + "
                                   f"{'RemoveExperts skilled-expert mask' if args.mask != 'none' else 'no mask'}"
                                   f"{' + union Wanda mask' if args.mask == 'union' else ''}, "
                                   f"{8 * cfg.sample_size}^2 (4x{cfg.sample_size}x{cfg.sample_size} latents), "
                                   f"{args.inference_steps} {args.scheduler.upper()} steps, CFG 7.5"
                                   f"{' + CLIP text encoder + VAE decode to 512^2 RGB' if args.decode else ''}",
                       "prompts_per_gpu": args.batch, "global_batch": world * args.batch,
                       "parallelism": f"dp{world}"},
            # TFLOP_PER_IMAGE is quoted for 50 U-Net calls; scale to this run's call count
            "step_mfma_frac": round(value / world * TFLOP_PER_IMAGE[args.model] *
                                    (args.inference_steps + (1 if args.scheduler == "pndm" else 0)) / 50 /
                                    PEAK_FP16_TFLOPS, 4),
            "roofline": roof, "cpu_baseline": cpu, "outputs_finite": finite, "end_to_end": end_to_end,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
