"""Per-launch device time of U-Net ops at the bench's shapes (16 images), under one or more sdmoe_tune settings.

usage: python tools/micro_ab.py FAMILY [--tune "k=v,k=v"]... [--iters 50]
FAMILY: gn | linear | geglu | keep | conv | attn | topk | all. Each case is launched back to back `iters` times between two HIP events on
the launch stream (warm L2: a relative A/B tool, not the pipeline's cold-cache numbers: tools/op_breakdown.py)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import _lib, ops  # noqa: E402

DEV = "cuda"
N_IMG = 16


DEFAULTS = {"7": 1, "8": 1, "14": 1, "16": 1, "20": 1, "21": 1, "23": 1}  # sdmoe_tune knobs whose default is not 0


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).half()


def gn_cases():
    out = []
    for HW, C in [(4096, 320), (4096, 640), (4096, 960), (1024, 640), (1024, 1280), (1024, 1920), (1024, 960),
                  (256, 1280), (256, 2560), (256, 1920), (64, 1280), (64, 2560)]:
        x = rnd(N_IMG * HW, C)
        g, b = rnd(C) * 0.1 + 1, rnd(C) * 0.1
        y = torch.empty_like(x)
        out.append((f"groupnorm+silu HW={HW} C={C}", lambda x=x, g=g, b=b, y=y, HW=HW:
                    ops.groupnorm(x, N_IMG, HW, g, b, 1e-5, 32, True, out=y), 3 * x.numel() * 2, "B"))
        if HW > 256:
            out.append((f"groupnorm stats HW={HW} C={C}", lambda x=x, g=g, b=b, HW=HW:
                        ops.groupnorm_stats(x, N_IMG, HW, g, b, 1e-5, 32), x.numel() * 2, "B"))
    return out


def linear_cases():
    out = []
    for M, N, K, res in [(65536, 320, 320, True), (65536, 320, 320, False), (16384, 640, 640, True),
                         (16384, 640, 640, False), (4096, 1280, 1280, True), (4096, 1280, 1280, False),
                         (65536, 960, 320, False), (1024, 1280, 1280, True)]:
        M = M * N_IMG // 16  # the bench's rows at 16 images; --nimg 2 gives the one-prompt shapes
        x, w, bias = rnd(M, K), rnd(N, K, scale=K ** -0.5), rnd(N, scale=0.1)
        r = rnd(M, N) if res else None
        y = torch.empty(M, N, device=DEV, dtype=torch.float16)
        out.append((f"linear M={M} N={N} K={K}{' +res' if res else ''}",
                    lambda x=x, w=w, bias=bias, r=r, y=y: ops.linear(x, w, bias, residual=r, out=y), 2 * M * N * K, "F"))
    return out


def geglu_cases():
    """The fused routed GEGLU projection (relu, expert 20, top-k 0.2) and the LN-folded QKV at each U-Net level."""
    out = []
    for M, C in [(65536, 320), (16384, 640), (4096, 1280)]:
        M = M * N_IMG // 16
        F, E = 4 * C, 4 * C // 20
        x = rnd(M, C)
        w = rnd(2 * F, C, scale=C ** -0.5)
        routing = ops.Routing(torch.randperm(F) % E, E, E // 5, DEV)
        w_il, b_il = ops.interleave_geglu(w, rnd(2 * F, scale=0.1), routing.perm)
        score = torch.empty(M, E, device=DEV, dtype=torch.float16)
        o = torch.empty(M, F, device=DEV, dtype=torch.float16)
        out.append((f"geglu M={M} N={2 * F} K={C}", lambda x=x, w_il=w_il, b_il=b_il, score=score, o=o, r=routing:
                    ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=r.esize, out=o),
                    2 * M * 2 * F * C, "F"))
        fold = ops.LNFold(rnd(3 * C, C, scale=C ** -0.5), rnd(C) * 0.1 + 1, rnd(C) * 0.1, 1e-5)
        out.append((f"linear_ln M={M} N={3 * C} K={C}", lambda x=x, f=fold: ops.linear_ln(x, f), 2 * M * 3 * C * C, "F"))
    return out


def keep_cases():
    """The routed FFN down projection (keep-masked A operand, + residual) at each U-Net level (20 % of neurons kept)."""
    out = []
    for M, C in [(N_IMG * 4096, 320), (N_IMG * 1024, 640), (N_IMG * 256, 1280)]:
        F = 4 * C
        x, w, bias, r = rnd(M, F), rnd(C, F, scale=F ** -0.5), rnd(C, scale=0.1), rnd(M, C)
        g = torch.Generator(device="cpu").manual_seed(M + C)
        keep = torch.randint(0, 2 ** 62, (F // 64, M), generator=g, dtype=torch.int64).to(DEV)
        y = torch.empty(M, C, device=DEV, dtype=torch.float16)
        out.append((f"keep M={M} N={C} K={F} +res", lambda x=x, keep=keep, w=w, bias=bias, r=r, y=y:
                    ops.linear_keep(x, keep, w, bias, residual=r, out=y), 2 * M * C * F, "F"))
    return out


def conv_cases():
    out = []
    for H, Cin, Cout in [(64, 320, 320), (64, 640, 320), (32, 640, 640), (32, 1280, 640), (32, 1920, 640), (32, 960, 640),
                         (16, 1280, 1280), (8, 1280, 1280), (8, 2560, 1280)]:
        x = rnd(N_IMG * H * H, Cin)
        w = ops.conv_weight(rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5))
        out.append((f"conv {H}x{H} {Cin}->{Cout}", lambda x=x, w=w, H=H: ops.conv3x3(x, N_IMG, H, H, w),
                    2 * N_IMG * H * H * Cout * 9 * Cin, "F"))
    for H, C in [(32, 640), (16, 1280), (8, 1280)]:  # the nearest-2x upsample convs (input H x H)
        x = rnd(N_IMG * H * H, C)
        w = ops.conv_weight(rnd(C, 3, 3, C, scale=(9 * C) ** -0.5))
        out.append((f"conv up {H}->{2 * H} {C}->{C}", lambda x=x, w=w, H=H: ops.conv3x3(x, N_IMG, H, H, w, upsample=True),
                    2 * N_IMG * 4 * H * H * C * 9 * C, "F"))
    return out


def attn_cases():
    out = []
    for N, C, heads in [(4096, 320, 8), (1024, 640, 8), (256, 1280, 8), (64, 1280, 8), (4096, 640, 10), (1024, 1280, 20)]:
        q = rnd(N_IMG * N, 3 * C)
        d = C // heads
        out.append((f"attn N={N} d={d}", lambda q=q, C=C, N=N, heads=heads:
                    ops.attention(q[:, :C], q[:, C:2 * C], q[:, 2 * C:], N_IMG, N, N, heads),
                    4 * N_IMG * heads * N * N * d, "F"))
    for N, C, heads in [(4096, 320, 8), (1024, 640, 8), (256, 1280, 8)]:  # cross-attention, 77 text keys
        q = rnd(N_IMG * N, C)
        kv = rnd(N_IMG * 77, 2 * C)
        d = C // heads
        out.append((f"attn N={N} Nk=77 d={d}", lambda q=q, kv=kv, C=C, N=N, heads=heads:
                    ops.attention(q, kv[:, :C], kv[:, C:], N_IMG, N, 77, heads),
                    4 * N_IMG * heads * N * 77 * d, "F"))
    return out


def topk_cases():
    """Top-k expert selection (keep bits for the down projection) at the U-Net levels' token counts."""
    out = []
    for M, E in [(65536, 64), (16384, 128), (4096, 256), (1024, 256)]:
        routing = ops.Routing(torch.arange(20 * E) // 20, E, E // 5, DEV)
        score = rnd(M, E)
        out.append((f"topk_keep M={M} E={E}", lambda score=score, r=routing, M=M: ops.moe_topk_keep(score, r, M),
                    M * E * 2 + M * 20 * E // 8, "B"))
    return out


def run(cases, iters):
    res = {}
    for name, f, work, unit in cases:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            f()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / iters
        rate = work / (us * 1e-6) / (1e12 if unit == "F" else 1e9)
        res[name] = (us, f"{rate:8.1f} {'TF/s' if unit == 'F' else 'GB/s'}")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("family")
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--nimg", type=int, default=16, help="images per launch (2 = one prompt with CFG)")
    a = ap.parse_args()
    global N_IMG
    N_IMG = a.nimg
    lib = _lib.load()
    fam = {"gn": gn_cases, "linear": linear_cases, "geglu": geglu_cases, "conv": conv_cases, "attn": attn_cases,
           "topk": topk_cases, "keep": keep_cases}
    cases = [c for k in (fam if a.family == "all" else [a.family]) for c in fam[k]()]
    settings = a.tune or [""]
    table = {}
    for rep in range(2):  # interleaved twice
        for st in settings:
            for k, v in _lib.parse_tune(st):
                _lib.check(lib.sdmoe_tune(k, v), "tune")
            r = run(cases, a.iters)
            for k, _ in _lib.parse_tune(st):  # back to defaults (0) unless the knob's default differs
                _lib.check(lib.sdmoe_tune(k, DEFAULTS.get(str(k), 0)), "tune")
            for name, v in r.items():
                table.setdefault(name, {}).setdefault(st, []).append(v)
    for name, per in table.items():
        cols = "  ".join(f"[{st or 'default'}] " + " / ".join(f"{us:7.2f} us" for us, _ in v) + f" {v[-1][1]}"
                         for st, v in per.items())
        print(f"{name:36s} {cols}", flush=True)


if __name__ == "__main__":
    main()
