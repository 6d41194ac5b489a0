"""GEMM / conv tile x stages x split-K sweep in ONE process (warm L2, back-to-back launches between HIP events on the
launch stream): for every case, every config in --cfgs (tile:stages:ksplit, sdmoe_tune knobs 1 / 0 / 9; invalid
combinations fall back to the auto dispatch for that shape) is timed and the table printed with the auto config first.

usage: python tools/tile_sweep.py [--only SUBSTR] [--cfgs "0:0:0 1:2:0 ..."] [--iters 30]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import _lib, ops  # noqa: E402

DEV = "cuda"
N_IMG = 16


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).half()


def cases():
    out = []
    for H, Cin, Cout in [(8, 1280, 1280), (8, 2560, 1280), (16, 1280, 1280), (16, 2560, 1280), (32, 640, 640),
                         (32, 1280, 640), (64, 320, 320)]:
        x = rnd(N_IMG * H * H, Cin)
        w = ops.conv_weight(rnd(Cout, 3, 3, Cin, scale=(9 * Cin) ** -0.5))
        b = rnd(Cout, scale=0.1)
        y = torch.empty(N_IMG * H * H, Cout, device=DEV, dtype=torch.float16)
        out.append((f"conv {H}x{H} {Cin}->{Cout}", lambda x=x, w=w, b=b, y=y, H=H:
                    ops.conv3x3(x, N_IMG, H, H, w, b, out=y), 2.0 * N_IMG * H * H * Cout * 9 * Cin))
    for M, N, K, res in [(4096, 1280, 1280, True), (4096, 1280, 1280, False), (16384, 640, 640, True),
                         (65536, 320, 320, True), (65536, 320, 320, False), (1024, 1280, 1280, True)]:
        x, w, bias = rnd(M, K), rnd(N, K, scale=K ** -0.5), rnd(N, scale=0.1)
        r = rnd(M, N) if res else None
        y = torch.empty(M, N, device=DEV, dtype=torch.float16)
        out.append((f"linear M={M} N={N} K={K}{' +res' if res else ''}",
                    lambda x=x, w=w, bias=bias, r=r, y=y: ops.linear(x, w, bias, residual=r, out=y), 2.0 * M * N * K))
    for M, N, K in [(4096, 3840, 1280), (4096, 1280, 1280), (16384, 1920, 640), (65536, 960, 320)]:
        x, w = rnd(M, K), rnd(N, K, scale=K ** -0.5)
        fold = ops.LNFold(w, rnd(K) * 0.1 + 1, rnd(K) * 0.1, 1e-5)
        y = torch.empty(M, N, device=DEV, dtype=torch.float16)
        out.append((f"linear_ln M={M} N={N} K={K}", lambda x=x, fold=fold, y=y: ops.linear_ln(x, fold, out=y),
                    2.0 * M * N * K))
    for M, C in [(4096, 1280), (16384, 640), (65536, 320)]:
        F, E = 4 * C, C // 5
        x = rnd(M, C)
        w = rnd(2 * F, C, scale=C ** -0.5)
        b = rnd(2 * F, scale=0.1)
        routing = ops.Routing(torch.arange(F) % E, E, E // 5, DEV)
        w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
        score = torch.empty(M, E, device=DEV, dtype=torch.float16)
        pout = torch.empty(M, F, device=DEV, dtype=torch.float16)
        out.append((f"geglu M={M} F={F} K={C}", lambda x=x, w_il=w_il, b_il=b_il, score=score, pout=pout, e=routing.esize:
                    ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=e, out=pout), 2.0 * M * 2 * F * C))
    for M, C in [(4096, 1280), (16384, 640), (65536, 320)]:
        F, E = 4 * C, C // 5
        h = rnd(M, F)
        score = rnd(M, E)
        routing = ops.Routing(torch.arange(F) % E, E, E // 5, DEV)
        keep = ops.moe_topk_keep(score, routing, M)
        wd, r = rnd(C, F, scale=F ** -0.5), rnd(M, C)
        y = torch.empty(M, C, device=DEV, dtype=torch.float16)
        out.append((f"down-keep M={M} N={C} K={F} +res", lambda h=h, keep=keep, wd=wd, r=r, y=y:
                    ops.linear_keep(h, keep, wd, residual=r, out=y), 2.0 * M * C * F))
    return out


def time_us(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="'|'-separated substrings of case names")
    ap.add_argument("--cfgs", default="0:0:0 1:2:0 1:3:0 2:2:0 2:3:0 3:0:0 4:0:0 5:0:0 6:0:0 7:2:0 7:3:0 8:2:0 8:3:0")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    lib = _lib.load()
    cfgs = [tuple(int(v) for v in c.split(":")) for c in a.cfgs.split()]
    only = [o for o in a.only.split("|") if o]
    for name, fn, flop in cases():
        if only and not any(o in name for o in only):
            continue
        res = []
        ref = None
        bad = []
        for t, st, ks in cfgs:
            _lib.check(lib.sdmoe_tune(1, t), "tile")
            _lib.check(lib.sdmoe_tune(0, st), "stages")
            _lib.check(lib.sdmoe_tune(9, ks), "ksplit")
            y = fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.float().clone()
            else:  # every config must compute the same product (fp32 accumulation order may differ)
                err = ((y.float() - ref).norm() / ref.norm()).item()
                if not err < 1e-3:
                    bad.append(f"{t}:{st}:{ks} rel {err:.2e}")
            res.append((time_us(fn, a.iters), t, st, ks))
        _lib.check(lib.sdmoe_tune(1, 0), "tile")
        _lib.check(lib.sdmoe_tune(0, 0), "stages")
        _lib.check(lib.sdmoe_tune(9, 0), "ksplit")
        auto = res[0][0]
        best = min(res)
        line = "  ".join(f"{t}:{st}:{ks}={us:.1f}" for us, t, st, ks in res)
        if bad:
            print(f"MISMATCH {name}: {bad}", flush=True)
        print(f"{name:38s} auto {auto:8.1f} us ({flop / auto / 1e6:6.0f} TF/s) best {best[0]:8.1f} "
              f"[{best[1]}:{best[2]}:{best[3]}] | {line}", flush=True)


if __name__ == "__main__":
    main()
