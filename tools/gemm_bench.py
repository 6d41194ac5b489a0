"""Microbenchmark of the sdmoe GEMM / conv / attention kernels on the U-Net's real shapes (nimg = 2*B images).
usage: python tools/gemm_bench.py [--nimg 16] [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import ops  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nimg", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stages", type=int, default=0)
    ap.add_argument("--tile", type=int, default=0, help="forced GEMM tile (sdmoe_tune knob 1), 0 = auto")
    ap.add_argument("--only", default="", help="run only rows whose label contains this")
    ap.add_argument("--nqf", type=int, default=0, help="attention kernel (knob 4): 0 = auto, 1 = 32x32x16, 2/4 = 16x16x32 NQF")
    ap.add_argument("--diag", type=int, default=0, help="GEMM diagnostics (knob 6, bits): 1 = no K-loop loads, 2 = no MFMA, 4 = no epilogue")
    a = ap.parse_args()
    from sdmoe import _lib
    _lib.check(_lib.load().sdmoe_tune(0, a.stages), "tune")
    _lib.check(_lib.load().sdmoe_tune(1, a.tile), "tune")
    _lib.check(_lib.load().sdmoe_tune(4, a.nqf), "tune")
    _lib.check(_lib.load().sdmoe_tune(6, a.diag), "tune")
    print("stages", a.stages, "tile", a.tile)
    n = a.nimg
    dev = "cuda"
    rows = []
    # convs: (H, Cin, Cout, stride, upsample)
    for H, Cin, Cout, st, up in [(64, 320, 320, 1, 0), (64, 640, 320, 1, 0), (64, 960, 320, 1, 0),
                                  (32, 640, 640, 1, 0), (32, 960, 640, 1, 0), (32, 1280, 640, 1, 0),
                                  (32, 1920, 640, 1, 0), (16, 1280, 1280, 1, 0), (16, 2560, 1280, 1, 0),
                                  (8, 1280, 1280, 1, 0), (8, 2560, 1280, 1, 0), (64, 320, 320, 2, 0),
                                  (32, 640, 640, 2, 0), (16, 1280, 1280, 2, 0),
                                  (32, 640, 640, 1, 1), (16, 1280, 1280, 1, 1), (8, 1280, 1280, 1, 1),
                                  (64, 320, 8, 1, 0)]:
        x = torch.randn(n * H * H, Cin, device=dev).half()
        w = ops.conv_weight((torch.randn(Cout, 3, 3, Cin, device=dev) * (9 * Cin) ** -0.5).half())
        b = torch.zeros(Cout, device=dev).half()
        OH = 2 * H if up else (H - 1) // st + 1
        ms = timeit(lambda: ops.conv3x3(x, n, H, H, w, b, stride=st, upsample=bool(up)), a.iters)
        fl = 2.0 * n * OH * OH * Cout * 9 * Cin
        rows.append((f"conv {H}x{H} {Cin}->{Cout} s{st}{' up' if up else ''}", ms, fl / ms / 1e9))
    # linears: (M, N, K)
    for M, N, K in [(n * 4096, 960, 320), (n * 1024, 1920, 640), (n * 256, 3840, 1280), (n * 4096, 320, 320),
                    (n * 1024, 640, 640), (n * 256, 1280, 1280), (n * 4096, 2560, 320), (n * 4096, 320, 1280),
                    (n * 1024, 5120, 640), (n * 1024, 640, 2560), (n * 256, 10240, 1280), (n * 256, 1280, 5120),
                    (n * 64, 3840, 1280), (n * 77, 2560, 768)]:
        x = torch.randn(M, K, device=dev).half()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        ms = timeit(lambda: ops.linear(x, w), a.iters)
        rows.append((f"linear M={M} N={N} K={K}", ms, 2.0 * M * N * K / ms / 1e9))
    # transformer projections with the residual add epilogue (proj_out, to_out): the small-K, HBM-heavy shapes
    for M, N, K in [(n * 4096, 320, 320), (n * 1024, 640, 640), (n * 256, 1280, 1280), (n * 1024, 1920, 640),
                    (n * 256, 3840, 1280)]:
        x = torch.randn(M, K, device=dev).half()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        r = torch.randn(M, N, device=dev).half()
        ms = timeit(lambda: ops.linear(x, w, residual=r), a.iters)
        rows.append((f"linear+res M={M} N={N} K={K}", ms, 2.0 * M * N * K / ms / 1e9))
    # LayerNorm folded into the consuming GEMM (QKV / cross-attention Q at the three levels) vs LN + GEMM
    for M, N, K in [(n * 4096, 960, 320), (n * 4096, 320, 320), (n * 1024, 1920, 640), (n * 1024, 640, 640),
                    (n * 256, 3840, 1280), (n * 256, 1280, 1280)]:
        x = torch.randn(M, K, device=dev).half()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        gm, bt = torch.randn(K, device=dev).half(), torch.randn(K, device=dev).half()
        fold = ops.LNFold(w, gm, bt, 1e-5)
        ms = timeit(lambda: ops.linear_ln(x, fold), a.iters)
        rows.append((f"linear_ln M={M} N={N} K={K}", ms, 2.0 * M * N * K / ms / 1e9))
        ms = timeit(lambda: ops.linear(ops.layernorm(x, gm, bt, 1e-5), w), a.iters)
        rows.append((f"  ln+linear M={M} N={N} K={K}", ms, 2.0 * M * N * K / ms / 1e9))
    # fused routed GEGLU: projection GEMM with value*act(gate) + expert-score epilogue, then the top-k mask
    for M, C in [(n * 4096, 320), (n * 1024, 640), (n * 256, 1280)]:
        F, E = 4 * C, C // 5
        x = torch.randn(M, C, device=dev).half()
        w = (torch.randn(2 * F, C, device=dev) * C ** -0.5).half()
        b = torch.zeros(2 * F, device=dev).half()
        routing = ops.Routing(torch.arange(F) % E, E, E // 5, dev)
        w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
        score = torch.empty(M, E, device=dev).half()
        out = torch.empty(M, F, device=dev).half()
        ms = timeit(lambda: ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=routing.esize, out=out),
                    a.iters)
        rows.append((f"geglu-gemm M={M} F={F} K={C}", ms, 2.0 * M * 2 * F * C / ms / 1e9))
        gm, bt = torch.randn(C, device=dev).half(), torch.randn(C, device=dev).half()
        lnf = ops.interleave_ln_fold(ops.LNFold(w, gm, bt, 1e-5, b), routing.perm)
        ms = timeit(lambda: ops.linear_geglu(x, None, None, ops.ACT_RELU, score=score, esize=routing.esize, out=out,
                                             ln=lnf), a.iters)
        rows.append((f"geglu-gemm-ln M={M} F={F} K={C}", ms, 2.0 * M * 2 * F * C / ms / 1e9))
        score.copy_(torch.randn(M, E, device=dev).half())
        ms = timeit(lambda: ops.moe_topk_mask(out, score, routing), a.iters)
        rows.append((f"topk-mask M={M} F={F} (GB/s)", ms, (M * F * 2 * 0.8 + M * E * 2) / ms / 1e6))
        keep = ops.moe_topk_keep(score, routing, M)
        ms = timeit(lambda: ops.moe_topk_keep(score, routing, M, keep=keep), a.iters)
        rows.append((f"topk-keep M={M} E={E} (GB/s)", ms, (M * E * 2 + M * F / 8) / ms / 1e6))
        wd = (torch.randn(C, F, device=dev) * F ** -0.5).half()
        ms = timeit(lambda: ops.linear(out, wd), a.iters)
        rows.append((f"down M={M} N={C} K={F}", ms, 2.0 * M * C * F / ms / 1e9))
        ms = timeit(lambda: ops.linear_keep(out, keep, wd), a.iters)
        rows.append((f"down-keep M={M} N={C} K={F}", ms, 2.0 * M * C * F / ms / 1e9))
        y = torch.empty(M, 2 * F, device=dev).half()
        ms = timeit(lambda: ops.linear(x, w, b, out=y), a.iters)
        rows.append((f"  unfused proj M={M} N={2 * F} K={C}", ms, 2.0 * M * 2 * F * C / ms / 1e9))
        ms = timeit(lambda: ops.geglu_route(y, routing, ops.ACT_RELU, out=out), a.iters)
        rows.append((f"  unfused route M={M} F={F} (GB/s)", ms, (M * F * 6) / ms / 1e6))
    for N_, d, Nk in [(4096, 40, 4096), (4096, 40, 77), (1024, 80, 1024), (1024, 80, 77), (256, 160, 256),
                      (256, 160, 77), (4096, 64, 4096), (4096, 64, 77), (1024, 64, 1024)]:
        C = 8 * d
        q = torch.randn(n * N_, 3 * C, device=dev).half()
        kv = torch.randn(n * Nk, 2 * C, device=dev).half()
        if Nk == N_:
            f = lambda: ops.attention(q[:, :C], q[:, C:2 * C], q[:, 2 * C:], n, N_, Nk, 8)  # noqa: E731
        else:
            f = lambda: ops.attention(q[:, :C], kv[:, :C], kv[:, C:], n, N_, Nk, 8)  # noqa: E731
        ms = timeit(f, a.iters)
        rows.append((f"attn N={N_} d={d} Nk={Nk}", ms, 4.0 * n * 8 * N_ * Nk * d / ms / 1e9))
    # HBM-bound glue at the bench's shapes (GB/s = algorithmic bytes / time): GroupNorm statistics (read x once),
    # apply+SiLU (read + write), the one-call groupnorm, LayerNorm (read + write)
    for H, C in [(64, 320), (64, 640), (32, 640), (32, 1280), (16, 1280), (16, 2560), (8, 1280)]:
        x = torch.randn(n * H * H, C, device=dev).half()
        gm, bt = torch.randn(C, device=dev).half(), torch.randn(C, device=dev).half()
        byt = n * H * H * C * 2
        ms = timeit(lambda: ops.groupnorm_stats(x, n, H * H, gm, bt, 1e-5), a.iters)
        rows.append((f"gn-stats {H}x{H} C={C} (GB/s)", ms, byt / ms / 1e6))
        sc, sh = ops.groupnorm_stats(x, n, H * H, gm, bt, 1e-5)
        y = torch.empty_like(x)
        ms = timeit(lambda: ops.groupnorm_apply(x, n, H * H, sc, sh, True, out=y), a.iters)
        rows.append((f"gn-apply {H}x{H} C={C} (GB/s)", ms, 2 * byt / ms / 1e6))
        ms = timeit(lambda: ops.groupnorm(x, n, H * H, gm, bt, 1e-5, silu=True, out=y), a.iters)
        rows.append((f"groupnorm {H}x{H} C={C} (GB/s)", ms, 3 * byt / ms / 1e6))
    for M, C in [(n * 4096, 320), (n * 1024, 640), (n * 256, 1280), (n * 64, 1280)]:
        x = torch.randn(M, C, device=dev).half()
        gm, bt = torch.randn(C, device=dev).half(), torch.randn(C, device=dev).half()
        y = torch.empty_like(x)
        ms = timeit(lambda: ops.layernorm(x, gm, bt, 1e-5, out=y), a.iters)
        rows.append((f"layernorm M={M} C={C} (GB/s)", ms, 2 * M * C * 2 / ms / 1e6))
    for name, ms, tf in rows:
        if a.only and a.only not in name:
            continue
        print(f"{name:42s} {ms*1e3:9.1f} us {tf:8.1f} TF/s")


if __name__ == "__main__":
    main()
