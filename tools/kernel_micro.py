"""Run one kernel shape repeatedly (for rocprofv3 --pmc passes).
usage: python tools/kernel_micro.py attn|conv|linear|geglu [--iters 20] [--diag BITS] [--d 40] [--tune k=v,...]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nimg", type=int, default=16)
    ap.add_argument("--diag", type=int, default=0, help="GEMM diagnostics bits (sdmoe_tune knob 6)")
    ap.add_argument("--d", type=int, default=40, help="attn: head dim (8 heads, N = 4096)")
    ap.add_argument("--tune", default="", help="extra sdmoe_tune settings 'knob=value,...'")
    a = ap.parse_args()
    from sdmoe import _lib
    _lib.check(_lib.load().sdmoe_tune(6, a.diag), "tune")
    for k, v in _lib.parse_tune(a.tune):
        _lib.check(_lib.load().sdmoe_tune(k, v), "tune")
    n, dev = a.nimg, "cuda"
    if a.what == "attn":
        C = 8 * a.d
        q = torch.randn(n * 4096, 3 * C, device=dev).half()
        f = lambda: ops.attention(q[:, :C], q[:, C:2 * C], q[:, 2 * C:], n, 4096, 4096, 8)  # noqa: E731
    elif a.what == "conv":
        x = torch.randn(n * 4096, 320, device=dev).half()
        w = ops.conv_weight((torch.randn(320, 3, 3, 320, device=dev) * 0.02).half())
        f = lambda: ops.conv3x3(x, n, 64, 64, w)  # noqa: E731
    elif a.what == "geglu":  # the fused routed GEGLU projection at 64x64 (M = n*4096, F = 1280, K = 320)
        C, F, E = 320, 1280, 64
        x = torch.randn(n * 4096, C, device=dev).half()
        w = (torch.randn(2 * F, C, device=dev) * C ** -0.5).half()
        routing = ops.Routing(torch.arange(F) % E, E, E // 5, dev)
        w_il, b_il = ops.interleave_geglu(w, torch.zeros(2 * F, device=dev).half(), routing.perm)
        score = torch.empty(n * 4096, E, device=dev).half()
        out = torch.empty(n * 4096, F, device=dev).half()
        f = lambda: ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=routing.esize,  # noqa: E731
                                     out=out)
    else:
        x = torch.randn(n * 4096, 320, device=dev).half()
        w = (torch.randn(2560, 320, device=dev) * 0.05).half()
        f = lambda: ops.linear(x, w)  # noqa: E731
    for _ in range(a.iters):
        f()
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
