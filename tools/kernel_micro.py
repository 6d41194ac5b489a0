"""Run one kernel shape repeatedly (for rocprofv3 --pmc passes).
usage: python tools/kernel_micro.py attn|conv|linear [--iters 20]"""
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
    a = ap.parse_args()
    n, dev = a.nimg, "cuda"
    if a.what == "attn":
        C = 320
        q = torch.randn(n * 4096, 3 * C, device=dev).half()
        f = lambda: ops.attention(q[:, :C], q[:, C:2 * C], q[:, 2 * C:], n, 4096, 4096, 8)  # noqa: E731
    elif a.what == "conv":
        x = torch.randn(n * 4096, 320, device=dev).half()
        w = ops.conv_weight((torch.randn(320, 3, 3, 320, device=dev) * 0.02).half())
        f = lambda: ops.conv3x3(x, n, 64, 64, w)  # noqa: E731
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
