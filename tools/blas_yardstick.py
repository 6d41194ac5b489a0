"""Yardstick only (not a product path): torch.matmul (hipBLASLt/rocBLAS) fp16 throughput on the U-Net's GEMM
shapes next to sdmoe_linear / sdmoe_conv3x3 (conv shapes as their implicit-GEMM M x N x K)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
import torch  # noqa: E402

from sdmoe import ops  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


n = 16
for M, N, K, conv in [(n * 4096, 320, 2880, (64, 320)), (n * 1024, 640, 5760, (32, 640)), (n * 256, 1280, 11520, (16, 1280)),
                      (n * 64, 1280, 11520, (8, 1280)), (n * 4096, 2560, 320, None), (n * 4096, 320, 1280, None),
                      (n * 4096, 320, 320, None), (n * 1024, 640, 640, None), (n * 256, 1280, 1280, None),
                      (n * 1024, 5120, 640, None), (n * 256, 10240, 1280, None)]:
    a = torch.randn(M, K, device="cuda").half()
    b = torch.randn(K, N, device="cuda").half() * K ** -0.5
    ms = t(lambda: torch.matmul(a, b))
    line = f"M={M:6d} N={N:5d} K={K:5d}  torch.matmul {2 * M * N * K / ms / 1e9:7.1f} TF/s"
    if conv:
        H, C = conv
        x = torch.randn(n * H * H, C, device="cuda").half()
        w = ops.conv_weight((torch.randn(C, 3, 3, C, device="cuda") * (9 * C) ** -0.5).half())
        ms2 = t(lambda: ops.conv3x3(x, n, H, H, w))
        line += f" | sdmoe conv3x3 {2 * M * N * K / ms2 / 1e9:7.1f} TF/s"
    else:
        w = b.t().contiguous()
        ms2 = t(lambda: ops.linear(a, w))
        line += f" | sdmoe linear {2 * M * N * K / ms2 / 1e9:7.1f} TF/s"
    print(line, flush=True)
