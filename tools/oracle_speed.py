"""Time the CPU oracle U-Net (oracle/unet_ref.py) on this host: one SD-1.4 CFG evaluation at 64x64 latents (U-Net
batch 2), NCHW vs channels_last convs, plus the fp16 CPU linear of the reference hook vs fp32-then-round."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

if len(sys.argv) == 1:
    for v in ("0", "1"):
        subprocess.run([sys.executable, __file__, "run"], env=dict(os.environ, SDMOE_ORACLE_NHWC=v), check=True)
    sys.exit(0)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from sdmoe.config import UNetConfig  # noqa: E402
from sdmoe.weights import make_state_dict  # noqa: E402
from oracle import unet_ref  # noqa: E402

cfg = UNetConfig.sd14(64)
ref = unet_ref.UNetRef(make_state_dict(cfg, 0), cfg)
x = torch.randn(2, 4, 64, 64)
ctx = torch.randn(2, 77, 768) * 0.5
with torch.no_grad():
    ref(x, 500.0, ctx)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        ref(x, 500.0, ctx)
        ts.append(time.perf_counter() - t0)
print(f"NHWC={unet_ref.NHWC} threads={torch.get_num_threads()} eval s: {[round(t, 2) for t in ts]}", flush=True)
if unet_ref.NHWC:
    for M, K, N in [(8192, 320, 2560), (2048, 640, 5120), (512, 1280, 10240)]:
        a = torch.randn(M, K).half()
        w = (torch.randn(N, K) * K ** -0.5).half()
        b = (torch.randn(N) * 0.1).half()
        F.linear(a, w, b)
        t0 = time.perf_counter()
        y16 = F.linear(a, w, b)
        t1 = time.perf_counter()
        y32 = F.linear(a.float(), w.float(), b.float()).half()
        t2 = time.perf_counter()
        print(f"linear {M}x{K}x{N}: fp16 {t1 - t0:.3f} s, fp32+round {t2 - t1:.3f} s, mismatches "
              f"{int((y16 != y32).sum())}", flush=True)
