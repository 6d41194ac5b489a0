import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
import torch
import torch.nn.functional as F
from sdmoe import ops
torch.manual_seed(0)
for d in [32, 40, 64, 80, 160]:
    for Nq, Nk in [(16, 64), (128, 128), (128, 77), (256, 1024)]:
        nimg, heads = 1, 2
        C = heads * d
        q = torch.randn(nimg * Nq, C, device="cuda").half()
        k = torch.randn(nimg * Nk, C, device="cuda").half()
        v = torch.randn(nimg * Nk, C, device="cuda").half()
        out = ops.attention(q, k, v, nimg, Nq, Nk, heads).float()
        qf = q.float().reshape(nimg, Nq, heads, d).transpose(1, 2)
        kf = k.float().reshape(nimg, Nk, heads, d).transpose(1, 2)
        vf = v.float().reshape(nimg, Nk, heads, d).transpose(1, 2)
        ref = F.scaled_dot_product_attention(qf, kf, vf).transpose(1, 2).reshape(nimg * Nq, C)
        nan = torch.isnan(out)
        err = (out - ref).abs().nan_to_num(99).max().item()
        print(d, Nq, Nk, "nan", int(nan.sum()), "err", round(err, 4),
              "nan rows", nan.any(1).nonzero().flatten()[:8].tolist(), "nan cols", nan.any(0).nonzero().flatten()[:12].tolist())
