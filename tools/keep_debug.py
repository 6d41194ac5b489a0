"""Debug aid: compare sdmoe_moe_topk_mask's zero pattern with sdmoe_moe_topk_keep's keep bits on one case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdmoe import ops  # noqa: E402

DEV = "cuda:0"
M, C, E, k, nrem = 4096, 320, 64, 12, 5
g = torch.Generator().manual_seed(3 * M + C)
F = 4 * C
x = torch.randn(M, C, generator=g).half().to(DEV)
w = (torch.randn(2 * F, C, generator=g) * C ** -0.5).half().to(DEV)
b = (torch.randn(2 * F, generator=g) * 0.3).half().to(DEV)
routing = ops.Routing(torch.randperm(F, generator=g) % E, E, k, DEV)
rm_ids = torch.randperm(E, generator=g)[:nrem].tolist()
removed = ops.removed_bits(rm_ids, E, DEV)
w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
score = torch.empty((M, E), dtype=torch.float16, device=DEV)
P = ops.linear_geglu(x, w_il, b_il, ops.ACT_RELU, score=score, esize=routing.esize)
Pm = P.clone()
sel = torch.zeros((M, 2), dtype=torch.int32, device=DEV)
ops.moe_topk_mask(Pm, score, routing, removed=removed, sel_out=sel)
keep = ops.moe_topk_keep(score, routing, M, removed=removed)
torch.cuda.synchronize()
kb = keep.cpu().numpy().view(np.uint64)
bits = ((kb[:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(bool)
kmask = np.ascontiguousarray(bits.transpose(1, 0, 2).reshape(M, F))
Pn, Pmn = P.float().cpu().numpy(), Pm.float().cpu().numpy()
ref = np.where(kmask, Pn, 0)
bad = np.argwhere(ref != Pmn)
print("mismatches", len(bad), "of", M * F, "removed", rm_ids)
s = sel.cpu().numpy().view(np.uint32)
for m, n in bad[:10]:
    e = n // 20
    sb = (s[m, e >> 5] >> (e & 31)) & 1
    print(f"m={m} n={n} e={e} P={Pn[m, n]} Pm={Pmn[m, n]} keep={kmask[m, n]} sel={sb} removed={e in rm_ids}")
# expected keep from sel & ~removed
exp = np.zeros((M, F), bool)
for e in range(E):
    on = ((s[:, e >> 5] >> (e & 31)) & 1).astype(bool) & (e not in rm_ids)
    exp[:, 20 * e:20 * e + 20] = on[:, None]
print("keep bits vs sel&~removed mismatches:", int((exp != kmask).sum()))
print("mask-kernel zeros vs sel&~removed mismatches:", int(((np.where(exp, Pn, 0)) != Pmn).sum()))
