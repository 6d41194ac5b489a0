"""Shapes the U-Net's FeedForward down projections issue (test helper, no GPU).

A Transformer-block FFN at level i of a U-Net with latent side S runs its down projection (`ff.net.2`, reference
`LoRACompatibleLinear` hooked by remove_wanda_neurons_fast.py:107-112; fused keep-masked form in sdmoe/unet.py
FeedForward.run) as an M x K x N product with M = U-Net batch x (S / 2^i)^2 tokens, K = 4C, N = C. The U-Net batch
is 2 x prompts per call (CFG)."""
from sdmoe.config import UNetConfig

PROMPTS_PER_CALL = (1, 2, 8, 16)  # the reference's one-prompt call (base_receiver.py:73) .. 16 prompts per GPU


def _level(name, nblk):
    parts = name.split(".")
    if parts[0] == "mid_block":
        return nblk - 1
    i = int(parts[1])
    return i if parts[0] == "down_blocks" else nblk - 1 - i


def down_projection_shapes(model="sd14", prompts=PROMPTS_PER_CALL):
    """Sorted distinct (M, K, N) of the FFN down projections of `model` ('sd14' 512^2 or 'sdxl' 1024^2)."""
    cfg = UNetConfig.sd14() if model == "sd14" else UNetConfig.sdxl()
    nblk = len(cfg.block_out_channels)
    out = set()
    for name, C in cfg.geglu_layers():
        side = cfg.sample_size >> _level(name, nblk)
        for b in prompts:
            out.add((2 * b * side * side, 4 * C, C))
    return sorted(out)
