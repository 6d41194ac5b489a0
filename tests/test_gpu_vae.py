"""VAE decoder (diffusers AutoencoderKL.decode, restated in oracle/vae_ref.py — parity-unpinned
against diffusers itself): HIP decoder vs the fp32 oracle on the same fp16-rounded weights, plus
its two helper kernels vs torch fp32."""
import pytest
import torch

from oracle import vae_ref
from sdmoe import ops
from sdmoe.vae import AutoencoderKLDecoder, VAEConfig, make_vae_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def rel_l2(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("R,N", [(4096, 4096), (333, 64), (100, 1000), (7, 8192)])
def test_softmax_rows(R, N):
    g = torch.Generator().manual_seed(R + N)
    x = (torch.randn(R, N, generator=g) * 3).half().to(DEV)
    y = ops.softmax_rows(x)
    ref = torch.softmax(x.float(), dim=-1)
    assert (y.float() - ref).abs().max().item() <= 2e-3 * ref.abs().max().item() + 1e-6
    assert torch.allclose(y.float().sum(-1), torch.ones(R, device=DEV), atol=5e-3)


@pytest.mark.parametrize("R,C", [(4096, 512), (100, 70), (64, 64)])
def test_transpose(R, C):
    x = torch.randn(R, C + 8).half().to(DEV)[:, :C]
    assert torch.equal(ops.transpose(x), x.t().contiguous())


@pytest.mark.parametrize("cfg,h,B", [(VAEConfig.tiny(), 8, 2), (VAEConfig.sd14(), 8, 1)], ids=["tiny", "sd14"])
def test_decoder_vs_oracle(cfg, h, B):
    sd = make_vae_state_dict(cfg, 0)
    dec = AutoencoderKLDecoder(sd, cfg, DEV)
    lat = torch.randn(B, 4, h, h, generator=torch.Generator().manual_seed(3))
    got = dec.decode(lat).cpu()
    ref = vae_ref.decode({k: v.half().float() for k, v in sd.items()}, cfg, lat)
    assert got.shape == ref.shape == (B, 3, h * 2 ** (len(cfg.block_out_channels) - 1),
                                      h * 2 ** (len(cfg.block_out_channels) - 1))
    assert torch.isfinite(got).all()
    assert rel_l2(got, ref) <= 2e-2, rel_l2(got, ref)


def test_pipeline_decodes_with_vae():
    """output_type 'pt' runs the decoder on the denoised latents: images == postprocess(decode(latents))."""
    from sdmoe.config import UNetConfig
    from sdmoe.pipeline import StableDiffusionPipeline
    from sdmoe.vae import postprocess
    cfg = UNetConfig.tiny(8)
    pipe = StableDiffusionPipeline.synthetic(cfg, seed=0, device=DEV, num_inference_steps=2)
    lat = pipe(["a", "b"]).images
    pipe.vae = AutoencoderKLDecoder(make_vae_state_dict(VAEConfig.tiny(), 1), VAEConfig.tiny(), DEV)
    img = pipe(["a", "b"], output_type="pt").images
    assert img[0].shape == (3, 16, 16) and 0 <= float(img[0].min()) and float(img[0].max()) <= 1
    exp = postprocess(pipe.vae.decode(torch.stack(lat)))
    assert torch.equal(torch.stack(img), exp)
