"""Edge cases through the C ABI on the GPU: empty inputs are a no-op returning OK, unsupported shapes fail loudly
with SdmoeError (never a silent fallback), a prompt list of one and an empty prompt run the pipeline, and the
text encoder handles a maximum-length (truncated) prompt."""
import pytest
import torch

from sdmoe import _lib, ops
from sdmoe.config import UNetConfig
from sdmoe.pipeline import StableDiffusionPipeline

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_empty_inputs_are_noops():
    C = 320
    x = torch.empty((0, C), dtype=torch.float16, device=DEV)
    w = torch.randn(640, C, device=DEV).half()
    assert ops.linear(x, w).shape == (0, 640)
    y = torch.empty((0, 2 * 4 * C), dtype=torch.float16, device=DEV)
    routing = ops.Routing(torch.arange(4 * C) % 64, 64, 12, DEV)
    assert ops.geglu_route(y, routing, ops.ACT_RELU).shape == (0, 4 * C)
    q = torch.empty((0, C), dtype=torch.float16, device=DEV)
    assert ops.attention(q, q, q, 0, 64, 64, 8).shape == (0, C)
    table = torch.randn(10, 64, device=DEV).half()
    assert ops.gather_rows(table, torch.empty(0, dtype=torch.int32, device=DEV)).shape == (0, 64)
    torch.cuda.synchronize()


def test_unsupported_shapes_raise():
    x = torch.randn(16, 100, device=DEV).half()  # K % 64 != 0
    w = torch.randn(64, 100, device=DEV).half()
    with pytest.raises(_lib.SdmoeError):
        ops.linear(x, w)
    q = torch.randn(2 * 200, 8 * 48, device=DEV).half()  # head_dim 48 has no attention kernel
    with pytest.raises(_lib.SdmoeError):
        ops.attention(q, q, q, 2, 200, 200, 8)
    qs = torch.randn(200, 64, device=DEV).half()  # > 128 tokens for the short-sequence kernel
    with pytest.raises(_lib.SdmoeError):
        ops.attention_short(qs, qs, qs, 1, 200, 1)
    with pytest.raises(_lib.SdmoeError):  # CPU tensor: no CPU path
        ops.linear(torch.randn(16, 64).half(), torch.randn(64, 64).half())


def test_pipeline_single_and_empty_prompt_with_text_encoder():
    from sdmoe.clip import attach_text_encoders
    pipe = StableDiffusionPipeline.synthetic(UNetConfig.tiny(8), seed=0, device=DEV, num_inference_steps=2)
    attach_text_encoders(pipe, seed=1)
    a = pipe("", seed=0).images
    b = pipe("word " * 200, seed=0).images  # truncated to 77 tokens
    c = pipe(["a cat"], seed=0).images
    for imgs in (a, b, c):
        assert len(imgs) == 1 and imgs[0].shape == (4, 8, 8) and bool(torch.isfinite(imgs[0]).all())
    assert not torch.equal(a[0], c[0])  # the prompt reaches the U-Net through the encoder
