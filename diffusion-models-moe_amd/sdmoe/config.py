"""Model / run configuration. Field names follow the reference and diffusers' UNet2DConditionModel config.

The reference's experiment YAML keys (experiments/moefy_config.yaml, remove_skills.yaml) map onto RunConfig:
`expert_size`, `topk_experts`, `timesteps`, `n_layers`, `seed`.
"""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass(frozen=True)
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280, 1280)
    down_block_types: tuple = ("CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D",
                               "DownBlock2D")
    up_block_types: tuple = ("UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D")
    layers_per_block: int = 2
    attention_heads: int = 8          # SD-1.x "attention_head_dim": 8 is the number of heads
    cross_attention_dim: int = 768
    norm_num_groups: int = 32
    norm_eps: float = 1e-5            # ResnetBlock2D GroupNorm / conv_norm_out
    transformer_norm_eps: float = 1e-6  # Transformer2DModel.norm (GroupNorm)
    layer_norm_eps: float = 1e-5      # BasicTransformerBlock LayerNorms
    flip_sin_to_cos: bool = True
    freq_shift: float = 0.0
    sample_size: int = 64             # latent H = W (512^2 images)
    name: str = "sd-1.4"

    @property
    def time_embed_dim(self):
        return 4 * self.block_out_channels[0]

    def heads_for(self, C):
        return self.attention_heads

    @staticmethod
    def sd14(sample_size: int = 64):
        return UNetConfig(sample_size=sample_size)

    @staticmethod
    def tiny(sample_size: int = 16):
        """Same block structure as SD-1.x at 1/5 width (head_dim 64, 2 heads) for fast parity tests."""
        return UNetConfig(block_out_channels=(64, 128, 128, 128), attention_heads=2, cross_attention_dim=128,
                          sample_size=sample_size, name="tiny")

    def geglu_layers(self):
        """(name, C) of every Transformer-block GEGLU in execution order == sorted-name order
        (moefication/helper.py:77; SURVEY §8 layer table)."""
        out = []
        for i, t in enumerate(self.down_block_types):
            if t.startswith("CrossAttn"):
                for j in range(self.layers_per_block):
                    out.append((f"down_blocks.{i}.attentions.{j}.transformer_blocks.0.ff.net.0",
                                self.block_out_channels[i]))
        out.append(("mid_block.attentions.0.transformer_blocks.0.ff.net.0", self.block_out_channels[-1]))
        rev = list(reversed(self.block_out_channels))
        for i, t in enumerate(self.up_block_types):
            if t.startswith("CrossAttn"):
                for j in range(self.layers_per_block + 1):
                    out.append((f"up_blocks.{i}.attentions.{j}.transformer_blocks.0.ff.net.0", rev[i]))
        return out


@dataclass
class RunConfig:
    """One denoising job: the reference's YAML keys plus the pipeline knobs of StableDiffusionPipeline."""
    expert_size: int = 20
    topk_experts: float = 0.2
    timesteps: int = 50               # DDIM calls per image (the reference's PNDM run makes 51)
    n_layers: int = 16
    seed: int = 0
    num_inference_steps: int = 50
    guidance_scale: float = 7.5
    relufied: bool = True
    extra: dict = field(default_factory=dict)
