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
    # SDXL-family fields (diffusers UNet2DConditionModel config keys; SD-1.x defaults)
    transformer_layers_per_block: tuple = (1, 1, 1, 1)  # per down block; up blocks reversed; mid = last
    head_dim: int = 0                 # > 0: heads = C // head_dim (SDXL "attention_head_dim" = [5,10,20] heads)
    use_linear_projection: bool = False  # proj_in / proj_out as Linear [C, C] instead of 1x1 conv
    addition_embed_type: str = ""     # "text_time": SDXL micro-conditioning (pooled text + 6 time ids)
    addition_time_embed_dim: int = 256
    projection_class_embeddings_input_dim: int = 2816  # pooled text dim + 6 * addition_time_embed_dim

    @property
    def time_embed_dim(self):
        return 4 * self.block_out_channels[0]

    @property
    def pooled_dim(self):
        return self.projection_class_embeddings_input_dim - 6 * self.addition_time_embed_dim

    def heads_for(self, C):
        return C // self.head_dim if self.head_dim else self.attention_heads

    def depth_of(self, kind, i):
        """Transformer depth of down block i / the mid block / up block i (diffusers reverses the list)."""
        t = self.transformer_layers_per_block
        if kind == "down":
            return t[i]
        if kind == "mid":
            return t[-1]
        return tuple(reversed(t))[i]

    @staticmethod
    def sd14(sample_size: int = 64):
        return UNetConfig(sample_size=sample_size)

    @staticmethod
    def tiny(sample_size: int = 16):
        """Same block structure as SD-1.x at 1/5 width (head_dim 64, 2 heads) for fast parity tests."""
        return UNetConfig(block_out_channels=(64, 128, 128, 128), attention_heads=2, cross_attention_dim=128,
                          sample_size=sample_size, name="tiny")

    @staticmethod
    def sdxl(sample_size: int = 128):
        """stabilityai/stable-diffusion-xl-base-1.0 U-Net (2.57 B params; 70 GEGLU FFNs; 1024^2 -> 128^2)."""
        return UNetConfig(block_out_channels=(320, 640, 1280),
                          down_block_types=("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"),
                          up_block_types=("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"),
                          transformer_layers_per_block=(1, 2, 10), head_dim=64, cross_attention_dim=2048,
                          use_linear_projection=True, addition_embed_type="text_time",
                          addition_time_embed_dim=256, projection_class_embeddings_input_dim=2816,
                          sample_size=sample_size, name="sdxl-base")

    @staticmethod
    def tiny_xl(sample_size: int = 16):
        """SDXL block structure (no-attention first block, deep transformers, linear projections, text_time
        micro-conditioning) at small width/depth for fast parity tests: head_dim 64, 28 GEGLU FFNs."""
        return UNetConfig(block_out_channels=(64, 128, 128),
                          down_block_types=("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"),
                          up_block_types=("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"),
                          transformer_layers_per_block=(1, 2, 3), head_dim=64, cross_attention_dim=128,
                          use_linear_projection=True, addition_embed_type="text_time",
                          addition_time_embed_dim=32, projection_class_embeddings_input_dim=64 + 6 * 32,
                          sample_size=sample_size, name="tiny-xl")

    def geglu_layers(self):
        """(name, C) of every Transformer-block GEGLU in execution order == sorted-name order
        (moefication/helper.py:77; SURVEY §8 layer table)."""
        out = []
        for i, t in enumerate(self.down_block_types):
            if t.startswith("CrossAttn"):
                for j in range(self.layers_per_block):
                    for d in range(self.depth_of("down", i)):
                        out.append((f"down_blocks.{i}.attentions.{j}.transformer_blocks.{d}.ff.net.0",
                                    self.block_out_channels[i]))
        for d in range(self.depth_of("mid", 0)):
            out.append((f"mid_block.attentions.0.transformer_blocks.{d}.ff.net.0", self.block_out_channels[-1]))
        rev = list(reversed(self.block_out_channels))
        for i, t in enumerate(self.up_block_types):
            if t.startswith("CrossAttn"):
                for j in range(self.layers_per_block + 1):
                    for d in range(self.depth_of("up", i)):
                        out.append((f"up_blocks.{i}.attentions.{j}.transformer_blocks.{d}.ff.net.0", rev[i]))
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
