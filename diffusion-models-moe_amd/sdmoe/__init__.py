"""sdmoe — MI355X-native MoE-fied Stable-Diffusion denoising step."""
from .config import RunConfig, UNetConfig  # noqa: F401

__version__ = "0.1.0"
