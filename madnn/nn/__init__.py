"""madnn layers: fused-kernel norms and tensor-parallel (model-parallel) layers."""
from .norm import FusedBatchNorm2d, FusedLayerNorm, FusedRMSNorm, swap_layernorms

__all__ = ["FusedBatchNorm2d", "FusedLayerNorm", "FusedRMSNorm", "swap_layernorms"]
