"""madnn layers: fused-kernel norms / convolution and tensor-parallel (model-parallel) layers."""
from .conv import FusedConv2d
from .norm import (FusedBatchNorm2d, FusedGlobalAvgPool2d, FusedLayerNorm, FusedMaxPool2d, FusedRMSNorm,
                   swap_layernorms)
from .swap import use_madnn_kernels

__all__ = ["FusedBatchNorm2d", "FusedConv2d", "FusedGlobalAvgPool2d", "FusedLayerNorm", "FusedMaxPool2d", "FusedRMSNorm", "swap_layernorms",
           "use_madnn_kernels"]
from ..parallel.tp import (ColumnParallelLinear, MPBaseLinear, MPBaseReshape, MPInitialLinear, MPInitialReshape,
                           MPTanh, RowParallelLinear, set_debug_shapes)

__all__ += ["ColumnParallelLinear", "RowParallelLinear", "MPInitialLinear", "MPBaseLinear", "MPTanh",
            "MPInitialReshape", "MPBaseReshape", "set_debug_shapes"]
