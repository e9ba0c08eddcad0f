"""Model zoo (random init from configs; no network on the GPU box)."""
from .mlp import MLP, CifarConvNet, count_params
from .resnet import ResNet, resnet18, resnet50, resnet101

__all__ = ["MLP", "CifarConvNet", "count_params", "ResNet", "resnet18", "resnet50", "resnet101"]
