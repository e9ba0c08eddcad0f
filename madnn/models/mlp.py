"""Small models from the reference and BASELINE config 1.

* :class:`MLP` — "2-layer MLP auto-DP on CPU/gloo world_size=2" (BASELINE
  config 1), also the README model-parallel example shape 1024 -> 2048 -> 10
  (reference README.md:97-101) when built with ``MLP(1024, 2048, 10, act="tanh")``.
* :class:`CifarConvNet` — the reference example's network
  (cifar_example/sgd-torchad_nn-cifar.lua:88-118): conv 3->64 5x5, ReLU,
  maxpool 3/3, conv 64->64 5x5, ReLU, maxpool 3/3, view 64, dropout 0.5,
  linear 64->100, ReLU, linear 100->10 (114,838 parameters; the reference's
  LogSoftMax + CrossEntropyCriterion double-softmax, SURVEY A-17, is not
  replicated — the model returns logits).
"""
from __future__ import annotations

import torch
from torch import nn


class MLP(nn.Module):
    def __init__(self, d_in: int = 32, d_hidden: int = 64, d_out: int = 10, act: str = "relu"):
        super().__init__()
        self.fc1 = nn.Linear(d_in, d_hidden)
        self.act = nn.Tanh() if act == "tanh" else nn.ReLU()
        self.fc2 = nn.Linear(d_hidden, d_out)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x.flatten(1))))

    def tensor_parallel_pairs(self):
        """fc1 column-parallel -> elementwise act -> fc2 row-parallel (one all-reduce)."""
        return [(("fc1",), "fc2")]


class CifarConvNet(nn.Module):
    def __init__(self, num_classes: int = 10, dropout: float = 0.5):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 5), nn.ReLU(inplace=True), nn.MaxPool2d(3, 3),
            nn.Conv2d(64, 64, 5), nn.ReLU(inplace=True), nn.MaxPool2d(3, 3),
        )
        self.classifier = nn.Sequential(
            nn.Flatten(), nn.Dropout(dropout), nn.Linear(64, 100), nn.ReLU(inplace=True), nn.Linear(100, num_classes)
        )

    def forward(self, x):
        return self.classifier(self.features(x))


def count_params(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())
