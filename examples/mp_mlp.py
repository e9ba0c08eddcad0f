#!/usr/bin/env python3
"""Model-parallel MLP from the reference README (README.md:77-110), corrected math.

    python -m madnn.launch --nproc 4 examples/mp_mlp.py

Every rank holds 1/W of each Linear's input features; outputs are all-reduced,
input gradients all-gathered (the reference summed disjoint shards and tiled
gradients — exact only for W = 1).
"""
import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madnn  # noqa: E402
import madnn.nn as mnn  # noqa: E402


def main():
    madnn.init()
    madnn.seed_all(0)
    dev = madnn.device()
    model = nn.Sequential(mnn.MPInitialReshape(1024), mnn.MPInitialLinear(1024, 2048), mnn.MPTanh(),
                          mnn.MPBaseLinear(2048, 10)).to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=0.05)
    x = torch.randn(64, 32, 32, device=dev)   # identical on every rank (same seed): TP needs replicated inputs
    y = torch.randint(0, 10, (64,), device=dev)
    for it in range(20):
        loss = F.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if it % 5 == 0 and madnn.get_rank() == 0:
            print(f"iter {it} loss {loss.item():.4f}")
    madnn.shutdown()


if __name__ == "__main__":
    main()
