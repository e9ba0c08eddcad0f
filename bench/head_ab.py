#!/usr/bin/env python3
"""A/B the ResNet-50 global-average-pool head inside the full training step (batch 512):
``nn.AdaptiveAvgPool2d`` (ATen backward) vs ``madnn.nn.FusedGlobalAvgPool2d`` (one-pass,
layout-preserving backward).  One process, configurations interleaved round-robin."""
import json
import statistics
import time

import torch
import torch.nn.functional as F


def main():
    import madnn
    from madnn.models import resnet50
    from madnn.nn import FusedGlobalAvgPool2d
    from madnn.optim import FusedSGD

    madnn.init()
    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dmodel, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
    x, y = madnn.data.synthetic_batch("image", 512, madnn.device(), dtype=torch.bfloat16, channels_last=True,
                                      seed=1234)
    heads = {"aten": torch.nn.AdaptiveAvgPool2d((1, 1)), "fused": FusedGlobalAvgPool2d((1, 1))}

    def step():
        F.cross_entropy(dmodel(x).float(), y).backward()
        opt.step()

    for _ in range(8):
        step()
    times = {k: [] for k in heads}
    for rnd in range(6):
        for k, m in heads.items():
            model.avgpool = m
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(6):
                step()
            torch.cuda.synchronize()
            times[k].append((time.perf_counter() - t0) / 6 * 1e3)
        print(json.dumps({k: round(v[-1], 3) for k, v in times.items()}), flush=True)
    res = {k: {"median_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3)} for k, v in times.items()}
    print(json.dumps(res), flush=True)
    with open("gpurun_out/head_ab.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
