#!/usr/bin/env python3
"""Which ATen (non-madnn) elementwise ops run inside a ResNet-50 training step, with shapes and the
Python line that issued them (torch.profiler, record_shapes + with_stack):

    python bench/resnet_aten_ops.py [--batch 512] [--out gpurun_out/resnet_aten_ops.txt]
"""
import argparse
import collections
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = ("aten::copy_", "aten::add_", "aten::add", "aten::clone", "aten::contiguous", "aten::zero_", "aten::fill_",
       "aten::zeros_like", "aten::mul", "aten::to", "aten::_to_copy")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default="gpurun_out/resnet_aten_ops.txt")
    a = ap.parse_args()
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init(device="cuda", backend=None)
    assert madnn.ops.load_kernels()
    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
    dmodel, opt = madnn.distribute(model, opt, strategy="dp")
    x, y = madnn.data.synthetic_batch("image", a.batch, madnn.device(), channels_last=True, num_classes=1000)

    def step():
        loss = F.cross_entropy(dmodel(x).float(), y)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    rows = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        stack = [s for s in (ev.stack or []) if "madnn" in s or "bench" in s][:3]
        rows[(ev.name, str(ev.input_shapes)[:160], " <- ".join(stack)[:400])] += 1
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for (name, shapes, stack), n in sorted(rows.items(), key=lambda kv: -kv[1]):
            line = f"{n:3d}  {name}  {shapes}\n       {stack}\n"
            f.write(line)
            print(line, end="")


if __name__ == "__main__":
    main()
