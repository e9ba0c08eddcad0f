"""A few ResNet-50 DP training steps on one GPU (the bench.py model/optimizer, no timing or JSON):
the short target program for rocprofv3 PMC passes (scripts/gpu_bn_pmc.sh).

    python bench/resnet_steps.py --batch 512 --steps 2
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init()
    torch.manual_seed(0)
    m = resnet50()
    o = FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dm, o = madnn.distribute(m, o, strategy="dp")
    x, y = madnn.data.synthetic_batch("image", a.batch, madnn.device(), dtype=torch.bfloat16, channels_last=True)
    for _ in range(a.steps):
        F.cross_entropy(dm(x).float(), y).backward()
        o.step()
    torch.cuda.synchronize()
    print("ok")
    madnn.shutdown()


if __name__ == "__main__":
    main()
