#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes over K13 (fwd, data grad, weight grad) at one ResNet-50 shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from madnn import ops

    assert ops.load_kernels()
    C, H, B = (int(v) for v in os.environ.get("K13_SHAPE", "64,56,1536").split(","))
    x = torch.randn(B, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(memory_format=torch.channels_last)
    for _ in range(2):
        y, _ = torch.ops.madnn.conv3x3_fwd(x, w, True)
        torch.ops.madnn.conv3x3_wgrad(y, x, True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
