#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes over K12 at GPT-2 medium's c_fc shape (65536 tokens, 1024 -> 4096):
forward (row x row operands), data gradient (col x row) and split-K weight gradient (col x col)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from madnn import ops

    assert ops.load_kernels()
    m = torch.ops.madnn
    T, K, N = (int(v) for v in os.environ.get("K12_SHAPE", "65536,1024,4096").split(","))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.03
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
    splits = int(m.wgrad_splits(T, N, K))
    for _ in range(3):
        m.linear_fwd(x, w, None, None, 0, False)
        m.linear_dgrad(dy, w, None, False)
        m.linear_wgrad(dy, x, None, False, splits)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
