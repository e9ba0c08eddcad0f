#!/usr/bin/env python3
"""Minimal driver for profiling the K8 attention kernels under rocprofv3 (one shape, few iterations)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from madnn import ops

    B, S, H, HKV, D = (int(v) for v in (os.environ.get("ATTN_SHAPE", "16,1024,16,16,64").split(",")))
    causal = os.environ.get("ATTN_CAUSAL", "1") == "1"
    dev = torch.device("cuda")
    q = torch.randn(B, S, H, D, device=dev).bfloat16().requires_grad_(True)
    k = torch.randn(B, S, HKV, D, device=dev).bfloat16().requires_grad_(True)
    v = torch.randn(B, S, HKV, D, device=dev).bfloat16().requires_grad_(True)
    for _ in range(int(os.environ.get("ATTN_ITERS", "3"))):
        o = ops.attention(q, k, v, causal=causal)
        o.backward(torch.randn_like(o))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
