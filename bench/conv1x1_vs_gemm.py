#!/usr/bin/env python3
"""A/B: ResNet-50 1x1 convolutions (NHWC bf16) on MIOpen vs as plain GEMMs on hipBLASLt.

A stride-1 1x1 conv over an NHWC tensor is exactly x[M, Cin] @ W[Cout, Cin]^T with
M = N*H*W; forward, data-grad and weight-grad are three GEMMs.  Times fwd+bwd per shape
(median of interleaved rounds, one process — cdna_hip_programming.md §5.4 rule 24).
"""
import statistics
import sys

import torch
import torch.nn.functional as F


def t_of(fn, iters=10):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
              (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]
    dev = "cuda"
    tot_c = tot_g = 0.0
    for hw, cin, cout in shapes:
        x = torch.randn(N, cin, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)
        dy = torch.randn(N, cout, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)

        def conv():
            y = F.conv2d(x, w)
            torch.autograd.grad(y, (x, w), dy)

        x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, cin).requires_grad_(True)
        w2 = w.detach().reshape(cout, cin).requires_grad_(True)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)

        def gemm():
            y = x2 @ w2.t()
            torch.autograd.grad(y, (x2, w2), dy2)

        tc, tg = [], []
        for _ in range(3):
            tc.append(t_of(conv))
            tg.append(t_of(gemm))
        c, g = min(tc), min(tg)
        tot_c += c
        tot_g += g
        print(f"N={N} {hw}x{hw} {cin:5d}->{cout:5d}: miopen {c:7.3f} ms  gemm {g:7.3f} ms  ratio {c / g:5.2f}")
    print(f"total miopen {tot_c:.3f} ms  gemm {tot_g:.3f} ms")


if __name__ == "__main__":
    main()
