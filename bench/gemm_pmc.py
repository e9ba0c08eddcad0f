#!/usr/bin/env python3
"""Same-operand K12 vs hipBLASLt dispatches for rocprofv3 PMC passes: the forward GEMM at one
shape, ``GEMM_ITERS`` of each (random uniform [-1, 1) bf16 operands, cdna_hip_programming.md
§5.4 rule 25).  ``GEMM_SHAPE=M,N,K`` (default 8192,8192,8192); ``GEMM_K12=0`` runs hipBLASLt only;
``GEMM_OP=wgrad``: the weight gradient dW[N, K] = dY[M, N]^T X[M, K] on K12 (8 waves), K12W (4 waves)
and hipBLASLt instead.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES ... -- python3 bench/gemm_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from madnn import ops

    assert ops.load_kernels()
    m = torch.ops.madnn
    M, N, K = (int(v) for v in os.environ.get("GEMM_SHAPE", "8192,8192,8192").split(","))
    iters = int(os.environ.get("GEMM_ITERS", "5"))
    g = torch.Generator(device="cuda").manual_seed(0)
    if os.environ.get("GEMM_OP", "fwd") == "wgrad":
        dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).bfloat16()
        x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        for _ in range(iters):
            torch.mm(dy.t(), x)
            m.linear_wgrad(dy, x, None, False, 0)
            m.linear_wgrad4(dy, x, None, False, 0)
            if M % 128 == 0:
                m.linear_wgrad4h(dy, x, None, False, 0)
        torch.cuda.synchronize()
        return
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).bfloat16()
    for _ in range(iters):
        torch.mm(x, w.t())
        if os.environ.get("GEMM_K12", "1") == "1":
            m.linear_fwd(x, w, None, None, 0, False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
