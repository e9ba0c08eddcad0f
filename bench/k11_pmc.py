#!/usr/bin/env python3
"""Drive K11 (ops.bias_grad) at the GPT-2 medium c_fc shape [16384, 4096] bf16, plain and with the
fused GELU backward, for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_k11_pmc.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from madnn import ops  # noqa: E402


def main():
    assert ops.load_kernels()
    dy = torch.randn(16384, 4096, device="cuda").bfloat16()
    pre = torch.randn(16384, 4096, device="cuda").bfloat16()
    for _ in range(4):
        ops.bias_grad(dy, None, torch.bfloat16)
        ops.bias_grad(dy, pre, torch.bfloat16)
    torch.cuda.synchronize()
    print("k11 pmc driver done")


if __name__ == "__main__":
    main()
