"""K12P epilogue diagnosis on the GPT-2 c_fc forward (tokens x 1024 -> 4096, bias, tanh GELU):
plain epilogue vs GELU (+ pre-activation store) vs the diagnostic builds (MADNN_GEMMP_DIAG=3: no GELU
math, both stores; 4: GELU math, no pre-activation store) vs hipBLASLt + the K11 GELU pass.  Prints one
JSON line per case (us per call)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    from madnn import ops

    assert ops.load_kernels()
    M = int(os.environ.get("TOKENS", 131072))
    x = torch.randn(M, 1024, device="cuda").bfloat16()
    w = (torch.randn(4096, 1024, device="cuda") * 0.03).bfloat16()
    bias = torch.randn(4096, device="cuda").bfloat16()
    fp = torch.ops.madnn.linear_fwd_p
    out = {"diag": int(os.environ.get("MADNN_GEMMP_DIAG", "0")), "tokens": M,
           "k12p_plain_us": timed(lambda: fp(x, w, bias, 0)),
           "k12p_gelu_us": timed(lambda: fp(x, w, bias, 1))}
    lt = torch.nn.functional.linear
    out["lt_plain_us"] = timed(lambda: lt(x, w, bias))
    out["lt_gelu_k11_us"] = timed(lambda: torch.ops.madnn.gelu_fwd(lt(x, w, bias), 1))
    print(json.dumps({k: round(v, 1) if isinstance(v, float) else v for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
