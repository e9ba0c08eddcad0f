"""hipBLASLt's ranked candidates on the GPT-2 medium b128 Linear shapes: for each forward (bias) and
data-gradient (``w_kn``) GEMM, the heuristic's first choice (what PyTorch's ``F.linear`` / ``@`` run)
against every other candidate it offers (``lt_linear(..., algo=i)``).  One JSON line per shape:
us per call of each candidate, the best index and its gain over index 0."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=10):
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
    T = int(os.environ.get("TOKENS", 131072))
    lt = torch.ops.madnn.lt_linear
    cnt = torch.ops.madnn.lt_algo_count
    shapes = [  # name, M, K (reduction), N, bias, w_kn
        ("qkv_fwd", T, 1024, 3072, True, False), ("proj_fwd", T, 1024, 1024, True, False),
        ("fc2_fwd", T, 4096, 1024, True, False), ("fc1_fwd", T, 1024, 4096, True, False),
        ("lm_head_fwd", T, 1024, 50304, False, False),
        ("qkv_dgrad", T, 3072, 1024, False, True), ("proj_dgrad", T, 1024, 1024, False, True),
        ("fc1_dgrad", T, 4096, 1024, False, True), ("lm_head_dgrad", T, 50304, 1024, False, True),
    ]
    only = os.environ.get("ONLY", "")
    for name, M, K, N, has_bias, w_kn in shapes:
        if only and only not in name:
            continue
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(K, N, device="cuda") if w_kn else torch.randn(N, K, device="cuda")).mul_(0.03).bfloat16()
        bias = torch.randn(N, device="cuda").bfloat16() if has_bias else None
        n = int(cnt(x, w, bias, w_kn))
        ref = lt(x, w, bias, None, False, False, w_kn, 0)[0].float()
        rec = {"shape": name, "M": M, "K": K, "N": N, "candidates": n, "us": []}
        if w_kn:
            rec["torch_us"] = round(timed(lambda: x @ w), 1)
        else:
            rec["torch_us"] = round(timed(lambda: torch.nn.functional.linear(x, w, bias)), 1)
        for i in range(n):
            y = lt(x, w, bias, None, False, False, w_kn, i)[0].float()
            rel = float((y - ref).norm() / ref.norm())
            t = timed(lambda: lt(x, w, bias, None, False, False, w_kn, i))
            rec["us"].append(round(t, 1) if rel < 1e-2 else None)
        ok = [(t, i) for i, t in enumerate(rec["us"]) if t is not None]
        best = min(ok)
        rec["best"] = best[1]
        rec["gain_vs_0"] = round(rec["us"][0] / best[0] - 1, 4) if rec["us"][0] else None
        rec["tflops_best"] = round(2.0 * M * N * K / best[0] / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del x, w, bias, ref, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
