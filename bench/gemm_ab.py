#!/usr/bin/env python3
"""K12 (madnn MFMA GEMM) vs hipBLASLt (torch.mm) on the GPT-2 medium Linear shapes, same random
bf16 operands, interleaved rounds in one process (cdna_hip_programming.md §5.4 rules 24/25).

    python bench/gemm_ab.py [--tokens 65536] [--rounds 5] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    m = torch.ops.madnn
    M = a.tokens
    # (name, N, K): forward y[M,N] = x[M,K] w[N,K]^T ; dgrad dx[M,K] = dy[M,N] w[N,K]
    shapes = [("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
              ("lm_head", 50304, 1024), ("sq8192", 8192, 8192)]
    rows = []
    for name, N, K in shapes:
        MM = 8192 if name == "sq8192" else M
        x = (torch.rand(MM, K, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        dy = (torch.rand(MM, N, device="cuda") * 2 - 1).bfloat16()
        fl = 2.0 * MM * N * K
        import ctypes

        tune = ctypes.CDLL(str(ops.kernels_path())).madnn_gemm_tune

        def shape(v, f):
            def run():
                tune(0, v)
                return f()
            return run

        cands = {
            "fwd_lt": lambda: torch.mm(x, w.t()),
            "fwd_k12": shape(1, lambda: m.linear_fwd(x, w, None, None, 0, False)),
            "fwd_k12m32": shape(0, lambda: m.linear_fwd(x, w, None, None, 0, False)),
            "dgrad_lt": lambda: torch.mm(dy, w),
            "dgrad_k12": shape(1, lambda: m.linear_dgrad(dy, w, None, False)),
            "dgrad_k12m32": shape(0, lambda: m.linear_dgrad(dy, w, None, False)),
        }
        ref = torch.mm(x, w.t())
        tune(0, 1)
        err = float((m.linear_fwd(x, w, None, None, 0, False)[0].float() - ref.float()).abs().max())
        refd = torch.mm(dy, w)
        errd = float((m.linear_dgrad(dy, w, None, False).float() - refd.float()).abs().max())
        ts = {k: [] for k in cands}
        for k, f in cands.items():
            timeit(f, 2)
        for _ in range(a.rounds):
            for k, f in cands.items():
                ts[k].append(timeit(f))
        row = {"shape": name, "M": MM, "N": N, "K": K, "max_abs_diff_fwd": err, "max_abs_diff_dgrad": errd}
        for k, v in ts.items():
            med = statistics.median(v)
            row[k + "_us"] = round(med * 1e6, 1)
            row[k + "_tflops"] = round(fl / med / 1e12, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del x, w, dy, ref, refd
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
