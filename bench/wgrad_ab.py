#!/usr/bin/env python3
"""Linear weight gradients, GPT-2 medium at 64 x 1024 tokens: hipBLASLt (torch.mm into the bucket
slot, what ops.linear ran in round 2) vs K12 split-K (madnn.linear_wgrad, auto and fixed splits);
same random bf16 operands, interleaved rounds in one process.

    python bench/wgrad_ab.py [--tokens 65536] [--rounds 5] [--json out.json]
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
    rows = []
    for name, N, K in [("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
                       ("lm_head", 50304, 1024)]:
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        auto = int(m.wgrad_splits(M, N, K))
        import ctypes

        tune = ctypes.CDLL(str(ops.kernels_path())).madnn_gemm_tune

        def m32(f):
            def run():
                tune(0, 0)
                r = f()
                tune(0, 1)
                return r
            return run

        cands = {"lt": lambda: torch.mm(dy.t(), x, out=out), "k12_auto": lambda: m.linear_wgrad(dy, x, out, False, 0),
                 "k12_auto_m32": m32(lambda: m.linear_wgrad(dy, x, out, False, 0))}
        for sp in sorted({1, 2, 4, 8, 16} - {auto}):
            cands[f"k12_s{sp}"] = (lambda sp=sp: m.linear_wgrad(dy, x, out, False, sp))
        ref = torch.mm(dy.t(), x)
        err = float((m.linear_wgrad(dy, x, None, False, 0).float() - ref.float()).abs().max())
        ts = {k: [] for k in cands}
        for f in cands.values():
            timeit(f, 2)
        for _ in range(a.rounds):
            for k, f in cands.items():
                ts[k].append(timeit(f))
        row = {"shape": name, "M": M, "N": N, "K": K, "auto_splits": auto, "max_abs_diff_vs_lt": err}
        for k, v in ts.items():
            med = statistics.median(v)
            row[k + "_us"] = round(med * 1e6, 1)
            row[k + "_tflops"] = round(fl / med / 1e12, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del dy, x, out, ref
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
