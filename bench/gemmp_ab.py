#!/usr/bin/env python3
"""K12P (persistent, fused epilogues) vs hipBLASLt and one-tile K12 on GPT-2 medium's Linear
shapes; same random bf16 operands, interleaved rounds in one process (cdna_hip_programming.md
§5.4 rules 24/25).  Rows:

* ``fwd``: y = x W^T (+ bias) for qkv / proj / fc1 / fc2;
* ``dgrad``: dx = dy W for the same layers;
* ``fc1_gelu``: c_fc forward + GELU -- hipBLASLt (bias) + the K11 GELU pass vs K12P's GELU epilogue;
* ``fc2_dgrad_dgelu``: c_proj's data gradient + c_fc's GELU backward and bias gradient --
  hipBLASLt + the K11 dGELU/column-sum pass vs K12P's dGELU epilogue.

    python bench/gemmp_ab.py [--tokens 131072] [--rounds 5] [--json out.json]
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
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    m = torch.ops.madnn
    M = a.tokens
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*shape, scale=1.0):
        return ((torch.rand(*shape, device="cuda", generator=g) * 2 - 1) * scale).bfloat16()

    rows = []

    def run(name, fl, cands):
        ts = {k: [] for k in cands}
        for f in cands.values():
            timeit(f, 2)
        for _ in range(a.rounds):
            for k, f in cands.items():
                ts[k].append(timeit(f))
        row = {"case": name, "M": M}
        for k, v in ts.items():
            med = statistics.median(v)
            row[k + "_us"] = round(med * 1e6, 1)
            if fl:
                row[k + "_tflops"] = round(fl / med / 1e12, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)

    for name, N, K in [("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096)]:
        x, w, b, dy = rnd(M, K), rnd(N, K, scale=K ** -0.5), rnd(N).float(), rnd(M, N)
        fl = 2.0 * M * N * K
        run(f"{name}_fwd", fl, {
            "lt": lambda: torch.nn.functional.linear(x, w, b.bfloat16()),
            "k12": lambda: m.linear_fwd(x, w, b, None, 0, False),
            "k12p": lambda: m.linear_fwd_p(x, w, b, 0),
        })
        run(f"{name}_dgrad", fl, {
            "lt": lambda: torch.mm(dy, w),
            "k12": lambda: m.linear_dgrad(dy, w, None, False),
            "k12p": lambda: m.linear_dgrad_p(dy, w, None, torch.float32),
        })
        if name == "fc1":
            run("fc1_gelu", fl, {
                "lt+k11": lambda: m.gelu_fwd(torch.nn.functional.linear(x, w, b.bfloat16())),
                "k12p": lambda: m.linear_fwd_p(x, w, b, 1),
            })
        if name == "fc2":
            pre = rnd(M, K, scale=2.0)
            run("fc2_dgrad_dgelu", fl, {
                "lt+k11": lambda: m.bias_grad(torch.mm(dy, w), pre, torch.float32),
                "k12p": lambda: m.linear_dgrad_p(dy, w, pre, torch.float32),
            })
        del x, w, b, dy
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
