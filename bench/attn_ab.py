#!/usr/bin/env python3
"""K8 attention variants A/B in one process (interleaved rounds, same random operands): the
``madnn_attn_tune`` keys given with --knob KEY:OFF:ON, at the GPT-2 medium, BERT-large and Llama-3 8B (B = 2, S = 4096, GQA, D = 128) shapes.
Prints one JSON line per (shape, arm) with forward and backward times and TFLOP/s (forward
4*B*H*S^2*D, halved when causal; backward 2.5x forward).

    python bench/attn_ab.py --knob 7:0:1 [--batch 32] [--rounds 5]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", required=True, help="KEY:OFF:ON of madnn_attn_tune")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    tune = ctypes.CDLL(str(ops.kernels_path())).madnn_attn_tune
    key, off, on = (int(v) for v in a.knob.split(":"))
    rows = []
    for name, S, H, HKV, D, causal, B in [("gpt2-medium", 1024, 16, 16, 64, True, a.batch),
                                          ("bert-large", 512, 16, 16, 64, False, a.batch),
                                          ("llama3-8b", 4096, 32, 8, 128, True, 2)]:
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B, S, H, D, device="cuda", generator=g).bfloat16().requires_grad_(True)
        k, v = (torch.randn(B, S, HKV, D, device="cuda", generator=g).bfloat16().requires_grad_(True) for _ in range(2))
        do = torch.randn(B, S, H, D, device="cuda", generator=g).bfloat16()
        fl = 4.0 * B * H * S * S * D / (2 if causal else 1)
        o = ops.attention(q, k, v, causal=causal)
        outs = {}
        ts = {arm: {"fwd": [], "bwd": []} for arm in ("off", "on")}
        for arm, val in (("off", off), ("on", on)):
            tune(key, val)
            oo = ops.attention(q, k, v, causal=causal)
            outs[arm] = torch.autograd.grad(oo, (q, k, v), do)
        diff = max(float((x - y).float().abs().max()) for x, y in zip(outs["off"], outs["on"]))
        for _ in range(a.rounds):
            for arm, val in (("off", off), ("on", on)):
                tune(key, val)
                ts[arm]["fwd"].append(timeit(lambda: ops.attention(q, k, v, causal=causal)))
                o = ops.attention(q, k, v, causal=causal)
                ts[arm]["bwd"].append(timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)))
        for arm in ("off", "on"):
            f, b = statistics.median(ts[arm]["fwd"]), statistics.median(ts[arm]["bwd"])
            row = {"shape": name, "B": B, "knob": key, "arm": arm, "fwd_us": round(f * 1e6, 1),
                   "fwd_tflops": round(fl / f / 1e12, 1), "bwd_us": round(b * 1e6, 1),
                   "bwd_tflops": round(2.5 * fl / b / 1e12, 1), "max_abs_diff_off_vs_on": diff}
            rows.append(row)
            print(json.dumps(row), flush=True)
    tune(key, on)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
