#!/usr/bin/env python3
"""K13 (madnn 3x3 conv) vs MIOpen (shipped find-db) on ResNet-50's stride-1 3x3 shapes, forward,
data grad and weight grad, same random bf16 NHWC operands, interleaved rounds in one process.
    python bench/conv3x3_ab.py [--batch 1536] [--rounds 3] [--json out]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import madnn
    from madnn import ops

    madnn.init(device="cuda", backend=None)
    assert ops.load_kernels()
    rows = []
    for C, H, n in [(64, 56, 3), (128, 28, 3), (256, 14, 5), (512, 7, 2)]:
        B = a.batch
        x = torch.randn(B, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(C, C, 3, 3, device="cuda", dtype=torch.bfloat16) * (9 * C) ** -0.5).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        ref = F.conv2d(x.float()[:2], w.float(), None, 1, 1)
        got = torch.ops.madnn.conv3x3_fwd(x[:2].contiguous(memory_format=torch.channels_last), w, False)[0]
        err = float((got.float() - ref).abs().max())
        c = {"fwd_miopen": lambda: F.conv2d(x, w, None, 1, 1),
             "fwd_k13": lambda: torch.ops.madnn.conv3x3_fwd(x, w, True),
             "dgrad_miopen": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False,
                                                                          (0, 0), 1, (True, False, False)),
             "dgrad_k13": lambda: torch.ops.madnn.conv3x3_fwd(
                 dy, w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last), False),
             "wgrad_miopen": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False,
                                                                          (0, 0), 1, (False, True, False)),
             "wgrad_k13": lambda: torch.ops.madnn.conv3x3_wgrad(dy, x, True)}
        ts = {k: [] for k in c}
        for k, f in c.items():
            f()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for k, f in c.items():
                ts[k].append(timeit(f))
        fl = 2.0 * B * H * H * C * C * 9
        row = {"C": C, "H": H, "per_step": n, "max_abs_err_fwd": err}
        for k, v in ts.items():
            row[k + "_us"] = round(statistics.median(v), 1)
            row[k + "_tflops"] = round(fl / statistics.median(v) / 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del x, w, dy, wt
        torch.cuda.empty_cache()
    tot = {k: round(sum(r[k + "_us"] * r["per_step"] for r in rows) / 1e3, 2) for k in c}
    print(json.dumps({"per_step_ms": tot}), flush=True)
    if a.json:
        json.dump({"rows": rows, "per_step_ms": tot}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
