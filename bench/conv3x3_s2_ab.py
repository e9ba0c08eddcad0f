#!/usr/bin/env python3
"""K13 stride-2 forward (madnn/ops/csrc/conv3.hip, SD = 2) against the library forward PyTorch
dispatches (MIOpen / CK) at ResNet-50's three stride-2 3x3 shapes, interleaved rounds in one
process, same operands.  K13 also writes the BatchNorm statistics partial rows (the library path
needs a separate statistics pass for them; timed without it).

    python bench/conv3x3_s2_ab.py [--batch 2048] [--rounds 5] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

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
    ap.add_argument("--batch", type=int, nargs="+", default=[2048, 512])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    rows = []
    for B in a.batch:
        for Ci, H in ((128, 56), (256, 28), (512, 14)):
            x = torch.randn(B, Ci, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            w = (torch.randn(Ci, Ci, 3, 3, device="cuda") * (9 * Ci) ** -0.5).bfloat16()
            w = w.contiguous(memory_format=torch.channels_last)
            k13 = lambda: torch.ops.madnn.conv3x3_fwd_s2(x, w, True)  # noqa: E731
            lib = lambda: F.conv2d(x, w, None, 2, 1)  # noqa: E731
            diff = float((k13()[0].float() - lib().float()).abs().max())
            ts = {"k13": [], "lib": []}
            for _ in range(a.rounds):
                ts["k13"].append(timeit(k13))
                ts["lib"].append(timeit(lib))
            fl = 2.0 * B * (H // 2) ** 2 * Ci * Ci * 9
            row = {"batch": B, "Ci": Ci, "H": H, "k13_us": round(statistics.median(ts["k13"]) * 1e6, 1),
                   "lib_us": round(statistics.median(ts["lib"]) * 1e6, 1), "max_abs_diff": diff}
            row["k13_tflops"] = round(fl / (row["k13_us"] * 1e-6) / 1e12, 1)
            row["lib_tflops"] = round(fl / (row["lib_us"] * 1e-6) / 1e12, 1)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del x, w
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
