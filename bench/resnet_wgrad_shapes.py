#!/usr/bin/env python3
"""Per-shape weight-gradient candidates for ResNet-50's stride-1 convolutions at the bench batch:
MIOpen (aten convolution_backward), K12 split-K over the pixels (1x1: madnn.linear_wgrad on the
[pixels, C] rows), hipBLASLt (1x1: torch.mm), K13 (3x3: madnn.conv3x3_wgrad); time and TF/s each.

    python bench/resnet_wgrad_shapes.py [--batch 2048] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (cin, cout, k, H) of ResNet-50's stride-1 convolutions, with their count per step
SHAPES = [
    (64, 64, 1, 56, 1), (256, 64, 1, 56, 2), (64, 256, 1, 56, 4), (64, 64, 3, 56, 3),
    (256, 128, 1, 56, 1), (512, 128, 1, 28, 3), (128, 512, 1, 28, 4), (128, 128, 3, 28, 3),
    (512, 256, 1, 28, 1), (1024, 256, 1, 14, 5), (256, 1024, 1, 14, 6), (256, 256, 3, 14, 5),
    (1024, 512, 1, 14, 1), (2048, 512, 1, 7, 2), (512, 2048, 1, 7, 3), (512, 512, 3, 7, 2),
]


def timeit(fn, iters=6):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import madnn
    from madnn import ops

    madnn.init(device="cuda", backend=None)
    assert ops.load_kernels()
    B = a.batch
    rows = []
    tot = {}
    for cin, cout, k, H, n in SHAPES:
        x = torch.randn(B, cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, cout, H, H, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.zeros(cout, cin, k, k, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        pad = k // 2
        fl = 2.0 * B * H * H * cin * cout * k * k
        cand = {"miopen": lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, (1, 1), (pad, pad), (1, 1), False, (0, 0), 1, (False, True, False))[1]}
        if k == 1:
            dr, xr = ops._rows(dy), ops._rows(x)
            cand["k12"] = lambda: torch.ops.madnn.linear_wgrad(dr, xr, None, False, 0)
            cand["lt"] = lambda: torch.mm(dr.t(), xr)
        else:
            cand["k13"] = lambda: torch.ops.madnn.conv3x3_wgrad(dy, x, True)
        r = {"cin": cin, "cout": cout, "k": k, "H": H, "count": n}
        for name, fn in cand.items():
            try:
                t = timeit(fn)
            except RuntimeError as e:  # noqa: PERF203
                r[name + "_err"] = str(e)[:120]
                continue
            r[name + "_us"] = round(t, 1)
            r[name + "_tflops"] = round(fl / t / 1e6, 1)
        best = min((v, kk[:-3]) for kk, v in r.items() if kk.endswith("_us"))
        r["best"] = best[1]
        for kk, v in r.items():
            if kk.endswith("_us"):
                tot[kk] = tot.get(kk, 0.0) + v * n
        tot["best_us"] = tot.get("best_us", 0.0) + best[0] * n
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, dy, w
    summ = {k: round(v / 1e3, 2) for k, v in tot.items()}
    print(json.dumps({"per_step_ms": summ}), flush=True)
    if a.json:
        json.dump({"batch": B, "rows": rows, "per_step_ms": summ}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
