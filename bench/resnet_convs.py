#!/usr/bin/env python3
"""Every distinct ResNet-50 convolution shape on MIOpen (the shipped find-db's solvers), per pass,
against the MI355X roofline: time, TFLOP/s, GB/s of compulsory traffic, and the bound
max(FLOP / 2.5 PF, bytes / 5 TB/s).  python bench/resnet_convs.py [--batch 1536] [--json out]"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import madnn
    from madnn.models import resnet50

    madnn.init(device="cuda", backend=None)  # seeds the shipped MIOpen find-db
    model = resnet50()
    shapes = collections.Counter()
    hw = {}
    x = torch.zeros(1, 3, 224, 224)

    def hook(m, inp, out):
        key = (m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0], m.padding[0], inp[0].shape[2])
        shapes[key] += 1
        hw[key] = (out[0] if isinstance(out, tuple) else out).shape[2]

    hs = [m.register_forward_hook(hook) for m in model.modules() if isinstance(m, torch.nn.Conv2d)]
    with torch.no_grad():
        model.float()(x)
    for h in hs:
        h.remove()
    B = a.batch
    rows = []
    tot = collections.Counter()
    for (cin, cout, k, s, p, H), n in sorted(shapes.items()):
        Ho = hw[(cin, cout, k, s, p, H)]
        xi = torch.randn(B, cin, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, k, k, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(xi, w, None, s, p)
        dy = torch.randn_like(y)
        fl = 2.0 * B * Ho * Ho * cout * cin * k * k
        bx, by, bw = xi.numel() * 2, y.numel() * 2, w.numel() * 2
        passes = {
            "fwd": (lambda: F.conv2d(xi, w, None, s, p), bx + by + bw),
            "dgrad": (lambda: torch.ops.aten.convolution_backward(dy, xi, w, None, (s, s), (p, p), (1, 1), False,
                                                                   (0, 0), 1, (True, False, False)), by + bx + bw),
            "wgrad": (lambda: torch.ops.aten.convolution_backward(dy, xi, w, None, (s, s), (p, p), (1, 1), False,
                                                                   (0, 0), 1, (False, True, False)), by + bx + bw),
        }
        for name, (fn, byts) in passes.items():
            if name == "dgrad" and cin == 3:
                continue
            t = timeit(fn)
            bound = max(fl / 2.5e15, byts / 5.0e12)
            r = {"cin": cin, "cout": cout, "k": k, "stride": s, "H": H, "count": n, "pass": name,
                 "us": round(t * 1e6, 1), "tflops": round(fl / t / 1e12, 1), "gbps": round(byts / t / 1e9),
                 "bound_us": round(bound * 1e6, 1), "eff": round(bound / t, 3)}
            rows.append(r)
            tot[name] += t * n
            tot[name + "_bound"] += bound * n
            print(json.dumps(r), flush=True)
        del xi, w, y, dy
    summ = {k: round(v * 1e3, 2) for k, v in tot.items()}
    print(json.dumps({"per_step_ms": summ}), flush=True)
    if a.json:
        json.dump({"rows": rows, "per_step_ms": summ}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
