#!/usr/bin/env python3
"""Time one ResNet-50 3x3 convolution shape (fwd, dgrad, wgrad) on MIOpen with whatever db /
find settings the environment selects.  python bench/miopen_search_probe.py --cin 64 --hw 56 --batch 1536"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--hw", type=int, default=56)
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--benchmark", type=int, default=1)
    a = ap.parse_args()
    import madnn

    madnn.init(device="cuda", backend=None)
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    B, C, H = a.batch, a.cin, a.hw
    x = torch.randn(B, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device="cuda", dtype=torch.bfloat16) * 0.05).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t0 = time.time()
    fns = {"fwd": lambda: F.conv2d(x, w, None, 1, 1),
           "dgrad": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                                                                 (True, False, False)),
           "wgrad": lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                                                                 (False, True, False))}
    out = {"cin": C, "hw": H, "batch": B, "enforce": os.environ.get("MIOPEN_FIND_ENFORCE")}
    for k, f in fns.items():
        t1 = time.time()
        f()
        torch.cuda.synchronize()
        out[k + "_first_s"] = round(time.time() - t1, 1)
        print(json.dumps({k: "found", "s": out[k + "_first_s"]}), flush=True)
        out[k + "_us"] = round(timeit(f), 1)
    out["total_s"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
