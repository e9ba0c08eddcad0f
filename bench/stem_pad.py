#!/usr/bin/env python3
"""A/B: the ResNet stem (7x7/2 conv, 3 input channels, NHWC bf16) with the input channels
zero-padded to 4 or 8, forward + weight grad, MIOpen immediate mode (shipped find-db) and
with find (cudnn.benchmark).  Zero channels with zero weights leave the output unchanged."""
import json
import statistics
import sys

import torch
import torch.nn.functional as F


def t_of(fn, iters=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    import madnn

    madnn.init()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    res = {}
    for bench_mode in (False, True):
        torch.backends.cudnn.benchmark = bench_mode
        for c in (3, 4, 8):
            x = torch.randn(N, c, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            w = torch.randn(64, c, 7, 7, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            y = F.conv2d(x, w, stride=2, padding=3)
            dy = torch.randn_like(y)
            cb = torch.ops.aten.convolution_backward
            f = t_of(lambda: F.conv2d(x, w, stride=2, padding=3))
            wg = t_of(lambda: cb(dy, x, w, None, (2, 2), (3, 3), (1, 1), False, (0, 0), 1, (False, True, False)))
            xp = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            pad = t_of(lambda: F.pad(xp, (0, 0, 0, 0, 0, c - 3)).contiguous(memory_format=torch.channels_last)) \
                if c > 3 else 0.0
            res[f"C{c}_{'find' if bench_mode else 'db'}"] = {"fwd": round(f, 3), "wgrad": round(wg, 3), "pad": round(pad, 3)}
            print(json.dumps({f"C{c}_{'find' if bench_mode else 'db'}": res[f"C{c}_{'find' if bench_mode else 'db'}"]}),
                  flush=True)


if __name__ == "__main__":
    main()
