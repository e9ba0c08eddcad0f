#!/usr/bin/env python3
"""In-process A/B of one ResNet-50 DP1 model with a madnn.ops routing flag toggled between
interleaved timing windows (same box, same tensors):

    python bench/flag_ab.py --flag _K13 --windows 8 --steps 4 [--batch 1536]
    python bench/flag_ab.py --flag _K13_WGRAD --on auto --off miopen
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flag", default="_K13")
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--on", default="True", help="flag value of the 'on' arm (True/False or a string)")
    ap.add_argument("--off", default="False")
    a = ap.parse_args()
    import madnn
    from madnn import ops
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init()
    torch.manual_seed(0)
    m = resnet50()
    o = FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dm, o = madnn.distribute(m, o, strategy="dp")
    x, y = madnn.data.synthetic_batch("image", a.batch, madnn.device(), dtype=torch.bfloat16, channels_last=True)
    base = getattr(ops, a.flag)
    val = {True: {"True": True, "False": False}.get(a.on, a.on), False: {"True": True, "False": False}.get(a.off, a.off)}

    def window(on, n):
        setattr(ops, a.flag, val[on])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            F.cross_entropy(dm(x).float(), y).backward()
            o.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for on in (True, False):
        window(on, 2)
    res = {True: [], False: []}
    for w in range(a.windows):
        on = w % 2 == 0
        res[on].append(window(on, a.steps))
    setattr(ops, a.flag, base)
    out = {"flag": a.flag, "on": a.on, "off": a.off, "batch": a.batch, "on_ms": res[True], "off_ms": res[False],
           "on_median": statistics.median(res[True]), "off_median": statistics.median(res[False]),
           "on_img_s": round(a.batch / statistics.median(res[True]) * 1e3, 1),
           "off_img_s": round(a.batch / statistics.median(res[False]) * 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
