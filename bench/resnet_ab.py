"""In-process A/B of ResNet-50 DP1 variants that differ in how the model was distributed
(two engines built side by side, interleaved timing windows on the same box):

    python bench/resnet_ab.py --a bucket_mb=64 --b bucket_mb=0 --windows 6 --steps 6
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


def parse_kw(s):
    out = {}
    for part in filter(None, s.split(",")):
        k, v = part.split("=")
        try:
            v = float(v) if "." in v else int(v)
        except ValueError:
            pass
        out[k] = v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="bucket_mb=64")
    ap.add_argument("--b", default="bucket_mb=0")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init()
    arms = {}
    for name, kw in (("a", parse_kw(a.a)), ("b", parse_kw(a.b))):
        torch.manual_seed(0)
        m = resnet50()
        o = FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        dm, o = madnn.distribute(m, o, strategy="dp", **kw)
        arms[name] = (dm, o, len(dm.space.buckets))
    x, y = madnn.data.synthetic_batch("image", a.batch, madnn.device(), dtype=torch.bfloat16, channels_last=True)

    def window(arm, n):
        dm, o, _ = arms[arm]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            F.cross_entropy(dm(x).float(), y).backward()
            o.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for arm in arms:
        window(arm, 3)
    res = {"a": [], "b": []}
    for w in range(a.windows):
        arm = "a" if w % 2 == 0 else "b"
        res[arm].append(window(arm, a.steps))
    out = {"a": a.a, "b": a.b, "buckets": {k: v[2] for k, v in arms.items()}, "a_ms": res["a"], "b_ms": res["b"],
           "a_median": statistics.median(res["a"]), "b_median": statistics.median(res["b"])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
