"""In-process A/B of a ResNet-50 module-level switch (one model, one optimizer; the flag is
flipped between interleaved timing windows on the same box, so both arms see the same memory
state and clocks):

    python bench/resnet_flag_ab.py --flag madnn.models.resnet:_DUAL_BN --batch 1536 --windows 6 --steps 5
    python bench/resnet_flag_ab.py --flag bn_tune:multi --on 1=1,3=1 --off 1=3,3=0   # several native keys
"""
import argparse
import importlib
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
    ap.add_argument("--flag", default="madnn.models.resnet:_DUAL_BN", help="module:attribute")
    ap.add_argument("--on", default="true", help="value of the 'on' arm (true/false/int/string)")
    ap.add_argument("--off", default="false", help="value of the 'off' arm")
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    def val(v):
        return {"true": True, "false": False}.get(v.lower(), int(v) if v.lstrip("-").isdigit() else v)

    arm_val = {True: val(a.on), False: val(a.off)}
    mod_name, attr = a.flag.split(":")
    if mod_name == "bn_tune" or mod_name.startswith("native."):
        # a native tunable: bn_tune:KEY (madnn_bn_tune) or native.FUNC:KEY, e.g. native.madnn_conv1x1_tune:0
        import ctypes

        madnn_mod = importlib.import_module("madnn.ops")
        madnn_mod.load_kernels()
        fname = "madnn_bn_tune" if mod_name == "bn_tune" else mod_name[len("native."):]
        tune = getattr(ctypes.CDLL(str(madnn_mod.kernels_path())), fname)

        class _Native:
            def __setattr__(self, k, v):
                if k == "multi":   # --flag bn_tune:multi --on 3=1,1=2 --off 3=0,1=3: several keys per arm
                    for kv in str(v).split(","):
                        kk, vv = kv.split("=")
                        tune(int(kk), int(vv))
                else:
                    tune(int(k), int(v))

        mod = _Native()
    else:
        mod = importlib.import_module(mod_name)
    madnn.init()
    torch.manual_seed(0)
    m = resnet50()
    o = FusedSGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dm, o = madnn.distribute(m, o, strategy="dp")
    x, y = madnn.data.synthetic_batch("image", a.batch, madnn.device(), dtype=torch.bfloat16, channels_last=True)

    def window(on, n):
        setattr(mod, attr, arm_val[on])
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
        for on in ((True, False) if w % 2 == 0 else (False, True)):
            res[on].append(window(on, a.steps))
    out = {"flag": a.flag, "on": a.on, "off": a.off, "batch": a.batch, "windows": a.windows, "steps": a.steps,
           "on_ms": statistics.median(res[True]), "off_ms": statistics.median(res[False]),
           "on_all": res[True], "off_all": res[False]}
    out["on_img_s"] = a.batch / out["on_ms"] * 1e3
    out["off_img_s"] = a.batch / out["off_ms"] * 1e3
    out["speedup"] = out["off_ms"] / out["on_ms"]
    line = json.dumps(out)
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
