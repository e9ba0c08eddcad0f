#!/usr/bin/env python3
"""Where does the first step's time go?  (bench.py's warmup_s: 2.2 s in round 2, 76.6 s in round 3.)

Runs the ResNet-50 (or GPT-2 medium) bench step on one GPU and times each of the first
``--steps`` steps on its own (device-synchronised), counting the per-shape kernel timings madnn
does on first use (``ops._time_wgrad``: weight-gradient K12/K13 vs library, GELU-Linear forward)
and the size of MIOpen's user kernel cache before and after (runtime kernel compiles land there).
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _dir_bytes(p: Path) -> int:
    if not p.exists():
        return 0
    return sum(f.stat().st_size for f in p.rglob("*") if f.is_file())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "gpt2-medium"])
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import torch.nn.functional as F

    import madnn
    import madnn.ops as ops

    cache = Path(os.environ.get("MIOPEN_CUSTOM_CACHE_DIR", str(Path.home() / ".cache" / "miopen")))
    cache0 = _dir_bytes(cache)
    timings = {"n": 0, "s": 0.0, "keys": []}
    orig = ops._time_wgrad

    def counted(fn, iters: int = 3):
        t = time.perf_counter()
        r = orig(fn, iters)
        timings["n"] += 1
        timings["s"] += time.perf_counter() - t
        return r

    ops._time_wgrad = counted
    madnn.init()
    torch.manual_seed(0)
    dev = madnn.device()
    if args.model == "resnet50":
        from madnn.models import resnet50
        from madnn.optim import FusedSGD

        model = resnet50()
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        dmodel, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
        x, y = madnn.data.synthetic_batch("image", args.batch, dev, dtype=torch.bfloat16, channels_last=True, seed=1)

        def step():
            loss = F.cross_entropy(dmodel(x).float(), y)
            loss.backward()
            opt.step()
    else:
        from madnn.models.gpt2 import GPT2, gpt2_config
        from madnn.optim import FusedAdam

        cfg = gpt2_config("gpt2-medium")
        model = GPT2(cfg)
        opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
        engine, opt = madnn.distribute(model, opt, strategy="dp", checkpointing="none",
                                       example_input=torch.zeros(1, 1024, dtype=torch.long))
        ids = torch.randint(0, cfg.vocab_size, (args.batch, 1024)).to(dev)

        def step():
            engine.train_step(ids, ids)
            opt.step()

    per = []
    for i in range(args.steps):
        n0, s0 = timings["n"], timings["s"]
        torch.cuda.synchronize()
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        per.append({"step": i, "s": round(time.perf_counter() - t, 3), "timed_choices": timings["n"] - n0,
                    "timing_s": round(timings["s"] - s0, 3)})
        print(json.dumps(per[-1]), flush=True)
    rec = {"model": args.model, "batch": args.batch, "steps": per,
           "wgrad_choices": {str(k): v for k, v in ops._WGRAD_CHOICE.items()},
           "gelu_fwd_choices": {str(k): v for k, v in ops._GELU_FWD_CHOICE.items()},
           "miopen_cache_bytes_before": cache0, "miopen_cache_bytes_after": _dir_bytes(cache),
           "miopen_cache_dir": str(cache)}
    print(json.dumps(rec), flush=True)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
