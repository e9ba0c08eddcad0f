"""Planner accuracy at N=1: the modelled step time of a model (HIP-event layer costs, two-point
fixed + per-sample fit, one-chain calibration, optimizer pass) against the measured step of the
same model, batch and optimizer run through ``madnn.distribute``.

    python bench/plan_accuracy.py --cases resnet50:512,gpt2-medium:16 --json-out gpurun_out/plan_acc.json
"""
import argparse
import json
import statistics
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_case(model_name: str, batch: int, steps: int = 6, warmup: int = 3) -> dict:
    import madnn
    from madnn.config import Config
    from madnn.nn.swap import use_madnn_kernels
    from madnn.optim import FusedAdam, FusedSGD
    from madnn.planner import plan_model

    dev = madnn.device()
    torch.manual_seed(0)
    if model_name == "resnet50":
        from madnn.models import resnet50

        model = resnet50()
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        ex = torch.zeros(1, 3, 224, 224)
    else:
        from madnn.models.gpt2 import GPT2, gpt2_config

        model = GPT2(gpt2_config(model_name))
        opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
        ex = torch.zeros(1, 1024, dtype=torch.long)
    use_madnn_kernels(model)
    t0 = time.time()
    plan = plan_model(model, Config.from_env(strategy="dp", checkpointing="none"), 1, example_input=ex,
                      global_batch=batch, optimizer=opt)
    plan_s = time.time() - t0
    eng, opt = madnn.distribute(model, opt, strategy="dp", checkpointing="none")
    if model_name == "resnet50":
        x, y = madnn.data.synthetic_batch("image", batch, dev, dtype=torch.bfloat16, channels_last=True)

        def step():
            F.cross_entropy(eng(x).float(), y).backward()
            opt.step()
    else:
        ids = torch.randint(0, model.config.vocab_size, (batch, 1024), device=dev)

        def step():
            eng.train_step(ids, ids)
            opt.step()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    per = []
    for _ in range(steps):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        per.append(time.perf_counter() - t0)
    meas = statistics.median(per)  # one-off host stalls (allocator, first-use tuning) do not count
    eng.remove_hooks()
    del eng, opt, model
    torch.cuda.empty_cache()
    out = {"model": model_name, "batch": batch, "est_ms": plan.est_step_s * 1e3, "measured_ms": meas * 1e3,
           "ratio": plan.est_step_s / meas, "plan_s": round(plan_s, 1), "calibration": plan.calibration,
           "measured_costs": plan.measured,
           "step_ms": [round(t * 1e3, 2) for t in per]}
    print(json.dumps(out), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="resnet50:512,resnet50:2048,gpt2-medium:16,gpt2-medium:64")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import madnn

    madnn.init()
    res = []
    for c in a.cases.split(","):
        name, b = c.split(":")
        res.append(run_case(name, int(b)))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
