#!/usr/bin/env python3
"""Throughput for every BASELINE.json config through ``madnn.distribute``.

    python bench/throughput.py --model gpt2-medium --batch 16 --seq 1024 [--strategy auto|dp|pp|dp_pp]
    python -m madnn.launch --nproc 8 bench/throughput.py --model llama3-8b --strategy dp_pp --pp 2

Models: resnet50, gpt2-medium, bert-large, llama3-8b, llama3-1b, mlp; synthetic
data, random init; bf16 compute, fp32 masters; prints one JSON line (rank 0)
with samples/s, tokens/s and the plan madnn chose.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(name, meta: bool):
    from madnn.models import MLP, resnet50
    from madnn.models.bert import BertForPreTraining, bert_config
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.models.llama import Llama, llama_config

    ctx = torch.device("meta") if meta else torch.device("cpu")
    with ctx:
        if name == "resnet50":
            return resnet50()
        if name.startswith("gpt2"):
            return GPT2(gpt2_config(name))
        if name.startswith("bert"):
            return BertForPreTraining(bert_config(name))
        if name.startswith("llama3"):
            return Llama(llama_config(name))
        if name == "mlp":
            return MLP(1024, 4096, 10)
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--batch", type=int, default=8, help="GLOBAL batch")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--strategy", default="auto")
    ap.add_argument("--pp", type=int, default=None)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--checkpointing", default="auto")
    ap.add_argument("--optimizer", default="adam", choices=["adam", "sgd"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--meta-init", action="store_true", help="build on the meta device (8B models)")
    ap.add_argument("--metrics", default=None, help="after timing, run 3 metered steps (JSONL to this path)")
    a = ap.parse_args()

    import madnn
    from madnn.optim import FusedAdam, FusedSGD

    madnn.init()
    world, rank = madnn.get_world_size(), madnn.get_rank()
    dev = madnn.device()
    torch.manual_seed(0)
    meta = a.meta_init or a.model == "llama3-8b"
    model = build(a.model, meta)
    opt = (FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01) if a.optimizer == "adam"
           else FusedSGD(model.parameters(), lr=0.1, momentum=0.9))
    image = a.model == "resnet50" or a.model == "mlp"
    if a.model == "resnet50":
        example = torch.zeros(1, 3, 224, 224)
    elif a.model == "mlp":
        example = torch.zeros(1, 1024)
    else:
        example = torch.zeros(1, a.seq, dtype=torch.long)
    loss_fn = getattr(model, "loss_fn", None) or (lambda out, y: F.cross_entropy(out.float(), y))
    if meta and a.strategy in ("dp", "auto") and world == 1:
        from madnn.parallel.pp import materialize_

        materialize_(model, dev, getattr(model, "init_weights", None), opt)
    eng, opt = madnn.distribute(model, opt, strategy=a.strategy, pp_stages=a.pp, microbatches=a.microbatches,
                                checkpointing=a.checkpointing, example_input=example, loss_fn=loss_fn,
                                global_batch=a.batch)
    plan = getattr(eng, "plan", None)
    dp = plan.dp if plan is not None else world
    per_replica = a.batch // dp
    g = torch.Generator(device=dev).manual_seed(7 + (eng.groups.dp_idx if hasattr(eng, "groups") else rank))
    if a.model == "resnet50":
        x = torch.randn(per_replica, 3, 224, 224, device=dev, generator=g).bfloat16()
        y = torch.randint(0, 1000, (per_replica,), device=dev, generator=g)
    elif a.model == "mlp":
        x = torch.randn(per_replica, 1024, device=dev, generator=g)
        y = torch.randint(0, 10, (per_replica,), device=dev, generator=g)
    else:
        vocab = model.config.vocab_size
        x = torch.randint(0, vocab, (per_replica, a.seq), device=dev, generator=g)
        y = x

    def step():
        loss = eng.train_step(x, y)
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    madnn.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    madnn.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    metered = None
    if a.metrics:
        from madnn.utils.metrics import StepMeter

        meter = StepMeter(eng, samples_per_step=a.batch, path=a.metrics)
        for _ in range(3):
            meter.start()
            loss = step()
            metered = meter.stop(loss)
        meter.close()
    sps = a.batch * a.steps / dt
    out = {"model": a.model, "n_gpus": world, "global_batch": a.batch, "seq_len": None if image else a.seq,
           "samples_per_s": round(sps, 2), "tokens_per_s": None if image else round(sps * a.seq, 1),
           "ms_per_step": round(dt / a.steps * 1e3, 2), "plan": plan.describe() if plan is not None else "dp",
           "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 2), "dtype": "bf16",
           "data": "synthetic", "loss": float(loss) if loss is not None else None}
    if metered is not None:
        out["metrics"] = {k: round(v, 3) if isinstance(v, float) else v for k, v in metered.items()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    madnn.shutdown()


if __name__ == "__main__":
    main()
