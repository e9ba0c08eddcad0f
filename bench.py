#!/usr/bin/env python3
"""madnn headline benchmark (BASELINE.json metric):

  "samples/sec whole-node ResNet-50 DP + GPT-2 PP at 1/2/4/8 MI355X; scaling eff"

Default (the driver's contract): ResNet-50, automatic data parallelism
(``madnn.distribute``), bf16 compute with fp32 master weights and fp32 BatchNorm,
channels_last, FusedSGD (momentum 0.9, wd 5e-5) on the hand-written gfx950 kernel,
bucketed RCCL all-reduce overlapped with backward; synthetic ImageNet-shaped
data and random init (no network on the box); fixed per-GPU batch => weak
scaling.  ``--model gpt2-medium`` runs the GPT-2 medium pipeline-parallel
config instead.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Times exactly K steps between a barrier + device synchronize on both sides,
takes the MAX over ranks, and rank 0 prints ONE JSON line.
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

METRIC = "samples/sec whole-node ResNet-50 DP + GPT-2 PP at 1/2/4/8 MI355X; scaling eff"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "gpt2-medium"])
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (resnet50) / global batch (gpt2)")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--device", default="cuda", help="cuda (MI355X) or cpu (gloo; for testing the harness)")
    ap.add_argument("--backend", default=None,
                    help="process-group backend override (default: nccl=RCCL on cuda, gloo on cpu); gloo on cuda "
                         "lets tests run several ranks on one GPU, which RCCL refuses")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--miopen-benchmark", type=int, default=0,
                    help="torch.backends.cudnn.benchmark (MIOpen find).  Both modes read the shipped MI355X "
                         "find-db (madnn/tuning/miopen, seeded by madnn.init), so 0 already runs the tuned solvers")
    return ap.parse_args()


def _sync_all():
    if not torch.cuda.is_available():
        if dist.is_initialized():
            dist.barrier()
        return
    torch.cuda.synchronize()
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
        torch.cuda.synchronize()


def bench_resnet(args, world, rank):
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    # 512 images per GPU: sized for 288 GB HBM3E (a few tens of GB of activations), and large enough
    # that the per-step fixed costs (kernel boundaries, MIOpen workspace memsets) are amortised
    per_gpu = args.batch or 512
    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    kw = {}
    if args.bucket_mb:
        kw["bucket_mb"] = args.bucket_mb
    dmodel, opt = madnn.distribute(model, opt, strategy="dp", overlap=not args.no_overlap,
                                   channels_last=bool(args.channels_last), **kw)
    dev = madnn.device()
    x, y = madnn.data.synthetic_batch("image", per_gpu, dev, dtype=torch.bfloat16 if dev.type == "cuda" else
                                      torch.float32, channels_last=bool(args.channels_last), seed=1234 + rank,
                                      shape=(3, args.image_size, args.image_size))

    def step():
        out = dmodel(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    tw = time.perf_counter()
    for _ in range(args.warmup):
        step()
    _sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    _sync_all()
    dt = time.perf_counter() - t0
    return dt, per_gpu * world, {"warmup_s": round(t0 - tw, 1), "model": "resnet50", "global_batch": per_gpu * world, "per_gpu_batch": per_gpu,
                                 "seq_len": None, "image": [3, args.image_size, args.image_size], "parallelism": f"dp{world}",
                                 "optimizer": "FusedSGD(momentum=0.9)", "loss": float(loss.detach())}


def bench_gpt2(args, world, rank):
    import madnn
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    cfg = gpt2_config("gpt2-medium")
    gbatch = args.batch or 8 * max(world, 1)
    torch.manual_seed(0)
    model = GPT2(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    stages = min(4, world)
    strategy = "pp" if world > 1 else "dp"
    engine, opt = madnn.distribute(model, opt, strategy=strategy, pp_stages=stages if world > 1 else None,
                                   microbatches=args.microbatches)
    dev = madnn.device()
    ids, _ = madnn.data.synthetic_batch("tokens", gbatch, dev, seq_len=args.seq_len, vocab=cfg.vocab_size)

    def step():
        loss = engine.train_step(ids, ids)
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    _sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    _sync_all()
    dt = time.perf_counter() - t0
    par = f"pp{stages}" if strategy == "pp" and world == stages else (f"dp{world // stages}xpp{stages}"
                                                                     if strategy == "pp" else f"dp{world}")
    return dt, gbatch, {"model": "gpt2-medium", "global_batch": gbatch, "seq_len": args.seq_len,
                        "parallelism": par, "optimizer": "FusedAdam", "loss": float(loss.detach()) if loss is not None else None}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    import madnn

    torch.backends.cudnn.benchmark = bool(args.miopen_benchmark)
    madnn.init(device=args.device, backend=args.backend)
    rank = madnn.get_rank()
    if args.model == "resnet50":
        dt, samples_per_step, config = bench_resnet(args, world, rank)
    else:
        dt, samples_per_step, config = bench_gpt2(args, world, rank)
    t = torch.tensor([dt], dtype=torch.float64, device=madnn.device())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1000.0
    value = samples_per_step * args.steps / dt
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak" if args.model == "resnet50" else "strong",
        "vs_baseline": None,
        "dtype": "bf16" if madnn.device().type == "cuda" else "fp32",
        "data": "synthetic (random ImageNet-shaped images, random-init weights)" if args.model == "resnet50"
        else "synthetic (random tokens, random-init weights)",
        "config": config,
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    madnn.shutdown()


if __name__ == "__main__":
    main()
