#!/usr/bin/env python3
"""Llama-3 8B, automatic hybrid DP x PP on one 8x MI355X node (BASELINE config 4).

    python -m madnn.launch --nproc 8 examples/llama_hybrid.py --seq 4096 --batch 64

The model is built on the META device (no 32 GB host copy per rank); the planner
prices DP / PP / DPxPP with and without activation checkpointing against 288 GB
per GPU and picks the fastest feasible layout; each rank materialises only its
own stage on its GPU.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madnn  # noqa: E402
from madnn.models.llama import Llama, llama_config  # noqa: E402
from madnn.optim import FusedAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--strategy", default="auto")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    madnn.init()
    cfg = llama_config(a.model)
    with torch.device("meta"):
        model = Llama(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.1)
    eng, opt = madnn.distribute(model, opt, strategy=a.strategy, global_batch=a.batch,
                                example_input=torch.zeros(1, a.seq, dtype=torch.long))
    plan = eng.plan
    if madnn.get_rank() == 0:
        print(plan.describe())
        print(plan.table())
    per_replica = a.batch // plan.dp
    ids = madnn.data.synthetic_batch("tokens", per_replica, madnn.device(), seq_len=a.seq, vocab=cfg.vocab_size)[0]
    for step in range(a.steps):
        loss = eng.train_step(ids, ids)
        opt.step()
        if loss is not None and madnn.get_rank() == madnn.get_world_size() - 1:
            print(f"step {step} loss {float(loss):.4f}")
    madnn.shutdown()


if __name__ == "__main__":
    main()
