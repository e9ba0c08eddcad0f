#!/usr/bin/env python3
"""GPT-2 medium, automatic pipeline parallelism over xGMI (BASELINE config 3).

    python -m madnn.launch --nproc 4 examples/gpt2_pipeline.py --stages 4 --microbatches 8

The planner traces the model's spine (embedding, 24 blocks, tied LM head), costs
every layer on the meta device and cuts 4 balanced stages; the engine runs the
C++ 1F1B program with batched send/recv, sums the tied embedding gradient between
the first and last stage, and FusedAdam (HIP) steps each stage.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madnn  # noqa: E402
from madnn.models.gpt2 import GPT2, gpt2_config  # noqa: E402
from madnn.optim import FusedAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--stages", type=int, default=None)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--schedule", default="1f1b", choices=["1f1b", "gpipe"])
    a = ap.parse_args()
    madnn.init()
    torch.manual_seed(0)
    cfg = gpt2_config(a.model)
    model = GPT2(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    eng, opt = madnn.distribute(model, opt, strategy="pp", pp_stages=a.stages or madnn.get_world_size(),
                                microbatches=a.microbatches, schedule=a.schedule,
                                example_input=torch.zeros(1, a.seq, dtype=torch.long))
    if madnn.get_rank() == 0:
        print(eng.plan.describe())
        print(eng.plan.table())
    ids = madnn.data.synthetic_batch("tokens", a.batch, madnn.device(), seq_len=a.seq, vocab=cfg.vocab_size)[0]
    for step in range(a.steps):
        t0 = time.time()
        loss = eng.train_step(ids, ids)
        opt.step()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if eng.is_last:
            print(f"step {step} loss {float(loss):.4f} {a.batch / (time.time() - t0):.1f} samples/s")
    madnn.shutdown()


if __name__ == "__main__":
    main()
