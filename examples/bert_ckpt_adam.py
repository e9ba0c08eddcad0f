#!/usr/bin/env python3
"""BERT-large: auto-partition + activation checkpointing + fused Adam (BASELINE config 5).

    python -m madnn.launch --nproc 8 examples/bert_ckpt_adam.py --batch 256

``strategy="auto"`` lets the planner choose the placement; ``checkpointing="auto"``
lets it decide per block whether recomputation is needed to fit (force with "all").
Post-LN sublayers run the K3 LayerNorm kernel with the residual add fused; the
masked-LM loss is the K6 fused cross-entropy; FusedAdam is the K2 HIP kernel.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import madnn  # noqa: E402
from madnn.models.bert import BertForPreTraining, bert_config  # noqa: E402
from madnn.optim import FusedAdam  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-large")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--checkpointing", default="all")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    madnn.init()
    torch.manual_seed(0)
    cfg = bert_config(a.model)
    model = BertForPreTraining(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    eng, opt = madnn.distribute(model, opt, strategy="auto", checkpointing=a.checkpointing, global_batch=a.batch,
                                example_input=torch.zeros(1, a.seq, dtype=torch.long))
    if madnn.get_rank() == 0:
        print(eng.plan.describe() if eng.plan is not None else "dp")
    dp = eng.plan.dp if eng.plan is not None else madnn.get_world_size()
    ids = madnn.data.synthetic_batch("tokens", a.batch // dp, madnn.device(), seq_len=a.seq, vocab=cfg.vocab_size)[0]
    for step in range(a.steps):
        loss = eng.train_step(ids, ids)
        opt.clip_grad_norm_(1.0)
        opt.step()
        if loss is not None and madnn.get_rank() == 0:
            print(f"step {step} loss {float(loss):.4f}")
    madnn.shutdown()


if __name__ == "__main__":
    main()
