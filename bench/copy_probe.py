#!/usr/bin/env python3
"""Which ATen ops launch device copies / fills in one Llama training step (8B layer dims, 2 layers,
one GPU, the bench's distribute path): torch.profiler op table of copy_ / fill_ / contiguous /
clone / zero_ calls with their input shapes.  python bench/copy_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import madnn
    from madnn.models.llama import Llama, llama_config
    from madnn.optim import FusedAdam

    madnn.init()
    dev = madnn.device()
    cfg = llama_config("llama3-8b", layers=2, vocab_size=32000)
    torch.manual_seed(0)
    model = Llama(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4)
    engine, opt = madnn.distribute(model, opt, strategy="dp", checkpointing="none",
                                   example_input=torch.zeros(1, 2048, dtype=torch.long))
    ids = torch.randint(0, cfg.vocab_size, (2, 2048)).to(dev)

    def step():
        engine.train_step(ids, ids)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages(group_by_input_shape=True):
        if any(k in e.key for k in ("copy_", "fill_", "contiguous", "clone", "zero_", "to_copy", "cat", "add_", "add")):
            rows.append((e.count, e.key, str(e.input_shapes)[:150]))
    for r in sorted(rows, key=lambda r: -r[0])[:40]:
        print(r, flush=True)


if __name__ == "__main__":
    main()
