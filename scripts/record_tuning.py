#!/usr/bin/env python3
"""Regenerate madnn's shipped start-up tuning on one MI355X (run through gpurun).

Two things make a fresh process's first training step slow: madnn's per-shape timing of the
weight-gradient / GELU-Linear implementations (``ops.tuned_wgrad``), and MIOpen's search for
convolution problems its find-db does not hold yet (that is where round 3's 76 s warm-up went:
``profiles/r4_first_steps_resnet50_b2048_*.json``).  This script runs the bench
configurations (ResNet-50 at 2048 and 512 images, GPT-2 medium at every microbatch size the
pipeline planner may choose, BERT-large at 128 sequences) from an EMPTY choice table with MIOpen's user db pointed at
``--out``, then writes

  <out>/choices_gfx950.json   -> madnn/tuning/choices_gfx950.json
  <out>/miopen/*.txt          -> madnn/tuning/miopen/

and prints each model's first-step / steady-step times.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tuning")
    ap.add_argument("--resnet-batches", default="2048,512")
    ap.add_argument("--gpt2-batches", default="128,64,32,16,8,4")
    ap.add_argument("--bert-batches", default="128")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--keep-table", action="store_true",
                    help="start from the shipped choice table (time only the shapes it lacks) instead of an empty one")
    ap.add_argument("--retime", default="",
                    help="with --keep-table: comma list of table:kind entries to drop and time afresh, e.g. "
                         "wgrad:linear (every Linear weight gradient, with K12W as a candidate); table:* drops a whole table")
    args = ap.parse_args()
    out = Path(args.out)
    db = out / "miopen"
    db.mkdir(parents=True, exist_ok=True)
    for f in (ROOT / "madnn" / "tuning" / "miopen").iterdir():
        if f.is_file():
            shutil.copy2(f, db / f.name)
    os.environ["MIOPEN_USER_DB_PATH"] = str(db)
    if not args.keep_table:
        os.environ["MADNN_TUNE_TABLE"] = "0"      # decide every shape afresh

    import torch
    import torch.nn.functional as F

    import madnn
    import madnn.ops as ops

    madnn.init()
    if args.keep_table:
        ops.load_kernels()
        tables = {"wgrad": ops._WGRAD_CHOICE, "gelu_fwd": ops._GELU_FWD_CHOICE, "dgelu": ops._DGELU_CHOICE,
                  "dgrad": ops._DGRAD_CHOICE}
        for item in [v for v in args.retime.split(",") if v]:
            tab, kind = item.split(":")
            for k in [k for k in tables[tab] if k and (kind == "*" or k[0] == kind)]:
                del tables[tab][k]
    dev = madnn.device()
    rec = []

    def run(name, step, n):
        times = []
        for _ in range(n):
            torch.cuda.synchronize()
            t = time.perf_counter()
            step()
            torch.cuda.synchronize()
            times.append(round(time.perf_counter() - t, 3))
        rec.append({"model": name, "step_s": times, "timed_so_far": ops.tuning_timings()})
        print(json.dumps(rec[-1]), flush=True)

    from madnn.models import resnet50
    from madnn.optim import FusedAdam, FusedSGD

    for b in [int(v) for v in args.resnet_batches.split(",") if v]:
        torch.manual_seed(0)
        model = resnet50()
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
        dmodel, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
        x, y = madnn.data.synthetic_batch("image", b, dev, dtype=torch.bfloat16, channels_last=True, seed=1)

        def step():
            F.cross_entropy(dmodel(x).float(), y).backward()
            opt.step()

        run(f"resnet50_b{b}", step, args.steps)
        dmodel.remove_hooks()
        del model, opt, dmodel, x, y
        torch.cuda.empty_cache()

    from madnn.models.gpt2 import GPT2, gpt2_config

    for b in [int(v) for v in args.gpt2_batches.split(",") if v]:
        torch.manual_seed(0)
        cfg = gpt2_config("gpt2-medium")
        model = GPT2(cfg)
        opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
        engine, opt = madnn.distribute(model, opt, strategy="dp", checkpointing="none",
                                       example_input=torch.zeros(1, 1024, dtype=torch.long))
        ids = torch.randint(0, cfg.vocab_size, (b, 1024)).to(dev)

        def step():
            engine.train_step(ids, ids)
            opt.step()

        run(f"gpt2-medium_b{b}", step, args.steps)
        del model, opt, engine, ids
        torch.cuda.empty_cache()

    from madnn.models.bert import BertForPreTraining, bert_config

    for b in [int(v) for v in args.bert_batches.split(",") if v]:
        torch.manual_seed(0)
        cfg = bert_config("bert-large")
        model = BertForPreTraining(cfg)
        opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
        engine, opt = madnn.distribute(model, opt, strategy="dp", checkpointing="none",
                                       example_input=torch.zeros(1, 512, dtype=torch.long))
        ids = torch.randint(0, cfg.vocab_size, (b, 512)).to(dev)

        def step():
            engine.train_step(ids, ids)
            opt.step()

        run(f"bert-large_b{b}", step, args.steps)
        del model, opt, engine, ids
        torch.cuda.empty_cache()

    ops.export_choices(str(out / "choices_gfx950.json"))
    (out / "record.json").write_text(json.dumps(rec, indent=1) + "\n")
    # the per-shape A/B behind every choice (ms for 3 calls of each implementation)
    (out / "measurements.json").write_text(json.dumps(ops.tuning_measurements(), indent=1) + "\n")
    print(json.dumps({"choices": len(ops._WGRAD_CHOICE) + len(ops._GELU_FWD_CHOICE) + len(ops._DGELU_CHOICE)
                      + len(ops._DGRAD_CHOICE),
                      "miopen_db": sorted(p.name for p in db.iterdir())}), flush=True)


if __name__ == "__main__":
    main()
