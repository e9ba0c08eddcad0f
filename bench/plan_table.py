"""The planner's 8-GPU placement for each BASELINE model, costed with HIP-event layer timings on
this GPU (analytic costs on CPU) and the shipped MI355X hardware profile: the candidate table
(every dp x pp x tp x checkpointing option with its modelled compute, exposed communication,
bubble and memory) and the choice, as markdown.

    python bench/plan_table.py --world 8 --out gpurun_out/plan_tables.md
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cases():
    from madnn.models import resnet50
    from madnn.models.bert import BertForPreTraining, bert_config
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.models.llama import Llama, llama_config

    # (name, builder, example input per sample batch, global batch per GPU, optimizer kind, checkpointing,
    #  config overrides)
    return [
        ("ResNet-50 (bench: 2048 images/GPU)", lambda: resnet50(),
         lambda b: torch.randn(b, 3, 224, 224), 2048, "sgd", "none", {}),
        ("GPT-2 medium (128 x 1024 tokens/GPU, unconstrained)", lambda: GPT2(gpt2_config("gpt2-medium")),
         lambda b: torch.zeros(b, 1024, dtype=torch.long), 128, "adam", "none", {}),
        ("GPT-2 medium (bench's pipeline half: 128 x 1024 tokens/GPU, 4 stages pinned, everything else automatic)",
         lambda: GPT2(gpt2_config("gpt2-medium")), lambda b: torch.zeros(b, 1024, dtype=torch.long), 128, "adam",
         "none", {"pp_stages": 4}),
        ("BERT-large (64 x 512/GPU, checkpointing auto)", lambda: BertForPreTraining(bert_config("bert-large")),
         lambda b: torch.zeros(b, 512, dtype=torch.long), 64, "adam", "auto", {}),
        ("Llama-3 8B (4 x 2048/GPU, checkpointing auto)", lambda: Llama(llama_config("llama3-8b")),
         lambda b: torch.zeros(b, 2048, dtype=torch.long), 4, "adam", "auto", {}),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import threading

    def heartbeat():      # measured layer costs take minutes per model: show progress
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"[plan_table] still planning ({time.time() - t0:.0f} s)", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    if torch.cuda.is_available():
        # the shipped MIOpen find-db, as madnn.init() seeds it for every job: without it every
        # convolution the layer timing touches is searched first (ResNet-50: 317 s instead of seconds)
        from madnn.utils.miopen import setup_find_db

        setup_find_db()
    from madnn.config import Config
    from madnn.planner import plan_model

    lines = [f"# Planner placements at {a.world} GPUs "
             f"({'measured layer costs on ' + torch.cuda.get_device_name(0) if torch.cuda.is_available() else 'analytic costs'})",
             ""]
    for name, build, example, per_gpu, opt, ckpt, over in cases():
        if a.only and a.only.lower() not in name.lower():
            continue
        t0 = time.time()
        with torch.device("meta"):
            model = build()
        cfg = Config()
        cfg.checkpointing = ckpt
        for k, v in over.items():
            setattr(cfg, k, v)
        optim = torch.optim.SGD if opt == "sgd" else torch.optim.AdamW
        plan = plan_model(model, cfg, a.world, example_input=example(1), global_batch=per_gpu * a.world,
                          optimizer=optim([torch.nn.Parameter(torch.zeros(1))], lr=0.1))
        hw = getattr(plan, "machine", None)
        cal = getattr(plan, "calibration", None) or {}
        cal_line = ("calibration: " + ", ".join(
            f"{k} {v:.3g}" if isinstance(v, float) else f"{k} {v}" for k, v in cal.items())) if cal else \
            "calibration: none"
        lines += [f"## {name}", "", f"choice: **{plan.describe()}** (planned in {time.time() - t0:.1f} s)", "",
                  cal_line, "",
                  f"links priced at: all-reduce eff {hw.allreduce_eff:.2f} x {hw.link_gbps:.0f} GB/s per link, "
                  f"P2P {hw.p2p_gbps:.0f} GB/s ({hw.source}; a job at W > 1 replaces these with its own "
                  "measurement, comm.probe)" if hw else "", "", plan.table(), ""]
        print("\n".join(lines[-8:]), flush=True)
    txt = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
