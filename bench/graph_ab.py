"""ResNet-50 DP1 step: eager launches vs one HIP-graph replay per step (madnn.utils.graphs), same
process, interleaved timing windows; plus a parity check (graph-replayed training reaches the same
weights as eager training from the same initial state).

    python bench/graph_ab.py --batch 512 --windows 6 --steps 8
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(batch, seed=0):
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    torch.manual_seed(seed)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    eng, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
    x, y = madnn.data.synthetic_batch("image", batch, madnn.device(), dtype=torch.bfloat16, channels_last=True,
                                      seed=1234)

    def step():
        loss = F.cross_entropy(eng(x).float(), y)
        loss.backward()
        opt.step()
        return loss.detach()

    return eng, opt, step


def timed(fn, n):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import madnn
    from madnn.utils.graphs import capture_step

    madnn.init()
    # parity: 6 eager steps vs 3 eager warm-up steps + capture + 3 replays, same init
    eng_a, _, step_a = build(a.batch)
    for _ in range(6):
        la = step_a()
    wa = torch.cat([p.detach().float().flatten() for p in eng_a.module.parameters()])
    del eng_a, step_a
    torch.cuda.empty_cache()
    eng_b, _, step_b = build(a.batch)
    g = capture_step(step_b, warmup=3)
    for _ in range(3):
        lb = g()
    wb = torch.cat([p.detach().float().flatten() for p in eng_b.module.parameters()])
    diff = float((wa - wb).abs().max())
    parity = {"loss_eager": float(la), "loss_graph": float(lb), "max_abs_weight_diff": diff}
    print(json.dumps(parity), flush=True)
    # timing: interleaved windows on the same model
    eager, graph = [], []
    for w in range(a.windows):
        eager.append(timed(step_b, a.steps))
        graph.append(timed(g, a.steps))
        print(json.dumps({"window": w, "eager_ms": round(eager[-1], 3), "graph_ms": round(graph[-1], 3)}), flush=True)
    res = {"batch": a.batch, "eager_ms_median": statistics.median(eager), "graph_ms_median": statistics.median(graph),
           "speedup": statistics.median(eager) / statistics.median(graph), "parity": parity,
           "eager_ms": eager, "graph_ms": graph}
    print(json.dumps(res), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
