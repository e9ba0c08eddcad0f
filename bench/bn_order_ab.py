#!/usr/bin/env python3
"""A/B the fused-BN apply passes' walk order and grid size (madnn_bn_tune, bn.hip) inside the
full ResNet-50 training step at batch 512; one process, configurations interleaved round-robin
so box drift hits all of them alike (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes
import json
import statistics
import sys
import time

import torch
import torch.nn.functional as F


def main():
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init()
    assert madnn.ops.load_kernels()
    tune = ctypes.CDLL(str(madnn.ops.kernels_path())).madnn_bn_tune
    per_gpu = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dmodel, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
    x, y = madnn.data.synthetic_batch("image", per_gpu, madnn.device(), dtype=torch.bfloat16, channels_last=True,
                                      seed=1234)

    def step():
        F.cross_entropy(dmodel(x).float(), y).backward()
        opt.step()

    for _ in range(8):
        step()
    cfgs = [(0, 16), (1, 8), (0, 8), (1, 16)]  # (reverse, workgroups per CU); (0, 16) = the old fixed launch
    times = {c: [] for c in cfgs}
    for rnd in range(5):
        for rev, wg in cfgs:
            tune(0, rev)
            tune(1, wg)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(6):
                step()
            torch.cuda.synchronize()
            times[(rev, wg)].append((time.perf_counter() - t0) / 6 * 1e3)
        print(json.dumps({f"rev{r}_wg{w}": round(times[(r, w)][-1], 3) for r, w in cfgs}), flush=True)
    res = {f"rev{r}_wg{w}": {"median_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3)}
           for (r, w), v in times.items()}
    res["per_gpu_batch"] = per_gpu
    print(json.dumps(res), flush=True)
    with open("gpurun_out/bn_order_ab.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
