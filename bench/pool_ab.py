#!/usr/bin/env python3
"""A/B the k=3/s=2 max-pool kernels (madnn_maxpool_set_k3s2, pool.hip) against the generic
window-loop kernels: (1) the ResNet-50 stem pool alone at batch 512 (fwd and bwd, HIP events,
bytes vs the HBM roofline), (2) the full training step, configurations interleaved round-robin
in one process so box drift hits both alike."""
import ctypes
import json
import statistics
import time

import torch
import torch.nn.functional as F


MODES = (0, 1, 2)  # generic, unrolled, unrolled + XCD-contiguous workgroups


def _time(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    import madnn
    from madnn import ops
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    madnn.init()
    assert ops.load_kernels()
    sel = ctypes.CDLL(str(ops.kernels_path())).madnn_maxpool_set_k3s2
    res = {}
    x = torch.randn(512, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = ops.max_pool2d(x, 3, 2, 1)
    dy = torch.randn_like(y)
    outs = {}
    for on in MODES:
        sel(on)
        yy = ops.max_pool2d(x, 3, 2, 1)
        x.grad = None
        yy.backward(dy)
        outs[on] = (yy.detach().clone(), x.grad.clone())
        fwd = _time(lambda: ops.max_pool2d(x.detach(), 3, 2, 1))
        yk = ops.max_pool2d(x, 3, 2, 1)
        bwd = _time(lambda: torch.autograd.grad(yk, x, dy, retain_graph=True))
        nx, ny = x.numel() * 2, y.numel() * 2
        res[f"k3s2_{on}"] = {"fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1),
                             "fwd_TBps": round((nx + ny + y.numel() // 8 * 8 / 8) / fwd / 1e6, 2),
                             "bwd_TBps": round((nx + ny + y.numel()) / bwd / 1e6, 2)}
    res["bitwise_equal"] = all(torch.equal(outs[0][i], outs[m][i]) for m in MODES for i in (0, 1))
    print(json.dumps(res), flush=True)
    del x, y, dy, outs

    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    dmodel, opt = madnn.distribute(model, opt, strategy="dp", channels_last=True)
    xb, yb = madnn.data.synthetic_batch("image", 512, madnn.device(), dtype=torch.bfloat16, channels_last=True,
                                        seed=1234)

    def step():
        F.cross_entropy(dmodel(xb).float(), yb).backward()
        opt.step()

    for _ in range(8):
        step()
    times = {m: [] for m in MODES}
    for rnd in range(5):
        for on in MODES:
            sel(on)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(6):
                step()
            torch.cuda.synchronize()
            times[on].append((time.perf_counter() - t0) / 6 * 1e3)
        print(json.dumps({f"k3s2_{o}": round(times[o][-1], 3) for o in MODES}), flush=True)
    sel(1)
    res["step_ms"] = {f"k3s2_{o}": {"median": round(statistics.median(v), 3), "min": round(min(v), 3)}
                      for o, v in times.items()}
    print(json.dumps(res), flush=True)
    with open("gpurun_out/pool_ab.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
