"""Launch-shape sweep of the two streaming passes left in the GPT-2 medium step (GELU forward
after c_fc, LayerNorm forward) at the bench shape (64 x 1024 tokens): each setting of the native
launch knobs timed in interleaved rounds (rotated order, medians), with the analytic HBM rate.

    python bench/stream_tune.py --out gpurun_out/stream_tune.json
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def sweep(name, lib, setter, settings, fn, nbytes, rounds):
    times = {repr(st): [] for st in settings}
    for r in range(rounds):
        order = settings[r % len(settings):] + settings[:r % len(settings)]
        for st in order:
            setter(lib, st)
            times[repr(st)].append(_time(fn))
    out = []
    for st in settings:
        us = statistics.median(times[repr(st)])
        out.append({"kernel": name, "setting": st, "us": round(us, 1), "tbps": round(nbytes / us / 1e6, 2)})
        print(json.dumps(out[-1]), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from madnn import ops

    assert torch.cuda.is_available() and ops.load_kernels()
    lib = ctypes.CDLL(str(ops.kernels_path()))
    res = []
    x = torch.randn(a.rows, 4096, device="cuda", dtype=torch.bfloat16)

    def set_gelu(lib, st):
        lib.madnn_gelu_tune(0, st[0])
        lib.madnn_gelu_tune(1, st[1])

    res += sweep("gelu_fwd [M, 4096]", lib, set_gelu, [(1, 8), (8, 4), (1, 4), (2, 8)],
                 lambda: ops.gelu_tanh(x), 2 * x.numel() * 2, a.rounds)
    set_gelu(lib, (1, 8))
    # the fused GELU backward + bias-gradient pass (K11): workgroups per CU
    dy = torch.randn_like(x)
    res += sweep("bias_grad+gelu_bwd [M, 4096]", lib, lambda l, st: l.madnn_bias_tune(1, st), [4, 2, 1, 8],
                 lambda: ops.bias_grad(dy, x, torch.bfloat16), 3 * x.numel() * 2, a.rounds)
    lib.madnn_bias_tune(1, 4)
    del x, dy
    # FusedAdam over 64M parameters (fp32 master / m / v, bf16 grad and model copy)
    from madnn.optim import FusedAdam

    p = torch.nn.Parameter(torch.randn(64 << 20, device="cuda", dtype=torch.bfloat16))
    p.grad = torch.randn_like(p)
    opt = FusedAdam([p], lr=1e-4)
    opt.step()
    res += sweep("adam [64M]", lib, lambda l, st: l.madnn_optim_tune(0, st), [4, 2, 1, 8], opt.step,
                 p.numel() * (4 * 3 * 2 + 2 + 2), a.rounds)
    lib.madnn_optim_tune(0, 4)
    del p, opt
    h = torch.randn(a.rows, 1024, device="cuda", dtype=torch.bfloat16)
    w = torch.ones(1024, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(1024, device="cuda", dtype=torch.bfloat16)

    def set_norm(lib, st):
        lib.madnn_norm_tune(0, st)

    with torch.no_grad():
        res += sweep("norm_fwd [M, 1024]", lib, set_norm, [8, 16, 32], lambda: ops.layer_norm(h, w, b),
                     2 * h.numel() * 2, a.rounds)
    set_norm(lib, 8)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
