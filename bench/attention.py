#!/usr/bin/env python3
"""K8 attention (madnn MFMA kernels) vs PyTorch-ROCm SDPA: time and TFLOP/s.

    python bench/attention.py [--json out.json]

FLOPs use the standard accounting: forward 4*B*H*S^2*D (halved when causal),
backward 2.5x forward.  Both paths take the same bf16 [B, S, H, D] tensors; SDPA
gets them transposed to its [B, H, S, D] layout (views, as in a model).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # name, B, S, H, Hkv, D, causal
    ("gpt2-medium", 16, 1024, 16, 16, 64, True),
    ("bert-large", 32, 512, 16, 16, 64, False),
    ("llama3-8b", 4, 2048, 32, 8, 128, True),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--native", default="",
                    help="FUNC:KEY:ON:OFF -- A/B a native tunable (e.g. madnn_attn_tune:0:1:0): K8 only, both arms")
    a = ap.parse_args()
    if a.native:
        return ab_native(a)
    from madnn import ops

    assert ops.load_kernels()
    dev = torch.device("cuda")
    rows = []
    for name, B, S, H, HKV, D, causal in SHAPES:
        q = torch.randn(B, S, H, D, device=dev).bfloat16().requires_grad_(True)
        k = torch.randn(B, S, HKV, D, device=dev).bfloat16().requires_grad_(True)
        v = torch.randn(B, S, HKV, D, device=dev).bfloat16().requires_grad_(True)
        fl = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)

        def k8_f():
            return ops.attention(q, k, v, causal=causal)

        def sd_f():
            return F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                                  is_causal=causal, enable_gqa=H != HKV)

        o1, o2 = k8_f(), sd_f()
        do1 = torch.randn_like(o1)
        do2 = do1.transpose(1, 2)
        t_k8f = timeit(k8_f)
        t_sdf = timeit(sd_f)
        t_k8b = timeit(lambda: torch.autograd.grad(o1, (q, k, v), do1, retain_graph=True))
        t_sdb = timeit(lambda: torch.autograd.grad(o2, (q, k, v), do2, retain_graph=True))
        row = {"shape": name, "B": B, "S": S, "H": H, "Hkv": HKV, "D": D, "causal": causal,
               "k8_fwd_ms": round(t_k8f * 1e3, 3), "sdpa_fwd_ms": round(t_sdf * 1e3, 3),
               "k8_bwd_ms": round(t_k8b * 1e3, 3), "sdpa_bwd_ms": round(t_sdb * 1e3, 3),
               "k8_fwd_tflops": round(fl / t_k8f / 1e12, 1), "sdpa_fwd_tflops": round(fl / t_sdf / 1e12, 1),
               "k8_bwd_tflops": round(2.5 * fl / t_k8b / 1e12, 1), "sdpa_bwd_tflops": round(2.5 * fl / t_sdb / 1e12, 1),
               "max_abs_diff_fwd": float((o1.float() - o2.transpose(1, 2).float()).abs().max())}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=2)


def ab_native(a):
    """K8 forward / backward times with a native tunable ON vs OFF, interleaved rounds in one process."""
    import ctypes

    from madnn import ops

    assert ops.load_kernels()
    fn, key, von, voff = a.native.split(":")
    knob = getattr(ctypes.CDLL(str(ops.kernels_path())), fn)
    dev = torch.device("cuda")
    rows = []
    for name, B, S, H, HKV, D, causal in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, S, H, D, device=dev, generator=g).bfloat16().requires_grad_(True)
        k = torch.randn(B, S, HKV, D, device=dev, generator=g).bfloat16().requires_grad_(True)
        v = torch.randn(B, S, HKV, D, device=dev, generator=g).bfloat16().requires_grad_(True)
        fl = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        res = {True: {"f": [], "b": []}, False: {"f": [], "b": []}}
        outs = {}
        for rnd in range(6):
            for arm in ((True, False) if rnd % 2 == 0 else (False, True)):
                knob(int(key), int(von if arm else voff))
                o = ops.attention(q, k, v, causal=causal)
                do = torch.randn(o.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).bfloat16()
                res[arm]["f"].append(timeit(lambda: ops.attention(q, k, v, causal=causal)))
                res[arm]["b"].append(timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True)))
                if rnd == 0:
                    outs[arm] = (o.detach().float(), [t.float() for t in torch.autograd.grad(o, (q, k, v), do)])
        knob(int(key), int(von))
        med = {arm: {p: statistics.median(res[arm][p]) for p in "fb"} for arm in (True, False)}
        row = {"shape": name, "native": a.native,
               "on_fwd_ms": round(med[True]["f"] * 1e3, 3), "off_fwd_ms": round(med[False]["f"] * 1e3, 3),
               "on_bwd_ms": round(med[True]["b"] * 1e3, 3), "off_bwd_ms": round(med[False]["b"] * 1e3, 3),
               "on_fwd_tflops": round(fl / med[True]["f"] / 1e12, 1),
               "on_bwd_tflops": round(2.5 * fl / med[True]["b"] / 1e12, 1),
               "max_abs_diff_o": float((outs[True][0] - outs[False][0]).abs().max()),
               "max_abs_diff_grads": [float((x - y).abs().max()) for x, y in zip(outs[True][1], outs[False][1])]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=2)


if __name__ == "__main__":
    main()
