#!/usr/bin/env python3
"""Microbenchmarks of madnn's HIP kernels vs the HBM roofline (and vs the eager ops they replace).

    python bench/kernels.py [--n 268435456] [--json out.json]
    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -- python3 bench/kernels.py --iters 3

Each kernel runs on buffers far larger than the 256 MiB Infinity Cache, so the
bytes really come from HBM; achieved GB/s = analytic bytes moved / time
(HIP events, median of --iters).  Bytes per element per kernel:
  sgd (momentum, bf16 model copy): read p,g,m (12) + write p,m (8) + bf16 (2)  = 22 B
  adam (bf16 grad + bf16 model):   read p,m,v (12) + g (2) + write p,m,v (12) + 2 = 28 B
  pack bf16->fp32 (K4):            read 2 + write 4 = 6 B
  layernorm fwd bf16, H=1024:      read 2 + write 2 (+ stats)  = 4 B
  layernorm bwd bf16:              read x, dy (4) + write dx (2) = 6 B
  bn fwd (stats + apply, +res,+relu) bf16: read x (2) + read x,res (4) + write y (2) = 8 B
  xent fwd/bwd bf16:               read 2 / read 2 + write 2 B
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters):
    ts = []
    for _ in range(2):
        fn()
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
    ap.add_argument("--n", type=int, default=1 << 28, help="elements per buffer (default 256M)")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    dev = torch.device("cuda")
    n = a.n
    res = []

    def rec(name, t, nbytes, ref_t=None):
        row = {"kernel": name, "ms": round(t * 1e3, 3), "GBps": round(nbytes / t / 1e9, 1),
               "bytes": nbytes}
        if ref_t is not None:
            row["eager_ms"] = round(ref_t * 1e3, 3)
            row["speedup_vs_eager"] = round(ref_t / t, 2)
        res.append(row)
        print(json.dumps(row), flush=True)

    # K1 SGD
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.randn(n, device=dev)
    mb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.sgd_step(p, g, m, mb, lr=1e-3, momentum=0.9, weight_decay=1e-4), a.iters)
    tref = timeit(lambda: torch._foreach_add_([p], [g], alpha=-1e-3), a.iters)
    rec("K1 sgd_step (momentum, fp32 grad, bf16 copy)", t, 22 * n)
    del g
    # K2 Adam
    gb = torch.randn(n, device=dev).bfloat16()
    v = torch.rand(n, device=dev)
    t = timeit(lambda: ops.adam_step(p, gb, m, v, mb, lr=1e-4, step=3, weight_decay=0.01), a.iters)
    pr = [p.clone()]
    gr = [gb.float()]
    o = torch.optim.AdamW(pr, lr=1e-4, weight_decay=0.01, fused=True)
    pr[0].grad = gr[0]
    tref = timeit(lambda: o.step(), a.iters)
    rec("K2 adam_step (bf16 grad, bf16 copy)", t, 28 * n, tref)
    del pr, gr, o, v
    # K4 pack: 64 tensors bf16 -> fp32 flat, 1/W fused
    k = 64
    ts = [torch.randn(n // k, device=dev).bfloat16() for _ in range(k)]
    offs = [i * (n // k) for i in range(k)]
    flat = torch.empty(n, device=dev)
    t = timeit(lambda: ops.bucket_pack(ts, flat, offs, 0.125), a.iters)
    tref = timeit(lambda: torch.cat([x.float().mul_(0.125) for x in ts]), a.iters)
    rec("K4 bucket_pack (64 bf16 tensors -> fp32, x1/W)", t, 6 * n, tref)
    t = timeit(lambda: ops.bucket_unpack(ts, flat, offs, 1.0), a.iters)
    rec("K4 bucket_unpack (fp32 -> 64 bf16 tensors)", t, 6 * n)
    del ts, flat
    # K3 LayerNorm fwd/bwd bf16, H = 1024
    H = 1024
    rows = n // H
    x = torch.randn(rows, H, device=dev).bfloat16().requires_grad_(True)
    w = torch.ones(H, device=dev, requires_grad=True)
    b = torch.zeros(H, device=dev, requires_grad=True)
    t = timeit(lambda: ops.layer_norm(x.detach(), w.detach(), b.detach()), a.iters)
    tref = timeit(lambda: torch.nn.functional.layer_norm(x.detach(), (H,), w.detach().bfloat16(),
                                                          b.detach().bfloat16()), a.iters)
    rec("K3 layer_norm fwd bf16 H=1024", t, 4 * rows * H, tref)
    y = ops.layer_norm(x, w, b)
    dy = torch.randn_like(y)
    t = timeit(lambda: torch.autograd.grad(y, (x, w, b), dy, retain_graph=True), a.iters)
    rec("K3 layer_norm bwd bf16 H=1024", t, 6 * rows * H)
    del x, y, dy
    # K5 BN fwd (train) NHWC bf16, C=256, + residual + relu
    C = 256
    N = n // (C * 56 * 56) or 1
    xb = torch.randn(N, C, 56, 56, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(xb)
    wb, bb = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    t = timeit(lambda: ops.batch_norm_act(xb, wb, bb, rm, rv, training=True, relu=True, residual=r), a.iters)
    tref = timeit(lambda: torch.relu(torch.nn.functional.batch_norm(xb, rm, rv, wb, bb, True) + r), a.iters)
    rec(f"K5 batchnorm+add+relu fwd NHWC bf16 C={C}", t, 8 * xb.numel(), tref)
    del xb, r
    # K6 cross-entropy fwd+bwd, GPT-2 vocab
    V = 50257
    rows = max(n // 50304 // 4, 1)
    lg = torch.randn(rows, 50304, device=dev).bfloat16().requires_grad_(True)
    tg = torch.randint(0, V, (rows,), device=dev)

    def xent():
        loss = ops.cross_entropy(lg, tg, vocab=V)
        loss.backward()

    def xref():
        loss = torch.nn.functional.cross_entropy(lg[:, :V].float(), tg)
        loss.backward()

    t = timeit(xent, a.iters)
    tref = timeit(xref, a.iters)
    rec("K6 cross_entropy fwd+bwd bf16 V=50257", t, 6 * lg.numel(), tref)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(), "n": n, "results": res}, f, indent=2)


if __name__ == "__main__":
    main()
