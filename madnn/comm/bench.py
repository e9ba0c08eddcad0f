"""Collective microbenchmark — the working version of the
reference's dead ``comm_speed`` probe (datamodule.lua:280-303).

    python -m madnn.launch --nproc 8 -m madnn.comm.bench --out gpurun_out/comm.json

Sweeps message sizes for all_reduce / all_gather / reduce_scatter / broadcast
and a point-to-point ping-pong between ranks 0 and 1, reports algorithm and
bus bandwidth (busbw = algbw x 2(W-1)/W for all-reduce, (W-1)/W for gathers),
and with ``--hw-profile`` writes the measured large-message link bandwidth in
the planner's ``Machine`` format (``MADNN_HW_PROFILE``) so stage placement and
bucket sizing are priced with this node's numbers.
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist

from .. import runtime as rt


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _time(fn, iters, warmup):
    for _ in range(warmup):
        fn()
    _sync()
    rt.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    _sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], device=rt.device(), dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run(sizes, iters: int = 20, warmup: int = 5, dtype=torch.bfloat16, ops=("all_reduce", "all_gather",
                                                                              "reduce_scatter", "broadcast", "p2p")):
    rt.init()
    w = rt.get_world_size()
    dev = rt.device()
    res = []
    esz = torch.tensor([], dtype=dtype).element_size()
    for nbytes in sizes:
        n = max(nbytes // esz // max(w, 1) * max(w, 1), max(w, 1))
        x = torch.ones(n, dtype=dtype, device=dev)
        row = {"bytes": n * esz}
        if "all_reduce" in ops:
            t = _time(lambda: dist.all_reduce(x) if w > 1 else x.add_(0), iters, warmup)
            row["all_reduce_us"] = t * 1e6
            row["all_reduce_busbw_gbps"] = (n * esz / t) * (2 * (w - 1) / w) / 1e9 if w > 1 else 0.0
        if "all_gather" in ops and w > 1:
            out = torch.empty(n * w, dtype=dtype, device=dev)
            t = _time(lambda: dist.all_gather_into_tensor(out, x), iters, warmup)
            row["all_gather_us"] = t * 1e6
            row["all_gather_busbw_gbps"] = (n * w * esz / t) * ((w - 1) / w) / 1e9
        if "reduce_scatter" in ops and w > 1:
            out = torch.empty(n // w, dtype=dtype, device=dev)
            t = _time(lambda: dist.reduce_scatter_tensor(out, x), iters, warmup)
            row["reduce_scatter_us"] = t * 1e6
            row["reduce_scatter_busbw_gbps"] = (n * esz / t) * ((w - 1) / w) / 1e9
        if "broadcast" in ops and w > 1:
            t = _time(lambda: dist.broadcast(x, src=0), iters, warmup)
            row["broadcast_us"] = t * 1e6
            row["broadcast_algbw_gbps"] = n * esz / t / 1e9
        if "p2p" in ops and w > 1:
            r = rt.get_rank()

            def pingpong():
                if r == 0:
                    dist.send(x, 1)
                    dist.recv(x, 1)
                elif r == 1:
                    dist.recv(x, 0)
                    dist.send(x, 0)

            t = _time(pingpong, iters, warmup)
            row["p2p_roundtrip_us"] = t * 1e6
            row["p2p_gbps"] = 2 * n * esz / t / 1e9
        res.append(row)
    return res


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-bytes", type=int, default=1 << 10)
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--hw-profile", default=None, help="write measured link numbers for the planner")
    a = ap.parse_args(argv)
    sizes = []
    s = a.min_bytes
    while s <= a.max_bytes:
        sizes.append(s)
        s *= 4
    res = run(sizes, iters=a.iters)
    if rt.get_rank() == 0:
        w = rt.get_world_size()
        print(f"world={w} device={rt.device()}")
        for row in res:
            print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}))
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"world": w, "results": res}, f, indent=2)
        if a.hw_profile and w > 1:
            from ..planner.hw import Machine, dump

            big = res[-1]
            m = Machine()
            # busbw of one ring-spread all-reduce over min(links, W-1) links -> per-link bandwidth
            m.link_gbps = big["all_reduce_busbw_gbps"] / (min(m.links, w - 1) * m.allreduce_eff)
            if "p2p_gbps" in big:
                m.p2p_gbps = big["p2p_gbps"]
            dump(m, a.hw_profile)
    rt.shutdown()


if __name__ == "__main__":
    main()
