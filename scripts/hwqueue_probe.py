#!/usr/bin/env python3
"""Do two HIP streams of one process falsely serialise on a shared hardware queue?

For every ordered pair (A, B) of a set of streams, launch a bounded flag wait on A, then the
kernel that sets the flag on B (``madnn/ops/csrc/probe.hip``).  If A and B were given the same
hardware queue and that queue runs dispatches in submission order, the setter cannot start
until the waiter gives up: the waiter reports a timeout.  Otherwise the flag arrives in
microseconds.

Streams probed, in creation order (what a pipeline rank owns):
  * the default (null) stream -- the compute stream;
  * ``--low`` pool streams (``torch.cuda.Stream()``: madnn's DP comm stream, and what
    ProcessGroupNCCL takes for each communicator unless TORCH_NCCL_HIGH_PRIORITY=1);
  * ``--high`` high-priority pool streams.

Writes a JSON record: the blocked pairs, the classes of mutually blocking streams (= shared
hardware queues) and the environment (GPU_MAX_HW_QUEUES).  Every wait is bounded by
``--timeout-us``, so a blocked pair costs that and nothing more.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--low", type=int, default=12)
    ap.add_argument("--high", type=int, default=6)
    ap.add_argument("--timeout-us", type=int, default=20000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import madnn.ops as ops

    assert torch.cuda.is_available() and ops.load_kernels(), "needs the GPU and the madnn kernel library"
    dev = torch.device("cuda", 0)
    names, streams = ["default"], [torch.cuda.default_stream(dev)]
    for i in range(args.low):
        streams.append(torch.cuda.Stream(dev))
        names.append(f"low{i}")
    for i in range(args.high):
        streams.append(torch.cuda.Stream(dev, priority=-1))
        names.append(f"high{i}")
    n = len(streams)
    # touch every stream once (any lazy queue binding happens here, in creation order)
    for s in streams:
        with torch.cuda.stream(s):
            torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize()

    pairs = [(a, b) for a in range(n) for b in range(n) if a != b]
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(len(pairs), 2, dtype=torch.int32, device=dev)
    t0 = time.perf_counter()
    for k, (a, b) in enumerate(pairs):
        with torch.cuda.stream(streams[a]):
            torch.ops.madnn.hwq_wait(flag, k + 1, args.timeout_us, out[k])
        with torch.cuda.stream(streams[b]):
            torch.ops.madnn.hwq_set(flag, k + 1)
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    res = out.cpu().tolist()
    blocked = [(names[a], names[b]) for (a, b), (ok, _) in zip(pairs, res) if not ok]
    waited_us = {f"{names[a]}<-{names[b]}": t / 100.0 for (a, b), (_ok, t) in zip(pairs, res)}

    # classes of streams that block each other (union-find over blocked pairs)
    parent = list(range(n))

    def find(i):
        while parent[i] != i:
            parent[i] = parent[parent[i]]
            i = parent[i]
        return i

    idx = {nm: i for i, nm in enumerate(names)}
    for a, b in blocked:
        ra, rb = find(idx[a]), find(idx[b])
        if ra != rb:
            parent[rb] = ra
    classes = {}
    for i in range(n):
        classes.setdefault(find(i), []).append(names[i])
    rec = {
        "env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "HIP_FORCE_DEV_KERNARG", "AMD_SERIALIZE_KERNEL",
                                              "TORCH_NCCL_HIGH_PRIORITY")},
        "device": torch.cuda.get_device_name(0),
        "streams": names,
        "timeout_us": args.timeout_us,
        "pairs": len(pairs),
        "blocked_pairs": len(blocked),
        "blocked": blocked,
        "queue_classes": sorted(classes.values(), key=lambda c: names.index(c[0])),
        "max_unblocked_wait_us": max((t for (a, b), (ok, t) in zip(pairs, res) if ok), default=0) / 100.0,
        "wall_s": round(wall, 2),
    }
    line = json.dumps(rec)
    print(json.dumps({k: rec[k] for k in ("env", "blocked_pairs", "pairs", "queue_classes",
                                          "max_unblocked_wait_us", "wall_s")}), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            f.write(line + "\n")
        with open(args.out + ".waits.json", "w") as f:
            json.dump(waited_us, f)


if __name__ == "__main__":
    main()
