#!/usr/bin/env python3
"""Replay two pipeline ranks' programs on ONE MI355X's real hardware queues.

``scripts/hwqueue_probe.py`` shows that a process's streams share GPU_MAX_HW_QUEUES (4)
hardware queues and serialise across them.  This script runs the two ranks of an S = 2
pipeline inside one process, each on its OWN queue pool -- rank 0 on the default stream plus
normal-priority pool streams, rank 1 on high-priority pool streams (the probe measured that
the two pools never share a queue) -- with as many streams per rank as a real rank drives
(compute, WORLD, pipeline, gradient, tied, DP comm, side), so each rank's streams contend for
its 4 queues the way they do in a real job.

Messages use RCCL's rendezvous semantics (``hwq_batch``: a send waits for its receiver's
acknowledgement, one kernel per batch completes when all its messages met their peers);
compute is a busy kernel (``hwq_spin``).  Every wait is bounded, so a program that deadlocks
on the queues shows up as timed-out messages.  Two programs per schedule:

* ``engine``: madnn's ``issue_plan`` (boundary batches, activations / gradients on two
  communicators, receive-only parts on a side stream), at lag 0 and at lag 0.3 (boundaries on a
  clock with transfers; the engine times both on a job and keeps the faster);
* ``prepost``: the round-3 engine (every receive of the step posted up front on its channel's
  stream, sends after their producer).

Prints one JSON line per (schedule, design) with the number of timed-out messages.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro", type=int, default=8)
    ap.add_argument("--spin-us", type=int, default=200)
    ap.add_argument("--timeout-us", type=int, default=300000)
    ap.add_argument("--streams", type=int, default=7, help="streams per rank (compute + comm)")
    ap.add_argument("--reps", type=int, default=1, help="replays per (schedule, plan)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import madnn.ops as ops
    from madnn.utils.hwqueue import replay

    assert torch.cuda.is_available() and ops.load_kernels()
    results = []
    epoch = 0
    for kind, V in (("gpipe", 1), ("1f1b", 1), ("interleaved", 2)):
        for design, lag in (("engine", 0.0), ("engine", 0.3), ("prepost", 0.0)):
            for _rep in range(args.reps):
                epoch += 1
                rec = replay(kind, V, args.micro, design, args.spin_us, args.timeout_us, args.streams, epoch, lag)
                results.append(rec)
                print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"streams_per_rank": args.streams, "timeout_us": args.timeout_us, "spin_us": args.spin_us,
                       "results": results}, f, indent=1)


if __name__ == "__main__":
    main()
