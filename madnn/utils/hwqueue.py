"""Replay pipeline ranks' programs on ONE GPU's real hardware queues (see scripts/hwqueue_pipeline.py).

Two ranks of an S = 2 pipeline run inside one process, each on its OWN hardware-queue pool:
rank 0 on the default stream plus normal-priority pool streams, rank 1 on high-priority pool
streams (``scripts/hwqueue_probe.py`` measured that the two pools never share a queue).  Each rank
drives as many streams as a real rank (compute, WORLD, pipeline, gradient, tied, DP comm, side),
so its streams contend for its 4 queues as in a real job.  Messages have RCCL's rendezvous
semantics (``hwq_batch``), compute is a busy kernel (``hwq_spin``), every wait is bounded: a
program that deadlocks on the queues reports timed-out messages instead of hanging.
"""
from __future__ import annotations

import time

import torch


class _Rank:
    def __init__(self, stage, priority, nstreams):
        self.stage = stage
        self.pool = [torch.cuda.Stream(priority=priority) for _ in range(nstreams)]
        self.compute = torch.cuda.default_stream() if priority == 0 else self.pool[0]


_RANKS = {}


def _ranks(nstreams):
    if nstreams not in _RANKS:
        dev = torch.device("cuda", torch.cuda.current_device())
        ranks = [_Rank(0, 0, nstreams), _Rank(1, -1, nstreams)]
        for r in ranks:                     # bind every stream to its queue (creation order)
            for s in r.pool + [r.compute]:
                with torch.cuda.stream(s):
                    torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize()
        _RANKS[nstreams] = ranks
    return _RANKS[nstreams]


def replay(kind: str, V: int, M: int, design: str, spin_us: int = 200, timeout_us: int = 300000,
           streams: int = 7, epoch: int = 1, lag: float = 0.0) -> dict:
    """Run one training step of both ranks' programs (``design``: ``engine`` = madnn's
    ``issue_plan`` at ``lag``, ``prepost`` = the round-3 engine) and count the messages that
    timed out."""
    from ..ops import native_runtime
    from ..parallel.pp import issue_plan, recv_plan, virtual_stage

    dev = torch.device("cuda", torch.cuda.current_device())
    S = 2
    ranks = _ranks(streams)
    msg_id = {}

    def mid(key):
        if key not in msg_id:
            msg_id[key] = len(msg_id)
        return msg_id[key]

    a = torch.zeros(4096, dtype=torch.int32, device=dev)
    b = torch.zeros(4096, dtype=torch.int32, device=dev)

    def msg(d, k, c, m, s):
        vs = c * S + s
        if d == "recv":
            return (k, vs, m)
        return (k, vs + 1 if k == "act" else vs - 1, m)

    # 1) every rank's program as actions (nothing touches the GPU yet)
    progs = []
    for r in ranks:
        s = r.stage
        acts = []     # ("batch", stream_name, [(d, msg)], needs_last, is_recv) / ("compute", us)
        if design == "engine":
            for item in issue_plan(kind, s, S, M, V, lag):
                if item[0] == "X":
                    for k in ("act", "grad"):
                        part = [(d, msg(d, kk, c, m, s)) for d, kk, c, m, _p in item[1] if kk == k]
                        if part:
                            sends = any(d == "send" for d, _ in part)
                            acts.append(("batch", k, part, sends, any(d == "recv" for d, _ in part)))
                else:
                    acts.append(("compute", spin_us * (1 if item[1] == "F" else 2)))
        else:
            order = native_runtime.pipeline_order(kind, s, S, M, V)
            vst = [virtual_stage(c, s, S) for c in range(V)]
            for k, c, m in recv_plan(order, vst, S * V):
                acts.append(("batch", k + "_in", [("recv", msg("recv", k, c, m, s))], False, (k, c, m)))
            for op, c, m in order:
                vs = vst[c]
                key = ("act", c, m) if op == "F" and vs > 0 else (
                    ("grad", c, m) if op == "B" and vs < S * V - 1 else None)
                acts.append(("compute", spin_us * (1 if op == "F" else 2), key))
                k = "act" if op == "F" and vs < S * V - 1 else ("grad" if op == "B" and vs > 0 else None)
                if k is not None:
                    acts.append(("batch", k + "_out", [("send", msg("send", k, c, m, s))], True, None))
        progs.append(acts)
    # 2) the op tables of every batch in ONE device tensor, copied before anything runs
    kinds, msgs, idx = [], [], []
    for acts in progs:
        for act in acts:
            if act[0] == "batch":
                for d, m in act[2]:
                    kinds.append(0 if d == "send" else 1)
                    msgs.append(mid(m))
                    idx.append(len(idx))
    table = torch.tensor([kinds, msgs, idx], dtype=torch.int32, device=dev)
    ok = torch.full((len(idx),), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    # 3) issue: each rank's streams in its own queue pool
    t0 = time.perf_counter()
    pos = 0
    for r, acts in zip(ranks, progs):
        st = {"act": r.pool[1], "grad": r.pool[2], "act_in": r.pool[1], "grad_in": r.pool[2],
              "act_out": r.pool[3], "grad_out": r.pool[4]}
        last, pending, got = None, [], {}
        for act in acts:
            if act[0] == "batch":
                _, name, part, after_compute, tag = act
                stream = st[name]
                if after_compute and last is not None:
                    stream.wait_event(last)          # a send follows its producer
                n = len(part)
                with torch.cuda.stream(stream):
                    torch.ops.madnn.hwq_batch(table[0, pos:pos + n], table[1, pos:pos + n], a, b, epoch,
                                              timeout_us, ok, table[2, pos:pos + n])
                pos += n
                ev = torch.cuda.Event()
                ev.record(stream)
                if design == "engine" and tag:
                    pending.append(ev)
                elif design == "prepost" and tag is not None and not after_compute:
                    got[tag] = ev
            else:
                if design == "engine":
                    for ev in pending:
                        r.compute.wait_event(ev)
                    pending = []
                elif act[2] is not None:
                    r.compute.wait_event(got[act[2]])
                with torch.cuda.stream(r.compute):
                    torch.ops.madnn.hwq_spin(a, act[1])
                last = torch.cuda.Event()
                last.record(r.compute)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    res = ok.cpu()
    return {"schedule": kind, "V": V, "micro": M, "design": design, "lag": lag, "messages": len(idx),
            "timed_out": int((res == 0).sum()), "unset": int((res < 0).sum()), "wall_s": round(wall, 3)}
