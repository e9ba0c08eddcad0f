#!/usr/bin/env python3
"""Comm/compute overlap from a rocprofv3 ``*_kernel_trace.csv``.

For every RCCL kernel: which HIP queue/stream it ran on and how much of its lifetime
overlapped kernels on OTHER streams (the backward's compute kernels).  Evidence for
"RCCL all-reduce on the comm stream interleaved with backward kernels".

usage: comm_overlap.py <kernel_trace.csv> [--rccl-api rccl_api_trace.csv] [--step-kernel REGEX]
                        [--out file.md] [--max-rows 40]

With ``--rccl-api`` (rocprofv3 ``--rccl-trace``) it also places every ncclAllReduce CALL
inside its training step: which host thread issued it (the autograd engine thread = from a
gradient hook, mid-backward) and how much of that step's compute-stream kernel time still
ran after the call (work the reduction can overlap).  At world size 1 RCCL launches no
kernel for an in-place all-reduce, so the API trace is the evidence there.
"""
import argparse
import csv
import re
from collections import defaultdict

RCCL = re.compile(r"nccl|rccl", re.I)


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-rows", type=int, default=40)
    ap.add_argument("--rccl-api", default=None)
    ap.add_argument("--step-kernel", default=r"adam_kernel|sgd_kernel",
                    help="kernel name regex marking each step's optimizer (step boundary)")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        name = _col(r, "Kernel_Name", "KernelName", "Name")
        q = _col(r, "Stream_Id", "Queue_Id")
        rows.append((int(_col(r, "Start_Timestamp", "BeginNs")), int(_col(r, "End_Timestamp", "EndNs")), q, name))
    rows.sort()
    comm = [x for x in rows if RCCL.search(x[3])]
    other = [x for x in rows if not RCCL.search(x[3])]
    streams = defaultdict(int)
    for x in rows:
        streams[(x[2], bool(RCCL.search(x[3])))] += 1
    lines = [f"# RCCL / compute overlap: {a.csv}", "",
             f"kernels: {len(rows)}, RCCL kernels: {len(comm)}", "",
             "| stream/queue | RCCL kernels | other kernels |", "|---|---|---|"]
    for q in sorted({k[0] for k in streams}, key=str):
        lines.append(f"| {q} | {streams[(q, True)]} | {streams[(q, False)]} |")
    # overlap: for each RCCL kernel, time covered by kernels of other streams during its lifetime
    tot_comm = tot_ov = 0
    detail = []
    j0 = 0
    for (s, e, q, n) in comm:
        while j0 < len(other) and other[j0][1] < s:
            j0 += 1
        cov = []
        j = j0
        while j < len(other) and other[j][0] < e:
            os_, oe, oq, on = other[j]
            if oq != q and oe > s:
                cov.append((max(s, os_), min(e, oe), on))
            j += 1
        # union of covered intervals
        cov.sort()
        u, cur = 0, None
        for cs, ce, _ in cov:
            if cur is None or cs > cur[1]:
                if cur:
                    u += cur[1] - cur[0]
                cur = [cs, ce]
            else:
                cur[1] = max(cur[1], ce)
        if cur:
            u += cur[1] - cur[0]
        tot_comm += e - s
        tot_ov += u
        detail.append((s, e - s, q, u, len(cov), cov[0][2] if cov else "-", n))
    lines += ["", f"RCCL kernel time: {tot_comm / 1e6:.3f} ms; overlapped by other-stream kernels: "
              f"{tot_ov / 1e6:.3f} ms ({100.0 * tot_ov / max(tot_comm, 1):.1f}%)", "",
              f"## first {a.max_rows} RCCL kernels", "",
              "| t (ms from first) | dur us | stream | overlapped us | concurrent kernels | e.g. | RCCL kernel |",
              "|---|---|---|---|---|---|---|"]
    t0 = rows[0][0] if rows else 0
    for s, d, q, u, k, ex, n in detail[:a.max_rows]:
        ex = ex if len(ex) < 50 else ex[:47] + "..."
        n = n if len(n) < 50 else n[:47] + "..."
        lines.append(f"| {(s - t0) / 1e6:.3f} | {d / 1e3:.1f} | {q} | {u / 1e3:.1f} | {k} | `{ex}` | `{n}` |")
    if a.rccl_api:
        lines += _api_section(a, rows)
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


def _api_section(a, rows):
    calls = []
    for r in csv.DictReader(open(a.rccl_api)):
        calls.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r["Thread_Id"]))
    main_tid = min((c[3] for c in calls), key=lambda t: int(t)) if calls else None
    ar = sorted(c for c in calls if c[2] in ("ncclAllReduce", "ncclReduceScatter", "ncclAllGather"))
    step_pat = re.compile(a.step_kernel)
    # step boundaries: first optimizer kernel after a gap of non-optimizer kernels
    bounds, prev_opt = [], False
    for s_, e_, q, n in rows:
        is_opt = bool(step_pat.search(n))
        if is_opt and not prev_opt:
            bounds.append(s_)
        prev_opt = is_opt
    comp = [(s_, e_) for s_, e_, q, n in rows if q == "0" and not RCCL.search(n)]
    out = ["", "## RCCL calls inside the training steps (rccl API trace)", "",
           f"collective calls: {len(ar)}; issuing threads: "
           + ", ".join(f"{t} ({'main' if t == main_tid else 'autograd/hook'}): {sum(1 for c in ar if c[3] == t)}"
                       for t in sorted({c[3] for c in ar}))]
    rows_md = ["", "| step | calls | from hook thread | median compute after call (ms) | step compute (ms) |",
               "|---|---|---|---|---|"]
    lo = 0
    for k, b in enumerate(bounds):
        sc = [c for c in ar if lo <= c[0] < b]
        if sc:
            win = [(s_, e_) for s_, e_ in comp if lo <= s_ < b]
            tot = sum(e_ - s_ for s_, e_ in win)
            after = sorted(sum(e_ - max(s_, c[0]) for s_, e_ in win if e_ > c[0]) for c in sc)
            med = after[len(after) // 2]
            hook = sum(1 for c in sc if c[3] != main_tid)
            rows_md.append(f"| {k} | {len(sc)} | {hook} | {med / 1e6:.2f} | {tot / 1e6:.2f} |")
        lo = b
    return out + rows_md


if __name__ == "__main__":
    main()
