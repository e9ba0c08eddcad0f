#!/usr/bin/env python3
"""Per-step view of a rocprofv3 kernel trace: split the dispatches into steps at a marker kernel
(the optimizer's update kernel ends every step), keep the last N steps, and print per-kernel time
per step (steady state: no first-use tuning, no MIOpen find).

usage: trace_steps.py <kernel_trace.csv> [--marker sgd_kernel] [--last 4] [--top 40] [--out f.md]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="sgd_kernel|adam_kernel")
    ap.add_argument("--last", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import re

    mk = re.compile(a.marker)
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if mk.search(r["Kernel_Name"])]
    # one step may launch several optimizer kernels back to back: keep the last of each run
    step_ends = [e for j, e in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != e + 1]
    if len(step_ends) < a.last + 1:
        raise SystemExit(f"only {len(step_ends)} steps found")
    lo, hi = step_ends[-a.last - 1] + 1, step_ends[-1] + 1
    sel = rows[lo:hi]
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e6 / a.last
    per = defaultdict(lambda: [0.0, 0])
    for r in sel:
        name = r["Kernel_Name"]
        per[name][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        per[name][1] += 1
    busy = sum(v[0] for v in per.values()) / 1e3 / a.last
    lines = [f"steady-state steps: last {a.last}; wall {wall:.2f} ms/step, kernel busy {busy:.2f} ms/step "
             f"({len(sel) // a.last} dispatches/step)", "",
             "| kernel | calls/step | us/step | avg us | % busy |", "|---|---|---|---|---|"]
    for name, (us, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[: a.top]:
        short = name if len(name) < 90 else name[:87] + "..."
        lines.append(f"| `{short}` | {n / a.last:g} | {us / a.last:.0f} | {us / n:.1f} | "
                     f"{100 * us / 1e3 / a.last / busy:.1f} |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
