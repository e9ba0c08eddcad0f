#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into categories + top kernels.

usage: prof_summary.py <kernel_stats.csv> [--steps N] [--out file.md]
"""
import argparse
import csv
import re
from collections import defaultdict

CATS = [
    ("madnn (hand-written HIP)", r"bucket_copy|flat_scale_cast|sgd_kernel|adam_kernel|sqnorm|norm_fwd|norm_bwd|"
                                 r"norm_wgrad|norm_finalize|bn_|madnn"),
    ("conv fwd (MIOpen igemm)", r"igemm_fwd|conv.*fwd|ConvFwd|naive_conv.*fwd"),
    ("conv bwd-data (MIOpen)", r"igemm_bwd|ConvBwd|naive_conv.*bwd"),
    ("conv bwd-weight (MIOpen)", r"igemm_wrw|ConvWrw|naive_conv.*wrw"),
    ("batchnorm (MIOpen)", r"BatchNorm"),
    ("GEMM (hipBLASLt/rocBLAS)", r"^Cijk_|^Custom_Cijk_|gemm|Gemm"),
    ("attention", r"attn|flash|fmha"),
    ("RCCL", r"ncclDevKernel|rccl|nccl"),
    ("elementwise / reduce (ATen)", r"elementwise|vectorized|reduce_kernel|unrolled|SubTensorOp|Op2d|Op1d"),
    ("memset / copy", r"fillBuffer|copyBuffer|Memcpy|memset"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=float, default=None, help="steps in the profiled region (for ms/step)")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    cat = defaultdict(float)
    calls = defaultdict(int)
    for r in rows:
        name = r["Name"]
        for c, pat in CATS:
            if re.search(pat, name):
                break
        else:
            c = "other"
        cat[c] += float(r["TotalDurationNs"])
        calls[c] += int(r["Calls"])
    lines = [f"# kernel time summary: {a.csv}", "", f"total GPU kernel time: {tot / 1e6:.2f} ms"
             + (f" ({tot / 1e6 / a.steps:.2f} ms/step over {a.steps:g} steps)" if a.steps else ""), "",
             "| category | ms | % | calls |", "|---|---|---|---|"]
    for c, v in sorted(cat.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {c} | {v / 1e6:.2f} | {100 * v / tot:.1f} | {calls[c]} |")
    lines += ["", f"## top {a.top} kernels", "", "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        n = r["Name"]
        n = n if len(n) < 90 else n[:87] + "..."
        lines.append(f"| `{n}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {100 * float(r['TotalDurationNs']) / tot:.1f} |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)


if __name__ == "__main__":
    main()
