#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench/kernels.py for madnn kernels.

usage: pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> [--out md]
FETCH_SIZE/WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports half the bytes of a
16-B/lane streaming read (MI355X_MICROARCH.md §HBM), so 2x FETCH is shown too.
"""
import argparse
import csv
import re
from collections import defaultdict


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or "madnn::" not in r["Kernel_Name"]:
            continue
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
        per[name].append((float(r["Counter_Value"]) * 1024, dur, int(r["Grid_Size"]), int(r["VGPR_Count"])))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out")
    a = ap.parse_args()
    f = load(a.fetch, "FETCH_SIZE")
    w = load(a.write, "WRITE_SIZE")
    lines = ["| kernel | dispatches | VGPRs | time/dispatch (us) | FETCH MB | 2xFETCH MB | WRITE MB | (2xFETCH+WRITE)/time GB/s |",
             "|---|---|---|---|---|---|---|---|"]
    for k in sorted(f, key=lambda k: -max(x[1] for x in f[k])):
        fe = max(f[k], key=lambda x: x[1])   # the largest (roofline) dispatch of this kernel
        wr = max(w.get(k, [(0, fe[1], 0, 0)]), key=lambda x: x[1])
        t = fe[1]
        lines.append(f"| `{k}` | {len(f[k])} | {fe[3]} | {t * 1e6:.1f} | {fe[0] / 1e6:.1f} | {2 * fe[0] / 1e6:.1f} | "
                     f"{wr[0] / 1e6:.1f} | {(2 * fe[0] + wr[0]) / t / 1e9:.0f} |")
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write("# madnn kernels: rocprofv3 PMC (FETCH_SIZE / WRITE_SIZE), bench/kernels.py, MI355X\n\n"
                               + txt)


if __name__ == "__main__":
    main()
