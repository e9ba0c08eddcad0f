#!/usr/bin/env python3
"""Per-kernel table of rocprofv3 PMC counters (sums over dispatches) from one or more
counter_collection.csv files.  python scripts/pmc_table.py a.csv [b.csv ...] [--match substr]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    tab = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in a.csv:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")
                if a.match not in k:
                    continue
                k = k.split("(")[0][:70]
                tab[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((path, r.get("Dispatch_Id", "")))
    names = sorted({c for v in tab.values() for c in v})
    print("| kernel | " + " | ".join(names) + " |")
    print("|---|" + "---|" * len(names))
    for k, v in sorted(tab.items()):
        print(f"| `{k}` | " + " | ".join(f"{v.get(n, 0):.4g}" for n in names) + " |")


if __name__ == "__main__":
    main()
