"""Per-kernel time difference between two rocprofv3 kernel_stats.csv files (A/B arms)."""
import collections
import csv
import sys


def load(p):
    d = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(p)):
        k = r["Name"][:100]
        d[k][0] += int(r["Calls"])
        d[k][1] += float(r["TotalDurationNs"]) / 1e6
    return d


def main():
    a, b = load(sys.argv[1]), load(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    print(f"total ms: A {sum(v[1] for v in a.values()):.2f}  B {sum(v[1] for v in b.values()):.2f}")
    z = [0, 0.0]
    for k in sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, z)[1] - a.get(k, z)[1]))[:top]:
        x, y = a.get(k, z), b.get(k, z)
        print(f"{y[1] - x[1]:8.2f} ms | A {x[0]:5d} calls {x[1]:8.2f} | B {y[0]:5d} calls {y[1]:8.2f} | {k}")


if __name__ == "__main__":
    main()
