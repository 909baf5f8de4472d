"""Compare two rocprofv3 kernel_stats.csv files: per-kernel average time, as a markdown table.

    python scripts/compare_kernel_stats.py A.csv B.csv [--top 20]
"""
import argparse
import csv


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        out[r["Name"].split("(")[0][:48]] = (int(r["Calls"]), float(r["AverageNs"]) / 1000, float(r["TotalDurationNs"]) / 1000)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=20)
    args = ap.parse_args()
    a, b = load(args.a), load(args.b)
    print("| kernel | calls A | A avg us | B avg us | change |")
    print("|---|---|---|---|---|")
    for k in sorted(a, key=lambda k: -a[k][2])[:args.top]:
        if k in b:
            print(f"| {k} | {a[k][0]} | {a[k][1]:.1f} | {b[k][1]:.1f} | {100 * (b[k][1] / a[k][1] - 1):+.1f}% |")
    print(f"\ntotal kernel time: A {sum(v[2] for v in a.values()) / 1000:.2f} ms, B {sum(v[2] for v in b.values()) / 1000:.2f} ms")


if __name__ == "__main__":
    main()
