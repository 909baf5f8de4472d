"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (top kernels, per-step time).

    python scripts/summarize_prof.py gpurun_out/full/prof/run_kernel_stats.csv --steps 13 > top_kernels.md
"""
import argparse
import csv
import re


def short(name: str) -> str:
    m = re.match(r"(?:void )?([\w:]+(?:<\d+)?)", name)
    return (m.group(1) if m else name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="engine steps in the profiled run (per-step column)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | total us | avg us | % |" + (" us/step |" if a.steps else ""))
    print("|---|---|---|---|---|" + ("---|" if a.steps else ""))
    for r in rows[:a.top]:
        t = float(r["TotalDurationNs"])
        line = (f"| {short(r['Name'])} | {r['Calls']} | {t / 1e3:.0f} | {float(r['AverageNs']) / 1e3:.1f} | "
                f"{100 * t / total:.1f} |")
        if a.steps:
            line += f" {t / 1e3 / a.steps:.1f} |"
        print(line)
    print(f"\nall kernels: {total / 1e6:.2f} ms over the run")


if __name__ == "__main__":
    main()
