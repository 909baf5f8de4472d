"""Summarise a rocprofv3 kernel profile into a markdown table (top kernels, per-step time).

    python scripts/summarize_prof.py gpurun_out/full/prof/run_kernel_stats.csv --steps 13 > top_kernels.md
    python scripts/summarize_prof.py gpurun_out/full/prof/run_kernel_trace.csv > top_kernels.md

Given the per-dispatch trace (``*_kernel_trace.csv``) the table is split in two: one-time setup
(buffer allocation fills, registry upload, ...: every dispatch before the first engine step) and
the steady state, whose per-step column divides by the number of engine steps found in the trace
(dispatches of ``--step-kernel``).  The aggregate ``*_kernel_stats.csv`` cannot make that split,
so there the per-step column charges setup kernels to the steps too.
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    m = re.match(r"(?:void )?([\w:]+(?:<\d+)?)", name)
    s = (m.group(1) if m else name)
    f = re.search(r"at::native::(\w+Functor)<([\w ]+)>", name)      # torch fills: name the functor
    if f:
        s += f" {f.group(1)}<{f.group(2)}>"
    return s[:80]


def table(stats, steps=0, top=25):
    total = sum(t for _, t in stats.values())
    out = ["| kernel | calls | total us | avg us | % |" + (" us/step |" if steps else ""),
           "|---|---|---|---|---|" + ("---|" if steps else "")]
    for name, (calls, t) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:top]:
        line = f"| {name} | {calls} | {t / 1e3:.0f} | {t / 1e3 / calls:.1f} | {100 * t / max(total, 1):.1f} |"
        if steps:
            line += f" {t / 1e3 / steps:.1f} |"
        out.append(line)
    return out, total


def from_stats(path, steps, top):
    stats = {}
    for r in csv.DictReader(open(path)):
        c, t = stats.get(short(r["Name"]), (0, 0.0))
        stats[short(r["Name"])] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    lines, total = table(stats, steps, top)
    print("\n".join(lines))
    print(f"\nall kernels: {total / 1e6:.2f} ms over the run")


def from_trace(path, step_kernel, top):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = next((i for i, r in enumerate(rows) if step_kernel in r["Kernel_Name"]), len(rows))
    setup, steady = collections.defaultdict(lambda: [0, 0.0]), collections.defaultdict(lambda: [0, 0.0])
    steps = 0
    for i, r in enumerate(rows):
        d = (setup if i < first else steady)[short(r["Kernel_Name"])]
        d[0] += 1
        d[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        steps += i >= first and step_kernel in r["Kernel_Name"]
    lines, total = table({k: tuple(v) for k, v in steady.items()}, steps, top)
    print(f"## steady state: {steps} engine steps (from the first `{step_kernel}` dispatch)\n")
    print("\n".join(lines))
    print(f"\nsteady-state kernels: {total / 1e6:.2f} ms = {total / 1e3 / max(steps, 1):.1f} us/step\n")
    lines, total = table({k: tuple(v) for k, v in setup.items()}, 0, 10)
    print("## one-time setup (before the first step)\n")
    print("\n".join(lines))
    print(f"\nsetup kernels: {total / 1e6:.2f} ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="engine steps in the profiled run (stats csv only)")
    ap.add_argument("--step-kernel", default="k_decode_count", help="one dispatch of this kernel per engine step")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    with open(a.csv) as f:
        header = f.readline()
    if "Start_Timestamp" in header:
        from_trace(a.csv, a.step_kernel, a.top)
    else:
        from_stats(a.csv, a.steps, a.top)


if __name__ == "__main__":
    main()
