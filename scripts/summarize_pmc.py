"""Per-kernel HBM traffic and achieved bandwidth from rocprofv3 --pmc passes (scripts/gpu_pmc.sh).

FETCH_SIZE / WRITE_SIZE are in KB per dispatch; durations are the counter pass's own dispatch
timestamps.  SQ counters give waves and instruction mix.

    python scripts/summarize_pmc.py gpurun_out/pmc > profiles/r1_pmc/kernels.md
"""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?([\w:]+)", name)
    return (m.group(1) if m else name)[:40]


def load(path):
    rows = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(float)
    calls = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (r["Dispatch_Id"],)
        if key not in calls[k]:
            calls[k].add(key)
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return rows, dur, {k: len(v) for k, v in calls.items()}


def main():
    d = sys.argv[1]
    f, fd, fc = load(os.path.join(d, "fetch", "run_counter_collection.csv"))
    w, wd, _ = load(os.path.join(d, "write", "run_counter_collection.csv"))
    s, _, _ = load(os.path.join(d, "sq", "run_counter_collection.csv"))
    ks = sorted((k for k in f if k.startswith("k_")), key=lambda k: -fd[k])
    print("| kernel | calls | time us/call | read MB/call | write MB/call | achieved GB/s | waves/call | VALU/VMEM insts |")
    print("|---|---|---|---|---|---|---|---|")
    for k in ks:
        n = fc[k]
        rd = f[k]["FETCH_SIZE"] / 1024 / n
        wr = w.get(k, {}).get("WRITE_SIZE", 0.0) / 1024 / n
        t = (fd[k] + wd.get(k, fd[k])) / 2 / n
        bw = (rd + wr) / 1024 / t if t else 0.0
        sq = s.get(k, {})
        vm = sq.get("SQ_INSTS_VMEM_RD", 0) + sq.get("SQ_INSTS_VMEM_WR", 0)
        mix = f"{sq.get('SQ_INSTS_VALU', 0) / max(vm, 1):.1f}" if sq else "-"
        print(f"| {k} | {n} | {t * 1e6:.1f} | {rd:.2f} | {wr:.2f} | {bw:.0f} | {sq.get('SQ_WAVES', 0) / n:.0f} | {mix} |")


if __name__ == "__main__":
    main()
