"""Kernel dispatches of one steady-state engine step from a rocprofv3 database (``--kernel-trace``):
the sequence between two consecutive step starts (``k_vlen_tiles``, the varint framing that opens
every step of the bench), with each kernel's grid and time, and the per-step dispatch count.

    python scripts/step_dispatches.py gpurun_out/<run>_prof/run_results.db [--step 10]"""
from __future__ import annotations

import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=10, help="which step (0-based) to print")
    ap.add_argument("--first", default="k_vlen_tiles", help="kernel that opens a step")
    ap.add_argument("--stats", action="store_true",
                    help="instead: per-kernel totals over every complete steady-state step (from --step on)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, workgroup_x, duration / 1000.0, start from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if r[0].startswith(a.first)]
    if len(starts) < a.step + 2:
        raise SystemExit(f"only {len(starts)} steps in the trace")
    if a.stats:
        steps = [rows[starts[j]:starts[j + 1]] for j in range(a.step, len(starts) - 1)]
        agg: dict = {}
        for st in steps:
            for name, grid, wg, us, _ in st:
                k = name.split("(")[0]
                c_, t_, m_ = agg.get(k, (0, 0.0, 0.0))
                agg[k] = (c_ + 1, t_ + us, max(m_, us))
        tot = sum(v[1] for v in agg.values())
        n = len(steps)
        print(f"Steady-state engine steps {a.step}..{a.step + n - 1} ({n} steps) of the trace\n")
        print("| kernel | calls/step | us/step | mean us | max us | % |")
        print("|---|---:|---:|---:|---:|---:|")
        for k, (c_, t_, m_) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"| `{k}` | {c_ / n:.1f} | {t_ / n:.1f} | {t_ / c_:.1f} | {m_:.1f} | {100 * t_ / tot:.1f} |")
        print(f"\nkernel time per step: {tot / n:.1f} us; dispatches per step: {sum(v[0] for v in agg.values()) / n:.1f}")
        return
    i0, i1 = starts[a.step], starts[a.step + 1]
    step = rows[i0:i1]
    t0 = step[0][4]
    print("| # | kernel | workgroups | us | start us |")
    print("|---:|---|---:|---:|---:|")
    for k, (name, grid, wg, us, st) in enumerate(step):
        print(f"| {k + 1} | `{name.split('(')[0]}` | {grid // max(1, wg)} | {us:.1f} | {(st - t0) / 1000.0:.1f} |")
    span = (rows[i1][4] - t0) / 1000.0
    busy = sum(r[3] for r in step)
    counts = [starts[j + 1] - starts[j] for j in range(len(starts) - 1)]
    print(f"\n{len(step)} dispatches in step {a.step}; kernel time {busy:.1f} us of a {span:.1f} us step span; "
          f"dispatches per step over the run: min {min(counts)}, max {max(counts)}")


if __name__ == "__main__":
    main()
