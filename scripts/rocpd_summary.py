"""Per-kernel summary of a rocprofv3 run database (rocpd SQLite: ``-d DIR -o NAME`` writes
``DIR/NAME_results.db``): calls, total / mean / max microseconds and share, sorted by total time,
plus dispatches per step when ``--steps`` is given.  Usage:
    python scripts/rocpd_summary.py gpurun_out/r4_prof/run_results.db [--steps 25] [--md out.md]"""
from __future__ import annotations

import argparse
import sqlite3


def summary(db_path: str):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, count(*), sum(duration), avg(duration), max(duration) from kernels "
                      "group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(r[0], r[1], r[2] / 1e3, r[3] / 1e3, r[4] / 1e3, 100.0 * r[2] / total) for r in rows], total / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0, help="steps in the run (warmup included)")
    ap.add_argument("--md", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows, total_us = summary(a.db)
    lines = ["| kernel | calls | total us | mean us | max us | % |", "|---|---:|---:|---:|---:|---:|"]
    for name, n, tot, mean, mx, pct in rows[:a.top]:
        short = name.split("(")[0][:70]
        lines.append(f"| `{short}` | {n} | {tot:.1f} | {mean:.2f} | {mx:.2f} | {pct:.1f} |")
    calls = sum(r[1] for r in rows)
    lines.append(f"\nkernel time {total_us:.1f} us in {calls} dispatches")
    if a.steps:
        lines.append(f"per step: {total_us / a.steps:.1f} us of kernels, {calls / a.steps:.1f} dispatches")
    text = "\n".join(lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
