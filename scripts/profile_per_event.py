"""cProfile (per-thread CPU time, so GIL waits do not count) every thread of the in-process per-event pipeline (bench_reference_config.py,
``--path per-event --replicas 0``) and print the merged top functions.

    python scripts/profile_per_event.py --events 3000 --out /tmp/per_event_prof
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=3000)
    ap.add_argument("--out", default="/tmp/per_event_prof")
    ap.add_argument("--top", type=int, default=50)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    profs, lock = [], threading.Lock()

    def hook(*_):
        p = cProfile.Profile(time.thread_time)
        with lock:
            profs.append(p)
        sys.setprofile(None)
        p.enable()
    threading.setprofile(hook)
    main_p = cProfile.Profile(time.thread_time)
    profs.append(main_p)
    import bench_reference_config as b
    sys.argv = ["bench_reference_config.py", "--path", "per-event", "--replicas", "0", "--events", str(args.events),
                "--paced", "50"]
    main_p.enable()
    try:
        b.main()
    finally:
        threading.setprofile(None)
        st = None
        for p in list(profs):
            try:
                p.disable()
                p.create_stats()
            except Exception:
                continue
            if p.stats:
                st = pstats.Stats(p) if st is None else st.add(p)
        for key in ("tottime", "cumtime"):
            s = io.StringIO()
            st.stream = s
            st.sort_stats(key).print_stats(args.top)
            with open(os.path.join(args.out, f"{key}.txt"), "w") as f:
                f.write(s.getvalue())
        print(f"profiles written to {args.out}")


if __name__ == "__main__":
    main()
