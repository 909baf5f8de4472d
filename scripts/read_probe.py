"""Time listings against an existing bench store (``bench.py --durable-dir D``) on the host:
``python scripts/read_probe.py D/rank0 --n-customers 10000 --n-assets 0 [--kind list_customer]``.
Prints per-query latency and the store's phase split; ``--profile`` adds a cProfile of the queries."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--n-assignments", type=int, default=1 << 20)
    ap.add_argument("--n-customers", type=int, default=97)
    ap.add_argument("--n-areas", type=int, default=31)
    ap.add_argument("--n-assets", type=int, default=1009)
    ap.add_argument("--kind", default="list_customer")
    ap.add_argument("--queries", type=int, default=20)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from sitewhere_amd.persistence.read_load import ReadLoad, bench_dictionary
    from sitewhere_amd.persistence.segments import DurableEventStore, trailer_offset
    t0 = time.perf_counter()
    st = DurableEventStore(a.dir, rank=0)
    ents = st.seg.index()
    boots = sorted(set(int(b) for b in ents["boot"]))
    asg, ctx = bench_dictionary(a.n_assignments, a.n_customers, a.n_areas, a.n_assets)
    for b in boots:
        st.add_dictionary(b, asg=asg, ctx=ctx)
    blk = st.seg.read_block(ents[-1])
    print(json.dumps({"open_s": round(time.perf_counter() - t0, 2), "blocks": len(ents),
                      "rows": int(ents["n_rows"].sum()), "trailer": trailer_offset(blk) > 0}))
    rl = ReadLoad(st, a.n_assignments, n_area=a.n_areas, threads=1, n_cust=a.n_customers, n_asset=a.n_assets)
    rng = np.random.default_rng(3)
    rl._one(a.kind, rng)                                  # warm: block tables, trailers
    prof = None
    if a.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    lat, ph = [], []
    for _ in range(a.queries):
        dt, n = rl._one(a.kind, rng)
        lat.append(dt * 1e3)
        tl = getattr(st, "_tl", None)
        if tl is not None and getattr(tl, "phases", None):
            ph.append({k: round(v * 1e3, 2) for k, v in tl.phases.items()})
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("cumulative").print_stats(25)
    lat = np.array(lat)
    print(json.dumps({"kind": a.kind, "p50_ms": round(float(np.median(lat)), 2),
                      "p99_ms": round(float(np.percentile(lat, 99)), 2), "phases_first3": ph[:3]}))


if __name__ == "__main__":
    main()
