"""Read latencies of a large durable event store (~1B events, ListMeasurementsForIndex
page 1 < 50 ms, GetById / GetByAlternateId < 10 ms).

Opens the segment directory a ``bench.py --durable-dir DIR --durable-retention-gb 0`` run left
behind (one rank's ``DIR/rank0``), builds the block indexes (postings by assignment + type,
alternate-id hashes; memory-mapped sidecars), then times, each over ``--queries`` random targets:
  * list_events(Measurement, Assignment, [one device's assignment], page 1 of 100)
  * get_event_by_id(random stored event)
  * get_event_by_alternate_id(the alternate id of a random stored event), and of an id never stored
Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(xs, q):
    return round(float(np.percentile(np.asarray(xs) * 1e3, q)), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--queries", type=int, default=50)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    from sitewhere_amd.persistence.segments import DurableEventStore
    t0 = time.perf_counter()
    st = DurableEventStore(a.dir, index=True, index_threads=a.threads)
    t_open = time.perf_counter() - t0
    ents = st.seg.index()
    ents = ents[ents["n_rows"] > 0]
    rows = int(ents["n_rows"].sum())
    t0 = time.perf_counter()
    ok = False
    while time.perf_counter() - t0 < 1800 and not ok:
        ok = st.index_wait(10)
        print(json.dumps({"progress": "indexing", "s": round(time.perf_counter() - t0, 1), **st.index_stats()}),
              file=sys.stderr, flush=True)
    t_index = time.perf_counter() - t0
    ixs = st.index_stats()
    rng = np.random.default_rng(11)
    boot = int(ents[0]["boot"])
    # dictionary entries for the assignments queried (bench.py registers only a few)
    asg_ids = [int(x) for x in rng.integers(0, 1 << 20, a.queries)]
    st.add_dictionary(boot, asg={i: [f"asg-{i}", f"dev-{i}", None, None, None] for i in asg_ids})
    lat = {"list_page1": [], "by_id": [], "by_alt": [], "by_alt_miss": []}
    found = []
    for i in asg_ids:
        t = time.perf_counter()
        r = st.list_events("Measurement", "Assignment", [f"asg-{i}"], DateRangeSearchCriteria(page_size=100))
        lat["list_page1"].append(time.perf_counter() - t)
        found.append(r.num_results)
    picks = []
    for _ in range(a.queries):
        e = ents[int(rng.integers(0, len(ents)))]
        row = int(rng.integers(0, int(e["n_rows"])))
        eid = (int(e["first_seq"]) + row) * int(e["world"]) + int(e["rank"])
        picks.append(f"{int(e['boot']):x}-{eid}")
    alts = []
    for id_ in picks:
        t = time.perf_counter()
        ev = st.get_event_by_id(id_)
        lat["by_id"].append(time.perf_counter() - t)
        assert ev is not None and ev.id == id_, id_
        if ev.alternate_id:
            alts.append((ev.alternate_id, id_))
    for alt, id_ in alts:
        t = time.perf_counter()
        ev = st.get_event_by_alternate_id(alt)
        lat["by_alt"].append(time.perf_counter() - t)
        assert ev is not None and ev.alternate_id == alt
    for k in range(min(20, a.queries)):
        t = time.perf_counter()
        assert st.get_event_by_alternate_id(f"never-stored-{k}") is None
        lat["by_alt_miss"].append(time.perf_counter() - t)
    out = {"bench": "store_reads", "events": rows, "blocks": len(ents), "open_s": round(t_open, 2),
           "index_build_s": round(t_index, 1), "indexed_all": ok, "index_bytes_per_event": round(ixs["index_bytes"] / max(1, rows), 2),
           "list_page1_results_mean": round(float(np.mean(found)), 1)}
    for k, v in lat.items():
        if v:
            out[k + "_ms"] = {"p50": pct(v, 50), "p99": pct(v, 99), "max": round(max(v) * 1e3, 3), "n": len(v)}
    print(json.dumps(out), flush=True)
    st.close()


if __name__ == "__main__":
    main()
