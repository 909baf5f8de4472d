"""Read latencies of a durable event store: ListMeasurementsForIndex by Assignment
and by Area (page 1 of 100), GetDeviceEventById, GetDeviceEventByAlternateId (hit and miss).

Two modes:
  * ``--dir DIR``: open the segment directory a ``bench.py --durable-dir DIR --durable-retention-gb 0``
    run left behind (one rank's ``DIR/rank0``) and query it for ``--seconds`` (no ingest running).
  * reads while ingesting: ``bench.py --read-threads N`` runs the same query mix
    (``persistence/read_load.py``) against the store the bench is writing; see
    ``scripts/gpu_r5_reads.sh`` and ``profiles/r5_reads``.

Every block carries its index trailer (built on the GPU in the ingest step): there is nothing to
index after the fact.  Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--threads", type=int, default=1, help="reader threads")
    ap.add_argument("--devices", type=int, default=1 << 20, help="the bench fleet's assignments")
    a = ap.parse_args()
    from sitewhere_amd.persistence.read_load import ReadLoad, bench_dictionary
    from sitewhere_amd.persistence.segments import DurableEventStore
    t0 = time.perf_counter()
    st = DurableEventStore(a.dir)
    t_open = time.perf_counter() - t0
    ents = st.seg.index()
    boot = int(ents[0]["boot"]) if len(ents) else 0
    asg, ctx = bench_dictionary(a.devices)
    st.add_dictionary(boot, asg=asg, ctx=ctx)
    import gc
    gc.collect()
    gc.freeze()
    rl = ReadLoad(st, a.devices, threads=a.threads).start()
    time.sleep(a.seconds)
    out = {"bench": "store_reads", "events": int(ents["n_rows"].sum()), "blocks": int(len(ents)),
           "open_s": round(t_open, 2), **st.index_stats(), **rl.stop()}
    print(json.dumps(out), flush=True)
    st.close()


if __name__ == "__main__":
    main()
