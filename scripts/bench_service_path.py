"""Reference-architecture baseline (BASELINE.json config #1): events/s through the per-event
microservice path on CPU -- event sources decode -> decoded topic -> inbound processing (device +
assignment lookups) -> event management persist -> persisted topic -> enrichment -> enriched topic ->
device state.  Same machine, same wire payloads as bench.py, so the fused GPU engine's speedup over
the reference's design is measured rather than asserted.

    python scripts/bench_service_path.py --events 5000
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=5000)
    args = ap.parse_args()
    import logging
    logging.basicConfig(level=logging.ERROR)
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire

    sw = SiteWhereInstance().start()
    sw.wait_for_tenant("default", 60)
    es = sw.tenant_engine("event-sources")
    em_engine = sw.tenant_engine("event-management")
    ds_engine = sw.tenant_engine("device-state")
    tokens = [f"{t}-{i:03d}" for t in ("galaxytab", "meitrack", "raspberrypi", "iphone6s", "openhab") for i in range(4)]
    payloads = [wire.measurements(tokens[i % len(tokens)], {"m": float(i)}, event_date=1_700_000_000_000 + i)
                for i in range(args.events)]
    store = em_engine.store
    base = store.count() if hasattr(store, "count") else None
    t0 = time.perf_counter()
    for p in payloads:
        es.inject("default-protobuf", p)
    t_inj = time.perf_counter() - t0

    def persisted():
        return (store.count() - base) if base is not None else em_engine.management.store.stats().get("events", 0)

    while persisted() < args.events:
        time.sleep(0.01)
    t_persist = time.perf_counter() - t0
    while ds_engine.consumer.processed < args.events:
        time.sleep(0.01)
    t_state = time.perf_counter() - t0
    out = {"metric": "device_events_per_sec_reference_architecture_cpu", "events": args.events,
           "inject_s": round(t_inj, 3), "persisted_events_per_sec": round(args.events / t_persist, 1),
           "through_device_state_events_per_sec": round(args.events / t_state, 1),
           "path": "event-sources > decoded topic > inbound-processing > event-management > persisted topic > "
                   "enrichment > enriched topic > device-state (co-located, in-process bus)"}
    print(json.dumps(out))
    sw.stop()


if __name__ == "__main__":
    main()
