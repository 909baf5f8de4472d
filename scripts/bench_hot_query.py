"""Hot-store event queries (the read side of event management) over a full HBM event ring.

Fills a 2^27-event ring on the MI355X with the bench.py fleet, then times ``query_store`` --
``list*ForIndex`` for one assignment, 1,000 assignments and one customer (~1/97 of the fleet), each
as page 1 of 100, newest first -- on the GPU (one k_store_filter pass + device ordering) and, for
the same store contents, with the numpy path the CPU engines use.

    python scripts/bench_hot_query.py --store 134217728
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--store", type=int, default=1 << 27)
    ap.add_argument("--devices", type=int, default=1 << 20)
    ap.add_argument("--msgs", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cpu", action="store_true", help="also time the numpy query on a host copy of the ring")
    args = ap.parse_args()
    import torch

    from sitewhere_amd.models.columnar import EV_LOCATION, EV_MEASUREMENT
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.cpu_engine import CpuInboundEngine
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine

    cfg = EngineConfig(max_msgs=args.msgs, rec_cap=args.msgs + 4096, max_devices=int(args.devices * 1.1) + 1024,
                       max_assignments=int(args.devices * 1.1) + 1024, store_cap=args.store, dedup_slots=1 << 20,
                       name_slots=1 << 12, state_slots=2 * 20 * int(args.devices * 1.1))
    g = GpuInboundEngine(cfg)
    heap, offs = gen_tokens("dev-", 0, args.devices)
    lo, hi = fingerprints(heap, offs)
    d = g.register_devices(lo, hi)
    g.set_assignments(d, d, customer=d % 97, area=d % 31, asset=d % 1009)
    spec = FleetSpec(prefix="dev-", n_devices=args.devices, p_location=0.25, p_alert=0.05, mx_per_msg=1, n_names=16)
    now0 = int(time.time() * 1000)
    batches = []
    for b in range(4):
        raw, o = gen_payloads(spec, args.msgs, now0 - 3_600_000, seed=100 + b)
        batches.append((np.concatenate([raw, np.zeros(64, np.uint8)]), o))
    t0 = time.time()
    k = 0
    while g.cursor < args.store + args.msgs:              # fill and wrap the ring once
        raw, o = batches[k % 4]
        g.step(raw, o, now0 + k, presence=False)
        k += 1
    fill_s = time.time() - t0
    rng = np.random.default_rng(5)
    one = [int(rng.integers(0, args.devices))]
    thousand = rng.choice(args.devices, 1000, replace=False).tolist()
    customer = np.nonzero(d % 97 == 13)[0].tolist()
    queries = {"1 assignment": (EV_MEASUREMENT, one), "1000 assignments": (EV_MEASUREMENT, thousand),
               "1 customer (~10.8K assignments)": (EV_LOCATION, customer)}
    out = {"store_events": int(min(g.cursor, args.store)), "fill_s": round(fill_s, 1), "queries": {}}
    for name, (et, asg) in queries.items():
        g.query_store(et, asg, page_size=100)             # warm (bitmap / buffers)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            s = time.perf_counter()
            total, _, _ = g.query_store(et, asg, page_size=100)
            ts.append(1000 * (time.perf_counter() - s))
        out["queries"][name] = {"matches": int(total), "gpu_ms_p50": round(float(np.median(ts)), 3),
                                "gpu_ms_min": round(float(np.min(ts)), 3)}
    if args.cpu:
        c = CpuInboundEngine.__new__(CpuInboundEngine)       # numpy query over a host copy of the same ring
        c.cfg, c.cursor, c.world, c.rank = cfg, g.cursor, 1, 0
        c.store = {k2: v.cpu().numpy() for k2, v in g.store.items()}
        for name, (et, asg) in queries.items():
            s = time.perf_counter()
            total, _, _ = c.query_store(et, asg, page_size=100)
            out["queries"][name]["cpu_numpy_ms"] = round(1000 * (time.perf_counter() - s), 1)
            assert total == out["queries"][name]["matches"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
