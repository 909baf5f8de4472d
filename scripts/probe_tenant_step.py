"""Where a synchronous tenant-engine step spends its time (GPU): H2D staging, launch, sync, collect.

    python scripts/probe_tenant_step.py --batch 65536 --batch 262144
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
    ap.add_argument("--batch", type=int, action="append")
    ap.add_argument("--devices", type=int, default=20000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--mapped", action="store_true", help="read rows from the mapped host buffer (old path)")
    args = ap.parse_args()
    import torch

    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    from sitewhere_amd.persistence.columnar import ColumnarEventStore, encode_batch

    batches = args.batch or [65536, 262144]
    cfg = EngineConfig(max_msgs=max(batches), max_devices=1 << 16, max_assignments=1 << 16, store_cap=1 << 24,
                       dedup_slots=1 << 20, name_slots=1 << 12, gen_cap=1 << 16)
    e = GpuInboundEngine(cfg)
    heap, offs = gen_tokens("dev-", 0, args.devices)
    lo, hi = fingerprints(heap, offs)
    d = e.register_devices(lo, hi)
    e.set_assignments(d, d, customer=d % 7, area=d % 5, asset=d % 3)
    spec = FleetSpec(prefix="dev-", n_devices=args.devices, p_location=0.25, p_alert=0.05, mx_per_msg=1)
    out = {}
    for b in batches:
        raw, o = gen_payloads(spec, b, int(time.time() * 1000) - 1000, seed=3)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        for _ in range(3):
            e.step(raw, o, int(time.time() * 1000))
        t = {"total": [], "h2d": [], "launch": [], "sync": [], "collect": [], "encode": [], "store_add": []}
        store = ColumnarEventStore()
        for _ in range(args.iters):
            now = int(time.time() * 1000)
            t0 = time.perf_counter()
            raw_dev, off_dev = e._stage(raw, o)
            t1 = time.perf_counter()
            sel = e.step_async(raw_dev, off_dev, len(o) - 1, now, presence=False, out_to_device=not args.mapped)
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            r = e.collect(sel, raw, from_device=not args.mapped)
            t4 = time.perf_counter()
            p = encode_batch("boot", r.first_seq, 1, 0, now, r.out, {}, {})
            t5 = time.perf_counter()
            store.add_columnar(p)
            t6 = time.perf_counter()
            for k, v in zip(t, (t6 - t0, t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
                t[k].append(1000 * v)
        out[b] = {k: round(float(np.median(v)), 3) for k, v in t.items()}
        out[b]["events_per_sec_engine_only"] = round(r.n_events / (out[b]["total"] - out[b]["encode"]
                                                                   - out[b]["store_add"]) * 1000, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
