"""Where the block index build spends its time: one bench-shape step (1M payloads, 1M devices, 97
customers / 31 areas / 1009 assets) with the heads kernel's s_memrealtime stamps on (100 MHz), per
chunk [start, items loaded, heads selected, done].  Prints one JSON line: the kernel span, the
per-phase time distributions and how the chunks' start times spread over the span."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pct(x, q):
    return round(float(np.percentile(x, q)), 2) if len(x) else None


def main():
    import torch
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    n_dev = 1 << 20
    cfg = EngineConfig(max_msgs=1 << 20, rec_cap=(1 << 20) + 4096, gen_cap=1 << 19, max_devices=n_dev + 4096,
                       max_assignments=n_dev + 4096, store_cap=1 << 23, dedup_slots=1 << 22, name_slots=1 << 12,
                       state_slots=1 << 24)
    g = GpuInboundEngine(cfg, device="cuda:0")
    heap, offs = gen_tokens("dev-", 0, n_dev)
    lo, hi = fingerprints(heap, offs)
    d = g.register_devices(lo, hi)
    g.set_assignments(d, d, customer=d % 97, area=d % 31, asset=d % 1009)
    words = int(g.lib.sw_seg_index_stamp_words(g.out_cap))
    g.ix_stamps = torch.zeros(words, dtype=torch.int64, device="cuda:0")
    spec = FleetSpec(prefix="dev-", n_devices=n_dev, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.1)
    now = int(time.time() * 1000)
    out = {}
    for k in range(3):
        raw, off = gen_payloads(spec, 1 << 20, now - 30_000, seed=7 + k)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        res = g.step(raw, off, now + k, presence=False)
        g.ix_stamps.zero_()
        t0 = time.perf_counter()
        g.encode_block(now + k, res, boot=1)
        out["encode_block_ms"] = round(1000 * (time.perf_counter() - t0), 3)
    st = g.ix_stamps.cpu().numpy().reshape(-1, 4)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    us = lambda x: (x.astype(np.float64)) / 100.0      # noqa: E731  (100 MHz ticks -> us)
    start = us(st[:, 0] - t0)
    load = us(st[:, 1] - st[:, 0])
    sel = us(st[:, 2] - st[:, 1])
    rest = us(st[:, 3] - st[:, 2])
    total = us(st[:, 3] - st[:, 0])
    out.update({
        "chunks": int(len(st)),
        "span_us": round(float(us(st[:, 3].max() - t0)), 2),
        "chunk_us": {"p50": pct(total, 50), "p90": pct(total, 90), "p99": pct(total, 99), "max": pct(total, 100)},
        "load_us": {"p50": pct(load, 50), "p99": pct(load, 99)},
        "select_us": {"p50": pct(sel, 50), "p99": pct(sel, 99)},
        "write_merge_us": {"p50": pct(rest, 50), "p99": pct(rest, 99), "max": pct(rest, 100)},
        "start_us": {"p10": pct(start, 10), "p50": pct(start, 50), "p90": pct(start, 90), "max": pct(start, 100)},
    })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
