"""Host-side cost of the durable store's queries (no GPU): fill a store with ``--blocks`` blocks of
the bench fleet shape from the native CPU engine (same block + trailer format the GPU writes), then
time and cProfile each query kind of persistence/read_load.py.  Prints one JSON line of latencies
and, with ``--profile KIND``, the top functions of that kind."""
from __future__ import annotations

import argparse
import cProfile
import json
import os
import pstats
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=200)
    ap.add_argument("--msgs", type=int, default=1 << 16)
    ap.add_argument("--devices", type=int, default=1 << 16)
    ap.add_argument("--queries", type=int, default=40)
    ap.add_argument("--profile", default="")
    ap.add_argument("--dir", default="")
    a = ap.parse_args()
    from sitewhere_amd.persistence.read_load import KINDS, ReadLoad, bench_dictionary
    from sitewhere_amd.persistence.segments import DurableEventStore
    from sitewhere_amd.pipeline.config import EngineConfig
    from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens
    from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
    d = a.dir or tempfile.mkdtemp(prefix="sw-q-")
    cfg = EngineConfig(max_msgs=a.msgs, rec_cap=a.msgs * 2, gen_cap=a.msgs, max_devices=a.devices + 1024,
                       max_assignments=a.devices + 1024, store_cap=1 << 20, dedup_slots=1 << 22,
                       name_slots=1 << 12, state_slots=1 << 20)
    eng = NativeCpuEngine(cfg)
    heap, offs = gen_tokens("dev-", 0, a.devices)
    lo, hi = fingerprints(heap, offs)
    dev = eng.register_devices(lo, hi)
    eng.set_assignments(dev, dev, customer=dev % 97, area=dev % 31, asset=dev % 1009)
    st = DurableEventStore(d, rotate_bytes=1 << 30)
    boot = 0x1700000000
    asg, ctx = bench_dictionary(a.devices)
    st.add_dictionary(boot, asg=asg, ctx=ctx)
    spec = FleetSpec(prefix="dev-", n_devices=a.devices, p_location=0.25, p_alert=0.05, p_unregistered=0.005,
                     with_alternate_id=True, lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.1)
    now = 1_700_000_000_000
    t0 = time.perf_counter()
    for b in range(a.blocks):
        raw, off = gen_payloads(spec, a.msgs, now + 1000 * b - 30_000, seed=b + 1)
        raw = np.concatenate([raw, np.zeros(64, np.uint8)])
        res = eng.step(raw, off, now + 1000 * b, presence=False)
        st.add_encoded(eng.encode_block(now + 1000 * b, res, boot=boot))
    st.flush()
    fill_s = time.perf_counter() - t0
    rl = ReadLoad(st, a.devices, threads=1)
    rng = np.random.default_rng(3)
    prof = cProfile.Profile() if a.profile else None
    for q in range(a.queries):
        for kind in KINDS:
            if prof is not None and kind == a.profile:
                prof.enable()
            got = rl._one(kind, rng)
            if prof is not None and kind == a.profile:
                prof.disable()
            if got is not None:
                rl.lat[kind].append(got[0])
                rl.results[kind].append(got[1])
    out = {"blocks": a.blocks, "rows": int(st.seg.index()["n_rows"].sum()), "fill_s": round(fill_s, 1), **rl.summary()}
    print(json.dumps(out), flush=True)
    if prof is not None:
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(25)
    st.close()


if __name__ == "__main__":
    main()
