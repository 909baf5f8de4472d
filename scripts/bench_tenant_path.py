"""Service-level MI355X path: events/s through a ``gpu-columnar`` tenant of a whole co-located instance.

raw payload batches (the ``event-source-raw-payloads`` record format) -> inbound-processing GPU tenant
engine (decode, validate, dedup, persist, state, zone rules on the MI355X, block encode) -> durable
batch -> event-management segment store (fdatasync'd before the raw offset commits) +
``inbound-enriched-batches`` topic; rejected payloads routed per payload to the unregistered /
registration topics.  Devices and assignments are created through the device-management API and
mirrored into the engine by the change feed.  Every timed batch carries fresh alternate ids
(``--alt-ids``), so dedup does real work and nothing is dropped as a replay.

    python scripts/bench_tenant_path.py --devices 20000 --batch 65536 --batches 40
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


class _StackSampler:
    """SW_SAMPLE_STACKS=1: every 2 ms, the innermost frames of every Python thread (a sampling
    profiler without extra packages); the report goes to stderr, busiest (thread, frames) first."""

    IDLE = {"wait", "get", "_wait_for_tstate_lock", "select", "poll", "sleep", "accept", "recv", "_worker"}

    def __init__(self, period_s: float = 0.002, depth: int = 4):
        import collections
        import threading
        self.counts = collections.Counter()
        self.samples = 0
        self._stop = threading.Event()
        self._depth = depth
        self._t = threading.Thread(target=self._run, args=(period_s,), daemon=True)
        self._t.start()

    def _run(self, period_s):
        import threading
        me = threading.get_ident()
        names = {}
        while not self._stop.wait(period_s):
            names.update({t.ident: t.name for t in threading.enumerate()})
            for tid, f in sys._current_frames().items():
                if tid == me:
                    continue
                if f.f_code.co_name in self.IDLE:
                    continue                  # a thread waiting (lock, queue, event, sleep)
                stack = []
                while f is not None and len(stack) < self._depth:
                    stack.append(f"{os.path.basename(f.f_code.co_filename)}:{f.f_code.co_name}:{f.f_lineno}")
                    f = f.f_back
                self.counts[(names.get(tid, str(tid)), " < ".join(stack))] += 1
            self.samples += 1

    def report(self, top: int = 40):
        self._stop.set()
        self._t.join()
        print(f"stack samples: {self.samples}", file=sys.stderr)
        for (name, stack), n in self.counts.most_common(top):
            print(f"{n:6d} {100.0 * n / max(1, self.samples):5.1f}% [{name}] {stack}", file=sys.stderr)
        print("(share of samples in which that thread sat in that code; waiting threads are left out)", file=sys.stderr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", type=int, default=20000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--max-msgs", type=int, default=0, help="engine batch capacity override (0 = template)")
    ap.add_argument("--via-bus", action="store_true",
                    help="publish the batches to the tenant's raw-payload topic (zero-copy pinned records, as "
                         "event sources do) and time until the raw consumer has stored and committed them all")
    ap.add_argument("--zero-copy", action=argparse.BooleanOptionalAction, default=False,
                    help="frame columnar payloads around the rows in the engine's pinned buffers (zeroCopyRows)")
    ap.add_argument("--gc", choices=["default", "freeze"], default="default",
                    help="freeze: gc.freeze() the heap once the devices are loaded; default: leave the collector alone")
    ap.add_argument("--template", default="gpu-columnar", help="tenant template (gpu-memory: volatile store)")
    ap.add_argument("--alt-ids", action=argparse.BooleanOptionalAction, default=True)
    ap.add_argument("--p-unregistered", type=float, default=0.0, help="share of payloads from unknown devices")
    ap.add_argument("--p-register", type=float, default=0.0)
    ap.add_argument("--p-ack", type=float, default=0.0)
    ap.add_argument("--store-retention", type=int, default=0,
                    help="rows the columnar event store holds (0 = the template's); older batches are evicted "
                         "and their memory reused -- a store that only grows page-faults fresh memory per batch")
    args = ap.parse_args()
    import logging
    logging.basicConfig(level=logging.ERROR)
    import numpy as np

    from sitewhere_amd.assembly import SiteWhereInstance
    # a fresh data directory per run: a durable store left by an earlier run would be resumed
    # (its alternate ids seed the dedup filter, so the same synthetic batches read as replays)
    if not os.environ.get("SITEWHERE_DATA_DIR"):
        import tempfile
        os.environ["SITEWHERE_DATA_DIR"] = tempfile.mkdtemp(prefix="sw-tenant-bench-")
    from sitewhere_amd.pipeline.fleet import FleetSpec, gen_payloads

    numa_node = None
    if os.environ.get("SW_NUMA_BIND", "1") != "0":
        import torch
        if torch.cuda.is_available():   # the instance's threads and pinned pools next to the GPU
            from sitewhere_amd.utils.numa import bind_to_gpu_node
            numa_node = bind_to_gpu_node(0)
    sw = SiteWhereInstance().start()
    sw.wait_for_tenant("default", 60)
    tm = sw.api("TenantManagement")
    sw.instance.system_user.run(lambda: tm.create_tenant({"token": "fast", "name": "fast",
                                                          "configurationTemplateId": args.template,
                                                          "datasetTemplateId": "empty"}))
    sw.wait_for_tenant("fast", 120)
    if args.max_msgs or args.zero_copy:
        from sitewhere_amd.runtime.config import dump_document
        ms = sw["inbound-processing"]
        before = ms.get_tenant_engine("fast")
        cfg = dict(before.config)
        if args.max_msgs:
            cfg["capacity"] = dict(cfg.get("capacity", {}), max_msgs=args.max_msgs)
        cfg["zeroCopyRows"] = bool(args.zero_copy)
        sw.instance.coord.put(ms.tenant_config_path("fast"), dump_document(cfg))
        while ms.get_tenant_engine("fast") in (None, before) or ms.get_tenant_engine("fast").status.value != "Started":
            time.sleep(0.1)
    if args.store_retention and hasattr(sw.tenant_engine("event-management", "fast").store, "retention_rows"):
        # the same window on the enriched-batch topic, which references the same batch payloads
        sw.tenant_engine("event-management", "fast").store.retention_rows = args.store_retention
        t_out = sw.instance.naming.tenant_prefix("fast") + "inbound-enriched-batches"
        sw.instance.bus.topic(t_out)
        sw.instance.bus.set_retention(t_out, 32 * args.store_retention)
    run = lambda f: sw.instance.system_user.run(f, "fast")  # noqa: E731
    dm = sw.api("DeviceManagement", "fast")
    t0 = time.time()
    run(lambda: dm.create_device_type({"token": "sensor", "name": "Sensor"}))
    for i in range(args.devices):
        tok = f"dev-{i:010d}"
        run(lambda tok=tok: dm.create_device({"token": tok, "deviceTypeToken": "sensor"}))
        run(lambda tok=tok: dm.create_device_assignment({"deviceToken": tok}))
    ib = sw.tenant_engine("inbound-processing", "fast")
    while ib.engine.n_assignments < args.devices and time.time() - t0 < 600:
        time.sleep(0.1)
    setup_s = time.time() - t0
    from sitewhere_amd.pipeline.fleet import stamp_alt_epoch
    spec = FleetSpec(prefix="dev-", n_devices=args.devices, p_location=0.25, p_alert=0.05, mx_per_msg=1,
                     with_alternate_id=args.alt_ids, p_unregistered=args.p_unregistered, p_register=args.p_register,
                     p_ack=args.p_ack)
    now0 = int(time.time() * 1000)
    batches = []
    for b in range(4):
        raw, offs = gen_payloads(spec, args.batch, now0 - 1000, seed=7 + b)
        batches.append((np.concatenate([raw, np.zeros(64, np.uint8)]), offs))
    n_total = args.warmup + args.batches
    if args.alt_ids:
        # every batch its own alternate ids (stamped before the clock starts): cycling the 4
        # generated batches would otherwise make every batch after the 4th a set of duplicates
        base = batches
        batches = []
        for k in range(n_total):
            raw = base[k % 4][0].copy()
            stamp_alt_epoch(raw, base[k % 4][1], (0x7E17 << 48) | k)
            batches.append((raw, base[k % 4][1]))
    if args.gc == "freeze":
        import gc
        gc.collect()
        gc.freeze()                         # start-up objects leave the collector's generations
        gc.set_threshold(50_000, 20, 100)
    if args.via_bus:
        from sitewhere_amd.pipeline.bus_io import RawBatchRecord
        from sitewhere_amd.pipeline.framing import varint_lengths
        bus = sw.instance.bus
        t_raw = sw.instance.naming.tenant_prefix("fast") + "event-source-raw-payloads"
        import torch
        pin = torch.cuda.is_available()
        recs = [RawBatchRecord(r[:int(o[-1])], varint_lengths(o), len(o) - 1, pinned=pin) for r, o in batches]
        parts = bus.partitions(t_raw)

        def pump(n, k0):
            start = {p: bus.end_offset(t_raw, p) for p in range(parts)}
            for k in range(n):
                recs[(k0 + k) % len(recs)].publish(bus, t_raw, (k0 + k) % parts, ts=now0 + k0 + k)
            end = {p: bus.end_offset(t_raw, p) for p in range(parts)}
            while any(bus.committed(ib.raw_consumer.group, t_raw, p) < end[p] for p in range(parts)
                      if end[p] > start[p]):
                time.sleep(0.0005)
        pump(args.warmup, 0)
        ib.flush()
        base = ib.persisted_events.count
        ev0 = ib.processed_events.count
        sampler = _StackSampler() if os.environ.get("SW_SAMPLE_STACKS") == "1" else None
        t = t_timed = time.perf_counter()
        pump(args.batches, args.warmup)
        dt = time.perf_counter() - t
        if sampler is not None:
            sampler.report()
        ev = ib.processed_events.count - ev0
    else:
        for k in range(args.warmup):
            ib.process_batch(*batches[k % len(batches)])
        ib.flush()
        base = ib.persisted_events.count
        t = t_timed = time.perf_counter()
        ev = 0
        for k in range(args.batches):
            r = ib.process_batch(*batches[(args.warmup + k) % len(batches)])
            ev += r.n_events
        ib.flush()
        dt = time.perf_counter() - t
    em_store = sw.tenant_engine("event-management", "fast").store
    if os.environ.get("SW_PIN_REFERRERS") == "1":         # diagnostic: who holds the pooled row buffers
        import gc
        import sys as _sys
        for _pin, arr in getattr(ib.engine, "_pin_pool", [])[:3]:
            refs = gc.get_referrers(arr)
            print("pool buffer refcount", _sys.getrefcount(arr), [
                (type(r).__name__, getattr(r, "shape", None), str(type(getattr(r, "base", None)).__name__))
                for r in refs][:12], file=sys.stderr)
            for r in refs:
                if type(r).__name__ == "ndarray":
                    print("  view referrers:", [type(x).__name__ + ":" + str(x)[:60] for x in gc.get_referrers(r)
                                                if not isinstance(x, list) or len(x) < 50][:8], file=sys.stderr)
    trace = None
    if ib.trace:                # SW_TENANT_TRACE=1: medians over the second half of the timed batches
        # steps submitted inside the timed window only (warmup steps and the first step's set-up
        # are outside it); medians over its second half, the interval tail over all of it
        timed = [x for x in ib.trace if len(x) == 9 and x[0] >= t_timed]
        tr = timed[len(timed) // 2:]
        if tr:
            import numpy as np
            d = np.diff(np.asarray(tr), axis=1) * 1000
            gap = np.diff(np.asarray([x[0] for x in timed])) * 1000
            trace = {"submit_ms": d[:, 0], "to_complete_ms": d[:, 1], "queue_wait_ms": d[:, 2],
                     "payload_lock_ms": d[:, 3], "payload_dicts_ms": d[:, 4], "payload_encode_ms": d[:, 5],
                     "rpc_ms": d[:, 6], "publish_commit_ms": d[:, 7], "submit_interval_ms": gap}
            gap_pct = {f"submit_interval_p{q}_ms": round(float(np.percentile(gap, q)), 3) for q in (90, 99)} \
                if len(gap) else {}
            if len(gap):
                gap_pct["submit_interval_max_ms"] = round(float(gap.max()), 3)
                gap_pct["timed_steps"] = len(timed)
            trace = {k: round(float(np.median(v)), 3) for k, v in trace.items() if len(v)}
            trace.update(gap_pct)
    breakdown = {name: round(t.hist.snapshot()["mean"], 3)
                 for name, t in (("engine_step_ms", ib.step_timer), ("columnar_store_ms", ib.store_timer),
                                 ("publish_ms", ib.publish_timer), ("recheck_ms", ib.recheck_timer))}
    breakdown["recheck_max_ms"] = round(ib.recheck_timer.hist.snapshot()["max"], 3)
    breakdown["engine_step_max_ms"] = round(ib.step_timer.hist.snapshot()["max"], 3)
    print(json.dumps({"metric": "tenant_path_events_per_sec", "engine": ib.engine_kind, "via_bus": args.via_bus,
                      "gc": args.gc, "zero_copy_rows": ib.zero_copy_rows,
                      "payloads_framed": ib.zc_framed, "payloads_copied": ib.zc_copied,
                      "pinned_rows": getattr(ib.engine, "pin_stats", None),
                      "pinned_blocks": getattr(ib.engine, "pin_stats_blocks", None),
                      "framed_trace_ms_per_batch": {k: round(1000 * v / (args.warmup + args.batches), 3)
                                                    for k, v in (getattr(ib.engine, "framed_trace", None) or {}).items()},
                      "overlap_steps": ib.overlap,
                      "events": ev,
                      "events_per_sec": round(ev / dt, 1), "persisted": ib.persisted_events.count - base,
                      "ms_per_batch": round(1000 * dt / args.batches, 3), "batch": args.batch,
                      "engine_steps": ib.step_timer.count,
                      "devices": args.devices, "store_rows": getattr(em_store, "rows", None), "template": args.template,
                      "store": type(em_store).__name__,
                      "store_disk": em_store.seg.stats() if hasattr(em_store, "seg") else None,
                      "alt_ids": args.alt_ids, "p_unregistered": args.p_unregistered,
                      "duplicates": ib.engine.stats_dict().get("duplicates"),
                      "routed_payloads": ib.routed_payloads, "unregistered": ib.unregistered.count,
                      "raw_records_lost": getattr(ib.raw_consumer.consumer, "lost", None),
                      "backpressure_waits": getattr(sw.instance.bus, "backpressure_waits", None),
                      "numa_node": numa_node,
                      "store_retention_rows": getattr(em_store, "retention_rows", None),
                      "store_evicted_rows": getattr(em_store, "evicted_rows", None), "setup_s": round(setup_s, 1),
                      "mean_ms": breakdown, **({"median_ms_second_half": trace} if trace else {})}))
    sw.stop()


if __name__ == "__main__":
    main()
