"""Steady-state soak of an engine tenant through the bus.

A ``gpu-columnar-1m`` tenant of a whole co-located instance (1M devices and assignments, bulk
imported through device management) ingests for several phases of ``--phase-s`` seconds: a producer
publishes 1M-payload raw records (the event-sources record format, zero-copy pinned) to the tenant's
raw topic as fast as the tenant commits them, every record with FRESH alternate ids (a new id epoch
stamped in place natively, only into buffers whose records the tenant has committed) and 0.5% of
payloads from unregistered devices.  The tenant runs its real path: raw consumer -> MI355X engine
(decode, validation, window + store-backed dedup, persist, state, zones, block encode + index) ->
durable segment store (O_DIRECT, fdatasync before the raw offset commits), retention by rows bounded
to what the generational dedup filter holds.

Reported (one JSON line, plus a progress line every ~5 s): per phase events/s, the first and last
minute, submit-interval percentiles, dedup rechecks per payload, the filter's rotations against its
capacity, the store's retained / deleted rows (retention wraps), and a replay check at the end: a
sub-batch of a record published seconds before (still retained) is published again with the same
ids -- every valid event must come back a duplicate (filter recheck, settled against the store) and
the store must not grow.

    python scripts/soak_tenant.py --devices 1048576 --phases 3 --phase-s 70
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _trailer_diag(store, ib, lost) -> list:
    """For ids the store holds but its trailer lookup misses: the block holding each, the row and
    page, and what the block's in-memory trailer, its on-disk trailer and a CPU-rebuilt trailer
    each answer for the id (candidate pages)."""
    import ctypes
    import numpy as np
    from sitewhere_amd._native import native
    from sitewhere_amd.persistence import segments as sg
    from sitewhere_amd.pipeline.fleet import hash64
    lib = native()
    target = set(int(x) for x in lost[:64])
    out = []

    def pages_of(addr, h):
        bo, po = np.empty(64, np.int64), np.empty(64, np.int64)
        arr = (ctypes.c_void_p * 1)(addr)
        k = int(lib.swseg_ix_alt_pages(arr, 1, int(h), bo.ctypes.data, po.ctypes.data, 64))
        return po[:min(k, 64)].tolist()

    with store.seg.lease():
        tabs = store._boot_tables()
        for t in tabs.values():
            for bi in range(t["n"] - 1, -1, -1):
                if not target or len(out) >= 4:
                    break
                e = t["ents"][bi]
                hv = store._block_alt_hashes(e)
                hit = target & set(np.intersect1d(hv, np.array(sorted(target), np.uint64)).tolist())
                if not hit:
                    continue
                blk = store.seg.read_block(e)
                cols = sg.decode_block(blk, check=False)
                rows = {}
                for i in range(len(cols["date"])):
                    s = sg.row_strings(cols, i)[0]
                    if s is not None:
                        h = hash64(s)
                        if h in hit:
                            rows[h] = i
                toff = sg.trailer_offset(blk)
                disk_tr = np.ascontiguousarray(blk[toff:])
                mem_tr = t["tr"][bi]
                mem_bytes = np.asarray(mem_tr[3][:mem_tr[1]]) if mem_tr is not None and len(mem_tr) > 3 else None
                try:
                    ref = sg.index_block(_strip(blk), ib.engine.ctx_table())
                    cpu_tr = np.ascontiguousarray(ref[sg.trailer_offset(ref):])
                except Exception as ex:  # noqa: BLE001
                    cpu_tr = None
                    out.append({"cpu_rebuild_error": repr(ex)})
                d = {"block": int(bi), "of": int(t["n"]), "first_seq": int(e["first_seq"]), "n_rows": int(e["n_rows"]),
                     "hits": len(hit), "mem_equals_disk": None if mem_bytes is None else bool(np.array_equal(mem_bytes, disk_tr)),
                     "cpu_equals_disk": None if cpu_tr is None else bool(len(cpu_tr) == len(disk_tr) and np.array_equal(cpu_tr, disk_tr)),
                     "ids": []}
                if cpu_tr is not None and len(cpu_tr) == len(disk_tr):
                    diff = np.nonzero(cpu_tr != disk_tr)[0]
                    d["trailer_bytes_differ"] = int(len(diff))
                    d["first_diff"] = int(diff[0]) if len(diff) else None
                    hd = sg.parse_trailer(disk_tr)
                    d["trailer_sections"] = {k: int(hd[k]) for k in ("off_pages", "off_alt_dir", "off_alt", "n_alt",
                                                                      "alt_bits", "alt_pbits", "n_pages")}
                d["gpu_trailer"] = _tr_summary(disk_tr)
                if cpu_tr is not None:
                    d["cpu_trailer"] = _tr_summary(cpu_tr)
                    hg, hc = sg.parse_trailer(disk_tr), sg.parse_trailer(cpu_tr)
                    if int(hg["n_alt"]) == int(hc["n_alt"]) and int(hg["alt_bits"]) == int(hc["alt_bits"]):
                        nd = (1 << int(hg["alt_bits"])) + 1
                        dg = disk_tr[int(hg["off_alt_dir"]):int(hg["off_alt_dir"]) + 4 * nd].view(np.uint32)
                        dc = cpu_tr[int(hc["off_alt_dir"]):int(hc["off_alt_dir"]) + 4 * nd].view(np.uint32)
                        nw = (int(hg["n_alt"]) * 26 + 63) // 64
                        wg = np.frombuffer(disk_tr[int(hg["off_alt"]):int(hg["off_alt"]) + 8 * nw].tobytes(), np.uint64)
                        wc = np.frombuffer(cpu_tr[int(hc["off_alt"]):int(hc["off_alt"]) + 8 * nw].tobytes(), np.uint64)
                        bad = np.nonzero(wg != wc)[0]
                        d["alt_dir_differ"] = int((dg != dc).sum())
                        d["alt_words_differ"] = int(len(bad))
                        d["alt_words_first_last_bad"] = [int(bad[0]), int(bad[-1])] if len(bad) else None
                        pg_g, pg_c = sg.parse_trailer(disk_tr)["pages"], sg.parse_trailer(cpu_tr)["pages"]
                        d["pages_differ"] = int((pg_g != pg_c).sum()) if len(pg_g) == len(pg_c) else "len"
                for h in sorted(hit)[:6]:
                    r = rows.get(h)
                    d["ids"].append({"row": r, "page": None if r is None else r // sg.PAGE_ROWS,
                                     "disk": pages_of(disk_tr.ctypes.data, h),
                                     "mem": pages_of(int(mem_tr[0]), h) if mem_tr is not None else None,
                                     "cpu": pages_of(cpu_tr.ctypes.data, h) if cpu_tr is not None else None,
                                     "gpu_bucket": _bucket(disk_tr, h),
                                     "cpu_bucket": _bucket(cpu_tr, h) if cpu_tr is not None else None})
                out.append(d)
                target -= hit
    return out


def _tr_summary(tr) -> dict:
    from sitewhere_amd.persistence import segments as sg
    h = sg.parse_trailer(tr)
    return {k: (int(h[k]) if not hasattr(h[k], "__len__") else None) for k in
            ("n_rows", "n_pages", "n_alt", "alt_bits", "alt_pbits", "off_alt_dir", "off_alt", "bytes")}


def _bucket(tr, hv: int) -> dict:
    """The id's directory bucket in a trailer: its size and the (fingerprint, page) entries whose
    fingerprint is the id's."""
    import numpy as np
    from sitewhere_amd.persistence import segments as sg
    h = sg.parse_trailer(tr)
    bits, pb = int(h["alt_bits"]), int(h["alt_pbits"])
    EB = 26
    fb = EB - pb
    b = (hv >> (64 - bits)) if bits else 0
    want = (hv >> (64 - bits - fb)) & ((1 << fb) - 1)
    t = np.ascontiguousarray(tr)
    d0 = int(h["off_alt_dir"])
    dirs = t[d0:d0 + 4 * ((1 << bits) + 1)].view(np.uint32)
    lo, hi = int(dirs[b]), int(dirs[b + 1])
    words = t[int(h["off_alt"]):].view(np.uint64) if (len(t) - int(h["off_alt"])) % 8 == 0 else \
        np.frombuffer(t[int(h["off_alt"]):].tobytes() + b"\0" * 8, np.uint64)
    ents = []
    for e in range(lo, min(hi, int(h["n_alt"]))):
        bp = e * EB
        w0 = int(words[bp >> 6])
        sh = bp & 63
        v = w0 >> sh
        if sh + EB > 64:
            v |= int(words[(bp >> 6) + 1]) << (64 - sh)
        v &= (1 << EB) - 1
        ents.append((v >> pb, v & ((1 << pb) - 1)))
    return {"bucket": int(b), "size": hi - lo, "matches": [p for f, p in ents if f == want],
            "fps_sample": [f for f, _ in ents[:4]], "want_fp": int(want)}


def _strip(blk):
    """The block without its trailer (flag cleared, bytes = end of the pages, header re-sealed)."""
    from sitewhere_amd.persistence import segments as sg
    h = blk[:64].view(sg.HDR)[0]
    toff = sg.trailer_offset(blk)
    out = blk[:toff].copy()
    hv = out[:64].view(sg.HDR)
    hv["flags"] = 0
    hv["bytes"] = toff
    sg.seal(out, int(h["first_seq"]), int(h["recv_ms"]), int(h["boot"]), int(h["rank"]), int(h["world"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", type=int, default=1 << 20)
    ap.add_argument("--template", default="gpu-columnar-1m")
    ap.add_argument("--batch", type=int, default=1 << 20, help="payloads per raw record")
    ap.add_argument("--records", type=int, default=32, help="pinned raw records the producer cycles through")
    ap.add_argument("--ahead", type=int, default=28, help="records published ahead of the tenant's commits")
    ap.add_argument("--phases", type=int, default=3)
    ap.add_argument("--phase-s", type=float, default=70.0)
    ap.add_argument("--p-unregistered", type=float, default=0.005)
    ap.add_argument("--filter-ids", type=int, default=0, help="dedup filter ids per generation (0: template)")
    ap.add_argument("--replay", type=int, default=4096, help="payloads of the replayed sub-batch")
    ap.add_argument("--chunk", type=int, default=65536, help="devices per bulk import call")
    args = ap.parse_args()
    import logging
    logging.basicConfig(level=logging.ERROR)
    import numpy as np
    if not os.environ.get("SITEWHERE_DATA_DIR"):
        import tempfile
        os.environ["SITEWHERE_DATA_DIR"] = tempfile.mkdtemp(prefix="sw-soak-")
    data_dir = os.environ["SITEWHERE_DATA_DIR"]
    log("data dir", data_dir, "free GB", round(shutil.disk_usage(data_dir).free / 2 ** 30, 1))
    os.environ.setdefault("SW_TENANT_TRACE", "1")
    from sitewhere_amd.utils.stack_sampler import maybe_start
    maybe_start()                               # SW_STACK_SAMPLE=<prefix>: where the tenant's threads spend time
    import torch
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.pipeline.bus_io import VALUE_HDR, RawBatchRecord
    from sitewhere_amd.pipeline.fleet import FleetSpec, alt_positions, gen_payloads, stamp_alt_epoch, stamp_positions
    from sitewhere_amd.pipeline.framing import varint_lengths
    numa_node = None
    if torch.cuda.is_available() and os.environ.get("SW_NUMA_BIND", "1") != "0":
        from sitewhere_amd.utils.numa import bind_to_gpu_node
        numa_node = bind_to_gpu_node(0)
    t_setup = time.time()
    sw = SiteWhereInstance().start()
    sw.wait_for_tenant("default", 60)
    tm = sw.api("TenantManagement")
    sw.instance.system_user.run(lambda: tm.create_tenant({"token": "soak", "name": "soak",
                                                          "configurationTemplateId": args.template,
                                                          "datasetTemplateId": "empty"}))
    sw.wait_for_tenant("soak", 120)
    ms = sw["inbound-processing"]
    if args.filter_ids:
        from sitewhere_amd.runtime.config import dump_document
        before = ms.get_tenant_engine("soak")
        cfg = dict(before.config)
        cfg["capacity"] = dict(cfg.get("capacity", {}), dedup_filter_ids=args.filter_ids)
        sw.instance.coord.put(ms.tenant_config_path("soak"), dump_document(cfg))
        while ms.get_tenant_engine("soak") in (None, before) or ms.get_tenant_engine("soak").status.value != "Started":
            time.sleep(0.1)
    run = lambda f: sw.instance.system_user.run(f, "soak")  # noqa: E731
    dm = sw.api("DeviceManagement", "soak")
    run(lambda: dm.create_device_type({"token": "sensor", "name": "Sensor"}))
    # fleet import: devices, then their assignments (no "assignment Active" events -- an imported
    # fleet's activations happened before), in bulk: one change-feed record per 4096 entities
    for s in range(0, args.devices, args.chunk):
        toks = [f"dev-{i:010d}" for i in range(s, min(args.devices, s + args.chunk))]
        run(lambda: dm.create_devices([{"token": t, "deviceTypeToken": "sensor"} for t in toks]))
        run(lambda: dm.create_device_assignments([{"deviceToken": t} for t in toks], record_state_changes=False))
        log(f"imported {s + len(toks)} devices ({time.time() - t_setup:.0f} s)")
    ib = sw.tenant_engine("inbound-processing", "soak")
    while ib.engine.n_assignments < args.devices and time.time() - t_setup < 3600:
        time.sleep(0.2)
    while ib.dictionary_pending() >= ib.PRIME_DICTIONARY_MIN and time.time() - t_setup < 3600:
        time.sleep(0.2)                         # the imported fleet's dictionary reaches the store
    log(f"engine registry: {ib.engine.n_devices} devices, {ib.engine.n_assignments} assignments")
    ecfg = ib.engine.cfg
    store = sw.tenant_engine("event-management", "soak").store
    log("dedup sizing", json.dumps(ib.dedup_sizing_report, default=str))
    spec = FleetSpec(prefix="dev-", n_devices=args.devices, p_location=0.25, p_alert=0.05, mx_per_msg=1,
                     with_alternate_id=True, p_unregistered=args.p_unregistered)
    now0 = int(time.time() * 1000)
    base, recs, pos = [], [], []
    pin = torch.cuda.is_available()
    for b in range(args.records):
        raw, offs = gen_payloads(spec, args.batch, now0 - 1000, seed=11 + b)
        base.append((raw, offs))
        r = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1, pinned=pin)
        recs.append(r)
        pos.append(alt_positions(r.ptr + VALUE_HDR, offs))
    import gc
    gc.collect()
    gc.freeze()                                 # the fleet's objects leave the cyclic collector
    setup_s = time.time() - t_setup
    log(f"setup {setup_s:.0f} s")
    bus = sw.instance.bus
    t_raw = sw.instance.naming.tenant_prefix("soak") + "event-source-raw-payloads"
    parts = bus.partitions(t_raw)
    group = ib.raw_consumer.group
    slot_at = [None] * args.records            # (partition, offset) of each record's last publish
    epochs: list = []                          # (time, slot, epoch) of every publish

    def committed(p):
        return bus.committed(group, t_raw, p) or 0

    def done(po):
        return po is None or committed(po[0]) > po[1]

    k = 0
    samples = []                               # (t, processed, persisted, rechecks, duplicates, msgs)

    def sample():
        st = ib.engine.stats_dict()
        samples.append((time.perf_counter(), ib.processed_events.count, ib.persisted_events.count,
                        st["dedup_rechecks"], st["duplicates"], st["messages"], st["unregistered"]))

    t0 = time.perf_counter()
    sample()
    next_log = t0 + 5.0
    end = t0 + args.phases * args.phase_s
    inflight = []
    while time.perf_counter() < end:
        # flow control: at most `ahead` records past the tenant's commits
        while inflight and done(inflight[0]):
            inflight.pop(0)
        if len(inflight) >= args.ahead or not done(slot_at[k % args.records]):
            time.sleep(0.0005)
        else:
            s = k % args.records
            epoch = (0x50AC << 48) | k
            stamp_positions(recs[s].ptr + VALUE_HDR, pos[s], epoch, threads=8)     # fresh ids
            p = k % parts
            off = recs[s].publish(bus, t_raw, p, ts=now0 + k)
            slot_at[s] = (p, off)
            inflight.append((p, off))
            epochs.append((time.perf_counter(), s, epoch))
            k += 1
        now = time.perf_counter()
        if now >= next_log:
            sample()
            a, b_ = samples[-2], samples[-1]
            rate = (b_[1] - a[1]) / max(1e-9, b_[0] - a[0])
            fs = ib.engine.filter_state()
            rs = store.retention_state()
            log(f"t={now - t0:6.1f}s {rate / 1e6:7.1f}M ev/s records={k} rechecks={b_[3]} dups={b_[4]} "
                f"filter_rot={fs.get('rotations')} retained_rows={rs['retained_rows']} deleted_rows={rs['deleted_rows']}")
            next_log = now + 5.0
    while inflight:                             # drain: every published record stored and committed
        while inflight and done(inflight[0]):
            inflight.pop(0)
        time.sleep(0.001)
    ib.flush()
    sample()
    t_end = time.perf_counter()
    # ---- replay of a still-retained batch: the first `replay` payloads of a record published a few
    # seconds ago, with its ids
    rs0 = store.retention_state()
    recent = [e for e in epochs if t_end - e[0] >= 2.0] or epochs[:1]
    te, s, epoch = recent[-1]
    raw, offs = base[s]
    m = min(args.replay, len(offs) - 1)
    sub = np.concatenate([raw[:int(offs[m])], np.zeros(64, np.uint8)])
    stamp_alt_epoch(sub, offs[:m + 1], epoch)
    from sitewhere_amd.pipeline.fleet import cpu_decode
    dec = cpu_decode(sub, offs[:m + 1], now0)
    valid_alt = int(((dec["alt_hash"] != 0) & (dec["etype"] < 16)).sum())
    rdup0, rfp0 = ib.recheck_duplicates, ib.recheck_false_positives
    st0 = ib.engine.stats_dict()
    rows0 = store.rows
    # the stored event of every replayed id before the replay: a replay stored again would make its
    # id's newest stored event a different one
    hs0 = dec["alt_hash"][(dec["alt_hash"] != 0) & (dec["etype"] < 16)]
    stored_before = store.find_alternate_hashes(hs0.tolist(), indexed_only=False)
    rr = RawBatchRecord(sub[:int(offs[m])], varint_lengths(offs[:m + 1]), m, pinned=pin)
    p = k % parts
    off = rr.publish(bus, t_raw, p, ts=now0 + k)
    tw = time.time()
    while committed(p) <= off and time.time() - tw < 60:
        time.sleep(0.002)
    ib.flush()
    time.sleep(2.0)                            # the per-event path drops the rechecked replays
    st1 = ib.engine.stats_dict()
    replay = {"age_s": round(t_end - te, 2), "payloads": m, "events_with_alt_ids": valid_alt,
              "rechecks": st1["dedup_rechecks"] - st0["dedup_rechecks"],
              "window_duplicates": st1["duplicates"] - st0["duplicates"],
              "settled_duplicates": ib.recheck_duplicates - rdup0,
              "settled_false_positives": ib.recheck_false_positives - rfp0,
              "persisted_by_engine": st1["persisted"] - st0["persisted"],
              "store_rows_before": rows0, "store_rows_after": store.rows}
    # events of registered devices (the replay's unregistered payloads are routed, not deduplicated)
    replay["events_of_registered_devices"] = valid_alt - (st1["unregistered"] - st0["unregistered"])
    # diagnostics: the store's own answer for the replayed ids (indexed blocks, and every block)
    hs = dec["alt_hash"][(dec["alt_hash"] != 0) & (dec["etype"] < 16)]
    f_ix = store.find_alternate_hashes(hs.tolist(), indexed_only=True)
    f_all = store.find_alternate_hashes(hs.tolist(), indexed_only=False)
    replay["store_finds_indexed"], replay["store_finds_all"] = len(f_ix), len(f_all)
    # the stored id strings themselves (every block's id column decoded, newest first): are the
    # replayed ids in the store at all, or only missing from the trailers' lookups?
    want = set(int(x) for x in hs.tolist())
    in_cols, scanned = set(), 0
    for chunk in store.alternate_hash_chunks(max_ids=int(os.environ.get("SOAK_SCAN_IDS", 1 << 30))):
        scanned += len(chunk)
        in_cols |= want & set(np.intersect1d(chunk, hs).tolist())
        if len(in_cols) == len(want):
            break
    replay["store_decoded_has"], replay["store_decoded_scanned"] = len(in_cols), scanned
    miss = sorted(want - set(int(k) for k in f_ix))
    replay["missing_in_decoded"] = len(set(miss) - in_cols)
    if os.environ.get("SOAK_FORCE_DIAG"):           # exercise the diagnostics on found ids
        replay["trailer_diag_forced"] = _trailer_diag(store, ib, sorted(in_cols)[:8])
    if miss:
        # where the missing ids sit in the replayed sub-batch (payload index, device, event type)
        idx = np.nonzero(np.isin(dec["alt_hash"], np.array(miss[:2000], np.uint64)))[0]
        replay["missing_payload_idx_sample"] = idx[:40].tolist()
        replay["missing_etypes"] = np.bincount(dec["etype"][idx].astype(np.int64), minlength=4).tolist()
        replay["missing_first_last"] = [int(idx.min()), int(idx.max())] if len(idx) else None
        lost = sorted(set(miss) & in_cols)          # stored, yet not found through the trailers
        if lost:
            replay["trailer_diag"] = _trailer_diag(store, ib, lost)
    replay["store_blocks"] = store.index_stats()
    changed = [h for h, e in f_all.items() if stored_before.get(h) != e]
    replay["ids_stored_again"] = len(changed) + len(set(f_all) - set(stored_before))
    # other traffic may add rows meanwhile (presence scans, the per-event path): the test is that no
    # replayed id got a second stored event
    replay["all_duplicates"] = (replay["settled_duplicates"] + replay["window_duplicates"]
                                == replay["events_of_registered_devices"] and replay["persisted_by_engine"] == 0
                                and replay["ids_stored_again"] == 0)
    # ---- report
    ts = np.array([x[0] for x in samples]) - t0
    ev = np.array([x[1] for x in samples], np.float64)

    def rate_between(a, b):
        i, j = int(np.searchsorted(ts, a)), int(np.searchsorted(ts, b, side="right")) - 1
        if j <= i:
            return None
        return round(float((ev[j] - ev[i]) / (ts[j] - ts[i])), 1)

    phases = [rate_between(i * args.phase_s, (i + 1) * args.phase_s) for i in range(args.phases)]
    total_s = args.phases * args.phase_s
    first_min, last_min = rate_between(0, min(60.0, total_s)), rate_between(max(0.0, total_s - 60.0), total_s)
    st = ib.engine.stats_dict()
    fs = ib.engine.filter_state()
    rs = store.retention_state()
    msgs = st["messages"]
    trace = {}
    if ib.trace:
        tr = [x for x in ib.trace if len(x) == 9]
        gap = np.diff(np.asarray([x[0] for x in tr])) * 1000 if len(tr) > 1 else np.zeros(0)
        if len(gap):
            trace.update({f"submit_interval_p{q}_ms": round(float(np.percentile(gap, q)), 3) for q in (50, 90, 99)})
            trace["submit_interval_max_ms"] = round(float(gap.max()), 3)
            # per stage of a batch's life (submit, engine completion, store thread, durable commit):
            # median ms between consecutive trace stamps
            st_ = np.diff(np.asarray([x[:9] for x in tr], np.float64), axis=1) * 1000
            trace["stage_ms_p50"] = [round(float(x), 3) for x in np.median(st_, axis=0)]
            trace["stage_ms_p99"] = [round(float(x), 3) for x in np.percentile(st_, 99, axis=0)]
    ft = getattr(type(ib.engine), "framed_trace", None)
    if ft:
        n_sub = max(1, k)
        trace["framed_phase_ms_per_submit"] = {kk: round(v * 1000 / n_sub, 3) for kk, v in ft.items()}
    trace["pin_stats"] = {kk: v for kk, v in ib.engine.__dict__.items() if kk.startswith("pin_stats")}
    cap = ecfg.dedup_filter_gens * ecfg.dedup_filter_ids
    out = {"metric": "tenant_soak_events_per_sec", "template": args.template, "devices": args.devices,
           "batch": args.batch, "p_unregistered": args.p_unregistered, "alt_ids": True, "via_bus": True,
           "engine": ib.engine_kind, "numa_node": numa_node, "setup_s": round(setup_s, 1),
           "soak_s": round(t_end - t0, 1), "events": int(ev[-1] - ev[0]),
           "events_per_sec": round(float((ev[-1] - ev[0]) / (ts[-1] - ts[0])), 1),
           "phase_events_per_sec": phases, "first_minute_events_per_sec": first_min,
           "last_minute_events_per_sec": last_min,
           "last_vs_first": round(last_min / first_min, 3) if first_min and last_min else None,
           "records": k, "messages": msgs, "rechecks": st["dedup_rechecks"],
           "rechecks_per_payload": st["dedup_rechecks"] / max(1, msgs), "window_duplicates": st["duplicates"],
           "unregistered": st["unregistered"], "dedup_overflow": st["dedup_overflow"],
           "filter": {**fs, "capacity_ids": cap, "holds_ids": (ecfg.dedup_filter_gens - 1) * ecfg.dedup_filter_ids,
                      "bytes": ecfg.filter_bytes(), "ids_ingested_per_capacity": round(st["persisted"] / max(1, cap), 2)},
           "store": {**rs, "retention_wraps": round(rs["deleted_rows"] / max(1, rs["retention_rows"]), 2)},
           "trace": trace, "replay": replay,
           "timers_ms": {name: round(t.hist.snapshot()["mean"], 3)
                         for name, t in (("engine_step", ib.step_timer), ("columnar_store", ib.store_timer),
                                         ("recheck", ib.recheck_timer))},
           "series": [[round(float(a), 1), int(b)] for a, b in zip(ts, ev)]}
    print(json.dumps(out, default=str), flush=True)
    sw.stop()


if __name__ == "__main__":
    main()
