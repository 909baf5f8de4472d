"""Durable columnar event segments: block codec (csrc/include/swseg.h, csrc/native/swseg.cpp), the
native segment store (group commit, recovery, retention) and the DurableEventStore over it.  The
MI355X encoder is checked against the CPU encoder bit for bit in tests/test_gpu_segments.py."""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import pytest

from sitewhere_amd.models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE, NO_NAME, OUT_REC
from sitewhere_amd.persistence import segments as sg


def synth_rows(n, seed=0, full_precision=False, strings=True):
    """Inputs of one block shaped like an engine step's persisted output: decoded device events of a
    generated fleet (decimal sensor values, 6-decimal coordinates, alerts with varied messages,
    metadata on some events, alternate ids) enriched with assignments and name ids, then rule alerts
    and presence state changes (generated rows).  Returns (rows, records, string refs, raw batch)."""
    from sitewhere_amd.pipeline.fleet import FleetSpec, cpu_decode, gen_payloads
    rng = np.random.default_rng(seed)
    n_dev = max(1, n)
    spec = FleetSpec(prefix="s-", n_devices=n_dev, with_alternate_id=strings, p_meta=0.3 if strings else 0.0,
                     mx_per_msg=1 + seed % 2, lat0=33.0, lon0=-85.0, span_deg=2.0)
    n_msgs = max(1, int(n * 0.9) // spec.mx_per_msg)
    raw, offs = gen_payloads(spec, n_msgs, 1_700_000_000_000, seed=seed + 1)
    recs, spans = cpu_decode(raw, offs, 1_700_000_000_000, cap=4 * n_msgs + 16, spans=True)
    recs, spans = recs[:n], spans[:n]
    if not strings:
        spans[:] = 0
    g = n - len(recs)                                       # generated rows fill the rest
    gen = np.zeros(g, recs.dtype)
    gen["etype"] = np.where(rng.random(g) < 0.5, EV_ALERT, EV_STATE_CHANGE)
    gen["event_date"] = 1_700_000_100_000
    gen["level"] = np.where(gen["etype"] == EV_ALERT, rng.integers(0, 4, g), 0)
    recs = np.concatenate([recs, gen])
    spans = np.concatenate([spans, np.zeros(g, spans.dtype)])
    et = recs["etype"]
    rows = np.zeros(n, OUT_REC)
    rows["etype"] = et
    rows["event_date"] = recs["event_date"]
    rows["assignment"] = rng.integers(0, 1 << 20, n)
    loc = et == EV_LOCATION
    rows["name_id"] = np.where(loc, NO_NAME, rng.integers(0, 20, n))
    rows["v0"], rows["v1"], rows["level"] = recs["v0"], recs["v1"], recs["level"]
    if full_precision:
        rows["v0"] = np.where(loc, 33.0 + 2.0 * rng.random(n), rows["v0"])
        rows["v1"] = np.where(loc, -85.0 + 2.0 * rng.random(n), rows["v1"])
    return rows, recs, spans, raw


def expected_strings(recs, spans, raw):
    """(alternate id or None, alert message, metadata) of each row, read from the batch directly."""
    from sitewhere_amd.models.wire import iter_fields
    b = raw.tobytes()
    out = []
    for r, s in zip(recs, spans):
        alt = None
        if s["has"] & 1:
            alt = b[int(s["alt_off"]):int(s["alt_off"]) + int(s["alt_len"])].decode()
            if s["has"] & 4:
                alt += f":{int(s['k'])}"
        gen = int(r["fp_lo"]) == 0 and int(r["fp_hi"]) == 0
        msg = b[int(r["aux2_off"]):int(r["aux2_off"]) + int(r["aux2_len"])].decode() \
            if int(r["etype"]) == EV_ALERT and not gen else ""
        md = {}
        if s["has"] & 2:
            span = b[int(s["meta_off"]):int(s["meta_off"]) + int(s["meta_len"])]
            field = {EV_MEASUREMENT: 4, EV_LOCATION: 6, EV_ALERT: 5}[int(r["etype"])]
            for f, wt, v in iter_fields(span):
                if f == field:
                    kv = dict((f2, v2.decode()) for f2, _, v2 in iter_fields(v))
                    md[kv[1]] = kv[2]
        out.append((alt, msg, md))
    return out


def check_roundtrip(rows, recs, spans, raw):
    blk = sg.encode_block(rows, recs, spans, raw)
    sg.seal(blk, 1000, 1_700_000_100_000, 7, 0, 1)
    assert sg.verify(blk) == 0
    c = sg.decode_block(blk)
    assert c["header"]["n_rows"] == len(rows) and c["header"]["first_seq"] == 1000
    for col, key in (("etype", "etype"), ("level", "level"), ("date", "event_date"), ("asg", "assignment"),
                     ("name", "name_id")):
        np.testing.assert_array_equal(c[col], rows[key], err_msg=col)
    # values bit for bit (exceptions included); elevation only where one was sent
    np.testing.assert_array_equal(c["v0"].view(np.uint64), rows["v0"].view(np.uint64))
    np.testing.assert_array_equal(c["v1"].view(np.uint64), rows["v1"].view(np.uint64))
    has_elev = (recs["etype"] == EV_LOCATION) & ((recs["flags"] & 8) != 0)
    np.testing.assert_array_equal(c["v2"].view(np.uint64), np.where(has_elev, recs["v2"], 0.0).view(np.uint64))
    assert ((c["flags"] & sg.SEGF_HAS_ELEV) != 0).tolist() == has_elev.tolist()
    gen = (recs["fp_lo"] == 0) & (recs["fp_hi"] == 0)
    assert ((c["flags"] & sg.SEGF_GEN) != 0).tolist() == gen.tolist()
    us = np.where(gen, 0, recs["flags"] & 3)
    np.testing.assert_array_equal(c["flags"] & 3, us)
    want = expected_strings(recs, spans, raw)
    for i in range(len(rows)):
        assert sg.row_strings(c, i) == want[i], i
    # without strings: the same columns (the string-length columns are skipped), no heap
    c2 = sg.decode_block(blk, strings=False)
    assert c2["str_heap"] is None
    for col in ("etype", "level", "date", "asg", "name", "v0", "v1", "v2", "flags"):
        np.testing.assert_array_equal(c2[col].view(np.uint8), c[col].view(np.uint8), err_msg=col)
    return blk


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 5000])
def test_block_roundtrip(n):
    check_roundtrip(*synth_rows(n, seed=n))


def test_block_is_lossless_for_every_string_form():
    """Alternate ids in raw and hex pages, multi-measurement suffixes, alert messages, metadata on
    every event type, updateState true / false / absent, elevation sent or not."""
    from sitewhere_amd.models import wire
    from sitewhere_amd.pipeline.fleet import cpu_decode, pack_messages
    msgs = []
    for i in range(3000):
        md = {f"k{j}": f"value-{i}-{j}" for j in range(i % 3)}
        alt = [f"{i:08x}", f"uuid-{i * 7919 % 104729}-x", None, f"dev-9-{i}"][i % 4]
        us = [None, True, False][i % 3]
        k = i % 5
        if k == 0:
            msgs.append(wire.measurements(f"d-{i}", {"t": i / 100, "h": -i / 10}, alternate_id=alt, metadata=md,
                                          update_state=us))
        elif k == 1:
            msgs.append(wire.location(f"d-{i}", 33 + i / 1e6, -84 - i / 1e6, elevation=None if i % 2 else i / 10,
                                      alternate_id=alt, metadata=md, update_state=us))
        elif k == 2:
            msgs.append(wire.alert(f"d-{i}", f"type{i % 7}", f"alert number {i} 漢字", alternate_id=alt, metadata=md,
                                   update_state=us))
        else:
            msgs.append(wire.measurements(f"d-{i}", {"only": float(i)}, alternate_id=alt))
    raw, offs = pack_messages(msgs)
    recs, spans = cpu_decode(raw, offs, 1_700_000_000_000, cap=8000, spans=True)
    rows = np.zeros(len(recs), OUT_REC)
    for k in ("event_date", "v0", "v1", "etype", "level"):
        rows[k] = recs[k]
    rows["assignment"] = np.arange(len(recs)) % 77
    rows["name_id"] = np.where(recs["etype"] == EV_LOCATION, NO_NAME, 3)
    check_roundtrip(rows, recs, spans, raw)
    # pages of counter-style ids take the hex mode: no remainder bytes in the heap
    hexy = [wire.measurements(f"d-{i}", {"a": 1.0}, alternate_id=f"0123456789abcdef-{i:08x}") for i in range(2048)]
    raw, offs = pack_messages(hexy)
    recs, spans = cpu_decode(raw, offs, 1_700_000_000_000, cap=4096, spans=True)
    rows = np.zeros(len(recs), OUT_REC)
    rows["event_date"], rows["v0"], rows["name_id"] = recs["event_date"], recs["v0"], 1
    blk = check_roundtrip(rows, recs, spans, raw)
    assert len(blk) / len(rows) < 8, len(blk) / len(rows)        # a 26-byte id costs ~1.5 bytes


def test_block_compresses_decimal_data():
    rows, recs, spans, raw = synth_rows(100_000, seed=1, strings=False)
    blk = check_roundtrip(rows, recs, spans, raw)
    assert len(blk) / len(rows) < 9.0, len(blk) / len(rows)       # vs 32 B OUT_REC + 8 B elevation


def test_block_exceptions_are_lossless():
    rows, recs, spans, raw = synth_rows(20_000, seed=2, full_precision=True)
    rows["v0"][::7] = np.where(rows["etype"][::7] == EV_MEASUREMENT, np.nan, rows["v0"][::7])
    rows["v0"][1::11] = np.where(rows["etype"][1::11] == EV_MEASUREMENT, -0.0, rows["v0"][1::11])
    rows["v1"][::13] = np.where(rows["etype"][::13] == EV_LOCATION, np.inf, rows["v1"][::13])
    check_roundtrip(rows, recs, spans, raw)


def test_corruption_detected():
    blk = check_roundtrip(*synth_rows(3000, seed=3))
    for pos in (10, 64 + 4, len(blk) // 2, len(blk) - 8):
        bad = blk.copy()
        bad[pos] ^= 0x40
        assert sg.verify(bad) != 0, pos


def _store_blocks(st, nblocks, rows_per=3000):
    seq = 0
    blocks = []
    for b in range(nblocks):
        rows, recs, spans, raw = synth_rows(rows_per, seed=100 + b)
        blk = sg.encode_block(rows, recs, spans, raw)
        sg.seal(blk, seq, 1_700_000_000_000 + b, b, 0, 1)
        tok = st.append_block(blk)
        blocks.append((seq, rows, tok))
        seq += rows_per
    return blocks


def test_segment_store_durable_reopen_and_index(tmp_path):
    d = str(tmp_path / "seg")
    st = sg.SegmentStore(d, rotate_bytes=64 << 10, direct=True)
    blocks = _store_blocks(st, 12)
    assert st.flush(30)
    assert st.durable() == blocks[-1][2]
    stats = st.stats()
    assert stats["blocks_written"] == 12 and stats["files"] > 1 and stats["syncs"] >= 1
    st.close()
    st2 = sg.SegmentStore(d)
    idx = st2.index()
    assert list(idx["first_seq"]) == [b[0] for b in blocks]
    for ent, (seq, rows, _) in zip(idx, blocks):
        c = sg.decode_block(st2.read_block(ent))
        np.testing.assert_array_equal(c["date"], rows["event_date"])
        assert ent["min_date"] <= rows["event_date"].min() and ent["max_date"] >= rows["event_date"].max()
    st2.close()


def test_segment_store_torn_tail_recovery(tmp_path):
    d = str(tmp_path / "seg")
    st = sg.SegmentStore(d)
    blocks = _store_blocks(st, 5)
    st.flush(30)
    st.close()
    files = sorted(os.listdir(d))
    path = os.path.join(d, [f for f in files if f.endswith(".sweg")][-1])
    size = os.path.getsize(path)
    with open(path, "r+b") as f:               # crash mid-write of the last block: garbage tail
        f.seek(size - 4096 - 3000)              # (the block's last bytes are in its final 4 KiB)
        f.write(os.urandom(4096 + 3000))
    st2 = sg.SegmentStore(d)
    idx = st2.index()
    assert list(idx["first_seq"]) == [b[0] for b in blocks[:-1]]
    assert os.path.getsize(path) < size        # truncated at the last good block
    # appends continue after recovery
    blk = sg.encode_block(*synth_rows(100, seed=9))
    sg.seal(blk, blocks[-1][0], 1, 99, 0, 1)
    st2.wait(st2.append_block(blk), 30)
    assert len(st2.index()) == 5
    st2.close()


def test_segment_store_retention(tmp_path):
    d = str(tmp_path / "seg")
    st = sg.SegmentStore(d, rotate_bytes=48 << 10, retention_bytes=160 << 10)
    _store_blocks(st, 30)
    st.flush(30)
    s = st.stats()
    assert s["deleted_files"] > 0 and s["retained_bytes"] <= (160 << 10) + (48 << 10)
    idx = st.index()
    assert len(idx) < 30 and idx["first_seq"][-1] == 29 * 3000
    for ent in idx:
        assert sg.verify(st.read_block(ent)) == 0
    st.close()


def test_durable_event_store_queries_and_restart(tmp_path):
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    d = str(tmp_path / "es")
    es = sg.DurableEventStore(d)
    rows, recs, spans, raw = synth_rows(4000, seed=5)
    rows["assignment"] = np.arange(4000) % 50
    asg = {i: [f"asg-{i}", f"dev-{i}", f"cust-{i % 3}", f"area-{i % 2}", None] for i in range(50)}
    names = {i: f"mx.metric{i}" for i in range(20)}
    blk = sg.encode_block(rows, recs, spans, raw)
    sg.seal(blk, 0, 1_700_000_100_000, 0xb0, 0, 1)
    tok = es.add_encoded(blk, asg=asg, names=names)
    es.wait(tok)
    # replayed block (same sequence range) is skipped
    assert es.add_encoded(blk) == -1
    res = es.list_events("Measurement", "Assignment", ["asg-7"], DateRangeSearchCriteria(page_size=0))
    want = rows[(rows["assignment"] == 7) & (rows["etype"] == EV_MEASUREMENT)]
    assert res.num_results == len(want)
    assert sorted(e.value for e in res.results) == sorted(want["v0"].tolist())
    assert all(e.name.startswith("mx.metric") and e.device_id == "dev-7" for e in res.results)
    # the whole event comes back: alternate ids and metadata of the stored rows
    exp = expected_strings(recs, spans, raw)
    by_id = {e.id: e for e in res.results}
    for j in np.nonzero((rows["assignment"] == 7) & (rows["etype"] == EV_MEASUREMENT))[0]:
        e = by_id[f"b0-{int(j)}"]
        assert (e.alternate_id, e.metadata) == (exp[j][0], exp[j][2])
    ev = res.results[0]
    es.close()
    es2 = sg.DurableEventStore(d)                         # restart: everything from disk
    again = es2.list_events("Measurement", "Assignment", ["asg-7"], DateRangeSearchCriteria(page_size=0))
    assert [e.id for e in again.results] == [e.id for e in res.results]
    assert es2.get_event_by_id(ev.id).value == ev.value
    with_alt = [j for j in range(len(rows)) if exp[j][0] is not None]
    for j in with_alt[:5] + with_alt[-3:]:
        got = es2.get_event_by_alternate_id(exp[j][0])
        assert got is not None and got.id == f"b0-{j}" and got.alternate_id == exp[j][0]
    from sitewhere_amd.pipeline.fleet import hash64
    hashes = [hash64(exp[j][0]) for j in with_alt[:5]]
    found = es2.find_alternate_hashes(hashes)
    assert set(found) == set(hashes)
    assert all(v.startswith("b0-") for v in found.values())
    assert es2.get_event_by_alternate_id("no-such-id") is None
    # a new engine incarnation restarts its sequences and indices: its block is not a replay, and
    # its dictionary does not rewrite the first boot's
    rows2 = rows.copy()
    rows2["assignment"] = (np.arange(4000) + 25) % 50
    blk2 = sg.encode_block(rows2, recs, spans, raw)
    sg.seal(blk2, 0, 1_700_000_200_000, 0xb1, 0, 1)
    asg2 = {i: [f"asg-{(i + 1) % 50}", f"dev-{(i + 1) % 50}", None, None, None] for i in range(50)}
    es2.wait(es2.add_encoded(blk2, asg=asg2))
    both = es2.list_events("Measurement", "Assignment", ["asg-7"], DateRangeSearchCriteria(page_size=0))
    want2 = rows2[(rows2["assignment"] == 6) & (rows2["etype"] == EV_MEASUREMENT)]
    assert both.num_results == len(want) + len(want2)
    assert {e.id.split("-")[0] for e in both.results} == {"b0", "b1"}
    es2.close()


class _FakeHostBuffer:
    """Page-aligned host memory standing in for the MI355X pinned buffers (no GPU needed)."""

    def __init__(self, lib, n):
        import ctypes
        import mmap
        self.m = mmap.mmap(-1, n)
        self.nbytes = n
        self.host = ctypes.addressof(ctypes.c_char.from_buffer(self.m))


def test_block_sink_pool_bounded_and_commits_in_order(tmp_path):
    """DurableBlockSink: blocks published zero-copy to the enriched topic and queued to the store;
    buffers come back when both let go (growing blocks replace undersized buffers), and the caller
    tags come back as committable in order once durable."""
    import ctypes
    from sitewhere_amd.bus.log import EventBus
    store = sg.DurableEventStore(str(tmp_path / "s"))
    bus = EventBus(None, default_partitions=1)
    sink = sg.DurableBlockSink(store, None, 5, bus=bus, topic="t.out", max_buffers=16)
    sink._HostBuffer = _FakeHostBuffer
    bus.set_retention("t.out", 4 << 20)
    tags = []
    for k in range(60):
        blk = sg.encode_block(*synth_rows(20000 + 1000 * k, seed=k))
        host, buf = sink.target(len(blk))
        ctypes.memmove(host, blk.ctypes.data, len(blk))
        sink.publish(buf, len(blk), k * 200_000, 1, tag=k)
        tags += sink.committable()
    sink.flush()
    tags += sink.committable()
    assert tags == list(range(60))
    assert sink.n_alloc <= 16 and store.rows == sum(20000 + 1000 * k for k in range(60))
    # the topic carries the sealed blocks
    v = bus.read_views("t.out", 0, bus.begin_offset("t.out", 0), 1)[0].value
    assert sg.verify(np.frombuffer(v, np.uint8)) == 0
    store.close()


def test_failed_append_is_retried_not_skipped_as_a_replay(tmp_path):
    """the (boot, rank) high-water mark moves only once a block is queued.  A write that
    fails is retried as a write; a replay of queued-but-not-durable rows returns the token that makes
    them durable, and -1 only once they are on disk -- so a caller never commits offsets of rows that
    are not on disk."""
    es = sg.DurableEventStore(str(tmp_path / "es"))
    blk = sg.encode_block(*synth_rows(2000, seed=11))
    sg.seal(blk, 0, 1_700_000_100_000, 0xc0, 0, 1)
    real = es.seg.append
    calls = {"n": 0}

    def failing(*a, **k):
        calls["n"] += 1
        raise OSError(5, "injected write failure")
    es.seg.append = failing
    with pytest.raises(OSError):
        es.add_encoded(blk)
    es.seg.append = real
    tok = es.add_encoded(blk)                 # the retry writes the block (not a "replay" skip)
    assert tok >= 0 and calls["n"] == 1
    assert es.add_encoded(blk) in (tok, -1)   # a replay while queued: the same token (or -1 once durable)
    es.wait(tok)
    assert es.add_encoded(blk) == -1
    assert es.rows == 2000
    es.close()


def _ctx_store_blocks(tmp_path, n_blocks=5, rows_per=3000, dates="random", n_asg=40, trailers=True, seed=3,
                      n_cust=3, n_area=2, n_asset=5):
    """A store of engine-like blocks: assignment contexts with engine ids (customer i % n_cust, area
    i % n_area, asset i % n_asset), trailers built with that context table, dictionaries with the
    context ids."""
    es = sg.DurableEventStore(str(tmp_path / "es"), direct=False)
    asg = {i: [f"asg-{i}", f"dev-{i}", f"cust-{i % n_cust}", f"area-{i % n_area}", f"asset-{i % n_asset}"]
           for i in range(n_asg)}
    ctx_tab = np.array([[i, i % n_cust, i % n_area, i % n_asset] for i in range(n_asg)], np.int32)
    ctx = {0: {f"cust-{k}": k for k in range(n_cust)}, 1: {f"area-{k}": k for k in range(n_area)},
           2: {f"asset-{k}": k for k in range(n_asset)}}
    names = {i: f"mx.metric{i}" for i in range(20)}
    blocks, exp_all, n0 = [], [], 0
    rng = np.random.default_rng(seed)
    for b in range(n_blocks):
        rows, recs, spans, raw = synth_rows(rows_per, seed=20 + b)
        rows["assignment"] = rng.integers(0, n_asg, len(rows))
        if dates == "random":
            rows["event_date"] = 1_700_000_000_000 + rng.integers(0, 5_000_000, len(rows))   # out of order
        else:                           # real devices: each block newer than the last, a little jitter
            rows["event_date"] = 1_700_000_000_000 + b * 1_000_000 + rng.integers(0, 50_000, len(rows))
        # persist order clustered by assignment, the generated rows after the rest (what the engines
        # do: their trailers then carry SIX_F_CLUSTERED)
        gen = (recs["fp_lo"] == 0) & (recs["fp_hi"] == 0)
        o = np.lexsort((rows["assignment"], gen))
        rows, recs, spans = rows[o], recs[o], spans[o]
        blk = sg.encode_block(rows, recs, spans, raw, index=trailers, ctx=ctx_tab)
        sg.seal(blk, n0, 1_700_000_100_000 + b, 0xc0, 0, 1)
        es.wait(es.add_encoded(blk, asg=asg, names=names, ctx=ctx))
        blocks.append((blk.copy(), n0))
        exp_all += [(n0 + j, s_[0]) for j, s_ in enumerate(expected_strings(recs, spans, raw))]
        n0 += len(rows)
    return es, asg, blocks, exp_all


def _brute(blocks, asg, etype, index, ents, c):
    """What the store must answer: every block decoded and filtered, newest first (date, then id)."""
    from sitewhere_amd.persistence.segments import _CTX, _ETYPE
    from sitewhere_amd.models.domain import DeviceEventIndex, DeviceEventType
    et = _ETYPE[DeviceEventType(etype)]
    pos = _CTX[DeviceEventIndex(index)]
    hits = []
    for blk, n0 in blocks:
        cols = sg.decode_block(blk)
        for i in range(len(cols["date"])):
            d = int(cols["date"][i])
            if int(cols["etype"][i]) != et or asg[int(cols["asg"][i])][pos] not in ents:
                continue
            if (c.start_date is not None and d < c.start_date) or (c.end_date is not None and d > c.end_date):
                continue
            hits.append((d, n0 + i))
    hits.sort(key=lambda x: (-x[0], -x[1]))
    total = len(hits)
    if c.page_size > 0:
        start = (max(1, c.page_number) - 1) * c.page_size
        hits = hits[start:start + c.page_size]
    return total, [(f"c0-{e}", d) for d, e in hits]


@pytest.mark.parametrize("dates", ["random", "increasing"])
def test_block_indexes_answer_like_the_scan(tmp_path, dates):
    """Reads through the index trailers (assignment zone maps + leading-column page scans, context-key
    counts and heads merged across blocks, alternate-id buckets) return exactly what decoding and
    filtering every block returns: totals, newest-first order across blocks, date ranges (blocks
    straddling a bound), paging deep enough to exhaust blocks' heads, point lookups, dedup hashes.
    Dates out of order within and across blocks, or increasing block by block (real devices: page 1
    then comes from the newest block, whose heads run out)."""
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    from sitewhere_amd.pipeline.fleet import hash64
    es, asg, blocks, exp_all = _ctx_store_blocks(tmp_path, dates=dates)
    assert es.index_stats()["indexed"] == 5
    t0 = 1_700_000_000_000
    crits = [DateRangeSearchCriteria(page_size=0), DateRangeSearchCriteria(page_size=7),
             DateRangeSearchCriteria(page_number=3, page_size=5), DateRangeSearchCriteria(page_size=100),
             DateRangeSearchCriteria(page_number=2, page_size=40),
             DateRangeSearchCriteria(page_size=10, start_date=t0 + 1_000_000, end_date=t0 + 3_000_000),
             DateRangeSearchCriteria(page_size=0, start_date=t0 + 2_000_000)]
    queries = [(t, ix, ents) for t in ("Measurement", "Location", "Alert")
               for ix, ents in (("Assignment", ["asg-3"]), ("Assignment", ["asg-5", "asg-9", "nope"]),
                                ("Customer", ["cust-1"]), ("Area", ["area-0"]), ("Asset", ["asset-2", "asset-4"]),
                                ("Customer", ["nobody"]))]
    n_checked = 0
    for t, ix, ents in queries:
        for c in crits:
            r = es.list_events(t, ix, ents, c)
            got = (r.num_results, [(e.id, e.event_date) for e in r.results])
            want = _brute(blocks, asg, t, ix, set(ents), c)
            assert got == want, (t, ix, ents, c)
            n_checked += want[0]
    assert n_checked > 5000
    rng = np.random.default_rng(9)
    with_alt = [(eid, a) for eid, a in exp_all if a is not None]
    picks = [with_alt[i] for i in rng.choice(len(with_alt), 40, replace=False)]
    assert [es.get_event_by_alternate_id(a).id for _, a in picks] == [f"c0-{eid}" for eid, _ in picks]
    assert [es.get_event_by_id(f"c0-{eid}").alternate_id for eid, _ in picks] == [a for _, a in picks]
    found = es.find_alternate_hashes([hash64(a) for _, a in picks] + [12345])
    assert found == {hash64(a): f"c0-{eid}" for eid, a in picks}
    assert es.alternate_id_count() == len(with_alt)
    es.close()
    # reopen: the trailers are read from the segment files as they are
    es2 = sg.DurableEventStore(str(tmp_path / "es"), direct=False)
    c = DateRangeSearchCriteria(page_size=0)
    r = es2.list_events("Measurement", "Area", ["area-0"], c)
    assert (r.num_results, [(e.id, e.event_date) for e in r.results]) == \
        _brute(blocks, asg, "Measurement", "Area", {"area-0"}, c)
    # a segment file retention deletes while a lookup holds the block table: its candidates are
    # dropped (those ids are no longer stored), the lookup does not fail
    ents = es2.seg.index_tr()[0]
    gone = int(ents["file"][0])
    real = es2.seg.file_path
    es2.seg.file_path = lambda f: None if int(f) == gone else real(f)
    found2 = es2.find_alternate_hashes([hash64(a) for _, a in picks])
    assert set(found2.items()) <= set(found.items())
    es2.list_events("Measurement", "Assignment", ["asg-3"], DateRangeSearchCriteria(page_size=0))
    es2.seg.file_path = real
    es2.close()


def test_blocks_without_trailers_are_scanned(tmp_path):
    """Blocks from a writer that built no index trailer (an older store, a foreign producer) are
    answered by decoding them: same results as the indexed blocks."""
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    es, asg, blocks, exp_all = _ctx_store_blocks(tmp_path, n_blocks=3, trailers=False)
    assert es.index_stats()["indexed"] == 0
    for ix, ents in (("Assignment", ["asg-3"]), ("Area", ["area-1"]), ("Customer", ["cust-2"])):
        for c in (DateRangeSearchCriteria(page_size=0), DateRangeSearchCriteria(page_size=9)):
            r = es.list_events("Measurement", ix, ents, c)
            assert (r.num_results, [(e.id, e.event_date) for e in r.results]) == \
                _brute(blocks, asg, "Measurement", ix, set(ents), c)
    eid, alt = [(e, a) for e, a in exp_all if a is not None][17]
    assert es.get_event_by_alternate_id(alt).id == f"c0-{eid}"
    es.close()


def test_reopen_after_retention_deleted_a_file(tmp_path):
    """with retention deleting the oldest segment file between runs, every remaining block
    still answers from its own trailer (trailers live inside the block record: nothing keyed by
    process-local file ids, nothing left behind)."""
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    d = str(tmp_path / "es")
    ctx_tab = np.array([[i, i % 3, i % 2, i % 5] for i in range(40)], np.int32)
    asg = {i: [f"asg-{i}", f"dev-{i}", f"cust-{i % 3}", f"area-{i % 2}", f"asset-{i % 5}"] for i in range(40)}
    es = sg.DurableEventStore(d, direct=False, rotate_bytes=1 << 16)
    n0, kept = 0, []
    rng = np.random.default_rng(1)
    for b in range(6):
        rows, recs, spans, raw = synth_rows(1500, seed=50 + b)
        rows["assignment"] = np.sort(rng.integers(0, 40, len(rows)))
        blk = sg.encode_block(rows, recs, spans, raw, index=True, ctx=ctx_tab)
        sg.seal(blk, n0, 1_700_000_100_000 + b, 0xc0, 0, 1)
        es.wait(es.add_encoded(blk, asg=asg))
        kept.append((blk.copy(), n0))
        n0 += len(rows)
    es.close()
    files = sorted(f for f in os.listdir(d) if f.endswith(".sweg"))
    assert len(files) >= 3
    os.remove(os.path.join(d, files[0]))                 # retention, while the store was closed
    es2 = sg.DurableEventStore(d, direct=False)
    live = {int(e["first_seq"]) for e in es2.seg.index()}
    blocks = [(b, n) for b, n in kept if n in live]
    assert 0 < len(blocks) < 6
    c = DateRangeSearchCriteria(page_size=0)
    for ix, ents in (("Assignment", ["asg-7"]), ("Area", ["area-1"])):
        r = es2.list_events("Measurement", ix, ents, c)
        assert (r.num_results, [(e.id, e.event_date) for e in r.results]) == \
            _brute(blocks, asg, "Measurement", ix, set(ents), c)
    es2.close()


def test_point_fetch_equals_page_decode(tmp_path):
    """The store's native point reads (swseg_fetch_rows: a pass over the leading rows of a page, not
    a decode of the page) return exactly what decoding the whole page gives, strings included, in
    request order -- duplicates and several rows of one page included."""
    es, _, blocks, _ = _ctx_store_blocks(tmp_path, n_blocks=3, rows_per=2500)
    t = next(iter(es._boot_tables().values()))
    rng = np.random.default_rng(4)
    bis = rng.integers(0, t["n"], 200)
    rows = np.array([rng.integers(0, int(t["ents"][b]["n_rows"])) for b in bis])
    bis, rows = np.concatenate([bis, bis[:30], [0, 0]]), np.concatenate([rows, rows[:30] ^ 1, [0, 0]])
    got = es._fetch(t, bis, rows)
    for i, (b, r) in enumerate(zip(bis.tolist(), rows.tolist())):
        d = sg.decode_block(blocks[b][0], pages=(r // 1024, r // 1024 + 1))
        k = r - d["row0"]
        for col in ("etype", "level", "date", "asg", "name", "v0", "v1", "v2", "flags"):
            assert got[col][i] == d[col][k] or (np.isnan(got[col][i]) and np.isnan(d[col][k])), (col, b, r)
        assert sg.row_strings(got, i) == sg.row_strings(d, k)
        assert es._materialize(got, i).id == f"c0-{blocks[b][1] + r}"
    es.close()


def test_trailer_copies_in_memory_and_cap(tmp_path):
    """The segment store holds each block's index trailer in memory and, while the block is recent,
    its scan image (page headers + leading columns) -- made while the block is written, trailers on
    recovery too; beyond the caps the oldest copies are dropped and the reads fall back to the files
    -- same answers either way."""
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    es, _, blocks, exp_all = _ctx_store_blocks(tmp_path, n_blocks=4, rows_per=2000)
    with es.seg.lease():
        ents, ta, tl, ba = es.seg.index_tr()
        assert len(ents) == 4 and (ta != 0).all() and (tl > 0).all() and (ba != 0).all()
        for (blk, _), n, t, b in zip(blocks, tl.tolist(), ta.tolist(), ba.tolist()):
            toff = sg.trailer_offset(blk)
            assert n == len(blk) - toff
            assert np.array_equal(np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(t)), blk[toff:])
            npg = int(blk[:64].view(sg.HDR)[0]["n_pages"])
            io = np.ctypeslib.as_array((ctypes.c_uint32 * (2 + npg)).from_address(b))
            pt = blk[64:64 + 4 * (npg + 1)].view(np.uint32)
            assert io[0] == npg
            for p in range(npg):          # each page's first 256 bytes (header + leading columns)
                img = np.ctypeslib.as_array((ctypes.c_uint8 * 256).from_address(b + int(io[2 + p])))
                assert np.array_equal(img, blk[int(pt[p]):int(pt[p]) + 256])
    crit = DateRangeSearchCriteria(page_size=50)
    want = es.list_events("Measurement", "Area", ["area-1"], crit)
    want_a = es.list_events("Measurement", "Assignment", ["asg-3"], crit)
    alt = next(a for _, a in exp_all[::-1] if a is not None)
    want_alt = es.get_event_by_alternate_id(alt).id

    def same():
        got = es.list_events("Measurement", "Area", ["area-1"], crit)
        assert (got.num_results, [e.id for e in got.results]) == (want.num_results, [e.id for e in want.results])
        got = es.list_events("Measurement", "Assignment", ["asg-3"], crit)
        assert (got.num_results, [e.id for e in got.results]) == (want_a.num_results, [e.id for e in want_a.results])
        assert es.get_event_by_alternate_id(alt).id == want_alt

    es.seg.mem_caps(-1, 2 * (1 << 20))                   # scan images: the newest two (1 MiB slots)
    _, ta2, _, ba2 = es.seg.index_tr()
    assert (ba2[:2] == 0).all() and (ba2[2:] != 0).all() and (ta2 != 0).all()
    same()
    es.seg.mem_caps(int(tl[-1]), 0)                      # no scan images, one trailer copy
    _, ta3, _, ba3 = es.seg.index_tr()
    assert (ba3 == 0).all() and (ta3[:-1] == 0).all() and ta3[-1] != 0
    same()
    d = es.dir
    es.close()
    es2 = sg.DurableEventStore(d, direct=False)           # recovery copies the trailers again
    _, ta4, _, _ = es2.seg.index_tr()
    assert (ta4 != 0).all()
    got = es2.list_events("Measurement", "Area", ["area-1"], crit)
    assert [e.id for e in got.results] == [e.id for e in want.results]
    es2.close()


def test_read_lease_defers_reclaiming_copies(tmp_path):
    """A copy dropped while a read lease is held stays readable until the lease ends."""
    es, _, blocks, _ = _ctx_store_blocks(tmp_path, n_blocks=2, rows_per=1500)
    with es.seg.lease():
        _, _, _, ba = es.seg.index_tr()
        b0 = int(ba[0])
        before = np.ctypeslib.as_array((ctypes.c_uint8 * 4096).from_address(b0)).copy()
        es.seg.mem_caps(-1, 0)                           # drop every scan image
        assert (es.seg.index_tr()[3] == 0).all()
        assert np.array_equal(np.ctypeslib.as_array((ctypes.c_uint8 * 4096).from_address(b0)), before)
    es.close()


def test_high_cardinality_dimensions_route_through_assignments(tmp_path):
    """dimensions whose context ids pass SIX_CTX_MAX (an asset per device, 10K
    customers) are not in the trailers' key tables; their listings go through the id's assignments
    (one native pass over every block's page zone maps, one scan of those pages) and answer exactly
    like decoding every block -- totals, order, paging, date ranges."""
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    es, asg, blocks, _ = _ctx_store_blocks(tmp_path, n_blocks=4, rows_per=20000, dates="increasing",
                                           n_asg=20000, n_cust=10000, n_area=31, n_asset=20000)
    # clustered blocks: their pages without generated rows are binary-searched by assignment
    for blk, _ in blocks:
        off = sg.trailer_offset(blk)
        assert int(blk[off:off + 128].view(sg.IX_HDR)[0]["flags"]) & sg.IX_F_CLUSTERED
    t0 = 1_700_000_000_000
    crits = [DateRangeSearchCriteria(page_size=0), DateRangeSearchCriteria(page_size=100),
             DateRangeSearchCriteria(page_number=2, page_size=3),
             DateRangeSearchCriteria(page_size=10, start_date=t0 + 1_000_000, end_date=t0 + 2_500_000)]
    n = 0
    for t in ("Measurement", "Location"):
        for ix, ents in (("Asset", ["asset-17"]), ("Asset", ["asset-5", "asset-19999"]), ("Customer", ["cust-42"]),
                         ("Customer", ["cust-9999", "cust-3"]), ("Area", ["area-4"]), ("Asset", ["asset-none"])):
            for c in crits:
                r = es.list_events(t, ix, ents, c)
                got = (r.num_results, [(e.id, e.event_date) for e in r.results])
                want = _brute(blocks, asg, t, ix, set(ents), c)
                assert got == want, (t, ix, ents, c)
                n += want[0]
    assert n > 50
    es.close()


def test_trailer_clustered_flag():
    """SIX_F_CLUSTERED is set only when the data proves it: persisted rows first, their assignments
    non-decreasing, generated rows after them (readers then binary-search those pages)."""
    rows, recs, spans, raw = synth_rows(3000, seed=5)
    gen = (recs["fp_lo"] == 0) & (recs["fp_hi"] == 0)
    assert gen.any() and (~gen).any()

    def flag(o):
        blk = sg.encode_block(rows[o], recs[o], spans[o], raw, index=True)
        off = sg.trailer_offset(blk)
        return int(blk[off:off + 128].view(sg.IX_HDR)[0]["flags"]) & sg.IX_F_CLUSTERED

    assert flag(np.lexsort((rows["assignment"], gen))) == 1                  # engine order
    assert flag(np.argsort(rows["assignment"], kind="stable")) == 0          # generated rows interleaved
    assert flag(np.arange(len(rows))) == 0                                   # unsorted
