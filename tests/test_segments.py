"""Durable columnar event segments: block codec (csrc/include/swseg.h, csrc/native/swseg.cpp), the
native segment store (group commit, recovery, retention) and the DurableEventStore over it.  The
MI355X encoder is checked against the CPU encoder bit for bit in tests/test_gpu_segments.py."""
from __future__ import annotations

import os

import numpy as np
import pytest

from sitewhere_amd.models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE, NO_NAME, OUT_REC
from sitewhere_amd.persistence import segments as sg


def synth_rows(n, seed=0, full_precision=False):
    """Rows shaped like the engine's persisted output: decimal sensor values, 6-decimal coordinates,
    alerts, presence state changes; some alternate ids."""
    rng = np.random.default_rng(seed)
    et = rng.choice([EV_MEASUREMENT, EV_LOCATION, EV_ALERT, EV_STATE_CHANGE], n, p=[0.68, 0.25, 0.05, 0.02])
    rows = np.zeros(n, OUT_REC)
    rows["etype"] = et
    rows["event_date"] = 1_700_000_000_000 + rng.integers(0, 60_000, n)
    rows["assignment"] = rng.integers(0, 1 << 20, n)
    mx, loc, al = et == EV_MEASUREMENT, et == EV_LOCATION, et == EV_ALERT
    rows["name_id"] = np.where(loc, NO_NAME, rng.integers(0, 20, n))
    rows["v0"] = np.where(mx, rng.integers(0, 100000, n) / 100.0, 0.0)
    lat = 33.0 + rng.integers(0, 2_000_000, n) / 1e6
    lon = -85.0 + rng.integers(0, 2_000_000, n) / 1e6
    if full_precision:
        lat = 33.0 + 2.0 * rng.random(n)
        lon = -85.0 + 2.0 * rng.random(n)
    rows["v0"] = np.where(loc, lat, rows["v0"])
    rows["v1"] = np.where(loc, lon, 0.0)
    rows["level"] = np.where(al, rng.integers(0, 4, n), 0)
    v2 = np.where(loc, 10.0, 0.0)
    alt = np.where(rng.random(n) < 0.5, rng.integers(1, 1 << 62, n).astype(np.uint64) * 3, 0).astype(np.uint64)
    return rows, v2, alt


def check_roundtrip(rows, v2, alt):
    blk = sg.encode_block(rows, v2, alt)
    sg.seal(blk, 1000, 1_700_000_100_000, 7, 0, 1)
    assert sg.verify(blk) == 0
    c = sg.decode_block(blk)
    assert c["header"]["n_rows"] == len(rows) and c["header"]["first_seq"] == 1000
    for col, key in (("etype", "etype"), ("level", "level"), ("date", "event_date"), ("asg", "assignment"),
                     ("name", "name_id")):
        np.testing.assert_array_equal(c[col], rows[key], err_msg=col)
    # values bit for bit (exceptions included)
    np.testing.assert_array_equal(c["v0"].view(np.uint64), rows["v0"].view(np.uint64))
    np.testing.assert_array_equal(c["v1"].view(np.uint64), rows["v1"].view(np.uint64))
    np.testing.assert_array_equal(c["v2"].view(np.uint64), np.asarray(v2, np.float64).view(np.uint64))
    np.testing.assert_array_equal(c["alt"], alt)
    return blk


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 5000])
def test_block_roundtrip(n):
    rows, v2, alt = synth_rows(n, seed=n)
    check_roundtrip(rows, v2, alt)


def test_block_compresses_decimal_data():
    rows, v2, alt = synth_rows(100_000, seed=1)
    alt[:] = 0
    blk = check_roundtrip(rows, v2, alt)
    assert len(blk) / len(rows) < 9.0, len(blk) / len(rows)       # vs 32 B OUT_REC + 8 B elevation


def test_block_exceptions_are_lossless():
    rows, v2, alt = synth_rows(20_000, seed=2, full_precision=True)
    rows["v0"][::7] = np.where(rows["etype"][::7] == EV_MEASUREMENT, np.nan, rows["v0"][::7])
    rows["v0"][1::11] = np.where(rows["etype"][1::11] == EV_MEASUREMENT, -0.0, rows["v0"][1::11])
    rows["v1"][::13] = np.where(rows["etype"][::13] == EV_LOCATION, np.inf, rows["v1"][::13])
    check_roundtrip(rows, v2, alt)


def test_corruption_detected():
    rows, v2, alt = synth_rows(3000, seed=3)
    blk = check_roundtrip(rows, v2, alt)
    for pos in (10, 64 + 4, len(blk) // 2, len(blk) - 8):
        bad = blk.copy()
        bad[pos] ^= 0x40
        assert sg.verify(bad) != 0, pos


def _store_blocks(st, nblocks, rows_per=3000):
    seq = 0
    blocks = []
    for b in range(nblocks):
        rows, v2, alt = synth_rows(rows_per, seed=100 + b)
        blk = sg.encode_block(rows, v2, alt)
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
        f.seek(size - 3000)
        f.write(os.urandom(3000))
    st2 = sg.SegmentStore(d)
    idx = st2.index()
    assert list(idx["first_seq"]) == [b[0] for b in blocks[:-1]]
    assert os.path.getsize(path) < size        # truncated at the last good block
    # appends continue after recovery
    rows, v2, alt = synth_rows(100, seed=9)
    blk = sg.encode_block(rows, v2, alt)
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
    rows, v2, alt = synth_rows(4000, seed=5)
    rows["assignment"] = np.arange(4000) % 50
    asg = {i: [f"asg-{i}", f"dev-{i}", f"cust-{i % 3}", f"area-{i % 2}", None] for i in range(50)}
    names = {i: f"mx.metric{i}" for i in range(20)}
    blk = sg.encode_block(rows, v2, alt)
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
    ev = res.results[0]
    es.close()
    es2 = sg.DurableEventStore(d)                         # restart: everything from disk
    again = es2.list_events("Measurement", "Assignment", ["asg-7"], DateRangeSearchCriteria(page_size=0))
    assert [e.id for e in again.results] == [e.id for e in res.results]
    assert es2.get_event_by_id(ev.id).value == ev.value
    hashes = alt[alt != 0][:5]
    found = es2.find_alternate_hashes(hashes)
    assert set(found) == set(int(h) for h in hashes)
    assert all(v.startswith("b0-") for v in found.values())
    # a new engine incarnation restarts its sequences and indices: its block is not a replay, and
    # its dictionary does not rewrite the first boot's
    rows2 = rows.copy()
    rows2["assignment"] = (np.arange(4000) + 25) % 50
    blk2 = sg.encode_block(rows2, v2, alt)
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
        rows, v2, alt = synth_rows(20000 + 1000 * k, seed=k)
        blk = sg.encode_block(rows, v2, alt)
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
