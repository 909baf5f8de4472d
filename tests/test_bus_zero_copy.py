"""Zero-copy records in the commit log (csrc/native/swnative.cpp swlog_append_external/view/hold).

A producer whose record bytes already sit in DMA-able memory publishes them in place; consumers
read them in place (the MI355X engine DMAs a raw batch straight out of the topic) or copy them
like any other record.  Retention releases the buffers back to their owner, and a hold keeps
in-flight records from being released."""
from __future__ import annotations

import numpy as np
import pytest

from sitewhere_amd.bus.log import EventBus

H = 0


def _ext(bus, topic, payload: bytes, key: bytes = b"", released=None):
    buf = np.frombuffer(key + payload, np.uint8).copy()
    off = bus.append_external(topic, 0, buf, buf.ctypes.data, buf.nbytes, key_len=len(key), ts=123,
                              on_release=None if released is None else released.append)
    return buf, off


def test_external_record_reads_in_place_and_by_copy():
    bus = EventBus(default_partitions=1)
    bus.append("t", 0, [(b"k0", b"copied-before")])
    buf, off = _ext(bus, "t", b"zero-copy-value", key=b"dev-1")
    bus.append("t", 0, [(None, b"copied-after")])
    assert off == 1 and bus.end_offset("t", 0) == 3
    ptr, n, ts = bus.view("t", 0, 1)
    assert ptr == buf.ctypes.data + H + 5 and n == len(b"zero-copy-value") and ts == 123
    recs = bus.read("t", 0, 0)
    assert [(r.key, r.value) for r in recs] == [(b"k0", b"copied-before"), (b"dev-1", b"zero-copy-value"),
                                                (None, b"copied-after")]
    buf[H + 5] = ord("Z")                                   # the log reads the caller's memory in place
    assert bus.read("t", 0, 1, 1)[0].value == b"Zero-copy-value"
    assert bus.view("t", 0, 7) is None


def test_retention_releases_external_buffers_and_hold_defers_it():
    bus = EventBus(default_partitions=1)
    bus.topic("r")
    bus.set_retention("r", 1)                               # keep as little as possible
    rel = []
    bufs = [_ext(bus, "r", bytes([i]) * 1000, released=rel)[0] for i in range(2)]
    bus.hold("r", 0, 2)                                     # a consumer has records >= 2 in flight
    b2, off2 = _ext(bus, "r", b"x" * 1000, released=rel)
    b3, off3 = _ext(bus, "r", b"y" * 1000, released=rel)
    bus.reclaim()
    assert {id(o) for o in rel} == {id(b) for b in bufs}    # handed back to their pool
    assert bus.begin_offset("r", 0) == 2 and bus.view("r", 0, off2) is not None
    bus.hold("r", 0, None)                                  # released: retention catches up
    bus.reclaim()
    assert {id(o) for o in rel[2:]} == {id(b2)}
    assert bus.begin_offset("r", 0) == off3
    assert bus.read("r", 0, off3)[0].value == b"y" * 1000
    # owners without a pool are dropped by the log once released
    import weakref
    tmp = np.frombuffer(b"z" * 100, np.uint8).copy()
    ref = weakref.ref(tmp)
    bus.append_external("r", 0, tmp, tmp.ctypes.data, tmp.nbytes)
    del tmp
    _ext(bus, "r", b"w" * 1000)                             # pushes the previous record out
    bus.reclaim()
    assert ref() is None


def test_zero_copy_views_through_a_consumer():
    bus = EventBus(default_partitions=1)
    vals = [bytes([65 + i]) * (10 + i) for i in range(5)]
    keep = [_ext(bus, "v", v)[0] for v in vals]
    bus.append("v", 0, [(b"k", b"copied")])
    c = bus.consumer("g", ["v"])
    got = c.poll(100, views=True)[("v", 0)]
    assert [bytes(r.value) for r in got] == vals + [b"copied"]
    assert isinstance(got[0].value, memoryview) and got[0].value.readonly
    assert np.frombuffer(got[0].value, np.uint8).ctypes.data == keep[0].ctypes.data


def test_bytes_values_are_published_by_reference():
    bus = EventBus(default_partitions=1)
    v = b"immutable-columnar-batch" * 100
    off = bus.append_bytes("b", 0, v, ts=7)
    ptr, n, ts = bus.view("b", 0, off)
    import ctypes
    assert n == len(v) and ts == 7 and ctypes.string_at(ptr, n) == v
    assert ptr == ctypes.cast(ctypes.c_char_p(v), ctypes.c_void_p).value     # the bytes object itself
    assert bus.read("b", 0, off)[0].value == v


def test_durable_partitions_copy_zero_copy_records(tmp_path):
    """A durable partition writes a zero-copy record to its files (a copy) and releases the owner
    at once; the record survives a reopen."""
    released = []
    bus = EventBus(str(tmp_path / "log"), default_partitions=1)
    buf, off = _ext(bus, "d", b"value", key=b"k", released=released)
    assert off == 0 and bus.end_offset("d", 0) == 1 and not bus._ext and len(released) == 1
    buf[:] = 0                                  # the owner is free: the log holds its own copy
    r = bus.read("d", 0, 0)[0]
    assert (r.key, r.value) == (b"k", b"value")
    bus.close()
    bus = EventBus(str(tmp_path / "log"), default_partitions=1)
    assert bus.read("d", 0, 0)[0].value == b"value"
    bus.close()


def test_varint_framing_rejects_truncated_and_overlong():
    import numpy as np
    import pytest as _pt
    from sitewhere_amd.pipeline.framing import offsets_from_varint, varint_lengths
    ok = varint_lengths(np.array([0, 5, 300, 70000], np.int64))
    assert list(offsets_from_varint(ok)) == [0, 5, 300, 70000]
    with _pt.raises(ValueError):
        offsets_from_varint(np.concatenate([ok, np.array([0x85], np.uint8)]))      # truncated
    with _pt.raises(ValueError):
        offsets_from_varint(np.array([0xff] * 6 + [0x01], np.uint8))               # > 5 bytes


def test_native_varint_offsets_match_reference():
    """RawBatch.offsets (one native pass, sw_varint_offsets) == the numpy reference, and framing
    errors (truncated / over-long / wrong count / wrong total) are rejected."""
    import numpy as np
    import pytest as _pt
    from sitewhere_amd.pipeline.bus_io import RawBatch
    from sitewhere_amd.pipeline.framing import offsets_from_varint, varint_lengths
    rng = np.random.default_rng(3)
    lens = rng.choice([0, 1, 90, 127, 128, 300, 16383, 16384, 70000], 5000).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    st = varint_lengths(offs)
    b = RawBatch(len(lens), int(offs[-1]), None, lens=st)
    np.testing.assert_array_equal(b.offsets(), offsets_from_varint(st))
    for bad, n, total in ((st[:-1], len(lens), int(offs[-1])), (st, len(lens) + 1, int(offs[-1])),
                          (st, len(lens), int(offs[-1]) + 1),
                          (np.array([0xff] * 6 + [0x01], np.uint8), 1, 1)):
        with _pt.raises(ValueError):
            RawBatch(n, total, None, lens=bad).offsets()
