"""Zero-copy records in the commit log (csrc/native/swnative.cpp swlog_append_external/view/hold).

A producer whose record bytes already sit in DMA-able memory publishes them in place; consumers
read them in place (the MI355X engine DMAs a raw batch straight out of the topic) or copy them
like any other record.  Retention releases the buffers back to their owner, and a hold keeps
in-flight records from being released."""
from __future__ import annotations

import numpy as np
import pytest

from sitewhere_amd.bus.log import EventBus

H = EventBus.REC_HDR


def _ext(bus, topic, payload: bytes, key: bytes = b""):
    buf = np.zeros(H + len(key) + len(payload), np.uint8)
    buf[H:H + len(key)] = np.frombuffer(key, np.uint8) if key else []
    buf[H + len(key):] = np.frombuffer(payload, np.uint8)
    off = bus.append_external(topic, 0, buf, buf.ctypes.data, buf.nbytes, key_len=len(key), ts=123)
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
    bufs = [_ext(bus, "r", bytes([i]) * 1000)[0] for i in range(2)]
    bus.hold("r", 0, 2)                                     # a consumer has records >= 2 in flight
    b2, off2 = _ext(bus, "r", b"x" * 1000)
    b3, off3 = _ext(bus, "r", b"y" * 1000)
    got = bus.reclaim()
    assert [id(o) for o in got] == [id(bufs[1]), id(bufs[0])] or {id(o) for o in got} == {id(b) for b in bufs}
    assert bus.begin_offset("r", 0) == 2 and bus.view("r", 0, off2) is not None
    bus.hold("r", 0, None)                                  # released: retention catches up
    assert {id(o) for o in bus.reclaim()} == {id(b2)}
    assert bus.begin_offset("r", 0) == off3
    assert bus.read("r", 0, off3)[0].value == b"y" * 1000


def test_durable_partitions_refuse_zero_copy(tmp_path):
    bus = EventBus(str(tmp_path / "log"), default_partitions=1)
    with pytest.raises(RuntimeError, match="durable"):
        _ext(bus, "d", b"v")
    assert bus.end_offset("d", 0) == 0 and not bus._ext
    bus.close()
