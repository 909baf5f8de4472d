"""No silent loss: producers wait for a protected topic's consumer instead of retention dropping
what it has not read (``EventBus.protect``).

Reference: the MQTT receiver acknowledges a message only after handing it off
(``MqttInboundEventReceiver.java:166-215``), so a slow pipeline throttles publishers.  Here the
in-process log's memory retention would drop the oldest segments of a lagging topic; a protected
topic keeps every record its consumer group has not committed and makes producers wait for room."""
from __future__ import annotations

import threading
import time

import pytest

from sitewhere_amd.bus.log import BackpressureTimeout, EventBus

REC = 200 << 10          # 200 KB records, 1 MB retention: ~5 records fit


def _consume_slowly(bus, group, topic, n, got, delay=0.01):
    c = bus.consumer(group, [topic], auto_offset_reset="earliest")
    while len(got) < n:
        for recs in c.poll(200, 4).values():
            for r in recs:
                got.append(r.offset)
                time.sleep(delay)
            c.commit()
    c.close()
    return c


def test_protected_topic_throttles_producer_and_loses_nothing():
    bus = EventBus(default_partitions=1, retention_bytes=1 << 20)
    bus.protect("slow", "raw", max_wait_s=30)
    got: list = []
    th = threading.Thread(target=_consume_slowly, args=(bus, "slow", "raw", 60, got))
    th.start()
    t0 = time.time()
    for i in range(60):                       # 12 MB into a 1 MB topic
        bus.append_bytes("raw", 0, bytes([i % 256]) * REC)      # zero-copy: a segment per record
    th.join(60)
    assert got == list(range(60))             # every record read, in order, none skipped
    assert bus.backpressure_waits > 0 and time.time() - t0 > 0.3     # the producer was held back
    bus.close()


def test_unprotected_topic_drops_and_counts_the_loss():
    bus = EventBus(default_partitions=1, retention_bytes=1 << 20)
    c = bus.consumer("late", ["raw"], auto_offset_reset="earliest")
    c.poll(10)
    for i in range(60):
        bus.append_bytes("raw", 0, b"x" * REC)
    seen = []
    while len(seen) + c.lost < 60:
        for recs in c.poll(100, 100).values():
            seen += [r.offset for r in recs]
    assert c.lost > 0 and len(seen) + c.lost == 60          # retention dropped them; counted
    c.close()
    bus.close()


def test_backpressure_times_out_instead_of_dropping():
    bus = EventBus(default_partitions=1, retention_bytes=1 << 20)
    bus.protect("stuck", "raw", max_wait_s=0.3)
    with pytest.raises(BackpressureTimeout):
        for _ in range(20):
            bus.append_bytes("raw", 0, b"y" * REC)
    assert bus.begin_offset("raw", 0) == 0                  # nothing was dropped
    bus.unprotect("stuck", "raw")
    bus.append("raw", 0, [(None, b"z" * REC)])              # unprotected again: no wait
    bus.close()


def test_event_source_requeues_payloads_the_bus_refused():
    """A raw batch that cannot be published (backpressure timeout) goes back into the source's
    buffer: the next flush publishes it -- no payload is lost on the way."""
    from types import SimpleNamespace

    from sitewhere_amd.services.event_sources import EventSourcesManager

    class _Bus:
        def __init__(self):
            self.fail, self.records = True, []

        def partitions(self, name):
            return 1

        def append_external(self, name, p, owner, ptr, n):
            if self.fail:
                raise BackpressureTimeout("full")
            self.records.append(owner.value())

    bus = _Bus()
    eng = SimpleNamespace(ms=SimpleNamespace(instance=SimpleNamespace(bus=bus)), config={})
    m = EventSourcesManager.__new__(EventSourcesManager)
    m.engine, m.t_raw = eng, "raw"
    m._raw_buf, m._raw_lock, m._pub_lock = [], threading.Lock(), threading.Lock()
    for i in range(10):
        m._raw_buf.append(b"p%d" % i)
    with pytest.raises(BackpressureTimeout):
        m.flush_raw()
    assert len(m._raw_buf) == 10              # nothing lost
    bus.fail = False
    m.flush_raw()
    assert len(bus.records) == 1 and not m._raw_buf
