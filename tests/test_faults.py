"""Delivery semantics under injected faults: consumer redelivery after handler
failures, poison-batch skipping, buffered-writer retries, and the seeded fault injector itself."""
from __future__ import annotations

import threading
import time
from types import SimpleNamespace

import pytest

from sitewhere_amd.bus.log import EventBus
from sitewhere_amd.models.domain import DeviceMeasurement
from sitewhere_amd.persistence.events import BufferedEventWriter, MemoryEventStore
from sitewhere_amd.runtime.consumers import BusConsumer
from sitewhere_amd.utils.faults import FaultInjector, InjectedFault


def _engine(bus):
    return SimpleNamespace(ms=SimpleNamespace(instance=SimpleNamespace(bus=bus), producer=bus.producer()))


def _wait(cond, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end and not cond():
        time.sleep(0.01)
    return cond()


@pytest.mark.parametrize("threads", [0, 3])
def test_consumer_redelivers_failed_batches(threads):
    bus = EventBus(default_partitions=2)
    prod = bus.producer()
    for i in range(300):
        prod.send("t", f"k{i % 7}", str(i).encode())
    seen, lock = [], threading.Lock()
    fi = FaultInjector(seed=3)

    def handler(recs):
        if fi._roll(0.4 if threads == 0 else 0.15):      # threaded: a batch needs every slice to succeed
            raise InjectedFault("transient")
        with lock:
            seen.extend(int(r.value) for r in recs)
    c = BusConsumer(_engine(bus), "c", ["t"], handler, threads=threads, max_records=40, group="g-redeliver")
    c.max_attempts = 1000
    c.start(None)
    try:
        assert _wait(lambda: set(seen) == set(range(300)), 30)
        assert c.retries > 0 and c.failures > 0 and c.dropped == 0
        # committed positions cover everything once the last batch succeeded
        assert _wait(lambda: sum(bus.committed("g-redeliver", "t", p) for p in range(2)) == 300)
    finally:
        c._stop.set()
        c._t.join(5)
    # a fresh member of the group resumes after the committed positions: nothing redelivered
    c2 = bus.consumer("g-redeliver", ["t"])
    assert not any(c2.poll(50).values())


def test_consumer_skips_poison_batch():
    bus = EventBus(default_partitions=1)
    prod = bus.producer()
    for i in range(30):
        prod.send("p", "k", str(i).encode())
    ok = []

    def handler(recs):
        if any(r.value == b"13" for r in recs):
            raise ValueError("poison")
        ok.extend(int(r.value) for r in recs)
    c = BusConsumer(_engine(bus), "c", ["p"], handler, max_records=10, group="g-poison")
    c.max_attempts = 3
    c.start(None)
    try:
        assert _wait(lambda: c.dropped == 10 and len(ok) == 20, 30)
        assert sorted(ok) == list(range(10)) + list(range(20, 30))
        assert c.retries == 2
        dl = bus.consumer("dlq-reader", ["p.dead-letter"])
        got = []
        assert _wait(lambda: got.extend(r.value for rs in dl.poll(50).values() for r in rs) or len(got) == 10)
        assert sorted(int(v) for v in got) == list(range(10, 20))
        # once the cause is fixed, the parked records go back onto the topic and are processed
        from sitewhere_amd.runtime.consumers import replay_dead_letter
        poisoned = {b"13"}
        handler_ok = ok

        def fixed(recs):
            handler_ok.extend(int(r.value) for r in recs if r.value not in poisoned)
        c.handler = fixed
        poisoned.clear()
        assert replay_dead_letter(bus, "p") == 10
        assert _wait(lambda: sorted(ok) == list(range(30)))
        assert replay_dead_letter(bus, "p") == 0
    finally:
        c._stop.set()
        c._t.join(5)


def _events(n, prefix):
    out = []
    for i in range(n):
        e = DeviceMeasurement(name="m", value=float(i))
        e.id, e.alternate_id, e.device_assignment_id, e.event_date = f"{prefix}{i}", f"{prefix}alt{i}", "a", i
        out.append(e)
    return out


def test_buffered_writer_retries_until_store_recovers():
    store = MemoryEventStore()
    w = BufferedEventWriter(store, chunk=50, interval_ms=20)
    with FaultInjector(seed=1) as fi:
        fi.fail(store, "add_events", 1.0)                  # store down
        evs = _events(120, "bw")
        w.add(evs)
        assert w.pending_alternate("bwalt5") is evs[5]     # dedup sees buffered events
        assert _wait(lambda: w.failed_writes >= 3, 10)
        assert store.count() == 0
    assert _wait(lambda: store.count() == 120, 10)         # store back: everything written once
    assert _wait(lambda: w.pending_alternate("bwalt5") is None)
    w.close()


def test_fault_injector_is_seeded_and_restores():
    class Obj:
        def f(self):
            return 1
    o = Obj()
    runs = []
    for _ in range(2):
        with FaultInjector(seed=42) as fi:
            fi.fail(o, "f", 0.5)
            seq = []
            for _ in range(50):
                try:
                    seq.append(o.f())
                except InjectedFault:
                    seq.append(0)
            runs.append(seq)
        assert "f" not in o.__dict__ and o.f() == 1
    assert runs[0] == runs[1] and 0 < sum(runs[0]) < 50
    with FaultInjector(seed=0) as fi:
        fi.drop(o, "f", 1.0, empty=[])
        assert o.f() == []


def test_control_plane_consumer_never_dead_letters():
    """max_attempts=None (registry change feed, registration): a failing batch is retried until it
    succeeds -- skipping it would leave the consumer's mirror diverged from device management."""
    bus = EventBus(default_partitions=1)
    prod = bus.producer()
    for i in range(5):
        prod.send("cp", "k", str(i).encode())
    seen, fails = [], [0]

    def handler(recs):
        if fails[0] < 14:
            fails[0] += 1
            raise InjectedFault("model store down")
        seen.extend(int(r.value) for r in recs)
    c = BusConsumer(_engine(bus), "c", ["cp"], handler, max_records=10, group="g-cp", max_attempts=None)
    c.alert_every = 5
    c._stop.wait = lambda t: time.sleep(min(t, 0.01))      # keep the backoff short for the test
    c.start(None)
    try:
        assert _wait(lambda: seen == list(range(5)), 20)
        assert c.dropped == 0 and c.retries == 14
        assert bus.end_offset("cp.dead-letter", 0) == 0
    finally:
        c._stop.set()
        c._t.join(5)


def test_retry_from_rewinds_before_the_current_batch():
    """A handler may ask to re-read from an earlier offset (work handed off for batch k failed while
    batch k+1 is being handled): the consumer seeks there, and that never counts as a poison batch."""
    from sitewhere_amd.runtime.consumers import RetryFrom
    bus = EventBus(default_partitions=1)
    prod = bus.producer()
    for i in range(6):
        prod.send("rw", "k", str(i).encode())
    reads, state = [], {"rewound": False}

    def handler(recs):
        reads.extend(r.offset for r in recs)
        if recs[0].offset == 3 and not state["rewound"]:
            state["rewound"] = True
            raise RetryFrom({("rw", 0): 1}, InjectedFault("store of offset 1 failed"))
    c = BusConsumer(_engine(bus), "c", ["rw"], handler, max_records=3, group="g-rw")
    c.max_attempts = 1                                      # a RetryFrom must not dead-letter
    c.start(None)
    try:
        assert _wait(lambda: bus.committed("g-rw", "rw", 0) == 6, 10)
        assert reads[:6] == [0, 1, 2, 3, 4, 5] and reads[6:9] == [1, 2, 3]
        assert c.rewinds == 1 and c.dropped == 0
    finally:
        c._stop.set()
        c._t.join(5)
