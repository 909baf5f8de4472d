"""Azure Event Hubs over AMQP 1.0 (``edges/amqp10.py``, ``edges/eventhub.py``) against the in-process
stand-in (``edges/eventhub_server.py``).

Reference: ``EventHubInboundEventReceiver.java:60-174`` (EventProcessorHost: every partition of
the hub, offsets checkpointed per consumer group, partitions balanced over hosts)."""
from __future__ import annotations

import threading
import time
import uuid

import pytest

from sitewhere_amd.core.lifecycle import LifecycleProgressMonitor
from sitewhere_amd.edges import amqp10
from sitewhere_amd.edges.eventhub import CoordCheckpoints, EventHubAmqpReceiver, MemoryCheckpoints
from sitewhere_amd.edges.eventhub_server import EventHubServer


# Every delivery notifies this condition, so a wait wakes on the event that satisfies it (not on
# a poll tick).  The deadline only bounds a genuine failure: a loaded machine delays the
# receiver thread without changing what it must deliver.
_DELIVERED = threading.Condition()


class _Source:
    def __init__(self):
        self.got, self.lock = [], threading.Lock()

    def on_encoded_event_received(self, receiver, payload, md):
        with self.lock:
            self.got.append((bytes(payload), md))
        with _DELIVERED:
            _DELIVERED.notify_all()


def _wait(cond, t=60.0):
    end = time.time() + t
    with _DELIVERED:
        while not cond():
            left = end - time.time()
            if left <= 0:
                return False
            # link attach / credit changes do not deliver, so wake at least every 50 ms for them
            _DELIVERED.wait(min(left, 0.05))
    return True


def _receiver(srv, cps, **kw):
    r = EventHubAmqpReceiver(None, srv.hub, "RootManageSharedAccessKey", "secret", host="127.0.0.1", port=srv.port,
                             tls=False, checkpoints=cps, rebalance_s=0.2, checkpoint_every=5, **kw)
    r.source = _Source()
    return r


def test_codec_round_trip():
    v = [None, True, False, amqp10.UInt(0), amqp10.UInt(7), amqp10.UInt(70000), amqp10.ULong(1 << 40),
         amqp10.UByte(3), amqp10.UShort(513), -5, 1 << 40, 2.5, amqp10.Timestamp(1_700_000_000_000), "héllo",
         amqp10.Symbol("x-opt-offset"), b"\x00\x01" * 200, uuid.UUID(int=42), {"a": [1, 2, {"b": None}]},
         amqp10.Described(amqp10.ULong(0x75), b"data"), amqp10.Array(0xa3, [amqp10.Symbol("PLAIN")]),
         "x" * 300, list(range(300))]
    out = amqp10.decode_all(b"".join(amqp10.encode(x) for x in v))
    assert out[:-2] == v[:-2] and out[-2] == v[-2] and out[-1] == v[-1]
    assert isinstance(out[4], amqp10.UInt) and isinstance(out[6], amqp10.ULong) and isinstance(out[14], amqp10.Symbol)
    m = amqp10.Message(body=b"payload", annotations={amqp10.Symbol("x-opt-offset"): "42"},
                       app_properties={"k": 1})
    d = amqp10.Message.decode(m.encode())
    assert d.body == b"payload" and d.annotations["x-opt-offset"] == "42" and d.app_properties == {"k": 1}


def test_reads_every_partition_and_resumes_after_checkpoint():
    srv = EventHubServer(hub="telemetry", partitions=4).start()
    cps = MemoryCheckpoints()
    try:
        sent = {}
        for i in range(40):
            p = str(i % 4)
            sent.setdefault(p, []).append(f"ev-{i}".encode())
            srv.send(p, f"ev-{i}".encode(), key=f"dev-{i % 7}")
        r = _receiver(srv, cps)
        r.lifecycle_start(LifecycleProgressMonitor())
        assert r.partitions == ["0", "1", "2", "3"]            # from the $management node
        assert _wait(lambda: len(r.source.got) == 40)
        by_p = {}
        for body, md in r.source.got:
            by_p.setdefault(md["partition"], []).append(body)
            assert md["eventHub"] == "telemetry" and md["offset"] is not None
        assert by_p == sent                                    # every partition, in order
        r.lifecycle_stop(LifecycleProgressMonitor())           # checkpoints the last offsets
        assert set(cps.offsets) == {"0", "1", "2", "3"}
        for i in range(40, 48):
            srv.send(str(i % 4), f"ev-{i}".encode())
        r2 = _receiver(srv, cps)
        r2.lifecycle_start(LifecycleProgressMonitor())
        assert _wait(lambda: len(r2.source.got) == 8)
        # a sentinel behind each partition's events: once all four arrive, any replay of events
        # before the checkpoint (same partitions, earlier positions) would have arrived too
        for p in "0123":
            srv.send(p, f"end-{p}".encode())
        assert _wait(lambda: sum(b.startswith(b"end-") for b, _ in r2.source.got) == 4)
        assert sorted(b for b, _ in r2.source.got if not b.startswith(b"end-")) == \
            sorted(f"ev-{i}".encode() for i in range(40, 48))
        assert len(r2.source.got) == 12
        r2.lifecycle_stop(LifecycleProgressMonitor())
    finally:
        srv.stop()


def test_two_hosts_split_the_partitions():
    from sitewhere_amd.coord.store import Coordination
    srv = EventHubServer(hub="h", partitions=4).start()
    coord = Coordination()
    try:
        a = _receiver(srv, CoordCheckpoints(coord, "/t/eh"), host_name_prefix="a")
        a.lifecycle_start(LifecycleProgressMonitor())
        assert len(a.links) == 4
        b = _receiver(srv, CoordCheckpoints(coord, "/t/eh"), host_name_prefix="b")
        b.lifecycle_start(LifecycleProgressMonitor())
        assert _wait(lambda: len(a.links) == 2 and len(b.links) == 2)
        assert set(a.links) | set(b.links) == {"0", "1", "2", "3"}
        for i in range(20):
            srv.send(str(i % 4), f"x{i}".encode())
        assert _wait(lambda: len(a.source.got) + len(b.source.got) == 20)
        a.lifecycle_stop(LifecycleProgressMonitor())           # b takes the whole hub over
        assert _wait(lambda: len(b.links) == 4)
        for i in range(20, 24):
            srv.send(str(i % 4), f"x{i}".encode())
        assert _wait(lambda: len(b.source.got) >= 10 + 4)
        bodies = [p for p, _ in a.source.got + b.source.got]
        assert {f"x{i}".encode() for i in range(24)} <= set(bodies)
        b.lifecycle_stop(LifecycleProgressMonitor())
    finally:
        srv.stop()


def test_wrong_key_is_refused():
    srv = EventHubServer(hub="h", partitions=1).start()
    try:
        with pytest.raises(amqp10.AmqpError, match="SASL"):
            amqp10.AmqpConnection("127.0.0.1", srv.port, ("PLAIN", "RootManageSharedAccessKey", "wrong")).open()
        assert srv.auth_failures == 1
    finally:
        srv.stop()


def test_tenant_event_source_on_event_hubs():
    """A tenant's event source with an ``eventhub`` receiver (AMQP) stores what devices send."""
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    srv = EventHubServer(hub="devices", partitions=2).start()
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        ms = sw["event-sources"]
        doc = run(lambda: ms.management.get_tenant_configuration("default"))
        doc["sources"].append({"id": "hub", "decoder": "protobuf", "receivers": [{
            "type": "eventhub", "host": "127.0.0.1", "port": srv.port, "tls": False, "eventHub": "devices",
            "sasKeyName": "RootManageSharedAccessKey", "sasKey": "secret", "consumerGroup": "$Default"}]})
        run(lambda: ms.management.update_tenant_configuration("default", doc))
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        aid = run(lambda: dm.get_device_by_token("meitrack-001")).device_assignment_id
        assert _wait(lambda: srv.credited == {"0", "1"}, 30)     # both partition links receiving
        srv.send("1", wire.measurements("meitrack-001", {"hub.t": 3.5}), key="meitrack-001")
        assert _wait(lambda: any(m.name == "hub.t" for m in run(
            lambda: em.list_measurements_for_index("Assignment", [aid], {"pageSize": 0})).results), 30)
    finally:
        sw.stop()
        srv.stop()
