"""Kafka wire protocol: RecordBatch v2, the broker front end over the native commit log, the client,
the group protocol and KafkaEventBus (the bus surface on Kafka).

Parity unpinned against a real Apache Kafka (none in this environment): the broker and the client are
checked against each other, against the protocol's published constants (CRC-32C check value,
RecordBatch v2 layout) and against the native bus they share."""
import gzip
import struct
import threading
import time

import pytest

from sitewhere_amd.bus import kafka_wire as kw
from sitewhere_amd.bus.kafka_broker import KafkaBrokerServer
from sitewhere_amd.bus.kafka_client import KafkaClient, KafkaEventBus, range_assign
from sitewhere_amd.bus.log import EventBus


@pytest.fixture
def broker():
    bus = EventBus(None, default_partitions=4)
    srv = KafkaBrokerServer(bus, port=0).start()
    yield bus, srv
    srv.stop()
    bus.close()


def test_crc32c_and_record_batch_roundtrip():
    assert kw.crc32c(b"123456789") == 0xE3069283                 # CRC-32C check value
    recs = [(b"k1", b"v1", 1000), (None, b"", 1005), (b"k3", None, 999)]
    b = kw.encode_batch(recs, base_offset=42)
    base, blen, _, magic = struct.unpack_from(">qiib", b, 0)
    assert (base, magic, blen) == (42, 2, len(b) - 12)
    out = kw.decode_batches(b)
    assert [(o, k, v, t) for o, k, v, t in out] == [(42, b"k1", b"v1", 1000), (43, None, b"", 1005),
                                                     (44, b"k3", None, 999)]
    # a corrupted byte fails the CRC; a truncated trailing batch is ignored (fetch semantics)
    bad = bytearray(b)
    bad[-1] ^= 0xFF
    with pytest.raises(kw.KafkaError):
        kw.decode_batches(bytes(bad))
    assert kw.decode_batches(b + b[:30]) == out


def test_gzip_batch_is_read():
    plain = kw.encode_batch([(b"a", b"hello", 5), (b"b", b"world", 6)])
    head, rest = plain[:61], plain[61:]
    comp = gzip.compress(rest)
    attrs_and_rest = struct.pack(">h", 1) + plain[23:61] + comp       # attributes = gzip
    crc = kw.crc32c(attrs_and_rest)
    body = struct.pack(">iib", -1, 2, 0)[:0]
    batch = struct.pack(">qiib", 0, 4 + 1 + 4 + len(attrs_and_rest), -1, 2) + struct.pack(">I", crc) + attrs_and_rest
    assert [(k, v) for _, k, v, _ in kw.decode_batches(batch)] == [(b"a", b"hello"), (b"b", b"world")]
    assert head[:8] == batch[:8] and body == b""


def test_produce_fetch_metadata_offsets_shared_with_native_bus(broker):
    bus, srv = broker
    c = KafkaClient(srv.address)
    assert c.metadata(["sw.in"]) == {"sw.in": 4}                   # auto-created, default partitions
    base = c.produce("sw.in", 1, [(b"dev-1", b"m1"), (b"dev-1", b"m2")], ts=1000)
    assert base == 0
    # the native bus sees Kafka-produced records ...
    assert [r.value for r in bus.read("sw.in", 1, 0)] == [b"m1", b"m2"]
    # ... and Kafka clients see natively appended ones
    bus.append("sw.in", 1, [(b"dev-2", b"m3")], ts=2000)
    got = c.fetch_many([("sw.in", 1, 1)], max_wait_ms=0)
    recs, hw, err = got[("sw.in", 1)]
    assert err == 0 and hw == 3 and [(o, v) for o, _, v, _ in recs] == [(1, b"m2"), (2, b"m3")]
    assert c.list_offset("sw.in", 1, -2) == 0 and c.list_offset("sw.in", 1, -1) == 3
    assert c.list_offset("sw.in", 1, 1500) == 2                   # first record at/after ts
    # long-poll fetch wakes up on an append
    threading.Timer(0.2, lambda: bus.append("sw.in", 2, [(None, b"late")])).start()
    t0 = time.time()
    got = c.fetch_many([("sw.in", 2, 0)], max_wait_ms=5000)
    assert got[("sw.in", 2)][0][0][2] == b"late" and time.time() - t0 < 3
    # out-of-range fetch is reported, not silently empty
    assert c.fetch_many([("sw.in", 1, 99)], max_wait_ms=0)[("sw.in", 1)][2] == kw.OFFSET_OUT_OF_RANGE
    c.close()


def test_api_versions_probe_of_a_newer_client(broker):
    import socket
    _, srv = broker
    s = socket.create_connection(("127.0.0.1", srv.port))
    s.sendall(kw.request_frame(kw.API_VERSIONS, 3, 7, "java", b""))
    msg = kw.recv_frame(s)
    assert struct.unpack_from(">i", msg, 0)[0] == 7
    r = kw.decode(kw.RESPONSE[kw.API_VERSIONS], msg, 4)
    assert r["error_code"] == kw.UNSUPPORTED_VERSION
    assert {a["api_key"]: a["max_version"] for a in r["api_keys"]} == kw.VERSIONS
    s.close()


def test_range_assignor():
    plan = range_assign({"b": ["t"], "a": ["t", "u"]}, {"t": 5, "u": 2})
    assert plan["a"] == [("t", 0), ("t", 1), ("t", 2), ("u", 0), ("u", 1)]
    assert plan["b"] == [("t", 3), ("t", 4)]


def test_group_rebalance_leave_and_commits(broker):
    _, srv = broker
    c1, c2 = KafkaClient(srv.address, "c1"), KafkaClient(srv.address, "c2")
    c1.metadata(["sw.grp"])
    g1, m1, a1 = c1.join_group("g", ["sw.grp"], session_ms=6000)
    assert a1 == [("sw.grp", p) for p in range(4)]
    res = {}
    t = threading.Thread(target=lambda: res.update(j2=c2.join_group("g", ["sw.grp"], session_ms=6000)))
    t.start()
    # member 1 learns about the rebalance from its heartbeat and rejoins
    deadline = time.time() + 10
    while c1.heartbeat("g", g1, m1) != kw.REBALANCE_IN_PROGRESS and time.time() < deadline:
        time.sleep(0.05)
    g1b, m1b, a1b = c1.join_group("g", ["sw.grp"], m1, session_ms=6000)
    t.join(10)
    g2, m2, a2 = res["j2"]
    assert g1b == g2 > g1 and m1b == m1
    assert sorted(a1b + a2) == [("sw.grp", p) for p in range(4)] and len(a1b) == len(a2) == 2
    # commits are generation-checked and land in the shared bus offsets
    c1.commit("g", [("sw.grp", a1b[0][1], 17)], g1b, m1)
    assert c2.committed("g", "sw.grp", a1b[0][1]) == 17
    with pytest.raises(kw.KafkaError):
        c1.commit("g", [("sw.grp", 0, 1)], g1, m1)                 # stale generation
    # member 2 leaves: member 1 takes everything after rejoining
    c2.leave_group("g", m2)
    assert c1.heartbeat("g", g1b, m1) == kw.REBALANCE_IN_PROGRESS
    g1c, _, a1c = c1.join_group("g", ["sw.grp"], m1, session_ms=6000)
    assert g1c > g1b and a1c == [("sw.grp", p) for p in range(4)]
    c1.close()
    c2.close()


def test_sasl_plain(broker):
    bus, _ = broker
    srv = KafkaBrokerServer(bus, port=0, users={"$ConnectionString": "Endpoint=sb://x/;SharedAccessKey=k"}).start()
    try:
        ok = KafkaClient(srv.address, sasl_plain=("$ConnectionString", "Endpoint=sb://x/;SharedAccessKey=k"))
        assert ok.metadata(["hub"]) == {"hub": 4}
        with pytest.raises(kw.KafkaError):
            KafkaClient(srv.address, sasl_plain=("$ConnectionString", "wrong")).metadata(["hub"])
        with pytest.raises((ConnectionError, OSError, kw.KafkaError)):
            KafkaClient(srv.address).metadata(["hub"])             # unauthenticated: connection closed
        ok.close()
    finally:
        srv.stop()


def test_kafka_event_bus_runs_the_bus_consumer_and_producer(broker):
    bus, srv = broker
    kb = KafkaEventBus(srv.address, heartbeat_s=0.2)
    prod = kb.producer()
    with prod.batching():
        for i in range(40):
            prod.send("sw.events", f"dev-{i % 7}", f"e{i}".encode())
    # keyed records land where Kafka's default partitioner (murmur2) puts them
    from sitewhere_amd.bus.log import kafka_partition
    assert [r.value for r in bus.read("sw.events", kafka_partition(b"dev-0", 4), 0)][:2] == [b"e0", b"e7"]
    c = kb.consumer("svc", ["sw.events"])
    seen = []
    end = time.time() + 10
    while len(seen) < 40 and time.time() < end:
        for recs in c.poll(500).values():
            seen += [r.value for r in recs]
    c.commit()
    assert sorted(seen) == sorted(f"e{i}".encode() for i in range(40))
    c.close()
    # a new member of the group resumes after the committed offsets
    prod.send("sw.events", "dev-1", b"after")
    c2 = kb.consumer("svc", ["sw.events"])
    got = []
    end = time.time() + 10
    while not got and time.time() < end:
        for recs in c2.poll(500).values():
            got += [r.value for r in recs]
    assert got == [b"after"]
    c2.close()
    kb.close()


class _Source:
    def __init__(self):
        self.got = []

    def on_encoded_event_received(self, receiver, payload, metadata):
        self.got.append((payload, metadata))


def test_kafka_and_event_hub_receivers(broker):
    from sitewhere_amd.core.lifecycle import LifecycleProgressMonitor
    from sitewhere_amd.edges.receivers import build_receiver
    bus, srv = broker
    hub = KafkaBrokerServer(bus, port=0, users={"$ConnectionString": "Endpoint=sb://ns/;SharedAccessKey=k"}).start()
    try:
        recs = [build_receiver({"type": "kafka", "bootstrap": srv.address, "topic": "devices.in", "group": "r1"}),
                build_receiver({"type": "eventhub", "bootstrap": hub.address, "tls": False, "eventHub": "telemetry",
                                "connectionString": "Endpoint=sb://ns/;SharedAccessKey=k"})]
        srcs = [_Source(), _Source()]
        for r, s in zip(recs, srcs):
            r.source = s
            r.lifecycle_start(LifecycleProgressMonitor())
        c = KafkaClient(srv.address)
        c.produce("devices.in", 0, [(b"dev-1", b"payload-1")])
        c.produce("telemetry", 3, [(None, b"hub-1"), (None, b"hub-2")])
        end = time.time() + 10
        while (len(srcs[0].got) < 1 or len(srcs[1].got) < 2) and time.time() < end:
            time.sleep(0.05)
        assert srcs[0].got[0][0] == b"payload-1" and srcs[0].got[0][1]["key"] == "dev-1"
        assert [p for p, _ in srcs[1].got] == [b"hub-1", b"hub-2"]
        # delivered records were committed by the receivers' groups
        end = time.time() + 5
        while bus.committed("$Default", "telemetry", 3) != 2 and time.time() < end:
            time.sleep(0.05)
        assert bus.committed("r1", "devices.in", 0) == 1 and bus.committed("$Default", "telemetry", 3) == 2
        for r in recs:
            r.lifecycle_stop(LifecycleProgressMonitor())
        c.close()
    finally:
        hub.stop()


def test_whole_instance_runs_on_kafka(broker):
    """Every microservice's data plane on KafkaEventBus (the reference's deployment shape), through
    the broker front end: a device measurement flows to event management and device state."""
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    from sitewhere_amd.runtime.config import InstanceSettings
    from sitewhere_amd.runtime.microservice import Instance
    _, srv = broker
    inst = Instance(InstanceSettings(heartbeat_s=1.0), bus=KafkaEventBus(srv.address, heartbeat_s=0.5))
    sw = SiteWhereInstance(instance=inst).start()
    try:
        sw.wait_for_tenant("default", 120)
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        aid = run(lambda: dm.get_device_by_token("meitrack-003")).device_assignment_id
        sw.tenant_engine("event-sources").inject("default-protobuf",
                                                 wire.measurements("meitrack-003", {"kafka.temp": 7.5}))
        end, res = time.time() + 60, []
        while not res and time.time() < end:
            res = run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
            time.sleep(0.1)
        assert res and res[0].name == "kafka.temp" and res[0].value == 7.5
    finally:
        sw.stop()
