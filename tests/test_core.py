"""Unit tests: lifecycle FSM, JWT, tracing, metrics, bus, coordination, persistence."""
import threading
import time

import pytest

from sitewhere_amd.core.errors import ServerStartupException, SiteWhereException, UnauthorizedException
from sitewhere_amd.core.lifecycle import (CompositeLifecycleStep, LifecycleComponent, LifecycleProgressMonitor,
                                          LifecycleStatus, LifecycleComponentParameter, SimpleLifecycleStep)
from sitewhere_amd.core.metrics import MetricRegistry
from sitewhere_amd.core.security import (Authentication, TokenManagement, current_tenant, security_context,
                                         hash_password, verify_password)
from sitewhere_amd.core.tracing import Tracer


class Boom(LifecycleComponent):
    def __init__(self, where):
        super().__init__("boom")
        self.where = where

    def initialize(self, m):
        if self.where == "init":
            raise RuntimeError("init failed")

    def start(self, m):
        if self.where == "start":
            raise RuntimeError("start failed")


class Parent(LifecycleComponent):
    def __init__(self, child, require):
        super().__init__("parent")
        self.child, self.require = child, require

    def initialize(self, m):
        self.initialize_nested_component(self.child, m, self.require)

    def start(self, m):
        self.start_nested_component(self.child, m, self.require)


def test_lifecycle_happy_path_and_terminate():
    c = LifecycleComponent("c")
    seen = []
    c.add_status_listener(lambda comp, old, new: seen.append(new))
    c.lifecycle_initialize()
    assert c.status == LifecycleStatus.Stopped
    c.lifecycle_start()
    assert c.status == LifecycleStatus.Started
    c.lifecycle_stop()
    c.lifecycle_terminate()
    assert c.status == LifecycleStatus.Terminated
    assert seen[:2] == [LifecycleStatus.Initializing, LifecycleStatus.Stopped]


def test_lifecycle_errors_and_required_children():
    b = Boom("init")
    b.lifecycle_initialize()
    assert b.status == LifecycleStatus.InitializationError and b.lifecycle_error
    p = Parent(Boom("init"), require=True)
    p.lifecycle_initialize()
    assert p.status == LifecycleStatus.InitializationError
    assert isinstance(p.lifecycle_error.__cause__, ServerStartupException)
    # optional child failing at start -> StartedWithErrors
    p2 = Parent(Boom("start"), require=False)
    p2.lifecycle_initialize()
    p2.lifecycle_start()
    assert p2.status == LifecycleStatus.StartedWithErrors
    p2.lifecycle_stop()
    assert p2.status == LifecycleStatus.StoppedWithErrors


def test_required_parameter_validation():
    c = LifecycleComponent("p")
    c.parameters.append(LifecycleComponentParameter("host", required=True))
    c.lifecycle_initialize()
    assert c.status == LifecycleStatus.InitializationError


def test_composite_step_aborts_and_reports():
    msgs = []
    mon = LifecycleProgressMonitor(listener=msgs.append)
    order = []
    step = CompositeLifecycleStep("boot", [SimpleLifecycleStep("a", lambda m: order.append("a")),
                                           SimpleLifecycleStep("b", lambda m: (_ for _ in ()).throw(SiteWhereException("x"))),
                                           SimpleLifecycleStep("c", lambda m: order.append("c"))])
    with pytest.raises(SiteWhereException):
        step.execute(mon)
    assert order == ["a"] and [m["task"] for m in msgs] == ["a", "b"]


def test_jwt_roundtrip_and_tamper():
    tm = TokenManagement("s3cret", expiration_minutes=5)
    tok = tm.generate_token("admin", ["REST", "ADMINISTER_USERS"])
    assert tm.get_username(tok) == "admin"
    assert tm.get_granted_authorities(tok) == ["REST", "ADMINISTER_USERS"]
    with pytest.raises(UnauthorizedException):
        TokenManagement("other").get_claims(tok)
    with pytest.raises(UnauthorizedException):
        tm.get_claims(TokenManagement("s3cret", expiration_minutes=-1).generate_token("a", []))


def test_instance_jwt_secret_is_random_and_shared_through_coordination(monkeypatch):
    """No literal default secret: each instance gets a random one, created once in the coordination
    store, so every process of the instance verifies the others' tokens and nobody else can."""
    from sitewhere_amd.coord.store import Coordination
    from sitewhere_amd.runtime.config import InstanceSettings
    from sitewhere_amd.runtime.microservice import Instance
    monkeypatch.delenv("SITEWHERE_JWT_SECRET", raising=False)
    coord = Coordination()
    a = Instance(InstanceSettings(), coord=coord)
    b = Instance(InstanceSettings(), coord=coord)          # a second process of the same instance
    other = Instance(InstanceSettings())                    # a different instance
    assert a.tokens.secret == b.tokens.secret and len(a.tokens.secret) == 64
    assert other.tokens.secret != a.tokens.secret
    assert b.tokens.get_username(a.system_jwt())
    with pytest.raises(UnauthorizedException):
        other.tokens.get_claims(a.system_jwt())
    assert TokenManagement("sitewhere-instance-secret").secret != a.tokens.secret
    monkeypatch.setenv("SITEWHERE_JWT_SECRET", "from-env")
    assert Instance(InstanceSettings(), coord=Coordination()).tokens.secret == b"from-env"


def test_security_context_is_scoped_per_thread():
    out = {}

    def worker(name):
        with security_context(Authentication(name, tenant=name)):
            time.sleep(0.01)
            out[name] = current_tenant()

    ts = [threading.Thread(target=worker, args=(f"t{i}",)) for i in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert out == {f"t{i}": f"t{i}" for i in range(8)}
    assert current_tenant() is None


def test_password_hashing():
    h = hash_password("pw")
    assert verify_password("pw", h) and not verify_password("nope", h)


def test_tracing_propagation_and_errors():
    tr = Tracer(sample_rate=1.0)
    with tr.start_span("outer") as o:
        with tr.start_span("inner") as i:
            pass
        hdr = o.context_header()
    remote = tr.start_span("remote-child", child_of=hdr)
    remote.finish()
    spans = tr.export()
    names = [s["name"] for s in spans]
    assert names == ["inner", "outer", "remote-child"]
    assert spans[0]["parentId"] == spans[1]["spanId"]
    assert spans[2]["traceId"] == spans[1]["traceId"]
    with pytest.raises(ValueError):
        with tr.start_span("bad"):
            raise ValueError("x")
    assert tr.export()[-1]["tags"]["error"] is True


def test_metrics_and_prometheus():
    r = MetricRegistry()
    r.meter("t1.decodedEvents").mark(5)
    with r.timer("t1.eventStorage").time():
        pass
    r.counter("c").inc(3)
    snap = r.snapshot()
    assert snap["t1.decodedEvents"]["count"] == 5 and snap["c"]["count"] == 3
    text = r.prometheus()
    assert "sitewhere_t1_decodedEvents_total 5" in text


# ------------------------------------------------------------------------------ bus
def test_bus_key_partitioning_groups_and_commit(tmp_path):
    from sitewhere_amd.bus.log import EventBus
    bus = EventBus(str(tmp_path / "log"), default_partitions=4)
    p = bus.producer()
    for i in range(200):
        p.send("t", f"dev-{i % 10}", f"v{i}".encode())
    # same key -> same partition, in order
    parts = {}
    c = bus.consumer("g1", ["t"])
    got = []
    while True:
        batch = c.poll(200)
        if not batch:
            break
        for tp, recs in batch.items():
            for r in recs:
                parts.setdefault(r.key, set()).add(tp[1])
                got.append(r.value)
    assert len(got) == 200 and all(len(v) == 1 for v in parts.values())
    c.commit()
    # an independent group sees the full stream (fan-out)
    c2 = bus.consumer("g2", ["t"])
    n2 = sum(len(r) for r in c2.poll(500, max_records=1000).values())
    assert n2 == 200
    c.close()
    c2.close()
    bus.close()
    # durability: reopen, committed offsets resume where g1 left
    bus2 = EventBus(str(tmp_path / "log"), default_partitions=4)
    p2 = bus2.producer()
    p2.send("t", "dev-1", b"after-restart")
    c3 = bus2.consumer("g1", ["t"])
    vals = [r.value for recs in c3.poll(500).values() for r in recs]
    assert vals == [b"after-restart"]
    bus2.close()


def test_bus_rebalance_splits_partitions():
    from sitewhere_amd.bus.log import EventBus
    bus = EventBus(None, default_partitions=8)
    bus.topic("x")
    a = bus.consumer("g", ["x"], member_id="a")
    b = bus.consumer("g", ["x"], member_id="b")
    a.poll(10)
    b.poll(10)
    pa, pb = {p for _, p in a.assignment()}, {p for _, p in b.assignment()}
    assert len(pa) == len(pb) == 4 and not (pa & pb)
    b.close()
    a.poll(10)
    assert len(a.assignment()) == 8


def test_bus_at_least_once_redelivery_after_crash():
    from sitewhere_amd.bus.log import EventBus
    bus = EventBus(None, default_partitions=1)
    prod = bus.producer()
    for i in range(10):
        prod.send("q", "k", str(i).encode())
    c = bus.consumer("g", ["q"], member_id="m1")
    first = [r.value for recs in c.poll(100, max_records=5).values() for r in recs]
    c.commit()
    c.poll(100, max_records=5)  # processed but NOT committed -> "crash"
    c.close()
    c2 = bus.consumer("g", ["q"], member_id="m2")
    again = [r.value for recs in c2.poll(100).values() for r in recs]
    assert first == [b"0", b"1", b"2", b"3", b"4"] and again[0] == b"5" and len(again) == 5


def test_murmur2_matches_kafka_reference_values(native_lib):
    import ctypes
    # Kafka's Utils.murmur2 test vectors
    vecs = {b"21": -973932308, b"foobar": -790332482, b"a-little-bit-long-string": -985981536,
            b"a-little-bit-longer-string": -1486304829, b"lkjh234lh9fiuh90y23oiuhsafujhadof229phr9h19h89h8": -58897971,
            b"abc": 479470107}
    for k, want in vecs.items():
        buf = ctypes.create_string_buffer(k, len(k))
        assert native_lib.sw_murmur2(ctypes.cast(buf, ctypes.c_void_p), len(k)) == want


# ------------------------------------------------------------------------------ coordination
def test_coordination_watch_versions_ephemeral_and_mutex(tmp_path):
    from sitewhere_amd.coord.store import (BadVersionError, Coordination, InterProcessMutex, NODE_ADDED,
                                           NODE_UPDATED, NODE_REMOVED, INITIALIZED)
    co = Coordination(str(tmp_path / "zk.json"))
    co.create("/sw/conf/a.xml", b"1")
    events = []
    co.watch_tree("/sw/conf", lambda k, p, d: events.append((k, p)))
    time.sleep(0.05)
    st = co.set("/sw/conf/a.xml", b"2")
    with pytest.raises(BadVersionError):
        co.set("/sw/conf/a.xml", b"3", version=st.version - 1)
    s = co.open_session()
    co.create("/sw/live/m1", b"", ephemeral=True, session=s)
    co.delete("/sw/conf/a.xml")
    time.sleep(0.1)
    kinds = [k for k, _ in events]
    assert INITIALIZED in kinds and NODE_UPDATED in kinds and NODE_REMOVED in kinds and NODE_ADDED in kinds
    co.close_session(s)
    assert co.exists("/sw/live/m1") is None
    # mutex contention: only one holder at a time
    holders = []
    lock_log = []

    def worker(i):
        with InterProcessMutex(co, "/sw/locks/boot"):
            holders.append(i)
            lock_log.append(len(holders))
            time.sleep(0.02)
            holders.remove(i)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert max(lock_log) == 1 and len(lock_log) == 4
    # snapshot durability
    co.put("/sw/conf/b.xml", b"keep")
    co2 = Coordination(str(tmp_path / "zk.json"))
    assert co2.get_data("/sw/conf/b.xml") == b"keep"
    assert co2.exists("/sw/live/m1") is None


# ------------------------------------------------------------------------------ persistence
@pytest.mark.parametrize("kind", ["memory", "sqlite"])
def test_entity_store(kind):
    from sitewhere_amd.models.domain import Device, DeviceType
    from sitewhere_amd.persistence.store import create_store
    from sitewhere_amd.core.errors import SiteWhereSystemException
    s = create_store(kind)
    s.register("devices", Device)
    s.register("types", DeviceType)
    d = Device(token="d1", comments="x", metadata={"a": "b"})
    s.put("devices", d)
    assert s.get_by_token("devices", "d1").metadata == {"a": "b"}
    with pytest.raises(SiteWhereSystemException):
        s.put("devices", Device(token="d1"))
    d2 = s.get("devices", d.id)
    d2.comments = "y"
    s.put("devices", d2)
    assert s.get("devices", d.id).comments == "y"
    assert len(s.query("devices", lambda e: e.comments == "y")) == 1
    s.delete("devices", d.id)
    assert s.get_by_token("devices", "d1") is None


@pytest.mark.parametrize("kind", ["memory", "sqlite", "bucketed"])
def test_event_store_queries(kind):
    from sitewhere_amd.models.domain import (DateRangeSearchCriteria, DeviceEventIndex, DeviceEventType,
                                             DeviceMeasurement, DeviceCommandResponse)
    from sitewhere_amd.persistence.events import create_event_store
    es = create_event_store(kind, bucket_ms=1000)
    evs = [DeviceMeasurement(device_assignment_id="a1" if i % 2 else "a2", customer_id="c", name="t", value=i,
                             event_date=1000 * i, alternate_id=f"alt{i}") for i in range(20)]
    es.add_events(evs)
    r = es.list_events(DeviceEventType.Measurement, DeviceEventIndex.Assignment, ["a1"],
                       DateRangeSearchCriteria(page_size=3, start_date=2000, end_date=15000))
    assert r.num_results == 7 and [e.value for e in r.results] == [15, 13, 11]
    r2 = es.list_events(DeviceEventType.Measurement, DeviceEventIndex.Customer, ["c"], DateRangeSearchCriteria(page_size=0))
    assert r2.num_results == 20 and r2.results[0].value == 19
    assert es.get_event_by_alternate_id("alt4").value == 4
    resp = DeviceCommandResponse(originating_event_id=evs[0].id, device_assignment_id="a2", response="ok",
                                 event_date=5)
    es.add_events([resp])
    assert es.list_command_responses_for_invocation(evs[0].id).results[0].response == "ok"


def test_buffered_writer_and_influx_lines():
    from sitewhere_amd.models.domain import DeviceLocation, DeviceMeasurement
    from sitewhere_amd.persistence.events import BufferedEventWriter, InfluxLineWriter, MemoryEventStore
    st = MemoryEventStore()
    w = BufferedEventWriter(st, chunk=50, interval_ms=50)
    w.add([DeviceMeasurement(device_assignment_id="a", name="x", value=i, event_date=i) for i in range(120)])
    w.flush()
    w.close()
    assert st.count() == 120 and w.flushes >= 3
    posted = []
    iw = InfluxLineWriter("http://influx:8086", batch=2, post=lambda url, body: posted.append((url, body)))
    iw.add_events([DeviceMeasurement(device_assignment_id="a", name="temp", value=1.5, event_date=7),
                   DeviceLocation(device_assignment_id="a", latitude=1.0, longitude=2.0, event_date=8)])
    assert posted and b"mx_temp=1.5" in posted[0][1] and b"latitude=1.0" in posted[0][1]


def test_every_microservice_has_a_configuration_model():
    from sitewhere_amd.assembly import SERVICES_BY_ID
    from sitewhere_amd.configuration import model_for
    from sitewhere_amd.services.tenant_management import TENANT_TEMPLATES
    assert len(SERVICES_BY_ID) == 19
    for ident in SERVICES_BY_ID:
        m = model_for(ident)
        assert m is not None and m.to_dict()["root"]["role"] == ident
    # every tenant template document validates against its service's model
    for tpl in TENANT_TEMPLATES.values():
        for svc, doc in tpl["services"].items():
            assert model_for(svc).validate(doc) == [], (svc, doc)


def test_bus_memory_retention_frees_whole_segments():
    """Memory-only logs keep at most retention_bytes per partition (64 MB segments are freed and
    recycled whole); a consumer behind the retained range resumes at the oldest retained record."""
    import os
    from sitewhere_amd.bus.log import EventBus
    bus = EventBus(None, default_partitions=1, retention_bytes=100 << 20)
    v = os.urandom(1 << 20)
    for i in range(300):
        bus.append("big", 0, [(f"k{i}".encode(), v[:-8] + i.to_bytes(8, "little"))])
    begin, end = bus.begin_offset("big", 0), bus.end_offset("big", 0)
    assert end == 300 and 0 < begin and end - begin >= 100       # ~100-164 MB retained
    first = bus.read("big", 0, 0, 1, 2 << 20)[0]                  # behind the range: clamped
    assert first.offset == begin and first.value[-8:] == begin.to_bytes(8, "little")
    last = bus.read("big", 0, 299, 1, 2 << 20)[0]
    assert last.key == b"k299" and last.value[:-8] == v[:-8]
    bus.retain_from("big", 0, 290)
    assert bus.begin_offset("big", 0) == 290
    assert [r.offset for r in bus.read("big", 0, 0, 20, 32 << 20)] == list(range(290, 300))
    bus.close()


def test_bus_durable_reload_after_large_batches(tmp_path):
    """Durable partitions survive reopen with records spanning several appends (segments)."""
    import os
    from sitewhere_amd.bus.log import EventBus
    bus = EventBus(str(tmp_path / "d"), default_partitions=1)
    vals = [os.urandom(3 << 20) for _ in range(5)]
    for v in vals:
        bus.append("t", 0, [(None, v)])
    bus.close()
    bus2 = EventBus(str(tmp_path / "d"), default_partitions=1)
    assert bus2.end_offset("t", 0) == 5
    assert [r.value for r in bus2.read("t", 0, 0, 10, 32 << 20)] == vals
    bus2.append("t", 0, [(None, b"tail")])
    assert bus2.read("t", 0, 5, 1)[0].value == b"tail"
    bus2.close()


def test_columnar_store_dense_and_small_batches():
    """Large batches are kept zero-copy with ids computed on query; small ones are consolidated.
    Both serve get-by-id and index queries (newest first), and replays are skipped."""
    import numpy as np
    from sitewhere_amd.models.columnar import OUT_REC
    from sitewhere_amd.models.domain import DeviceEventIndex, DeviceEventType, DateRangeSearchCriteria
    from sitewhere_amd.persistence.columnar import ColumnarEventStore, encode_batch
    st = ColumnarEventStore(dense_rows=100)
    asg = {0: ["a0", "d0", "c0", "ar0", None], 1: ["a1", "d1", "c1", "ar1", None]}

    def rows(n, d0):
        r = np.zeros(n, OUT_REC)
        r["event_date"] = d0 + np.arange(n)
        r["v0"] = np.arange(n, dtype=np.float64)
        r["assignment"] = np.arange(n) % 2
        r["name_id"] = 0
        return r
    assert st.add_columnar(encode_batch("b", 0, 2, 1, 5, rows(500, 1000), asg, {0: "t"})) == 500     # dense
    assert st.add_columnar(encode_batch("b", 500, 2, 1, 6, rows(10, 9000), {}, {})) == 10            # small
    assert st.add_columnar(encode_batch("b", 0, 2, 1, 5, rows(500, 1000), {}, {})) == 0              # replay
    e = st.get_event_by_id(f"b-{(7 * 2) + 1}")                 # seq 7 of the dense batch
    assert e.value == 7.0 and e.device_assignment_id == "a1" and e.received_date == 5
    e = st.get_event_by_id(f"b-{(503 * 2) + 1}")               # seq 503 = row 3 of the small batch
    assert e.event_date == 9003 and e.received_date == 6
    assert st.get_event_by_id("b-2") is None                   # rank 0 id: not this shard's
    res = st.list_events(DeviceEventType.Measurement, DeviceEventIndex.Assignment, ["a0"],
                         DateRangeSearchCriteria(page_size=3))
    assert res.num_results == 255 and [m.event_date for m in res.results] == [9008, 9006, 9004]


def test_codec_clone_matches_wire_round_trip():
    """LocalChannel's clone mode returns what a wire round trip would, without sharing mutables."""
    from sitewhere_amd.models import domain
    from sitewhere_amd.rpc import codec
    n = 0
    for cls in codec._REGISTRY.values():
        try:
            obj = cls()
        except TypeError:
            continue
        if hasattr(obj, "metadata"):
            obj.metadata = {"k": "v", "n": "1"}
        c = codec.clone(obj)
        assert type(c) is cls and c == codec.loads(codec.dumps(obj)) and c is not obj
        if hasattr(obj, "metadata"):
            c.metadata["k"] = "changed"
            assert obj.metadata["k"] == "v"
        n += 1
    assert n > 40
    m = domain.DeviceMeasurement(name="t", value=1.5, metadata={"a": "b"})
    payload = {"args": [[{"name": "x", "value": 2.0}], m, (1, 2), b"\x00\x01"], "kwargs": {"res": domain.SearchResults(1, [m])}}
    c = codec.clone(payload)
    assert c == codec.loads(codec.dumps(payload))
    assert c["args"][1] is not m and c["kwargs"]["res"].results[0] is not m


def test_columnar_store_retention_evicts_oldest_batches():
    """The in-memory columnar store holds at most ``retentionRows`` rows: whole oldest batches go,
    queries and id lookups see only what is held, and the newest batch always stays."""
    import numpy as np

    from sitewhere_amd.models.columnar import EV_MEASUREMENT, OUT_REC
    from sitewhere_amd.models.domain import DateRangeSearchCriteria
    from sitewhere_amd.persistence.columnar import encode_batch
    from sitewhere_amd.persistence.events import create_event_store
    st = create_event_store("columnar", retentionRows=10_000)
    for b in range(5):
        rows = np.zeros(4096, OUT_REC)
        rows["etype"], rows["assignment"], rows["name_id"] = EV_MEASUREMENT, 0, 1
        rows["event_date"] = 1_700_000_000_000 + b * 10_000 + np.arange(4096)
        rows["v0"] = b
        st.add_columnar(encode_batch("boot", b * 4096, 1, 0, 1, rows, {0: ["a0", "d0", None, None, None]},
                                     {1: "m"} if b == 0 else {}))
    assert st.rows == 8192 and st.evicted_rows == 3 * 4096 and st.count() == 8192
    res = st.list_events("Measurement", "Assignment", ["a0"], DateRangeSearchCriteria(page_size=0))
    assert res.num_results == 8192 and {e.value for e in res.results} == {3.0, 4.0}
    assert st.get_event_by_id("boot-0") is None and st.get_event_by_id(f"boot-{4 * 4096}").value == 4.0
    one = create_event_store("columnar", retentionRows=10)
    rows = np.zeros(4096, OUT_REC)
    one.add_columnar(encode_batch("b", 0, 1, 0, 1, rows, {}, {}))
    assert one.rows == 4096                              # a batch larger than the window is kept whole


def test_near_cache_lru_ttl_and_max_idle(monkeypatch):
    """Reference near-cache policy (HazelcastManager: LRU, TTL 60 s, max-idle 20 s)."""
    import sitewhere_amd.runtime.consumers as cons
    now = [1000.0]
    monkeypatch.setattr(cons.time, "time", lambda: now[0])
    c = cons.NearCache(capacity=2, ttl_s=60.0, max_idle_s=20.0)
    loads = []
    load = lambda k: loads.append(k) or f"v-{k}"  # noqa: E731
    assert c.get("a", load) == "v-a" and c.get("a", load) == "v-a" and loads == ["a"]
    now[0] += 15
    assert c.get("a", load) == "v-a" and loads == ["a"]          # touched: idle clock restarts
    now[0] += 15
    assert c.get("a", load) == "v-a" and loads == ["a"]
    now[0] += 21
    assert c.get("a", load) == "v-a" and loads == ["a", "a"]     # idle > 20 s: reloaded
    for _ in range(5):                                           # busy entry still expires at the TTL
        now[0] += 15
        c.get("a", load)
    assert loads.count("a") == 3
    c.get("b", load)
    c.get("c", load)                                             # capacity 2: oldest insert evicted
    assert len(c) == 2 and c.get("a") is None
    c.invalidate("b")
    assert c.get("b") is None


def test_zero_copy_columnar_frame_matches_encoded_batch():
    """A columnar batch framed in place around rows that already sit in a buffer (the MI355X
    engine's pinned row buffers) reads back like the copied encoding, is shared (not copied) by the
    in-process RPC codec, travels as bytes over the network codec, and is stored without a copy."""
    import numpy as np

    from sitewhere_amd.models.columnar import OUT_REC
    from sitewhere_amd.persistence.columnar import ColumnarEventStore, decode_batch, encode_batch, frame_batch
    from sitewhere_amd.rpc import codec
    n, head = 5000, 1 << 16
    buf = np.zeros(head + n * OUT_REC.itemsize, np.uint8)
    rows = buf[head:].view(OUT_REC)
    rows["event_date"] = 1000 + np.arange(n)
    rows["assignment"] = np.arange(n) % 2
    rows["v0"] = np.arange(n) * 0.5
    asg = {0: ["a0", "d0", "c0", "ar0", None], 1: ["a1", "d1", "c1", "ar1", None]}
    names = {1: "temp"}
    v = frame_batch((buf, head), rows.nbytes, "boot1", 7, 1, 0, 99, asg, names, {"zone.x": "in zone"})
    assert v is not None and not v.flags.writeable and np.shares_memory(v, buf)
    a, b = decode_batch(v), decode_batch(encode_batch("boot1", 7, 1, 0, 99, rows, asg, names, {"zone.x": "in zone"}))
    assert {k: a[k] for k in a if k != "rows"} == {k: b[k] for k in b if k != "rows"}
    assert np.array_equal(a["rows"], b["rows"]) and np.shares_memory(a["rows"], buf)
    assert codec.clone(v) is v                                   # in-process RPC: shared
    assert codec.from_wire(codec.to_wire(v)) == bytes(v)         # network RPC: bytes
    st = ColumnarEventStore(dense_rows=100)
    assert st.add_columnar(v) == n and st.rows == n
    assert np.shares_memory(st._chunks[-1]["rows"], buf)       # stored without a copy
    assert frame_batch((buf, 16), rows.nbytes, "boot1", 7, 1, 0, 99, asg, names) is None   # header too big


def test_pinned_row_pool_sizes_recycles_and_spills(monkeypatch):
    """The engine's pinned row buffers (GpuInboundEngine._pinned_out): sized to the step's rows plus
    slack (not the full output capacity), reused once nothing references them, and -- when every
    pooled buffer is held downstream (zero-copy payloads retained by the store / topic) -- a small
    set of recycled spill buffers marked not-retainable instead of a pinned allocation per step.
    Pinning itself is stubbed: the pool logic is host code."""
    import torch

    from sitewhere_amd.pipeline.gpu_engine import GpuInboundEngine
    monkeypatch.setattr(torch.Tensor, "pin_memory", lambda self: self)
    eng = object.__new__(GpuInboundEngine)
    eng.out_cap = 1 << 20                                     # 32 MB of rows at full capacity
    eng.PIN_POOL, eng.PIN_SPILL = 3, 2
    need = 65536 * 32
    pin, arr, pooled = eng._pinned_out(need)
    assert pooled and need + eng.ROW_HEADROOM <= arr.nbytes <= 4 << 20
    del pin, arr
    _, again, pooled = eng._pinned_out(need)                  # released: the same buffer comes back
    assert pooled and eng.pin_stats["reused"] == 1
    held = [again] + [eng._pinned_out(need)[1] for _ in range(2)]   # the pool (3) is now all held
    assert eng.pin_stats["new_pooled"] == 3
    s1 = eng._pinned_out(need)
    assert s1[2] is False and eng.pin_stats["spill"] == 1
    addr = s1[1].ctypes.data
    del s1
    s2 = eng._pinned_out(need)                                 # the spill buffer is recycled
    assert s2[2] is False and s2[1].ctypes.data == addr and eng.pin_stats["new_unpooled"] == 0
    s3 = eng._pinned_out(need)
    s4 = eng._pinned_out(need)                                 # spill set exhausted: unpooled, last resort
    assert s3[2] is False and s4[2] is False and eng.pin_stats["new_unpooled"] == 1
    big = eng._pinned_out(eng.out_cap * 32)                    # a full-capacity step fits too
    assert big[1].nbytes >= eng.out_cap * 32 + eng.ROW_HEADROOM
    del held
