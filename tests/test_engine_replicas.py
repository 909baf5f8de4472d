"""Several inbound-processing engine replicas on one tenant (one process per GPU in production).

Reference parallelism: decoded events are keyed by device token, so Kafka's
partitioner sends every event of one device to one partition and a consumer group spreads the
partitions over the inbound-processing replicas.  The MI355X path keeps that contract for raw
batches: event sources split each batch by ``murmur2(device token) % partitions``
(``sw_partition_payloads``), the engine replicas share the raw-payload consumer group, and each
device's state, dedup window and events live on exactly one replica.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.bus.log import murmur2
from sitewhere_amd.models import wire
from sitewhere_amd.pipeline.bus_io import parse_raw_batch, partition_payloads
from sitewhere_amd.runtime.microservice import run_microservice, shutdown_microservice


def wait(cond, t=30.0):
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.05)
    return cond()


def test_payload_partitioner_matches_kafka_key_partitioning():
    toks = [f"dev-{i:05d}" for i in range(300)]
    payloads = [wire.measurements(t, {"m": 1.0}) for t in toks] + [b"\x01\x02garbage"]
    parts = partition_payloads(payloads, 8)
    assert parts[-1] == -1
    assert parts[:-1].tolist() == [(murmur2(t.encode()) & 0x7FFFFFFF) % 8 for t in toks]
    assert len(set(parts[:-1].tolist())) == 8


def test_two_engine_replicas_split_devices_by_partition():
    _replicas_scenario()


@pytest.mark.gpu
@pytest.mark.skipif(not __import__("conftest").gpu_available(), reason="needs an MI355X GPU")
def test_two_gpu_engine_replicas_split_devices_by_partition():
    """Same on the MI355X: both replicas run the HIP engine (here sharing the box's one GPU)."""
    _replicas_scenario(kind="gpu")


def _replicas_scenario(kind: str | None = None):
    from sitewhere_amd.services.inbound_processing import InboundProcessingMicroservice
    sw = SiteWhereInstance().start()
    replica = None
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "rep", "name": "rep",
                                                              "configurationTemplateId": "gpu",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("rep", 120)
        replica = InboundProcessingMicroservice(sw.instance)
        assert run_microservice(replica) == 0
        r1 = sw.tenant_engine("inbound-processing", "rep")
        r2 = replica.wait_for_tenant_engine("rep", 60)
        if kind is not None:
            assert r1.engine_kind == r2.engine_kind == kind
        run = lambda f: sw.instance.system_user.run(f, "rep")  # noqa: E731
        dm = sw.api("DeviceManagement", "rep")
        devs = [d for d in run(lambda: dm.list_devices({"pageSize": 0})).results
                if d.device_assignment_id and not d.token[0].isdigit()]          # demo fleet: no history
        assert len(devs) >= 8
        for e in (r1, r2):          # both replicas mirror the registry (change feed + initial load)
            assert wait(lambda e=e: all(e.asg_index.idx.get(d.device_assignment_id) is not None for d in devs))
        t_raw = sw.instance.naming.tenant_prefix("rep") + "event-source-raw-payloads"
        bus = sw.instance.bus

        def split():    # the group has converged: disjoint non-empty assignments covering every partition
            a1, a2 = set(r1.raw_consumer.consumer.assignment()), set(r2.raw_consumer.consumer.assignment())
            return a1 and a2 and not (a1 & a2) and len(a1 | a2) == bus.partitions(t_raw)
        assert wait(split), (r1.raw_consumer.consumer.assignment(), r2.raw_consumer.consumer.assignment())
        es = sw.tenant_engine("event-sources", "rep")
        n = 400
        for i in range(n):
            d = devs[i % len(devs)]
            es.inject("default-protobuf", wire.measurements(d.token, {"rep": float(i)}, alternate_id=f"rep-{i}"))
        es.manager.flush_raw()
        assert wait(lambda: r1.processed_events.count + r2.processed_events.count >= n)
        assert r1.processed_events.count > 0 and r2.processed_events.count > 0
        # every raw record carries the payloads of one partition's devices only
        for p in range(bus.partitions(t_raw)):
            for rec in bus.read(t_raw, p, bus.begin_offset(t_raw, p), max_records=10_000, max_bytes=64 << 20):
                rb = parse_raw_batch(rec.value)
                raw, offs = np.asarray(rb.payload), rb.offsets()
                payloads = [bytes(raw[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
                assert set(partition_payloads(payloads, bus.partitions(t_raw)).tolist()) == {p}
        # each device's state lives on exactly one replica
        owners = {}
        for d in devs:
            held = [k for k, e in enumerate((r1, r2))
                    if e.engine.device_state(e.asg_index.idx[d.device_assignment_id]).get("measurements")]
            owners[d.token] = held
        assert all(len(h) == 1 for h in owners.values()), owners
        assert {h[0] for h in owners.values()} == {0, 1}
        # stored exactly once, each event by its device's replica
        em = sw.api("DeviceEventManagement", "rep")
        r1.flush()
        r2.flush()
        assert r1.persisted_events.count + r2.persisted_events.count == n
        stored = sum(run(lambda d=d: em.list_measurements_for_index("Assignment", [d.device_assignment_id],
                                                                    {"pageSize": 0})).num_results for d in devs)
        assert stored == n
    finally:
        if replica is not None:
            shutdown_microservice(replica)
        sw.stop()


def test_raw_batches_cut_at_the_count_bound_per_partition():
    """A source reaching rawBatchSize x partitions cuts a batch at once (not only on the delay
    timer), splits it by device token and publishes it -- concurrently injecting threads included."""
    import threading
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        es_ms = sw["event-sources"]
        eng = es_ms.get_tenant_engine("default")
        eng.raw_batch, eng.raw_delay_s = 16, 3600.0             # count bound only
        src = eng.manager.sources["default-protobuf"]
        src.forward_raw = True
        t_raw = eng.manager.t_raw
        bus = sw.instance.bus
        nparts = bus.partitions(t_raw)
        before = sum(bus.end_offset(t_raw, p) for p in range(nparts))

        def inject(k):
            for i in range(16 * nparts):
                eng.inject("default-protobuf", wire.measurements(f"cnt-{k}-{i % 40}", {"x": float(i)}))
        ths = [threading.Thread(target=inject, args=(k,)) for k in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(30)
        assert not any(t.is_alive() for t in ths), "raw batch cut deadlocked"
        eng.manager.flush_raw()
        recs = [r for p in range(nparts) for r in bus.read(t_raw, p, 0, max_records=100_000, max_bytes=64 << 20)]
        assert sum(bus.end_offset(t_raw, p) for p in range(nparts)) - before == len(recs) > nparts
        assert sum(parse_raw_batch(r.value).n_msgs for r in recs) == 4 * 16 * nparts
    finally:
        sw.stop()
