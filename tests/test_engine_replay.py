"""Replay safety of the fused inbound engine tenant (services/gpu_inbound.py).

engine.step advances the event cursor, the alternate-id dedup table and device state, so it must
run once per raw record: when storing a stepped batch fails, the raw consumer re-reads the batch
and only the storage is retried with the kept StepResult.  These tests run on the CPU engine (the
same tenant code drives the MI355X engine) and check that a failed store loses nothing, stores
nothing twice and never drops a replayed event as an alternate-id duplicate."""
from __future__ import annotations

import struct
import time

import pytest
from conftest import engine_knows

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.models import wire
from sitewhere_amd.services.event_sources import RAW_PAYLOADS
from sitewhere_amd.utils.faults import FaultInjector


def _engine_rows(store):
    """Rows the engine persisted (a durable store also holds API-added events in blocks)."""
    return getattr(store, "engine_rows", store.rows)


def wait_until(cond, timeout=20.0, step=0.02):
    end = time.time() + timeout
    while time.time() < end:
        if cond():
            return True
        time.sleep(step)
    return bool(cond())


def _raw_batch(b, n=20, token="galaxytab-001"):
    msgs = [wire.measurements(token, {"v": float(100 * b + i)}, event_date=1_700_000_000_000 + 100 * b + i,
                              alternate_id=f"rp-{b}-{i}") for i in range(n)]
    return struct.pack(f"<I{len(msgs)}I", len(msgs), *[len(m) for m in msgs]) + b"".join(msgs)


@pytest.fixture(scope="module")
def inst():
    sw = SiteWhereInstance().start()
    sw.wait_for_tenant("default", 60)
    yield sw
    sw.stop()


def _tenant(inst, token, template):
    tm = inst.api("TenantManagement")
    inst.instance.system_user.run(lambda: tm.create_tenant({"token": token, "name": token,
                                                            "configurationTemplateId": template,
                                                            "datasetTemplateId": "construction"}))
    inst.wait_for_tenant(token, 60)
    ib = inst.tenant_engine("inbound-processing", token)
    run = lambda f: inst.instance.system_user.run(f, token)  # noqa: E731
    dev = run(lambda: inst.api("DeviceManagement", token).get_device_by_token("galaxytab-001"))
    assert wait_until(lambda: engine_knows(ib, dev))
    return ib, run, dev


def _values(inst, run, token, dev):
    em = inst.api("DeviceEventManagement", token)
    res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id], {"pageSize": 0}))
    return res.results


@pytest.mark.parametrize("overlap", [False, True])
def test_async_store_failure_rewinds_and_stores_once(inst, overlap):
    """gpu-columnar (asyncStore on): the store thread fails batch k while batch k+1 is queued.
    Nothing is committed past k, the consumer rewinds to k, both batches are stored from their kept
    results (not re-stepped) and every event lands exactly once.  ``overlap``: the engine completes
    each batch when the next is submitted (the MI355X overlapped steps; the CPU engine keeps the
    same one-deep lag), so a rewind also has to complete the batch still in the engine."""
    tok = "rpo" if overlap else "rpa"
    ib, run, dev = _tenant(inst, tok, "gpu-columnar")
    ib.overlap = overlap
    assert ib.async_store
    store = inst.tenant_engine("event-management", tok).store
    topic = inst.instance.naming.tenant_prefix(tok) + RAW_PAYLOADS
    group = ib.raw_consumer.group
    ingest = "add_batch" if hasattr(store, "add_batch") else "add_columnar"     # durable / in-memory store
    with FaultInjector() as fi:
        fi.fail_next(store, ingest, 2)
        for b in range(6):
            inst.instance.bus.append(topic, 0, [(None, _raw_batch(b))], ts=1_700_000_100_000 + b)
        assert wait_until(lambda: _engine_rows(store) == 120, 30), _engine_rows(store)
        assert fi.injected[(ingest, "fail")] == 2
    assert ib.engine.stats_dict()["persisted"] == 120          # each batch stepped exactly once
    assert ib.replayed_batches >= 1 and ib.raw_consumer.rewinds >= 1
    assert wait_until(lambda: inst.instance.bus.committed(group, topic, 0) == 6)
    res = _values(inst, run, tok, dev)
    assert sorted(m.value for m in res) == sorted(float(100 * b + i) for b in range(6) for i in range(20))
    assert len({m.id for m in res}) == 120
    assert not ib._stepped and not ib.engine.framed_pending


def test_overlapped_steps_on_zero_copy_records(inst):
    """Raw batches published as zero-copy framed records (what event sources write) through a tenant
    with overlapped engine steps: each record is read in place, stays retained (engine hold) until the
    engine returned its result, unregistered devices still reach the slow path from the held bytes,
    and every offset is committed once its batch is stored."""
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord
    from sitewhere_amd.pipeline.fleet import pack_messages
    from sitewhere_amd.pipeline.framing import varint_lengths
    ib, run, dev = _tenant(inst, "rpz", "gpu-columnar")
    ib.overlap = True
    bus = inst.instance.bus
    store = inst.tenant_engine("event-management", "rpz").store
    topic = inst.instance.naming.tenant_prefix("rpz") + RAW_PAYLOADS
    unreg = bus.consumer("rpz-unreg", [inst.instance.naming.unregistered_device_events("rpz")])
    recs = []
    for b in range(5):
        msgs = [wire.measurements("galaxytab-001", {"v": float(100 * b + i)}, event_date=1_700_000_300_000 + 100 * b + i)
                for i in range(30)] + [wire.measurements(f"stranger-{b}", {"v": 1.0})]
        raw, offs = pack_messages(msgs)
        rec = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1, pinned=False)
        recs.append(rec)
        rec.publish(bus, topic, 0, ts=1_700_000_400_000 + b)
    assert wait_until(lambda: _engine_rows(store) == 150, 30), _engine_rows(store)
    assert wait_until(lambda: bus.committed(ib.raw_consumer.group, topic, 0) == bus.end_offset(topic, 0))
    assert not ib.engine.framed_pending and not ib._stepped
    assert not ib._holds.get((topic, 0))                     # every engine hold released
    seen = []
    assert wait_until(lambda: seen.extend(r.key for rs in unreg.poll(50).values() for r in rs) or len(seen) >= 5)
    assert sorted(seen) == [f"stranger-{b}".encode() for b in range(5)]
    res = _values(inst, run, "rpz", dev)
    assert sorted(m.value for m in res) == sorted(float(100 * b + i) for b in range(5) for i in range(30))


def test_sync_store_failure_retries_store_not_step(inst):
    """gpu template (synchronous object storage): the event-management call fails after the step.
    The re-read batch reuses its StepResult -- before the fix it was re-stepped and every event with
    an alternate id was rejected as a duplicate of itself and silently lost."""
    ib, run, dev = _tenant(inst, "rps", "gpu")
    assert not ib.async_store
    mgmt = inst.tenant_engine("event-management", "rps").management
    topic = inst.instance.naming.tenant_prefix("rps") + RAW_PAYLOADS
    with FaultInjector() as fi:
        fi.fail_next(mgmt, "add_enriched_events", 2)
        for b in range(4):
            inst.instance.bus.append(topic, 0, [(None, _raw_batch(b))], ts=1_700_000_200_000 + b)
        assert wait_until(lambda: len(_values(inst, run, "rps", dev)) >= 80, 30)
    assert ib.engine.stats_dict()["persisted"] == 80
    assert ib.engine.stats_dict().get("duplicates", 0) == 0
    res = _values(inst, run, "rps", dev)
    assert sorted(m.value for m in res) == sorted(float(100 * b + i) for b in range(4) for i in range(20))
    assert len({m.id for m in res}) == 80
    assert ib.replayed_batches >= 1


def test_checkpoint_refuses_unstored_batches(inst, tmp_path):
    ib, _, _ = _tenant(inst, "rpc", "gpu-columnar")
    ib.ckpt_path = str(tmp_path / "shard.safetensors")
    ib._stepped[("t", 0, 5)] = object()
    try:
        with pytest.raises(RuntimeError, match="refusing to checkpoint"):
            ib.checkpoint()
    finally:
        ib._stepped.clear()
        ib.ckpt_path = None


def test_poison_raw_record_is_dead_lettered_not_retried(inst):
    """A raw record that fails validation before it is stepped (truncated varint lengths, framing that
    does not add up) goes to ``<topic>.dead-letter`` and its offset is committed in order; the good
    batches around it are stored exactly once."""
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord
    from sitewhere_amd.runtime.consumers import BusConsumer
    ib, run, dev = _tenant(inst, "rpp", "gpu-columnar")
    topic = inst.instance.naming.tenant_prefix("rpp") + RAW_PAYLOADS
    bus = inst.instance.bus
    good = [wire.measurements("galaxytab-001", {"v": float(i)}, event_date=1_700_000_000_000 + i,
                              alternate_id=f"pp-{i}") for i in range(10)]
    rec = RawBatchRecord.from_payloads(good, pinned=False).value()
    bad = bytearray(rec)
    bad[-1] |= 0x80                     # the last varint length now has its continuation bit set
    bus.append(topic, 0, [(None, rec[:64] + b"")], ts=1_700_000_200_000)   # header only: corrupt
    bus.append(topic, 0, [(None, bytes(bad))], ts=1_700_000_200_001)
    bus.append(topic, 0, [(None, rec)], ts=1_700_000_200_002)
    end = bus.end_offset(topic, 0)
    assert wait_until(lambda: bus.committed(ib.raw_consumer.group, topic, 0) == end)
    assert ib.dead_lettered == 2
    dl = topic + BusConsumer.DEAD_LETTER_SUFFIX
    assert sum(bus.end_offset(dl, p) for p in range(bus.partitions(dl))) == 2
    assert wait_until(lambda: sorted(e.value for e in _values(inst, run, "rpp", dev)) == [float(i) for i in range(10)])


def test_durable_wait_failure_rewinds_without_loss_or_duplicates(inst):
    """The durable store's token check fails while blocks are in flight: every batch not yet
    finalized is stored again after the rewind (replayed blocks the store already holds are skipped
    by sequence), offsets commit only behind durable blocks, and each event is on disk once."""
    ib, run, dev = _tenant(inst, "rpd", "gpu-columnar")
    store = inst.tenant_engine("event-management", "rpd").store
    assert ib.storage == "durable" and hasattr(store, "add_batch")
    topic = inst.instance.naming.tenant_prefix("rpd") + RAW_PAYLOADS
    with FaultInjector() as fi:
        fi.fail_next(store, "durable", 2)
        for b in range(6):
            inst.instance.bus.append(topic, 0, [(None, _raw_batch(b))], ts=1_700_000_700_000 + b)
        assert wait_until(lambda: inst.instance.bus.committed(ib.raw_consumer.group, topic, 0) == 6, 30)
        assert fi.injected[("durable", "fail")] == 2
    assert _engine_rows(store) == 120
    res = _values(inst, run, "rpd", dev)
    assert sorted(m.value for m in res) == sorted(float(100 * b + i) for b in range(6) for i in range(20))
    assert not ib._stepped and not ib._durable_wait


def test_waiting_records_coalesce_into_one_step_and_store_once(inst):
    """Framed raw records already waiting in a partition are stepped together (``coalesceRaw``): one
    engine step for several records, the rejects of each routed from its own bytes, and -- with the
    first store of the coalesced batch failing -- a rewind to its first record that stores every
    event exactly once and commits every offset."""
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord
    from sitewhere_amd.pipeline.fleet import pack_messages
    from sitewhere_amd.pipeline.framing import varint_lengths
    ib, run, dev = _tenant(inst, "rpk", "gpu-columnar")
    ib.overlap = True
    bus = inst.instance.bus
    store = inst.tenant_engine("event-management", "rpk").store
    topic = inst.instance.naming.tenant_prefix("rpk") + RAW_PAYLOADS
    unreg = bus.consumer("rpk-unreg", [inst.instance.naming.unregistered_device_events("rpk")])
    ingest = "add_batch" if hasattr(store, "add_batch") else "add_columnar"
    values, batch_values = [], []
    for b in range(8):
        msgs = [wire.measurements("galaxytab-001", {"v": float(100 * b + i)}, event_date=1_700_000_500_000 + 100 * b + i,
                                  alternate_id=f"ck-{b}-{i}") for i in range(25)] + \
               [wire.measurements(f"newcomer-{b}", {"v": 1.0})]
        values += [float(100 * b + i) for i in range(25)]
        raw, offs = pack_messages(msgs)
        rec = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1, pinned=False)
        batch_values.append(rec.value())
    steps0 = ib.step_timer.count
    with FaultInjector() as fi:
        fi.fail_next(store, ingest, 1)
        # all eight records in one append: the consumer finds them waiting together
        bus.append(topic, 0, [(None, v) for v in batch_values], ts=1_700_000_600_000)
        assert wait_until(lambda: _engine_rows(store) == 200, 30), _engine_rows(store)
        assert fi.injected[(ingest, "fail")] == 1
    assert wait_until(lambda: bus.committed(ib.raw_consumer.group, topic, 0) == bus.end_offset(topic, 0))
    assert ib.step_timer.count - steps0 < 8                    # coalesced: fewer steps than records
    assert ib.engine.stats_dict()["persisted"] == 200           # each record stepped exactly once
    assert not ib._stepped and not ib.engine.framed_pending
    res = _values(inst, run, "rpk", dev)
    assert sorted(m.value for m in res) == sorted(values) and len({m.id for m in res}) == 200
    seen = []
    assert wait_until(lambda: seen.extend(r.key for rs in unreg.poll(50).values() for r in rs) or len(seen) >= 8)
    assert sorted(seen) == sorted(f"newcomer-{b}".encode() for b in range(8))
