"""End-to-end service tests over a whole co-located instance (all microservices in one process).

Mirrors the reference's behavioural expectations: bootstrap of users / tenants /
datasets, the inbound event flow decode -> validate -> persist -> enrich -> device state / rules /
connectors, registration of unknown devices, command delivery, batch operations, schedules, labels.
"""
from __future__ import annotations

import base64
import json
import time

import pytest
from conftest import engine_knows

from sitewhere_amd.assembly import SiteWhereInstance
from sitewhere_amd.models import wire
from sitewhere_amd.models.domain import DeviceEventType


def _engine_diag(ib, dev) -> str:
    """What an inbound engine did with a device's events: its counters, and the device's registry
    row on the host and (GPU engine) in HBM."""
    import numpy as np
    e = ib.engine
    out = {"stats": {k: v for k, v in e.stats_dict().items() if v}}
    with ib._lock:
        di = ib.dev_index.idx.get(dev.id)
        slot = int(e.dev_slot[di]) if di is not None else -1
        out["dev"], out["slot"] = di, slot
        if slot >= 0:
            out["host_row"] = e.packed_registry(np.array([slot])).tolist()
            if isinstance(getattr(e, "t", None), dict) and "reg" in e.t:
                out["gpu_row"] = e.t["reg"].view(-1, 4)[slot].cpu().tolist()
                from sitewhere_amd.models.columnar import EVENT_REC
                r = e.t["recs"][:4 * EVENT_REC.itemsize].cpu().numpy().view(EVENT_REC)
                out["recs"] = [(int(x["fp_lo"]), int(x["fp_hi"]), int(x["etype"]), int(x["flags"])) for x in r]
                out["reg_ptr_ok"] = (e.args.reg == e.t["reg"].data_ptr(), int(e.args.reg_mask), e.cfg.reg_slots)
                out["reg_rows"] = int((e.t["reg"].view(-1, 4)[:, 0] != 0).sum().item())
                out["graph"] = (e.use_graph, e._graph is not None)
    for k in ("processed_events", "persisted_events"):
        m = getattr(ib, k, None)
        out[k] = getattr(m, "_count", None)
    out["store_error"] = repr(getattr(ib, "_store_error", None))
    out["stepped"] = len(getattr(ib, "_stepped", ()))
    print("engine diag:", out)
    return str(out)


def wait_until(cond, timeout=10.0, step=0.02):
    end = time.time() + timeout
    while time.time() < end:
        v = cond()
        if v:
            return v
        time.sleep(step)
    return cond()


@pytest.fixture(scope="module")
def sw():
    inst = SiteWhereInstance().start()
    inst.wait_for_tenant("default", 60)
    yield inst
    inst.stop()


def as_system(sw, fn, tenant="default"):
    return sw.instance.system_user.run(fn, tenant)


def test_instance_bootstrap(sw):
    um = sw.api("UserManagement")
    tm = sw.api("TenantManagement")
    users = as_system(sw, lambda: um.list_users())
    assert {u.username for u in users.results} >= {"admin", "noadmin"}
    t = as_system(sw, lambda: tm.get_tenant_by_token("default"))
    assert t is not None and t.dataset_template_id == "construction"
    dm = sw.api("DeviceManagement", "default")
    assert as_system(sw, lambda: dm.list_devices({"pageSize": 0}).num_results) == 23      # 3 scripted + 20 demo
    am = sw.api("AssetManagement", "default")
    assert as_system(sw, lambda: am.list_assets().num_results) == 21
    sm = sw.api("ScheduleManagement", "default")
    assert as_system(sw, lambda: sm.get_schedule_by_token("every-hour")) is not None


def test_authentication(sw):
    um = sw.api("UserManagement")
    u = as_system(sw, lambda: um.authenticate("admin", "password", True))
    assert u.username == "admin"
    with pytest.raises(Exception):
        as_system(sw, lambda: um.authenticate("admin", "wrong", False))


def test_event_flow_measurement_to_state(sw):
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    em = sw.api("DeviceEventManagement", "default")
    dev = as_system(sw, lambda: dm.get_device_by_token("meitrack-001"))
    aid = dev.device_assignment_id
    n = es.inject("default-protobuf", wire.measurements("meitrack-001", {"engine.temp": 91.5}, event_date=1_700_000_000_000))
    assert n == 1
    res = wait_until(lambda: as_system(sw, lambda: em.list_measurements_for_index("Assignment", [aid])).results)
    assert res and res[0].name == "engine.temp" and res[0].value == 91.5
    assert res[0].device_id == dev.id and res[0].customer_id is not None
    ds = sw.api("DeviceStateManagement", "default")
    st = wait_until(lambda: as_system(sw, lambda: ds.get_device_state_by_device_assignment_id(aid)))
    assert st is not None
    assert wait_until(lambda: "engine.temp" in (as_system(sw, lambda: ds.get_device_state_by_device_assignment_id(aid))
                                                .last_measurement_event_ids or {}))


def test_event_flow_location_and_alert(sw):
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    em = sw.api("DeviceEventManagement", "default")
    aid = as_system(sw, lambda: dm.get_device_by_token("meitrack-002")).device_assignment_id
    es.inject("default-protobuf", wire.location("meitrack-002", 34.1025, -84.2420, 300.0))
    es.inject("default-protobuf", wire.alert("meitrack-002", "engine.overheat", "too hot"))
    locs = wait_until(lambda: as_system(sw, lambda: em.list_locations_for_index("Assignment", [aid])).results)
    assert abs(locs[0].latitude - 34.1025) < 1e-9 and locs[0].elevation == 300.0
    alerts = wait_until(lambda: as_system(sw, lambda: em.list_alerts_for_index("Assignment", [aid])).results)
    assert alerts[0].type == "engine.overheat" and alerts[0].message == "too hot"


def test_json_decoder_and_duplicates(sw):
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    em = sw.api("DeviceEventManagement", "default")
    aid = as_system(sw, lambda: dm.get_device_by_token("iphone6s-000")).device_assignment_id
    import json
    body = json.dumps({"deviceToken": "iphone6s-000", "type": "DeviceMeasurement",
                       "request": {"name": "battery", "value": 0.5, "alternateId": "alt-batt-1"}}).encode()
    es.inject("default-json", body)
    got = wait_until(lambda: as_system(sw, lambda: em.get_device_event_by_alternate_id("alt-batt-1")))
    assert got is not None and got.device_assignment_id == aid
    es.inject("default-json", body)       # duplicate alternate id -> dropped by the deduplicator
    time.sleep(0.3)
    res = as_system(sw, lambda: em.list_measurements_for_index("Assignment", [aid])).results
    assert sum(1 for e in res if e.alternate_id == "alt-batt-1") == 1


def test_unregistered_device_registration(sw):
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    es.inject("default-protobuf", wire.registration("new-device-001", "raspberrypi"))
    dev = wait_until(lambda: as_system(sw, lambda: dm.get_device_by_token("new-device-001")), timeout=10)
    assert dev is not None
    assert wait_until(lambda: as_system(sw, lambda: dm.get_device_by_token("new-device-001")).device_assignment_id)


def test_command_invocation_delivery(sw):
    dm = sw.api("DeviceManagement", "default")
    em = sw.api("DeviceEventManagement", "default")
    dev = as_system(sw, lambda: dm.get_device_by_token("galaxytab-000"))
    cmd = as_system(sw, lambda: dm.get_device_command_by_token("galaxytab-ping"))
    inv = as_system(sw, lambda: em.add_command_invocations(dev.device_assignment_id, {
        "initiator": "REST", "initiatorId": "admin", "target": "Assignment", "commandToken": cmd.token,
        "deviceCommandId": cmd.id, "parameterValues": {}}))
    assert inv[0].event_type == DeviceEventType.CommandInvocation
    cd = sw.tenant_engine("command-delivery")
    prov = cd.destinations["default"].provider
    assert wait_until(lambda: len(prov.delivered) >= 1)


def test_batch_operation(sw):
    dm = sw.api("DeviceManagement", "default")
    bm = sw.api("BatchManagement", "default")
    ids = [as_system(sw, lambda t=t: dm.get_device_by_token(t)).id for t in ("openhab-000", "openhab-001")]
    op = as_system(sw, lambda: bm.create_batch_command_invocation({"token": "batch-1", "commandToken": "openhab-ping",
                                                                  "deviceIds": ids}))
    done = wait_until(lambda: as_system(sw, lambda: bm.get_batch_operation(op.id)).processing_status.value
                      .startswith("Finished"))
    assert done
    els = as_system(sw, lambda: bm.list_batch_operation_elements(op.id)).results
    assert [e.processing_status.value for e in els] == ["Succeeded", "Succeeded"]


def test_label_generation_png(sw):
    lg = sw.api("LabelGeneration", "default")
    dm = sw.api("DeviceManagement", "default")
    dev = as_system(sw, lambda: dm.get_device_by_token("galaxytab-001"))
    label = as_system(sw, lambda: lg.get_device_label("qrcode", dev.id))
    assert label.content.startswith(b"\x89PNG")


def test_tenant_engine_state_and_topology(sw):
    dm_ms = sw["device-management"]
    assert dm_ms.mt_management.check_tenant_engine_available("default")
    tree = dm_ms.state_tree()
    assert tree["tenantEngines"]["default"] in ("Started", "StartedWithErrors")


def test_new_tenant_gpu_template_cpu_engine():
    """Tenant on the MI355X template: inbound runs the fused engine (CPU oracle when no GPU)."""
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "fast", "name": "Fast",
                                                                "configurationTemplateId": "gpu",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("fast", 60)
        # route the protobuf source through the raw path
        ib = inst.tenant_engine("inbound-processing", "fast")
        assert ib.engine_kind in ("cpu", "gpu")
        dm = inst.api("DeviceManagement", "fast")
        em = inst.api("DeviceEventManagement", "fast")
        run = lambda f: inst.instance.system_user.run(f, "fast")  # noqa: E731
        dev = run(lambda: dm.get_device_by_token("meitrack-000"))
        assert wait_until(lambda: engine_knows(ib, dev))
        api = inst.api("InboundProcessing", "fast")
        r = run(lambda: api.process_payloads([wire.measurements("meitrack-000", {"rpm": 1200.0}),
                                              wire.location("meitrack-000", 34.10, -84.24),
                                              wire.measurements("nobody", {"x": 1.0})]))
        assert r["persisted"] == 2, (r, _engine_diag(ib, dev))
        ms = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id])).results
        assert ms and ms[0].name == "rpm" and ms[0].value == 1200.0
        st = run(lambda: api.get_statistics())
        assert st["engine.unregistered"] >= 1
        # an assignment's update ahead of its device's (the change feed does not order them): the
        # engine registers the device from device management at once, not when its event comes
        from types import SimpleNamespace
        from sitewhere_amd.pipeline.fleet import fingerprint_str
        late = SimpleNamespace(id="late-dev-id", token="late-device-1", device_type_id=None)
        dm_stub = SimpleNamespace(get_device=lambda i: late if i == late.id else None)
        ib._dm = lambda: dm_stub
        try:
            ib._upsert_assignment(SimpleNamespace(id="late-asg-id", device_id=late.id, status="Active",
                                                  customer_id=None, area_id=None, asset_id=None))
        finally:
            del ib._dm
        di = ib.dev_index.idx.get(late.id)
        assert di is not None and ib.engine.lookup_device(*fingerprint_str(late.token)) == di
        assert int(ib.engine.dev_asg[di]) == ib.asg_index.idx.get("late-asg-id")
    finally:
        inst.stop()


@pytest.mark.gpu
@pytest.mark.skipif(not __import__("conftest").gpu_available(), reason="needs an MI355X GPU")
def test_gpu_tenant_engine_on_device():
    """On an MI355X the MI355X tenant template runs the HIP engine (no silent CPU fallback)."""
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "fastgpu", "name": "Fast",
                                                                "configurationTemplateId": "gpu",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("fastgpu", 120)
        ib = inst.tenant_engine("inbound-processing", "fastgpu")
        assert ib.engine_kind == "gpu"
        run = lambda f: inst.instance.system_user.run(f, "fastgpu")  # noqa: E731
        dm = inst.api("DeviceManagement", "fastgpu")
        em = inst.api("DeviceEventManagement", "fastgpu")
        dev = run(lambda: dm.get_device_by_token("meitrack-000"))
        assert wait_until(lambda: engine_knows(ib, dev))
        api = inst.api("InboundProcessing", "fastgpu")
        r = run(lambda: api.process_payloads([wire.measurements("meitrack-000", {"rpm": 1200.0}),
                                              wire.location("meitrack-000", 34.10, -84.24),
                                              wire.measurements("nobody", {"x": 1.0})]))
        assert r["persisted"] == 2, (r, _engine_diag(ib, dev))
        ms = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id])).results
        assert ms and ms[0].name == "rpm" and ms[0].value == 1200.0
        st = run(lambda: api.get_device_state(dev.device_assignment_id))
        assert "rpm" in st["measurements"]
    finally:
        inst.stop()


def test_streaming_media_chunks(sw):
    sm = sw.api("StreamingMedia", "default")
    dm = sw.api("DeviceManagement", "default")
    dev = as_system(sw, lambda: dm.get_device_by_token("openhab-002"))
    ack = as_system(sw, lambda: sm.handle_device_stream_request("openhab-002", {"streamId": "cam1",
                                                                                 "contentType": "video/mp4"}))
    assert ack["state"] == "STREAM_CREATED"
    assert as_system(sw, lambda: sm.handle_device_stream_request("openhab-002", {"streamId": "cam1"}))["state"] == \
        "STREAM_EXISTS"
    for seq, chunk in ((2, b"world"), (1, b"hello ")):          # out of order
        as_system(sw, lambda seq=seq, chunk=chunk: sm.add_device_stream_data(dev.device_assignment_id, "cam1", seq, chunk))
    assert as_system(sw, lambda: sm.get_stream_content(dev.device_assignment_id, "cam1")) == b"hello world"
    with pytest.raises(Exception):
        as_system(sw, lambda: sm.add_device_stream_data(dev.device_assignment_id, "nope", 1, b"x"))


def test_stream_chunks_are_durable_in_the_configured_datastore(tmp_path):
    """Chunks go to the tenant's datastore (SQLite here): a new manager over the same file --
    a restarted streaming-media engine -- reassembles the stream; a re-sent chunk replaces itself."""
    from types import SimpleNamespace

    from sitewhere_amd.persistence.store import create_store
    from sitewhere_amd.services.labels_media_search import DeviceStreamManager
    dm = SimpleNamespace(get_device_stream_by_stream_id=lambda a, s: object())
    eng = SimpleNamespace(ms=SimpleNamespace(api=lambda *a: dm), tenant=SimpleNamespace(token="t"))
    path = str(tmp_path / "media.db")
    m1 = DeviceStreamManager(eng, create_store("sqlite", path=path))
    for seq, chunk in ((3, b"!"), (1, b"\x00bin"), (2, b"ary"), (2, b"ARY")):
        m1.add_device_stream_data("asg-1", "cam", seq, chunk)
    m2 = DeviceStreamManager(eng, create_store("sqlite", path=path))
    assert m2.get_stream_content("asg-1", "cam") == b"\x00binARY!"
    assert m2.get_device_stream_data("asg-1", "cam", 1).data == b"\x00bin"
    assert m2.list_device_stream_data("asg-1", "cam").num_results == 3


def test_event_search_providers(sw):
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    aid = as_system(sw, lambda: dm.get_device_by_token("raspberrypi-002")).device_assignment_id
    es.inject("default-protobuf", wire.measurements("raspberrypi-002", {"humidity": 55.0}))
    search = sw.api("EventSearch", "default")
    assert [p["id"] for p in as_system(sw, lambda: search.list_search_providers())] == ["events"]
    hits = wait_until(lambda: as_system(sw, lambda: search.search("events", f"assignment:{aid} name:humidity")))
    assert hits and hits[0]["value"] == 55.0
    # Solr provider against a canned response (no Solr in the image)
    from sitewhere_amd.services.labels_media_search import SolrSearchProvider
    urls = []
    p = SolrSearchProvider("solr", "http://solr:8983/solr", get=lambda u: (urls.append(u) or
                           b'{"response": {"docs": [{"id": "e1"}]}}'))
    assert p.search("eventType:Measurement", 10) == [{"id": "e1"}]
    assert "q=eventType%3AMeasurement" in urls[0] and "rows=10" in urls[0]


def test_global_configuration_update_restarts_engines(sw):
    """Global config change -> every tenant engine of that service restarts (MultitenantMicroservice:381-409)."""
    from sitewhere_amd.runtime.config import dump_document
    ms = sw["asset-management"]
    before = ms.get_tenant_engine("default")
    sw.instance.coord.put(ms.config_path(), dump_document({"note": "changed"}))
    assert wait_until(lambda: ms.get_tenant_engine("default") is not None and
                      ms.get_tenant_engine("default") is not before and
                      ms.get_tenant_engine("default").status.value == "Started", 20)
    assert ms.config.get("note") == "changed"


def test_columnar_tenant_end_to_end():
    """gpu-columnar template: engine rows stored as columns, queried through the normal event API."""
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "col", "name": "Columnar",
                                                                "configurationTemplateId": "gpu-columnar",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("col", 60)
        run = lambda f: inst.instance.system_user.run(f, "col")  # noqa: E731
        dm = inst.api("DeviceManagement", "col")
        em = inst.api("DeviceEventManagement", "col")
        ib = inst.tenant_engine("inbound-processing", "col")
        dev = run(lambda: dm.get_device_by_token("galaxytab-001"))
        assert wait_until(lambda: engine_knows(ib, dev))
        topic = inst.instance.naming.tenant_prefix("col") + "inbound-enriched-batches"
        cons = inst.instance.bus.consumer("col-batches", [topic])
        api = inst.api("InboundProcessing", "col")
        msgs = [wire.measurements("galaxytab-001", {"temp": 20.0 + i}, event_date=1_700_000_000_000 + i)
                for i in range(50)] + [wire.location("galaxytab-001", 34.0, -84.0, event_date=1_700_000_001_000)]
        r = run(lambda: api.process_payloads(msgs))
        assert r["persisted"] == 51
        res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id],
                                                         {"pageSize": 10}))
        assert res.num_results == 50 and len(res.results) == 10
        assert [m.value for m in res.results[:3]] == [69.0, 68.0, 67.0]          # newest first
        assert res.results[0].name == "temp" and res.results[0].customer_id is not None
        loc = run(lambda: em.list_locations_for_index("Customer", [res.results[0].customer_id],
                                                      {"pageSize": 0})).results
        loc = [x for x in loc if x.latitude == 34.0 and x.device_assignment_id == dev.device_assignment_id]
        assert len(loc) == 1              # (the rest is the construction dataset's location history)
        one = run(lambda: em.get_device_event_by_id(res.results[0].id))
        assert one.value == 69.0
        rng = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id],
                                                         {"startDate": 1_700_000_000_010, "endDate": 1_700_000_000_019,
                                                          "pageSize": 0}))
        assert rng.num_results == 10
        # the same reads served from the engine's event ring (hot store) agree with event management
        hot = run(lambda: api.list_hot_events("Measurement", "Assignment", [dev.device_assignment_id], None, None,
                                              1, 10))
        assert hot["numResults"] == 50
        assert [(h.id, h.value, h.name) for h in hot["results"]] == [(m.id, m.value, m.name) for m in res.results]
        hl = run(lambda: api.list_hot_events("Location", "Customer", [res.results[0].customer_id]))
        assert hl["results"][0].latitude == 34.0 and hl["results"][0].id == loc[0].id
        got = []
        end = time.time() + 5
        while not got and time.time() < end:
            for recs in cons.poll(200).values():
                got += recs
        from sitewhere_amd.persistence.columnar import decode_batch
        b = decode_batch(got[0].value)
        assert len(b["rows"]) == 51 and "temp" in b["names"].values()
        cons.close()
    finally:
        inst.stop()


def test_gpu_template_routes_protobuf_raw_and_json_per_event():
    """gpu template: protobuf payloads reach the fused engine as raw micro-batches (size- or
    time-flushed); JSON measurements join them transcoded to protobuf (``pipeline/json_transcode``),
    metadata included: the engine rows become event objects through the step's block, which
    carries the strings (alternate ids, messages, metadata).  All end up persisted."""
    import json as _json
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "mix", "name": "Mixed",
                                                                "configurationTemplateId": "gpu",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("mix", 60)
        run = lambda f: inst.instance.system_user.run(f, "mix")  # noqa: E731
        dm = inst.api("DeviceManagement", "mix")
        em = inst.api("DeviceEventManagement", "mix")
        ib = inst.tenant_engine("inbound-processing", "mix")
        es = inst.tenant_engine("event-sources", "mix")
        dev = run(lambda: dm.get_device_by_token("iphone6s-001"))
        assert wait_until(lambda: engine_knows(ib, dev))
        for i in range(7):                                   # < rawBatchSize: flushed by the timer
            es.inject("default-protobuf", wire.measurements("iphone6s-001", {"pb": float(i)}))
        es.inject("default-json", _json.dumps({"deviceToken": "iphone6s-001", "type": "DeviceMeasurement",
                                               "request": {"name": "js", "value": 9.0}}).encode())
        es.inject("default-json", _json.dumps({"deviceToken": "iphone6s-001", "type": "DeviceMeasurement",
                                               "request": {"name": "jm", "value": 3.0,
                                                           "metadata": {"unit": "C"}}}).encode())

        def names():
            res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id],
                                                             {"pageSize": 0})).results
            return sorted(m.name for m in res)
        assert wait_until(lambda: names() == ["jm", "js"] + ["pb"] * 7, 20), names()
        assert ib.engine.stats_dict()["events"] >= 9               # 7 protobuf + the 2 transcoded JSON
        assert es.manager.sources["default-json"].transcoded == 2
        res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id],
                                                         {"pageSize": 0})).results
        assert next(m for m in res if m.name == "jm").metadata == {"unit": "C"}   # the engine path kept it
    finally:
        inst.stop()


def test_device_stream_over_the_wire(sw):
    """Stream create + out-of-order chunks sent as protobuf device messages reach streaming media."""
    es = sw.tenant_engine("event-sources")
    dm = sw.api("DeviceManagement", "default")
    sm = sw.api("StreamingMedia", "default")
    dev = as_system(sw, lambda: dm.get_device_by_token("openhab-003"))
    es.inject("default-protobuf", wire.stream_create("openhab-003", "mic", "audio/wav"))
    assert wait_until(lambda: as_system(sw, lambda: dm.get_device_stream_by_stream_id(dev.device_assignment_id, "mic")))
    es.inject("default-protobuf", wire.stream_data("openhab-003", "mic", 2, b"-two"))
    es.inject("default-protobuf", wire.stream_data("openhab-003", "mic", 1, b"one"))
    assert wait_until(lambda: as_system(sw, lambda: sm.get_stream_content(dev.device_assignment_id, "mic")) == b"one-two")
    # the device requests chunk 2 back: delivered as a system command through command delivery
    prov = sw.tenant_engine("command-delivery").destinations["default"].provider
    es.inject("default-protobuf", wire.stream_data_request("openhab-003", "mic", 2))

    def _chunk(p):
        body = json.loads(p[2]).get("systemCommand", {})
        return base64.b64decode(body["data"]["base64"]) if body.get("type") == "DeviceStreamData" else None
    assert wait_until(lambda: any(_chunk(p) == b"-two" for p in prov.delivered))


def test_protobuf_system_command_downlinks():
    """Stream acks / chunks use the typed Device.proto downlinks (ACK_DEVICE_STREAM, RECEIVE_DEVICE_STREAM_DATA)."""
    from types import SimpleNamespace

    from sitewhere_amd.services.command_delivery import ProtobufEncoder
    enc = ProtobufEncoder()
    nest = {"gateway": SimpleNamespace(token="gw-1"), "path": "bus/sensor"}
    cmd, path, body = wire.decode_device_command(
        enc.encode_system({"type": "DeviceStreamAck", "streamId": "mic", "state": "STREAM_EXISTS"}, nest))
    assert (cmd, path, body.streamId, body.state) == (wire.ACK_DEVICE_STREAM, "bus/sensor", "mic", 2)
    cmd, path, body = wire.decode_device_command(
        enc.encode_system({"type": "DeviceStreamData", "streamId": "mic", "sequenceNumber": 7, "data": b"\x00\x01"}, nest))
    assert cmd == wire.RECEIVE_DEVICE_STREAM_DATA and body.hardwareId == "gw-1"
    assert (body.streamId, body.sequenceNumber, body.data) == ("mic", 7, b"\x00\x01")
    cmd, _, body = wire.decode_device_command(enc.encode_system({"type": "RegistrationAck", "state": "NEW_REGISTRATION"}, {}))
    assert cmd == wire.ACK_REGISTRATION and body.state == 1


def test_gpu_tenant_checkpoint_resume_replays_exactly(tmp_path):
    """Checkpoint-aligned commits: after an unclean restart the MI355X tenant engine restores its
    snapshot, replays the raw batches after it with the same event ids, and the columnar store
    skips the rows it already holds -- every payload persisted exactly once."""
    import struct

    from sitewhere_amd.runtime.config import dump_document
    from sitewhere_amd.services.event_sources import RAW_PAYLOADS
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "ck", "name": "ck",
                                                                "configurationTemplateId": "gpu-columnar",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("ck", 60)
        ms = inst["inbound-processing"]
        path = str(tmp_path / "ck-shard.safetensors")

        def reconfigure(note):
            cfg = dict(ms.get_tenant_engine("ck").config)
            cfg.update(checkpoint={"path": path, "everyBatches": 2}, note=note)
            before = ms.get_tenant_engine("ck")
            inst.instance.coord.put(ms.tenant_config_path("ck"), dump_document(cfg))
            assert wait_until(lambda: ms.get_tenant_engine("ck") is not None and ms.get_tenant_engine("ck") is not before
                              and ms.get_tenant_engine("ck").status.value == "Started", 30)
            return ms.get_tenant_engine("ck")

        ib = reconfigure(1)
        run = lambda f: inst.instance.system_user.run(f, "ck")  # noqa: E731
        dm = inst.api("DeviceManagement", "ck")
        dev = run(lambda: dm.get_device_by_token("galaxytab-001"))
        assert wait_until(lambda: engine_knows(ib, dev))
        topic = inst.instance.naming.tenant_prefix("ck") + RAW_PAYLOADS

        def raw_batch(b):
            msgs = [wire.measurements("galaxytab-001", {"v": float(100 * b + i)}, event_date=1_700_000_000_000 + 100 * b + i)
                    for i in range(20)]
            return struct.pack(f"<I{len(msgs)}I", len(msgs), *[len(m) for m in msgs]) + b"".join(msgs)

        for b in range(5):
            inst.instance.bus.append(topic, 0, [(None, raw_batch(b))], ts=1_700_000_100_000 + b)
        assert wait_until(lambda: ib.engine.stats_dict()["persisted"] == 100, 20)
        assert ib.checkpoints == 2                       # after batches 2 and 4; batch 5 not yet covered
        store = inst.tenant_engine("event-management", "ck").store
        # stored (on disk) on the store thread; the store also holds the dataset's API-added events
        assert wait_until(lambda: getattr(store, "engine_rows", store.rows) == 100, 20)
        ib._since_ckpt = 0                               # "crash": no final snapshot on stop
        ib2 = reconfigure(2)
        assert ib2 is not ib
        assert wait_until(lambda: ib2.engine.stats_dict()["persisted"] == 100, 20)   # 80 restored + 20 replayed
        assert getattr(store, "engine_rows", store.rows) == 100      # the replayed batch was not stored twice
        em = inst.api("DeviceEventManagement", "ck")
        res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id], {"pageSize": 0}))
        vals = sorted(m.value for m in res.results)
        assert vals == sorted(float(100 * b + i) for b in range(5) for i in range(20))
        assert len({m.id for m in res.results}) == 100
    finally:
        inst.stop()


@pytest.mark.gpu
@pytest.mark.skipif(not __import__("conftest").gpu_available(), reason="needs an MI355X GPU")
@pytest.mark.parametrize("zero_copy_rows", [False, True])
def test_gpu_columnar_tenant_overlapped_steps_from_pinned_records(zero_copy_rows):
    """The MI355X columnar tenant steps raw batches overlapped (H2D of batch k+1 and the row D2H of
    batch k-1 beside the compute of batch k), straight from pinned zero-copy topic records: every
    measurement stored once, unregistered devices routed, offsets committed, record holds released.
    With ``zeroCopyRows`` the columnar payloads are framed in the engine's pinned row buffers and
    the engine's enriched batches stay on one topic partition."""
    from sitewhere_amd.pipeline.bus_io import RawBatchRecord
    from sitewhere_amd.pipeline.fleet import pack_messages
    from sitewhere_amd.pipeline.framing import varint_lengths
    from sitewhere_amd.services.event_sources import RAW_PAYLOADS
    inst = SiteWhereInstance().start()
    try:
        inst.wait_for_tenant("default", 60)
        tm = inst.api("TenantManagement")
        inst.instance.system_user.run(lambda: tm.create_tenant({"token": "ovl", "name": "ovl",
                                                                "configurationTemplateId": "gpu-columnar",
                                                                "datasetTemplateId": "construction"}))
        inst.wait_for_tenant("ovl", 120)
        if zero_copy_rows:
            from sitewhere_amd.runtime.config import dump_document
            ms = inst["inbound-processing"]
            before = ms.get_tenant_engine("ovl")
            inst.instance.coord.put(ms.tenant_config_path("ovl"), dump_document(dict(before.config, zeroCopyRows=True)))
            assert wait_until(lambda: ms.get_tenant_engine("ovl") not in (None, before)
                              and ms.get_tenant_engine("ovl").status.value == "Started", 120)
        ib = inst.tenant_engine("inbound-processing", "ovl")
        assert ib.engine_kind == "gpu" and ib.overlap and ib.async_store and ib.zero_copy_rows == zero_copy_rows
        run = lambda f: inst.instance.system_user.run(f, "ovl")  # noqa: E731
        dev = run(lambda: inst.api("DeviceManagement", "ovl").get_device_by_token("galaxytab-001"))
        assert wait_until(lambda: engine_knows(ib, dev))
        _engine_diag(ib, dev)                   # printed (shown on failure): the registry row before the batches
        bus = inst.instance.bus
        topic = inst.instance.naming.tenant_prefix("ovl") + RAW_PAYLOADS
        unreg = bus.consumer("ovl-unreg", [inst.instance.naming.unregistered_device_events("ovl")])
        store = inst.tenant_engine("event-management", "ovl").store
        recs = []
        for b in range(8):
            msgs = [wire.measurements("galaxytab-001", {"v": float(1000 * b + i)},
                                      event_date=1_700_000_000_000 + 1000 * b + i) for i in range(200)]
            msgs.append(wire.measurements(f"stranger-{b}", {"v": 1.0}))
            raw, offs = pack_messages(msgs)
            rec = RawBatchRecord(raw[:int(offs[-1])], varint_lengths(offs), len(offs) - 1)
            recs.append(rec)
            rec.publish(bus, topic, 0, ts=1_700_000_500_000 + b)
        assert wait_until(lambda: getattr(store, "engine_rows", store.rows) == 1600, 60), \
            (getattr(store, "engine_rows", store.rows), _engine_diag(ib, dev))
        assert wait_until(lambda: bus.committed(ib.raw_consumer.group, topic, 0) == bus.end_offset(topic, 0), 30)
        assert not ib.engine.framed_pending and not ib._stepped and not ib._holds.get((topic, 0))
        seen = []
        assert wait_until(lambda: seen.extend(r.key for rs in unreg.poll(50).values() for r in rs) or len(seen) >= 8)
        assert sorted(seen) == sorted(f"stranger-{b}".encode() for b in range(8))
        em = inst.api("DeviceEventManagement", "ovl")
        res = run(lambda: em.list_measurements_for_index("Assignment", [dev.device_assignment_id], {"pageSize": 0}))
        assert sorted(m.value for m in res.results) == sorted(float(1000 * b + i) for b in range(8) for i in range(200))
        t_out = inst.instance.naming.tenant_prefix("ovl") + "inbound-enriched-batches"
        used = [p for p in range(bus.partitions(t_out)) if bus.end_offset(t_out, p) > 0]
        # durable batches are framed around the GPU-encoded block in its pinned buffer either way
        assert ib.storage == "durable" and ib.zc_framed > 0
        if zero_copy_rows:
            assert used == [ib._sticky_part]
        else:
            assert len(used) > 1                                      # round-robin partitions
    finally:
        inst.stop()
