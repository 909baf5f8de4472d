"""Data-plane topic payloads as the reference's protobuf messages.

* the schema keeps the reference's field numbers and types, checked message by message against
  the reference ``.proto`` files (when the reference tree is present);
* every payload kind round-trips through protobuf, including values the reference messages
  have no field for (non-UUID ids, deviceCommandId, undelivered errors);
* a whole instance runs with ``SITEWHERE_TOPIC_CODEC=protobuf``: decoded / persisted / enriched /
  unregistered records on the bus are reference-format protobuf and the pipeline outcome is the
  same as with JSON.
"""
from __future__ import annotations

import os
import re
import time

import pytest

from sitewhere_amd.bus import payloads
from sitewhere_amd.models import domain

REF = "/root/reference"
REF_PROTOS = [f"{REF}/sitewhere-grpc-model/src/main/proto/sitewhere-common.proto",
              f"{REF}/sitewhere-grpc-event-management/src/main/proto/device-event-model.proto",
              f"{REF}/sitewhere-grpc-model/src/main/proto/sitewhere-kafka.proto"]


def _ref_messages() -> dict:
    """{message: {field: (number, type)}} from the reference .proto text (regex level)."""
    out: dict = {}
    for path in REF_PROTOS:
        text = re.sub(r"//[^\n]*", "", open(path).read())
        for m in re.finditer(r"message\s+(\w+)\s*\{", text):
            depth, i = 1, m.end()
            while depth:
                depth += {"{": 1, "}": -1}.get(text[i], 0)
                i += 1
            body = text[m.end():i - 1]
            fields = {}
            for f in re.finditer(r"(?:repeated\s+)?(map<[^>]+>|[\w.]+)\s+(\w+)\s*=\s*(\d+)\s*;", body):
                fields[f.group(2)] = (int(f.group(3)), f.group(1).split(".")[-1].replace(" ", ""))
            out[m.group(1)] = fields
    return out


@pytest.mark.skipif(not all(os.path.exists(p) for p in REF_PROTOS), reason="reference protos not present")
def test_schema_matches_the_reference_field_numbers_and_types():
    from google.protobuf.descriptor import FieldDescriptor as FD
    ref = _ref_messages()
    scalar = {FD.TYPE_DOUBLE: "double", FD.TYPE_STRING: "string", FD.TYPE_UINT64: "uint64", FD.TYPE_BOOL: "bool",
              FD.TYPE_FIXED64: "fixed64", FD.TYPE_INT64: "int64", FD.TYPE_INT32: "int32", FD.TYPE_BYTES: "bytes"}
    checked = 0
    for name, cls in payloads.messages().items():
        if not hasattr(cls, "DESCRIPTOR") or not hasattr(cls.DESCRIPTOR, "fields"):
            continue
        assert name in ref, f"{name} is not a reference message"
        for f in cls.DESCRIPTOR.fields:
            assert f.name in ref[name], f"{name}.{f.name} not in the reference"
            num, rtype = ref[name][f.name]
            assert f.number == num, (name, f.name)
            if f.message_type is not None and f.message_type.GetOptions().map_entry:
                k, v = f.message_type.fields
                want = f"map<{scalar[k.type]},{scalar[v.type]}>"
            elif f.message_type is not None:
                want = f.message_type.name
            elif f.enum_type is not None:
                want = f.enum_type.name
            else:
                want = scalar[f.type]
            assert want == rtype, (name, f.name, want, rtype)
            checked += 1
        assert len(cls.DESCRIPTOR.fields) == len(ref[name]), name
    assert checked > 100


@pytest.fixture
def protobuf_codec():
    prev = payloads.set_topic_codec("protobuf")
    yield
    payloads.set_topic_codec(prev)


def test_inbound_and_registration_round_trip(protobuf_codec):
    cases = [
        ("DeviceMeasurement", {"name": "temp", "value": 21.5, "eventDate": 1_700_000_000_123, "alternateId": "a1",
                               "updateState": True, "metadata": {"k": "v"}}),
        ("DeviceLocation", {"latitude": 33.5, "longitude": -84.25, "elevation": 310.0, "metadata": {}}),
        ("DeviceAlert", {"type": "engine.overheat", "message": "hot", "level": "Critical", "source": "Device",
                         "metadata": {}}),
        ("DeviceCommandResponse", {"originatingEventId": "6f1c7a4e-53a4-4f3e-9a57-6c2b7b9d0e11",
                                   "responseEventId": "gpu17-42", "response": "ok", "metadata": {}}),
        ("DeviceStateChange", {"attribute": "presence", "type": "presence", "previousState": "PRESENT",
                               "newState": "NOT_PRESENT", "metadata": {}}),
        ("DeviceCommandInvocation", {"initiator": "Script", "initiatorId": "s1", "targetId": "asg-1",
                                     "commandToken": "ping", "deviceCommandId": "c7", "parameterValues": {"n": "3"},
                                     "metadata": {}}),
    ]
    for t, req in cases:
        p = {"sourceId": "src", "deviceToken": "dev-1", "originator": "orig-9",
             "eventCreateRequest": {"type": t, "request": req}}
        b = payloads.encode_inbound(p)
        assert b[:1] != b"{"
        back = payloads.decode_inbound(b)
        assert back["deviceToken"] == "dev-1" and back["originator"] == "orig-9" and back["sourceId"] == "src"
        assert back["eventCreateRequest"]["type"] == t
        got = back["eventCreateRequest"]["request"]
        for k, v in req.items():
            if k == "target":
                continue
            assert got.get(k) == v, (t, k, got.get(k), v)
    reg = {"sourceId": "src", "deviceToken": "new-dev", "originator": None, "eventCreateRequest": {
        "type": "RegisterDevice", "request": {"deviceTypeToken": "sensor", "areaToken": "a", "metadata": {"m": "1"}}}}
    back = payloads.decode_inbound(payloads.encode_inbound(reg), registration=True)
    assert back["eventCreateRequest"] == {"type": "RegisterDevice", "request": {
        "deviceTypeToken": "sensor", "areaToken": "a", "metadata": {"m": "1"}}}
    # request types the reference message has no member for stay JSON (readers detect it)
    ack = {"sourceId": "s", "deviceToken": "d", "originator": None,
           "eventCreateRequest": {"type": "Acknowledge", "request": {"response": "r"}}}
    assert payloads.encode_inbound(ack)[:1] == b"{"
    assert payloads.decode_inbound(payloads.encode_inbound(ack))["eventCreateRequest"]["type"] == "Acknowledge"


def test_persisted_and_enriched_round_trip(protobuf_codec):
    ids = dict(device_id=domain.new_id(), device_assignment_id=domain.new_id(), customer_id=domain.new_id(),
               area_id=None, asset_id="forklift-7")                  # an asset referenced by token
    evs = [domain.DeviceMeasurement(name="speed", value=12.5, event_date=10, received_date=11, alternate_id="x",
                                    metadata={"q": "1"}, **ids),
           domain.DeviceLocation(id="5b3e-77", latitude=1.0, longitude=2.0, elevation=None, **ids),  # GPU-style id
           domain.DeviceAlert(source=domain.AlertSource.System, level=domain.AlertLevel.Error, type="zone.enter",
                              message="entered", **ids),
           domain.DeviceCommandInvocation(initiator=domain.CommandInitiator.BatchOperation, initiator_id="b1",
                                          target_id="t", device_command_id=domain.new_id(), command_token="reboot",
                                          parameter_values={"delay": "5"}, **ids),
           domain.DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                                    new_state="NOT_PRESENT", **ids)]
    for e in evs:
        back = payloads.decode_persisted(payloads.encode_persisted(e))
        assert type(back) is type(e) and back.to_dict() == e.to_dict(), (back.to_dict(), e.to_dict())
    ctx = {"deviceId": ids["device_id"], "deviceTypeId": domain.new_id(), "parentDeviceId": None,
           "deviceStatus": "ok", "deviceMetadata": {"fw": "1.2"}, "assignmentStatus": "Active",
           "assignmentMetadata": {"site": "a"}, "deviceToken": "dev-1"}
    b = payloads.encode_enriched(evs[3], ctx, error="no route")
    m = payloads.messages()["GEnrichedEventPayload"].FromString(b)
    assert m.event.WhichOneof("event") == "commandInvocation" and m.context.assignmentStatus == 1
    ev, back_ctx, err = payloads.decode_enriched(b, b"dev-1")
    assert ev.to_dict() == evs[3].to_dict() and err == "no route" and back_ctx == ctx
    # JSON records keep decoding whatever the writer mode
    payloads.set_topic_codec("json")
    ev2, ctx2, err2 = payloads.decode_enriched(payloads.encode_enriched(evs[0], ctx), None)
    assert ev2.to_dict() == evs[0].to_dict() and ctx2 == ctx and err2 is None


def test_whole_instance_on_protobuf_topics(protobuf_codec):
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.models import wire
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        n, bus = sw.instance.naming, sw.instance.bus
        topics = {"decoded": n.decoded_events("default"), "persisted": n.inbound_persisted_events("default"),
                  "enriched": n.inbound_enriched_events("default"), "unregistered": n.unregistered_device_events("default")}
        cons = {k: bus.consumer(f"pb-check-{k}", [t], auto_offset_reset="latest") for k, t in topics.items()}
        for c in cons.values():
            c.poll(10)
        es = sw.tenant_engine("event-sources")
        em_engine = sw.tenant_engine("event-management")
        base = em_engine.store.count()
        t0 = int(time.time() * 1000)
        for i in range(40):
            # strictly increasing event dates: device state keeps the newest by date, and events
            # injected within one millisecond would tie
            es.inject("default-protobuf", wire.measurements("meitrack-002", {"pb": float(i)}, alternate_id=f"pb-{i}",
                                                            event_date=t0 + i))
        es.inject("default-protobuf", wire.measurements("ghost-pb", {"x": 1.0}))
        end = time.time() + 30
        while em_engine.store.count() - base < 40 and time.time() < end:
            time.sleep(0.05)
        assert all(em_engine.store.get_event_by_alternate_id(f"pb-{i}") for i in range(40))
        got: dict = {k: [] for k in topics}
        end = time.time() + 20
        while time.time() < end and (len(got["enriched"]) < 40 or not got["unregistered"]):
            for k, c in cons.items():
                for recs in c.poll(100).values():
                    got[k] += recs
        M = payloads.messages()
        for k, cls in (("decoded", "GInboundEventPayload"), ("persisted", "GPersistedEventPayload"),
                       ("enriched", "GEnrichedEventPayload"), ("unregistered", "GInboundEventPayload")):
            assert got[k], k
            for r in got[k]:
                assert bytes(r.value[:1]) != b"{", k
                M[cls].FromString(bytes(r.value))             # reference-format protobuf
        enriched = [payloads.decode_enriched(r.value, r.key) for r in got["enriched"]]
        assert {e.metadata.get("sw.id") for e, _, _ in enriched} == {None}
        assert all(ctx["deviceToken"] == "meitrack-002" and ctx["assignmentStatus"] == "Active"
                   for _, ctx, _ in enriched)
        assert payloads.decode_inbound(got["unregistered"][0].value)["deviceToken"] == "ghost-pb"
        # a downstream consumer (device state) reads the protobuf records
        dm = sw.api("DeviceManagement", "default")
        dsm = sw.api("DeviceStateManagement", "default")
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dev = run(lambda: dm.get_device_by_token("meitrack-002"))
        last = em_engine.store.get_event_by_alternate_id("pb-39").id
        end = time.time() + 20
        while time.time() < end:
            st = run(lambda: dsm.get_device_state_by_device_assignment_id(dev.device_assignment_id))
            if st is not None and st.last_measurement_event_ids.get("pb") == last:
                break
            time.sleep(0.05)
        assert st.last_measurement_event_ids.get("pb") == last
        for c in cons.values():
            c.close()
    finally:
        sw.stop()


def test_instance_log_messages(protobuf_codec):
    m = {"microservice": "event-sources", "hostname": "es-1", "level": "ERROR", "logger": "x",
         "message": "decode failed", "timestamp": 1_700_000_000_000, "tenant": "default",
         "exception": {"message": "ValueError: bad", "frames": [
             {"module": "event_sources", "function": "decode", "file": "/a/event_sources.py", "line": 42}]}}
    b = payloads.encode_log(m)
    p = payloads.messages()["GMicroserviceLogMessage"].FromString(b)
    assert p.level == 4 and p.microserviceContainerId == "es-1" and p.exception.elements[0].lineNumber == 42
    back = payloads.decode_log(b)
    assert back["message"] == "[default] decode failed" and back["level"] == "ERROR"
    assert back["exception"]["frames"][0]["function"] == "decode"
    tid = domain.new_id()
    assert payloads.decode_log(payloads.encode_log(dict(m, tenant=tid)))["tenant"] == tid
