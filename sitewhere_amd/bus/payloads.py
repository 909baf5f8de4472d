"""Data-plane record values: the payload messages of SURVEY §2.4, as JSON or as protobuf.

The reference puts protobuf on every data-plane topic (``GInboundEventPayload`` on decoded /
unregistered / reprocess events, ``GDeviceRegistationPayload`` on registrations,
``GPersistedEventPayload`` on persisted events, ``GEnrichedEventPayload`` on enriched events,
enriched command invocations and undelivered commands -- ``KafkaModelMarshaler`` /
``EventModelMarshaler``).  This module writes either

* ``json`` (default) -- this framework's codec (``rpc/codec.py``) documents, or
* ``protobuf`` -- the reference's messages (``models/proto/kafka_payloads.proto``, same field
  numbers), so reference producers and consumers can share the topics,

chosen by ``SITEWHERE_TOPIC_CODEC`` (or :func:`set_topic_codec`).  Readers accept both: a JSON
record starts with ``{``, a protobuf one never does (its first byte is a field tag).

Values the reference messages have no field for travel in the event's metadata under ``sw.*``
keys and are restored on read: ids that are not UUIDs (``GUUID`` is two fixed64 words; GPU
engine event ids are ``<boot>-<sequence>``, assets may be referenced by token), an invocation's
``deviceCommandId``, and an undelivered command's error.  The device token of an enriched event
is the record key, as in the reference (``EnrichedEventsProducer`` keys by device token).
"""
from __future__ import annotations

import json
import os
import uuid
from pathlib import Path

from ..models import domain
from ..rpc import codec

_MODE = os.environ.get("SITEWHERE_TOPIC_CODEC", "json").lower()
_M = None
_MASK = (1 << 64) - 1


def set_topic_codec(mode: str) -> str:
    """Switch the writer format (``json`` | ``protobuf``); returns the previous one."""
    global _MODE
    if mode not in ("json", "protobuf"):
        raise ValueError(f"topic codec must be 'json' or 'protobuf', not {mode!r}")
    prev, _MODE = _MODE, mode
    return prev


def topic_codec() -> str:
    return _MODE


def messages() -> dict:
    global _M
    if _M is None:
        from ..models.protoschema import load_proto
        text = (Path(__file__).resolve().parent.parent / "models" / "proto" / "kafka_payloads.proto").read_text()
        _M = load_proto(text, "sitewhere_amd/kafka_payloads.proto")
    return _M


def _is_json(value) -> bool:
    return bool(value) and bytes(value[:1]) == b"{"


# ------------------------------------------------------------------------------ small helpers
def _set_uuid(msg, field: str, value, meta: dict):
    if not value:
        return
    try:
        u = uuid.UUID(str(value)).int
    except ValueError:
        meta[f"sw.{field}"] = str(value)
        return
    g = getattr(msg, field)
    g.msb, g.lsb = u >> 64, u & _MASK


def _get_uuid(msg, field: str, meta: dict):
    stashed = meta.pop(f"sw.{field}", None)
    if stashed is not None:
        return stashed
    if not msg.HasField(field):
        return None
    g = getattr(msg, field)
    return str(uuid.UUID(int=(g.msb << 64) | g.lsb))


def _opt(msg, field: str):
    return getattr(msg, field).value if msg.HasField(field) else None


_LEVELS = ["Info", "Warning", "Error", "Critical"]
_SOURCES = ["Device", "System"]
_INITIATORS = ["REST", "BatchOperation", "Script", "Scheduler"]
_ASSN = {"Active": 1, "Missing": 2, "Released": 3}
_ASSN_BACK = {v: k for k, v in _ASSN.items()}
_ONEOF = {"DeviceMeasurement": "measurement", "DeviceAlert": "alert", "DeviceLocation": "location",
          "DeviceCommandInvocation": "commandInvocation", "DeviceCommandResponse": "commandResponse",
          "DeviceStateChange": "stateChange"}
_ONEOF_BACK = {v: k for k, v in _ONEOF.items()}
_EVENT_ONEOF = {domain.DeviceEventType.Measurement: "measurement", domain.DeviceEventType.Alert: "alert",
                domain.DeviceEventType.Location: "location",
                domain.DeviceEventType.CommandInvocation: "commandInvocation",
                domain.DeviceEventType.CommandResponse: "commandResponse",
                domain.DeviceEventType.StateChange: "stateChange"}
_EVENT_CLASS = {v: domain.EVENT_CLASSES[k] for k, v in _EVENT_ONEOF.items()}
_ETYPE_NUM = {"measurement": 0, "location": 1, "alert": 2, "commandInvocation": 3, "commandResponse": 4,
              "stateChange": 5}


# ------------------------------------------------------------------------------ create requests
def _create_header(h, req: dict):
    meta = {str(k): str(v) for k, v in (req.get("metadata") or {}).items()}
    for k in ("alternateId", "customerToken", "areaToken", "assetToken"):
        if req.get(k) is not None:
            getattr(h, k).value = str(req[k])
    if req.get("eventDate") is not None:
        h.eventDate = int(req["eventDate"])
    if req.get("updateState") is not None:
        h.updateState.value = bool(req["updateState"])
    return meta


def _create_request(any_req, type_: str, req: dict) -> bool:
    """Fill ``GAnyDeviceEventCreateRequest``; False for request types it has no member for."""
    name = _ONEOF.get(type_)
    if name is None:
        return False
    m = getattr(any_req, name)
    meta = _create_header(m.event, req)
    if name == "measurement":
        m.name, m.value = str(req.get("name", "")), float(req.get("value", 0.0))
    elif name == "location":
        for k in ("latitude", "longitude", "elevation"):
            if req.get(k) is not None:
                getattr(m, k).value = float(req[k])
    elif name == "alert":
        m.source = _SOURCES.index(req.get("source") or "Device")
        m.level = _LEVELS.index(req.get("level") or "Info")
        m.type, m.alertMessage = str(req.get("type", "")), str(req.get("message", ""))
    elif name == "commandInvocation":
        m.initiator = _INITIATORS.index(req.get("initiator") or "REST")
        m.initiatorId = str(req.get("initiatorId") or "")
        if req.get("targetId"):
            m.targetId.value = str(req["targetId"])
        m.commandToken = str(req.get("commandToken") or "")
        m.parameterValues.update({str(k): str(v) for k, v in (req.get("parameterValues") or {}).items()})
        if req.get("deviceCommandId"):
            meta["sw.deviceCommandId"] = str(req["deviceCommandId"])
    elif name == "commandResponse":
        _set_uuid(m, "originatingEventId", req.get("originatingEventId"), meta)
        _set_uuid(m, "responseEventId", req.get("responseEventId"), meta)
        if req.get("response") is not None:
            m.response.value = str(req["response"])
    elif name == "stateChange":
        m.attribute, m.type = str(req.get("attribute", "")), str(req.get("type", ""))
        for k in ("previousState", "newState"):
            if req.get(k) is not None:
                getattr(m, k).value = str(req[k])
    m.event.metadata.update(meta)
    return True


def _request_dict(any_req) -> tuple[str, dict]:
    name = any_req.WhichOneof("event")
    if name is None:
        raise ValueError("GAnyDeviceEventCreateRequest without an event")
    m = getattr(any_req, name)
    h = m.event
    meta = dict(h.metadata)
    req: dict = {"metadata": meta}
    for k in ("alternateId", "customerToken", "areaToken", "assetToken"):
        if h.HasField(k):
            req[k] = getattr(h, k).value
    if h.eventDate:
        req["eventDate"] = h.eventDate
    if h.HasField("updateState"):
        req["updateState"] = h.updateState.value
    if name == "measurement":
        req.update(name=m.name, value=m.value)
    elif name == "location":
        for k in ("latitude", "longitude", "elevation"):
            if m.HasField(k):
                req[k] = getattr(m, k).value
    elif name == "alert":
        req.update(source=_SOURCES[m.source], level=_LEVELS[m.level], type=m.type, message=m.alertMessage)
    elif name == "commandInvocation":
        req.update(initiator=_INITIATORS[m.initiator], initiatorId=m.initiatorId or None, target="Assignment",
                   commandToken=m.commandToken or None, parameterValues=dict(m.parameterValues))
        if m.HasField("targetId"):
            req["targetId"] = m.targetId.value
        if "sw.deviceCommandId" in meta:
            req["deviceCommandId"] = meta.pop("sw.deviceCommandId")
    elif name == "commandResponse":
        req.update(originatingEventId=_get_uuid(m, "originatingEventId", meta),
                   responseEventId=_get_uuid(m, "responseEventId", meta), response=_opt(m, "response"))
    elif name == "stateChange":
        req.update(attribute=m.attribute, type=m.type, previousState=_opt(m, "previousState"),
                   newState=_opt(m, "newState"))
    return _ONEOF_BACK[name], req


# ------------------------------------------------------------------------------ inbound / registration
def encode_inbound(payload: dict) -> bytes:
    """``{"sourceId", "deviceToken", "originator", "eventCreateRequest": {"type", "request"}}`` ->
    record value (``GInboundEventPayload``, or ``GDeviceRegistationPayload`` for RegisterDevice)."""
    if _MODE == "protobuf":
        M = messages()
        ecr = payload.get("eventCreateRequest") or {}
        t, req = ecr.get("type"), ecr.get("request") or {}
        if t == "RegisterDevice":
            p = M["GDeviceRegistationPayload"](sourceId=payload.get("sourceId") or "",
                                               deviceToken=payload.get("deviceToken") or "")
            if payload.get("originator"):
                p.originator.value = str(payload["originator"])
            for k in ("deviceTypeToken", "customerToken", "areaToken"):
                if req.get(k):
                    getattr(p.registration, k).value = str(req[k])
            p.registration.metadata.update({str(k): str(v) for k, v in (req.get("metadata") or {}).items()})
            return p.SerializeToString()
        p = M["GInboundEventPayload"](sourceId=payload.get("sourceId") or "",
                                      deviceToken=payload.get("deviceToken") or "")
        if payload.get("originator"):
            p.originator.value = str(payload["originator"])
        if _create_request(p.event, t, req):
            return p.SerializeToString()
        # acks / streams have no member in the reference message: keep the JSON form for those
    return json.dumps(codec.to_wire(payload)).encode()


def decode_inbound(value, registration: bool = False) -> dict:
    """Record value of a decoded / unregistered / reprocess (or, with ``registration``, the
    registration) topic -> the payload dict :func:`encode_inbound` takes."""
    if _is_json(value):
        return codec.from_wire(json.loads(value))
    M = messages()
    if registration:
        p = M["GDeviceRegistationPayload"].FromString(bytes(value))
        r = p.registration
        req = {k: getattr(r, k).value for k in ("deviceTypeToken", "customerToken", "areaToken") if r.HasField(k)}
        req["metadata"] = dict(r.metadata)
        t = "RegisterDevice"
    else:
        p = M["GInboundEventPayload"].FromString(bytes(value))
        t, req = _request_dict(p.event)
    return {"sourceId": p.sourceId, "deviceToken": p.deviceToken, "originator": _opt(p, "originator"),
            "eventCreateRequest": {"type": t, "request": req}}


# ------------------------------------------------------------------------------ events
def _event_message(any_ev, e: domain.DeviceEvent) -> dict:
    name = _EVENT_ONEOF[e.event_type]
    m = getattr(any_ev, name)
    h = m.event
    meta = {str(k): str(v) for k, v in (e.metadata or {}).items()}
    _set_uuid(h, "id", e.id, meta)
    if e.alternate_id:
        h.alternateId.value = e.alternate_id
    h.eventType = _ETYPE_NUM[name]
    for f, v in (("deviceId", e.device_id), ("deviceAssignmentId", e.device_assignment_id),
                 ("customerId", e.customer_id), ("areaId", e.area_id), ("assetId", e.asset_id)):
        _set_uuid(h, f, v, meta)
    h.eventDate, h.receivedDate = int(e.event_date or 0), int(e.received_date or 0)
    if name == "measurement":
        m.name, m.value = e.name, float(e.value)
    elif name == "location":
        m.latitude.value, m.longitude.value = float(e.latitude), float(e.longitude)
        if e.elevation is not None:
            m.elevation.value = float(e.elevation)
    elif name == "alert":
        m.source = _SOURCES.index(getattr(e.source, "value", e.source) or "Device")
        m.level = _LEVELS.index(getattr(e.level, "value", e.level) or "Info")
        m.type, m.alertMessage = e.type or "", e.message or ""
    elif name == "commandInvocation":
        m.initiator = _INITIATORS.index(getattr(e.initiator, "value", e.initiator) or "REST")
        m.initiatorId = e.initiator_id or ""
        if e.target_id:
            m.targetId.value = e.target_id
        m.commandToken = e.command_token or ""
        m.parameterValues.update({str(k): str(v) for k, v in (e.parameter_values or {}).items()})
        if e.device_command_id:
            meta["sw.deviceCommandId"] = e.device_command_id
    elif name == "commandResponse":
        _set_uuid(m, "originatingEventId", e.originating_event_id, meta)
        _set_uuid(m, "responseEventId", e.response_event_id, meta)
        if e.response is not None:
            m.response.value = e.response
    elif name == "stateChange":
        m.attribute, m.type = e.attribute or "", e.type or ""
        if e.previous_state is not None:
            m.previousState.value = e.previous_state
        if e.new_state is not None:
            m.newState.value = e.new_state
    h.metadata.update(meta)
    return meta


def _event_object(any_ev) -> domain.DeviceEvent:
    name = any_ev.WhichOneof("event")
    if name is None:
        raise ValueError("GAnyDeviceEvent without an event")
    m = getattr(any_ev, name)
    h = m.event
    meta = dict(h.metadata)
    kw = dict(alternate_id=_opt(h, "alternateId"), event_date=h.eventDate or None,
              received_date=h.receivedDate or None)
    ident = _get_uuid(h, "id", meta)
    if ident:
        kw["id"] = ident
    for f, attr in (("deviceId", "device_id"), ("deviceAssignmentId", "device_assignment_id"),
                    ("customerId", "customer_id"), ("areaId", "area_id"), ("assetId", "asset_id")):
        kw[attr] = _get_uuid(h, f, meta)
    if name == "measurement":
        kw.update(name=m.name, value=m.value)
    elif name == "location":
        kw.update(latitude=m.latitude.value, longitude=m.longitude.value, elevation=_opt(m, "elevation"))
    elif name == "alert":
        kw.update(source=domain.AlertSource(_SOURCES[m.source]), level=domain.AlertLevel(_LEVELS[m.level]),
                  type=m.type, message=m.alertMessage)
    elif name == "commandInvocation":
        kw.update(initiator=domain.CommandInitiator(_INITIATORS[m.initiator]), initiator_id=m.initiatorId or None,
                  target_id=_opt(m, "targetId"), command_token=m.commandToken or None,
                  parameter_values=dict(m.parameterValues), device_command_id=meta.pop("sw.deviceCommandId", None))
    elif name == "commandResponse":
        kw.update(originating_event_id=_get_uuid(m, "originatingEventId", meta),
                  response_event_id=_get_uuid(m, "responseEventId", meta), response=_opt(m, "response"))
    elif name == "stateChange":
        kw.update(attribute=m.attribute, type=m.type, previous_state=_opt(m, "previousState"),
                  new_state=_opt(m, "newState"))
    kw["metadata"] = meta
    return _EVENT_CLASS[name](**kw)


def encode_persisted(event: domain.DeviceEvent) -> bytes:
    if _MODE == "protobuf":
        p = messages()["GPersistedEventPayload"]()
        meta: dict = {}
        _set_uuid(p, "deviceId", event.device_id, meta)
        _event_message(p.event, event)
        return p.SerializeToString()
    return json.dumps({"event": codec.to_wire(event)}).encode()


def decode_persisted(value) -> domain.DeviceEvent:
    if _is_json(value):
        return codec.from_wire(json.loads(value)["event"])
    return _event_object(messages()["GPersistedEventPayload"].FromString(bytes(value)).event)


def encode_enriched(event: domain.DeviceEvent, context: dict | None, error: str | None = None) -> bytes:
    """Enriched event (+ ``GDeviceEventContext``); ``error`` marks an undelivered command."""
    if _MODE == "protobuf":
        p = messages()["GEnrichedEventPayload"]()
        _event_message(p.event, event)
        if error:
            getattr(p.event, p.event.WhichOneof("event")).event.metadata["sw.error"] = str(error)
        ctx, c = context or {}, p.context
        cmeta: dict = {}
        for f in ("deviceId", "deviceTypeId", "parentDeviceId"):
            _set_uuid(c, f, ctx.get(f), cmeta)
        if ctx.get("deviceStatus") is not None:
            c.deviceStatus.value = str(ctx["deviceStatus"])
        c.deviceMetadata.update({str(k): str(v) for k, v in (ctx.get("deviceMetadata") or {}).items()})
        c.deviceMetadata.update(cmeta)
        c.assignmentStatus = _ASSN.get(str(ctx.get("assignmentStatus") or ""), 0)
        c.assignmentMetadata.update({str(k): str(v) for k, v in (ctx.get("assignmentMetadata") or {}).items()})
        return p.SerializeToString()
    body = {"event": codec.to_wire(event), "context": context}
    if error:
        body["error"] = str(error)
    return json.dumps(body).encode()


def decode_enriched(value, key=None) -> tuple[domain.DeviceEvent, dict, str | None]:
    """-> (event, context, error).  The context's ``deviceToken`` comes from the record key when the
    value does not carry it (protobuf, as in the reference)."""
    token = key.decode() if isinstance(key, (bytes, bytearray)) else key
    if _is_json(value):
        m = json.loads(value)
        ctx = m.get("context") or {}
        if token and not ctx.get("deviceToken"):
            ctx["deviceToken"] = token
        return codec.from_wire(m["event"]), ctx, m.get("error")
    p = messages()["GEnrichedEventPayload"].FromString(bytes(value))
    ev = _event_object(p.event)
    error = ev.metadata.pop("sw.error", None)
    c = p.context
    dmeta = dict(c.deviceMetadata)
    ctx = {"deviceId": _get_uuid(c, "deviceId", dmeta), "deviceTypeId": _get_uuid(c, "deviceTypeId", dmeta),
           "parentDeviceId": _get_uuid(c, "parentDeviceId", dmeta), "deviceStatus": _opt(c, "deviceStatus"),
           "deviceMetadata": dmeta, "assignmentStatus": _ASSN_BACK.get(c.assignmentStatus),
           "assignmentMetadata": dict(c.assignmentMetadata), "deviceToken": token}
    return ev, ctx, error


# ------------------------------------------------------------------------------ instance logging
_LOG_LEVELS = {"TRACE": 0, "DEBUG": 1, "INFO": 2, "WARNING": 3, "WARN": 3, "ERROR": 4, "CRITICAL": 4}
_LOG_BACK = {0: "TRACE", 1: "DEBUG", 2: "INFO", 3: "WARNING", 4: "ERROR"}


def encode_log(m: dict) -> bytes:
    """Log record (``BusLogHandler``) -> ``instance-logging`` value; ``GMicroserviceLogMessage`` in
    protobuf mode (the tenant travels as ``tenantId`` when it is a UUID, otherwise as a
    ``[tenant]`` prefix of the text)."""
    if _MODE != "protobuf":
        return json.dumps(m).encode()
    p = messages()["GMicroserviceLogMessage"](microserviceIdentifier=m.get("microservice") or "",
                                              microserviceContainerId=m.get("hostname") or "",
                                              timestamp=int(m.get("timestamp") or 0),
                                              level=_LOG_LEVELS.get(str(m.get("level", "INFO")).upper(), 2))
    text, tenant = m.get("message") or "", m.get("tenant")
    if tenant:
        meta: dict = {}
        _set_uuid(p, "tenantId", tenant, meta)
        if meta:
            text = f"[{tenant}] {text}"
    p.messageText = text
    exc = m.get("exception")
    if exc:
        p.exception.messageText = exc.get("message", "")
        for fr in exc.get("frames", []):
            p.exception.elements.add(clazz=fr.get("module", ""), method=fr.get("function", ""),
                                     file=fr.get("file", ""), lineNumber=int(fr.get("line") or 0))
    return p.SerializeToString()


def decode_log(value) -> dict:
    if _is_json(value):
        return json.loads(value)
    p = messages()["GMicroserviceLogMessage"].FromString(bytes(value))
    out = {"microservice": p.microserviceIdentifier, "hostname": p.microserviceContainerId,
           "level": _LOG_BACK.get(p.level, "INFO"), "message": p.messageText, "timestamp": p.timestamp,
           "tenant": _get_uuid(p, "tenantId", {})}
    if p.HasField("exception"):
        out["exception"] = {"message": p.exception.messageText, "frames": [
            {"module": e.clazz, "function": e.method, "file": e.file, "line": e.lineNumber}
            for e in p.exception.elements]}
    return out
