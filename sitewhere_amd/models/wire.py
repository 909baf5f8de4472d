"""SiteWhere device wire protocol, built with the protobuf runtime (no protoc needed).

Schema parity with ``sitewhere-communication/src/main/proto/sitewhere.proto``
(proto2): ``Model`` (Metadata, DeviceLocation, DeviceAlert, Measurement,
DeviceMeasurements, DeviceStream, DeviceStreamData), ``SiteWhere`` (Command enum,
Header, RegisterDevice, Acknowledge, DeviceStreamDataRequest) and ``Device``
(Command, Header, RegistrationAck, DeviceStreamAck).  One extension: optional
``alternateId = 15`` on the three event bodies (unknown field to reference parsers).

A payload is ``varint(len(Header)) Header varint(len(Body)) Body`` -- the
``parseDelimitedFrom`` framing used by ``ProtobufDeviceEventDecoder.java:79-281``.
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf.internal import decoder as _pbdec
from google.protobuf.internal import encoder as _pbenc

_F = descriptor_pb2.FieldDescriptorProto
_REQ, _OPT, _REP = _F.LABEL_REQUIRED, _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
_T = {
    "string": _F.TYPE_STRING, "double": _F.TYPE_DOUBLE, "fixed64": _F.TYPE_FIXED64, "bool": _F.TYPE_BOOL,
    "bytes": _F.TYPE_BYTES, "enum": _F.TYPE_ENUM, "msg": _F.TYPE_MESSAGE,
}


def _msg(parent, name, fields, enums=None, nested=None):
    m = parent.add() if hasattr(parent, "add") else parent
    m.name = name
    for en, vals in (enums or {}).items():
        e = m.enum_type.add()
        e.name = en
        for vn, vv in vals:
            v = e.value.add()
            v.name, v.number = vn, vv
    for nm, fn in (nested or []):
        fn(m.nested_type, nm)
    for fname, num, label, typ, tname in fields:
        f = m.field.add()
        f.name, f.number, f.label, f.type = fname, num, label, _T[typ]
        if tname:
            f.type_name = tname
    return m


def _build():
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "sitewhere_amd/sitewhere.proto"
    fd.package = "sitewhere_amd.wire"
    fd.syntax = "proto2"
    P = ".sitewhere_amd.wire."
    meta = P + "Model.Metadata"

    def model(nt, name):
        m = nt.add()
        m.name = name
        _msg(m.nested_type, "Metadata", [("name", 1, _REQ, "string", None), ("value", 2, _REQ, "string", None)])
        _msg(m.nested_type, "DeviceLocation", [
            ("hardwareId", 1, _REQ, "string", None), ("latitude", 2, _REQ, "double", None),
            ("longitude", 3, _REQ, "double", None), ("elevation", 4, _OPT, "double", None),
            ("eventDate", 5, _OPT, "fixed64", None), ("metadata", 6, _REP, "msg", meta),
            ("updateState", 7, _OPT, "bool", None), ("alternateId", 15, _OPT, "string", None)])
        _msg(m.nested_type, "DeviceAlert", [
            ("hardwareId", 1, _REQ, "string", None), ("alertType", 2, _REQ, "string", None),
            ("alertMessage", 3, _REQ, "string", None), ("eventDate", 4, _OPT, "fixed64", None),
            ("metadata", 5, _REP, "msg", meta), ("updateState", 6, _OPT, "bool", None),
            ("alternateId", 15, _OPT, "string", None)])
        _msg(m.nested_type, "Measurement", [
            ("measurementId", 1, _REQ, "string", None), ("measurementValue", 2, _REQ, "double", None)])
        _msg(m.nested_type, "DeviceMeasurements", [
            ("hardwareId", 1, _REQ, "string", None), ("measurement", 2, _REP, "msg", P + "Model.Measurement"),
            ("eventDate", 3, _OPT, "fixed64", None), ("metadata", 4, _REP, "msg", meta),
            ("updateState", 5, _OPT, "bool", None), ("alternateId", 15, _OPT, "string", None)])
        _msg(m.nested_type, "DeviceStream", [
            ("hardwareId", 1, _REQ, "string", None), ("streamId", 2, _REQ, "string", None),
            ("contentType", 3, _REQ, "string", None), ("metadata", 4, _REP, "msg", meta)])
        _msg(m.nested_type, "DeviceStreamData", [
            ("hardwareId", 1, _REQ, "string", None), ("streamId", 2, _REQ, "string", None),
            ("sequenceNumber", 3, _REQ, "fixed64", None), ("data", 4, _REQ, "bytes", None),
            ("eventDate", 5, _OPT, "fixed64", None), ("metadata", 6, _REP, "msg", meta)])

    def sitewhere(nt, name):
        m = nt.add()
        m.name = name
        e = m.enum_type.add()
        e.name = "Command"
        for vn, vv in [("SEND_REGISTRATION", 1), ("SEND_ACKNOWLEDGEMENT", 2), ("SEND_DEVICE_LOCATION", 3),
                       ("SEND_DEVICE_ALERT", 4), ("SEND_DEVICE_MEASUREMENTS", 5), ("SEND_DEVICE_STREAM", 6),
                       ("SEND_DEVICE_STREAM_DATA", 7), ("REQUEST_DEVICE_STREAM_DATA", 8)]:
            v = e.value.add()
            v.name, v.number = vn, vv
        _msg(m.nested_type, "Header", [("command", 1, _REQ, "enum", P + "SiteWhere.Command"),
                                       ("originator", 2, _OPT, "string", None)])
        _msg(m.nested_type, "RegisterDevice", [
            ("hardwareId", 1, _REQ, "string", None), ("deviceTypeToken", 2, _REQ, "string", None),
            ("metadata", 3, _REP, "msg", meta), ("areaToken", 4, _OPT, "string", None)])
        _msg(m.nested_type, "Acknowledge", [("hardwareId", 1, _REQ, "string", None),
                                            ("message", 2, _OPT, "string", None)])
        _msg(m.nested_type, "DeviceStreamDataRequest", [
            ("hardwareId", 1, _REQ, "string", None), ("streamId", 2, _REQ, "string", None),
            ("sequenceNumber", 3, _REQ, "fixed64", None)])

    def device(nt, name):
        m = nt.add()
        m.name = name
        for en, vals in [("Command", [("ACK_REGISTRATION", 1), ("ACK_DEVICE_STREAM", 2),
                                      ("RECEIVE_DEVICE_STREAM_DATA", 3)]),
                         ("RegistrationAckState", [("NEW_REGISTRATION", 1), ("ALREADY_REGISTERED", 2),
                                                   ("REGISTRATION_ERROR", 3)]),
                         ("RegistrationAckError", [("INVALID_SPECIFICATION", 1), ("SITE_TOKEN_REQUIRED", 2),
                                                   ("NEW_DEVICES_NOT_ALLOWED", 3)]),
                         ("DeviceStreamAckState", [("STREAM_CREATED", 1), ("STREAM_EXISTS", 2),
                                                   ("STREAM_FAILED", 3)])]:
            e = m.enum_type.add()
            e.name = en
            for vn, vv in vals:
                v = e.value.add()
                v.name, v.number = vn, vv
        _msg(m.nested_type, "Header", [("command", 1, _REQ, "enum", P + "Device.Command"),
                                       ("originator", 2, _OPT, "string", None),
                                       ("nestedPath", 3, _OPT, "string", None),
                                       ("nestedSpec", 4, _OPT, "string", None)])
        _msg(m.nested_type, "RegistrationAck", [
            ("state", 1, _REQ, "enum", P + "Device.RegistrationAckState"),
            ("errorType", 2, _OPT, "enum", P + "Device.RegistrationAckError"),
            ("errorMessage", 3, _OPT, "string", None)])
        _msg(m.nested_type, "DeviceStreamAck", [("streamId", 1, _REQ, "string", None),
                                                ("state", 2, _REQ, "enum", P + "Device.DeviceStreamAckState")])

    model(fd.message_type, "Model")
    sitewhere(fd.message_type, "SiteWhere")
    device(fd.message_type, "Device")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    classes = {}
    for full in ["Model.Metadata", "Model.DeviceLocation", "Model.DeviceAlert", "Model.Measurement",
                 "Model.DeviceMeasurements", "Model.DeviceStream", "Model.DeviceStreamData", "SiteWhere.Header",
                 "SiteWhere.RegisterDevice", "SiteWhere.Acknowledge", "SiteWhere.DeviceStreamDataRequest",
                 "Device.Header", "Device.RegistrationAck", "Device.DeviceStreamAck"]:
        desc = pool.FindMessageTypeByName("sitewhere_amd.wire." + full)
        classes[full] = message_factory.GetMessageClass(desc)
    return classes


M = _build()
Metadata = M["Model.Metadata"]
DeviceLocation = M["Model.DeviceLocation"]
DeviceAlert = M["Model.DeviceAlert"]
Measurement = M["Model.Measurement"]
DeviceMeasurements = M["Model.DeviceMeasurements"]
DeviceStream = M["Model.DeviceStream"]
DeviceStreamData = M["Model.DeviceStreamData"]
Header = M["SiteWhere.Header"]
RegisterDevice = M["SiteWhere.RegisterDevice"]
Acknowledge = M["SiteWhere.Acknowledge"]
DeviceStreamDataRequest = M["SiteWhere.DeviceStreamDataRequest"]
DeviceHeader = M["Device.Header"]
RegistrationAck = M["Device.RegistrationAck"]
DeviceStreamAck = M["Device.DeviceStreamAck"]

SEND_REGISTRATION, SEND_ACKNOWLEDGEMENT, SEND_DEVICE_LOCATION, SEND_DEVICE_ALERT = 1, 2, 3, 4
SEND_DEVICE_MEASUREMENTS, SEND_DEVICE_STREAM, SEND_DEVICE_STREAM_DATA, REQUEST_DEVICE_STREAM_DATA = 5, 6, 7, 8
ACK_REGISTRATION, ACK_DEVICE_STREAM, RECEIVE_DEVICE_STREAM_DATA = 1, 2, 3

_BODY = {
    SEND_REGISTRATION: RegisterDevice, SEND_ACKNOWLEDGEMENT: Acknowledge, SEND_DEVICE_LOCATION: DeviceLocation,
    SEND_DEVICE_ALERT: DeviceAlert, SEND_DEVICE_MEASUREMENTS: DeviceMeasurements, SEND_DEVICE_STREAM: DeviceStream,
    SEND_DEVICE_STREAM_DATA: DeviceStreamData, REQUEST_DEVICE_STREAM_DATA: DeviceStreamDataRequest,
}


def delimited(msg) -> bytes:
    body = msg.SerializeToString()
    return _pbenc._VarintBytes(len(body)) + body


def read_delimited(buf: bytes, pos: int, cls):
    n, pos = _pbdec._DecodeVarint(buf, pos)
    m = cls()
    m.ParseFromString(buf[pos:pos + n])
    return m, pos + n


def iter_fields(buf: bytes):
    """Raw protobuf fields of ``buf``: (field number, wire type, value) with value = int (varint),
    bytes (length-delimited, fixed64, fixed32).  Stops at the first malformed field."""
    p, n = 0, len(buf)
    while p < n:
        try:
            key, p = _pbdec._DecodeVarint(buf, p)
        except Exception:  # noqa: BLE001
            return
        f, wt = key >> 3, key & 7
        if wt == 0:
            try:
                v, p = _pbdec._DecodeVarint(buf, p)
            except Exception:  # noqa: BLE001
                return
        elif wt == 2:
            try:
                ln, p = _pbdec._DecodeVarint(buf, p)
            except Exception:  # noqa: BLE001
                return
            if p + ln > n:
                return
            v, p = bytes(buf[p:p + ln]), p + ln
        elif wt == 1 or wt == 5:
            w = 8 if wt == 1 else 4
            if p + w > n:
                return
            v, p = bytes(buf[p:p + w]), p + w
        else:
            return
        yield f, wt, v


def encode(command: int, body, originator: str | None = None) -> bytes:
    h = Header(command=command)
    if originator is not None:
        h.originator = originator
    return delimited(h) + delimited(body)


def decode(payload: bytes):
    """Decode one payload -> (command, originator or None, body message)."""
    h, pos = read_delimited(payload, 0, Header)
    cls = _BODY.get(h.command)
    if cls is None or not h.IsInitialized():
        raise ValueError(f"unknown command {h.command if h.HasField('command') else None}")
    body, _ = read_delimited(payload, pos, cls)
    if not body.IsInitialized():
        # protobuf-java's parseDelimitedFrom refuses a message missing a `required` field
        # (ProtobufDeviceEventDecoder.java:79-95); the python runtime parses it, so check here
        raise ValueError(f"{cls.DESCRIPTOR.name} misses required fields: {body.FindInitializationErrors()}")
    return h.command, (h.originator if h.HasField("originator") else None), body


def encode_device_command(command: int, body, originator: str | None = None, nested_path: str | None = None,
                          nested_spec: str | None = None) -> bytes:
    """Downlink (system -> device) framing: Device.Header + body (reference ProtobufEncoder)."""
    h = DeviceHeader(command=command)
    if originator is not None:
        h.originator = originator
    if nested_path is not None:
        h.nestedPath = nested_path
    if nested_spec is not None:
        h.nestedSpec = nested_spec
    return delimited(h) + delimited(body)


def decode_device_command(payload: bytes):
    """Device-side decode of a system downlink -> (command, nested path or None, body message)."""
    h, pos = read_delimited(payload, 0, DeviceHeader)
    cls = {ACK_REGISTRATION: RegistrationAck, ACK_DEVICE_STREAM: DeviceStreamAck,
           RECEIVE_DEVICE_STREAM_DATA: DeviceStreamData}.get(h.command)
    if cls is None:
        raise ValueError(f"unknown downlink command {h.command}")
    body, _ = read_delimited(payload, pos, cls)
    return h.command, (h.nestedPath if h.HasField("nestedPath") else None), body


# convenience builders -----------------------------------------------------------
def measurements(hardware_id: str, values: dict, event_date: int | None = None, alternate_id: str | None = None,
                 metadata: dict | None = None, update_state: bool | None = None, originator: str | None = None) -> bytes:
    b = DeviceMeasurements(hardwareId=hardware_id)
    for k, v in values.items():
        b.measurement.add(measurementId=k, measurementValue=float(v))
    if event_date is not None:
        b.eventDate = int(event_date)
    if alternate_id is not None:
        b.alternateId = alternate_id
    for k, v in (metadata or {}).items():
        b.metadata.add(name=k, value=v)
    if update_state is not None:
        b.updateState = update_state
    return encode(SEND_DEVICE_MEASUREMENTS, b, originator)


def location(hardware_id: str, lat: float, lon: float, elevation: float | None = None, event_date: int | None = None,
             alternate_id: str | None = None, originator: str | None = None, metadata: dict | None = None,
             update_state: bool | None = None) -> bytes:
    b = DeviceLocation(hardwareId=hardware_id, latitude=lat, longitude=lon)
    if elevation is not None:
        b.elevation = elevation
    if event_date is not None:
        b.eventDate = int(event_date)
    for k, v in (metadata or {}).items():
        b.metadata.add(name=k, value=v)
    if update_state is not None:
        b.updateState = update_state
    if alternate_id is not None:
        b.alternateId = alternate_id
    return encode(SEND_DEVICE_LOCATION, b, originator)


def alert(hardware_id: str, alert_type: str, message: str, event_date: int | None = None,
          alternate_id: str | None = None, originator: str | None = None, metadata: dict | None = None,
          update_state: bool | None = None) -> bytes:
    b = DeviceAlert(hardwareId=hardware_id, alertType=alert_type, alertMessage=message)
    if event_date is not None:
        b.eventDate = int(event_date)
    for k, v in (metadata or {}).items():
        b.metadata.add(name=k, value=v)
    if update_state is not None:
        b.updateState = update_state
    if alternate_id is not None:
        b.alternateId = alternate_id
    return encode(SEND_DEVICE_ALERT, b, originator)


def registration(hardware_id: str, device_type_token: str, area_token: str | None = None,
                 metadata: dict | None = None, originator: str | None = None) -> bytes:
    b = RegisterDevice(hardwareId=hardware_id, deviceTypeToken=device_type_token)
    if area_token is not None:
        b.areaToken = area_token
    for k, v in (metadata or {}).items():
        b.metadata.add(name=k, value=v)
    return encode(SEND_REGISTRATION, b, originator)


def acknowledge(hardware_id: str, message: str | None = None, originator: str | None = None) -> bytes:
    b = Acknowledge(hardwareId=hardware_id)
    if message is not None:
        b.message = message
    return encode(SEND_ACKNOWLEDGEMENT, b, originator)


def stream_create(hardware_id: str, stream_id: str, content_type: str = "application/octet-stream",
                  originator: str | None = None) -> bytes:
    return encode(SEND_DEVICE_STREAM, DeviceStream(hardwareId=hardware_id, streamId=stream_id,
                                                   contentType=content_type), originator)


def stream_data(hardware_id: str, stream_id: str, sequence_number: int, data: bytes,
                event_date: int | None = None, originator: str | None = None) -> bytes:
    b = DeviceStreamData(hardwareId=hardware_id, streamId=stream_id, sequenceNumber=sequence_number, data=data)
    if event_date is not None:
        b.eventDate = event_date
    return encode(SEND_DEVICE_STREAM_DATA, b, originator)


def stream_data_request(hardware_id: str, stream_id: str, sequence_number: int,
                        originator: str | None = None) -> bytes:
    return encode(REQUEST_DEVICE_STREAM_DATA, DeviceStreamDataRequest(hardwareId=hardware_id, streamId=stream_id,
                                                                      sequenceNumber=sequence_number), originator)
