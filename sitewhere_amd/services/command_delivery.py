"""service-command-delivery: command invocation -> target -> encoding -> routing -> delivery.

Reference: ``EnrichedCommandInvocationsConsumer.java:53-171`` (5-thread pool),
``DefaultCommandProcessingStrategy.java:61-85`` (command lookup -> ``DefaultCommandExecutionBuilder``
-> ``DefaultCommandTargetResolver`` -> ``NestedDeviceSupport`` -> routing), ``CommandRoutingLogic.java:38-63``
(router -> ``CommandDestination`` = encoder + parameter extractor + delivery provider), encoders
(protobuf / JSON / Groovy), providers (MQTT QoS 1 ``MqttCommandDeliveryProvider.java:87-111``, CoAP,
Twilio SMS), routers (single-choice, device-type mapping, Groovy, no-op); failures go to the
``undelivered-command-invocations`` topic.
"""
from __future__ import annotations

import base64
import json
import threading

from ..core.errors import SiteWhereException
from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from ..edges.mqtt import MQTT_OPTIONS, client_from_config, parse_qos
from ..models import wire
from ..models.domain import ParameterType
from ..runtime.consumers import BusConsumer
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads

_CONVERT = {
    ParameterType.Double: float, ParameterType.Float: float, ParameterType.Bool: lambda v: str(v).lower() in ("1", "true"),
    ParameterType.String: str, ParameterType.Bytes: lambda v: v if isinstance(v, bytes) else str(v).encode(),
}


def convert_parameter(ptype: ParameterType, value):
    if value is None:
        return None
    return _CONVERT.get(ptype, int)(value)


class CommandExecution(dict):
    """{command, invocation, parameters(typed), nesting}."""


def build_execution(command, invocation) -> CommandExecution:
    """DefaultCommandExecutionBuilder: typed parameters, required-parameter check."""
    params = {}
    for p in command.parameters:
        raw = invocation.parameter_values.get(p.name)
        if raw is None:
            if p.required:
                raise SiteWhereException(f"required parameter {p.name!r} missing for command {command.name}")
            continue
        params[p.name] = convert_parameter(p.type, raw)
    return CommandExecution(command={"name": command.name, "namespace": command.namespace, "token": command.token},
                            invocation={"id": invocation.id, "initiator": invocation.initiator.value
                                        if hasattr(invocation.initiator, "value") else invocation.initiator},
                            parameters=params)


def nesting_of(dm, device) -> dict:
    """NestedDeviceSupport: deliver to the top-level gateway with the path of the nested device."""
    path, cur = [], device
    seen = set()
    while cur.parent_device_id and cur.parent_device_id not in seen:
        seen.add(cur.id)
        parent = dm.get_device(cur.parent_device_id)
        if parent is None:
            break
        maps = [m for m in parent.device_element_mappings if m.device_token == cur.token]
        path.insert(0, maps[0].device_element_schema_path if maps else cur.token)
        cur = parent
    return {"gateway": cur, "nested": device if cur.id != device.id else None, "path": "/".join(path) or None}


# ------------------------------------------------------------------------------ encoders
class JsonEncoder:
    def encode(self, execution, nesting, assignment) -> bytes:
        return json.dumps({"command": execution["command"], "parameters": _jsonable(execution["parameters"]),
                           "invocationId": execution["invocation"]["id"], "nestedPath": nesting.get("path"),
                           "assignmentId": assignment.id if assignment else None}).encode()

    def encode_system(self, command: dict, nesting) -> bytes:
        cmd = {k: ({"base64": base64.b64encode(v).decode()} if isinstance(v, bytes) else v) for k, v in command.items()}
        return json.dumps({"systemCommand": cmd, "nestedPath": nesting.get("path")}).encode()


class ProtobufEncoder:
    """System commands use the reference's typed downlink messages (``Device.Header`` + e.g.
    ``RegistrationAck``).  Custom commands are framed as three delimited ``Model.Metadata`` messages
    (command name, JSON parameters, nested path) -- the reference instead generated a protobuf schema
    per device type (``ProtobufSpecificationBuilder``)."""

    def encode(self, execution, nesting, assignment) -> bytes:
        return (wire.delimited(wire.Metadata(name="command", value=execution["command"]["name"])) +
                wire.delimited(wire.Metadata(name="parameters", value=json.dumps(_jsonable(execution["parameters"])))) +
                wire.delimited(wire.Metadata(name="nestedPath", value=nesting.get("path") or "")))

    def encode_system(self, command: dict, nesting) -> bytes:
        if command.get("type") == "RegistrationAck":
            st = {"NEW_REGISTRATION": 1, "ALREADY_REGISTERED": 2, "REGISTRATION_ERROR": 3}[command["state"]]
            ack = wire.RegistrationAck(state=st)
            if command.get("errorType"):
                ack.errorType = {"INVALID_SPECIFICATION": 1, "SITE_TOKEN_REQUIRED": 2,
                                 "NEW_DEVICES_NOT_ALLOWED": 3}[command["errorType"]]
            return wire.encode_device_command(wire.ACK_REGISTRATION, ack, nested_path=nesting.get("path"))
        if command.get("type") == "DeviceStreamAck":
            st = {"STREAM_CREATED": 1, "STREAM_EXISTS": 2, "STREAM_FAILED": 3}[command["state"]]
            return wire.encode_device_command(wire.ACK_DEVICE_STREAM,
                                              wire.DeviceStreamAck(streamId=command["streamId"], state=st),
                                              nested_path=nesting.get("path"))
        if command.get("type") == "DeviceStreamData":
            # reference Device.proto RECEIVE_DEVICE_STREAM_DATA carries the Model.DeviceStreamData chunk
            body = wire.DeviceStreamData(hardwareId=nesting["gateway"].token, streamId=command["streamId"],
                                         sequenceNumber=command["sequenceNumber"], data=command.get("data") or b"")
            return wire.encode_device_command(wire.RECEIVE_DEVICE_STREAM_DATA, body, nested_path=nesting.get("path"))
        return JsonEncoder().encode_system(command, nesting)


class ScriptEncoder:
    def __init__(self, runner, source):
        self.runner, self.source = runner, source

    def encode(self, execution, nesting, assignment) -> bytes:
        out = self.runner.call(self.source, "encode", dict(execution), {"path": nesting.get("path")},
                               assignment.to_dict() if assignment else None, name="command-encoder")
        return out if isinstance(out, bytes) else str(out).encode()

    def encode_system(self, command, nesting) -> bytes:
        return JsonEncoder().encode_system(command, nesting)


def _jsonable(d):
    return {k: (v.decode("latin-1") if isinstance(v, bytes) else v) for k, v in d.items()}


# ------------------------------------------------------------------------------ providers
class LogProvider:
    def __init__(self):
        self.delivered = []

    def deliver(self, nesting, assignment, payload: bytes, params: dict):
        self.delivered.append((nesting["gateway"].token, params, payload))


class MqttProvider:
    """MQTT publish of encoded commands (reference ``MqttCommandDeliveryProvider.java:87-111``, QoS 1
    by default); ``mqtt``: the ``MqttLifecycleComponent`` attributes (TLS, credentials, client id)."""

    def __init__(self, host, port, qos=1, **mqtt):
        self.host, self.port, self.qos = host, port, parse_qos(qos)
        self.mqtt = {k: v for k, v in mqtt.items() if v is not None}
        self.client = None
        self._lock = threading.Lock()

    def deliver(self, nesting, assignment, payload, params):
        with self._lock:
            if self.client is None:
                self.client = client_from_config(dict(self.mqtt, host=self.host, port=self.port),
                                                 reconnect=True).connect()
        self.client.publish(params["topic"], payload, qos=self.qos)


class CoapProvider:
    """CoAP request to the device (reference ``CoapCommandDeliveryProvider`` with
    ``MetadataCoapParameterExtractor``: host, port, resource path and method from device metadata)."""

    _METHODS = {"POST": 2, "PUT": 3}

    def deliver(self, nesting, assignment, payload, params):
        host, port = params.get("hostname"), params.get("port")
        if not host:
            raise SiteWhereException("Hostname not found in device metadata. Unable to deliver command.")
        method = self._METHODS.get(str(params.get("method") or "POST").upper())
        if method is None:
            raise SiteWhereException(f"unsupported CoAP delivery method {params.get('method')!r}")
        from ..edges.receivers import coap_request
        r = coap_request(host, int(port or 5683), params.get("path") or "commands", payload, method)
        if r is None or (r["code"] >> 5) != 2:
            raise SiteWhereException("CoAP delivery not acknowledged" if r is None else
                                     f"CoAP delivery refused: {r['code'] >> 5}.{r['code'] & 31:02d}")


class SmsProvider:
    """Twilio SMS over its REST API (reference ``twilio/TwilioCommandDeliveryProvider``: the encoded
    command is the message body, sent ``From`` the configured number ``To`` the number in the
    gateway's metadata).  ``POST {api}/2010-04-01/Accounts/{sid}/Messages.json`` with HTTP basic
    auth -- no Twilio SDK needed.  System commands are not delivered by SMS (as in the reference)."""

    def __init__(self, account_sid: str | None, auth_token: str | None, from_phone: str | None,
                 api_base: str = "https://api.twilio.com", timeout: float = 10.0):
        if not account_sid:
            raise SiteWhereException("Twilio command delivery provider missing account SID.")
        if not auth_token:
            raise SiteWhereException("Twilio command delivery provider missing auth token.")
        self.sid, self.from_phone, self.api, self.timeout = account_sid, from_phone, api_base.rstrip("/"), timeout
        self._auth = "Basic " + base64.b64encode(f"{account_sid}:{auth_token}".encode()).decode()
        self.sent: list = []

    def deliver(self, nesting, assignment, payload, params):
        import urllib.error
        import urllib.parse
        import urllib.request
        to = params.get("phone")
        if not to:
            raise SiteWhereException("No phone number found in device metadata. Unable to deliver.")
        body = payload.decode() if isinstance(payload, (bytes, bytearray)) else str(payload)
        req = urllib.request.Request(f"{self.api}/2010-04-01/Accounts/{urllib.parse.quote(self.sid)}/Messages.json",
                                     data=urllib.parse.urlencode({"To": to, "From": self.from_phone or "",
                                                                  "Body": body}).encode(),
                                     headers={"Authorization": self._auth,
                                              "Content-Type": "application/x-www-form-urlencoded"}, method="POST")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                res = json.loads(r.read() or b"{}")
        except urllib.error.HTTPError as e:
            try:
                msg = json.loads(e.read()).get("message", "")
            except ValueError:
                msg = ""
            raise SiteWhereException(f"Unable to send Twilio SMS message: HTTP {e.code} {msg}".strip()) from e
        except OSError as e:
            raise SiteWhereException(f"Unable to send Twilio SMS message: {e}") from e
        self.sent.append(res.get("sid"))
        return res

    def deliver_system(self, nesting, assignment, payload, params):
        raise SiteWhereException("system commands are not delivered by SMS")


def mqtt_extractor(tenant: str, command_topic: str, system_topic: str):
    def extract(nesting, assignment, system: bool = False):
        tpl = system_topic if system else command_topic
        return {"topic": tpl.format(tenant=tenant, deviceToken=nesting["gateway"].token)}
    return extract


def metadata_extractor(keys: dict):
    """Read delivery parameters from device metadata (CoAP host/port, SMS number)."""
    def extract(nesting, assignment, system: bool = False):
        md = nesting["gateway"].metadata or {}
        return {k: md.get(src) for k, src in keys.items()}
    return extract


class CommandDestination(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.CommandDestination

    def __init__(self, did, encoder, extractor, provider):
        super().__init__(f"destination:{did}")
        self.did, self.encoder, self.extractor, self.provider = did, encoder, extractor, provider
        self.delivered = 0

    def deliver_command(self, execution, nesting, assignment):
        payload = self.encoder.encode(execution, nesting, assignment)
        self.provider.deliver(nesting, assignment, payload, self.extractor(nesting, assignment))
        self.delivered += 1

    def deliver_system_command(self, command, nesting, assignment):
        payload = self.encoder.encode_system(command, nesting)
        deliver = getattr(self.provider, "deliver_system", self.provider.deliver)
        deliver(nesting, assignment, payload, self.extractor(nesting, assignment, True))
        self.delivered += 1


# ------------------------------------------------------------------------------ routers
class SingleChoiceRouter:
    def __init__(self, destination):
        self.destination = destination

    def route(self, execution, nesting, assignment, device_type_token):
        return [self.destination]


class DeviceTypeMappingRouter:
    def __init__(self, mapping: dict, default=None):
        self.mapping, self.default = mapping, default

    def route(self, execution, nesting, assignment, device_type_token):
        d = self.mapping.get(device_type_token, self.default)
        return [d] if d else []


class ScriptRouter:
    def __init__(self, runner, source):
        self.runner, self.source = runner, source

    def route(self, execution, nesting, assignment, device_type_token):
        r = self.runner.call(self.source, "route", dict(execution), nesting["gateway"].token,
                             assignment.id if assignment else None, name="command-router")
        return [r] if isinstance(r, str) else list(r or [])


class NoOpRouter:
    def route(self, *a):
        return []


class CommandDeliveryTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        t = self.tenant.token
        self.destinations: dict[str, CommandDestination] = {}
        for dc in self.config.get("destinations", []):
            d = self.build_destination(dc)
            d.tenant_engine = self
            self.initialize_nested_component(d, monitor, require=False)
            self.destinations[d.did] = d
        rc = self.config.get("router", {"type": "single-choice", "destination": "default"})
        rt = rc.get("type")
        if rt == "single-choice":
            self.router = SingleChoiceRouter(rc.get("destination") or next(iter(self.destinations), None))
        elif rt == "device-type-mapping":
            self.router = DeviceTypeMappingRouter(rc.get("mappings", {}), rc.get("default"))
        elif rt == "script":
            self.router = ScriptRouter(self.ms.scripts, self.script_source(rc["script"]))
        else:
            self.router = NoOpRouter()
        n = self.ms.instance.naming
        self.t_undelivered = n.undelivered_command_invocations(t)
        self.consumer = BusConsumer(self, "enriched-command-invocations", [n.enriched_command_invocations(t)],
                                    self._process, threads=int(self.config.get("processingThreads", 5)))
        self.undelivered = 0
        self.api = {"CommandDelivery": CommandDeliveryApi(self)}

    def build_destination(self, dc) -> CommandDestination:
        enc = {"json": JsonEncoder, "protobuf": ProtobufEncoder}.get(dc.get("encoder", "json"))
        encoder = enc() if enc else ScriptEncoder(self.ms.scripts, self.script_source(dc["encoderScript"]))
        p = dc.get("provider", "log")
        if p == "mqtt":
            provider = MqttProvider(dc.get("hostname") or dc.get("host", "127.0.0.1"), int(dc.get("port", 1883)),
                                    dc.get("qos", 1), **{k: dc.get(k) for k in MQTT_OPTIONS})
            extractor = mqtt_extractor(self.tenant.token, dc.get("commandTopic", "SiteWhere/{tenant}/command/{deviceToken}"),
                                       dc.get("systemTopic", "SiteWhere/{tenant}/system/{deviceToken}"))
        elif p == "coap":
            provider = CoapProvider()       # metadata field names: MetadataCoapParameterExtractor defaults
            extractor = metadata_extractor({"hostname": dc.get("hostnameMetadata", "coap_hostname"),
                                            "port": dc.get("portMetadata", "coap_port"),
                                            "path": dc.get("urlMetadata", "coap_url"),
                                            "method": dc.get("methodMetadata", "coap_method")})
        elif p == "sms":
            provider = SmsProvider(dc.get("accountSid"), dc.get("authToken"), dc.get("fromPhone"),
                                   dc.get("apiBase", "https://api.twilio.com"))
            extractor = metadata_extractor({"phone": dc.get("phoneMetadata", "sms_phone")})
        else:
            provider = LogProvider()
            extractor = lambda nesting, a, system=False: {}  # noqa: E731
        return CommandDestination(dc["id"], encoder, extractor, provider)

    def _dm(self):
        return self.ms.api("DeviceManagement", self.tenant.token)

    def _process(self, recs):
        for r in recs:
            ev, ctx, _ = payloads.decode_enriched(r.value, r.key)
            try:
                self.deliver_command(ev)
            except Exception as e:  # noqa: BLE001
                self.undelivered += 1
                self.ms.producer.send(self.t_undelivered, ev.device_id, payloads.encode_enriched(ev, ctx, str(e)))

    def deliver_command(self, invocation) -> int:
        dm = self._dm()
        cmd = dm.get_device_command(invocation.device_command_id) if invocation.device_command_id else \
            dm.get_device_command_by_token(invocation.command_token)
        if cmd is None:
            raise SiteWhereException(f"unknown command {invocation.command_token or invocation.device_command_id}")
        execution = build_execution(cmd, invocation)
        assignment = dm.get_device_assignment(invocation.device_assignment_id)
        device = dm.get_device(assignment.device_id)
        nesting = nesting_of(dm, device)
        dtype = dm.get_device_type(device.device_type_id)
        dests = self.router.route(execution, nesting, assignment, dtype.token if dtype else None)
        if not dests:
            raise SiteWhereException("no command destination")
        for did in dests:
            d = self.destinations.get(did)
            if d is None:
                raise SiteWhereException(f"unknown destination {did}")
            d.deliver_command(execution, nesting, assignment)
        return len(dests)

    def deliver_system_command(self, device_token: str, command: dict) -> int:
        dm = self._dm()
        device = dm.get_device_by_token(device_token)
        if device is None:
            raise SiteWhereException(f"unknown device {device_token}")
        nesting = nesting_of(dm, device)
        assignment = dm.get_device_assignment(device.device_assignment_id) if device.device_assignment_id else None
        dtype = dm.get_device_type(device.device_type_id)
        n = 0
        for did in self.router.route({"system": command}, nesting, assignment, dtype.token if dtype else None):
            self.destinations[did].deliver_system_command(command, nesting, assignment)
            n += 1
        return n

    def tenant_start(self, monitor):
        for d in self.destinations.values():
            self.start_nested_component(d, monitor, require=False)
        self.start_nested_component(self.consumer, monitor, require=True)

    def tenant_stop(self, monitor):
        self.consumer.lifecycle_stop(monitor)


class CommandDeliveryApi:
    def __init__(self, e):
        self._e = e

    def deliver_system_command(self, device_token: str, command: dict) -> int:
        return self._e.deliver_system_command(device_token, command)

    def list_destinations(self) -> list[dict]:
        return [{"id": d.did, "status": d.status.value, "delivered": d.delivered} for d in self._e.destinations.values()]

    def get_statistics(self) -> dict:
        return {"undelivered": self._e.undelivered,
                "delivered": sum(d.delivered for d in self._e.destinations.values())}


class CommandDeliveryMicroservice(MultitenantMicroservice):
    identifier = "command-delivery"
    name = "Command Delivery"

    def service_names(self):
        return ["CommandDelivery"]

    def create_tenant_engine(self, tenant):
        return CommandDeliveryTenantEngine(self, tenant)
