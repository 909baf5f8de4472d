"""service-event-sources: protocol receivers -> decoders -> dedup -> decoded-events topic (multitenant).

Reference: ``service-event-sources`` --
  * ``InboundEventSource.java:40-283``: one decoder, optional deduplicator, N receivers;
    ``onEncodedEventReceived`` -> decode -> meter -> dedup -> ``EventSourcesManager.handleDecodedEvent``
  * ``EventSourcesManager.java:153-197``: event requests -> decoded-events topic keyed by device token,
    registrations -> registration topic, decode failures -> failed-decode topic
  * decoders: protobuf (``ProtobufDeviceEventDecoder.java:79-281``), JSON ``DeviceRequest``
    (``JsonDeviceRequestMarshaler.java:62-148``), JSON batch, scripted (Groovy -> Python), composite
    (per-device-type choice with a metadata extractor), echo / payload logger (debug)
  * deduplicators: ``AlternateIdDeduplicator``, scripted
  * receivers: MQTT, CoAP, socket, WebSocket, REST polling, ActiveMQ/RabbitMQ/EventHub (see
    :mod:`sitewhere_amd.edges`); plus an in-process ``direct`` receiver for embedding and tests.
The MI355X path: a source configured with ``"forward": "raw"`` skips per-message decoding and ships
raw payload batches to ``event-source-raw-payloads`` for the GPU inbound engine.
"""
from __future__ import annotations

import json
import threading
import time

from ..core.errors import EventDecodeException
from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from ..models import wire
from ..rpc import codec
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads

RAW_PAYLOADS = "event-source-raw-payloads"

REQUEST_TYPES = ("DeviceMeasurement", "DeviceLocation", "DeviceAlert", "DeviceCommandResponse", "DeviceStateChange",
                 "RegisterDevice", "Acknowledge", "DeviceStream", "DeviceStreamData", "SendDeviceStreamData")


def decoded(token: str, type_: str, request: dict, originator: str | None = None) -> dict:
    return {"deviceToken": token, "type": type_, "request": request, "originator": originator}


# ------------------------------------------------------------------------------ decoders
class Decoder:
    def decode(self, payload: bytes, metadata: dict) -> list[dict]:
        raise NotImplementedError


class ProtobufDecoder(Decoder):
    """SiteWhere device protocol (delimited Header + body)."""

    def decode(self, payload, metadata):
        try:
            cmd, orig, b = wire.decode(bytes(payload))
        except Exception as e:
            raise EventDecodeException(f"protobuf decode failed: {e}") from e
        md = {m.name: m.value for m in getattr(b, "metadata", [])}
        base = {"metadata": md}
        if hasattr(b, "HasField") and "updateState" in b.DESCRIPTOR.fields_by_name and b.HasField("updateState"):
            base["updateState"] = b.updateState
        if "eventDate" in b.DESCRIPTOR.fields_by_name and b.HasField("eventDate"):
            base["eventDate"] = b.eventDate
        if "alternateId" in b.DESCRIPTOR.fields_by_name and b.HasField("alternateId"):
            base["alternateId"] = b.alternateId
        if cmd == wire.SEND_DEVICE_MEASUREMENTS:
            out = []
            for i, m in enumerate(b.measurement):
                r = dict(base, name=m.measurementId, value=m.measurementValue)
                if "alternateId" in base:
                    r["alternateId"] = f"{base['alternateId']}:{i}" if len(b.measurement) > 1 else base["alternateId"]
                out.append(decoded(b.hardwareId, "DeviceMeasurement", r, orig))
            return out
        if cmd == wire.SEND_DEVICE_LOCATION:
            r = dict(base, latitude=b.latitude, longitude=b.longitude)
            if b.HasField("elevation"):
                r["elevation"] = b.elevation
            return [decoded(b.hardwareId, "DeviceLocation", r, orig)]
        if cmd == wire.SEND_DEVICE_ALERT:
            return [decoded(b.hardwareId, "DeviceAlert", dict(base, type=b.alertType, message=b.alertMessage,
                                                               level="Info"), orig)]
        if cmd == wire.SEND_REGISTRATION:
            r = {"deviceTypeToken": b.deviceTypeToken, "metadata": md}
            if b.HasField("areaToken"):
                r["areaToken"] = b.areaToken
            return [decoded(b.hardwareId, "RegisterDevice", r, orig)]
        if cmd == wire.SEND_ACKNOWLEDGEMENT:
            return [decoded(b.hardwareId, "Acknowledge", {"originatingEventId": orig, "response": b.message}, orig)]
        if cmd == wire.SEND_DEVICE_STREAM:
            return [decoded(b.hardwareId, "DeviceStream", {"streamId": b.streamId, "contentType": b.contentType,
                                                            "metadata": md}, orig)]
        if cmd == wire.SEND_DEVICE_STREAM_DATA:
            return [decoded(b.hardwareId, "DeviceStreamData", {"streamId": b.streamId, "sequenceNumber": b.sequenceNumber,
                                                                "data": b.data, "eventDate": base.get("eventDate")}, orig)]
        if cmd == wire.REQUEST_DEVICE_STREAM_DATA:
            return [decoded(b.hardwareId, "SendDeviceStreamData", {"streamId": b.streamId,
                                                                    "sequenceNumber": b.sequenceNumber}, orig)]
        raise EventDecodeException(f"unsupported command {cmd}")


class JsonDeviceRequestDecoder(Decoder):
    """``{"deviceToken", "originator", "type", "request"}`` (reference JsonDeviceRequestMarshaler)."""

    def decode(self, payload, metadata):
        try:
            d = json.loads(payload)
        except Exception as e:
            raise EventDecodeException(f"invalid JSON: {e}") from e
        return [self._one(d)]

    @staticmethod
    def _one(d: dict) -> dict:
        t = d.get("type")
        if t not in REQUEST_TYPES:
            raise EventDecodeException(f"unknown request type {t!r}")
        if not d.get("deviceToken"):
            raise EventDecodeException("deviceToken missing")
        if d.get("request") is None:
            raise EventDecodeException("request missing")
        return decoded(d["deviceToken"], t, d["request"], d.get("originator"))


class JsonBatchDecoder(Decoder):
    """``{"deviceToken", "measurements": [...], "locations": [...], "alerts": [...]}`` (DeviceEventBatch)."""

    def decode(self, payload, metadata):
        try:
            d = json.loads(payload)
        except Exception as e:
            raise EventDecodeException(f"invalid JSON: {e}") from e
        tok = d.get("hardwareId") or d.get("deviceToken")
        if not tok:
            raise EventDecodeException("deviceToken missing")
        out = [decoded(tok, "DeviceMeasurement", m) for m in d.get("measurements", [])]
        out += [decoded(tok, "DeviceLocation", m) for m in d.get("locations", [])]
        out += [decoded(tok, "DeviceAlert", m) for m in d.get("alerts", [])]
        return out


class CoapJsonDecoder(Decoder):
    """Body of a CoAP request routed by the receiver's path (reference
    ``decoder/coap/CoapJsonDecoder.java``): ``eventType`` / ``token`` come from the receiver's
    metadata, the JSON body is the request itself."""

    def decode(self, payload, metadata):
        t, tok = metadata.get("eventType"), metadata.get("token")
        if t not in REQUEST_TYPES or not tok:
            raise EventDecodeException(f"CoAP payload without a routed event type/token ({t!r}, {tok!r})")
        try:
            req = json.loads(payload) if payload else {}
        except Exception as e:
            raise EventDecodeException(f"invalid JSON: {e}") from e
        if not isinstance(req, dict):
            raise EventDecodeException("CoAP request body must be a JSON object")
        return [decoded(tok, t, req)]


class ScriptedDecoder(Decoder):
    """User script ``decode(payload, metadata) -> list[dict]`` (reference Groovy decoders)."""

    def __init__(self, runner, source: str, name: str = "decoder"):
        self.runner, self.source, self.name = runner, source, name

    def decode(self, payload, metadata):
        try:
            res = self.runner.call(self.source, "decode", payload, metadata, name=self.name)
        except Exception as e:
            raise EventDecodeException(f"script decoder failed: {e}") from e
        return [JsonDeviceRequestDecoder._one(r) for r in (res or [])]


class CompositeDecoder(Decoder):
    """Metadata extractor picks the device token, then a decoder chosen by device type
    (reference ``decoder/composite/*``)."""

    def __init__(self, extractor, choices: dict, device_type_of, default: Decoder | None = None):
        self.extractor, self.choices, self.device_type_of, self.default = extractor, choices, device_type_of, default

    def decode(self, payload, metadata):
        try:
            token, inner = self.extractor(payload, metadata)
        except Exception as e:
            raise EventDecodeException(f"composite decoder metadata extraction failed: {e}") from e
        dt = self.device_type_of(token)
        dec = self.choices.get(dt, self.default)
        if dec is None:         # reference: no choice applies -> nothing decoded
            return []
        # the chosen decoder sees the device context too (CompositeDeviceEventDecoder META_DEVICE*)
        out = dec.decode(inner, dict(metadata or {}, deviceToken=token, deviceTypeToken=dt))
        for r in out:
            r.setdefault("deviceToken", token)
        return out


class EchoStringDecoder(Decoder):
    def __init__(self, logger):
        self.logger = logger

    def decode(self, payload, metadata):
        self.logger.info("echo payload: %r", bytes(payload)[:256])
        return []


class PayloadLoggerDecoder(Decoder):
    """Debug wrapper: log the payload, then delegate."""

    def __init__(self, inner: Decoder, logger):
        self.inner, self.logger = inner, logger

    def decode(self, payload, metadata):
        self.logger.info("payload (%d bytes): %r", len(payload), bytes(payload)[:128])
        return self.inner.decode(payload, metadata)


# ------------------------------------------------------------------------------ deduplicators
class AlternateIdDeduplicator:
    """Drop requests whose alternate id already exists (event store lookup + recent-id window)."""

    def __init__(self, event_lookup, window: int = 100_000):
        self.lookup = event_lookup
        self.window = window
        self._recent: dict[str, float] = {}
        self._lock = threading.Lock()

    def is_duplicate(self, req: dict) -> bool:
        alt = (req.get("request") or {}).get("alternateId")
        if not alt:
            return False
        with self._lock:
            if alt in self._recent:
                return True
            self._recent[alt] = time.time()
            if len(self._recent) > self.window:
                for k in list(self._recent)[: self.window // 10]:
                    del self._recent[k]
        try:
            return self.lookup(alt) is not None
        except Exception:
            return False


class ScriptedDeduplicator:
    def __init__(self, runner, source: str):
        self.runner, self.source = runner, source

    def is_duplicate(self, req: dict) -> bool:
        return bool(self.runner.call(self.source, "is_duplicate", req, name="deduplicator"))


# ------------------------------------------------------------------------------ sources
class DirectReceiver(TenantEngineLifecycleComponent):
    """In-process receiver: ``inject(payload)`` hands bytes to the owning source."""

    component_type = LifecycleComponentType.InboundEventReceiver

    def __init__(self, rid: str = "direct"):
        super().__init__(f"receiver:{rid}")
        self.source = None
        self.received = 0

    def inject(self, payload: bytes, metadata: dict | None = None):
        self.received += 1
        return self.source.on_encoded_event_received(self, payload, metadata or {})


class InboundEventSource(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.InboundEventSource

    def __init__(self, source_id: str, decoder: Decoder | None, deduplicator=None, receivers=(), manager=None,
                 forward_raw: bool = False):
        super().__init__(f"source:{source_id}")
        self.source_id = source_id
        self.decoder = decoder
        self.deduplicator = deduplicator
        self.receivers = list(receivers)
        self.manager = manager
        self.forward_raw = forward_raw
        self.transcoded = 0                   # JSON payloads forwarded to the engine as protobuf
        for r in self.receivers:
            r.source = self

    def initialize(self, monitor):
        self.decoded_events = self.create_meter("decodedEvents")
        self.decode_failures = self.create_meter("decodeFailures")
        self.duplicates = self.create_meter("duplicates")
        for r in self.receivers:
            r.tenant_engine = self.tenant_engine
            self.initialize_nested_component(r, monitor, require=True)

    def start(self, monitor):
        for r in self.receivers:
            self.start_nested_component(r, monitor, require=False)

    def stop(self, monitor):
        for r in self.receivers:
            r.lifecycle_stop(monitor)

    def on_encoded_event_received(self, receiver, payload: bytes, metadata: dict) -> int:
        if self.forward_raw:
            raw = payload
            if isinstance(self.decoder, JsonDeviceRequestDecoder):
                # JSON devices join the fused engine path as the protobuf payloads they are
                # equivalent to; a request the engine path cannot represent exactly (metadata,
                # registrations, ...) or an invalid one keeps the per-event path below
                from ..pipeline.json_transcode import to_protobuf
                raw = to_protobuf(payload)
                if raw is not None:
                    self.transcoded += 1
            if raw is not None:
                self.manager.handle_raw_payload(self.source_id, raw, getattr(self.tenant_engine, "raw_batch", 4096))
                return 1
        try:
            reqs = self.decoder.decode(payload, metadata)
        except Exception as e:
            self.decode_failures.mark()
            self.manager.handle_failed_decode(self.source_id, payload, e)
            return 0
        n = 0
        for r in reqs:
            self.decoded_events.mark()
            if self.deduplicator is not None and self.deduplicator.is_duplicate(r):
                self.duplicates.mark()
                continue
            self.manager.handle_decoded_event(self.source_id, r)
            n += 1
        return n


class EventSourcesManager(TenantEngineLifecycleComponent):
    """Routes decoded requests to the bus (EventSourcesManager.java:153-197)."""

    def __init__(self, engine: "EventSourcesTenantEngine"):
        super().__init__("event-sources-manager")
        self.engine = engine
        self.tenant_engine = engine
        ms = engine.ms
        t = engine.tenant.token
        self.producer = ms.producer
        self.t_decoded = ms.instance.naming.decoded_events(t)
        self.t_failed = ms.instance.naming.failed_decode_events(t)
        self.t_registration = ms.instance.naming.device_registration_events(t)
        self.t_raw = ms.instance.naming.tenant_prefix(t) + RAW_PAYLOADS
        self.sources: dict[str, InboundEventSource] = {}
        self._raw_buf: list = []
        self._raw_lock = threading.Lock()      # the payload buffer
        self._pub_lock = threading.Lock()      # cut + publish of raw batches, in order

    def handle_decoded_event(self, source_id: str, req: dict):
        payload = {"sourceId": source_id, "deviceToken": req["deviceToken"], "originator": req.get("originator"),
                   "eventCreateRequest": {"type": req["type"], "request": req["request"]}}
        body = payloads.encode_inbound(payload)
        if req["type"] == "RegisterDevice":
            self.producer.send(self.t_registration, req["deviceToken"], body)
        else:
            self.producer.send(self.t_decoded, req["deviceToken"], body)

    def handle_failed_decode(self, source_id: str, payload: bytes, err: Exception):
        self.producer.send(self.t_failed, source_id, json.dumps(
            {"sourceId": source_id, "error": str(err), "payload": codec.to_wire(bytes(payload))}).encode())

    def _raw_partitions(self) -> int:
        """Partitions raw batches are split over (1 with ``rawPartitioning: false``)."""
        n = getattr(self, "_raw_nparts", None)
        if n is None:
            bus = self.engine.ms.instance.bus
            n = bus.partitions(self.t_raw) if hasattr(bus, "partitions") else 1
            if not self.engine.config.get("rawPartitioning", True):
                n = 1
            self._raw_nparts = n
        return n

    def handle_raw_payload(self, source_id: str, payload: bytes, flush_at: int = 4096):
        """Buffer a raw payload; the count bound is per partition (a flush splits the buffer over
        the partitions, so each record still carries ~``flush_at`` payloads at full rate)."""
        with self._raw_lock:
            self._raw_buf.append(bytes(payload))
            full = len(self._raw_buf) >= flush_at * self._raw_partitions()
        if full:
            self.flush_raw()

    def flush_raw(self):
        """Ship the buffered raw payloads as framed batch records (``pipeline/bus_io.py``), one per
        partition of the raw-payload topic: payloads are key-partitioned by device token, so with
        several engine replicas in the consumer group each device is processed -- its state merged,
        its alternate ids deduplicated -- by exactly one of them.  On the in-process bus a record is
        published in place: its bytes sit in pinned host memory when a GPU is present, so the
        MI355X engine DMAs the batch straight out of the topic."""
        with self._pub_lock:            # batches are published in the order they were cut
            with self._raw_lock:
                buf, self._raw_buf = self._raw_buf, []
            if buf:
                self._publish_raw(buf)

    def _publish_raw(self, buf: list):
        from ..pipeline.bus_io import RawBatchRecord, partition_payloads
        bus = self.engine.ms.instance.bus
        n = self._raw_partitions()
        if n > 1:
            parts = partition_payloads(buf, n)
            groups: dict[int, list] = {}
            for payload, p in zip(buf, parts.tolist()):
                groups.setdefault(max(p, 0), []).append(payload)      # unparsable: partition 0
        else:
            groups = {0: buf}
        items = sorted(groups.items())
        for i, (p, payloads) in enumerate(items):
            try:
                if hasattr(bus, "append_external"):
                    # on a protected raw topic this waits while the engine's consumer is behind
                    # (EventBus.protect): the receiving thread -- and so the device -- is throttled
                    rec = RawBatchRecord.from_payloads(payloads)
                    bus.append_external(self.t_raw, p, rec, rec.ptr, rec.value_len)
                else:
                    self.producer.send(self.t_raw, None, RawBatchRecord.from_payloads(payloads, pinned=False).value(),
                                       partition=p)
            except Exception:
                # nothing is dropped: the unpublished payloads go back to the front of the buffer
                rest = [x for _, ps in items[i:] for x in ps]
                with self._raw_lock:
                    self._raw_buf[:0] = rest
                raise


class EventSourcesTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        self.manager = EventSourcesManager(self)
        # raw batches for the MI355X engine are shipped at rawBatchSize payloads or every rawMaxDelayMs
        self.raw_batch = int(self.config.get("rawBatchSize", 4096))
        self.raw_delay_s = float(self.config.get("rawMaxDelayMs", 5)) / 1000.0
        self._flush_stop = threading.Event()
        ms = self.ms
        for sc in self.config.get("sources", []):
            src = self.build_source(sc)
            src.tenant_engine = self
            self.manager.sources[src.source_id] = src
            self.initialize_nested_component(src, monitor, require=False)
        self.api = {"EventSources": EventSourcesApi(self)}

    def build_source(self, sc: dict) -> InboundEventSource:
        from ..edges.receivers import build_receiver
        d = sc.get("decoder", "json")
        if sc.get("script") and (d == "script" or isinstance(d, dict) and d.get("type") == "script" and "script" not in d):
            d = {"type": "script", "script": sc["script"]}      # source-level script (imported templates)
        dec = self.build_decoder(d)
        if sc.get("logPayloads"):
            dec = PayloadLoggerDecoder(dec, self.logger)
        dd = None
        dcfg = sc.get("deduplicator", self.config.get("deduplicator"))
        if dcfg:
            if dcfg.get("type") == "alternate-id":
                ev = lambda alt: self.ms.api("DeviceEventManagement", self.tenant.token).get_device_event_by_alternate_id(alt)  # noqa
                dd = AlternateIdDeduplicator(ev)
            elif dcfg.get("type") == "script":
                dd = ScriptedDeduplicator(self.ms.scripts, self.script_source(dcfg["script"]))
        recs = [DirectReceiver("direct")] + [build_receiver(self._resolve_receiver_scripts(rc), self.ms.scripts)
                                            for rc in sc.get("receivers", [])]
        return InboundEventSource(sc["id"], dec, dd, recs, self.manager, forward_raw=sc.get("forward") == "raw")

    def _resolve_receiver_scripts(self, rc: dict) -> dict:
        """Receiver script references (socket interaction handler, REST polling ``scriptId``) -> source."""
        ref = rc.get("script") or rc.get("scriptId")
        return dict(rc, script=self.script_source(ref)) if ref else rc

    def build_decoder(self, d) -> Decoder:
        if isinstance(d, str):
            d = {"type": d}
        t = d.get("type")
        if t == "protobuf":
            return ProtobufDecoder()
        if t in ("json", "json-string"):          # JsonStringDeviceRequestDecoder: same document as text
            return JsonDeviceRequestDecoder()
        if t == "coap-json":
            return CoapJsonDecoder()
        if t == "json-batch":
            return JsonBatchDecoder()
        if t == "script":
            return ScriptedDecoder(self.ms.scripts, self.script_source(d["script"]))
        if t == "echo":
            return EchoStringDecoder(self.logger)
        if t == "composite":
            choices = {k: self.build_decoder(v) for k, v in d.get("choices", {}).items()}
            dm = lambda tok: self.ms.api("DeviceManagement", self.tenant.token)  # noqa: E731

            def dtype_of(tok):
                dev = dm(tok).get_device_by_token(tok)
                if dev is None:
                    return None
                dt = dm(tok).get_device_type(dev.device_type_id)
                return dt.token if dt else None

            if d.get("extractorScript"):
                # GroovyMessageMetadataExtractor: extract(payload, metadata) -> (token, payload) or
                # {"deviceToken": ..., "payload": ...}; works on binary payloads
                src, runner = self.script_source(d["extractorScript"]), self.ms.scripts

                def extractor(payload, md):
                    r = runner.call(src, "extract", bytes(payload), dict(md or {}), name="metadata-extractor")
                    tok, inner = (r["deviceToken"], r["payload"]) if isinstance(r, dict) else r
                    return tok, inner if isinstance(inner, (bytes, bytearray)) else str(inner).encode()
            else:
                def extractor(payload, md):
                    obj = json.loads(payload)
                    return obj[d.get("tokenField", "deviceToken")], json.dumps(obj.get(d.get("payloadField", "payload"), obj)).encode()
            return CompositeDecoder(extractor, choices, dtype_of, self.build_decoder(d["default"]) if d.get("default") else None)
        raise ValueError(f"unknown decoder {t!r}")

    def tenant_start(self, monitor):
        for s in self.manager.sources.values():
            self.start_nested_component(s, monitor, require=False)
        if any(s.forward_raw for s in self.manager.sources.values()):
            self._flush_stop.clear()
            threading.Thread(target=self._flusher, daemon=True, name=f"raw-flush-{self.tenant.token}").start()

    def _flusher(self):
        """Latency bound of the raw micro-batches (the count bound is checked on every payload)."""
        while not self._flush_stop.wait(self.raw_delay_s):
            try:
                self.manager.flush_raw()
            except Exception:
                self.logger.exception("raw batch flush failed")

    def tenant_stop(self, monitor):
        self._flush_stop.set()
        for s in self.manager.sources.values():
            s.lifecycle_stop(monitor)
        self.manager.flush_raw()

    def source(self, sid: str) -> InboundEventSource:
        return self.manager.sources[sid]

    def inject(self, source_id: str, payload: bytes, metadata: dict | None = None) -> int:
        return self.source(source_id).receivers[0].inject(payload, metadata)


class EventSourcesApi:
    """Management view of the tenant's sources (used by the admin REST API)."""

    def __init__(self, engine: EventSourcesTenantEngine):
        self._e = engine

    def list_event_sources(self) -> list[dict]:
        return [{"id": s.source_id, "status": s.status.value, "decoder": type(s.decoder).__name__ if s.decoder else None,
                 "receivers": [r.component_name for r in s.receivers],
                 "decodedEvents": s.decoded_events.count, "decodeFailures": s.decode_failures.count,
                 "duplicates": s.duplicates.count} for s in self._e.manager.sources.values()]

    def inject(self, source_id: str, payload: bytes, metadata: dict | None = None) -> int:
        return self._e.inject(source_id, payload, metadata)


class EventSourcesMicroservice(MultitenantMicroservice):
    identifier = "event-sources"
    name = "Event Sources"

    def service_names(self):
        return ["EventSources"]

    def create_tenant_engine(self, tenant):
        return EventSourcesTenantEngine(self, tenant)
