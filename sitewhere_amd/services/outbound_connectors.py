"""service-outbound-connectors: fan-out of enriched events to external systems (multitenant).

Reference: ``KafkaOutboundConnectorHost.java:77-246`` (consumer group ``...connector.<id>``, pool of
``numProcessingThreads``), ``FilteredOutboundConnector`` (area / device-type / script filters),
``SerialOutboundConnector.java:37-75`` (per-event-type dispatch) and the connectors: MQTT (437),
RabbitMQ (295), SQS (188), EventHub (247), Dweet.io, InitialState, Solr, Groovy.

Delivery semantics: the reference commits offsets *before* the batch is processed (at-most-once,
SURVEY §5.2); :class:`~sitewhere_amd.runtime.consumers.BusConsumer` commits after processing
(at-least-once).
"""
from __future__ import annotations

import json
import os
import threading
import urllib.request

from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from ..edges.mqtt import MQTT_OPTIONS, client_from_config, parse_qos
from ..runtime.consumers import BusConsumer
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice


class OutboundConnector(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.OutboundConnector

    def __init__(self, cid: str, filters: list | None = None):
        super().__init__(f"connector:{cid}")
        self.cid = cid
        self.filters = filters or []
        self.delivered = 0
        self.filtered = 0

    def accept(self, ev, ctx) -> bool:
        return not any(f(ev, ctx) for f in self.filters)

    def process_batch(self, items):
        keep = [(ev, ctx) for ev, ctx in items if self.accept(ev, ctx)]
        self.filtered += len(items) - len(keep)
        if keep:
            self.deliver(keep)
            self.delivered += len(keep)

    def deliver(self, items):
        """Default: serial per-event dispatch (SerialOutboundConnector)."""
        for ev, ctx in items:
            self.on_event(ev, ctx)

    def on_event(self, ev, ctx):
        raise NotImplementedError


def event_json(ev, ctx) -> dict:
    return {"event": ev.to_dict(), "context": ctx}


class LogConnector(OutboundConnector):
    def __init__(self, cid, filters=None, keep: int = 10000):
        super().__init__(cid, filters)
        self.seen = []
        self.keep = keep

    def on_event(self, ev, ctx):
        if len(self.seen) < self.keep:
            self.seen.append(event_json(ev, ctx))


class MqttConnector(OutboundConnector):
    """Publish each event as JSON to ``topic`` (``{deviceToken}``/``{eventType}`` placeholders);
    ``mqtt`` carries the reference's ``MqttLifecycleComponent`` attributes (TLS, credentials, client
    id, clean session).  The client reconnects and retransmits unacknowledged QoS>0 publishes."""

    def __init__(self, cid, host, port, topic="SiteWhere/{tenant}/outbound/{deviceToken}", qos=0, filters=None,
                 **mqtt):
        super().__init__(cid, filters)
        self.host, self.port, self.topic, self.qos = host, port, topic, parse_qos(qos)
        self.mqtt = {k: v for k, v in mqtt.items() if v is not None}
        self.client = None

    def start(self, monitor):
        self.client = client_from_config(dict(self.mqtt, host=self.host, port=self.port), reconnect=True).connect()

    def on_event(self, ev, ctx):
        t = self.topic.format(tenant=self.tenant_engine.tenant.token, deviceToken=ctx.get("deviceToken"),
                              eventType=ev.event_type.value)
        self.client.publish(t, json.dumps(event_json(ev, ctx)).encode(), qos=self.qos)

    def stop(self, monitor):
        if self.client:
            self.client.disconnect()


class HttpConnector(OutboundConnector):
    """POST JSON batches to a webhook (covers the Dweet.io / InitialState style connectors)."""

    def __init__(self, cid, url, headers=None, batch=True, filters=None, post=None):
        super().__init__(cid, filters)
        self.url, self.headers, self.batch = url, headers or {}, batch
        self._post = post

    def _send(self, body):
        if self._post:
            return self._post(self.url, body)
        req = urllib.request.Request(self.url, data=json.dumps(body).encode(), method="POST",
                                     headers={"Content-Type": "application/json", **self.headers})
        urllib.request.urlopen(req, timeout=10).read()

    def deliver(self, items):
        if self.batch:
            self._send([event_json(ev, ctx) for ev, ctx in items])
        else:
            for ev, ctx in items:
                self._send(event_json(ev, ctx))


class SolrConnector(HttpConnector):
    """Index events as Solr documents via the JSON update handler (reference SolrOutboundConnector)."""

    def __init__(self, cid, solr_url, collection="SiteWhere", filters=None, post=None):
        super().__init__(cid, f"{solr_url.rstrip('/')}/{collection}/update?commit=true", filters=filters, post=post)

    def deliver(self, items):
        docs = []
        for ev, ctx in items:
            d = {"id": ev.id, "eventType": ev.event_type.value, "assignmentId": ev.device_assignment_id,
                 "deviceId": ev.device_id, "eventDate": ev.event_date, "receivedDate": ev.received_date}
            for k, v in ev.to_dict().items():
                if isinstance(v, (int, float, str)) and k not in d:
                    d[f"{k}_s" if isinstance(v, str) else f"{k}_d"] = v
            docs.append(d)
        self._send(docs)


class FileArchiveConnector(OutboundConnector):
    """Append events as JSON lines (cold archive / audit)."""

    def __init__(self, cid, path, filters=None):
        super().__init__(cid, filters)
        self.path = path
        self._lock = threading.Lock()

    def deliver(self, items):
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        with self._lock, open(self.path, "a") as f:
            for ev, ctx in items:
                f.write(json.dumps(event_json(ev, ctx)) + "\n")


class ScriptConnector(OutboundConnector):
    def __init__(self, cid, source, filters=None):
        super().__init__(cid, filters)
        self.source = source

    def on_event(self, ev, ctx):
        self.tenant_engine.ms.scripts.call(self.source, "process", ev.to_dict(), ctx, name=f"connector-{self.cid}")


def build_filters(engine, cfgs) -> list:
    out = []
    for f in cfgs or []:
        t = f.get("type")
        op = f.get("operation", "include")
        if t == "area":
            want = f["areaToken"]
            dm = lambda: engine.ms.api("DeviceManagement", engine.tenant.token)  # noqa: E731
            area_id = {}

            def area_filter(ev, ctx, want=want, op=op):
                if "id" not in area_id:
                    a = dm().get_area_by_token(want)
                    area_id["id"] = a.id if a else None
                hit = ev.area_id == area_id["id"]
                return (not hit) if op == "include" else hit
            out.append(area_filter)
        elif t == "device-type":
            want = f["deviceTypeToken"]
            cache = {}

            def dt_filter(ev, ctx, want=want, op=op):
                if "id" not in cache:
                    d = engine.ms.api("DeviceManagement", engine.tenant.token).get_device_type_by_token(want)
                    cache["id"] = d.id if d else None
                hit = ctx.get("deviceTypeId") == cache["id"]
                return (not hit) if op == "include" else hit
            out.append(dt_filter)
        elif t == "event-type":
            types = set(f["eventTypes"])
            out.append(lambda ev, ctx, types=types: ev.event_type.value not in types)
        elif t == "script":
            src = engine.script_source(f["script"])
            out.append(lambda ev, ctx, src=src: bool(engine.ms.scripts.call(src, "filter", ev.to_dict(), ctx,
                                                                            name="connector-filter")))
    return out


def build_connector(engine, cfg) -> OutboundConnector:
    t, cid = cfg.get("type"), cfg["id"]
    filters = build_filters(engine, cfg.get("filters"))
    if t == "log":
        return LogConnector(cid, filters)
    if t == "mqtt":
        return MqttConnector(cid, cfg.get("host", "127.0.0.1"), int(cfg.get("port", 1883)),
                             cfg.get("topic", "SiteWhere/{tenant}/outbound/{deviceToken}"), cfg.get("qos", 0), filters,
                             **{k: cfg.get(k) for k in MQTT_OPTIONS})
    if t == "http":
        return HttpConnector(cid, cfg["url"], cfg.get("headers"), cfg.get("batch", True), filters)
    from .cloud_connectors import build_cloud_connector
    cloud = build_cloud_connector(t, cid, cfg, filters)
    if cloud is not None:
        return cloud
    if t == "solr":
        return SolrConnector(cid, cfg["url"], cfg.get("collection", "SiteWhere"), filters)
    if t == "file":
        return FileArchiveConnector(cid, cfg["path"], filters)
    if t == "script":
        return ScriptConnector(cid, engine.script_source(cfg["script"]), filters)
    raise ValueError(f"unknown connector {t!r}")


class OutboundConnectorsTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        from .enriched_batches import EnrichedBatchReader, enriched_topics
        self.connectors, self.hosts, self.readers = [], [], []
        # per-event enriched records and engine tenants' enriched batches (one block per step)
        topics = enriched_topics(self)
        for cc in self.config.get("connectors", []):
            c = build_connector(self, cc)
            c.tenant_engine = self
            self.initialize_nested_component(c, monitor, require=False)
            self.connectors.append(c)
            reader = EnrichedBatchReader(self)
            self.readers.append(reader)
            self.hosts.append(BusConsumer(self, f"connector.{c.cid}", topics, self._handler(c, reader),
                                          threads=int(cc.get("numProcessingThreads", 0))))
        self.api = {"OutboundConnectors": OutboundConnectorsApi(self)}

    @staticmethod
    def _handler(c, reader):
        from .enriched_batches import expand_records

        def handle(recs):
            # processed before the consumer commits (at-least-once; the reference commits first)
            c.process_batch(expand_records(reader, recs))
        return handle

    def tenant_start(self, monitor):
        for c, h in zip(self.connectors, self.hosts):
            self.start_nested_component(c, monitor, require=False)
            self.start_nested_component(h, monitor, require=True)

    def tenant_stop(self, monitor):
        for c, h in zip(self.connectors, self.hosts):
            h.lifecycle_stop(monitor)
            c.lifecycle_stop(monitor)


class OutboundConnectorsApi:
    def __init__(self, e):
        self._e = e

    def list_connectors(self) -> list[dict]:
        return [{"id": c.cid, "type": type(c).__name__, "status": c.status.value, "delivered": c.delivered,
                 "filtered": c.filtered} for c in self._e.connectors]


class OutboundConnectorsMicroservice(MultitenantMicroservice):
    identifier = "outbound-connectors"
    name = "Outbound Connectors"

    def service_names(self):
        return ["OutboundConnectors"]

    def create_tenant_engine(self, tenant):
        return OutboundConnectorsTenantEngine(self, tenant)
