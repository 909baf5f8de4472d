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

import numpy as np

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
        self.threads = 0                          # numProcessingThreads: deliveries of a batch in parallel
        self._pool = None
        self._count_lock = threading.Lock()

    def accept(self, ev, ctx) -> bool:
        return not any(f(ev, ctx) for f in self.filters)

    def process_batch(self, items):
        keep = [(ev, ctx) for ev, ctx in items if self.accept(ev, ctx)]
        self.filtered += len(items) - len(keep)
        if keep:
            self._deliver_all(keep)

    def process_records(self, reader, recs):
        """A poll of enriched records.  Engine batches are filtered on their columns (area /
        device type / event type: one vectorised mask per batch) and only the rows that pass are
        materialized; per-event records and filters without a column form (scripts) go event by
        event.  Delivery of what passes runs on the connector's pool (``numProcessingThreads``)."""
        from .enriched_batches import is_batch
        keep, single = [], []
        for r in recs:
            if not is_batch(r.value):
                single.append(r)
                continue
            cols = reader.columns(r.value)
            n = len(cols["date"])
            excl = np.zeros(n, bool)
            per_row = []
            for f in self.filters:
                m = f.exclude(cols, reader) if hasattr(f, "exclude") else None
                if m is None:
                    per_row.append(f)
                else:
                    excl |= m
            rows = np.nonzero(~excl)[0]
            items = [(reader.event(cols, int(i)), reader.context(cols, int(i))) for i in rows]
            if per_row:
                items = [(ev, ctx) for ev, ctx in items if not any(f(ev, ctx) for f in per_row)]
            self.filtered += n - len(items)
            keep.extend(items)
        if single:
            from .enriched_batches import expand_records
            items = expand_records(reader, single)
            passed = [(ev, ctx) for ev, ctx in items if self.accept(ev, ctx)]
            self.filtered += len(items) - len(passed)
            keep.extend(passed)
        if keep:
            self._deliver_all(keep)

    def _deliver_all(self, items):
        if self._pool is None or len(items) < 2 * max(1, self.threads):
            self.deliver(items)
        else:
            step = -(-len(items) // self.threads)
            for f in [self._pool.submit(self.deliver, items[i:i + step]) for i in range(0, len(items), step)]:
                f.result()
        with self._count_lock:
            self.delivered += len(items)

    def set_threads(self, n: int):
        from concurrent.futures import ThreadPoolExecutor
        self.threads = max(0, int(n))
        self._pool = ThreadPoolExecutor(self.threads, thread_name_prefix=f"connector-{self.cid}") \
            if self.threads > 1 else None

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

    def _topic(self, ev, ctx):
        return self.topic.format(tenant=self.tenant_engine.tenant.token, deviceToken=ctx.get("deviceToken"),
                                 eventType=ev.event_type.value)

    def on_event(self, ev, ctx):
        self.client.publish(self._topic(ev, ctx), json.dumps(event_json(ev, ctx)).encode(), qos=self.qos)

    def deliver(self, items):
        """A batch's events in one write (QoS 0) / with their acknowledgements awaited together."""
        for i in range(0, len(items), 1024):
            self.client.publish_many([(self._topic(ev, ctx), json.dumps(event_json(ev, ctx)).encode())
                                      for ev, ctx in items[i:i + 1024]], qos=self.qos)

    # rows per native delivery job (JSON + framing of one job hold no interpreter lock)
    NATIVE_CHUNK = 16384

    def process_records(self, reader, recs):
        """Engine batches at QoS 0 behind column filters, natively: the kept rows of a decoded block
        are written as the same JSON documents (``EnrichedBatchReader.outbound_json``, byte for byte
        ``json.dumps(event_json(...))``) with their topics, framed as PUBLISH packets and sent in one
        write per block -- blocks on the delivery pool, no event object per row.  A durable block is
        selected natively (``select_json``: unselected rows are never decoded); a columnar batch is
        decoded and filtered on its columns.  Anything else (per-event records, QoS 1 / 2, script
        filters) takes the generic path."""
        from .enriched_batches import is_batch
        if self.qos != 0 or self.client is None or any(not hasattr(f, "select") for f in self.filters):
            return super().process_records(reader, recs)
        batches = [r for r in recs if is_batch(r.value)]
        single = [r for r in recs if not is_batch(r.value)]
        if single:
            super().process_records(reader, single)
        if not batches:
            return
        tpl = self.topic.replace("{tenant}", str(self.tenant_engine.tenant.token))
        selector = combined_selector(self.filters, reader)

        def frame(buf, off, tbuf, toff, n):
            from .._native import native
            tb = np.ascontiguousarray(tbuf, np.uint8) if len(tbuf) else np.zeros(1, np.uint8)
            cap = len(buf) + len(tbuf) + 8 * n + 64
            out = reader._buf("mqtt_frames", cap, np.uint8)
            k = int(native().swmqtt_publish_qos0(tb.ctypes.data, toff.ctypes.data, buf.ctypes.data, off.ctypes.data,
                                                 n, 0, out.ctypes.data, cap))
            self.client.publish_framed_qos0(memoryview(out[:k]))

        # one block in this poll: its pages are selected on the connector's threads instead (the
        # native pass splits them); several: one block per pool thread
        inner = max(1, self.threads) if len(batches) == 1 else 1

        def send_block(r):
            """A durable block: selection + JSON in one native pass, unselected rows never decoded."""
            got = reader.select_json(r.value, selector, topic=tpl, threads=inner)
            if got is None:
                return None
            buf, off, tbuf, toff, kept, total = got
            if kept:
                frame(buf, off, tbuf, toff, kept)
            with self._count_lock:
                self.filtered += total - kept
            return kept

        done, rest = 0, []
        if self._pool is None or len(batches) < 2:
            for r in batches:
                k = send_block(r)
                if k is None:
                    rest.append(r)
                else:
                    done += k
        else:
            futs = [(r, self._pool.submit(send_block, r)) for r in batches]
            for r, f in futs:
                k = f.result()
                if k is None:
                    rest.append(r)
                else:
                    done += k
        jobs = []
        for r in rest:
            cols = reader.columns(r.value)
            n = len(cols["date"])
            excl = np.zeros(n, bool)
            for f in self.filters:
                m = f.exclude(cols, reader)
                if m is not None:
                    excl |= m
            rows = np.nonzero(~excl)[0]
            self.filtered += n - len(rows)
            for i in range(0, len(rows), self.NATIVE_CHUNK):
                jobs.append((cols, rows[i:i + self.NATIVE_CHUNK]))

        def send(job):
            cols, rows = job
            got = reader.outbound_json(cols, rows, topic=tpl)
            if got is None:                       # a row the native writer leaves to Python
                self.deliver([(reader.event(cols, int(i)), reader.context(cols, int(i))) for i in rows])
                return len(rows)
            buf, off, tbuf, toff = got
            frame(buf, off, tbuf, toff, len(rows))
            return len(rows)

        if self._pool is None or len(jobs) < 2:
            done += sum(send(j) for j in jobs)
        else:
            done += sum(f.result() for f in [self._pool.submit(send, j) for j in jobs])
        with self._count_lock:
            self.delivered += done

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


ALL_ETYPES = -1                           # event-type bit mask of every type (int32: all bits)


def combined_selector(filters, reader):
    """``selector(boot) -> (event-type bit mask, keep per assignment index or None, keep beyond it)``
    of a connector's column filters together (a row passes when every filter keeps it), for
    :meth:`EnrichedBatchReader.select_json`."""
    def selector(boot):
        etmask, keep, dflt = ALL_ETYPES, None, True
        for f in filters:
            em, k, d = f.select(reader, boot)
            etmask &= em
            if k is None:
                continue
            if keep is None:
                keep, dflt = np.asarray(k, bool), bool(d)
                continue
            n = max(len(keep), len(k))
            a = np.full(n, dflt)
            a[:len(keep)] = keep
            b = np.full(n, bool(d))
            b[:len(k)] = k
            keep, dflt = a & b, dflt and bool(d)
        return etmask, keep, dflt
    return selector


class _Filter:
    """A connector filter (``FilteredOutboundConnector``): ``f(ev, ctx)`` is True for an event to
    leave out; ``exclude(cols, reader)`` is the same test over an engine batch's columns (a bool per
    row), or None where the filter has no column form; ``select(reader, boot)`` the same test as
    (event-type bit mask, keep per assignment index, keep beyond it) for the native block selection."""
    op = "include"

    def _out(self, hit):
        return ~hit if self.op == "include" else hit

    def exclude(self, cols, reader):
        return None

    def _select_attr(self, reader, boot, pos, value):
        m = reader.asg_mask(boot, pos, value)
        return (ALL_ETYPES, m, False) if self.op == "include" else (ALL_ETYPES, ~m, True)


class AreaFilter(_Filter):
    """``connectors/filter/AreaFilter.java``: events of (or not of) one area."""

    def __init__(self, engine, token: str, op: str):
        self.engine, self.token, self.op = engine, token, op
        self._id = None

    def area_id(self):
        if self._id is None:
            a = self.engine.ms.api("DeviceManagement", self.engine.tenant.token).get_area_by_token(self.token)
            self._id = (a.id if a else None,)
        return self._id[0]

    def __call__(self, ev, ctx):
        hit = ev.area_id == self.area_id()
        return (not hit) if self.op == "include" else hit

    def exclude(self, cols, reader):
        return self._out(reader.attr_mask(cols, 3, self.area_id()))

    def select(self, reader, boot):
        return self._select_attr(reader, boot, 3, self.area_id())


class DeviceTypeFilter(_Filter):
    """``connectors/filter/DeviceTypeFilter.java``: events of devices of (or not of) one type."""

    def __init__(self, engine, token: str, op: str):
        self.engine, self.token, self.op = engine, token, op
        self._id = None

    def type_id(self):
        if self._id is None:
            d = self.engine.ms.api("DeviceManagement", self.engine.tenant.token).get_device_type_by_token(self.token)
            self._id = (d.id if d else None,)
        return self._id[0]

    def __call__(self, ev, ctx):
        hit = ctx.get("deviceTypeId") == self.type_id()
        return (not hit) if self.op == "include" else hit

    def exclude(self, cols, reader):
        return self._out(reader.attr_mask(cols, 6, self.type_id()))

    def select(self, reader, boot):
        return self._select_attr(reader, boot, 6, self.type_id())


class EventTypeFilter(_Filter):
    def __init__(self, types):
        from ..persistence.api_blocks import _ETYPE
        from ..models.domain import DeviceEventType
        self.types = set(types)
        self.codes = np.array(sorted(_ETYPE[DeviceEventType(t)] for t in self.types), np.uint8)

    def __call__(self, ev, ctx):
        return ev.event_type.value not in self.types

    def exclude(self, cols, reader):
        return ~np.isin(np.asarray(cols["etype"]), self.codes)

    def select(self, reader, boot):
        m = 0
        for c in self.codes:
            m |= 1 << int(c)
        return (m - (1 << 32) if m >= 1 << 31 else m), None, True


class ScriptFilter(_Filter):
    def __init__(self, engine, src):
        self.engine, self.src = engine, src

    def __call__(self, ev, ctx):
        return bool(self.engine.ms.scripts.call(self.src, "filter", ev.to_dict(), ctx, name="connector-filter"))


def build_filters(engine, cfgs) -> list:
    out = []
    for f in cfgs or []:
        t = f.get("type")
        op = f.get("operation", "include")
        if t == "area":
            out.append(AreaFilter(engine, f["areaToken"], op))
        elif t == "device-type":
            out.append(DeviceTypeFilter(engine, f["deviceTypeToken"], op))
        elif t == "event-type":
            out.append(EventTypeFilter(f["eventTypes"]))
        elif t == "script":
            out.append(ScriptFilter(engine, engine.script_source(f["script"])))
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
            c.set_threads(int(cc.get("numProcessingThreads", 0)))
            self.initialize_nested_component(c, monitor, require=False)
            self.connectors.append(c)
            reader = EnrichedBatchReader(self)
            self.readers.append(reader)
            # the connector's pool delivers a poll's events (engine batches are single records: a
            # per-record split would leave one thread busy)
            self.hosts.append(BusConsumer(self, f"connector.{c.cid}", topics, self._handler(c, reader)))
        self.api = {"OutboundConnectors": OutboundConnectorsApi(self)}

    @staticmethod
    def _handler(c, reader):
        def handle(recs):
            # processed before the consumer commits (at-least-once; the reference commits first)
            c.process_records(reader, recs)
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
