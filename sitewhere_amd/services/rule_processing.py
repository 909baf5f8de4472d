"""service-rule-processing: per-event rule processors on the enriched stream (multitenant).

Reference: ``KafkaRuleProcessorHost.java:77-250`` (one consumer group per processor, thread pool,
dispatch by event type to ``onMeasurement/onLocation/onAlert/...``), ``RuleProcessor`` base,
``ZoneTestRuleProcessor.java:47-62`` (JTS ``Polygon.contains`` per zone test -> alert through
event management, ``alert.setEventDate(new Date())``).  Added: a scripted processor and a threshold
processor; the zone test batches its point-in-polygon work onto the GPU when available
(:func:`sitewhere_amd.core.geo.batch_contains`).
"""
from __future__ import annotations

import numpy as np

from ..core.geo import batch_contains, polygon_of
from ..models.columnar import EV_LOCATION, EV_MEASUREMENT
from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from ..models.domain import DeviceEventType
from ..runtime.consumers import BusConsumer
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads


class RuleProcessor(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.RuleProcessor

    def __init__(self, pid: str):
        super().__init__(f"rule:{pid}")
        self.pid = pid
        self.alerts = 0

    def process_records(self, reader, recs):
        """A poll of enriched records: per-event records and engine batches (every row as an
        event).  Column-capable processors override :meth:`process_columns` for batches."""
        from .enriched_batches import expand_records, is_batch
        single = []
        for r in recs:
            if is_batch(r.value) and type(self).process_columns is not RuleProcessor.process_columns:
                self.process_columns(reader, reader.columns(r.value, strings=self.column_strings))
            else:
                single.append(r)
        if single:
            self.process_batch(expand_records(reader, single))

    column_strings = False        # the column forms read numbers and dictionaries, not the string heap

    def process_columns(self, reader, cols):
        """An engine batch as columns (``EnrichedBatchReader.columns``); default: row by row."""
        self.process_batch([(reader.event(cols, i), reader.context(cols, i)) for i in range(len(cols["date"]))])

    def raise_alerts(self, pairs):
        """Alerts of one batch in one durable add (``DeviceEventManagement.add_alert_batch``)."""
        if pairs:
            self.events_api().add_alert_batch(pairs)
            self.alerts += len(pairs)

    def process_batch(self, items: list[tuple]):
        for ev, ctx in items:
            h = {DeviceEventType.Measurement: self.on_measurement, DeviceEventType.Location: self.on_location,
                 DeviceEventType.Alert: self.on_alert, DeviceEventType.CommandInvocation: self.on_command_invocation,
                 DeviceEventType.CommandResponse: self.on_command_response,
                 DeviceEventType.StateChange: self.on_state_change}[ev.event_type]
            h(ctx, ev)

    def on_measurement(self, ctx, ev): pass
    def on_location(self, ctx, ev): pass
    def on_alert(self, ctx, ev): pass
    def on_command_invocation(self, ctx, ev): pass
    def on_command_response(self, ctx, ev): pass
    def on_state_change(self, ctx, ev): pass

    def events_api(self):
        e = self.tenant_engine
        return e.ms.api("DeviceEventManagement", e.tenant.token)


class ZoneTestRuleProcessor(RuleProcessor):
    """zoneTests: [{zoneToken, condition: inside|outside, alertType, alertLevel, alertMessage}]."""

    def __init__(self, pid: str, tests: list[dict]):
        super().__init__(pid)
        self.tests = tests
        self._polys: dict[str, object] = {}
        self.alerts = 0

    def _poly(self, token: str):
        p = self._polys.get(token)
        if p is None:
            e = self.tenant_engine
            z = e.ms.api("DeviceManagement", e.tenant.token).get_zone_by_token(token)
            if z is None:
                raise ValueError(f"Invalid zone token in zone test: {token}")
            p = self._polys[token] = polygon_of(z.bounds)
        return p

    def process_batch(self, items):
        locs = [(ev, ctx) for ev, ctx in items if ev.event_type == DeviceEventType.Location]
        if not locs or not self.tests:
            return
        polys = [self._poly(t["zoneToken"]) for t in self.tests]
        inside = batch_contains(polys, [(ev.latitude, ev.longitude) for ev, _ in locs])
        self.raise_alerts([(ev.device_assignment_id, self._request(t))
                           for i, (ev, _) in enumerate(locs) for j, t in enumerate(self.tests)
                           if (t.get("condition", "inside") == "inside") == bool(inside[i, j])])

    @staticmethod
    def _request(t):
        return {"type": t.get("alertType", "zone.alert"), "level": t.get("alertLevel", "Warning"),
                "message": t.get("alertMessage", ""), "source": "System", "updateState": False}

    def process_columns(self, reader, cols):
        """Location rows of an engine batch: one point-in-polygon pass over their columns, alerts
        for the hits in one add."""
        if not self.tests:
            return
        rows = np.nonzero(np.asarray(cols["etype"]) == EV_LOCATION)[0]
        if not len(rows):
            return
        polys = [self._poly(t["zoneToken"]) for t in self.tests]
        inside = batch_contains(polys, np.stack([cols["v0"][rows], cols["v1"][rows]], 1))
        ctx = cols["asg_ctx"]
        pairs = []
        for j, t in enumerate(self.tests):
            want = t.get("condition", "inside") == "inside"
            for i in np.nonzero(inside[:, j] == want)[0].tolist():
                a = ctx.get(int(cols["asg"][rows[i]]))
                if a:
                    pairs.append((a[0], self._request(t)))
        self.raise_alerts(pairs)


class ThresholdRuleProcessor(RuleProcessor):
    """Alert when a named measurement crosses a bound: {measurement, min?, max?, alertType, alertLevel}."""

    def __init__(self, pid: str, rules: list[dict]):
        super().__init__(pid)
        self.rules = rules
        self.alerts = 0

    @staticmethod
    def _request(r, name, value):
        lo, hi = r.get("min"), r.get("max")
        return {"type": r.get("alertType", f"{name}.threshold"), "level": r.get("alertLevel", "Warning"),
                "message": f"{name}={value} outside [{lo}, {hi}]", "source": "System"}

    def process_batch(self, items):
        pairs = []
        for ev, ctx in items:
            if ev.event_type != DeviceEventType.Measurement:
                continue
            for r in self.rules:
                lo, hi = r.get("min"), r.get("max")
                if r["measurement"] == ev.name and ((lo is not None and ev.value < lo) or
                                                    (hi is not None and ev.value > hi)):
                    pairs.append((ev.device_assignment_id, self._request(r, ev.name, ev.value)))
        self.raise_alerts(pairs)

    def process_records(self, reader, recs):
        """Durable engine batches natively (``EnrichedBatchReader.threshold_rows``: the block's
        measurement rows are tested where they lie packed, nothing else is decoded); anything else
        as :meth:`RuleProcessor.process_records`."""
        from .enriched_batches import is_batch
        rest, pairs = [], []
        for rec in recs:
            got = reader.threshold_rows(rec.value, self.rules) if is_batch(rec.value) else None
            if got is None:
                rest.append(rec)
                continue
            for r, hits in zip(self.rules, got):
                for a, v in hits:
                    if a:
                        pairs.append((a[0], self._request(r, r["measurement"], v)))
        self.raise_alerts(pairs)
        if rest:
            super().process_records(reader, rest)

    def process_columns(self, reader, cols):
        """Measurement rows of an engine batch against each rule on the columns (name id and value
        masks); only the rows out of bounds become alerts, all of the batch's in one add."""
        et = np.asarray(cols["etype"])
        name = np.asarray(cols["name"])
        v = np.asarray(cols["v0"])
        ctx = cols["asg_ctx"]
        pairs = []
        for r in self.rules:
            ids = reader.name_ids(cols, r["measurement"])
            if not ids:
                continue
            lo, hi = r.get("min"), r.get("max")
            m = (et == EV_MEASUREMENT) & np.isin(name, np.asarray(ids, name.dtype))
            out = np.zeros(len(v), bool)
            if lo is not None:
                out |= v < lo
            if hi is not None:
                out |= v > hi
            for i in np.nonzero(m & out)[0].tolist():
                a = ctx.get(int(cols["asg"][i]))
                if a:
                    pairs.append((a[0], self._request(r, r["measurement"], float(v[i]))))
        self.raise_alerts(pairs)


class ScriptedRuleProcessor(RuleProcessor):
    """User script defining any of ``on_measurement(ctx, ev, api)`` ... ``on_state_change``."""

    def __init__(self, pid: str, source: str):
        super().__init__(pid)
        self.source = source

    def _call(self, name, ctx, ev):
        ns = self.tenant_engine.ms.scripts.compile(self.source, f"rule-{self.pid}")
        if name in ns:
            self.tenant_engine.ms.scripts.call(self.source, name, ctx, ev.to_dict(), self.events_api(),
                                               name=f"rule-{self.pid}")

    def on_measurement(self, ctx, ev): self._call("on_measurement", ctx, ev)
    def on_location(self, ctx, ev): self._call("on_location", ctx, ev)
    def on_alert(self, ctx, ev): self._call("on_alert", ctx, ev)


def build_processor(cfg: dict, engine=None) -> RuleProcessor:
    t = cfg.get("type")
    if t == "zone-test":
        return ZoneTestRuleProcessor(cfg["id"], cfg.get("zoneTests", []))
    if t == "threshold":
        return ThresholdRuleProcessor(cfg["id"], cfg.get("rules", []))
    if t == "script":
        return ScriptedRuleProcessor(cfg["id"], engine.script_source(cfg["script"]) if engine else cfg["script"])
    raise ValueError(f"unknown rule processor {t!r}")


class RuleProcessingTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        self.processors = []
        self.hosts = []
        from .enriched_batches import EnrichedBatchReader, enriched_topics
        topics = enriched_topics(self)          # per-event records + engine tenants' batches
        for pc in self.config.get("processors", []):
            p = build_processor(pc, self)
            p.tenant_engine = self
            self.initialize_nested_component(p, monitor, require=False)
            self.processors.append(p)
            # one consumer group per processor: each sees the full enriched stream
            self.hosts.append(BusConsumer(self, f"rule-{p.pid}", topics, self._handler(p, EnrichedBatchReader(self)),
                                          threads=int(pc.get("numThreads", 0))))
        self.api = {"RuleProcessing": RuleProcessingApi(self)}

    @staticmethod
    def _handler(p: RuleProcessor, reader):
        def handle(recs):
            p.process_records(reader, recs)
        return handle

    def tenant_start(self, monitor):
        for h in self.hosts:
            self.start_nested_component(h, monitor, require=True)

    def tenant_stop(self, monitor):
        for h in self.hosts:
            h.lifecycle_stop(monitor)


class RuleProcessingApi:
    def __init__(self, e):
        self._e = e

    def list_rule_processors(self) -> list[dict]:
        return [{"id": p.pid, "type": type(p).__name__, "status": p.status.value,
                 "alerts": getattr(p, "alerts", 0)} for p in self._e.processors]


class RuleProcessingMicroservice(MultitenantMicroservice):
    identifier = "rule-processing"
    name = "Rule Processing"

    def service_names(self):
        return ["RuleProcessing"]

    def create_tenant_engine(self, tenant):
        return RuleProcessingTenantEngine(self, tenant)
