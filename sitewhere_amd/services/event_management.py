"""service-event-management: device-event persistence + the persisted-event trigger (multitenant).

Reference: ``EventManagementImpl.java`` routed by ``EventManagementRouter.java:80-150``; backend chosen
by ``spring/EventManagementParser.java:72-160`` (MongoDB / Cassandra / InfluxDB); the store is wrapped
by ``KafkaEventPersistenceTriggers.java:72-97`` which forwards every stored event to
``inbound-persisted-events`` keyed by assignment id.  RPCs (``device-event-management.proto``, 16):
AddDeviceEventBatch, GetDeviceEventById, GetDeviceEventByAlternateId, Add/List{Measurements, Locations,
Alerts, CommandInvocations, StateChanges}(ForIndex), AddCommandResponses,
ListCommandResponsesForInvocation, ListCommandResponsesForIndex.
"""
from __future__ import annotations

import numpy as np


from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException
from ..models.domain import (AlertLevel, AlertSource, DateRangeSearchCriteria, DeviceAlert, DeviceCommandInvocation,
                             DeviceCommandResponse, DeviceEvent, DeviceEventIndex, DeviceEventType, DeviceLocation,
                             DeviceMeasurement, DeviceStateChange, now_ms)
from ..persistence.events import BufferedEventWriter, DeviceEventStore, create_event_store
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads

_BASE = ("alternateId", "eventDate", "metadata", "updateState")


def _dr(c) -> DateRangeSearchCriteria:
    if c is None:
        return DateRangeSearchCriteria(page_size=100)
    if isinstance(c, DateRangeSearchCriteria):
        return c
    return DateRangeSearchCriteria(c.get("pageNumber", 1), c.get("pageSize", 100), c.get("startDate"), c.get("endDate"))


class DeviceEventManagement:
    """IDeviceEventManagement: validates the assignment, stamps context, stores, fires triggers."""

    def __init__(self, store: DeviceEventStore, assignment_lookup, on_persisted=None, buffered: bool = False):
        self.store = store
        self._writer = BufferedEventWriter(store) if buffered else None
        self._lookup = assignment_lookup           # id -> DeviceAssignment | None
        self._on_persisted = on_persisted or (lambda events: None)

    def _context(self, assignment_id: str):
        a = self._lookup(assignment_id)
        if a is None:
            raise NotFoundException(ErrorCode.InvalidDeviceAssignmentToken, assignment_id)
        return a

    def _stamp(self, e: DeviceEvent, a, req: dict) -> DeviceEvent:
        e.device_id, e.device_assignment_id = a.device_id, a.id
        e.customer_id, e.area_id, e.asset_id = a.customer_id, a.area_id, a.asset_id
        e.alternate_id = req.get("alternateId")
        e.event_date = req.get("eventDate") or now_ms()
        e.received_date = now_ms()
        e.metadata = dict(req.get("metadata") or {})
        return e

    def _persist(self, events: list[DeviceEvent]) -> list[DeviceEvent]:
        if self._writer is not None:
            self._writer.add(events)
        else:
            self.store.add_events(events)
        self._on_persisted(events)
        return events

    def _add(self, assignment_id: str, requests, build) -> list:
        """Idempotent by alternate id: a redelivered request whose alternate id is already stored
        returns the stored event instead of persisting a second copy (at-least-once delivery +
        alternate-id dedup = exactly-once storage)."""
        a = self._context(assignment_id)
        reqs = requests if isinstance(requests, list) else [requests]
        out, new, seen = [], [], {}
        for r in reqs:
            alt = r.get("alternateId")
            if alt:
                ex = seen.get(alt) or (self._writer is not None and self._writer.pending_alternate(alt)) \
                    or self.store.get_event_by_alternate_id(alt)
                if ex is not None:
                    out.append(ex)
                    continue
            e = self._stamp(build(r), a, r)
            if alt:
                seen[alt] = e
            new.append(e)
            out.append(e)
        if new:
            self._persist(new)
        return out

    # ---- adds ------------------------------------------------------------------
    def add_measurements(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceMeasurement(name=r.get("name", ""), value=float(r.get("value", 0.0))))

    def add_locations(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceLocation(latitude=float(r.get("latitude", 0)), longitude=float(r.get("longitude", 0)),
                                                  elevation=r.get("elevation")))

    def add_alerts(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceAlert(source=AlertSource(r.get("source", "Device")),
                                               level=AlertLevel(r.get("level", "Info")), type=r.get("type", ""),
                                               message=r.get("message", "")))

    def add_alert_batch(self, pairs) -> int:
        """Alerts of many assignments in one durable add: ``pairs`` = [(assignment id, alert request)]
        (what a rule processor raises over one engine batch).  Requests carrying an alternate id go
        through the idempotent per-assignment path."""
        out, ctx = [], {}
        for aid, r in pairs:
            if r.get("alternateId"):
                self.add_alerts(aid, r)
                continue
            a = ctx.get(aid)
            if a is None:
                a = ctx[aid] = self._context(aid)
            out.append(self._stamp(DeviceAlert(source=AlertSource(r.get("source", "Device")),
                                               level=AlertLevel(r.get("level", "Info")), type=r.get("type", ""),
                                               message=r.get("message", "")), a, r))
        if out:
            self._persist(out)
        return len(pairs)

    # event builders per type (the per-type add_* methods above use the same constructors)
    _BUILD = {
        "Measurement": lambda r: DeviceMeasurement(name=r.get("name", ""), value=float(r.get("value", 0.0))),
        "Location": lambda r: DeviceLocation(latitude=float(r.get("latitude", 0)), longitude=float(r.get("longitude", 0)),
                                             elevation=r.get("elevation")),
        "Alert": lambda r: DeviceAlert(source=AlertSource(r.get("source", "Device")), level=AlertLevel(r.get("level", "Info")),
                                       type=r.get("type", ""), message=r.get("message", "")),
        "StateChange": lambda r: DeviceStateChange(attribute=r.get("attribute", ""), type=r.get("type", ""),
                                                   previous_state=r.get("previousState"), new_state=r.get("newState")),
        "CommandResponse": lambda r: DeviceCommandResponse(originating_event_id=r.get("originatingEventId"),
                                                           response_event_id=r.get("responseEventId"),
                                                           response=r.get("response")),
    }

    def add_event_batch(self, items, assignments: list | None = None) -> list:
        """Events of many assignments in ONE durable add: ``items`` = [(assignment id, event type,
        request)] -- a consumer's whole poll batch (the reference's DecodedEventsConsumer hands each
        event to its own add, DecodedEventsConsumer.java:155-204, and only the Mongo buffer batches the
        writes, DeviceEventBuffer.java:99-135).  Alternate ids are checked in one pass: already stored
        or repeated within the batch, the stored (or first) event is returned instead of a new one
        (exactly-once storage, as :meth:`_add`).  Returns the events, in item order; an item whose
        assignment is unknown raises like the per-event add (nothing of the batch is stored).
        ``assignments``: the items' assignment entities when the caller has them (device management
        announcing its own bulk create), instead of one lookup each."""
        ctx = {a.id: a for a in assignments or ()}
        out, new, seen = [], [], {}
        for aid, etype, r in items:
            a = ctx.get(aid)
            if a is None:
                a = ctx[aid] = self._context(aid)
            alt = r.get("alternateId")
            if alt:
                ex = seen.get(alt) or (self._writer is not None and self._writer.pending_alternate(alt)) \
                    or self.store.get_event_by_alternate_id(alt)
                if ex is not None:
                    out.append(ex)
                    continue
            build = self._BUILD.get(str(getattr(etype, "value", etype)))
            if build is None:
                raise SiteWhereSystemException(ErrorCode.Error, detail=f"batch add of {etype} events")
            e = self._stamp(build(r), a, r)
            if alt:
                seen[alt] = e
            new.append(e)
            out.append(e)
        if new:
            self._persist(new)
        return out

    def add_command_invocations(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceCommandInvocation(initiator=r.get("initiator", "REST"),
                                                           initiator_id=r.get("initiatorId"),
                                                           target=r.get("target", "Assignment"),
                                                           target_id=r.get("targetId") or assignment_id,
                                                           command_token=r.get("commandToken"),
                                                           device_command_id=r.get("deviceCommandId"),
                                                           parameter_values=dict(r.get("parameterValues") or {})))

    def add_command_responses(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceCommandResponse(originating_event_id=r.get("originatingEventId"),
                                                         response_event_id=r.get("responseEventId"),
                                                         response=r.get("response")))

    def add_state_changes(self, assignment_id: str, *requests):
        return self._add(assignment_id, _flat(requests),
                         lambda r: DeviceStateChange(attribute=r.get("attribute", ""), type=r.get("type", ""),
                                                     previous_state=r.get("previousState"),
                                                     new_state=r.get("newState")))

    def add_enriched_events(self, events: list, fire_triggers: bool = False) -> int:
        """Bulk insert of events already stamped and enriched upstream (the GPU inbound engine does
        lookup/validation/enrichment on device, so persisted triggers are normally not re-fired)."""
        if self._writer is not None:
            self._writer.add(events)
        else:
            self.store.add_events(events)
        if fire_triggers:
            self._on_persisted(events)
        return len(events)

    def durable_source_offset(self, topic: str, partition: int) -> int | None:
        """Next input offset of (topic, partition) whose events the durable store holds (commit
        records of engine tenants' blocks); None when the store keeps no such record."""
        f = getattr(self.store, "source_offset", None)
        return None if f is None else f(topic, int(partition))

    def durable_dictionary(self, boot, asg_ids=(), name_ids=()) -> dict:
        """Dictionary entries of an engine tenant's batches (see ``DurableEventStore.dictionary``):
        enriched-batch consumers resolve the indices their batches' deltas did not carry."""
        f = getattr(self.store, "dictionary", None)
        return f(boot, asg_ids, name_ids) if f is not None else {"asg": {}, "names": {}, "rules": {}}

    def add_durable_dictionary(self, boot, asg: dict | None = None, names: dict | None = None,
                               rules: dict | None = None, ctx: dict | None = None) -> bool:
        """Dictionary entries of an engine incarnation ahead of its blocks (an engine tenant with a
        large registry sends them once at start instead of inside its first block's delta)."""
        f = getattr(self.store, "add_dictionary", None)
        if f is None:
            return False
        f(boot, asg=asg, names=names, rules=rules, ctx=ctx)
        return True

    def durable_alternate_hashes(self, max_ids: int = 1 << 24, skip: int = 0) -> bytes:
        """Alternate-id hashes of the durable store, newest first (u64 little endian): ids ``skip`` to
        ``skip + max_ids`` of that order -- an engine tenant seeds its store-backed dedup filter with
        them on start, chunk by chunk."""
        f = getattr(self.store, "alternate_hash_chunks", None)
        if f is None:
            return b""
        return b"".join(np.ascontiguousarray(c, np.uint64).tobytes() for c in f(int(max_ids), skip=int(skip)))

    def durable_retention(self) -> dict:
        """Retention limits and holdings of the durable store ({} for other stores)."""
        f = getattr(self.store, "retention_state", None)
        return f() if f is not None else {}

    def durable_limit_retention_rows(self, rows: int) -> int:
        """Bound the durable store to ``rows`` event rows (only ever tightens): an engine tenant's
        store-backed dedup filter remembers its newest N ids, and the store then holds no id the
        filter forgot.  Returns the limit in force (0: the store has no such limit)."""
        f = getattr(self.store, "limit_retention_rows", None)
        return int(f(int(rows))) if f is not None else 0

    def durable_alternate_id_count(self) -> int:
        """Alternate ids the durable store holds (from its block index trailers)."""
        f = getattr(self.store, "alternate_id_count", None)
        return int(f()) if f is not None else 0

    def durable_find_alternate_hashes(self, hashes: bytes, covered: list | None = None,
                                      indexed_only: bool = False) -> bytes:
        """Which of these alternate-id hashes (u64 little endian) the durable store holds: the engine
        tenant settles the ids its store-backed filter sent back with one lookup per step.
        ``covered`` = [boot, rank, sequence]: the engine's dedup window holds every id of its rows
        from that sequence on (see ``DurableEventStore.find_alternate_hashes``); ``indexed_only``:
        look in the blocks the store has indexed, no scans."""
        f = getattr(self.store, "find_alternate_hashes", None)
        h = np.frombuffer(hashes, np.uint64)
        if f is None or not len(h):
            return b""
        found = f(h.tolist(), tuple(int(x) for x in covered) if covered else None, indexed_only=indexed_only)
        return np.array(sorted(found), np.uint64).tobytes()

    def add_durable_batch(self, payload) -> tuple[int, int]:
        """Queue an engine tenant's durable batch: (rows, token).  The rows are on disk once
        :meth:`durable_token` reaches the token (-1: a replay the store already holds)."""
        add = getattr(self.store, "add_batch", None)
        if add is None:                 # a store without durability tokens: synchronous
            return self.add_columnar_batch(payload), -1
        return add(payload)

    def durable_token(self) -> int:
        f = getattr(self.store, "durable", None)
        return f() if f is not None else 1 << 62

    def wait_durable(self, token: int, timeout_s: float = 60.0) -> bool:
        f = getattr(self.store, "wait", None)
        return True if f is None or token < 0 else bool(f(int(token), timeout_s))

    def add_columnar_batch(self, payload: bytes) -> int:
        """Append a columnar batch of GPU-enriched rows (MI355X tenants; needs the columnar datastore)."""
        if not hasattr(self.store, "add_columnar"):
            raise SiteWhereSystemException(ErrorCode.Error, detail="event store is not columnar")
        return self.store.add_columnar(payload)

    def add_device_event_batch(self, assignment_id: str, batch: dict) -> dict:
        """Measurements + locations + alerts in one call (reference AddDeviceEventBatch)."""
        return {"measurements": self.add_measurements(assignment_id, batch.get("measurements", [])),
                "locations": self.add_locations(assignment_id, batch.get("locations", [])),
                "alerts": self.add_alerts(assignment_id, batch.get("alerts", []))}

    # ---- reads -----------------------------------------------------------------
    def get_device_event_by_id(self, id: str):
        return self.store.get_event_by_id(id)

    def get_device_event_by_alternate_id(self, alt: str):
        return (self._writer is not None and self._writer.pending_alternate(alt)) or \
            self.store.get_event_by_alternate_id(alt)

    def _list(self, et, index, ids, criteria):
        return self.store.list_events(et, DeviceEventIndex(index) if isinstance(index, str) else index, list(ids),
                                      _dr(criteria))

    def list_measurements_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.Measurement, index, entity_ids, criteria)

    def list_locations_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.Location, index, entity_ids, criteria)

    def list_alerts_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.Alert, index, entity_ids, criteria)

    def list_command_invocations_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.CommandInvocation, index, entity_ids, criteria)

    def list_command_responses_for_invocation(self, invocation_id: str, criteria=None):
        return self.store.list_command_responses_for_invocation(invocation_id, _dr(criteria))

    def list_command_responses_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.CommandResponse, index, entity_ids, criteria)

    def list_state_changes_for_index(self, index, entity_ids, criteria=None):
        return self._list(DeviceEventType.StateChange, index, entity_ids, criteria)

    def flush(self):
        if self._writer is not None:
            self._writer.flush()


def _flat(requests):
    out = []
    for r in requests:
        if isinstance(r, list):
            out.extend(r)
        else:
            out.append(r)
    return out


class EventManagementTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        self.store = create_event_store(ds.get("type", "memory"), **{k: v for k, v in ds.items() if k != "type"})
        topic = self.ms.instance.naming.inbound_persisted_events(self.tenant.token)
        self.ms.instance.bus.topic(topic)
        prod = self.ms.producer

        def triggers(events):
            """KafkaEventPersistenceTriggers: forward each persisted event keyed by assignment id."""
            prod.send_batch(topic, [(e.device_assignment_id, payloads.encode_persisted(e)) for e in events])

        dm_api = lambda: self.ms.api("DeviceManagement", self.tenant.token)  # noqa: E731
        cache: dict = {}

        def lookup(aid):
            a = cache.get(aid)
            if a is None:
                a = dm_api().get_device_assignment(aid)
                if a is not None:
                    cache[aid] = a
            return a

        self.management = DeviceEventManagement(self.store, lookup, triggers, bool(self.config.get("buffered")))
        self.api = {"DeviceEventManagement": self.management}

    def tenant_stop(self, monitor):
        self.management.flush()
        close = getattr(self.store, "close", None)
        if close is not None and hasattr(self.store, "seg"):
            close()                     # durable segments: a restarted engine reopens the directory
        super().tenant_stop(monitor)


class EventManagementMicroservice(MultitenantMicroservice):
    identifier = "event-management"
    name = "Event Management"

    def service_names(self):
        return ["DeviceEventManagement"]

    def create_tenant_engine(self, tenant):
        return EventManagementTenantEngine(self, tenant)
