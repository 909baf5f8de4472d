"""service-device-state: last-known state per assignment + presence detection (multitenant).

Reference: ``DeviceStateEnrichedEventsConsumer.java:75-187`` -> ``DeviceStateProcessingLogic.java:116-200``
(merge last interaction, last location, last measurement per name, last alert per type) and
``DevicePresenceManager.java:50-200`` (scan every ``checkInterval`` for states whose last interaction
is older than ``missingInterval``; emit a presence state-change event, send-once strategy).
RPCs (``device-state.proto``, 6): CreateDeviceState, GetDeviceState, GetDeviceStateByDeviceAssignmentId,
SearchDeviceStates, UpdateDeviceState, DeleteDeviceState.

Merge rule: the newest *event date* wins per slot (ties -> newest event), identical to the GPU
engine's two-pass merge, so batch and stream processing agree; the reference keeps the last
*processed* event, which depends on arrival order.
"""
from __future__ import annotations

import re
import threading

from ..core.errors import ErrorCode
from ..models.domain import DeviceEventType, DeviceState, SearchResults, now_ms
from ..persistence.store import create_store
from ..runtime.consumers import BusConsumer
from ..runtime.microservice import MicroserviceTenantEngine, MultitenantMicroservice
from ..bus import payloads
from .common import Crud, criteria_of

_ISO = re.compile(r"P(?:(\d+)D)?(?:T(?:(\d+)H)?(?:(\d+)M)?(?:(\d+)S)?)?")


def parse_period_ms(s) -> int:
    """ISO-8601 period (``PT10M``, ``PT8H``, ``P1D``) or a number of seconds."""
    if isinstance(s, (int, float)):
        return int(s * 1000)
    m = _ISO.fullmatch(s.strip().upper())
    if not m:
        raise ValueError(f"bad period {s!r}")
    d, h, mi, se = (int(x or 0) for x in m.groups())
    return ((d * 24 + h) * 60 + mi) * 60_000 + se * 1000


class DeviceStateManagement:
    def __init__(self, store=None):
        self.states = Crud(store or create_store("memory"), "deviceStates", DeviceState, ErrorCode.InvalidDeviceStateId,
                           ("token", "device_assignment_id"))
        self._lock = threading.RLock()
        self._dates: dict[str, dict] = {}   # assignment -> {slot: event date}

    def create_device_state(self, request: dict) -> DeviceState:
        return self.states.create(request)

    def get_device_state(self, id: str):
        return self.states.get(id)

    def get_device_state_by_device_assignment_id(self, assignment_id: str):
        return self.states.s.get_by(self.states.c, "device_assignment_id", assignment_id)

    def search_device_states(self, criteria=None) -> SearchResults:
        c = criteria or {}
        before = c.get("lastInteractionDateBefore") if isinstance(c, dict) else None
        sets = {k: set(c.get(k) or []) for k in ("deviceTypeIds", "customerIds", "areaIds", "assetIds")} if isinstance(c, dict) else {}

        def pred(s: DeviceState):
            if before and (s.last_interaction_date or 0) >= before:
                return False
            for k, f in (("deviceTypeIds", "device_type_id"), ("customerIds", "customer_id"), ("areaIds", "area_id"),
                         ("assetIds", "asset_id")):
                if sets.get(k) and getattr(s, f) not in sets[k]:
                    return False
            return True
        return self.states.list(criteria_of(c if isinstance(c, dict) and "pageSize" in c else None), pred,
                                sort=lambda s: s.last_interaction_date or 0, reverse=True)

    def update_device_state(self, id: str, request: dict):
        return self.states.update(id, request)

    def delete_device_state(self, id: str):
        return self.states.delete(id)

    # ---- DeviceStateProcessingLogic --------------------------------------------------
    def merge_event(self, event, context: dict, now: int | None = None) -> DeviceState | None:
        et = event.event_type
        with self._lock:
            st = self.get_device_state_by_device_assignment_id(event.device_assignment_id)
            if et not in (DeviceEventType.Alert, DeviceEventType.Location, DeviceEventType.Measurement):
                return st
            if st is None:
                st = self.states.create({}, device_assignment_id=event.device_assignment_id)
            st.device_id = event.device_id
            st.device_type_id = context.get("deviceTypeId")
            st.customer_id, st.area_id, st.asset_id = event.customer_id, event.area_id, event.asset_id
            st.last_interaction_date = max(st.last_interaction_date or 0, now or now_ms())
            st.presence_missing_date = None
            dates = self._dates.setdefault(event.device_assignment_id, {})
            d = event.event_date or 0
            if et == DeviceEventType.Location:
                slot = "location"
                if d >= dates.get(slot, -1):
                    dates[slot] = d
                    st.last_location_event_id = event.id
            elif et == DeviceEventType.Measurement:
                slot = "mx:" + event.name
                if d >= dates.get(slot, -1):
                    dates[slot] = d
                    st.last_measurement_event_ids[event.name] = event.id
            else:
                slot = "alert:" + event.type
                if d >= dates.get(slot, -1):
                    dates[slot] = d
                    st.last_alert_event_ids[event.type] = event.id
            return self.states.put(st)

    def find_missing(self, now_ms_: int, missing_ms: int) -> list[DeviceState]:
        limit = now_ms_ - missing_ms
        return self.states.query(lambda s: s.last_interaction_date is not None and s.last_interaction_date < limit
                                 and s.presence_missing_date is None)


class DevicePresenceManager(threading.Thread):
    def __init__(self, engine, check_ms: int, missing_ms: int):
        super().__init__(daemon=True, name=f"presence-{engine.tenant.token}")
        self.engine, self.check_ms, self.missing_ms = engine, check_ms, missing_ms
        self._stop = threading.Event()
        self.sent = 0

    def run(self):
        while not self._stop.wait(self.check_ms / 1000.0):
            try:
                self.check(now_ms())
            except Exception:
                self.engine.logger.exception("presence check failed")

    def check(self, now: int) -> int:
        mgmt = self.engine.management
        n = 0
        for st in mgmt.find_missing(now, self.missing_ms):
            ev_api = self.engine.ms.api("DeviceEventManagement", self.engine.tenant.token)
            ev_api.add_state_changes(st.device_assignment_id, {"attribute": "presence", "type": "automated",
                                                               "previousState": "PRESENT", "newState": "NOT_PRESENT"})
            st.presence_missing_date = now      # send-once: flag until the device interacts again
            mgmt.states.put(st)
            n += 1
        self.sent += n
        return n

    def stop(self):
        self._stop.set()


def latest_state_rows(cols: dict) -> list[int]:
    """Rows of a decoded engine batch that :meth:`DeviceStateManagement.merge_event` can keep: per
    (assignment, location | measurement name | alert type) the row with the newest event date, the
    later row on ties (merge order of the per-event path).  Vectorised: a 1M-row block materializes
    one event per state slot, not one per row."""
    import numpy as np
    from ..models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT
    et = np.asarray(cols["etype"])
    rows = np.flatnonzero((et == EV_MEASUREMENT) | (et == EV_LOCATION) | (et == EV_ALERT))
    if not len(rows):
        return []
    asg = np.asarray(cols["asg"])[rows].astype(np.int64)
    name = np.where(et[rows] == EV_LOCATION, 0, np.asarray(cols["name"])[rows].astype(np.int64) + 1)
    key = (asg << 34) | (et[rows].astype(np.int64) << 32) | (name & 0xffffffff)
    date = np.asarray(cols["date"])[rows].astype(np.int64)
    order = np.lexsort((rows, date, key))              # by key, then date, then row
    k = key[order]
    last = np.ones(len(k), bool)
    last[:-1] = k[1:] != k[:-1]
    return [int(i) for i in np.sort(rows[order[last]])]


class DeviceStateTenantEngine(MicroserviceTenantEngine):
    def tenant_initialize(self, monitor):
        ds = self.config.get("datastore", {"type": "memory"})
        self.management = DeviceStateManagement(create_store(ds.get("type", "memory"),
                                                             **{k: v for k, v in ds.items() if k != "type"}))
        from .enriched_batches import EnrichedBatchReader, enriched_topics
        # per-event enriched records and engine tenants' enriched batches (one durable block per step)
        self.reader = EnrichedBatchReader(self)
        self.consumer = BusConsumer(self, "device-state-enriched", enriched_topics(self), self._process)
        pres = self.config.get("presence", {})
        self.presence = DevicePresenceManager(self, parse_period_ms(pres.get("checkInterval", "PT10M")),
                                              parse_period_ms(pres.get("missingInterval", "PT8H")))
        self.api = {"DeviceStateManagement": self.management}

    def _process(self, recs):
        from .enriched_batches import is_batch
        for r in recs:
            if is_batch(r.value):
                # an engine batch: only the newest row of each state slot can change the state
                cols = self.reader.columns(r.value)
                for i in latest_state_rows(cols):
                    self.management.merge_event(self.reader.event(cols, i), self.reader.context(cols, i))
                continue
            ev, ctx, _ = payloads.decode_enriched(r.value, r.key)
            self.management.merge_event(ev, ctx)

    def tenant_start(self, monitor):
        self.start_nested_component(self.consumer, monitor, require=True)
        self.presence.start()

    def tenant_stop(self, monitor):
        self.consumer.lifecycle_stop(monitor)
        self.presence.stop()


class DeviceStateMicroservice(MultitenantMicroservice):
    identifier = "device-state"
    name = "Device State"

    def service_names(self):
        return ["DeviceStateManagement"]

    def create_tenant_engine(self, tenant):
        return DeviceStateTenantEngine(self, tenant)
