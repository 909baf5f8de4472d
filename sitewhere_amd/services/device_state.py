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


class _EngineStates:
    """Device state of one engine incarnation's enriched batches, column-wise: per assignment index
    the last interaction and, per state slot ((event type, name id): last location, last value of
    each measurement name, last alert of each type), the newest (event date, event id).  A batch
    merges with numpy only; DeviceState objects are written when a read needs them (``dirty``)."""

    def __init__(self, boot: int, header: dict):
        import numpy as np
        self.boot, self.world, self.rank = boot, int(header.get("world", 1)), int(header.get("rank", 0))
        self.n = 0
        self.last = np.zeros(0, np.int64)
        self.dirty = np.zeros(0, bool)
        self.slots: dict[tuple, list] = {}      # (etype, name id) -> [date int64[n], eid + 1 int64[n]]
        self._slot_lut = np.full(3 << 16, -1, np.int64)   # (etype << 16 | name id) -> dense slot number
        self._slot_keys: list[tuple] = []
        self.ctx: dict = {}                      # assignment index -> context list (reader dictionary)
        self._by_aid: dict = {}                  # assignment id -> index (rebuilt when ctx grows)
        self._by_aid_n = -1
        self.names: dict = {}                    # name id -> name

    def _grow(self, m: int):
        import numpy as np
        if m <= self.n:
            return
        m = max(m, 2 * self.n, 1024)
        pad = m - self.n
        self.last = np.concatenate([self.last, np.zeros(pad, np.int64)])
        self.dirty = np.concatenate([self.dirty, np.zeros(pad, bool)])
        for v in self.slots.values():
            v[0] = np.concatenate([v[0], np.full(pad, -1, np.int64)])
            v[1] = np.concatenate([v[1], np.zeros(pad, np.int64)])
        self.n = m

    def merge(self, cols: dict):
        """Newest (date, event id) per slot wins -- DeviceStateManagement.merge_event's rule."""
        import numpy as np
        from ..models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT
        self.ctx, self.names = cols.get("asg_ctx") or self.ctx, cols.get("names") or self.names
        et = np.asarray(cols["etype"])
        rows = np.flatnonzero((et == EV_MEASUREMENT) | (et == EV_LOCATION) | (et == EV_ALERT))
        if not len(rows):
            return
        h = cols["header"]
        asg = np.asarray(cols["asg"])[rows].astype(np.int64)
        keep = asg >= 0
        rows, asg = rows[keep], asg[keep]
        if not len(rows):
            return
        self._grow(int(asg.max()) + 1)
        ets = et[rows].astype(np.int64)
        name = np.where(ets == EV_LOCATION, 0xffff, np.asarray(cols["name"])[rows].astype(np.int64))
        date = np.asarray(cols["date"])[rows].astype(np.int64)
        eid1 = (int(h["first_seq"]) + int(cols.get("row0", 0)) + rows.astype(np.int64)) * self.world + self.rank + 1
        slot = (ets << 16) | name
        # dense slot numbers through a lookup table (no sort over the batch)
        lut = self._slot_lut
        new = np.unique(slot[lut[slot] < 0]) if (lut[slot] < 0).any() else ()
        for s in np.asarray(new).tolist():
            lut[s] = len(self._slot_keys)
            self._slot_keys.append((s >> 16, s & 0xffff))
            self.slots[(s >> 16, s & 0xffff)] = [np.full(self.n, -1, np.int64), np.zeros(self.n, np.int64)]
        sid = lut[slot]
        # the newest row per (slot, assignment): one max over (date, row) packed in an int64 (dates of
        # a batch span far less than 2^31 ms; rows < 2^32), per dense (slot, assignment) cell
        base = int(date.min())
        span = date - base
        cells = len(self._slot_keys) * self.n
        if int(span.max()) >= 1 << 31 or cells > max(1 << 24, 4 * len(rows)):   # sort instead
            order = np.lexsort((rows, date, sid * self.n + asg))
            k = (sid * self.n + asg)[order]
            lastm = np.ones(len(k), bool)
            lastm[:-1] = k[1:] != k[:-1]
            win = order[lastm]
        else:
            cell = sid * self.n + asg
            best = np.full(len(self._slot_keys) * self.n, -1, np.int64)
            np.maximum.at(best, cell, (span << 32) | np.arange(len(rows), dtype=np.int64))
            hit = best[best >= 0]
            win = (hit & 0xffffffff).astype(np.int64)
        recv = int(h.get("recv_ms") or now_ms())
        mark = np.zeros(self.n, bool)
        mark[asg] = True
        touched = np.flatnonzero(mark)
        self.last[touched] = np.maximum(self.last[touched], recv)
        self.dirty[touched] = True
        ws = sid[win]
        for j in np.flatnonzero(np.bincount(ws, minlength=len(self._slot_keys))).tolist():
            g = win[ws == j]
            t = self.slots[self._slot_keys[j]]
            a, d, e = asg[g], date[g], eid1[g]
            up = (d > t[0][a]) | ((d == t[0][a]) & (e > t[1][a]))
            t[0][a[up]] = d[up]
            t[1][a[up]] = e[up]

    def index_of(self, aid: str):
        """Assignment index of an assignment id (None: no engine row of it)."""
        if self._by_aid_n != len(self.ctx):
            self._by_aid = {c[0]: i for i, c in self.ctx.items() if c}
            self._by_aid_n = len(self.ctx)
        return self._by_aid.get(aid)

    def event_id(self, eid1: int) -> str:
        return f"{self.boot:x}-{int(eid1) - 1}"


class DeviceStateManagement:
    def __init__(self, store=None):
        self.states = Crud(store or create_store("memory"), "deviceStates", DeviceState, ErrorCode.InvalidDeviceStateId,
                           ("token", "device_assignment_id"))
        self._lock = threading.RLock()
        self._dates: dict[str, dict] = {}   # assignment -> {slot: event date}
        # (engine incarnation, rank) -> column-wise states: ranks of one incarnation number their
        # events apart (event id = (first_seq + row) * world + rank)
        self._engine: dict[tuple, _EngineStates] = {}

    def create_device_state(self, request: dict) -> DeviceState:
        return self.states.create(request)

    def get_device_state(self, id: str):
        self._sync()
        return self.states.get(id)

    def get_device_state_by_device_assignment_id(self, assignment_id: str):
        self._sync(assignment_id)            # that assignment's engine rows only
        return self.states.s.get_by(self.states.c, "device_assignment_id", assignment_id)

    # ---- engine batches ----------------------------------------------------------------
    def merge_batch(self, cols: dict):
        """An engine tenant's enriched batch (decoded block + dictionaries, EnrichedBatchReader):
        merged column-wise; the affected states are written on the next read."""
        h = cols["header"]
        key = (int(h["boot"]), int(h.get("rank", 0)), int(h.get("world", 1)))
        with self._lock:
            t = self._engine.get(key)
            if t is None:
                t = self._engine[key] = _EngineStates(key[0], h)
            t.merge(cols)

    def _sync(self, assignment_id: str | None = None):
        """Write the states engine batches changed since the last read (merge_event's slot rule
        against what the per-event path stored): every changed assignment, or only
        ``assignment_id``'s -- a per-assignment read (and every per-event merge) must not
        materialise a million-device fleet's states in Python on the way."""
        import numpy as np
        from ..models.columnar import EV_ALERT, EV_LOCATION
        with self._lock:
            for t in self._engine.values():
                if assignment_id is not None:
                    i0 = t.index_of(assignment_id)
                    idx = np.array([i0] if i0 is not None and i0 < len(t.dirty) and t.dirty[i0] else [], np.int64)
                else:
                    idx = np.flatnonzero(t.dirty)
                if not len(idx):
                    continue
                t.dirty[idx] = False
                for i in idx.tolist():
                    ctx = t.ctx.get(i)
                    if not ctx:
                        continue
                    aid = ctx[0]
                    st = self.states.s.get_by(self.states.c, "device_assignment_id", aid)
                    if st is None:
                        st = self.states.create({}, device_assignment_id=aid)
                    st.device_id = ctx[1] if len(ctx) > 1 else st.device_id
                    st.customer_id, st.area_id, st.asset_id = (ctx[2], ctx[3], ctx[4]) if len(ctx) > 4 else \
                        (st.customer_id, st.area_id, st.asset_id)
                    if len(ctx) > 6:
                        st.device_type_id = ctx[6]
                    st.last_interaction_date = max(st.last_interaction_date or 0, int(t.last[i]))
                    st.presence_missing_date = None
                    dates = self._dates.setdefault(aid, {})
                    for (et, nid), (dv, ev) in t.slots.items():
                        if ev[i] == 0:
                            continue
                        d = int(dv[i])
                        if et == EV_LOCATION:
                            key = "location"
                        else:
                            nm = t.names.get(nid, "")
                            key = ("alert:" if et == EV_ALERT else "mx:") + nm
                        if d < dates.get(key, -1):
                            continue
                        dates[key] = d
                        eid = t.event_id(int(ev[i]))
                        if et == EV_LOCATION:
                            st.last_location_event_id = eid
                        elif et == EV_ALERT:
                            st.last_alert_event_ids[t.names.get(nid, "")] = eid
                        else:
                            st.last_measurement_event_ids[t.names.get(nid, "")] = eid
                    self.states.put(st)

    def search_device_states(self, criteria=None) -> SearchResults:
        self._sync()
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
        self._sync()
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
                # an engine batch: merged column-wise (numpy, no per-event objects); states are
                # materialized when read
                self.management.merge_batch(self.reader.columns(r.value, strings=False))   # slots, dates, ids only
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
