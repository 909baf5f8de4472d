"""Engine tenants' enriched events for the enriched-event consumers.

Reference: outbound connectors, rule processors and device state all consume the enriched topic
(``KafkaOutboundConnectorHost.java:89``, ``KafkaRuleProcessorHost.java:89``,
``DeviceStateEnrichedEventsConsumer.java:75``), fed one ``GEnrichedEventPayload`` per event by
``OutboundPayloadEnrichmentLogic.java:54-92``.  An engine tenant (MI355X or native engine) publishes
its persisted events per step instead: one durable block per batch on ``inbound-enriched-batches``
(``services/gpu_inbound.py``; the same bytes the durable store writes), or a columnar row batch for
memory tenants.  The consumers subscribe to both topics; :class:`EnrichedBatchReader` turns a batch
record into the same ``(event, context)`` items a per-event record gives -- the whole event
(alternate id, metadata, alert message) and the context the reference's enrichment adds (device
id and token, device type, assignment status).

A batch carries only the dictionary entries its receiver has not seen (assignment contexts, name
ids).  A consumer group that starts later than the batch that carried an entry resolves it from
event management's store (``DeviceEventManagement.durable_dictionary``), once per entry.

Columnar consumers can ask for the decoded block instead (:meth:`EnrichedBatchReader.columns`) and
materialize only the rows they keep (vectorised filters, threshold rules).
"""
from __future__ import annotations

import threading

import numpy as np

from ..persistence import segments as sg

BATCH_MAGICS = (b"SWD1", b"SWC1")


def is_batch(value) -> bool:
    """Is a record value an engine batch (durable block or columnar rows) rather than one event?"""
    try:
        return bytes(memoryview(value)[:4]) in BATCH_MAGICS
    except TypeError:
        return False


class EnrichedBatchReader:
    """Per-consumer expansion of engine batches (thread-safe; dictionaries cached per incarnation)."""

    def __init__(self, engine):
        self.engine = engine                    # the consuming tenant engine (event management access)
        self._asg: dict[int, dict] = {}          # boot -> assignment index -> context list
        self._names: dict[int, dict] = {}        # boot -> name id -> name
        self._rules: dict[str, str] = {}
        self._lock = threading.Lock()
        self._masks: dict = {}                    # (boot, field, value) -> (bool per assignment, dictionary version)
        self._ver: dict[int, int] = {}            # boot -> version: bumped by every assignment delta applied
        self.rows = self.batches = self.resolved = 0

    # ------------------------------------------------------------------ dictionaries
    def _apply(self, boot: int, d: dict):
        with self._lock:
            asg = d.get("asg") or {}
            if asg:
                # a delta may rewrite known assignments in place (an assignment moved to another
                # area, a device's type changed): every cached mask of the boot is stale then
                self._ver[boot] = self._ver.get(boot, 0) + 1
            self._asg.setdefault(boot, {}).update({int(k): v for k, v in asg.items()})
            self._names.setdefault(boot, {}).update({int(k): v for k, v in (d.get("names") or {}).items()})
            self._rules.update(d.get("rules") or {})

    def _resolve(self, boot: int, asg_ids, name_ids):
        """Fetch the entries this consumer never saw a delta for (it started after their batch)."""
        a, n = self._asg.setdefault(boot, {}), self._names.setdefault(boot, {})
        miss_a = [int(x) for x in asg_ids if int(x) not in a and int(x) >= 0]
        miss_n = [int(x) for x in name_ids if int(x) not in n and int(x) != sg.NO_NAME]
        if not miss_a and not miss_n:
            return
        em = self.engine.ms.api("DeviceEventManagement", self.engine.tenant.token)
        got = em.durable_dictionary(boot, miss_a, miss_n)
        self.resolved += len(miss_a) + len(miss_n)
        self._apply(boot, got)

    # ------------------------------------------------------------------ batches
    def columns(self, value, strings: bool = True) -> dict:
        """Decoded block of a batch record with its dictionaries current: block columns + header
        (see ``persistence.segments.decode_block``) and ``cols["asg_ctx"]`` / ``["names"]`` /
        ``["rules"]`` for :func:`~sitewhere_amd.persistence.segments.materialize_row`.  A consumer
        that reads no alternate id, message or metadata passes ``strings=False`` (the string heap
        is not decoded; ``cols["str_heap"]`` is None)."""
        buf = memoryview(value).cast("B") if not isinstance(value, (bytes, bytearray)) else value
        if bytes(buf[:4]) == b"SWD1":
            d, blk = sg.decode_durable_batch(value)
            cols = sg.decode_block(np.ascontiguousarray(blk), strings=strings,
                                   check=isinstance(value, (bytes, bytearray)))
            boot = int(cols["header"]["boot"])
        else:
            from ..persistence.columnar import decode_batch
            d = decode_batch(value)
            rows = d["rows"]
            boot = sg.boot_id(d["boot"])
            n = len(rows)
            cols = {"etype": rows["etype"], "level": rows["level"], "date": rows["event_date"],
                    "asg": rows["assignment"], "name": rows["name_id"], "v0": rows["v0"], "v1": rows["v1"],
                    "v2": np.zeros(n), "flags": np.zeros(n, np.uint8), "str_heap": None, "str_off": None,
                    "row0": 0, "header": {"boot": boot, "first_seq": int(d["first_seq"]), "world": int(d["world"]),
                                          "rank": int(d["rank"]), "recv_ms": int(d["now"]), "n_rows": n}}
        self._apply(boot, d)
        self._resolve(boot, np.unique(cols["asg"]), np.unique(cols["name"]))
        cols["asg_ctx"], cols["names"], cols["rules"] = self._asg[boot], self._names[boot], self._rules
        self.batches += 1
        self.rows += len(cols["date"])
        return cols

    def attr_mask(self, cols: dict, pos: int, value) -> np.ndarray:
        """bool per row of ``cols``: does the row's assignment context field ``pos`` (0 assignment,
        1 device, 2 customer, 3 area, 4 asset, 5 device token, 6 device type) equal ``value``?  The
        per-assignment answer is cached for the batch's engine incarnation and rebuilt only when an
        assignment delta was applied since (new entries or changed ones) -- a filter costs one gather
        per batch, not a Python call per row."""
        boot = int(cols["header"]["boot"])
        key = (boot, pos, value)
        with self._lock:
            a = self._asg.get(boot, {})
            ver = self._ver.get(boot, 0)
            m, seen = self._masks.get(key, (None, -1))
            if m is None or seen != ver:
                n = (max(a) + 1) if a else 0
                m = np.zeros(n, bool)
                for i, ctx in a.items():
                    if len(ctx) > pos and ctx[pos] == value:
                        m[i] = True
                self._masks[key] = (m, ver)
        asg = np.asarray(cols["asg"], np.int64)
        ok = (asg >= 0) & (asg < len(m))
        out = np.zeros(len(asg), bool)
        out[ok] = m[asg[ok]]
        return out

    def name_ids(self, cols: dict, name: str) -> list[int]:
        """The batch incarnation's name ids of ``name`` (measurement name / alert type)."""
        boot = int(cols["header"]["boot"])
        with self._lock:
            return [int(i) for i, v in self._names.get(boot, {}).items() if v == name]

    def context(self, cols: dict, i: int) -> dict:
        """Enrichment context of row i (``OutboundPayloadEnrichmentLogic``: device and assignment)."""
        ctx = cols["asg_ctx"].get(int(cols["asg"][i])) or []
        return {"deviceId": ctx[1] if len(ctx) > 1 else None, "deviceToken": ctx[5] if len(ctx) > 5 else None,
                "deviceTypeId": ctx[6] if len(ctx) > 6 else None, "assignmentStatus": "Active", "engine": "batch"}

    def event(self, cols: dict, i: int):
        return sg.materialize_row(cols, i, cols["asg_ctx"], cols["names"], cols["rules"])

    def items(self, value, rows=None) -> list[tuple]:
        """(event, context) of every row (or of ``rows``) of a batch record."""
        cols = self.columns(value)
        idx = range(len(cols["date"])) if rows is None else rows
        return [(self.event(cols, int(i)), self.context(cols, int(i))) for i in idx]


def expand_records(reader: EnrichedBatchReader, recs) -> list[tuple]:
    """Records of the enriched topics -> (event, context) items, in record order: one per event
    record (``GEnrichedEventPayload`` / JSON), every row of an engine batch record."""
    from ..bus import payloads
    items = []
    for r in recs:
        if is_batch(r.value):
            items.extend(reader.items(r.value))
        else:
            ev, ctx, _ = payloads.decode_enriched(r.value, r.key)
            items.append((ev, ctx))
    return items


def enriched_topics(engine) -> list[str]:
    """The enriched-event topics of a tenant: per-event records and engine batches."""
    from .gpu_inbound import ENRICHED_BATCHES
    n = engine.ms.instance.naming
    return [n.inbound_enriched_events(engine.tenant.token), n.tenant_prefix(engine.tenant.token) + ENRICHED_BATCHES]
