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
        self._tabs: dict = {}                     # boot -> (version, native string tables) for outbound JSON
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

    def asg_mask(self, boot: int, pos: int, value) -> np.ndarray:
        """bool per assignment index of the incarnation ``boot``: does its context field ``pos`` equal
        ``value``?  Cached until an assignment delta is applied (see :meth:`attr_mask`)."""
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
        return m

    def attr_mask(self, cols: dict, pos: int, value) -> np.ndarray:
        """bool per row of ``cols``: does the row's assignment context field ``pos`` (0 assignment,
        1 device, 2 customer, 3 area, 4 asset, 5 device token, 6 device type) equal ``value``?  The
        per-assignment answer is cached for the batch's engine incarnation and rebuilt only when an
        assignment delta was applied since (new entries or changed ones) -- a filter costs one gather
        per batch, not a Python call per row."""
        m = self.asg_mask(int(cols["header"]["boot"]), pos, value)
        asg = np.asarray(cols["asg"], np.int64)
        ok = (asg >= 0) & (asg < len(m))
        out = np.zeros(len(asg), bool)
        out[ok] = m[asg[ok]]
        return out

    # ------------------------------------------------------------------ native outbound JSON
    @staticmethod
    def _strtab(entries, n: int):
        """(heap, offsets [n + 1], presence [n]) of n optional strings (``entries``: index -> str)."""
        present = np.zeros(max(n, 1), np.uint8)
        parts, lens = [], np.zeros(max(n, 1), np.int64)
        for k, v in entries:
            if 0 <= k < n and v is not None:
                b_ = v.encode() if isinstance(v, str) else bytes(v)
                parts.append((k, b_))
                present[k] = 1
                lens[k] = len(b_)
        off = np.zeros(max(n, 1) + 1, np.int64)
        np.cumsum(lens, out=off[1:])
        heap = np.zeros(max(int(off[-1]), 8), np.uint8)
        for k, b_ in parts:
            heap[off[k]:off[k] + len(b_)] = np.frombuffer(b_, np.uint8)
        return heap, off, present

    def _tables(self, boot: int):
        """The boot's dictionaries as native string tables, rebuilt when a delta was applied."""
        with self._lock:
            ver = (self._ver.get(boot, 0), len(self._names.get(boot, {})), len(self._rules))
            t = self._tabs.get(boot)
            if t is not None and t[0] == ver:
                return t[1]
            a = self._asg.get(boot, {})
            n_asg = (max(a) + 1) if a else 0
            asg = self._strtab(((7 * i + k, (ctx[k] if k < len(ctx) else None)) for i, ctx in a.items()
                                for k in range(7)), 7 * n_asg)
            nm = self._names.get(boot, {})
            n_names = (max(nm) + 1) if nm else 0
            names = self._strtab(nm.items(), n_names)
            rules = self._strtab(((i, self._rules.get(v)) for i, v in nm.items() if v in self._rules), n_names)
            known = np.zeros(max(n_asg, 1), np.uint8)
            if a:
                known[np.fromiter(a.keys(), np.int64, len(a))] = 1
            tabs = (n_asg, asg, n_names, names, rules, known)
            self._tabs[boot] = (ver, tabs)
            return tabs

    def outbound_json(self, cols: dict, rows, topic: str | None = None):
        """Rows of a decoded batch as the outbound connectors' JSON documents ({"event", "context"},
        exactly ``json.dumps(event_json(event, context))``), written natively (``swjson_rows``): (payload
        bytes, offsets [n + 1], topic bytes, offsets) -- topics from ``topic`` (a template whose
        ``{deviceToken}`` / ``{eventType}`` are filled per row; None: no topics).  Rows the native
        writer does not handle (API-added JSON rows) come back as None for the Python path."""
        from .._native import native
        rows = np.ascontiguousarray(rows, np.int64)
        n = len(rows)
        if not n:
            return b"", np.zeros(1, np.int64), b"", np.zeros(1, np.int64)
        if cols.get("str_off") is None:
            raise ValueError("outbound JSON needs the batch's strings (columns(strings=True))")
        h = cols["header"]
        boot = int(h["boot"])
        n_asg, (ah, ao, ap), n_names, (nh, no, npr), (rh, ro, rp), _ = self._tables(boot)
        tpl = b""
        if topic is not None:
            tpl = topic.replace("{deviceToken}", "\x01").replace("{eventType}", "\x02").encode()
        P = lambda a: a.ctypes.data  # noqa: E731
        c = {k: np.ascontiguousarray(cols[k]) for k in ("etype", "level", "date", "asg", "name", "v0", "v1", "v2", "flags")}
        heap, soff = np.ascontiguousarray(cols["str_heap"]), np.ascontiguousarray(cols["str_off"], np.int64)
        cap, tcap = 480 * n + 4096, (len(tpl) + 96) * n + 64
        tb = np.frombuffer(tpl + b"\0", np.uint8)
        for _ in range(2):
            out, ooff = np.empty(cap, np.uint8), np.empty(n + 1, np.int64)
            tout, toff = np.empty(tcap, np.uint8), np.empty(n + 1, np.int64)
            k = int(native().swjson_rows(P(rows), n, *(P(c[x]) for x in ("etype", "level", "date", "asg", "name", "v0",
                                                                          "v1", "v2", "flags")), P(heap), P(soff),
                                         boot, int(h["first_seq"]), int(h["world"]), int(h["rank"]), int(h["recv_ms"]),
                                         int(cols.get("row0", 0)), P(ah), P(ao), P(ap), n_asg, P(nh), P(no), P(npr),
                                         n_names, P(rh), P(ro), P(rp), P(tb), len(tpl), P(out), cap, P(ooff),
                                         P(tout) if topic is not None else None, tcap, P(toff), None))
            if k >= 0:
                return (out[:k], ooff, tout[:int(toff[-1])] if topic is not None else b"",
                        toff if topic is not None else None)
            if -k - 1 < n:                    # row -k - 1 is not for the native writer
                return None
            need = -k - 1 - n                 # a buffer was too small: once more, sized
            cap, tcap = max(cap, need + 4096), max(tcap, need + 4096)
        return None

    def _buf(self, name: str, n: int, dtype) -> np.ndarray:
        """A scratch / output array of this thread, grown as needed and reused across calls (fresh
        tens of megabytes per block cost more in page faults than the JSON writing)."""
        tl = self.__dict__.get("_tl")
        if tl is None:
            with self._lock:
                tl = self.__dict__.setdefault("_tl", threading.local())
        bufs = tl.__dict__.setdefault("bufs", {})
        a = bufs.get(name)
        if a is None or len(a) < n:
            a = bufs[name] = np.empty(int(n * 1.25) + 64, dtype)
        return a

    def durable_block(self, value):
        """(boot, verified block) of a durable batch record with its dictionary deltas applied, or
        None for another record kind (a columnar batch).  A record handed over in process (a
        zero-copy view) is the engine's own sealed block; bytes from a bus are verified."""
        buf = memoryview(value).cast("B") if not isinstance(value, (bytes, bytearray)) else value
        if bytes(buf[:4]) != b"SWD1":
            return None
        d, blk = sg.decode_durable_batch(value)
        blk = np.ascontiguousarray(blk)
        if isinstance(value, (bytes, bytearray)):
            rc = sg.verify(blk)
            if rc:
                raise ValueError(f"corrupt event block (code {rc})")
        boot = int(sg.header(blk)["boot"])
        self._apply(boot, d)
        return boot, blk

    def threshold_rows(self, value, rules, threads: int = 1):
        """Per threshold rule ({measurement, min?, max?}): (assignment context, value) of the rows of
        a durable batch record whose measurement is out of bounds (``swseg_threshold_rows``: only the
        measurement rows' type, name and value are unpacked), or None for a record that is not a
        durable block.  Contexts the consumer has not seen are resolved as :meth:`columns` does."""
        from .._native import native
        got = self.durable_block(value)
        if got is None:
            return None
        boot, blk = got
        self.batches += 1
        self.rows += int(sg.header(blk)["n_rows"])
        out = []
        for r in rules:
            with self._lock:
                names = self._names.get(boot, {})
                ids = [int(i) for i, v in names.items() if v == r["measurement"]]
            lo, hi = r.get("min"), r.get("max")
            if not ids or (lo is None and hi is None):
                out.append([])
                continue
            mask = np.zeros(max(ids) + 1, np.uint8)
            mask[ids] = 1
            cap = 4096
            while True:
                rows, asg, vals = np.empty(cap, np.int64), np.empty(cap, np.int32), np.empty(cap, np.float64)
                k = int(native().swseg_threshold_rows(blk.ctypes.data, mask.ctypes.data, len(mask),
                                                      float(lo if lo is not None else 0.0),
                                                      float(hi if hi is not None else 0.0), int(lo is not None),
                                                      int(hi is not None), int(threads), rows.ctypes.data,
                                                      asg.ctypes.data, vals.ctypes.data, cap))
                if k < 0:
                    raise ValueError("event block decode failed")
                if k <= cap:
                    break
                cap = k
            asg, vals = asg[:k], vals[:k]
            if k:
                self._resolve(boot, np.unique(asg), [])
            ctx = self._asg.get(boot, {})
            out.append([(ctx.get(int(a)), float(v)) for a, v in zip(asg.tolist(), vals.tolist())])
        return out

    def select_json(self, value, selector, topic: str | None = None, threads: int = 1):
        """A durable batch record's rows that pass ``selector(boot) -> (event-type bit mask, keep per
        assignment index or None, keep for indexes beyond it)`` as :meth:`outbound_json` documents,
        straight from the block (``swjson_select_block``: event type and assignment are read from the
        packed columns, only kept rows are decoded; pages on ``threads`` threads): (payload bytes,
        offsets, topic bytes, offsets, kept rows, block rows), or None where the record needs the
        decoded path (not a durable block, or rows the native writer leaves to Python).  Dictionary
        entries the consumer has not seen are resolved from event management, as :meth:`columns`.
        The arrays returned are this thread's reused buffers: valid until its next call."""
        from .._native import native
        got = self.durable_block(value)
        if got is None:
            return None
        boot, blk = got
        tpl = b""
        if topic is not None:
            tpl = topic.replace("{deviceToken}", "\x01").replace("{eventType}", "\x02").encode()
        tb = np.frombuffer(tpl + b"\0", np.uint8)
        P = lambda a: a.ctypes.data  # noqa: E731
        n_rows = int(sg.header(blk)["n_rows"])
        threads = max(1, int(threads))
        scap, tscap = 600 * n_rows + 4096 * threads, (len(tpl) + 100) * n_rows + 4096 * threads
        counts, miss = np.zeros(3, np.int64), np.zeros(1 << 16, np.int64)
        for _ in range(6):
            etmask, keep, keep_default = selector(boot)
            n_keep = len(keep) if keep is not None else 0
            keep = np.ascontiguousarray(keep if keep is not None else np.zeros(1, bool), np.uint8)
            n_asg, (ah, ao, ap), n_names, (nh, no, npr), (rh, ro, rp), known = self._tables(boot)
            scratch, tscratch = self._buf("scratch", scap, np.uint8), self._buf("tscratch", tscap, np.uint8)
            out, ooff = self._buf("out", scap, np.uint8), self._buf("ooff", n_rows + 1, np.int64)
            tout, toff = self._buf("tout", tscap, np.uint8), self._buf("toff", n_rows + 1, np.int64)
            k = int(native().swjson_select_block(P(blk), int(etmask), P(keep), n_keep, int(bool(keep_default)), P(known),
                                                 n_asg, P(ah), P(ao), P(ap), P(nh), P(no), P(npr), n_names, P(rh),
                                                 P(ro), P(rp), P(tb), len(tpl), threads, P(scratch), len(scratch),
                                                 P(tscratch), len(tscratch), P(out), len(out), P(ooff),
                                                 P(tout) if topic is not None else None, len(tout), P(toff), P(counts),
                                                 P(miss), len(miss)))
            if k >= 0:
                kept = int(counts[0])
                self.batches += 1
                self.rows += int(counts[1])
                return (out[:k], ooff[:kept + 1], tout[:int(toff[kept])] if topic is not None else b"",
                        toff[:kept + 1] if topic is not None else None, kept, int(counts[1]))
            if k == -(1 << 42):
                m = miss[:int(counts[2])]
                self._resolve(boot, m[m >= 0], -1 - m[m < 0])
                with self._lock:                # entries the store does not hold either: no context
                    a = self._asg.setdefault(boot, {})
                    gone = [int(x) for x in m[m >= 0] if int(x) not in a]
                    if gone:
                        a.update({x: [] for x in gone})
                        self._ver[boot] = self._ver.get(boot, 0) + 1
                continue
            if k > -(1 << 40):                  # a buffer too small
                scap = tscap = max(scap, tscap, -k + 4096)
                continue
            return None
        return None

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
