"""Columnar event store for MI355X tenants: enriched GPU output rows kept as numpy columns.

The fused inbound engine emits 32-byte ``OUT_REC`` rows (date, value(s), assignment index, interned
name, type, level) with implicit event ids.  Turning each into a Python event object before storage
caps a tenant at ~10^5 events/s on the host; this store appends the rows as columns (zero-copy
``frombuffer`` of the batch payload) plus small dictionaries (assignment index -> assignment /
device / customer / area / asset ids, name id -> name), and materialises domain objects only for
the page a query returns.  It implements :class:`~sitewhere_amd.persistence.events.DeviceEventStore`
(object events -- e.g. command invocations added over REST -- go to an embedded memory store and
are merged into query results), so event management serves GPU tenants through the same 16 RPCs.

Batch wire format (:func:`encode_batch` / :func:`decode_batch`): ``b"SWC1"``, a u32 header length,
a msgpack header ``{"boot", "first_seq", "world", "rank", "now", "asg": {idx: [assignment, device,
customer, area, asset]}, "names": {name_id: name}, "rules": {alert_type: message}}``, then the
OUT_REC rows as raw bytes.  The rows are copied once when the batch is built and viewed in place
(``np.frombuffer``) when it is read -- a 64K-row batch is 2 MB, and packing it inside msgpack cost
two more copies (0.45 ms per batch on the MI355X tenant path).
"""
from __future__ import annotations

import ctypes
import struct
import threading

import msgpack
import numpy as np

from .._native import native
from ..models.columnar import EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_STATE_CHANGE, NO_NAME, OUT_REC
from ..models.domain import (AlertLevel, AlertSource, DateRangeSearchCriteria, DeviceAlert, DeviceEventIndex,
                             DeviceEventType, DeviceLocation, DeviceMeasurement, DeviceStateChange, SearchResults)
from .events import DeviceEventStore, MemoryEventStore

_ETYPE = {DeviceEventType.Measurement: EV_MEASUREMENT, DeviceEventType.Location: EV_LOCATION,
          DeviceEventType.Alert: EV_ALERT, DeviceEventType.StateChange: EV_STATE_CHANGE}
_LEVELS = [AlertLevel.Info, AlertLevel.Warning, AlertLevel.Error, AlertLevel.Critical]
_CTX = {DeviceEventIndex.Assignment: 0, DeviceEventIndex.Customer: 2, DeviceEventIndex.Area: 3,
        DeviceEventIndex.Asset: 4}


_MAGIC = b"SWC1"
_COPY_THREADS = int(__import__("os").environ.get("SW_MEMCPY_THREADS", "0"))     # 0: one per 4 MB, <= 16


_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = (ctypes.c_void_p, ctypes.c_ssize_t)


def _header(boot: str, first_seq: int, world: int, rank: int, now: int, asg: dict, names: dict,
            rules: dict | None) -> bytes:
    return msgpack.packb({"boot": boot, "first_seq": int(first_seq), "world": int(world), "rank": int(rank),
                          "now": int(now), "asg": {int(k): list(v) for k, v in asg.items()},
                          "names": {int(k): v for k, v in names.items()}, "rules": rules or {}}, use_bin_type=True)


def encode_batch(boot: str, first_seq: int, world: int, rank: int, now: int, rows: np.ndarray, asg: dict,
                 names: dict, rules: dict | None = None) -> bytes:
    hdr = _header(boot, first_seq, world, rank, now, asg, names, rules)
    rows = np.ascontiguousarray(rows, OUT_REC)
    head = b"".join((_MAGIC, struct.pack("<I", len(hdr)), hdr))
    if rows.nbytes < (1 << 20):
        return head + memoryview(rows).cast("B")
    # a fresh (not yet shared) bytes object filled in place: the rows are copied once, over several
    # threads and without the GIL (one core copied ~7 GB/s: 5 ms per 1M-row batch)
    out = _new_bytes(None, len(head) + rows.nbytes)
    base = ctypes.cast(ctypes.c_char_p(out), ctypes.c_void_p).value
    ctypes.memmove(base, head, len(head))
    native().sw_memcpy_mt(base + len(head), rows.ctypes.data, rows.nbytes, _COPY_THREADS)
    return out


def frame_batch(frame: tuple, rows_nbytes: int, boot: str, first_seq: int, world: int, rank: int, now: int,
                asg: dict, names: dict, rules: dict | None = None) -> np.ndarray | None:
    """Zero-copy form of :func:`encode_batch` for rows that sit at ``offset`` of a host buffer with
    free bytes in front of them (``frame = (buffer, offset)``, the MI355X engine's pinned row
    buffers): the header is written right before the rows and the payload is the read-only view
    header + rows -- no row copy.  None when the header does not fit the free bytes."""
    buf, off = frame
    hdr = _header(boot, first_seq, world, rank, now, asg, names, rules)
    start = off - 8 - len(hdr)
    if start < 0:
        return None
    buf[start:start + 4] = np.frombuffer(_MAGIC, np.uint8)
    buf[start + 4:start + 8] = np.frombuffer(struct.pack("<I", len(hdr)), np.uint8)
    buf[start + 8:off] = np.frombuffer(hdr, np.uint8)
    view = buf[start:off + rows_nbytes]
    view.flags.writeable = False
    return view


def decode_batch(payload) -> dict:
    """``bytes`` or a zero-copy buffer (read-only array / memoryview) -> header dict + row view."""
    buf = payload if isinstance(payload, (bytes, bytearray)) else memoryview(payload).cast("B")
    if bytes(buf[:4]) == b"SWD1":             # durable batch: an encoded block (persistence/segments.py)
        from .segments import decode_block, decode_durable_batch, rows_of
        d, blk = decode_durable_batch(payload)
        cols = decode_block(blk)
        h = cols["header"]
        d.update(boot=f"{h['boot']:x}", first_seq=h["first_seq"], world=h["world"], rank=h["rank"],
                 now=h["recv_ms"], rows=rows_of(cols))
        return d
    if bytes(buf[:4]) != _MAGIC:              # batches written before the framed format
        d = msgpack.unpackb(bytes(buf), raw=False, strict_map_key=False)
        d["rows"] = np.frombuffer(d["rows"], OUT_REC)
        return d
    (n,) = struct.unpack_from("<I", buf, 4)
    d = msgpack.unpackb(bytes(buf[8:8 + n]), raw=False, strict_map_key=False)
    d["rows"] = np.frombuffer(buf, OUT_REC, offset=8 + n)
    return d


class ColumnarEventStore(DeviceEventStore):
    """``retention_rows`` bounds the rows held (oldest batches are evicted first, whole batches at a
    time): an MI355X tenant stores ~32 B x 10^8 events/s, so an unbounded in-memory store is a
    test/bench setting.  Evicted memory goes back to the allocator and is reused by the next
    batches -- fresh pages cost a page fault and a zeroing each, which halves the store's copy rate
    (4.8 vs 1.8 ms per 1M-row batch on 8 cores).  Durable history belongs to a persistent event
    store or to a consumer of the enriched-batch topic."""

    def __init__(self, consolidate_every: int = 64, dense_rows: int = 4096, retention_rows: int | None = None):
        self._objects = MemoryEventStore()
        self._chunks: list[dict] = []
        self._pending: list[dict] = []
        self._asg: dict[int, list] = {}         # assignment index -> [assignment, device, customer, area, asset]
        self._names: dict[int, str] = {}
        self._rules: dict[str, str] = {}
        self._boots: list[str] = []
        self._high: dict[tuple, int] = {}       # (boot, rank) -> next store sequence not yet held
        self._lock = threading.RLock()
        self.consolidate_every = consolidate_every
        self.dense_rows = dense_rows
        self.retention_rows = int(retention_rows) if retention_rows else None
        self.rows = 0               # rows held
        self.evicted_rows = 0

    # ------------------------------------------------------------------ ingest
    def dictionary(self, boot, asg_ids=(), name_ids=()) -> dict:
        """Assignment contexts / names of the rows held here (one engine incarnation at a time)."""
        return {"asg": {int(i): self._asg[int(i)] for i in asg_ids if int(i) in self._asg},
                "names": {int(i): self._names[int(i)] for i in name_ids if int(i) in self._names},
                "rules": dict(getattr(self, "_rules", {}) or {})}

    def add_columnar(self, payload: bytes | dict) -> int:
        d = payload if isinstance(payload, dict) else decode_batch(payload)
        rows = d["rows"]
        n = len(rows)
        with self._lock:
            self._asg.update({int(k): v for k, v in d["asg"].items()})
            self._names.update({int(k): v for k, v in d["names"].items()})
            self._rules.update(d.get("rules") or {})
            if d["boot"] not in self._boots:
                self._boots.append(d["boot"])
            # idempotent by store sequence: a shard restored from a checkpoint replays the batches
            # after it with the same (boot, sequence) ids -- rows already held are skipped
            key = (d["boot"], int(d["rank"]))
            high = self._high.get(key, 0)
            first = int(d["first_seq"])
            if first < high:
                skip = min(n, high - first)
                rows, first, n = rows[skip:], first + skip, n - skip
                d = dict(d, first_seq=first)
            if n:
                self._high[key] = max(high, first + n)
                bi = self._boots.index(d["boot"])
                if n >= self.dense_rows:
                    # large batch: zero-copy rows + scalar metadata, ids computed when queried
                    self._chunks.append({"rows": rows, "boot_i": bi, "first": first, "world": int(d["world"]),
                                         "rank": int(d["rank"]), "now": int(d["now"])})
                else:
                    eid = (first + np.arange(n, dtype=np.int64)) * d["world"] + d["rank"]
                    self._pending.append({"boot": np.full(n, bi, np.int16), "eid": eid,
                                          "rows": rows, "recv": np.full(n, d["now"], np.int64)})
                    if len(self._pending) >= self.consolidate_every:
                        self._consolidate()
                self.rows += n
                if self.retention_rows is not None and self.rows > self.retention_rows:
                    self._evict()
        return n

    def _evict(self):
        """Drop the oldest whole chunks until the rows held fit ``retention_rows`` (the newest chunk
        always stays)."""
        self._consolidate()
        while len(self._chunks) > 1 and self.rows > self.retention_rows:
            n = len(self._chunks.pop(0)["rows"])
            self.rows -= n
            self.evicted_rows += n

    # chunk accessors: dense chunks (scalar metadata) and consolidated small batches (per-row arrays)
    @staticmethod
    def _eids(ch: dict, idx: np.ndarray) -> np.ndarray:
        if "eid" in ch:
            return ch["eid"][idx]
        return (ch["first"] + np.asarray(idx, np.int64)) * ch["world"] + ch["rank"]

    @staticmethod
    def _boot_of(ch: dict, i: int) -> int:
        return int(ch["boot"][i]) if "boot" in ch else ch["boot_i"]

    @staticmethod
    def _recv_of(ch: dict, i: int) -> int:
        return int(ch["recv"][i]) if "recv" in ch else ch["now"]

    @staticmethod
    def _find_eid(ch: dict, b: int, eid: int) -> int:
        """Row of event id ``eid`` (boot index ``b``) in ``ch``, -1 if absent."""
        if "eid" in ch:
            hit = np.nonzero((ch["eid"] == eid) & (ch["boot"] == b))[0]
            return int(hit[0]) if len(hit) else -1
        if ch["boot_i"] != b or (eid - ch["rank"]) % ch["world"]:
            return -1
        row = (eid - ch["rank"]) // ch["world"] - ch["first"]
        return int(row) if 0 <= row < len(ch["rows"]) else -1

    def _consolidate(self):
        if not self._pending:
            return
        parts = self._pending
        self._pending = []
        self._chunks.append({"boot": np.concatenate([p["boot"] for p in parts]),
                             "eid": np.concatenate([p["eid"] for p in parts]),
                             "rows": np.concatenate([p["rows"] for p in parts]),
                             "recv": np.concatenate([p["recv"] for p in parts])})

    def _all_chunks(self) -> list[dict]:
        with self._lock:
            self._consolidate()
            return list(self._chunks)

    # ------------------------------------------------------------------ DeviceEventStore
    def add_events(self, events):
        return self._objects.add_events(events)

    def count(self) -> int:
        return self.rows + self._objects.count()

    def get_event_by_alternate_id(self, alt: str):
        return self._objects.get_event_by_alternate_id(alt)   # GPU rows carry only the alt-id hash

    def get_event_by_id(self, id: str):
        boot, sep, num = id.rpartition("-")
        if sep and boot in self._boots and num.isdigit():
            b, eid = self._boots.index(boot), int(num)
            for c in self._all_chunks():
                row = self._find_eid(c, b, eid)
                if row >= 0:
                    return self._materialize(c, row)
            return None
        return self._objects.get_event_by_id(id)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        return self._objects.list_command_responses_for_invocation(invocation_id, criteria)

    def list_events(self, event_type, index, entity_ids, criteria: DateRangeSearchCriteria | None = None):
        c = criteria or DateRangeSearchCriteria(page_size=100)
        et = _ETYPE.get(DeviceEventType(event_type))
        objs = self._objects.list_events(event_type, index, entity_ids, DateRangeSearchCriteria(page_size=0,
                                         start_date=c.start_date, end_date=c.end_date)).results
        if et is None:
            return SearchResults(len(objs), c.slice(objs))
        pos = _CTX[DeviceEventIndex(index)]
        want = set(entity_ids)
        with self._lock:
            asg_idx = np.array([i for i, ctx in self._asg.items() if ctx[pos] in want], np.int32)
        hits = []                                   # (date, chunk, row)
        for ci, ch in enumerate(self._all_chunks()):
            r = ch["rows"]
            m = (r["etype"] == et) & np.isin(r["assignment"], asg_idx)
            if c.start_date is not None:
                m &= r["event_date"] >= c.start_date
            if c.end_date is not None:
                m &= r["event_date"] <= c.end_date
            idx = np.nonzero(m)[0]
            if len(idx):
                hits.append((r["event_date"][idx], np.full(len(idx), ci, np.int32), idx, self._eids(ch, idx)))
        total = sum(len(h[0]) for h in hits) + len(objs)
        if not hits:
            return SearchResults(total, c.slice(objs))
        dates = np.concatenate([h[0] for h in hits])
        cis = np.concatenate([h[1] for h in hits])
        ris = np.concatenate([h[2] for h in hits])
        eids = np.concatenate([h[3] for h in hits])
        order = np.lexsort((-eids, -dates))         # newest first, then latest id
        chunks = self._all_chunks()
        if objs:
            merged = [self._materialize(chunks[cis[o]], int(ris[o])) for o in order] + objs
            merged.sort(key=lambda e: -(e.event_date or 0))
            return SearchResults(total, c.slice(merged))
        if c.page_size > 0:
            start = (max(1, c.page_number) - 1) * c.page_size
            order = order[start:start + c.page_size]
        return SearchResults(total, [self._materialize(chunks[cis[o]], int(ris[o])) for o in order])

    # ------------------------------------------------------------------ materialisation
    def _materialize(self, ch: dict, i: int):
        r = ch["rows"][i]
        ctx = self._asg.get(int(r["assignment"]), [None] * 5)
        base = dict(id=f"{self._boots[self._boot_of(ch, i)]}-{int(self._eids(ch, np.array([i]))[0])}",
                    device_assignment_id=ctx[0], device_id=ctx[1], customer_id=ctx[2], area_id=ctx[3],
                    asset_id=ctx[4], event_date=int(r["event_date"]), received_date=self._recv_of(ch, i))
        et = int(r["etype"])
        name = self._names.get(int(r["name_id"]), "") if int(r["name_id"]) != NO_NAME else ""
        if et == EV_MEASUREMENT:
            return DeviceMeasurement(name=name, value=float(r["v0"]), **base)
        if et == EV_LOCATION:
            return DeviceLocation(latitude=float(r["v0"]), longitude=float(r["v1"]), **base)
        if et == EV_ALERT:
            rule = self._rules.get(name)
            return DeviceAlert(source=AlertSource.System if rule is not None else AlertSource.Device,
                               level=_LEVELS[min(int(r["level"]), 3)], type=name, message=rule or "", **base)
        return DeviceStateChange(attribute="presence", type="presence", previous_state="PRESENT",
                                 new_state="NOT_PRESENT", **base)
