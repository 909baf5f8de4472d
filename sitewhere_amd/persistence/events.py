"""Device-event persistence backends for the event-management service.

Reference: ``service-event-management/.../persistence/**``:
  * MongoDB (``MongoDeviceEventManagement.java``) with the bulk ``DeviceEventBuffer``
    (10,000-entry queue, flush every 250 ms or 200 docs, ``DeviceEventBuffer.java:40-43, 99-135``)
  * Cassandra (``CassandraDeviceEventManagement.java``): 7 denormalised tables partitioned by
    ``(entity, event_type, bucket)`` clustered by ``event_date DESC`` (``:374-398, 419-495``)
  * InfluxDB (``InfluxDbDeviceEventManagement.java``): batched points (``InfluxDbClient.java:77``)
Here: :class:`MemoryEventStore` (indexed, bisect-sorted), :class:`SQLiteEventStore` (durable),
:class:`MongoEventStore` (the reference's MongoDB layout over the native wire client),
:class:`BucketedEventStore` (the Cassandra time-bucket layout, in memory), :class:`InfluxLineWriter`
(line protocol over HTTP, batched) and :class:`BufferedEventWriter` (the bulk buffer).  The GPU
engine's enriched rows are stored column-wise by :mod:`sitewhere_amd.persistence.columnar`.
"""
from __future__ import annotations

import bisect
import json
import logging
import queue
import sqlite3
import threading
import time
from collections import defaultdict

from ..models.domain import (DateRangeSearchCriteria, DeviceEvent, DeviceEventIndex, DeviceEventType, SearchResults,
                             event_from_dict)

_INDEX_FIELD = {
    DeviceEventIndex.Assignment: "device_assignment_id",
    DeviceEventIndex.Customer: "customer_id",
    DeviceEventIndex.Area: "area_id",
    DeviceEventIndex.Asset: "asset_id",
}


def _in_range(e: DeviceEvent, c: DateRangeSearchCriteria | None) -> bool:
    if c is None:
        return True
    d = e.event_date or 0
    if c.start_date is not None and d < c.start_date:
        return False
    if c.end_date is not None and d > c.end_date:
        return False
    return True


class DeviceEventStore:
    def add_events(self, events: list[DeviceEvent]) -> list[DeviceEvent]:
        raise NotImplementedError

    def get_event_by_id(self, id: str) -> DeviceEvent | None:
        raise NotImplementedError

    def get_event_by_alternate_id(self, alt: str) -> DeviceEvent | None:
        raise NotImplementedError

    def list_events(self, event_type: DeviceEventType, index: DeviceEventIndex, entity_ids: list[str],
                    criteria: DateRangeSearchCriteria | None = None) -> SearchResults:
        raise NotImplementedError

    def list_command_responses_for_invocation(self, invocation_id: str,
                                              criteria: DateRangeSearchCriteria | None = None) -> SearchResults:
        raise NotImplementedError

    def count(self) -> int:
        raise NotImplementedError


class MemoryEventStore(DeviceEventStore):
    def __init__(self):
        self._lock = threading.RLock()
        self._by_id: dict[str, DeviceEvent] = {}
        self._by_alt: dict[str, str] = {}
        # (event_type, index, entity_id) -> sorted list of (-date, seq, id)
        self._idx: dict[tuple, list] = defaultdict(list)
        self._resp: dict[str, list] = defaultdict(list)
        self._seq = 0

    def add_events(self, events):
        with self._lock:
            for e in events:
                self._by_id[e.id] = e
                if e.alternate_id:
                    self._by_alt[e.alternate_id] = e.id
                self._seq += 1
                key = (-(e.event_date or 0), self._seq, e.id)
                for ix, f in _INDEX_FIELD.items():
                    v = getattr(e, f)
                    if v:
                        bisect.insort(self._idx[(e.event_type, ix, v)], key)
                if e.event_type == DeviceEventType.CommandResponse and getattr(e, "originating_event_id", None):
                    bisect.insort(self._resp[e.originating_event_id], key)
        return events

    def get_event_by_id(self, id):
        with self._lock:
            return self._by_id.get(id)

    def get_event_by_alternate_id(self, alt):
        with self._lock:
            i = self._by_alt.get(alt)
            return self._by_id.get(i) if i else None

    def _collect(self, keys_lists, criteria):
        merged = sorted(set(k for lst in keys_lists for k in lst))
        with self._lock:
            evs = [self._by_id[k[2]] for k in merged]
        evs = [e for e in evs if _in_range(e, criteria)]
        c = criteria or DateRangeSearchCriteria()
        return SearchResults(len(evs), c.slice(evs))

    def list_events(self, event_type, index, entity_ids, criteria=None):
        with self._lock:
            lists = [list(self._idx.get((event_type, index, i), [])) for i in entity_ids]
        return self._collect(lists, criteria)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        with self._lock:
            lst = list(self._resp.get(invocation_id, []))
        return self._collect([lst], criteria)

    def count(self):
        with self._lock:
            return len(self._by_id)


class SQLiteEventStore(DeviceEventStore):
    def __init__(self, path: str = ":memory:"):
        self._lock = threading.RLock()
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("""CREATE TABLE IF NOT EXISTS events (id TEXT PRIMARY KEY, alt TEXT, type TEXT,
                            asg TEXT, cust TEXT, area TEXT, asset TEXT, orig TEXT, date INTEGER, doc TEXT)""")
        for c in ("alt", "orig"):
            self._db.execute(f"CREATE INDEX IF NOT EXISTS ev_{c} ON events({c})")
        for c in ("asg", "cust", "area", "asset"):
            self._db.execute(f"CREATE INDEX IF NOT EXISTS ev_{c} ON events(type, {c}, date DESC)")

    def add_events(self, events):
        rows = [(e.id, e.alternate_id, e.event_type.value, e.device_assignment_id, e.customer_id, e.area_id,
                 e.asset_id, getattr(e, "originating_event_id", None), e.event_date or 0, json.dumps(e.to_dict()))
                for e in events]
        with self._lock:
            self._db.execute("BEGIN")
            self._db.executemany("INSERT OR REPLACE INTO events VALUES (?,?,?,?,?,?,?,?,?,?)", rows)
            self._db.execute("COMMIT")
        return events

    def _one(self, where, arg):
        with self._lock:
            r = self._db.execute(f"SELECT doc FROM events WHERE {where}=?", (arg,)).fetchone()
        return event_from_dict(json.loads(r[0])) if r else None

    def get_event_by_id(self, id):
        return self._one("id", id)

    def get_event_by_alternate_id(self, alt):
        return self._one("alt", alt)

    def _search(self, where, args, criteria):
        c = criteria or DateRangeSearchCriteria()
        if c.start_date is not None:
            where += " AND date >= ?"
            args.append(c.start_date)
        if c.end_date is not None:
            where += " AND date <= ?"
            args.append(c.end_date)
        with self._lock:
            total = self._db.execute(f"SELECT COUNT(*) FROM events WHERE {where}", args).fetchone()[0]
            q = f"SELECT doc FROM events WHERE {where} ORDER BY date DESC"
            if c.page_size > 0:
                q += f" LIMIT {int(c.page_size)} OFFSET {int((max(1, c.page_number) - 1) * c.page_size)}"
            rows = self._db.execute(q, args).fetchall()
        return SearchResults(total, [event_from_dict(json.loads(r[0])) for r in rows])

    def list_events(self, event_type, index, entity_ids, criteria=None):
        col = {DeviceEventIndex.Assignment: "asg", DeviceEventIndex.Customer: "cust", DeviceEventIndex.Area: "area",
               DeviceEventIndex.Asset: "asset"}[index]
        if not entity_ids:
            return SearchResults(0, [])
        qs = ",".join("?" for _ in entity_ids)
        return self._search(f"type=? AND {col} IN ({qs})", [event_type.value, *entity_ids], criteria)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        return self._search("type=? AND orig=?", [DeviceEventType.CommandResponse.value, invocation_id], criteria)

    def count(self):
        with self._lock:
            return self._db.execute("SELECT COUNT(*) FROM events").fetchone()[0]


class MongoEventStore(DeviceEventStore):
    """The reference's MongoDB event layout (``MongoDeviceEventManagement.java``): one ``events``
    collection, one document per event (``_id`` = event id) with the index fields at top level,
    compound indexes (type, entity, date desc) per index, alternate-id and originating-event
    indexes.  Writes are bulk inserts (wrap in :class:`BufferedEventWriter` for the reference's
    200-document / 250 ms buffer).  Over the native wire client (``mongo_wire.py``)."""

    _FIELD = {DeviceEventIndex.Assignment: "deviceAssignmentId", DeviceEventIndex.Customer: "customerId",
              DeviceEventIndex.Area: "areaId", DeviceEventIndex.Asset: "assetId"}

    def __init__(self, uri: str = "mongodb://localhost:27017", database: str = "sitewhere", collection: str = "events"):
        from .mongo_wire import MongoClient
        self._client = MongoClient(uri)
        self._c = self._client[database][collection]
        for f in self._FIELD.values():
            self._c.create_index({"eventType": 1, f: 1, "eventDate": -1})
        self._c.create_index({"alternateId": 1}, sparse=True)
        self._c.create_index({"originatingEventId": 1}, sparse=True)

    def add_events(self, events):
        docs = []
        for e in events:
            d = e.to_dict()
            d["_id"] = e.id
            d["eventType"] = e.event_type.value
            d["eventDate"] = e.event_date or 0
            docs.append(d)
        if docs:
            self._c.bulk_replace(docs)
        return events

    @staticmethod
    def _load(d):
        if d is None:
            return None
        d = dict(d)
        d.pop("_id", None)
        return event_from_dict(d)

    def get_event_by_id(self, id):
        return self._load(self._c.find_one({"_id": id}))

    def get_event_by_alternate_id(self, alt):
        return self._load(self._c.find_one({"alternateId": alt}))

    def _search(self, flt, criteria):
        c = criteria or DateRangeSearchCriteria()
        rng = {}
        if c.start_date is not None:
            rng["$gte"] = c.start_date
        if c.end_date is not None:
            rng["$lte"] = c.end_date
        if rng:
            flt["eventDate"] = rng
        total = self._c.count_documents(flt)
        skip = (max(1, c.page_number) - 1) * c.page_size if c.page_size > 0 else 0
        docs = self._c.find(flt, sort={"eventDate": -1}, skip=skip, limit=c.page_size if c.page_size > 0 else 0)
        return SearchResults(total, [self._load(d) for d in docs])

    def list_events(self, event_type, index, entity_ids, criteria=None):
        if not entity_ids:
            return SearchResults(0, [])
        return self._search({"eventType": event_type.value, self._FIELD[index]: {"$in": list(entity_ids)}}, criteria)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        return self._search({"eventType": DeviceEventType.CommandResponse.value,
                             "originatingEventId": invocation_id}, criteria)

    def count(self):
        return self._c.count_documents({})


class CassandraEventStore(DeviceEventStore):
    """Events in Cassandra over the native CQL client (``persistence/cql_wire.py``), in the
    reference's denormalised layout (``CassandraEventManagementClient.java:138-160``): one table per
    index partitioned by ``(entity, event_type, bucket)`` and clustered by ``event_date DESC``,
    plus ``events_by_id`` / ``events_by_alt_id``; the bucket is ``event_date // bucket_ms``
    (``CassandraDeviceEventManagement.getBucketValue``).  Event bodies are stored as JSON documents
    (the reference uses frozen UDTs per event type).  ``event_buckets`` lists the buckets written per
    entity so unbounded ranges know which partitions to read."""

    _IDX = {DeviceEventIndex.Assignment: ("events_by_assignment", "assignment_id", 0),
            DeviceEventIndex.Customer: ("events_by_customer", "customer_id", 1),
            DeviceEventIndex.Area: ("events_by_area", "area_id", 2),
            DeviceEventIndex.Asset: ("events_by_asset", "asset_id", 3)}
    _TYPES = [t for t in DeviceEventType]

    def __init__(self, address: str = "127.0.0.1:9042", keyspace: str = "sitewhere", bucket_ms: int = 3600_000,
                 username: str | None = None, password: str | None = None):
        from .cql_wire import CqlSession
        self.bucket_ms = int(bucket_ms)
        self.s = CqlSession(address, None, username, password)
        keyspace = "".join(ch if ch.isalnum() else "_" for ch in keyspace).lower()
        self.ks = keyspace
        self._lock = threading.RLock()
        self.s.execute(f"CREATE KEYSPACE IF NOT EXISTS {keyspace} WITH replication = "
                       "{'class': 'SimpleStrategy', 'replication_factor': 1}")
        self.s.execute(f"USE {keyspace}")
        self.s.execute("CREATE TABLE IF NOT EXISTS events_by_id (event_id text PRIMARY KEY, event_type tinyint, "
                       "doc text)")
        self.s.execute("CREATE TABLE IF NOT EXISTS events_by_alt_id (alt_id text PRIMARY KEY, event_id text, doc text)")
        for table, col, _ in self._IDX.values():
            self.s.execute(f"CREATE TABLE IF NOT EXISTS {table} ({col} text, event_type tinyint, bucket int, "
                           f"event_date timestamp, event_id text, doc text, PRIMARY KEY (({col}, event_type, bucket), "
                           "event_date, event_id)) WITH CLUSTERING ORDER BY (event_date DESC, event_id ASC)")
        self.s.execute("CREATE TABLE IF NOT EXISTS responses_by_invocation (orig_id text, event_date timestamp, "
                       "event_id text, doc text, PRIMARY KEY ((orig_id), event_date, event_id)) "
                       "WITH CLUSTERING ORDER BY (event_date DESC, event_id ASC)")
        self.s.execute("CREATE TABLE IF NOT EXISTS event_buckets (entity_id text, index_kind tinyint, "
                       "event_type tinyint, bucket int, PRIMARY KEY ((entity_id, index_kind, event_type), bucket)) "
                       "WITH CLUSTERING ORDER BY (bucket DESC)")
        self.s.execute("CREATE TABLE IF NOT EXISTS event_counts (k text PRIMARY KEY, n bigint)")

    def bucket_of(self, date_ms: int) -> int:
        return int(date_ms) // self.bucket_ms

    def _tcode(self, et) -> int:
        return self._TYPES.index(et)

    def add_events(self, events):
        with self._lock:
            for e in events:
                doc = json.dumps(e.to_dict(), separators=(",", ":"))
                d = int(e.event_date or 0)
                b = self.bucket_of(d)
                tc = self._tcode(e.event_type)
                new = not self.s.execute("SELECT event_id FROM events_by_id WHERE event_id = ?", [e.id])
                self.s.execute("INSERT INTO events_by_id (event_id, event_type, doc) VALUES (?, ?, ?)", [e.id, tc, doc])
                if e.alternate_id:
                    self.s.execute("INSERT INTO events_by_alt_id (alt_id, event_id, doc) VALUES (?, ?, ?)",
                                   [e.alternate_id, e.id, doc])
                for idx, (table, col, kind) in self._IDX.items():
                    ent = getattr(e, _INDEX_FIELD[idx])
                    if not ent:
                        continue
                    self.s.execute(f"INSERT INTO {table} ({col}, event_type, bucket, event_date, event_id, doc) "
                                   "VALUES (?, ?, ?, ?, ?, ?)", [ent, tc, b, d, e.id, doc])
                    self.s.execute("INSERT INTO event_buckets (entity_id, index_kind, event_type, bucket) "
                                   "VALUES (?, ?, ?, ?)", [ent, kind, tc, b])
                orig = getattr(e, "originating_event_id", None)
                if orig and e.event_type == DeviceEventType.CommandResponse:
                    self.s.execute("INSERT INTO responses_by_invocation (orig_id, event_date, event_id, doc) "
                                   "VALUES (?, ?, ?, ?)", [orig, d, e.id, doc])
                if new:
                    cur = self.s.execute("SELECT n FROM event_counts WHERE k = ?", ["events"])
                    self.s.execute("INSERT INTO event_counts (k, n) VALUES (?, ?)",
                                   ["events", (cur[0]["n"] if cur else 0) + 1])
        return events

    def get_event_by_id(self, id):
        r = self.s.execute("SELECT doc FROM events_by_id WHERE event_id = ?", [id])
        return event_from_dict(json.loads(r[0]["doc"])) if r else None

    def get_event_by_alternate_id(self, alt):
        r = self.s.execute("SELECT doc FROM events_by_alt_id WHERE alt_id = ?", [alt])
        return event_from_dict(json.loads(r[0]["doc"])) if r else None

    @staticmethod
    def _page(rows, c):
        rows.sort(key=lambda r: (-r["event_date"], r["event_id"]))
        total = len(rows)
        if c.page_size > 0:
            lo = (max(1, c.page_number) - 1) * c.page_size
            rows = rows[lo:lo + c.page_size]
        return SearchResults(total, [event_from_dict(json.loads(r["doc"])) for r in rows])

    def list_events(self, event_type, index, entity_ids, criteria=None):
        c = criteria or DateRangeSearchCriteria()
        table, col, kind = self._IDX[index]
        tc = self._tcode(event_type)
        lo = c.start_date if c.start_date is not None else -(1 << 62)
        hi = c.end_date if c.end_date is not None else (1 << 62)
        blo = max(self.bucket_of(max(lo, -(1 << 50))), -(1 << 31))
        bhi = min(self.bucket_of(min(hi, 1 << 50)), (1 << 31) - 1)
        rows = []
        for ent in entity_ids:
            buckets = self.s.execute("SELECT bucket FROM event_buckets WHERE entity_id = ? AND index_kind = ? AND "
                                     "event_type = ? AND bucket >= ? AND bucket <= ?", [ent, kind, tc, blo, bhi])
            for bk in buckets:                    # newest bucket first (clustering order)
                rows += self.s.execute(f"SELECT event_date, event_id, doc FROM {table} WHERE {col} = ? AND "
                                       "event_type = ? AND bucket = ? AND event_date >= ? AND event_date <= ?",
                                       [ent, tc, bk["bucket"], lo, hi])
        return self._page(rows, c)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        rows = self.s.execute("SELECT event_date, event_id, doc FROM responses_by_invocation WHERE orig_id = ?",
                              [invocation_id])
        return self._page(rows, criteria or DateRangeSearchCriteria())

    def count(self):
        r = self.s.execute("SELECT n FROM event_counts WHERE k = ?", ["events"])
        return int(r[0]["n"]) if r else 0


class BucketedEventStore(DeviceEventStore):
    """Cassandra layout: partition = (entity, event type, time bucket); rows clustered by date DESC.

    Range queries walk buckets newest-first and stop once the page is full, exactly like the
    reference's bucketed CQL reads (``CassandraDeviceEventManagement.java:419-495``).
    """

    def __init__(self, bucket_ms: int = 60 * 60 * 1000):
        self.bucket_ms = bucket_ms
        self._lock = threading.RLock()
        self._parts: dict[tuple, list] = defaultdict(list)        # (ix, entity, type, bucket) -> [(-date, id)]
        self._buckets: dict[tuple, list] = defaultdict(list)      # (ix, entity, type) -> sorted buckets
        self._by_id: dict[str, DeviceEvent] = {}
        self._by_alt: dict[str, str] = {}
        self._resp: dict[str, list] = defaultdict(list)

    def bucket_of(self, date_ms: int) -> int:
        return int(date_ms // self.bucket_ms)

    def add_events(self, events):
        with self._lock:
            for e in events:
                self._by_id[e.id] = e
                if e.alternate_id:
                    self._by_alt[e.alternate_id] = e.id
                d = e.event_date or 0
                b = self.bucket_of(d)
                for ix, f in _INDEX_FIELD.items():
                    v = getattr(e, f)
                    if not v:
                        continue
                    pk = (ix, v, e.event_type)
                    bl = self._buckets[pk]
                    j = bisect.bisect_left(bl, b)
                    if j == len(bl) or bl[j] != b:
                        bl.insert(j, b)
                    bisect.insort(self._parts[pk + (b,)], (-d, e.id))
                if e.event_type == DeviceEventType.CommandResponse and getattr(e, "originating_event_id", None):
                    bisect.insort(self._resp[e.originating_event_id], (-d, e.id))
        return events

    def get_event_by_id(self, id):
        return self._by_id.get(id)

    def get_event_by_alternate_id(self, alt):
        i = self._by_alt.get(alt)
        return self._by_id.get(i) if i else None

    def list_events(self, event_type, index, entity_ids, criteria=None):
        c = criteria or DateRangeSearchCriteria()
        rows = []
        with self._lock:
            for ent in entity_ids:
                pk = (index, ent, event_type)
                for b in reversed(self._buckets.get(pk, [])):
                    if c.end_date is not None and b * self.bucket_ms > c.end_date:
                        continue
                    if c.start_date is not None and (b + 1) * self.bucket_ms <= c.start_date:
                        break
                    rows.extend(self._parts[pk + (b,)])
        rows.sort()
        evs = [self._by_id[i] for _, i in rows]
        evs = [e for e in evs if _in_range(e, c)]
        return SearchResults(len(evs), c.slice(evs))

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        c = criteria or DateRangeSearchCriteria()
        evs = [self._by_id[i] for _, i in self._resp.get(invocation_id, [])]
        return SearchResults(len(evs), c.slice(evs))

    def count(self):
        return len(self._by_id)


class BufferedEventWriter:
    """Bulk write buffer in front of any store (reference DeviceEventBuffer: queue 10,000,
    flush at 200 docs or every 250 ms).  ``add`` blocks when the queue is full (back-pressure).

    A failed bulk write is retried with backoff (0.05 s doubling to 2 s) until it succeeds -- the
    events stay buffered, never dropped, while the store is unavailable.  Buffered events are
    indexed by alternate id (``pending_alternate``) so a redelivery arriving before the flush is
    still deduplicated."""

    def __init__(self, store: DeviceEventStore, max_queue: int = 10_000, chunk: int = 200, interval_ms: int = 250):
        self.store, self.chunk, self.interval = store, chunk, interval_ms / 1000.0
        self.q: queue.Queue = queue.Queue(max_queue)
        self._stop = threading.Event()
        self._pending: dict = {}
        self._plock = threading.Lock()
        self._t = threading.Thread(target=self._run, daemon=True, name="event-buffer")
        self.flushes = 0
        self.failed_writes = 0
        self._t.start()

    def add(self, events):
        with self._plock:
            for e in events:
                if e.alternate_id:
                    self._pending[e.alternate_id] = e
        for e in events:
            self.q.put(e)

    def pending_alternate(self, alt: str):
        with self._plock:
            return self._pending.get(alt)

    def _write(self, buf):
        backoff = 0.05
        while True:
            try:
                self.store.add_events(buf)
                break
            except Exception:
                self.failed_writes += 1
                if self._stop.is_set() and backoff >= 2.0:
                    logging.getLogger(__name__).exception("dropping %d buffered events at shutdown", len(buf))
                    break
                logging.getLogger(__name__).warning("bulk write of %d events failed; retrying in %.2fs",
                                                    len(buf), backoff, exc_info=True)
                time.sleep(backoff)
                backoff = min(2.0, backoff * 2)
        self.flushes += 1
        with self._plock:
            for e in buf:
                if e.alternate_id and self._pending.get(e.alternate_id) is e:
                    del self._pending[e.alternate_id]

    def _run(self):
        buf = []
        last = time.time()
        while not self._stop.is_set() or not self.q.empty():
            try:
                buf.append(self.q.get(timeout=self.interval / 4))
            except queue.Empty:
                pass
            if buf and (len(buf) >= self.chunk or time.time() - last >= self.interval):
                self._write(buf)
                buf = []
                last = time.time()
        if buf:
            self._write(buf)

    def flush(self, timeout: float = 5.0):
        end = time.time() + timeout
        while (not self.q.empty() or self._pending) and time.time() < end:
            time.sleep(0.01)
        time.sleep(self.interval * 1.5)

    def close(self):
        self._stop.set()
        self._t.join(timeout=5)


class InfluxLineWriter:
    """InfluxDB line-protocol writer with batching (reference InfluxDbClient enableBatch)."""

    def __init__(self, url: str, database: str = "sitewhere", batch: int = 1000, post=None):
        self.url = url.rstrip("/") + f"/write?db={database}&precision=ms"
        self.batch = batch
        self.buf: list[str] = []
        self._post = post
        self.sent = 0

    @staticmethod
    def _esc(s: str) -> str:
        return str(s).replace(" ", r"\ ").replace(",", r"\,").replace("=", r"\=")

    @staticmethod
    def _str_field(v: str) -> str:
        return '"' + str(v).replace("\\", "\\\\").replace('"', '\\"') + '"'

    def line(self, e: DeviceEvent) -> str:
        tags = {"type": e.event_type.value, "assignment": e.device_assignment_id or "", "device": e.device_id or "",
                "customer": e.customer_id or "", "area": e.area_id or "", "asset": e.asset_id or ""}
        fields = {"eid": f'"{e.id}"'}
        if e.alternate_id:
            fields["alt"] = self._str_field(e.alternate_id)
        orig = getattr(e, "originating_event_id", None)
        if orig:
            fields["orig"] = self._str_field(orig)
        fields["doc"] = self._str_field(json.dumps(e.to_dict(), separators=(",", ":")))
        if e.event_type == DeviceEventType.Measurement:
            fields[f"mx_{self._esc(e.name)}"] = repr(float(e.value))
        elif e.event_type == DeviceEventType.Location:
            fields.update(latitude=repr(e.latitude), longitude=repr(e.longitude))
        elif e.event_type == DeviceEventType.Alert:
            fields.update(alertType=f'"{e.type}"', alertLevel=f'"{e.level.value}"',
                          message=json.dumps(e.message))
        tag_s = ",".join(f"{k}={self._esc(v)}" for k, v in tags.items() if v)
        field_s = ",".join(f"{k}={v}" for k, v in fields.items())
        return f"events,{tag_s} {field_s} {int(e.event_date or 0)}"

    def add_events(self, events):
        self.buf.extend(self.line(e) for e in events)
        if len(self.buf) >= self.batch:
            self.flush()
        return events

    def flush(self):
        if not self.buf:
            return
        body = "\n".join(self.buf).encode()
        if self._post is not None:
            self._post(self.url, body)
        else:
            import urllib.request
            urllib.request.urlopen(urllib.request.Request(self.url, data=body, method="POST"), timeout=10).read()
        self.sent += len(self.buf)
        self.buf = []


class InfluxEventStore(DeviceEventStore):
    """Events in InfluxDB, the reference's layout (``InfluxDbDeviceEvent.java``): measurement
    ``events``, tags type/assignment/device/customer/area/asset, field ``eid``; written in batched
    line protocol (:class:`InfluxLineWriter`) and read back with the reference's InfluxQL queries
    (``SELECT * FROM events WHERE type='..' AND (assignment='..' OR ..) AND time >= .. ORDER BY time
    DESC LIMIT .. OFFSET ..`` and ``SELECT count(eid) ...``) over the HTTP ``/query`` API.  Each point
    also carries the full event document (``doc``) so reads are lossless."""

    _TAG = {DeviceEventIndex.Assignment: "assignment", DeviceEventIndex.Customer: "customer",
            DeviceEventIndex.Area: "area", DeviceEventIndex.Asset: "asset"}

    def __init__(self, url: str = "http://localhost:8086", database: str = "sitewhere", batch: int = 1000, http=None):
        self.base, self.database = url.rstrip("/"), database
        self._http = http
        self.writer = InfluxLineWriter(self.base, database, batch, post=self._post if http else None)
        self._lock = threading.RLock()
        self.query_raw(f"CREATE DATABASE {database}", db=None)

    def _post(self, url, body):
        return self._http("POST", url, body)

    def query_raw(self, q: str, db: str | None = "") -> list:
        import urllib.parse
        import urllib.request
        params = {"q": q, "epoch": "ms"}
        if db is not None:
            params["db"] = db or self.database
        url = f"{self.base}/query?{urllib.parse.urlencode(params)}"
        if self._http:
            body = self._http("POST" if q.upper().startswith("CREATE") else "GET", url, None)
        else:
            req = urllib.request.Request(url, method="POST" if q.upper().startswith("CREATE") else "GET")
            body = urllib.request.urlopen(req, timeout=10).read()
        res = json.loads(body)["results"][0]
        if "error" in res:
            raise RuntimeError(f"influxdb: {res['error']}")
        return res.get("series", [])

    @staticmethod
    def _q(v) -> str:
        return "'" + str(v).replace("\\", "\\\\").replace("'", "\\'") + "'"

    def add_events(self, events):
        with self._lock:
            self.writer.add_events(events)
            self.writer.flush()                  # the buffered writer batches upstream
        return events

    def _rows(self, series) -> list:
        out = []
        for s in series:
            cols = s["columns"]
            for v in s.get("values", []):
                d = dict(zip(cols, v))
                if d.get("doc"):
                    out.append(event_from_dict(json.loads(d["doc"])))
        return out

    def _one(self, where: str):
        r = self._rows(self.query_raw(f"SELECT * FROM events WHERE {where} LIMIT 1"))
        return r[0] if r else None

    def get_event_by_id(self, id):
        return self._one(f"eid={self._q(id)}")

    def get_event_by_alternate_id(self, alt):
        return self._one(f"alt={self._q(alt)}")

    def _search(self, where: str, criteria):
        c = criteria or DateRangeSearchCriteria()
        if c.start_date is not None:
            where += f" AND time >= {int(c.start_date)}ms"
        if c.end_date is not None:
            where += f" AND time <= {int(c.end_date)}ms"
        cnt = self.query_raw(f"SELECT count(eid) FROM events WHERE {where}")
        total = int(cnt[0]["values"][0][1]) if cnt and cnt[0].get("values") else 0
        q = f"SELECT * FROM events WHERE {where} ORDER BY time DESC"
        if c.page_size > 0:
            q += f" LIMIT {int(c.page_size)} OFFSET {int((max(1, c.page_number) - 1) * c.page_size)}"
        return SearchResults(total, self._rows(self.query_raw(q)))

    def list_events(self, event_type, index, entity_ids, criteria=None):
        if not entity_ids:
            return SearchResults(0, [])
        tag = self._TAG[index]
        ors = " OR ".join(f"{tag}={self._q(i)}" for i in entity_ids)
        return self._search(f"type={self._q(event_type.value)} AND ({ors})", criteria)

    def list_command_responses_for_invocation(self, invocation_id, criteria=None):
        return self._search(f"type={self._q(DeviceEventType.CommandResponse.value)} AND orig={self._q(invocation_id)}",
                            criteria)

    def count(self):
        cnt = self.query_raw("SELECT count(eid) FROM events")
        return int(cnt[0]["values"][0][1]) if cnt and cnt[0].get("values") else 0


def create_event_store(kind: str = "memory", **kw) -> DeviceEventStore:
    kind = (kind or "memory").lower()
    if kind == "memory":
        return MemoryEventStore()
    if kind == "sqlite":
        return SQLiteEventStore(kw.get("path", ":memory:"))
    if kind == "cassandra" and kw.get("address"):
        return CassandraEventStore(kw["address"], kw.get("keyspace", "sitewhere"), kw.get("bucket_ms", 3600_000),
                                   kw.get("username"), kw.get("password"))
    if kind in ("cassandra", "bucketed"):
        return BucketedEventStore(kw.get("bucket_ms", 3600_000))
    if kind == "columnar":
        from .columnar import ColumnarEventStore
        return ColumnarEventStore(retention_rows=kw.get("retentionRows"))
    if kind in ("segments", "durable"):
        # durable columnar segments of engine tenants (persistence/segments.py)
        from .segments import DurableEventStore
        return DurableEventStore(kw.get("path", "/tmp/sitewhere/segments"), int(kw.get("rank", 0)),
                                 rotate_bytes=int(kw.get("rotateBytes", 1 << 30)),
                                 retention_bytes=int(kw.get("retentionBytes", 0)),
                                 direct=bool(kw.get("directIo", True)))
    if kind in ("mongo", "mongodb"):
        return MongoEventStore(kw.get("uri", "mongodb://localhost:27017"), kw.get("database", "sitewhere"))
    if kind == "influxdb":
        return InfluxEventStore(kw.get("url", "http://localhost:8086"), kw.get("database", "sitewhere"))
    raise ValueError(f"unknown event store {kind!r}")
