"""Event bus over the native partitioned commit log (the Kafka data plane, rebuilt).

Reference behaviour reproduced:
  * keyed records, Kafka-compatible murmur2 partitioning (records for one device token stay
    ordered on one partition) -- ``MicroserviceKafkaProducer.java:89-107``
  * consumer groups with partition assignment and rebalance on join/leave, manual offset
    commits (``enable.auto.commit=false``), at-least-once ``commitAsync`` after processing --
    ``MicroserviceKafkaConsumer.java:53-133``, ``DirectKafkaConsumer.java:28-41``
  * independent groups each see the full stream (fan-out: state / rules / connectors)
  * durable logs + committed offsets survive restarts (``SURVEY §5.4``)
The storage engine is ``libswnative``'s ``swlog_*`` (C++, CRC-checked append-only segments,
torn-tail recovery).  Topics are auto-created on first use, as the reference relied on broker
auto-creation.
"""
from __future__ import annotations

import ctypes
import os
import itertools
import struct
import threading
import time
import uuid
from dataclasses import dataclass

import numpy as np

from .._native import native, native_gil

_FRAME = struct.Struct("<qqII")


def murmur2(data: bytes) -> int:
    """Kafka's murmur2 (``Utils.murmur2``, seed 0x9747b28c) -- same values as the native sw_murmur2."""
    m, r = 0x5BD1E995, 24
    length = len(data)
    h = (0x9747B28C ^ length) & 0xFFFFFFFF
    n4 = length & ~3
    for i in range(0, n4, 4):
        k = data[i] | (data[i + 1] << 8) | (data[i + 2] << 16) | (data[i + 3] << 24)
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> r
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    rem = length & 3
    if rem == 3:
        h ^= data[n4 + 2] << 16
    if rem >= 2:
        h ^= data[n4 + 1] << 8
    if rem >= 1:
        h ^= data[n4]
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h


_PART_CACHE: dict = {}


def kafka_partition(key: bytes, n: int) -> int:
    """``toPositive(murmur2(key)) % n`` with a bounded memo (device tokens repeat)."""
    ck = (key, n)
    p = _PART_CACHE.get(ck)
    if p is None:
        if len(_PART_CACHE) > 200_000:
            _PART_CACHE.clear()
        p = _PART_CACHE[ck] = (murmur2(key) & 0x7FFFFFFF) % n
    return p


def parse_frames(name: str, partition: int, n: int, raw: bytes) -> list:
    """Framed records (``EventBus.read_framed``) -> Record objects."""
    out, pos = [], 0
    for _ in range(n):
        off, ts, kl, vl = _FRAME.unpack_from(raw, pos)
        pos += _FRAME.size
        key = raw[pos:pos + kl] if kl else None
        pos += kl
        out.append(Record(name, partition, off, key, raw[pos:pos + vl], ts))
        pos += vl
    return out


@dataclass
class Record:
    topic: str
    partition: int
    offset: int
    key: bytes | None
    value: bytes
    timestamp: int


class _Group:
    def __init__(self):
        self.members: dict[str, tuple] = {}   # member_id -> (topics tuple, last heartbeat)
        self.generation = 0
        self.assignment: dict[str, list[tuple[str, int]]] = {}


class BackpressureTimeout(RuntimeError):
    """A producer waited too long for a protected topic's consumer (see :meth:`EventBus.protect`)."""


class EventBus:
    """In-process broker: topics, partitions, consumer-group coordinator, committed offsets."""

    def __init__(self, directory: str | None = None, default_partitions: int = 8, fsync: bool = False,
                 session_timeout_s: float = 30.0, retention_bytes: int | None = None):
        self.lib = native()
        self.h = self.lib.swlog_open(directory.encode() if directory else None, 1 if fsync else 0)
        # microsecond calls keep the GIL (PyDLL); opening, flushing and closing go through CDLL
        self.fast = native_gil() if not fsync else self.lib
        self._tls = threading.local()
        # memory-only logs keep at most this many bytes per partition (Kafka retention.bytes);
        # lagging consumers resume at the oldest retained offset.  Durable logs keep everything.
        if retention_bytes is None:
            retention_bytes = 0 if directory else (1 << 30)
        self.lib.swlog_set_retention(self.h, -1, int(retention_bytes))
        self._ret_default = int(retention_bytes)
        self._ret_topic: dict[str, int] = {}
        # protected topics (protect): consumer group -> longest a producer waits for room
        self._protected: dict[str, dict[str, float]] = {}
        self._room = threading.Condition(threading.Lock())
        self.backpressure_waits = 0
        self.directory = directory
        # identity of this log's offsets: a memory-only log starts over at offset 0 each time, so
        # offsets recorded elsewhere (durable commit records) are scoped by it
        self.incarnation = self._incarnation(directory)
        self.default_partitions = default_partitions
        self.session_timeout_s = session_timeout_s
        self._topics: dict[str, int] = {}
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self._groups: dict[str, _Group] = {}
        self._nparts: dict[str, int] = {}
        self._waiters: dict[str, set] = {}       # topic -> Events of consumers subscribed to it
        self._ext: dict[int, object] = {}        # zero-copy record id -> buffer owner (kept alive)
        self._ext_ids = itertools.count()
        self._holds: dict[tuple[str, int], dict] = {}
        self._closed = False

    # ------------------------------------------------------------------ topics
    def topic(self, name: str, partitions: int | None = None) -> int:
        t = self._topics.get(name)            # hot path: no lock once the topic exists
        if t is not None:
            return t
        with self._lock:
            t = self._topics.get(name)
            if t is None:
                t = self.fast.swlog_topic(self.h, name.encode(), partitions or self.default_partitions)
                self._topics[name] = t
            return t

    def partitions(self, name: str) -> int:
        n = self._nparts.get(name)
        if n is None:
            n = self._nparts[name] = self.fast.swlog_partitions(self.h, self.topic(name))
        return n

    @staticmethod
    def _incarnation(directory: str | None) -> str:
        import uuid
        if not directory:
            return uuid.uuid4().hex
        path = os.path.join(directory, "bus.id")
        try:
            with open(path) as f:
                return f.read().strip()
        except FileNotFoundError:
            os.makedirs(directory, exist_ok=True)
            ident = uuid.uuid4().hex
            tmp = path + ".tmp"
            with open(tmp, "w") as f:
                f.write(ident)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, path)
            return ident

    def topics(self) -> list[str]:
        with self._lock:
            return sorted(self._topics)

    def end_offset(self, name: str, partition: int) -> int:
        return self.fast.swlog_end_offset(self.h, self.topic(name), partition)

    def begin_offset(self, name: str, partition: int) -> int:
        return self.fast.swlog_begin_offset(self.h, self.topic(name), partition)

    def partition_for(self, name: str, key: bytes | None) -> int:
        n = self.partitions(name)
        if key is None:
            return next(self._rr) % n
        return kafka_partition(bytes(key), n)

    _rr = itertools.count()

    # ------------------------------------------------------------------ produce
    def append(self, name: str, partition: int, records: list[tuple[bytes | None, bytes]], ts: int | None = None) -> int:
        if not records:
            return -1
        if name in self._protected:
            self._await_room(name, partition, sum(len(v) + len(k or b"") for k, v in records))
        t = self.topic(name)
        if len(records) == 1:
            k, v = records[0]
            k = k or b""
            first = self.fast.swlog_append(self.h, t, partition, k, len(k), v, len(v),
                                          ts if ts is not None else int(time.time() * 1000))
            if first < 0:
                raise RuntimeError(f"append to {name}[{partition}] failed")
            self._wake(name)
            return first
        keys = [k or b"" for k, _ in records]
        vals = [v for _, v in records]
        koff = np.zeros(len(records) + 1, np.int64)
        koff[1:] = np.cumsum([len(k) for k in keys])
        voff = np.zeros(len(records) + 1, np.int64)
        voff[1:] = np.cumsum([len(v) for v in vals])
        kb = np.frombuffer(b"".join(keys) + b"\0", np.uint8)
        vb = np.frombuffer(b"".join(vals) + b"\0", np.uint8)
        tsa = np.full(len(records), ts if ts is not None else int(time.time() * 1000), np.int64)
        first = self.fast.swlog_append_batch(self.h, t, partition, kb.ctypes.data, koff.ctypes.data, vb.ctypes.data,
                                            voff.ctypes.data, tsa.ctypes.data, len(records))
        if first < 0:
            raise RuntimeError(f"append to {name}[{partition}] failed")
        self._wake(name)
        return first

    # ------------------------------------------------------------------ zero-copy records
    def append_external(self, name: str, partition: int, owner, ptr: int, nbytes: int, key_len: int = 0,
                        ts: int | None = None, on_release=None) -> int:
        """Publish a record whose bytes already sit in caller memory, without copying them.

        ``ptr`` points at ``nbytes`` bytes: the key (``key_len`` bytes, usually none) then the value.
        The log references them in place, so consumers that read the record in place see that
        memory (pinned host memory lets an MI355X consumer DMA it straight from the topic).
        ``owner`` (the object owning the bytes: a pinned tensor, a ``bytes`` object, ...) is kept
        alive, and must not change, until retention drops the record; then ``on_release(owner)`` is
        called (a buffer pool takes it back) or, without a callback, the reference is dropped.
        A durable partition (files) copies the record instead and releases ``owner`` at once."""
        if name in self._protected:
            self._await_room(name, partition, int(nbytes))
        self._drain_released()
        ext = next(self._ext_ids)
        with self._lock:
            self._ext[ext] = (owner, on_release)
        first = self.fast.swlog_append_external(self.h, self.topic(name), partition, ptr, int(nbytes), int(key_len),
                                               ts if ts is not None else int(time.time() * 1000), ext)
        if first == -2:                 # durable partition: the record goes to its files (a copy)
            with self._lock:
                self._ext.pop(ext, None)
            raw = ctypes.string_at(ptr, int(nbytes))
            first = self.append(name, partition, [(raw[:key_len] or None, raw[key_len:])], ts=ts)
            if on_release is not None:
                on_release(owner)
            return first
        if first < 0:
            with self._lock:
                self._ext.pop(ext, None)
            raise RuntimeError(f"zero-copy append to {name}[{partition}] failed ({first})")
        self._wake(name)
        return first

    def append_bytes(self, name: str, partition: int, value: bytes, ts: int | None = None) -> int:
        """Publish an immutable ``bytes`` value by reference (no copy into the log)."""
        addr = ctypes.cast(ctypes.c_char_p(value), ctypes.c_void_p).value
        return self.append_external(name, partition, value, addr, len(value), ts=ts)

    def view(self, name: str, partition: int, offset: int):
        """(address, length, timestamp) of a retained record's value, read in place, or None.  The
        address stays valid while the record is retained; DMA readers :meth:`hold` it first."""
        ptr, n, ts = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        if self.fast.swlog_view(self.h, self.topic(name), partition, offset, ctypes.byref(ptr), ctypes.byref(n),
                                ctypes.byref(ts)):
            return None
        return ptr.value, n.value, ts.value

    def hold(self, name: str, partition: int, offset: int | None, holder=None):
        """Retention keeps every record at or after ``offset`` (None releases the hold).  Each
        ``holder`` (e.g. one zero-copy consumer) has its own hold; the partition honours the lowest."""
        with self._lock:
            hs = self._holds.setdefault((name, partition), {})
            if offset is None:
                hs.pop(holder, None)
            else:
                hs[holder] = int(offset)
            low = min(hs.values()) if hs else (1 << 63) - 1
            self.fast.swlog_hold(self.h, self.topic(name), partition, low)

    def _drain_released(self) -> list:
        """Hand zero-copy records that retention dropped back to their owners' ``on_release``;
        returns the owners that had none (their references are dropped once the caller lets go)."""
        # a scratch array per call: the event-source flush thread and the tenant store thread both
        # append externally, and a shared array could be overwritten between the native take and
        # the read below -- those owners would never be released
        ids = np.zeros(256, np.int64)
        out = []
        while True:
            n = self.fast.swlog_take_released(self.h, ids.ctypes.data, len(ids))
            if n:
                with self._lock:
                    got = [self._ext.pop(int(i), None) for i in ids[:n]]
                for e in got:
                    if e is None:
                        continue
                    if e[1] is not None:
                        e[1](e[0])
                    else:
                        out.append(e[0])
            if n < len(ids):
                return out

    def reclaim(self) -> list:
        """Release what retention dropped (see :meth:`append_external`); returns the owners that
        registered no ``on_release``."""
        return self._drain_released()

    def read_views(self, name: str, partition: int, offset: int, max_records: int = 500) -> list:
        """Like :meth:`read` but zero-copy: each record's ``value`` is a read-only memoryview of the
        log's own memory (keys are not returned).  A view is valid while the record is retained --
        take a :meth:`hold` at ``offset`` before reading and release it when done."""
        t = self.topic(name)
        end = self.fast.swlog_end_offset(self.h, t, partition)
        out = []
        ptr, n, ts = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        for off in range(max(offset, self.fast.swlog_begin_offset(self.h, t, partition)),
                         min(end, offset + max_records)):
            if self.fast.swlog_view(self.h, t, partition, off, ctypes.byref(ptr), ctypes.byref(n), ctypes.byref(ts)):
                continue
            mv = memoryview((ctypes.c_uint8 * n.value).from_address(ptr.value)).cast("B").toreadonly() \
                if n.value else memoryview(b"")
            out.append(Record(name, partition, off, None, mv, ts.value))
        return out

    # ------------------------------------------------------------------ fetch
    def read(self, name: str, partition: int, offset: int, max_records: int = 500, max_bytes: int = 1 << 20):
        t = self.topic(name)
        if offset >= self.fast.swlog_end_offset(self.h, t, partition):
            return []                                   # nothing new: no buffer, no copy
        buf = getattr(self._tls, "buf", None)           # per-thread fetch buffer, reused
        if buf is None or len(buf) < max_bytes:
            buf = self._tls.buf = np.empty(max_bytes, np.uint8)
        n = ctypes.c_int64(0)
        w = self.fast.swlog_read(self.h, t, partition, offset, max_records, buf.ctypes.data, max_bytes, ctypes.byref(n))
        if w < 0:
            return self.read(name, partition, offset, max_records, -w + 64)
        out = []
        raw = buf[:w].tobytes()
        pos = 0
        for _ in range(n.value):
            off, ts, kl, vl = _FRAME.unpack_from(raw, pos)
            pos += _FRAME.size
            key = raw[pos:pos + kl] if kl else None
            pos += kl
            val = raw[pos:pos + vl]
            pos += vl
            out.append(Record(name, partition, off, key, val, ts))
        return out

    def wait(self, timeout_s: float):
        with self._cond:
            self._cond.wait(timeout_s)

    # Targeted wake-ups: an append wakes only consumers subscribed to that topic (a global
    # notify_all per record woke every poller in the process -- a GIL storm under load).
    def _wake(self, name: str):
        for ev in list(self._waiters.get(name, ())):
            ev.set()

    def subscribe_event(self, topics, ev: threading.Event):
        with self._lock:
            for t in topics:
                self._waiters.setdefault(t, set()).add(ev)

    def unsubscribe_event(self, topics, ev: threading.Event):
        with self._lock:
            for t in topics:
                self._waiters.get(t, set()).discard(ev)

    def wait_topics(self, topics, timeout_s: float) -> bool:
        ev = threading.Event()
        self.subscribe_event(topics, ev)
        try:
            return ev.wait(timeout_s)
        finally:
            self.unsubscribe_event(topics, ev)

    def fetch_raw(self, reads, max_records: int, timeout_s: float, group: str | None = None,
                  member: str | None = None):
        """One consumer round trip (the Kafka Fetch request): group heartbeat, then up to
        ``max_records`` framed records from ``reads`` = [(topic, partition, offset)], blocking up to
        ``timeout_s`` until one of them has data.  The waiter is subscribed *before* the first read,
        so an append landing between the read and the wait still wakes it.  Returns
        (generation, [(topic, partition, n, framed bytes)]); an empty batch is also returned as soon
        as the group generation changes (the member must refresh its assignment)."""
        gen = self.heartbeat(group, member) if group else 0
        deadline = time.time() + timeout_s
        topics = {r[0] for r in reads}
        ev = threading.Event()
        self.subscribe_event(topics, ev)
        try:
            while True:
                ev.clear()
                out, budget = [], max_records
                for name, p, off in reads:
                    if budget <= 0:
                        break
                    n, raw = self.read_framed(name, p, off, budget)
                    if n:
                        out.append((name, p, n, raw))
                        budget -= n
                if out:
                    return gen, out
                left = deadline - time.time()
                if left <= 0:
                    return gen, out
                ev.wait(min(left, 0.25))
                if group and self.heartbeat(group, member) != gen:
                    return -2, []
        finally:
            self.unsubscribe_event(topics, ev)

    def read_framed(self, name: str, partition: int, offset: int, max_records: int = 500,
                    max_bytes: int = 1 << 20) -> tuple[int, bytes]:
        """(count, framed bytes) -- the wire form of :meth:`read` (``_FRAME`` header + key + value)."""
        t = self.topic(name)
        if offset >= self.fast.swlog_end_offset(self.h, t, partition):
            return 0, b""
        buf = getattr(self._tls, "buf", None)
        if buf is None or len(buf) < max_bytes:
            buf = self._tls.buf = np.empty(max_bytes, np.uint8)
        n = ctypes.c_int64(0)
        w = self.fast.swlog_read(self.h, t, partition, offset, max_records, buf.ctypes.data, max_bytes, ctypes.byref(n))
        if w < 0:
            return self.read_framed(name, partition, offset, max_records, -w + 64)
        return n.value, buf[:w].tobytes()

    def append_arrays(self, name: str, partition: int, keys: np.ndarray, key_off: np.ndarray, vals: np.ndarray,
                      val_off: np.ndarray, ts: int | None = None) -> int:
        """Append len(key_off) - 1 records whose keys / values sit back to back in two heaps (offsets
        [n+1] into each) in one native call -- natively built record batches (routed rejects)."""
        n = len(key_off) - 1
        if n <= 0:
            return -1
        if name in self._protected:
            self._await_room(name, partition, int(val_off[-1]) + int(key_off[-1]))
        t = self.topic(name)
        kb = np.ascontiguousarray(keys, np.uint8) if len(keys) else np.zeros(1, np.uint8)
        vb = np.ascontiguousarray(vals, np.uint8) if len(vals) else np.zeros(1, np.uint8)
        ko = np.ascontiguousarray(key_off, np.int64)
        vo = np.ascontiguousarray(val_off, np.int64)
        tsa = np.full(n, ts if ts is not None else int(time.time() * 1000), np.int64)
        # a multi-MB copy releases the GIL (CDLL); small batches stay on the GIL-holding fast path
        fn = self.lib if vb.nbytes >= (1 << 20) else self.fast
        first = fn.swlog_append_batch(self.h, t, partition, kb.ctypes.data, ko.ctypes.data, vb.ctypes.data,
                                      vo.ctypes.data, tsa.ctypes.data, n)
        if first < 0:
            raise RuntimeError(f"append to {name}[{partition}] failed")
        self._wake(name)
        return first

    def append_routed(self, names, routed, ts: int | None = None) -> list:
        """Append a router's output (``pipeline.routing.RoutedRejects``: records grouped by (kind,
        partition), heaps back to back) to ``names[kind]`` in one native call.  Returns the records
        appended per kind.  Protected topics take the per-group path (producer backpressure)."""
        n = len(routed)
        counts = [0, 0, 0, 0]
        if not n:
            return counts
        if any(nm in self._protected for nm in names):
            for kind, part, kh, ko, vh, vo in routed.groups():
                self.append_arrays(names[kind], max(part, 0), kh, ko, vh, vo, ts)
                counts[kind] += len(ko) - 1
            return counts
        tids = np.array([self.topic(nm) for nm in names], np.int32)
        rec = np.ascontiguousarray(routed.rec, np.int32)
        kb = routed.keys if len(routed.keys) else np.zeros(1, np.uint8)
        vb = routed.vals if len(routed.vals) else np.zeros(1, np.uint8)
        per = np.zeros(4, np.int64)
        fn = self.lib if vb.nbytes >= (1 << 20) else self.fast
        r = fn.swlog_append_routed(self.h, tids.ctypes.data, rec.ctypes.data, n, kb.ctypes.data, vb.ctypes.data,
                                   ts if ts is not None else int(time.time() * 1000), per.ctypes.data)
        if r < 0:
            raise RuntimeError("append of routed rejects failed")
        for kind, nm in enumerate(names):
            if per[kind]:
                self._wake(nm)
        return [int(x) for x in per]

    def append_many(self, batches, ts: int | None = None):
        """[(topic, partition, [(key, value)])] in one call (a producer's flushed batches)."""
        for name, p, recs in batches:
            self.append(name, p, recs, ts)

    # ------------------------------------------------------------------ offsets
    def commit_many(self, group: str, offsets):
        """[(topic, partition, offset)] in one call."""
        for name, p, off in offsets:
            self.commit(group, name, p, off)

    def commit(self, group: str, name: str, partition: int, offset: int):
        self.fast.swlog_commit(self.h, group.encode(), self.topic(name), partition, offset)
        prot = self._protected.get(name)
        if prot and group in prot:
            self.hold(name, partition, offset, holder=("group", group))
            with self._room:
                self._room.notify_all()

    def committed(self, group: str, name: str, partition: int) -> int:
        return self.fast.swlog_committed(self.h, group.encode(), self.topic(name), partition)

    def set_retention(self, name: str, retention_bytes: int):
        """Cap the retained bytes of every partition of a memory-only topic (0 = unlimited)."""
        self.lib.swlog_set_retention(self.h, self.topic(name), int(retention_bytes))
        self._ret_topic[name] = int(retention_bytes)

    def retention(self, name: str) -> int:
        """Retained bytes per partition of ``name`` (0 = unlimited)."""
        return int(self._ret_topic.get(name, self._ret_default))

    # ------------------------------------------------------------------ backpressure
    def protect(self, group: str, name: str, max_wait_s: float = 60.0):
        """No silent loss on ``name`` for consumer ``group``: retention never drops a record the
        group has not committed (a hold at its committed offset), and producers appending to the
        topic wait -- up to ``max_wait_s``, then :class:`BackpressureTimeout` -- while the group's
        unread bytes in the partition would pass the topic's retention.  Event sources then throttle
        (an MQTT publisher is acknowledged only after the hand-off) instead of the log dropping
        batches nobody read (reference: ``MqttInboundEventReceiver.java:166-215``)."""
        with self._room:
            self._protected.setdefault(name, {})[group] = float(max_wait_s)
        for p in range(self.partitions(name)):
            c = self.committed(group, name, p)
            self.hold(name, p, c if c >= 0 else self.begin_offset(name, p), holder=("group", group))

    def unprotect(self, group: str, name: str):
        with self._room:
            self._protected.get(name, {}).pop(group, None)
            if not self._protected.get(name):
                self._protected.pop(name, None)
            self._room.notify_all()
        for p in range(self.partitions(name)):
            self.hold(name, p, None, holder=("group", group))

    def unread_bytes(self, group: str, name: str, partition: int) -> int:
        c = self.committed(group, name, partition)
        return int(self.lib.swlog_bytes_from(self.h, self.topic(name), partition, c if c >= 0 else 0))

    def _await_room(self, name: str, partition: int, nbytes: int):
        groups = self._protected.get(name)
        if not groups:
            return
        limit = self._ret_topic.get(name, self._ret_default)
        if limit <= 0:
            return
        import time as _t
        deadline = _t.monotonic() + max(groups.values())
        waited = False
        while True:
            unread = max(self.unread_bytes(g, name, partition) for g in list(groups))
            if unread == 0 or unread + nbytes <= limit:
                return
            if not waited:
                self.backpressure_waits += 1
                waited = True
            left = deadline - _t.monotonic()
            if left <= 0:
                raise BackpressureTimeout(f"{name}[{partition}]: {unread} unread bytes of {limit} for "
                                          f"{sorted(groups)}; the consumer is not keeping up")
            with self._room:
                self._room.wait(min(left, 0.05))
            groups = self._protected.get(name)
            if not groups:
                return

    def retain_from(self, name: str, partition: int, offset: int) -> int:
        return self.lib.swlog_retain_from(self.h, self.topic(name), partition, offset)

    # ------------------------------------------------------------------ group coordinator
    def join(self, group: str, member_id: str, topics: list[str]) -> int:
        with self._lock:
            g = self._groups.setdefault(group, _Group())
            g.members[member_id] = (tuple(topics), time.time())
            self._rebalance(group, g)
            return g.generation

    def leave(self, group: str, member_id: str):
        with self._lock:
            g = self._groups.get(group)
            if g and member_id in g.members:
                del g.members[member_id]
                self._rebalance(group, g)

    def heartbeat(self, group: str, member_id: str) -> int:
        with self._lock:
            g = self._groups.get(group)
            if g is None or member_id not in g.members:
                return -1
            topics, _ = g.members[member_id]
            g.members[member_id] = (topics, time.time())
            # evict members whose session expired (crashed consumers)
            dead = [m for m, (_, hb) in g.members.items() if time.time() - hb > self.session_timeout_s]
            if dead:
                for m in dead:
                    del g.members[m]
                self._rebalance(group, g)
            return g.generation

    def _rebalance(self, group: str, g: _Group):
        """Range assignor per topic over the sorted member ids."""
        g.generation += 1
        g.assignment = {m: [] for m in g.members}
        topics = sorted({t for ts, _ in g.members.values() for t in ts})
        for t in topics:
            subs = sorted(m for m, (ts, _) in g.members.items() if t in ts)
            if not subs:
                continue
            n = self.partitions(t)
            per, extra = divmod(n, len(subs))
            p = 0
            for i, m in enumerate(subs):
                cnt = per + (1 if i < extra else 0)
                g.assignment[m].extend((t, q) for q in range(p, p + cnt))
                p += cnt
        self._cond.notify_all()
        for evs in self._waiters.values():
            for ev in evs:
                ev.set()

    def assignment(self, group: str, member_id: str) -> tuple[int, list]:
        with self._lock:
            g = self._groups.get(group)
            if g is None:
                return -1, []
            return g.generation, list(g.assignment.get(member_id, []))

    def group_members(self, group: str) -> list[str]:
        with self._lock:
            g = self._groups.get(group)
            return sorted(g.members) if g else []

    # ------------------------------------------------------------------ clients
    def producer(self) -> "Producer":
        return Producer(self)

    def consumer(self, group: str, topics: list[str], auto_offset_reset: str = "earliest",
                 member_id: str | None = None) -> "Consumer":
        return Consumer(self, group, topics, auto_offset_reset, member_id)

    def flush(self):
        self.lib.swlog_flush(self.h)

    def close(self):
        if not self._closed:
            self._closed = True
            self.lib.swlog_close(self.h)


class Producer:
    """Keyed producer.  Inside ``with producer.batching():`` sends made by the *calling thread* are
    buffered and appended per (topic, partition) when the block exits -- one round trip for a whole
    poll batch on a remote bus (Kafka's producer batching).  Per-partition order is preserved, and a
    consumer that wraps its handler in the block commits only after the flush (at-least-once)."""

    def __init__(self, bus: EventBus):
        self.bus = bus
        self.sent = 0
        self._tls = threading.local()

    def batching(self):
        return _ProducerBatch(self)

    def send(self, topic: str, key: str | bytes | None, value: bytes, partition: int | None = None) -> tuple[int, int]:
        kb = key.encode() if isinstance(key, str) else key
        p = self.bus.partition_for(topic, kb) if partition is None else partition
        buf = getattr(self._tls, "buf", None)
        if buf is not None:
            buf.setdefault((topic, p), []).append((kb, value))
            self.sent += 1
            return p, -1
        off = self.bus.append(topic, p, [(kb, value)])
        self.sent += 1
        return p, off

    def _flush_tls(self):
        buf = getattr(self._tls, "buf", None)
        if buf:
            self._tls.buf = {}
            self.bus.append_many([(t, p, recs) for (t, p), recs in buf.items()])

    def send_arrays(self, topic: str, partition: int, keys, key_off, vals, val_off):
        """Records of one partition from a key heap and a value heap (offsets [n+1] into each): one
        native append on the in-process bus, (key, value) pairs elsewhere."""
        n = len(key_off) - 1
        if n <= 0:
            return
        buf = getattr(self._tls, "buf", None)
        if buf is None and hasattr(self.bus, "append_arrays"):
            self.bus.append_arrays(topic, partition, keys, key_off, vals, val_off)
        else:
            kb, vb = bytes(keys), bytes(vals)
            recs = [(kb[key_off[i]:key_off[i + 1]] or None, vb[val_off[i]:val_off[i + 1]]) for i in range(n)]
            if buf is not None:
                buf.setdefault((topic, partition), []).extend(recs)
            else:
                self.bus.append_many([(topic, partition, recs)])
        self.sent += n

    def send_batch(self, topic: str, records: list[tuple[str | bytes | None, bytes]]):
        """Group by partition and append each group in one native call (batched produce)."""
        groups: dict[int, list] = {}
        for k, v in records:
            kb = k.encode() if isinstance(k, str) else k
            groups.setdefault(self.bus.partition_for(topic, kb), []).append((kb, v))
        buf = getattr(self._tls, "buf", None)
        if buf is not None:
            for p, recs in groups.items():
                buf.setdefault((topic, p), []).extend(recs)
        else:
            self.bus.append_many([(topic, p, recs) for p, recs in groups.items()])
        self.sent += len(records)


class _ProducerBatch:
    def __init__(self, producer: Producer):
        self.p = producer
        self.outer = False

    def __enter__(self):
        tls = self.p._tls
        self.outer = getattr(tls, "buf", None) is None
        if self.outer:
            tls.buf = {}
        return self.p

    def __exit__(self, et, ev, tb):
        if self.outer:
            try:
                if et is None:
                    self.p._flush_tls()
            finally:
                self.p._tls.buf = None
        return False


class Consumer:
    """Group member: polls its assigned partitions from committed positions; manual commit."""

    def __init__(self, bus: EventBus, group: str, topics: list[str], auto_offset_reset: str = "earliest",
                 member_id: str | None = None):
        self.bus, self.group, self.topics = bus, group, list(topics)
        for t in self.topics:
            bus.topic(t)
        self.member_id = member_id or f"{group}-{uuid.uuid4().hex[:8]}"
        self.reset = auto_offset_reset
        self._ev = threading.Event()
        self._local = hasattr(bus, "subscribe_event")
        if self._local:
            bus.subscribe_event(self.topics, self._ev)
        self.generation = bus.join(group, self.member_id, self.topics)
        self.positions: dict[tuple[str, int], int] = {}
        self._assigned: list = []
        self._held: set = set()             # partitions poll() holds for a zero-copy reader
        self.lost = 0                       # records retention dropped before this consumer read them
        self._refresh()
        self.closed = False

    def _refresh(self):
        gen, asg = self.bus.assignment(self.group, self.member_id)
        self.generation = gen
        self._assigned = asg
        newpos = {}
        for tp in asg:
            if tp in self.positions:
                newpos[tp] = self.positions[tp]
                continue
            c = self.bus.committed(self.group, *tp)
            if c >= 0:
                newpos[tp] = c
            else:
                newpos[tp] = self.bus.begin_offset(*tp) if self.reset == "earliest" else self.bus.end_offset(*tp)
        self.positions = newpos

    def assignment(self) -> list:
        return list(self._assigned)

    def _poll_fetch(self, timeout_ms: int, max_records: int) -> dict[tuple[str, int], list[Record]]:
        """Remote bus: heartbeat + wait + read of every assigned partition in one round trip."""
        deadline = time.time() + timeout_ms / 1000.0
        while True:
            reads = [(t, p, self.positions[(t, p)]) for t, p in self._assigned]
            gen, got = self.bus.fetch_raw(reads, max_records, max(0.0, deadline - time.time()), self.group,
                                          self.member_id)
            if gen == -1:
                self.generation = self.bus.join(self.group, self.member_id, self.topics)
                self._refresh()
            elif gen == -2 or gen != self.generation:
                self._refresh()
            out = {}
            for name, p, n, raw in got:
                tp = (name, p)
                if tp not in self.positions:      # reassigned while the fetch was in flight
                    continue
                recs = parse_frames(name, p, n, raw)
                recs = [r for r in recs if r.offset >= self.positions[tp]]
                if recs:
                    out[tp] = recs
                    self.positions[tp] = recs[-1].offset + 1
            if out or time.time() >= deadline:
                return out

    def poll(self, timeout_ms: int = 1000, max_records: int = 500, views: bool = False,
             holder=None) -> dict[tuple[str, int], list[Record]]:
        """``views=True`` on the in-process bus: record values are zero-copy views of the log
        (:meth:`EventBus.read_views`); other buses return copies as usual.  With ``holder`` the poll
        takes a retention hold (owned by ``holder``) on every partition before reading it in place --
        after any rebalance refresh, so a partition gained mid-poll is held too -- and remembers
        which it holds; :meth:`release_holds` drops exactly those, including partitions the
        rebalance took away."""
        if not self._local and hasattr(self.bus, "fetch_raw"):
            return self._poll_fetch(timeout_ms, max_records)
        views = views and hasattr(self.bus, "read_views")
        read = self.bus.read_views if views else self.bus.read
        hold = views and holder is not None and hasattr(self.bus, "hold")
        deadline = time.time() + timeout_ms / 1000.0
        while True:
            self._ev.clear()
            gen = self.bus.heartbeat(self.group, self.member_id)
            if gen < 0:
                self.generation = self.bus.join(self.group, self.member_id, self.topics)
                gen = self.generation
            if gen != self.generation:
                self._refresh()
            out = {}
            budget = max_records
            for tp in self._assigned:
                if budget <= 0:
                    break
                if hold:
                    self.bus.hold(tp[0], tp[1], self.positions[tp], holder=holder)
                    self._held.add(tp)
                recs = read(tp[0], tp[1], self.positions[tp], budget)
                if recs:
                    if recs[0].offset > self.positions[tp]:
                        # retention dropped records this group never read (an unprotected topic
                        # whose consumer fell behind): counted, never silent
                        self.lost += recs[0].offset - self.positions[tp]
                    out[tp] = recs
                    self.positions[tp] = recs[-1].offset + 1
                    budget -= len(recs)
            if out or time.time() >= deadline:
                return out
            left = max(0.0, deadline - time.time())
            if self._local:
                self._ev.wait(min(1.0, left))
            else:
                self.bus.wait_topics(self.topics, min(1.0, left))

    def release_holds(self, holder):
        """Drop the retention holds :meth:`poll` took for ``holder``."""
        held, self._held = self._held, set()
        for tp in held:
            self.bus.hold(tp[0], tp[1], None, holder=holder)

    def commit(self, offsets: dict[tuple[str, int], int] | None = None):
        """Commit positions (next offset to read); default: current positions of all partitions."""
        last = self.__dict__.setdefault("_last_commit", {})
        items = [(tp, off) for tp, off in (offsets or self.positions).items() if last.get(tp) != off]
        if not items:
            return                               # nothing moved since the last commit
        if hasattr(self.bus, "commit_many"):
            self.bus.commit_many(self.group, [(tp[0], tp[1], off) for tp, off in items])
        else:
            for tp, off in items:
                self.bus.commit(self.group, tp[0], tp[1], off)
        last.update(items)

    commit_async = commit

    def seek(self, topic: str, partition: int, offset: int):
        self.positions[(topic, partition)] = offset

    def lag(self) -> int:
        return sum(self.bus.end_offset(*tp) - self.positions.get(tp, 0) for tp in self._assigned)

    def close(self):
        if not self.closed:
            self.closed = True
            if self._local:
                self.bus.unsubscribe_event(self.topics, self._ev)
            self.bus.leave(self.group, self.member_id)
