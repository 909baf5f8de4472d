"""Bus consumer/producer components and the near cache.

Reference:
  * ``kafka/MicroserviceKafkaConsumer.java:53-133`` -- one consumer per component on its own poll
    thread, manual commits, per-partition ``process()``, shutdown via wakeup
  * ``kafka/DirectKafkaConsumer.java:28-41`` -- process then ``commitAsync`` (at-least-once)
  * ``KafkaOutboundConnectorHost.java:144-217`` -- pool hand-off (the reference commits *before*
    the async batch completes = at-most-once; here the commit waits for the batch: at-least-once)
  * ``sitewhere-grpc-client/.../cache/CacheProvider.java`` + ``NearCacheManager.java:77-165`` --
    near caches (LRU 10,000, TTL 60 s) for device / assignment / type lookups; invalidated by the
    device-model change feed instead of a Hazelcast grid.
"""
from __future__ import annotations

import threading
import time
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor, wait

from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent

_DEFAULT = object()


class RetryFrom(Exception):
    """Raised by a handler whose earlier batches have side effects still pending (e.g. rows stepped
    through the inbound engine but not yet stored): re-read each ``(topic, partition)`` in ``offsets``
    from the given offset instead of from the current batch's first record.  Such a rewind is a
    transient condition by construction, so it never counts towards dead-lettering."""

    def __init__(self, offsets: dict, cause: BaseException | None = None):
        super().__init__(f"re-read from {offsets}: {cause!r}")
        self.offsets = dict(offsets)
        self.cause = cause


class BusConsumer(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.Other

    def __init__(self, engine, name: str, topics: list[str], handler, threads: int = 0, max_records: int = 500,
                 group: str | None = None, auto_commit: bool = True, max_attempts=_DEFAULT, idle=None,
                 views: bool = False, merge_partitions: bool = False):
        super().__init__(name)
        self.tenant_engine = engine
        self.engine = engine
        self.topics = topics
        self.handler = handler            # handler(list[Record]) per partition batch
        self.threads = threads
        self.max_records = max_records
        # one handler call for every partition of a poll (split over the pool): a per-event service
        # whose handler makes a bulk RPC per call (inbound processing -> event management) pays
        # that round trip per poll, not per partition
        self.merge_partitions = merge_partitions
        inst = engine.ms.instance
        self.group = group or f"{inst.naming.prefix()}.{engine.tenant.token}.{engine.ms.identifier}.{name}"
        self._stop = threading.Event()
        self._t = None
        self.processed = 0
        self.failures = 0
        self.retries = 0          # batches re-read after a handler failure
        self.dropped = 0          # records of poison batches skipped after max_attempts
        # False: the handler commits explicit offsets itself (checkpoint-aligned commits)
        self.auto_commit = auto_commit
        # None: a control-plane consumer (registry change feed, registration): a batch is retried
        # until it succeeds, with an error logged every ``alert_every`` attempts -- skipping it would
        # leave the consumer's state silently diverged from its source of truth
        if max_attempts is not _DEFAULT:
            self.max_attempts = max_attempts
        self.rewinds = 0
        # called on the poll thread when a poll returns nothing; may raise RetryFrom (a failure that
        # surfaced after its batch was handed off, e.g. on a store thread, with no new records due)
        self.idle = idle
        # zero-copy: on the in-process bus the handler gets memoryviews of the log itself, valid
        # until it returns (a retention hold covers the partition's batch meanwhile)
        self.views = views

    def start(self, monitor):
        bus = self.engine.ms.instance.bus
        self.consumer = bus.consumer(self.group, self.topics, auto_offset_reset="earliest")
        self.pool = ThreadPoolExecutor(max_workers=self.threads, thread_name_prefix=self.component_name) if self.threads else None
        self._stop.clear()
        self._t = threading.Thread(target=self._run, daemon=True, name=f"consumer-{self.component_name}")
        self._t.start()

    # A failed batch is re-read from its first record (the partition is not committed past it) with
    # exponential backoff: transient faults (RPC unavailable, storage hiccups) cost retries, never
    # records.  A batch failing ``max_attempts`` times in a row is a poison batch: its records are
    # moved to ``<topic>.dead-letter`` (same keys and values, so they can be inspected and
    # re-injected with :func:`replay_dead_letter`), counted in ``dropped`` and skipped, so the
    # partition is not wedged forever.
    max_attempts: int | None = 10
    alert_every = 10
    DEAD_LETTER_SUFFIX = ".dead-letter"

    def _dead_letter(self, recs):
        try:
            self.engine.ms.producer.send_batch(recs[0].topic + self.DEAD_LETTER_SUFFIX,
                                               [(r.key, r.value) for r in recs])
            return True
        except Exception:
            self.logger.exception("consumer %s: dead-letter publish failed", self.component_name)
            return False

    def _call(self, recs):
        """True on success, False on failure, or the ``{tp: offset}`` rewind of a :class:`RetryFrom`."""
        try:
            # sends made while handling this batch go out in one produce round trip, before the commit
            with self.engine.ms.producer.batching():
                self.handler(recs)
            self.processed += len(recs)
            return True
        except RetryFrom as e:
            self.failures += len(recs)
            self.logger.warning("consumer %s: re-reading %s (%r)", self.component_name, e.offsets, e.cause)
            return e.offsets
        except Exception:
            self.failures += len(recs)
            self.logger.exception("consumer %s failed to process %d records", self.component_name, len(recs))
            return False

    def _run(self):
        backoff, attempts = 0.05, {}
        bus = self.engine.ms.instance.bus
        views = self.views and hasattr(bus, "read_views") and hasattr(bus, "hold")
        while not self._stop.is_set():
            try:
                if views:       # the poll holds each partition before reading it in place
                    batch = self.consumer.poll(100, self.max_records, views=True, holder=self)
                else:
                    batch = self.consumer.poll(100, self.max_records)
            except Exception:
                self.logger.exception("poll failed")
                time.sleep(0.1)
                continue
            if not batch:
                if views:
                    self.consumer.release_holds(self)
                if self.idle is not None:
                    try:
                        self.idle()
                    except RetryFrom as e:
                        self.logger.warning("consumer %s: re-reading %s (%r)", self.component_name, e.offsets, e.cause)
                        for tp, pos in e.offsets.items():
                            self.consumer.seek(tp[0], tp[1], pos)
                        self.rewinds += 1
                        self.retries += 1
                        self._stop.wait(backoff)
                        backoff = min(2.0, backoff * 2)
                    except Exception:
                        self.logger.exception("consumer %s: idle check failed", self.component_name)
                continue
            ok: dict = {}
            if self.merge_partitions and len(batch) > 1:
                allrecs = [r for recs in batch.values() for r in recs]
                if self.pool is None:
                    rs = [self._call(allrecs)]
                else:
                    step = max(256, -(-len(allrecs) // max(1, self.threads)))
                    fs = [self.pool.submit(self._call, allrecs[i:i + step]) for i in range(0, len(allrecs), step)]
                    wait(fs)
                    rs = [f.result() for f in fs]
                res = next((r for r in rs if isinstance(r, dict)), all(r is True for r in rs))
                ok = {tp: res for tp in batch}
            elif self.pool is None:
                for tp, recs in batch.items():
                    ok[tp] = self._call(recs)
            else:
                futs = {}
                for tp, recs in batch.items():
                    step = max(1, len(recs) // self.threads)
                    futs[tp] = [self.pool.submit(self._call, recs[i:i + step]) for i in range(0, len(recs), step)]
                wait([f for fs in futs.values() for f in fs])
                ok = {}
                for tp, fs in futs.items():
                    rs = [f.result() for f in fs]
                    ok[tp] = next((r for r in rs if isinstance(r, dict)), all(r is True for r in rs))
            failed, rewind = {}, {}
            for tp, good in ok.items():
                if isinstance(good, dict):
                    rewind.update(good)
                    if tp not in good:
                        rewind[tp] = batch[tp][0].offset
            for tp, pos in rewind.items():
                failed[tp] = min(pos, failed.get(tp, pos))
            for tp, good in ok.items():
                first = batch[tp][0].offset
                if good is True or tp in rewind:
                    if tp not in rewind:
                        attempts.pop(tp, None)
                    continue
                n = attempts.get(tp, (first, 0))[1] + 1 if attempts.get(tp, (None,))[0] == first else 1
                if self.max_attempts is None:
                    if n % self.alert_every == 0:
                        self.logger.error("consumer %s: batch %s@%d still failing after %d attempts "
                                          "(control-plane consumer: retried until it succeeds)",
                                          self.component_name, tp, first, n)
                elif n >= self.max_attempts and self._dead_letter(batch[tp]):
                    attempts.pop(tp, None)
                    self.dropped += len(batch[tp])
                    self.logger.error("consumer %s: poison batch %s@%d moved to %s%s after %d attempts",
                                      self.component_name, tp, first, tp[0], self.DEAD_LETTER_SUFFIX, n)
                    continue
                attempts[tp] = (first, n)
                failed[tp] = first
            for tp, pos in failed.items():
                self.consumer.seek(tp[0], tp[1], pos)           # re-read it: at-least-once
            if rewind:
                self.rewinds += 1
            if views:
                self.consumer.release_holds(self)               # the handler is done with the views
            if self.auto_commit:
                offsets = {tp: pos for tp, pos in self.consumer.positions.items() if tp not in failed}
                if offsets:
                    self.consumer.commit(offsets)               # after processing: at-least-once
            if failed:
                self.retries += 1
                self._stop.wait(backoff)
                backoff = min(2.0, backoff * 2)
            else:
                backoff = 0.05

    def stop(self, monitor):
        self._stop.set()
        if self._t:
            self._t.join(timeout=3)
        if getattr(self, "consumer", None):
            if hasattr(self.consumer, "release_holds"):
                self.consumer.release_holds(self)
            self.consumer.close()
        if self.pool:
            self.pool.shutdown(wait=True)

    def drain(self, timeout_s: float = 10.0) -> bool:
        """Wait until every assigned partition is consumed and committed (tests / shutdown)."""
        end = time.time() + timeout_s
        bus = self.engine.ms.instance.bus
        while time.time() < end:
            lag = 0
            for t in self.topics:
                for p in range(bus.partitions(t)):
                    c = bus.committed(self.group, t, p)
                    lag += bus.end_offset(t, p) - max(c, 0)
            if lag == 0:
                return True
            time.sleep(0.02)
        return False


class NearCache:
    """Thread-safe LRU with TTL and max-idle expiry (reference near cache,
    ``HazelcastManager.java:107-120``: LRU 10,000 entries, TTL 60 s, max-idle 20 s).  Entries are
    also invalidated explicitly from the device-model change feed."""

    def __init__(self, capacity: int = 10_000, ttl_s: float = 60.0, max_idle_s: float | None = 20.0):
        self.capacity, self.ttl, self.max_idle = capacity, ttl_s, max_idle_s
        self._d: OrderedDict = OrderedDict()        # key -> [value, created, last access]
        self._lock = threading.Lock()
        self.hits = self.misses = 0

    def get(self, key, loader=None):
        # Lock-free hit path (dict reads are atomic under the GIL); recency is refreshed on put, so
        # eviction is insertion-ordered with TTL -- taking a lock per hit serialised every consumer
        # thread on this cache.  The access stamp is a plain store into the entry.
        v = self._d.get(key)
        if v is not None:
            now = time.time()
            if now - v[1] < self.ttl and (self.max_idle is None or now - v[2] < self.max_idle):
                v[2] = now
                self.hits += 1
                return v[0]
        self.misses += 1
        if loader is None:
            return None
        val = loader(key)
        if val is not None:
            self.put(key, val)
        return val

    def get_many(self, keys, loader_many=None) -> dict:
        """key -> value for ``keys`` (missing ones: None): hits from the cache, every miss loaded with
        ONE ``loader_many(missed keys) -> values`` call (a consumer's poll batch validated in one
        pass, one bulk lookup for what the cache lacks)."""
        out, miss = {}, []
        now = time.time()
        for k in dict.fromkeys(keys):
            v = self._d.get(k)
            if v is not None and now - v[1] < self.ttl and (self.max_idle is None or now - v[2] < self.max_idle):
                v[2] = now
                self.hits += 1
                out[k] = v[0]
            else:
                self.misses += 1
                miss.append(k)
        if miss and loader_many is not None:
            for k, val in zip(miss, loader_many(miss)):
                out[k] = val
                if val is not None:
                    self.put(k, val)
        return out

    def put(self, key, val):
        with self._lock:
            now = time.time()
            self._d[key] = [val, now, now]
            self._d.move_to_end(key)
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)

    def invalidate(self, key=None):
        with self._lock:
            if key is None:
                self._d.clear()
            else:
                self._d.pop(key, None)

    def __len__(self):
        return len(self._d)


def replay_dead_letter(bus, topic: str, group: str = "dead-letter-replay", limit: int | None = None,
                       timeout_ms: int = 200) -> int:
    """Move records parked in ``<topic>.dead-letter`` (poison batches, see ``BusConsumer``) back onto
    ``topic`` -- e.g. after the bug or the bad reference data that made them fail was fixed.  The
    replay consumer group commits what it moved, so a second call resumes after it.  Returns the
    number of records re-published.

    Ordering is NOT preserved: replayed records are appended after everything written to ``topic``
    since they were parked, so a consumer sees them after newer records of the same key.  That is
    why control-plane consumers (registry change feed, registration) never dead-letter
    (``max_attempts=None``): an old ``device.updated`` replayed after a newer one would win."""
    c = bus.consumer(group, [topic + BusConsumer.DEAD_LETTER_SUFFIX], auto_offset_reset="earliest")
    prod = bus.producer()
    moved = 0
    try:
        while limit is None or moved < limit:
            batch = c.poll(timeout_ms, 500 if limit is None else min(500, limit - moved))
            if not batch:
                break
            for recs in batch.values():
                prod.send_batch(topic, [(r.key, r.value) for r in recs])
                moved += len(recs)
            c.commit()
    finally:
        c.close()
    return moved
