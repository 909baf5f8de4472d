"""Network infrastructure service: the event bus (Kafka role) and the coordination store (ZooKeeper
role) served to other processes over gRPC, plus drop-in remote clients.

Reference deployment: every microservice process talks to a Kafka cluster (``MicroserviceKafkaConsumer``/
``Producer``), a ZooKeeper ensemble (``ZookeeperManager.java:30-80``, Curator ``TreeCache`` in
``ConfigurationMonitor.java:69-125``, ``InterProcessMutex`` in ``BootstrapTenantEngineOperation.java:57-117``).
Here one ``InfraServer`` hosts :class:`EventBus` (native ``swlog`` storage) and :class:`Coordination`;
:class:`RemoteEventBus` / :class:`RemoteCoordination` implement the same Python surface so
``Producer``/``Consumer``/``InterProcessMutex``/the microservice runtime run unchanged across processes.

Wire format: unary gRPC ``/sitewhere.infra/<object>.<method>`` with msgpack ``[args, kwargs]`` bodies.
Fetches return the native log's raw frame buffer (no re-encoding); long polls (``wait``,
``wait_for``, ``watch_poll``) block server-side with a bounded timeout.  ZooKeeper session semantics:
clients heartbeat their session; the server expires silent sessions and deletes their ephemeral
nodes (crashed processes release locks and leave the topology).
"""
from __future__ import annotations

import itertools
import queue
import threading
import time
import uuid
from concurrent import futures

import grpc
import msgpack

from ..bus.log import _FRAME, Consumer, EventBus, Producer, Record
from ..coord.store import (BadVersionError, Coordination, NodeExistsError, NoNodeError,
                           NotEmptyError, Stat)

_ERRORS = {c.__name__: c for c in (NoNodeError, NodeExistsError, BadVersionError, NotEmptyError, KeyError,
                                   ValueError, TimeoutError, RuntimeError)}


def _pack(obj) -> bytes:
    return msgpack.packb(obj, use_bin_type=True, default=_default)


def _default(o):
    if isinstance(o, Stat):
        return {"__stat__": [o.version, o.ctime, o.mtime, o.ephemeral_owner, o.num_children]}
    if isinstance(o, (set, tuple)):
        return list(o)
    raise TypeError(f"cannot pack {type(o).__name__}")


def _hook(d):
    if "__stat__" in d:
        return Stat(*d["__stat__"])
    return d


def _unpack(b: bytes):
    return msgpack.unpackb(b, raw=False, object_hook=_hook, strict_map_key=False)


# ============================================================================ server side
class _BusFacade:
    """Bus methods exposed over the wire (raw frame fetch instead of Record objects)."""

    def __init__(self, bus: EventBus):
        self.b = bus

    def topic(self, name, partitions=None):
        return self.b.topic(name, partitions)

    def partitions(self, name):
        return self.b.partitions(name)

    def topics(self):
        return self.b.topics()

    def end_offset(self, name, p):
        return self.b.end_offset(name, p)

    def begin_offset(self, name, p):
        return self.b.begin_offset(name, p)

    def append(self, name, p, records, ts=None):
        return self.b.append(name, p, [(k, v) for k, v in records], ts)

    def read_raw(self, name, p, offset, max_records=500, max_bytes=1 << 20):
        import ctypes

        import numpy as np
        t = self.b.topic(name)
        while True:
            buf = np.empty(max_bytes, np.uint8)
            n = ctypes.c_int64(0)
            w = self.b.lib.swlog_read(self.b.h, t, p, offset, max_records, buf.ctypes.data, max_bytes, ctypes.byref(n))
            if w >= 0:
                return [n.value, buf[:w].tobytes()]
            max_bytes = -w + 64

    def wait(self, timeout_s):
        self.b.wait(min(float(timeout_s), 1.0))

    def wait_topics(self, topics, timeout_s):
        return self.b.wait_topics(topics, min(float(timeout_s), 1.0))

    def fetch_raw(self, reads, max_records, timeout_s, group=None, member=None):
        gen, got = self.b.fetch_raw([tuple(r) for r in reads], int(max_records), min(float(timeout_s), 1.0),
                                    group, member)
        return [gen, [list(x) for x in got]]

    def append_many(self, batches, ts=None):
        self.b.append_many([(t, p, [tuple(r) for r in recs]) for t, p, recs in batches], ts)

    def commit_many(self, group, offsets):
        self.b.commit_many(group, [tuple(o) for o in offsets])

    def commit(self, group, name, p, offset):
        self.b.commit(group, name, p, offset)

    def committed(self, group, name, p):
        return self.b.committed(group, name, p)

    def retain_from(self, name, p, offset):
        return self.b.retain_from(name, p, offset)

    def join(self, group, member, topics):
        return self.b.join(group, member, topics)

    def leave(self, group, member):
        self.b.leave(group, member)

    def heartbeat(self, group, member):
        return self.b.heartbeat(group, member)

    def assignment(self, group, member):
        gen, asg = self.b.assignment(group, member)
        return [gen, [list(x) for x in asg]]

    def group_members(self, group):
        return self.b.group_members(group)

    def flush(self):
        self.b.flush()


class _CoordFacade:
    def __init__(self, coord: Coordination, session_timeout_s: float):
        self.c = coord
        self.session_timeout_s = session_timeout_s
        self._last: dict[str, float] = {}
        self._watches: dict[str, tuple[queue.Queue, callable]] = {}
        self._lock = threading.Lock()

    # sessions
    def open_session(self):
        s = self.c.open_session()
        self._last[s] = time.time()
        return s

    def keepalive(self, session):
        if session not in self._last:
            return False
        self._last[session] = time.time()
        return True

    def close_session(self, session):
        self._last.pop(session, None)
        self.c.close_session(session)

    def expire(self):
        now = time.time()
        for s, t in list(self._last.items()):
            if now - t > self.session_timeout_s:
                self.close_session(s)

    # CRUD
    def create(self, path, data=b"", ephemeral=False, sequential=False, make_parents=True, session=None):
        return self.c.create(path, data, ephemeral, sequential, make_parents, session)

    def ensure(self, path, data=b""):
        return self.c.ensure(path, data)

    def exists(self, path):
        return self.c.exists(path)

    def get(self, path):
        d, st = self.c.get(path)
        return [d, st]

    def get_data(self, path, default=None):
        return self.c.get_data(path, default)

    def set(self, path, data, version=-1):
        return self.c.set(path, data, version)

    def put(self, path, data):
        return self.c.put(path, data)

    def delete(self, path, version=-1, recursive=False):
        return self.c.delete(path, version, recursive)

    def children(self, path):
        return self.c.children(path)

    def walk(self, prefix="/"):
        return self.c.walk(prefix)

    def wait_for(self, path, timeout_s):
        return self.c.wait_for(path, min(float(timeout_s), 1.0))

    # watches (server-side queues drained by long polls)
    def watch_open(self, prefix, initial=True):
        wid = uuid.uuid4().hex
        q: queue.Queue = queue.Queue()
        cancel = self.c.watch_tree(prefix, lambda k, p, d: q.put([k, p, d]), initial)
        with self._lock:
            self._watches[wid] = (q, cancel)
        return wid

    def watch_poll(self, wid, timeout_s=1.0, max_events=1000):
        w = self._watches.get(wid)
        if w is None:
            return None
        q = w[0]
        out = []
        try:
            out.append(q.get(timeout=min(float(timeout_s), 1.0)))
            while len(out) < max_events:
                out.append(q.get_nowait())
        except queue.Empty:
            pass
        return out

    def watch_close(self, wid):
        with self._lock:
            w = self._watches.pop(wid, None)
        if w:
            w[1]()


class InfraServer:
    """Hosts the bus and the coordination store for a multi-process instance."""

    def __init__(self, bus: EventBus | None = None, coord: Coordination | None = None, port: int = 0,
                 host: str = "127.0.0.1", workers: int = 64, session_timeout_s: float = 15.0):
        self.bus = bus or EventBus(None)
        self.coord = coord or Coordination()
        self.objects = {"bus": _BusFacade(self.bus), "coord": _CoordFacade(self.coord, session_timeout_s)}
        self.host, self.port, self.workers = host, port, workers
        self._server = None
        self._stop = threading.Event()

    def _handler(self, obj, method):
        def handle(request: bytes, context):
            try:
                args, kwargs = _unpack(request)
                return _pack({"ok": getattr(obj, method)(*args, **kwargs)})
            except Exception as e:  # noqa: BLE001
                return _pack({"err": type(e).__name__, "msg": str(e)})
        return handle

    def start(self):
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=self.workers),
                          options=[("grpc.max_send_message_length", 64 << 20),
                                   ("grpc.max_receive_message_length", 64 << 20)])

        class _Generic(grpc.GenericRpcHandler):
            def __init__(s, outer):
                s.outer = outer

            def service(s, details):
                path = details.method  # /sitewhere.infra/<obj>.<method>
                if not path.startswith("/sitewhere.infra/"):
                    return None
                name, _, meth = path[len("/sitewhere.infra/"):].partition(".")
                obj = s.outer.objects.get(name)
                if obj is None or meth.startswith("_") or not hasattr(obj, meth):
                    return None
                return grpc.unary_unary_rpc_method_handler(s.outer._handler(obj, meth))

        srv.add_generic_rpc_handlers([_Generic(self)])
        self.port = srv.add_insecure_port(f"{self.host}:{self.port}")
        srv.start()
        self._server = srv
        threading.Thread(target=self._expiry, daemon=True, name="infra-session-expiry").start()
        return self

    def _expiry(self):
        while not self._stop.wait(1.0):
            self.objects["coord"].expire()

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def stop(self):
        self._stop.set()
        if self._server is not None:
            self._server.stop(0.5)
            self._server = None


# ============================================================================ client side
class _Remote:
    def __init__(self, address: str, obj: str):
        self.address, self.obj = address, obj
        self._ch = grpc.insecure_channel(address, options=[("grpc.max_send_message_length", 64 << 20),
                                                           ("grpc.max_receive_message_length", 64 << 20)])
        self._stubs: dict = {}

    def call(self, method: str, *args, **kwargs):
        st = self._stubs.get(method)
        if st is None:
            st = self._stubs[method] = self._ch.unary_unary(f"/sitewhere.infra/{self.obj}.{method}")
        r = _unpack(st(_pack([list(args), kwargs]), timeout=30.0))
        if "err" in r:
            raise _ERRORS.get(r["err"], RuntimeError)(r["msg"])
        return r["ok"]

    def close(self):
        self._ch.close()


class RemoteEventBus:
    """Client for a bus hosted by :class:`InfraServer` (same surface as :class:`EventBus`)."""

    _rr = itertools.count()

    def __init__(self, address: str):
        self.r = _Remote(address, "bus")
        self._parts: dict[str, int] = {}
        from .._native import native
        self.lib = native()
        self.directory = None

    def topic(self, name, partitions=None):
        return self.r.call("topic", name, partitions)

    def partitions(self, name):
        n = self._parts.get(name)
        if n is None:
            n = self._parts[name] = self.r.call("partitions", name)
        return n

    def topics(self):
        return self.r.call("topics")

    def end_offset(self, name, p):
        return self.r.call("end_offset", name, p)

    def begin_offset(self, name, p):
        return self.r.call("begin_offset", name, p)

    def partition_for(self, name, key):
        n = self.partitions(name)
        if key is None:
            return next(self._rr) % n
        # Kafka's murmur2 partitioner, natively, keeping the GIL (a per-record call: no copy, no
        # release / re-acquire)
        from .._native import native_gil
        return native_gil().sw_partition_for_key(bytes(key), len(key), n)

    def append(self, name, p, records, ts=None):
        return self.r.call("append", name, p, [[k, v] for k, v in records], ts)

    def read(self, name, p, offset, max_records=500, max_bytes=1 << 20):
        n, raw = self.r.call("read_raw", name, p, offset, max_records, max_bytes)
        out, pos = [], 0
        for _ in range(n):
            off, ts, kl, vl = _FRAME.unpack_from(raw, pos)
            pos += _FRAME.size
            key = raw[pos:pos + kl] if kl else None
            pos += kl
            out.append(Record(name, p, off, key, raw[pos:pos + vl], ts))
            pos += vl
        return out

    def fetch_raw(self, reads, max_records, timeout_s, group=None, member=None):
        gen, got = self.r.call("fetch_raw", [list(r) for r in reads], max_records, min(float(timeout_s), 1.0),
                               group, member)
        return gen, [tuple(x) for x in got]

    def append_many(self, batches, ts=None):
        self.r.call("append_many", [[t, p, [[k, v] for k, v in recs]] for t, p, recs in batches], ts)

    def commit_many(self, group, offsets):
        self.r.call("commit_many", group, [list(o) for o in offsets])

    def wait(self, timeout_s):
        self.r.call("wait", timeout_s)

    def wait_topics(self, topics, timeout_s):
        return self.r.call("wait_topics", list(topics), timeout_s)

    def commit(self, group, name, p, offset):
        self.r.call("commit", group, name, p, offset)

    def committed(self, group, name, p):
        return self.r.call("committed", group, name, p)

    def retain_from(self, name, p, offset):
        return self.r.call("retain_from", name, p, offset)

    def join(self, group, member, topics):
        return self.r.call("join", group, member, list(topics))

    def leave(self, group, member):
        self.r.call("leave", group, member)

    def heartbeat(self, group, member):
        return self.r.call("heartbeat", group, member)

    def assignment(self, group, member):
        gen, asg = self.r.call("assignment", group, member)
        return gen, [tuple(x) for x in asg]

    def group_members(self, group):
        return self.r.call("group_members", group)

    def producer(self):
        return Producer(self)

    def consumer(self, group, topics, auto_offset_reset="earliest", member_id=None):
        return Consumer(self, group, topics, auto_offset_reset, member_id)

    def flush(self):
        self.r.call("flush")

    def close(self):
        self.r.close()


class RemoteCoordination:
    """Client for a coordination store hosted by :class:`InfraServer` (same surface as :class:`Coordination`)."""

    def __init__(self, address: str, keepalive_s: float = 3.0):
        self.r = _Remote(address, "coord")
        self._cond = threading.Condition()      # InterProcessMutex polls on this
        self._sessions: set[str] = set()
        self._stop = threading.Event()
        self._ka = threading.Thread(target=self._keepalive, args=(keepalive_s,), daemon=True, name="coord-keepalive")
        self._ka.start()
        self._watch_threads: list = []

    def _keepalive(self, period):
        while not self._stop.wait(period):
            for s in list(self._sessions):
                try:
                    self.r.call("keepalive", s)
                except Exception:
                    pass

    def open_session(self):
        s = self.r.call("open_session")
        self._sessions.add(s)
        return s

    def close_session(self, session):
        self._sessions.discard(session)
        self.r.call("close_session", session)

    def create(self, path, data=b"", ephemeral=False, sequential=False, make_parents=True, session=None):
        if ephemeral and session is None:
            session = self._default_session()
        return self.r.call("create", path, bytes(data), ephemeral, sequential, make_parents, session)

    def _default_session(self):
        if not hasattr(self, "_dflt"):
            self._dflt = self.open_session()
        return self._dflt

    def ensure(self, path, data=b""):
        return self.r.call("ensure", path, bytes(data))

    def exists(self, path):
        return self.r.call("exists", path)

    def get(self, path):
        d, st = self.r.call("get", path)
        return d, st

    def get_data(self, path, default=None):
        return self.r.call("get_data", path, default)

    def set(self, path, data, version=-1):
        return self.r.call("set", path, bytes(data), version)

    def put(self, path, data):
        return self.r.call("put", path, bytes(data))

    def delete(self, path, version=-1, recursive=False):
        return self.r.call("delete", path, version, recursive)

    def children(self, path):
        return self.r.call("children", path)

    def walk(self, prefix="/"):
        return self.r.call("walk", prefix)

    def wait_for(self, path, timeout_s):
        end = time.time() + timeout_s
        while True:
            if self.r.call("wait_for", path, max(0.0, min(1.0, end - time.time()))):
                return True
            if time.time() >= end:
                return False

    def watch_tree(self, prefix, callback, initial=True):
        wid = self.r.call("watch_open", prefix, initial)
        stop = threading.Event()

        def run():
            while not stop.is_set() and not self._stop.is_set():
                try:
                    evs = self.r.call("watch_poll", wid, 1.0)
                except Exception:
                    time.sleep(0.2)
                    continue
                if evs is None:
                    return
                for k, p, d in evs:
                    try:
                        callback(k, p, d)
                    except Exception:
                        pass

        t = threading.Thread(target=run, daemon=True, name=f"coord-watch-{prefix}")
        t.start()
        self._watch_threads.append(t)

        def cancel():
            stop.set()
            try:
                self.r.call("watch_close", wid)
            except Exception:
                pass
        return cancel

    def close(self):
        self._stop.set()
        for s in list(self._sessions):
            try:
                self.close_session(s)
            except Exception:
                pass
        self.r.close()
