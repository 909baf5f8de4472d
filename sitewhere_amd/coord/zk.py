"""Apache ZooKeeper over its wire protocol (jute) -- no client-library dependency.

The reference keeps configuration, bootstrap markers and locks in ZooKeeper through Curator
(``ZookeeperManager.java:30-80``: namespace = product id, ``ExponentialBackoffRetry``;
``ConfigurationMonitor`` = TreeCache; ``BootstrapTenantEngineOperation`` = InterProcessMutex).
:class:`ZooKeeperCoordination` implements this package's coordination surface
(:class:`~sitewhere_amd.coord.store.Coordination`) on a ZooKeeper ensemble:

* one ZooKeeper session per :meth:`open_session` (ephemeral nodes live and die with it) plus a
  default session; the namespace is a chroot (``host:port/sitewhere``);
* CRUD, versions, ephemeral / sequential nodes, recursive delete;
* ``watch_tree`` is a TreeCache: one-shot data + child watches re-armed on every event, diffed
  into NODE_ADDED / NODE_UPDATED / NODE_REMOVED callbacks (dispatched off the I/O thread).

Protocol: connect handshake (``ConnectRequest``/``ConnectResponse``), request header
``(xid, type)``, reply header ``(xid, zxid, err)``, notifications on xid -1, pings on xid -2.
``coord/zk_server.py`` serves the same protocol in process.
"""
from __future__ import annotations

import queue
import socket
import struct
import threading
import time
from concurrent.futures import ThreadPoolExecutor

from .store import (INITIALIZED, NODE_ADDED, NODE_REMOVED, NODE_UPDATED, BadVersionError, NodeExistsError,
                    NoNodeError, NotEmptyError, Stat, _norm, _parent)

# op codes
CREATE, DELETE, EXISTS, GET_DATA, SET_DATA, GET_CHILDREN, PING, CLOSE = 1, 2, 3, 4, 5, 8, 11, -11
# error codes
OK, NONODE, BADVERSION, NODEEXISTS, NOTEMPTY, SESSIONEXPIRED = 0, -101, -103, -110, -111, -112
# flags / events
EPHEMERAL, SEQUENTIAL = 1, 2
EV_CREATED, EV_DELETED, EV_DATA, EV_CHILDREN = 1, 2, 3, 4
WORLD_ANYONE_ALL = [(31, "world", "anyone")]

STAT = struct.Struct(">qqqqiiiqiiq")          # czxid mzxid ctime mtime version cversion aversion owner len nkids pzxid


class ZkError(RuntimeError):
    def __init__(self, code: int, path: str = ""):
        super().__init__(f"zookeeper error {code} {path}")
        self.code = code


def raise_for(code: int, path: str):
    if code == NONODE:
        raise NoNodeError(path)
    if code == NODEEXISTS:
        raise NodeExistsError(path)
    if code == BADVERSION:
        raise BadVersionError(path)
    if code == NOTEMPTY:
        raise NotEmptyError(path)
    raise ZkError(code, path)


# ---------------------------------------------------------------------------------- jute
class W:
    def __init__(self):
        self.parts = []

    def int(self, v):
        self.parts.append(struct.pack(">i", v))
        return self

    def long(self, v):
        self.parts.append(struct.pack(">q", v))
        return self

    def bool(self, v):
        self.parts.append(b"\x01" if v else b"\x00")
        return self

    def buffer(self, b: bytes | None):
        if b is None:
            return self.int(-1)
        self.int(len(b))
        self.parts.append(bytes(b))
        return self

    def string(self, s: str | None):
        return self.buffer(None if s is None else s.encode())

    def acl(self, acls):
        self.int(len(acls))
        for perms, scheme, ident in acls:
            self.int(perms).string(scheme).string(ident)
        return self

    def strings(self, xs):
        self.int(len(xs))
        for x in xs:
            self.string(x)
        return self

    def bytes(self) -> bytes:
        return b"".join(self.parts)

    def frame(self) -> bytes:
        b = self.bytes()
        return struct.pack(">i", len(b)) + b


class R:
    def __init__(self, b: bytes, pos: int = 0):
        self.b, self.pos = b, pos

    def int(self):
        (v,) = struct.unpack_from(">i", self.b, self.pos)
        self.pos += 4
        return v

    def long(self):
        (v,) = struct.unpack_from(">q", self.b, self.pos)
        self.pos += 8
        return v

    def bool(self):
        v = self.b[self.pos] != 0
        self.pos += 1
        return v

    def buffer(self):
        n = self.int()
        if n < 0:
            return None
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return bytes(v)

    def string(self):
        v = self.buffer()
        return None if v is None else v.decode()

    def strings(self):
        return [self.string() for _ in range(self.int())]

    def stat(self):
        v = STAT.unpack_from(self.b, self.pos)
        self.pos += STAT.size
        return v

    def acl(self):
        return [(self.int(), self.string(), self.string()) for _ in range(self.int())]


def recv_exact(sock, n):
    parts, got = [], 0
    while got < n:
        b = sock.recv(min(n - got, 1 << 20))
        if not b:
            raise ConnectionError("connection closed")
        parts.append(b)
        got += len(b)
    return b"".join(parts)


def recv_frame(sock) -> bytes:
    (n,) = struct.unpack(">i", recv_exact(sock, 4))
    if n < 0 or n > (64 << 20):
        raise ZkError(0, f"bad frame length {n}")
    return recv_exact(sock, n)


def to_stat(st) -> Stat:
    czxid, mzxid, ctime, mtime, version, cversion, aversion, owner, dlen, nkids, pzxid = st
    return Stat(version=version, ctime=ctime / 1000.0, mtime=mtime / 1000.0,
                ephemeral_owner=(f"{owner:x}" if owner else None), num_children=nkids)


# ---------------------------------------------------------------------------------- session
class ZkSession:
    """One ZooKeeper session on one TCP connection: pipelined requests matched by xid, a reader
    thread, pings at a third of the negotiated timeout, watch events to ``on_event(type, path)``."""

    def __init__(self, host: str, port: int, chroot: str = "", timeout_ms: int = 10000, on_event=None):
        self.chroot = chroot.rstrip("/")
        self.sock = socket.create_connection((host, port), timeout=30)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock.sendall(W().int(0).long(0).int(timeout_ms).long(0).buffer(b"\0" * 16).bool(False).frame())
        r = R(recv_frame(self.sock))
        r.int()
        self.timeout_ms = r.int()
        self.session_id = r.long()
        if self.timeout_ms <= 0:
            raise ZkError(SESSIONEXPIRED, "session rejected")
        self.sock.settimeout(None)
        self.on_event = on_event
        self._xid = 0
        self._send_lock = threading.Lock()
        self._pending: dict[int, queue.Queue] = {}
        self._closed = threading.Event()
        threading.Thread(target=self._reader, daemon=True, name="zk-reader").start()
        threading.Thread(target=self._pinger, daemon=True, name="zk-ping").start()

    def path(self, p: str) -> str:
        p = _norm(p)
        return (self.chroot + p) if p != "/" else (self.chroot or "/")

    def unpath(self, p: str) -> str:
        if self.chroot and p.startswith(self.chroot):
            p = p[len(self.chroot):] or "/"
        return p

    def _reader(self):
        try:
            while not self._closed.is_set():
                r = R(recv_frame(self.sock))
                xid, _zxid, err = r.int(), r.long(), r.int()
                if xid == -1:                              # watch notification
                    etype, _state, path = r.int(), r.int(), r.string()
                    if self.on_event and etype > 0:
                        self.on_event(etype, self.unpath(path))
                    continue
                if xid == -2:                              # ping reply
                    continue
                q = self._pending.pop(xid, None)
                if q is not None:
                    q.put((err, r))
        except (ConnectionError, OSError, struct.error):
            pass
        finally:
            self._closed.set()
            for q in list(self._pending.values()):
                q.put((SESSIONEXPIRED, None))

    def _pinger(self):
        period = max(0.2, self.timeout_ms / 3000.0)
        while not self._closed.wait(period):
            try:
                with self._send_lock:
                    self.sock.sendall(W().int(-2).int(PING).frame())
            except OSError:
                return

    def call(self, op: int, body: W):
        if self._closed.is_set():
            raise ZkError(SESSIONEXPIRED, "session closed")
        q: queue.Queue = queue.Queue(1)
        with self._send_lock:
            self._xid += 1
            xid = self._xid
            self._pending[xid] = q
            w = W().int(xid).int(op)
            w.parts += body.parts
            self.sock.sendall(w.frame())
        err, r = q.get(timeout=30)
        return err, r

    def close(self):
        if self._closed.is_set():
            return
        try:
            self.call(CLOSE, W())
        except (ZkError, OSError, queue.Empty):
            pass
        self._closed.set()
        try:
            self.sock.close()
        except OSError:
            pass


# ---------------------------------------------------------------------------------- coordination
class ZooKeeperCoordination:
    """The coordination surface of :class:`~sitewhere_amd.coord.store.Coordination` on ZooKeeper.

    ``ZooKeeperCoordination("zk1:2181,zk2:2181/sitewhere")`` -- the chroot is the namespace."""

    def __init__(self, connect: str, timeout_ms: int = 10000, watch_threads: int = 3):
        hosts, _, chroot = connect.partition("/")
        self.hosts = [(h, int(p)) for h, p in (x.rsplit(":", 1) for x in hosts.split(","))]
        self.chroot = "/" + chroot if chroot else ""
        self.timeout_ms = timeout_ms
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self._pool = ThreadPoolExecutor(max_workers=watch_threads, thread_name_prefix="zk-watch")
        self._trees: list[_TreeCache] = []
        self._sessions: dict[str, ZkSession] = {}
        if self.chroot:                                    # make sure the namespace exists
            boot = self._connect("")
            try:
                acc = ""
                for part in self.chroot.strip("/").split("/"):
                    acc += "/" + part
                    err, _ = boot.call(CREATE, W().string(acc).buffer(b"").acl(WORLD_ANYONE_ALL).int(0))
                    if err not in (OK, NODEEXISTS):
                        raise_for(err, acc)
            finally:
                boot.close()
        self.main = self._connect(self.chroot)

    def _connect(self, chroot) -> ZkSession:
        last = None
        for h, p in self.hosts:
            try:
                return ZkSession(h, p, chroot, self.timeout_ms, self._on_event)
            except OSError as e:
                last = e
        raise ConnectionError(f"no ZooKeeper server reachable: {last}")

    def _on_event(self, etype, path):
        with self._cond:
            self._cond.notify_all()
        for t in list(self._trees):
            self._pool.submit(t.on_event, etype, path)

    def _s(self, session: str | None) -> ZkSession:
        return self._sessions.get(session, self.main) if session else self.main

    # sessions
    def open_session(self) -> str:
        s = self._connect(self.chroot)
        sid = f"{s.session_id:x}"
        self._sessions[sid] = s
        return sid

    def close_session(self, session: str):
        s = self._sessions.pop(session, None)
        if s is not None:
            s.close()

    # CRUD
    def create(self, path: str, data: bytes = b"", ephemeral: bool = False, sequential: bool = False,
               make_parents: bool = True, session: str | None = None) -> str:
        path = _norm(path)
        s = self._s(session)
        flags = (EPHEMERAL if ephemeral else 0) | (SEQUENTIAL if sequential else 0)
        for _ in range(2):
            err, r = s.call(CREATE, W().string(s.path(path)).buffer(bytes(data)).acl(WORLD_ANYONE_ALL).int(flags))
            if err == OK:
                return s.unpath(r.string())
            if err == NONODE and make_parents and path != "/":
                self.ensure(_parent(path))
                continue
            raise_for(err, path)
        raise_for(err, path)

    def ensure(self, path: str, data: bytes = b"") -> str:
        path = _norm(path)
        if path == "/":
            return path
        try:
            return self.create(path, data)
        except NodeExistsError:
            return path

    def exists(self, path: str, watch: bool = False):
        s = self.main
        err, r = s.call(EXISTS, W().string(s.path(path)).bool(watch))
        if err == NONODE:
            return None
        if err:
            raise_for(err, path)
        return to_stat(r.stat())

    def get(self, path: str, watch: bool = False) -> tuple[bytes, Stat]:
        s = self.main
        err, r = s.call(GET_DATA, W().string(s.path(path)).bool(watch))
        if err:
            raise_for(err, path)
        data = r.buffer() or b""
        return data, to_stat(r.stat())

    def get_data(self, path: str, default: bytes | None = None):
        try:
            return self.get(path)[0]
        except NoNodeError:
            return default

    def set(self, path: str, data: bytes, version: int = -1) -> Stat:
        s = self.main
        err, r = s.call(SET_DATA, W().string(s.path(path)).buffer(bytes(data)).int(version))
        if err:
            raise_for(err, path)
        return to_stat(r.stat())

    def put(self, path: str, data: bytes):
        try:
            self.set(path, data)
        except NoNodeError:
            try:
                self.create(path, data)
            except NodeExistsError:
                self.set(path, data)

    def delete(self, path: str, version: int = -1, recursive: bool = False):
        path = _norm(path)
        if recursive:
            for c in self.children(path):
                try:
                    self.delete(path.rstrip("/") + "/" + c, recursive=True)
                except NoNodeError:
                    pass
        s = self.main
        err, _ = s.call(DELETE, W().string(s.path(path)).int(version))
        if err:
            raise_for(err, path)

    def children(self, path: str, watch: bool = False) -> list[str]:
        s = self.main
        err, r = s.call(GET_CHILDREN, W().string(s.path(path)).bool(watch))
        if err:
            raise_for(err, path)
        return sorted(r.strings())

    def walk(self, prefix: str = "/") -> list[str]:
        prefix = _norm(prefix)
        out = []
        stack = [prefix]
        while stack:
            p = stack.pop()
            try:
                kids = self.children(p)
            except NoNodeError:
                continue
            out.append(p)
            stack += [p.rstrip("/") + "/" + k for k in kids]
        return sorted(out)

    def wait_for(self, path: str, timeout_s: float) -> bool:
        end = time.time() + timeout_s
        while True:
            if self.exists(path, watch=True) is not None:
                return True
            left = end - time.time()
            if left <= 0:
                return False
            with self._cond:
                self._cond.wait(min(left, 0.5))

    def watch_tree(self, prefix: str, callback, initial: bool = True):
        t = _TreeCache(self, _norm(prefix), callback)
        self._trees.append(t)
        if initial:
            self._pool.submit(t.start, True)
        else:
            # load the current tree before returning: a node created after this call must fire
            # NODE_ADDED.  Loading in the background let a node created between the caller's own
            # listing and the cache's first read be absorbed silently into the initial state (a
            # tenant bootstrapped in that window never started an engine).
            t.start(False)

        def cancel():
            if t in self._trees:
                self._trees.remove(t)
            t.cancelled = True
        return cancel

    def close(self):
        for s in list(self._sessions.values()):
            s.close()
        self._sessions.clear()
        self.main.close()
        self._pool.shutdown(wait=False)


class _TreeCache:
    """Curator TreeCache semantics over one-shot watches (ConfigurationMonitor.java:69-125)."""

    def __init__(self, zk: ZooKeeperCoordination, prefix: str, callback):
        self.zk, self.prefix, self.cb = zk, prefix, callback
        self.nodes: dict[str, bytes] = {}
        self.lock = threading.RLock()
        self.cancelled = False

    def _under(self, p: str) -> bool:
        return p == self.prefix or p.startswith(self.prefix.rstrip("/") + "/")

    def _load(self, path: str, fire: bool):
        try:
            data, _ = self.zk.get(path, watch=True)
            kids = self.zk.children(path, watch=True)
        except NoNodeError:
            self.zk.exists(path, watch=True)            # learn when it appears
            return
        new = path not in self.nodes
        old = self.nodes.get(path)
        self.nodes[path] = data
        if fire and (new or old != data):
            self.cb(NODE_ADDED if new else NODE_UPDATED, path, data)
        for k in kids:
            c = path.rstrip("/") + "/" + k
            if c not in self.nodes:
                self._load(c, fire)

    def start(self, initial: bool):
        with self.lock:
            self._load(self.prefix, initial)
        if initial:
            self.cb(INITIALIZED, self.prefix, None)

    def on_event(self, etype: int, path: str):
        if self.cancelled or not self._under(path):
            return
        with self.lock:
            if etype == EV_DELETED:
                gone = sorted((p for p in self.nodes if p == path or p.startswith(path.rstrip("/") + "/")),
                              key=len, reverse=True)
                for p in gone:
                    del self.nodes[p]
                    self.cb(NODE_REMOVED, p, None)
                if path == self.prefix:
                    self.zk.exists(path, watch=True)
            elif etype in (EV_CREATED, EV_CHILDREN):
                self._load(path, True)
            elif etype == EV_DATA:
                try:
                    data, _ = self.zk.get(path, watch=True)
                except NoNodeError:
                    return
                if self.nodes.get(path) != data:
                    new = path not in self.nodes
                    self.nodes[path] = data
                    self.cb(NODE_ADDED if new else NODE_UPDATED, path, data)
