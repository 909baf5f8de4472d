"""In-process ZooKeeper stand-in speaking the wire protocol of ``coord/zk.py``.

Sessions (ephemeral nodes removed when a session closes or stops pinging), versions, sequential
nodes (``%010d`` of the parent's child-create counter, as ZooKeeper does), and one-shot data /
exists / child watches delivered as notifications (xid -1).  For tests and single-node use.
"""
from __future__ import annotations

import itertools
import socket
import socketserver
import threading
import time

from .zk import (CLOSE, CREATE, DELETE, EPHEMERAL, EV_CHILDREN, EV_CREATED, EV_DATA, EV_DELETED, EXISTS, GET_CHILDREN,
                 GET_DATA, NODEEXISTS, NONODE, NOTEMPTY, BADVERSION, OK, PING, SEQUENTIAL, SET_DATA, STAT, R, W,
                 recv_frame)


class _Node:
    __slots__ = ("data", "czxid", "mzxid", "ctime", "mtime", "version", "cversion", "owner", "children", "seq")

    def __init__(self, data, zxid, owner):
        now = int(time.time() * 1000)
        self.data, self.czxid, self.mzxid, self.ctime, self.mtime = data, zxid, zxid, now, now
        self.version = self.cversion = 0
        self.owner = owner
        self.children: set = set()
        self.seq = 0

    def stat(self) -> bytes:
        return STAT.pack(self.czxid, self.mzxid, self.ctime, self.mtime, self.version, self.cversion, 0,
                         self.owner, len(self.data), len(self.children), self.mzxid)


class _Conn:
    def __init__(self, sock, sid, timeout_ms):
        self.sock, self.sid, self.timeout_ms = sock, sid, timeout_ms
        self.lock = threading.Lock()
        self.last = time.time()
        self.alive = True

    def send(self, payload: bytes):
        with self.lock:
            self.sock.sendall(payload)


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        srv: MiniZooKeeperServer = self.server.zk      # type: ignore[attr-defined]
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            r = R(recv_frame(sock))
            r.int()
            r.long()
            timeout = max(2000, min(r.int(), 60000))
            conn = srv._open(sock, timeout)
            conn.send(W().int(0).int(timeout).long(conn.sid).buffer(b"\0" * 16).bool(False).frame())
            while conn.alive:
                r = R(recv_frame(sock))
                xid, op = r.int(), r.int()
                conn.last = time.time()
                if op == PING:
                    conn.send(W().int(-2).long(srv.zxid).int(OK).frame())
                    continue
                if op == CLOSE:
                    srv._close(conn)
                    conn.send(W().int(xid).long(srv.zxid).int(OK).frame())
                    return
                err, body = srv.execute(conn, op, r)
                w = W().int(xid).long(srv.zxid).int(err)
                if err == OK and body is not None:
                    w.parts += body.parts
                conn.send(w.frame())
        except (ConnectionError, OSError):
            pass
        finally:
            c = srv._by_sock.get(sock)
            if c is not None:
                srv._close(c)


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class MiniZooKeeperServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 2181):
        self._srv = _Server((host, port), _Handler)
        self._srv.zk = self
        self.host, self.port = host, self._srv.server_address[1]
        self._lock = threading.RLock()
        self.nodes: dict[str, _Node] = {"/": _Node(b"", 0, 0)}
        self.zxid = 0
        self._sids = itertools.count(0x1000)
        self._conns: dict[int, _Conn] = {}
        self._by_sock: dict = {}
        self._dw: dict[str, set] = {}       # data / exists watches: path -> conns
        self._cw: dict[str, set] = {}       # child watches
        self._stop = threading.Event()

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def start(self):
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="mini-zk").start()
        threading.Thread(target=self._reaper, daemon=True, name="mini-zk-sessions").start()
        return self

    def stop(self):
        self._stop.set()
        self._srv.shutdown()
        self._srv.server_close()

    # sessions
    def _open(self, sock, timeout) -> _Conn:
        with self._lock:
            c = _Conn(sock, next(self._sids), timeout)
            self._conns[c.sid] = c
            self._by_sock[sock] = c
            return c

    def _close(self, conn: _Conn):
        with self._lock:
            if not conn.alive:
                return
            conn.alive = False
            self._conns.pop(conn.sid, None)
            self._by_sock.pop(conn.sock, None)
            for ws in list(self._dw.values()) + list(self._cw.values()):
                ws.discard(conn)
            doomed = sorted((p for p, n in self.nodes.items() if n.owner == conn.sid), key=len, reverse=True)
            for p in doomed:
                if p in self.nodes and not self.nodes[p].children:
                    self._delete(p)

    def _reaper(self):
        while not self._stop.wait(0.5):
            now = time.time()
            for c in list(self._conns.values()):
                if now - c.last > c.timeout_ms / 1000.0:
                    self._close(c)
                    try:
                        c.sock.close()
                    except OSError:
                        pass

    # watches
    def _notify(self, table, path, etype):
        for c in table.pop(path, set()):
            if c.alive:
                try:
                    c.send(W().int(-1).long(self.zxid).int(0).int(etype).int(3).string(path).frame())
                except OSError:
                    pass

    @staticmethod
    def _parent(p):
        return p.rsplit("/", 1)[0] or "/"

    def _delete(self, path):
        self.zxid += 1
        del self.nodes[path]
        par = self.nodes.get(self._parent(path))
        if par is not None:
            par.children.discard(path.rsplit("/", 1)[1])
            par.cversion += 1
        self._notify(self._dw, path, EV_DELETED)
        self._notify(self._cw, path, EV_DELETED)
        self._notify(self._cw, self._parent(path), EV_CHILDREN)

    # operations
    def execute(self, conn, op, r: R):
        with self._lock:
            if op == CREATE:
                path, data, _acl, flags = r.string(), r.buffer() or b"", r.acl(), r.int()
                par = self.nodes.get(self._parent(path))
                if par is None:
                    return NONODE, None
                if flags & SEQUENTIAL:
                    path = f"{path}{par.seq:010d}"
                if path in self.nodes:
                    return NODEEXISTS, None
                par.seq += 1
                self.zxid += 1
                self.nodes[path] = _Node(data, self.zxid, conn.sid if flags & EPHEMERAL else 0)
                par.children.add(path.rsplit("/", 1)[1])
                par.cversion += 1
                self._notify(self._dw, path, EV_CREATED)
                self._notify(self._cw, self._parent(path), EV_CHILDREN)
                return OK, W().string(path)
            if op == DELETE:
                path, version = r.string(), r.int()
                n = self.nodes.get(path)
                if n is None:
                    return NONODE, None
                if version >= 0 and version != n.version:
                    return BADVERSION, None
                if n.children:
                    return NOTEMPTY, None
                self._delete(path)
                return OK, None
            if op == EXISTS:
                path, watch = r.string(), r.bool()
                n = self.nodes.get(path)
                if watch:
                    self._dw.setdefault(path, set()).add(conn)
                if n is None:
                    return NONODE, None
                w = W()
                w.parts.append(n.stat())
                return OK, w
            if op == GET_DATA:
                path, watch = r.string(), r.bool()
                n = self.nodes.get(path)
                if n is None:
                    return NONODE, None
                if watch:
                    self._dw.setdefault(path, set()).add(conn)
                w = W().buffer(n.data)
                w.parts.append(n.stat())
                return OK, w
            if op == SET_DATA:
                path, data, version = r.string(), r.buffer() or b"", r.int()
                n = self.nodes.get(path)
                if n is None:
                    return NONODE, None
                if version >= 0 and version != n.version:
                    return BADVERSION, None
                self.zxid += 1
                n.data, n.version, n.mzxid, n.mtime = data, n.version + 1, self.zxid, int(time.time() * 1000)
                self._notify(self._dw, path, EV_DATA)
                w = W()
                w.parts.append(n.stat())
                return OK, w
            if op == GET_CHILDREN:
                path, watch = r.string(), r.bool()
                n = self.nodes.get(path)
                if n is None:
                    return NONODE, None
                if watch:
                    self._cw.setdefault(path, set()).add(conn)
                return OK, W().strings(sorted(n.children))
            return -6, None                               # UNIMPLEMENTED
