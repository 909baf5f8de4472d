"""Hierarchical coordination store (the ZooKeeper + Curator layer, rebuilt).

Reference usage:
  * ``ZookeeperManager.java:30-80`` -- namespaced client, retries
  * ``ConfigurationMonitor.java:40-239`` -- Curator TreeCache over ``/<instance>/conf`` dispatching
    INITIALIZED / ADDED / UPDATED / REMOVED on a 3-thread pool
  * ``BootstrapTenantEngineOperation.java:57-117`` -- ``InterProcessMutex`` + ``bootstrapped`` markers
  * ``ZookeeperScriptManagement.java`` -- versioned script content in znodes
Semantics kept: versioned set (optimistic concurrency), ephemeral nodes bound to a session,
sequential nodes, persistent tree watches, mutex recipe by lowest ephemeral-sequential child.
Backends: :class:`Coordination` (in-memory, optionally snapshotted to a JSON file for durability);
:mod:`sitewhere_amd.coord.net` serves it over TCP for multi-process deployments.
"""
from __future__ import annotations

import base64
import json
import os
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field


class NoNodeError(KeyError):
    pass


class NodeExistsError(KeyError):
    pass


class BadVersionError(ValueError):
    pass


class NotEmptyError(ValueError):
    pass


@dataclass
class Stat:
    version: int = 0
    ctime: float = 0.0
    mtime: float = 0.0
    ephemeral_owner: str | None = None
    num_children: int = 0


@dataclass
class _Node:
    data: bytes = b""
    stat: Stat = field(default_factory=Stat)
    children: set = field(default_factory=set)
    seq: int = 0


NODE_ADDED, NODE_UPDATED, NODE_REMOVED, INITIALIZED = "NODE_ADDED", "NODE_UPDATED", "NODE_REMOVED", "INITIALIZED"


def _norm(path: str) -> str:
    if not path.startswith("/"):
        path = "/" + path
    if len(path) > 1 and path.endswith("/"):
        path = path[:-1]
    return path


def _parent(path: str) -> str:
    p = path.rsplit("/", 1)[0]
    return p or "/"


class Coordination:
    def __init__(self, snapshot_file: str | None = None, watch_threads: int = 3):
        self._lock = threading.RLock()
        self._cond = threading.Condition(self._lock)
        self._nodes: dict[str, _Node] = {"/": _Node(stat=Stat(ctime=time.time(), mtime=time.time()))}
        self._watches: list[tuple[str, callable]] = []
        self._pool = ThreadPoolExecutor(max_workers=watch_threads, thread_name_prefix="coord-watch")
        self._sessions: dict[str, float] = {}
        self.snapshot_file = snapshot_file
        if snapshot_file and os.path.exists(snapshot_file):
            self._load()

    # ------------------------------------------------------------------ sessions
    def open_session(self) -> str:
        s = uuid.uuid4().hex
        with self._lock:
            self._sessions[s] = time.time()
        return s

    def close_session(self, session: str):
        """Session loss: every ephemeral node it owns disappears (watches fire)."""
        with self._lock:
            self._sessions.pop(session, None)
            doomed = [p for p, n in self._nodes.items() if n.stat.ephemeral_owner == session]
        for p in sorted(doomed, key=len, reverse=True):
            try:
                self.delete(p, recursive=True)
            except NoNodeError:
                pass

    # ------------------------------------------------------------------ CRUD
    def create(self, path: str, data: bytes = b"", ephemeral: bool = False, sequential: bool = False,
               make_parents: bool = True, session: str | None = None) -> str:
        path = _norm(path)
        with self._lock:
            parent = _parent(path)
            if parent not in self._nodes:
                if not make_parents:
                    raise NoNodeError(parent)
                self.create(parent, b"", make_parents=True)
            pn = self._nodes[parent]
            if sequential:
                path = f"{path}{pn.seq:010d}"
                pn.seq += 1
            if path in self._nodes:
                raise NodeExistsError(path)
            now = time.time()
            self._nodes[path] = _Node(data=bytes(data), stat=Stat(0, now, now, session if ephemeral else None))
            pn.children.add(path.rsplit("/", 1)[1])
            pn.stat.num_children = len(pn.children)
            self._changed()
        self._fire(NODE_ADDED, path, bytes(data))
        return path

    def ensure(self, path: str, data: bytes = b"") -> str:
        try:
            return self.create(path, data)
        except NodeExistsError:
            return _norm(path)

    def exists(self, path: str) -> Stat | None:
        with self._lock:
            n = self._nodes.get(_norm(path))
            return None if n is None else Stat(**n.stat.__dict__)

    def get(self, path: str) -> tuple[bytes, Stat]:
        with self._lock:
            n = self._nodes.get(_norm(path))
            if n is None:
                raise NoNodeError(path)
            return n.data, Stat(**n.stat.__dict__)

    def get_data(self, path: str, default: bytes | None = None) -> bytes | None:
        try:
            return self.get(path)[0]
        except NoNodeError:
            return default

    def set(self, path: str, data: bytes, version: int = -1) -> Stat:
        path = _norm(path)
        with self._lock:
            n = self._nodes.get(path)
            if n is None:
                raise NoNodeError(path)
            if version >= 0 and version != n.stat.version:
                raise BadVersionError(f"{path}: expected v{version}, have v{n.stat.version}")
            n.data = bytes(data)
            n.stat.version += 1
            n.stat.mtime = time.time()
            st = Stat(**n.stat.__dict__)
            self._changed()
        self._fire(NODE_UPDATED, path, bytes(data))
        return st

    def put(self, path: str, data: bytes):
        """Create-or-set convenience."""
        try:
            self.set(path, data)
        except NoNodeError:
            try:
                self.create(path, data)
            except NodeExistsError:
                self.set(path, data)

    def delete(self, path: str, version: int = -1, recursive: bool = False):
        path = _norm(path)
        removed = []
        with self._lock:
            n = self._nodes.get(path)
            if n is None:
                raise NoNodeError(path)
            if n.children and not recursive:
                raise NotEmptyError(path)
            if version >= 0 and version != n.stat.version:
                raise BadVersionError(path)
            for p in sorted([p for p in self._nodes if p == path or p.startswith(path + "/")], key=len, reverse=True):
                removed.append(p)
                del self._nodes[p]
            pn = self._nodes.get(_parent(path))
            if pn is not None:
                pn.children.discard(path.rsplit("/", 1)[1])
                pn.stat.num_children = len(pn.children)
            self._changed()
        for p in removed:
            self._fire(NODE_REMOVED, p, None)

    def children(self, path: str) -> list[str]:
        with self._lock:
            n = self._nodes.get(_norm(path))
            if n is None:
                raise NoNodeError(path)
            return sorted(n.children)

    def walk(self, prefix: str = "/") -> list[str]:
        prefix = _norm(prefix)
        with self._lock:
            return sorted(p for p in self._nodes if p == prefix or p.startswith(prefix.rstrip("/") + "/"))

    # ------------------------------------------------------------------ watches
    def watch_tree(self, prefix: str, callback, initial: bool = True) -> callable:
        """TreeCache-like: ADDED for existing nodes (if initial), then INITIALIZED, then live events."""
        prefix = _norm(prefix)
        entry = (prefix, callback)
        with self._lock:
            self._watches.append(entry)
            existing = [(p, self._nodes[p].data) for p in self.walk(prefix)] if initial else []

        def _init():
            for p, d in existing:
                callback(NODE_ADDED, p, d)
            callback(INITIALIZED, prefix, None)

        self._pool.submit(_init)

        def cancel():
            with self._lock:
                if entry in self._watches:
                    self._watches.remove(entry)
        return cancel

    def _fire(self, kind, path, data):
        with self._lock:
            ws = [cb for pre, cb in self._watches if path == pre or path.startswith(pre.rstrip("/") + "/")]
            self._cond.notify_all()
        for cb in ws:
            self._pool.submit(cb, kind, path, data)

    def wait_for(self, path: str, timeout_s: float) -> bool:
        """Block until ``path`` exists (bootstrap markers, ``InitializeTenantEngineOperation``)."""
        end = time.time() + timeout_s
        with self._cond:
            while _norm(path) not in self._nodes:
                left = end - time.time()
                if left <= 0:
                    return False
                self._cond.wait(left)
            return True

    # ------------------------------------------------------------------ durability
    def _changed(self):
        if self.snapshot_file:
            snap = {p: {"d": base64.b64encode(n.data).decode(), "v": n.stat.version, "c": n.stat.ctime,
                        "m": n.stat.mtime, "s": n.seq} for p, n in self._nodes.items() if not n.stat.ephemeral_owner}
            tmp = self.snapshot_file + ".tmp"
            with open(tmp, "w") as f:
                json.dump(snap, f)
            os.replace(tmp, self.snapshot_file)

    def _load(self):
        with open(self.snapshot_file) as f:
            snap = json.load(f)
        for p in sorted(snap, key=len):
            e = snap[p]
            n = _Node(base64.b64decode(e["d"]), Stat(e["v"], e["c"], e["m"]), set(), e.get("s", 0))
            self._nodes[p] = n
            if p != "/":
                par = self._nodes.get(_parent(p))
                if par is not None:
                    par.children.add(p.rsplit("/", 1)[1])
                    par.stat.num_children = len(par.children)

    def close(self):
        self._pool.shutdown(wait=False)


class InterProcessMutex:
    """Curator InterProcessMutex: ephemeral-sequential lock nodes, lowest sequence owns the lock."""

    def __init__(self, coord: Coordination, path: str, session: str | None = None):
        self.coord, self.path = coord, _norm(path)
        self.session = session or coord.open_session()
        self._own_session = session is None
        self._node = None

    def acquire(self, timeout_s: float = 30.0) -> bool:
        self._node = self.coord.create(self.path + "/lock-", b"", ephemeral=True, sequential=True, session=self.session)
        name = self._node.rsplit("/", 1)[1]
        end = time.time() + timeout_s
        while True:
            kids = sorted(self.coord.children(self.path))
            if kids and kids[0] == name:
                return True
            left = end - time.time()
            if left <= 0:
                self.release()
                return False
            with self.coord._cond:
                self.coord._cond.wait(min(left, 0.1))

    def release(self):
        if self._node:
            try:
                self.coord.delete(self._node)
            except NoNodeError:
                pass
            self._node = None
        if self._own_session:
            pass

    def __enter__(self):
        if not self.acquire():
            raise TimeoutError(f"lock {self.path} not acquired")
        return self

    def __exit__(self, *a):
        self.release()
        return False
