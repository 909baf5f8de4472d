"""Isolated script worker: extension-point scripts in a separate process under rlimits + seccomp.

Reference: Groovy scripts run inside the microservice JVM (``GroovyComponent.java:25-166``) with
full privileges.  ``ScriptRunner(isolation="process")`` (``runtime/scripting.py``) sends the
data-in / data-out entry points -- decoders, deduplicators, metadata extractors, command encoders
and routers, connector filters -- to this worker instead.  The worker

1. caps its address space, written file size (stderr), core dumps and open files (``resource.setrlimit``),
2. imports every module scripts may use (the allow-list of ``runtime/scripting.py``) and msgpack,
3. locks itself with ``sw_sandbox_lock`` (``csrc/native/swsandbox.cpp``): a seccomp-BPF allow-list
   of compute / memory / pipe syscalls; ``open``, sockets, ``execve``, ``fork`` ... fail with EPERM,

then serves length-prefixed msgpack requests on stdin/stdout.  Scripts are compiled with the same
restricted builtins and source check as in-process ones and cached per (name, source).  A call
that outlives its time limit kills the worker; the next call starts a fresh one.  Microservices
start the worker when they are created (``ensure_started``), before a tenant engine opens a GPU in
the process: a replacement after a timeout is forked from a process that may have opened one.
"""
from __future__ import annotations

import os
import select
import struct
import subprocess
import sys
import threading
import time

_HDR = struct.Struct("<I")
_PLAIN = (type(None), bool, int, float, str, bytes)


def is_plain(v, depth: int = 0) -> bool:
    """True when ``v`` is msgpack-plain data (what crosses to the worker unchanged)."""
    if depth > 32:
        return False
    if isinstance(v, _PLAIN):
        return True
    if isinstance(v, (bytearray, memoryview)):
        return True
    if isinstance(v, (list, tuple)):
        return all(is_plain(x, depth + 1) for x in v)
    if isinstance(v, dict):
        return all(isinstance(k, (str, int)) and is_plain(x, depth + 1) for k, x in v.items())
    return False


def _plain(v):
    if isinstance(v, (bytearray, memoryview)):
        return bytes(v)
    if isinstance(v, tuple):
        return [_plain(x) for x in v]
    if isinstance(v, list):
        return [_plain(x) for x in v]
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    return v


def _read_exact(fd: int, n: int, deadline: float | None) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        if deadline is not None:
            left = deadline - time.monotonic()
            if left <= 0 or not select.select([fd], [], [], left)[0]:
                raise TimeoutError
        chunk = os.read(fd, n - len(buf))
        if not chunk:
            raise EOFError("script worker closed its pipe")
        buf += chunk
    return bytes(buf)


class SandboxedScripts:
    """Client side: one worker process, calls serialised (the worker is single-threaded)."""

    def __init__(self, memory_mb: int = 1024, require_seccomp: bool = True):
        self.memory_mb, self.require_seccomp = memory_mb, require_seccomp
        self._p: subprocess.Popen | None = None
        self._lock = threading.Lock()
        self.mode = None
        self.restarts = 0

    def ensure_started(self):
        with self._lock:
            if self._p is None or self._p.poll() is not None:
                self._start()

    def _start(self):
        import msgpack
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        self._p = subprocess.Popen([sys.executable, "-u", "-m", "sitewhere_amd.runtime.script_sandbox",
                                    str(self.memory_mb)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                   cwd=root, env=env, close_fds=True)
        hello = msgpack.unpackb(self._recv(time.monotonic() + 60), raw=False)
        self.mode = hello["sandbox"]
        if self.require_seccomp and self.mode != "seccomp":
            self._kill()
            raise RuntimeError(f"script sandbox unavailable: {hello.get('detail')}")

    def _recv(self, deadline):
        fd = self._p.stdout.fileno()
        n, = _HDR.unpack(_read_exact(fd, 4, deadline))
        return _read_exact(fd, n, deadline)

    def _kill(self):
        p, self._p = self._p, None
        if p is not None:
            p.kill()
            p.wait()

    def call(self, source: str, entry: str, args=(), kwargs=None, name: str = "<script>", timeout_s: float = 5.0):
        import msgpack

        from ..core.errors import SiteWhereException
        req = msgpack.packb({"src": source, "entry": entry, "name": name, "args": _plain(list(args)),
                             "kwargs": _plain(dict(kwargs or {}))}, use_bin_type=True)
        with self._lock:
            if self._p is None or self._p.poll() is not None:
                self._start()
            try:
                self._p.stdin.write(_HDR.pack(len(req)) + req)
                self._p.stdin.flush()
                resp = msgpack.unpackb(self._recv(time.monotonic() + timeout_s), raw=False)
            except TimeoutError:
                self.restarts += 1
                self._kill()
                raise SiteWhereException(f"script {name}.{entry} timed out (sandbox worker killed)") from None
            except (EOFError, BrokenPipeError, OSError) as e:
                self.restarts += 1
                self._kill()
                raise SiteWhereException(f"script {name}.{entry}: sandbox worker died ({e})") from None
        if "err" in resp:
            raise SiteWhereException(f"script {name}.{entry}: {resp['err']}")
        return resp["ok"]

    def close(self):
        with self._lock:
            if self._p is not None:
                try:
                    self._p.stdin.close()
                    self._p.wait(2)
                except Exception:  # noqa: BLE001
                    pass
                self._kill()


# ------------------------------------------------------------------------------------ worker
def _limit(memory_mb: int):
    """Soft AND hard limits: code escaping the restricted namespace cannot raise them again (the
    seccomp filter also refuses prlimit64 writes, csrc/native/swsandbox.cpp)."""
    import resource
    for lim, v in ((resource.RLIMIT_AS, memory_mb << 20), (resource.RLIMIT_FSIZE, 64 << 20), (resource.RLIMIT_CORE, 0),
                   (resource.RLIMIT_NOFILE, 64)):
        try:
            soft, hard = resource.getrlimit(lim)
            v = v if hard == resource.RLIM_INFINITY else min(v, hard)
            resource.setrlimit(lim, (v, v))
        except (ValueError, OSError):
            pass


def _lock() -> tuple[str, str]:
    import ctypes
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(here, "_lib", "libswnative.so")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        return "rlimits", f"libswnative.so not loadable: {e}"
    rc = lib.sw_sandbox_lock()
    if rc != 0:
        return "rlimits", f"seccomp refused (rc={rc}, errno={ctypes.get_errno()})"
    return "seccomp", ""


def _serve(memory_mb: int):
    import msgpack

    from .scripting import _ALLOWED_MODULES, _SAFE_BUILTINS, _restricted_import, check_source
    for m in sorted(_ALLOWED_MODULES):
        __import__(m)
    import _strptime  # noqa: F401 -- time.strptime imports it lazily
    import encodings.idna  # noqa: F401
    fin = sys.stdin.buffer.raw
    proto = os.dup(1)               # the protocol keeps the pipe; a script's print() goes to stderr
    os.dup2(2, 1)
    _limit(memory_mb)
    mode, detail = _lock()

    def send(obj):
        b = msgpack.packb(obj, use_bin_type=True, default=repr)
        out = _HDR.pack(len(b)) + b
        while out:
            out = out[os.write(proto, out):]

    send({"sandbox": mode, "detail": detail})
    cache: dict = {}
    while True:
        try:
            n, = _HDR.unpack(_read_exact(fin.fileno(), 4, None))
            req = msgpack.unpackb(_read_exact(fin.fileno(), n, None), raw=False)
        except EOFError:
            return
        try:
            key = (req["name"], req["src"])
            ns = cache.get(key)
            if ns is None:
                check_source(req["src"], req["name"])
                ns = {"__builtins__": dict(_SAFE_BUILTINS, __import__=_restricted_import), "__name__": req["name"]}
                exec(compile(req["src"], req["name"], "exec"), ns)  # noqa: S102 -- sandboxed worker
                if len(cache) > 256:
                    cache.clear()
                cache[key] = ns
            fn = ns.get(req["entry"])
            if not callable(fn):
                raise NameError(f"script does not define {req['entry']}()")
            send({"ok": _plain(fn(*req["args"], **req["kwargs"]))})
        except BaseException as e:  # noqa: BLE001 -- report any script failure, keep serving
            send({"err": f"{type(e).__name__}: {e}"})


if __name__ == "__main__":
    _serve(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
