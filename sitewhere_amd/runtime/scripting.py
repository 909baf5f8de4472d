"""Versioned user scripts stored in the coordination tree, executed in a restricted interpreter.

Reference: ``sitewhere-microservice/.../scripting/ZookeeperScriptManagement.java:55-287`` (create /
update / clone / activate / delete versions, content in znodes), ``GroovyComponent.java:25-166`` and
``GroovyConfiguration.java:33-90`` (script engine on a 3-thread pool), script templates served by
management gRPC ``GetScriptTemplates`` / ``GetScriptTemplateContent``.  Groovy decoders, encoders,
filters, routers and dataset initializers become Python scripts; each script defines the entry
point its extension point expects (``decode(payload, metadata)``, ``encode(execution)``,
``filter(event)``, ``route(execution)``, ``initialize(api)``...).

Trust model (the reference runs Groovy with full JVM privileges):

* ``isolation="thread"`` (default): scripts run in this process with restricted builtins, a module
  allow-list and a source check (``check_source``: no ``_``-prefixed attributes or dunder names, no
  frame / code / traceback introspection attributes).  That stops accidents and the well-known
  ``().__class__.__base__.__subclasses__()`` escape, but CPython offers no in-process sandbox:
  scripts in this mode are tenant-administrator code and are trusted like the reference's Groovy.
* ``isolation="process"`` (``SITEWHERE_SCRIPT_ISOLATION=process``): data-in / data-out entry points
  (decoders, deduplicators, metadata extractors, command encoders / routers, connector filters)
  run in a worker process (``runtime/script_sandbox.py``) under rlimits and a seccomp-BPF syscall
  allow-list (``csrc/native/swsandbox.cpp``): no files, sockets, exec or fork, whatever the script
  does to the interpreter.  A call that times out kills the worker.  Entry points handed live API
  objects (rule scripts, REST poll scripts, dataset initializers) always run in-process.
"""
from __future__ import annotations

import builtins
import json
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from concurrent.futures import TimeoutError as FutTimeout

from ..core.errors import ErrorCode, NotFoundException, SiteWhereException
from ..models.domain import ScriptMetadata

_SAFE_BUILTINS = {n: getattr(builtins, n) for n in (
    "abs", "all", "any", "bool", "bytes", "bytearray", "chr", "dict", "divmod", "enumerate", "filter", "float",
    "format", "frozenset", "hash", "hex", "int", "isinstance", "issubclass", "iter", "len", "list", "map", "max",
    "min", "next", "oct", "ord", "pow", "print", "range", "repr", "reversed", "round", "set", "slice", "sorted",
    "str", "sum", "tuple", "zip", "Exception", "ValueError", "KeyError", "TypeError", "IndexError",
    "ArithmeticError", "ZeroDivisionError", "True", "False", "None")}
_ALLOWED_MODULES = {"json", "math", "struct", "re", "time", "datetime", "base64", "binascii", "hashlib"}


def _restricted_import(name, globals=None, locals=None, fromlist=(), level=0):
    if name.split(".")[0] not in _ALLOWED_MODULES:
        raise ImportError(f"module {name!r} is not available to scripts")
    return __import__(name, globals, locals, fromlist, level)


# attributes that reach frames, code objects or module globals without a leading underscore
_DENIED_ATTRS = frozenset((
    "gi_frame", "gi_code", "gi_yieldfrom", "cr_frame", "cr_code", "cr_await", "ag_frame", "ag_code", "ag_await",
    "f_back", "f_globals", "f_locals", "f_builtins", "f_code", "f_trace", "tb_frame", "tb_next", "func_globals",
    "co_code", "co_consts", "mro"))


def check_source(source: str, name: str = "<script>"):
    """Reject script source that reaches interpreter internals (see the module docstring): any
    ``_``-prefixed attribute, any dunder name other than ``__name__``, and the introspection
    attributes in ``_DENIED_ATTRS``.  Raises ``SiteWhereException`` naming the line."""
    import ast
    try:
        tree = ast.parse(source, name)
    except SyntaxError as e:
        raise SiteWhereException(f"script {name}: {e}") from e
    for node in ast.walk(tree):
        bad = None
        if isinstance(node, ast.Attribute) and (node.attr.startswith("_") or node.attr in _DENIED_ATTRS):
            bad = node.attr
        elif isinstance(node, ast.Name) and node.id.startswith("__") and node.id != "__name__":
            bad = node.id
        elif isinstance(node, (ast.FunctionDef, ast.ClassDef)) and node.name.startswith("__"):
            bad = node.name
        if bad is not None:
            raise SiteWhereException(f"script {name} line {node.lineno}: access to {bad!r} is not allowed")


class ScriptManagement:
    """CRUD + versioning of scripts under ``/<instance>/scripts/<scope>/<microservice>``."""

    def __init__(self, coord, root: str):
        self.coord = coord
        self.root = root.rstrip("/")

    def _base(self, scope: str, ms: str) -> str:
        return f"{self.root}/{scope}/{ms}"

    def _meta_path(self, scope, ms, sid):
        return f"{self._base(scope, ms)}/{sid}/meta"

    def list_scripts(self, scope: str, ms: str) -> list[ScriptMetadata]:
        try:
            ids = self.coord.children(self._base(scope, ms))
        except KeyError:
            return []
        return [self.get_script(scope, ms, i) for i in ids]

    def get_script(self, scope, ms, sid) -> ScriptMetadata:
        d = self.coord.get_data(self._meta_path(scope, ms, sid))
        if d is None:
            raise NotFoundException(ErrorCode.InvalidScript, f"script {sid}")
        return ScriptMetadata.from_dict(json.loads(d))

    def _save(self, scope, ms, meta: ScriptMetadata):
        self.coord.put(self._meta_path(scope, ms, meta.id), json.dumps(meta.to_dict()).encode())

    def create_script(self, scope, ms, sid: str, name: str, content: str, description: str = "",
                      interpreter: str = "python") -> ScriptMetadata:
        ver = uuid.uuid4().hex[:12]
        meta = ScriptMetadata(id=sid, name=name, description=description, interpreter_type=interpreter,
                              active_version=ver, versions=[{"versionId": ver, "comment": "initial",
                                                             "createdDate": int(time.time() * 1000)}])
        self.coord.put(f"{self._base(scope, ms)}/{sid}/versions/{ver}", content.encode())
        self._save(scope, ms, meta)
        return meta

    def get_content(self, scope, ms, sid, version: str | None = None) -> str:
        meta = self.get_script(scope, ms, sid)
        v = version or meta.active_version
        d = self.coord.get_data(f"{self._base(scope, ms)}/{sid}/versions/{v}")
        if d is None:
            raise NotFoundException(ErrorCode.InvalidScript, f"script {sid} version {v}")
        return d.decode()

    def update_script(self, scope, ms, sid, version: str, content: str, name=None, description=None):
        meta = self.get_script(scope, ms, sid)
        if not any(v["versionId"] == version for v in meta.versions):
            raise NotFoundException(ErrorCode.InvalidScript, f"version {version}")
        self.coord.put(f"{self._base(scope, ms)}/{sid}/versions/{version}", content.encode())
        if name is not None:
            meta.name = name
        if description is not None:
            meta.description = description
        self._save(scope, ms, meta)
        return meta

    def clone_script(self, scope, ms, sid, version: str, comment: str = "") -> ScriptMetadata:
        content = self.get_content(scope, ms, sid, version)
        meta = self.get_script(scope, ms, sid)
        ver = uuid.uuid4().hex[:12]
        self.coord.put(f"{self._base(scope, ms)}/{sid}/versions/{ver}", content.encode())
        meta.versions.append({"versionId": ver, "comment": comment or f"clone of {version}",
                              "createdDate": int(time.time() * 1000)})
        self._save(scope, ms, meta)
        return meta

    def activate_script(self, scope, ms, sid, version: str) -> ScriptMetadata:
        meta = self.get_script(scope, ms, sid)
        if not any(v["versionId"] == version for v in meta.versions):
            raise NotFoundException(ErrorCode.InvalidScript, f"version {version}")
        meta.active_version = version
        self._save(scope, ms, meta)
        return meta

    def delete_script(self, scope, ms, sid) -> ScriptMetadata:
        meta = self.get_script(scope, ms, sid)
        self.coord.delete(f"{self._base(scope, ms)}/{sid}", recursive=True)
        return meta


class ScriptRunner:
    """Compile + run scripts in a restricted namespace on a small pool with a time limit; with
    ``isolation="process"`` the data-only entry points go to the sandboxed worker instead."""

    def __init__(self, threads: int = 3, timeout_s: float = 5.0, isolation: str | None = None):
        import os
        self.pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="script")
        self.timeout = timeout_s
        self._cache: dict[str, dict] = {}
        self._lock = threading.Lock()
        self.isolation = isolation or os.environ.get("SITEWHERE_SCRIPT_ISOLATION", "thread")
        if self.isolation not in ("thread", "process"):
            raise ValueError(f"script isolation {self.isolation!r}: expected 'thread' or 'process'")
        self._sandbox = None

    def compile(self, source: str, name: str = "<script>", extra_globals: dict | None = None) -> dict:
        key = f"{name}:{hash(source)}"
        with self._lock:
            ns = self._cache.get(key)
        if ns is None:
            ns = {"__builtins__": dict(_SAFE_BUILTINS, __import__=_restricted_import), "__name__": name}
            if extra_globals:
                ns.update(extra_globals)
            check_source(source, name)
            code = compile(source, name, "exec")
            exec(code, ns)  # noqa: S102 -- restricted builtins, module allow-list
            with self._lock:
                self._cache[key] = ns
        return ns

    def call(self, source: str, entry: str, *args, name: str = "<script>", extra_globals=None, **kwargs):
        if self.isolation == "process" and not extra_globals:
            from .script_sandbox import is_plain
            if is_plain(args) and is_plain(kwargs):
                return self.sandbox().call(source, entry, args, kwargs, name=name, timeout_s=self.timeout)
        ns = self.compile(source, name, extra_globals)
        fn = ns.get(entry)
        if not callable(fn):
            raise SiteWhereException(f"script {name} does not define {entry}()")
        fut = self.pool.submit(fn, *args, **kwargs)
        try:
            return fut.result(timeout=self.timeout)
        except FutTimeout as e:
            raise SiteWhereException(f"script {name}.{entry} timed out") from e

    def sandbox(self):
        with self._lock:
            if self._sandbox is None:
                from .script_sandbox import SandboxedScripts
                self._sandbox = SandboxedScripts()
            return self._sandbox

    def close(self):
        self.pool.shutdown(wait=False)
        if self._sandbox is not None:
            self._sandbox.close()


SCRIPT_TEMPLATES = {
    "event-sources": {
        "decoder.py": '"""Decode a raw payload into device requests."""\n\ndef decode(payload, metadata):\n'
                      '    import json\n    d = json.loads(payload)\n    return [{"deviceToken": d["device"], '
                      '"type": "DeviceMeasurement", "request": {"name": d["name"], "value": d["value"]}}]\n',
        "deduplicator.py": 'def is_duplicate(request):\n    return False\n',
    },
    "command-delivery": {
        "encoder.py": 'def encode(execution, nesting, assignment):\n    import json\n'
                      '    return json.dumps({"command": execution["command"]["name"], '
                      '"parameters": execution["parameters"]}).encode()\n',
        "router.py": 'def route(execution, device, assignment):\n    return "default"\n',
    },
    "outbound-connectors": {
        "filter.py": 'def filter(event, context):\n    """Return True to SKIP the event."""\n    return False\n',
        "connector.py": 'def process(event, context):\n    pass\n',
    },
    "instance-management": {
        "initializer.py": 'def initialize(api):\n    pass\n',
    },
}
