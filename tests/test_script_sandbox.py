"""Script isolation (``runtime/scripting.py`` trust model, ``runtime/script_sandbox.py``,
``csrc/native/swsandbox.cpp``).

Reference: Groovy scripts run in the microservice JVM with full privileges
(``GroovyComponent.java:25-166``).  Here in-process scripts are source-checked against interpreter
escapes, and ``isolation="process"`` runs extension-point scripts in a worker locked down by
rlimits + a seccomp-BPF syscall allow-list."""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

from sitewhere_amd.core.errors import SiteWhereException
from sitewhere_amd.runtime.scripting import ScriptRunner, check_source

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ESCAPES = [
    "x = ().__class__.__base__.__subclasses__()",
    "def g():\n    yield 1\ngen = g()\nf = gen.gi_frame.f_back",
    "b = __builtins__",
    "def f():\n    pass\nc = f.__code__",
    "try:\n    1/0\nexcept Exception as e:\n    t = e.__traceback__.tb_frame",
    "class __X:\n    pass",
]


@pytest.mark.parametrize("src", ESCAPES)
def test_source_check_rejects_interpreter_escapes(src):
    with pytest.raises(SiteWhereException, match="not allowed"):
        check_source(src)
    r = ScriptRunner()
    with pytest.raises(SiteWhereException):
        r.call(src + "\ndef decode(p, m):\n    return []\n", "decode", b"", {})
    r.close()


def test_source_check_allows_ordinary_scripts():
    check_source("import json\ndef decode(payload, md):\n    d = json.loads(payload)\n"
                 "    return [{'deviceToken': d['device'], 'name': __name__, 'n': len(d.keys())}]\n")


DECODER = '''
import json, math
def decode(payload, metadata):
    print("scripts may print: it goes to stderr, not the protocol pipe")
    d = json.loads(payload)
    return [{"deviceToken": d["device"], "value": math.sqrt(d["x"]), "topic": metadata.get("topic")}]
def spin(payload, metadata):
    while True:
        pass
def reach_out(payload, metadata):
    return open("/etc/hostname").read()
'''


def test_process_isolation_runs_decoders_and_survives_timeouts():
    r = ScriptRunner(isolation="process", timeout_s=2.0)
    try:
        out = r.call(DECODER, "decode", b'{"device": "d1", "x": 9}', {"topic": "t"}, name="dec")
        assert out == [{"deviceToken": "d1", "value": 3.0, "topic": "t"}]
        assert r.sandbox().mode == "seccomp"
        with pytest.raises(SiteWhereException, match="open"):
            r.call(DECODER, "reach_out", b"", {}, name="dec")
        r.timeout = 0.5
        with pytest.raises(SiteWhereException, match="timed out"):
            r.call(DECODER, "spin", b"", {}, name="dec")
        r.timeout = 2.0
        assert r.call(DECODER, "decode", b'{"device": "d2", "x": 4}', {}, name="dec")[0]["value"] == 2.0
        assert r.sandbox().restarts == 1
    finally:
        r.close()


def test_seccomp_lock_denies_files_sockets_and_processes():
    """What a script could do after escaping the restricted namespace: the locked worker cannot
    open files, create sockets or start processes, but still computes and allocates."""
    code = (
        "import os, socket\n"
        "from sitewhere_amd.runtime.script_sandbox import _lock\n"
        "mode, detail = _lock()\n"
        "assert mode == 'seccomp', detail\n"
        "x = [i * i for i in range(200000)]\n"
        "res = []\n"
        "for f in (lambda: open('/etc/hostname'), lambda: socket.socket(), lambda: os.fork(),\n"
        "          lambda: os.execv('/bin/true', ['true'])):\n"
        "    try:\n"
        "        f()\n"
        "        res.append('allowed')\n"
        "    except PermissionError:\n"
        "        res.append('denied')\n"
        "print(','.join(res), len(x))\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, p.stderr
    assert p.stdout.split() == ["denied,denied,denied,denied", "200000"]
