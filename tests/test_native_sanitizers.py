"""Host sanitizer runs of the native runtime (the reference has no race detection).

``csrc/native/tests/stress_native.cpp`` drives the commit log (producers, waiting / copying /
in-place readers, retention recycling segments across partitions, adopted external buffers,
consumer-group offsets, a durable directory), the CPU engine's fork-join pool and the
device-protocol decoder (20,000 corrupted payloads, string refs included) from many threads, and
encodes / verifies / decodes a lossless durable block of the decoded events (strings copied from an
exactly sized batch).  It is compiled together with ``swnative.cpp``, ``swcpuengine.cpp`` and
``swseg.cpp`` / ``swindex.cpp`` twice: with ThreadSanitizer, and with
AddressSanitizer + UndefinedBehaviorSanitizer.  Host code only -- no GPU code is instrumented.
"""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "native", "tests", "stress_native.cpp"),
       os.path.join(ROOT, "csrc", "native", "swnative.cpp"),
       os.path.join(ROOT, "csrc", "native", "swcpuengine.cpp"),
       os.path.join(ROOT, "csrc", "native", "swseg.cpp"),
       os.path.join(ROOT, "csrc", "native", "swindex.cpp"),
       os.path.join(ROOT, "csrc", "native", "swrowjson.cpp")]
CXX = shutil.which("g++")

SANITIZERS = {
    "thread": ["-fsanitize=thread"],
    "address_undefined": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                          "-fno-omit-frame-pointer"],
}


@pytest.mark.skipif(CXX is None, reason="needs g++")
@pytest.mark.parametrize("kind", sorted(SANITIZERS))
def test_native_runtime_is_sanitizer_clean(kind, tmp_path):
    exe = tmp_path / f"stress_{kind}"
    cmd = [CXX, "-std=c++17", "-O1", "-g", *SANITIZERS[kind], f"-I{os.path.join(ROOT, 'csrc', 'include')}",
           *SRC, "-o", str(exe), "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "sanitize" in b.stderr and "cannot find" in b.stderr:
        pytest.skip(f"{kind} sanitizer runtime not installed")
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1 abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path / "durable")], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-5000:]
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out and "runtime error" not in out, out[-5000:]
    assert "all native stress checks passed" in r.stdout
