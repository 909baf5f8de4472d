"""Small shared helpers (dense id maps, power-of-two sizing, wall-clock timing)."""
from __future__ import annotations

import os
import random

import time


def pow2_at_least(n: int) -> int:
    """Smallest power of two >= n (hash-table capacities; masks are capacity - 1)."""
    p = 1
    while p < n:
        p <<= 1
    return p


_rng = random.Random(int.from_bytes(os.urandom(16), "little"))
if hasattr(os, "register_at_fork"):
    os.register_at_fork(after_in_child=lambda: _rng.seed(int.from_bytes(os.urandom(16), "little")))


def fast_uuid4() -> str:
    """Random (version 4) UUID string from a process-local PRNG seeded by ``os.urandom``.

    Entity and event ids need uniqueness, not unpredictability.  ``uuid.uuid4()`` reads
    ``os.urandom`` per call, and that syscall releases the GIL: with the service threads busy,
    re-acquiring it costs ~200 us per id (measured on the per-event path) -- more than the rest of
    the event's processing.  ``getrandbits`` never releases the GIL."""
    n = (_rng.getrandbits(128) & ~(0xF000 << 64) | (0x4000 << 64)) & ~(0xC000 << 48) | (0x8000 << 48)
    h = f"{n:032x}"
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


def fast_hex(bits: int = 64) -> str:
    """Random hex id of ``bits`` bits (trace / span ids)."""
    return f"{_rng.getrandbits(bits):0{bits // 4}x}"


class IndexMap:
    """Stable dense int indices for string ids (device / assignment / customer / area / asset):
    the GPU tables are indexed by these, the control plane keeps the strings."""

    def __init__(self):
        self.idx: dict[str, int] = {}
        self.ids: list[str] = []

    def get(self, key: str | None) -> int:
        if key is None:
            return -1
        i = self.idx.get(key)
        if i is None:
            i = self.idx[key] = len(self.ids)
            self.ids.append(key)
        return i

    def id_of(self, i: int) -> str | None:
        return self.ids[i] if 0 <= i < len(self.ids) else None

    def __len__(self):
        return len(self.ids)


class Stopwatch:
    """``with Stopwatch() as sw: ...; sw.ms`` -- perf_counter based."""

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        self.s = time.perf_counter() - self.t0
        self.ms = 1000.0 * self.s
        return False


_MALLOC_TUNED = False


def retain_large_allocations() -> bool:
    """Keep multi-MB host allocations in the heap instead of fresh mmaps (glibc ``mallopt``).

    An engine tenant builds one tens-of-MB columnar batch per step; with glibc's default dynamic
    mmap threshold each one is a fresh mapping whose first touch page-faults at 1-2 GB/s in a
    container (4.3 ms per 37 MB batch measured, 1.5-2.7 ms once the heap keeps and reuses the
    memory).  Process-wide and idempotent; ``SW_MALLOC_RETAIN=0`` disables it."""
    global _MALLOC_TUNED
    if _MALLOC_TUNED or os.environ.get("SW_MALLOC_RETAIN", "1") == "0":
        return _MALLOC_TUNED
    try:
        import ctypes
        libc = ctypes.CDLL("libc.so.6")
        m_trim_threshold, m_mmap_threshold = -1, -3
        _MALLOC_TUNED = bool(libc.mallopt(m_mmap_threshold, 1 << 30)) and bool(libc.mallopt(m_trim_threshold, 1 << 31))
    except (OSError, AttributeError):
        _MALLOC_TUNED = False
    return _MALLOC_TUNED


_GC_TUNED = False


def tune_gc_for_streaming() -> bool:
    """Freeze the start-up heap out of the cyclic collector and raise the gen-0 threshold.

    An engine tenant holds tens of thousands of long-lived objects (the registry mirror, domain
    entities, service state) while its data plane allocates few Python objects per batch; a full
    collection walks the whole heap under the GIL.  Opt-in (tenant ``tuneGc``): on the MI355X
    tenant path a freeze after the registry is loaded measured +10-48% at 1M-payload batches, but
    tuning at tenant start was within run-to-run noise or slower (``profiles/r2_tenant_gc``).
    Objects created later are collected as usual.  Process-wide and idempotent; ``SW_GC_TUNE=0``
    disables it."""
    global _GC_TUNED
    if _GC_TUNED or os.environ.get("SW_GC_TUNE", "1") == "0":
        return _GC_TUNED
    import gc
    gc.collect()
    gc.freeze()
    gc.set_threshold(50_000, 20, 100)
    _GC_TUNED = True
    return True
