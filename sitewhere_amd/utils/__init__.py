"""Small shared helpers (dense id maps, power-of-two sizing, wall-clock timing)."""
from __future__ import annotations

import time


def pow2_at_least(n: int) -> int:
    """Smallest power of two >= n (hash-table capacities; masks are capacity - 1)."""
    p = 1
    while p < n:
        p <<= 1
    return p


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
