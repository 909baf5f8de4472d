"""Store-backed alternate-id dedup filter: generational fingerprint tables (Python oracle).

The reference checks every alternate id against the event store for as long as the store holds the
event (``AlternateIdDeduplicator.java:43-56`` over the unique sparse ``alternateId`` index,
``MongoDeviceEventManagement.java:130-131``).  The engines keep an exact HBM window of recent ids and,
behind it, this filter: an id new to the window that the filter holds goes to the host as a recheck
(``SW_ST_RECHECK``), where the durable store settles it.

Layout and rules are those of ``csrc/include/swtypes.h`` (``SW_FF_*``), implemented by the MI355X
kernels (``ff_has`` / ``ff_add`` / ``ff_clear_gen`` in ``csrc/hip/swgpu.hip``) and the native C++
engine (``csrc/native/swcpuengine.cpp``); this module is the bit-exact oracle:

* ``gens`` generations; a generation is a linear-probed table of ``buckets`` 16-slot buckets of
  32-bit fingerprints (0 = empty).  Bucket ``b`` of generation ``g`` sits at slot
  ``(b * gens + g) * 16``: one probe of every generation reads ``gens * 64`` contiguous bytes.
* An id's bucket is the low bits of ``mix(h)``, its fingerprint the high 32 bits (0 -> 1).
* Persisted ids go into the live generation.  At the end of a step whose persisted ids bring the live
  generation to ``ids_per_gen``, the oldest generation is cleared and becomes the live one.  So the
  filter always holds the newest ``(gens - 1) * ids_per_gen`` ids, and forgets what is older -- the
  durable store's retention is bounded by rows to match (``EngineConfig.filter_retention_rows``), so
  every id the store still holds stays checked.
"""
from __future__ import annotations

import numpy as np

SLOTS = 16            # SW_FF_SLOTS
MAX_PROBE = 64        # SW_FF_MAX_PROBE
META = 16             # SW_FF_META
MAX_GENS = 8          # SW_FF_MAX_GENS
_M64 = (1 << 64) - 1


def _mix64(x: int) -> int:
    x &= _M64
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & _M64
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & _M64
    return x ^ (x >> 31)


def ff_key(h: int, bmask: int) -> tuple[int, int]:
    """(home bucket, fingerprint) of alternate-id hash ``h`` (sw_ff_mix / sw_ff_bucket / sw_ff_fp)."""
    m = _mix64(int(h) ^ 0x5bd1e9955bd1e995)
    fp = m >> 32
    return m & bmask, fp if fp else 1


def meta_words(gens: int, ids_per_gen: int) -> np.ndarray:
    m = np.zeros(META + MAX_GENS, np.int64)
    m[2] = ids_per_gen
    m[3] = gens
    return m


class FingerprintFilter:
    """Generational fingerprint tables of persisted alternate ids (see the module docstring)."""

    def __init__(self, buckets: int, gens: int, ids_per_gen: int):
        if buckets & (buckets - 1) or not 2 <= gens <= MAX_GENS or ids_per_gen <= 0:
            raise ValueError("filter: buckets a power of two, 2..8 generations, ids per generation > 0")
        self.buckets, self.gens, self.bmask = int(buckets), int(gens), int(buckets) - 1
        self.tab = np.zeros(self.buckets * self.gens * SLOTS, np.uint32)
        self.meta = meta_words(gens, ids_per_gen)

    # ------------------------------------------------------------------ probes
    def has(self, h: int) -> bool:
        """Does a live generation hold ``h``'s fingerprint (ff_has)?"""
        b, fp = ff_key(h, self.bmask)
        open_ = (1 << self.gens) - 1
        G, t = self.gens, self.tab
        for _ in range(MAX_PROBE):
            if not open_:
                break
            for g in range(G):
                if not (open_ >> g) & 1:
                    continue
                s = t[(b * G + g) * SLOTS:(b * G + g + 1) * SLOTS]
                if (s == fp).any():
                    return True
                if (s == 0).any():
                    open_ &= ~(1 << g)
            b = (b + 1) & self.bmask
        return False

    def add(self, h: int, g: int | None = None) -> bool:
        """Add ``h`` to generation ``g`` (default: the live one) -- the first free slot of its chain;
        False when the probe bound was hit (dropped, counted in meta[5])."""
        g = int(self.meta[0]) if g is None else g
        b, fp = ff_key(h, self.bmask)
        G, t = self.gens, self.tab
        for _ in range(MAX_PROBE):
            base = (b * G + g) * SLOTS
            s = t[base:base + SLOTS]
            if (s == fp).any():
                return True
            free = np.nonzero(s == 0)[0]
            if len(free):
                t[base + int(free[0])] = fp
                return True
            b = (b + 1) & self.bmask
        self.meta[5] += 1
        return False

    def clear(self, g: int):
        v = self.tab.reshape(self.buckets, self.gens, SLOTS)
        v[:, g, :] = 0

    # ------------------------------------------------------------------ checkpoints
    def export(self) -> tuple[np.ndarray, np.ndarray]:
        """The non-empty buckets: (indices into [buckets * gens], [k, 16] fingerprints) -- the sparse
        form every engine checkpoints (a multi-GB filter of a small tenant is a few KB)."""
        v = self.tab.reshape(-1, SLOTS)
        idx = np.nonzero(v.any(axis=1))[0].astype(np.int64)
        return idx, v[idx].copy()

    def load(self, idx, rows):
        v = self.tab.reshape(-1, SLOTS)
        v[:] = 0
        v[np.asarray(idx, np.int64)] = np.asarray(rows, np.uint32).reshape(-1, SLOTS)

    # ------------------------------------------------------------------ step rules
    def add_persisted(self, hashes):
        """A step's persisted ids (k_persist): into the live generation, counted (meta[6])."""
        n = 0
        for h in np.asarray(hashes, np.uint64).tolist():
            if h:
                n += 1
                self.add(int(h))
        self.meta[6] += n

    def end_step(self, cursor: int):
        """The rotation rule (k_state_p2 clears, k_step_end flips): once the live generation has taken
        its ids, the oldest is cleared and becomes the live one."""
        if self.meta[6] >= self.meta[2]:
            self.rotate(cursor)

    def rotate(self, cursor: int):
        nxt = (int(self.meta[0]) + 1) % self.gens
        self.clear(nxt)
        self.meta[0] = nxt
        self.meta[META + nxt] = cursor
        self.meta[6] = 0
        self.meta[4] += 1


def filter_state(meta) -> dict:
    """Readable view of a filter's meta words (every engine's ``filter_state``)."""
    m = [int(x) for x in meta]
    g = m[3]
    return {"live": m[0], "ids_per_gen": m[2], "gens": g, "rotations": m[4], "dropped": m[5],
            "live_ids": m[6], "gen_cursor": m[META:META + g]}
