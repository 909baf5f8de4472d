"""Routing of the messages an engine step rejected, per payload and in native code.

``csrc/native/swroute.cpp`` finds the payload of every reject record (its offset points into it),
parses only those payloads and writes the reference's Kafka payloads: ``GInboundEventPayload`` per
event of an unregistered / unassigned device (``InboundPayloadProcessingLogic.java:199-218``),
``GDeviceRegistationPayload`` for registrations (``EventSourcesManager.java:153-182``), the payload
itself for acknowledgements / streams (decoded on the host: the reference message has no member for
them) and for undecodable payloads (failed-decode topic, ``EventSourcesManager.java:189-197``).
Records come back grouped by (kind, Kafka partition of the device token), keys and values in two
heaps, so each group is one native append to its topic.  Duplicates are dropped (dedup)."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .._native import native

UNREGISTERED, REGISTRATION, CONTROL, FAILED = 0, 1, 2, 3


@dataclass
class RoutedRejects:
    rec: np.ndarray          # int32 [n, 4]: kind, partition, key length, value length
    keys: np.ndarray         # uint8 heap
    vals: np.ndarray         # uint8 heap
    payloads: int            # payloads looked at

    def __len__(self):
        return len(self.rec)

    def groups(self):
        """(kind, partition, key heap, key offsets [m+1], value heap, value offsets [m+1]) per group."""
        n = len(self.rec)
        if not n:
            return
        koff = np.zeros(n + 1, np.int64)
        voff = np.zeros(n + 1, np.int64)
        np.cumsum(self.rec[:, 2], out=koff[1:])
        np.cumsum(self.rec[:, 3], out=voff[1:])
        kp = self.rec[:, 0].astype(np.int64) << 32 | (self.rec[:, 1].astype(np.int64) & 0xFFFFFFFF)
        cut = np.nonzero(np.diff(kp))[0] + 1
        starts = np.concatenate([[0], cut])
        ends = np.concatenate([cut, [n]])
        for a, b in zip(starts, ends):
            ko, vo = koff[a:b + 1], voff[a:b + 1]
            yield (int(self.rec[a, 0]), int(self.rec[a, 1]), self.keys[ko[0]:ko[-1]], ko - ko[0],
                   self.vals[vo[0]:vo[-1]], vo - vo[0])

    def values(self, kind: int):
        """(key bytes, value bytes) of every record of one kind (small kinds: control, failed)."""
        n = len(self.rec)
        koff = np.concatenate([[0], np.cumsum(self.rec[:, 2], dtype=np.int64)])
        voff = np.concatenate([[0], np.cumsum(self.rec[:, 3], dtype=np.int64)])
        for i in np.nonzero(self.rec[:, 0] == kind)[0] if n else []:
            yield bytes(self.keys[koff[i]:koff[i + 1]]), bytes(self.vals[voff[i]:voff[i + 1]])


def concat(parts: list) -> RoutedRejects:
    """Routed rejects of several records, in record order (each record's groups stay contiguous,
    so per-key order holds)."""
    if not parts:
        return RoutedRejects(np.zeros((0, 4), np.int32), np.zeros(0, np.uint8), np.zeros(0, np.uint8), 0)
    if len(parts) == 1:
        return parts[0]
    return RoutedRejects(np.concatenate([p.rec for p in parts]), np.concatenate([p.keys for p in parts]),
                         np.concatenate([p.vals for p in parts]), sum(p.payloads for p in parts))


def _call(fn, args_head: tuple, n_rej: int) -> RoutedRejects:
    need = np.zeros(3, np.int64)
    npay = np.zeros(1, np.int64)
    # generous first guess (np.empty does not touch the pages): a too-small heap makes the native
    # router do all its work twice (a payload with several measurements routes to several records)
    cap = (max(16, 8 * n_rej), max(1024, 160 * n_rej), max(4096, 1024 * n_rej))
    for _ in range(2):
        rec = np.empty((cap[0], 4), np.int32)         # the first n rows are written
        keys = np.empty(cap[1], np.uint8)
        vals = np.empty(cap[2], np.uint8)
        n = fn(*args_head, rec.ctypes.data, cap[0], keys.ctypes.data, cap[1], vals.ctypes.data, cap[2],
               need.ctypes.data, npay.ctypes.data)
        if n >= 0:
            return RoutedRejects(rec[:n], keys[:need[1]], vals[:need[2]], int(npay[0]))
        cap = tuple(int(x) for x in need)
    raise RuntimeError("reject routing: output sizing failed")


def route_refs(compact, refs: np.ndarray, rank: int = 0, source_id: str = "gpu-inbound",
               partitions=(1, 1, 1, 1), raw=None) -> RoutedRejects:
    """Route the MI355X step's reject snapshot (``k_reject_refs``: u32 [n, 4] = payload start, end,
    status | src_rank << 8, copy offset) from the compact payload copies ``compact`` the GPU made;
    ``raw`` (the batch bytes, a numpy array or address) only serves refs whose copy did not fit."""
    refs = np.ascontiguousarray(refs, np.uint32).reshape(-1)
    n = len(refs) // 4

    def ptr(x):
        return None if x is None else (x if isinstance(x, int) else np.asarray(x).ctypes.data)
    comp = np.ascontiguousarray(compact, np.uint8) if not isinstance(compact, int) else compact
    parts = np.asarray(partitions, np.int32)
    return _call(native().sw_route_refs, (ptr(comp), ptr(raw), refs.ctypes.data if n else None, n, int(rank),
                                          source_id.encode(), parts.ctypes.data), n)


def route_rejects(raw: np.ndarray, offs: np.ndarray, rej_off: np.ndarray, rej_status: np.ndarray,
                  source_id: str = "gpu-inbound", partitions=(1, 1, 1, 1)) -> RoutedRejects:
    """``raw`` / ``offs``: the raw batch; ``rej_off`` / ``rej_status``: the step's reject records
    (``EVENT_REC["aux_off"]``, engine status).  ``partitions``: partition counts of the
    unregistered, registration, decoded and failed-decode topics."""
    raw = np.ascontiguousarray(raw, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint32)
    ro = np.ascontiguousarray(rej_off, np.uint32)
    rs = np.ascontiguousarray(rej_status, np.uint8)
    parts = np.asarray(partitions, np.int32)
    n_rej = len(ro)
    return _call(native().sw_route_rejects, (raw.ctypes.data, offs.ctypes.data, len(offs) - 1,
                                             ro.ctypes.data if n_rej else None, rs.ctypes.data if n_rej else None,
                                             n_rej, source_id.encode(), parts.ctypes.data), n_rej)
