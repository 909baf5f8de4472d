"""JSON device requests -> device protobuf payloads (``csrc/native/swjson.cpp``).

A JSON event source that forwards raw batches (``forward: raw``) hands the fused engine the same
protobuf payloads a protobuf device would send: measurements, locations and Info-level device
alerts, with alternate ids, messages and metadata (the engine path stores them losslessly: durable
blocks, and event objects materialized from the step's block).  Anything else (registrations,
acks, non-integer dates, invalid JSON) is not transcoded and keeps the per-event path, so its
handling -- including decode-failure reporting -- is the reference's."""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from .._native import native

OK, INVALID, NOT_REPRESENTABLE = 0, -1, -2


_tls = threading.local()


def to_protobuf(payload: bytes) -> bytes | None:
    """Protobuf form of one JSON device request, or None when it stays on the per-event path."""
    b = payload if isinstance(payload, bytes) else bytes(payload)
    cap = 2 * len(b) + 64            # the protobuf form is never longer than the JSON plus its tags
    out = getattr(_tls, "out", None)
    if out is None or len(out) < cap:
        out = _tls.out = ctypes.create_string_buffer(max(cap, 4096))
    n = native().sw_json_to_pb(b, len(b), out, len(out))
    return ctypes.string_at(out, n) if n >= 0 else None


def batch_to_protobuf(payloads: list) -> tuple[list, np.ndarray]:
    """(protobuf payloads, status per input: 0 transcoded, -1 invalid, -2 not representable)."""
    n = len(payloads)
    lens = np.fromiter(map(len, payloads), np.int64, n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    heap = b"".join(payloads)
    cap = 2 * len(heap) + 64 * n + 64
    out = np.empty(cap, np.uint8)
    out_offs = np.zeros(n + 1, np.int64)
    status = np.zeros(n, np.int8)
    w = native().sw_json_to_pb_batch(heap, offs.ctypes.data, n, out.ctypes.data, cap, out_offs.ctypes.data,
                                     status.ctypes.data)
    if w < 0:
        raise RuntimeError("JSON transcode buffer too small")
    flat, o, st = out[:w].tobytes(), out_offs.tolist(), status.tolist()
    res = [flat[o[i]:o[i + 1]] if st[i] == OK else None for i in range(n)]
    return res, status
