"""Synthetic device fleets: tokens, fingerprints and protobuf wire payloads.

Thin numpy wrappers over ``libswnative`` (``sw_gen_payloads`` / ``sw_gen_tokens`` /
``sw_fingerprint_batch``).  Payloads use the reference device protocol
(``sitewhere-communication/src/main/proto/sitewhere.proto``): a delimited
``SiteWhere.Header`` followed by a delimited body message.  Used by bench.py,
the tests and the load-generator edge (the reference's equivalents are the
manual harnesses ``MqttTests.java`` / ``SiteWhereClientTester.java``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .._native import native


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def gen_tokens(prefix: str, first: int, n: int):
    """Device tokens ``<prefix><index:010d>`` as (heap uint8, offsets int64[n+1])."""
    lib = native()
    cap = n * (len(prefix.encode()) + 10) + 16
    heap = np.empty(cap, np.uint8)
    offs = np.empty(n + 1, np.int64)
    r = lib.sw_gen_tokens(prefix.encode(), first, n, _ptr(heap), cap, _ptr(offs))
    if r < 0:
        raise RuntimeError("token heap overflow")
    return heap[:r], offs


def token_list(prefix: str, first: int, n: int):
    heap, offs = gen_tokens(prefix, first, n)
    b = heap.tobytes()
    return [b[offs[i]:offs[i + 1]].decode() for i in range(n)]


def fingerprints(heap: np.ndarray, offs: np.ndarray):
    """128-bit device-token fingerprints (same function the GPU decoder uses)."""
    lib = native()
    n = len(offs) - 1
    lo = np.empty(n, np.uint64)
    hi = np.empty(n, np.uint64)
    heap = np.ascontiguousarray(heap, np.uint8)
    offs = np.ascontiguousarray(offs, np.int64)
    lib.sw_fingerprint_batch(_ptr(heap), _ptr(offs), n, _ptr(lo), _ptr(hi))
    return lo, hi


def fingerprint_str(s: str):
    b = np.frombuffer(s.encode(), np.uint8)
    lo, hi = fingerprints(b, np.array([0, len(b)], np.int64))
    return int(lo[0]), int(hi[0])


def hash64_strs(strs):
    lib = native()
    enc = [s.encode() for s in strs]
    offs = np.zeros(len(enc) + 1, np.int64)
    offs[1:] = np.cumsum([len(e) for e in enc])
    heap = np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy()
    out = np.empty(len(enc), np.uint64)
    lib.sw_hash64_batch(_ptr(heap), _ptr(offs), len(enc), _ptr(out))
    return out


def hash64(s: str) -> int:
    return int(hash64_strs([s])[0])


def hash64_heap(heap: np.ndarray, start: np.ndarray, end: np.ndarray) -> np.ndarray:
    """sw_hash64 of the strings heap[start[i]:end[i]] (vectorised over a string heap)."""
    lib = native()
    n = len(start)
    offs = np.empty(2 * n, np.int64)
    out = np.empty(n, np.uint64)
    if not n:
        return out
    heap = np.ascontiguousarray(heap, np.uint8)
    lib.sw_hash64_ranges(_ptr(heap), _ptr(np.ascontiguousarray(start, np.int64)),
                         _ptr(np.ascontiguousarray(end, np.int64)), n, _ptr(out))
    return out


@dataclass
class FleetSpec:
    prefix: str = "dev-"
    n_devices: int = 1 << 20
    p_location: float = 0.25
    p_alert: float = 0.05
    p_unregistered: float = 0.0
    mx_per_msg: int = 1
    n_names: int = 16
    with_alternate_id: bool = False
    lat0: float = 33.75
    lon0: float = -84.39
    span_deg: float = 0.5
    p_register: float = 0.0          # registration requests from new devices (control plane)
    p_ack: float = 0.0               # command acknowledgements (control plane)
    device_type: str = "default-type"
    p_meta: float = 0.0              # events carrying metadata (firmware version + gateway entries)
    alt_base: int = 0                # alternate ids "<epoch>-<alt_base + message index>" (8 hex digits)


def gen_payloads(spec: FleetSpec, n_msgs: int, ts0: int, seed: int, out: np.ndarray | None = None,
                 offs: np.ndarray | None = None):
    """Generate ``n_msgs`` encoded payloads. Returns (raw uint8[nbytes], offs uint32[n+1])."""
    lib = native()
    per = 112 + len(spec.prefix) + 10 + spec.mx_per_msg * 32 + (48 if spec.with_alternate_id else 0) + \
        (48 if spec.p_meta > 0 else 0)
    cap = n_msgs * per + 64
    if out is None or out.nbytes < cap:
        out = np.empty(cap, np.uint8)
    if offs is None or offs.size < n_msgs + 1:
        offs = np.empty(n_msgs + 1, np.uint32)
    r = lib.sw_gen_payloads(n_msgs, spec.prefix.encode(), spec.n_devices, spec.p_location, spec.p_alert,
                            spec.p_unregistered, spec.mx_per_msg, spec.n_names, ts0, seed,
                            1 if spec.with_alternate_id else 0, spec.lat0, spec.lon0, spec.span_deg,
                            float(spec.p_meta), _ptr(out), out.nbytes, _ptr(offs), int(spec.alt_base) & (2 ** 64 - 1))
    if r < 0:
        raise RuntimeError(f"payload buffer too small (need {-r})")
    raw, offs = out[:r], offs[:n_msgs + 1]
    if spec.p_register > 0 or spec.p_ack > 0:
        raw, offs = _splice_control(spec, raw, offs, seed)
    return raw, offs


def _splice_control(spec: FleetSpec, raw: np.ndarray, offs: np.ndarray, seed: int):
    """Replace a fraction of the payloads with registrations (new devices, reference
    ``SendRegistration``) and acknowledgements (registered devices) -- messages the engine hands to
    the control plane."""
    from ..models import wire
    n = len(offs) - 1
    rng = np.random.default_rng(seed + 0x5eed)
    u = rng.random(n)
    reg = np.nonzero(u < spec.p_register)[0]
    ack = np.nonzero((u >= spec.p_register) & (u < spec.p_register + spec.p_ack))[0]
    repl = {}
    for i in reg:
        repl[int(i)] = wire.registration(f"{spec.prefix}new-{seed}-{int(i)}", spec.device_type)
    for i in ack:
        d = int(rng.integers(0, spec.n_devices))
        repl[int(i)] = wire.acknowledge(f"{spec.prefix}{d:010d}", "ok", originator=f"cmd-{seed}-{int(i)}")
    if not repl:
        return raw, offs
    idx = np.array(sorted(repl), np.int64)
    lens = np.diff(offs.astype(np.int64))
    lens[idx] = [len(repl[int(i)]) for i in idx]
    new_offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=new_offs[1:])
    parts, prev = [], 0
    for i in idx:
        parts.append(raw[offs[prev]:offs[i]])
        parts.append(np.frombuffer(repl[int(i)], np.uint8))
        prev = int(i) + 1
    parts.append(raw[offs[prev]:offs[n]])
    return np.concatenate(parts), new_offs.astype(np.uint32)


def cpu_decode(raw: np.ndarray, offs: np.ndarray, now_ms: int, rank: int = 0, cap: int | None = None,
               threads: int = 4, out: np.ndarray | None = None, spans: np.ndarray | bool | None = None):
    """Decode a raw batch on the CPU with the shared decoder; returns an EVENT_REC array, or
    ``(records, STR_REF string refs)`` when ``spans`` is True or an array to fill.

    ``out`` (EVENT_REC, reused across batches) avoids a fresh allocation per batch; the decoder
    writes every byte of each record it returns, so it need not be zeroed."""
    from ..models.columnar import EVENT_REC, STR_REF

    lib = native()
    n_msgs = len(offs) - 1
    if out is not None:
        cap = len(out) if cap is None else min(cap, len(out))
    else:
        if cap is None:
            cap = max(16, n_msgs * 4)
        out = np.zeros(cap, EVENT_REC)
    want = spans is not None and spans is not False
    sp = None
    if want:
        sp = spans if isinstance(spans, np.ndarray) and len(spans) >= cap else np.zeros(cap, STR_REF)
    raw = np.ascontiguousarray(raw, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint32)
    n = lib.sw_cpu_decode(_ptr(raw) if raw.size else 0, _ptr(offs), n_msgs, now_ms, rank, _ptr(out),
                          _ptr(sp) if sp is not None else 0, cap, threads)
    return (out[:n], sp[:n]) if want else out[:n]


def stamp_alt_epoch(raw, offs: np.ndarray, epoch: int, threads: int = 8) -> int:
    """Give a generated batch fresh alternate ids in place (a producer replaying pre-generated
    payloads): the 16-hex-digit epoch of every fixed-width id (``sw_gen_payloads``) becomes
    ``epoch``.  ``raw`` is a numpy array or a host address.  Returns the payloads stamped."""
    offs = np.ascontiguousarray(offs, np.uint32)
    ptr = raw if isinstance(raw, int) else raw.ctypes.data
    return int(native().sw_stamp_alt_epoch(ptr, offs.ctypes.data, len(offs) - 1, int(epoch) & (2 ** 64 - 1),
                                           int(threads)))


def alt_positions(raw, offs: np.ndarray) -> np.ndarray:
    """Positions of the alternate-id epochs of a generated batch (``stamp_positions``); -1: none."""
    offs = np.ascontiguousarray(offs, np.uint32)
    pos = np.empty(len(offs) - 1, np.int64)
    ptr = raw if isinstance(raw, int) else raw.ctypes.data
    native().sw_alt_positions(ptr, offs.ctypes.data, len(offs) - 1, pos.ctypes.data)
    return pos


def stamp_positions(raw, pos: np.ndarray, epoch: int, threads: int = 4) -> int:
    """``stamp_alt_epoch`` at precomputed positions with streaming stores (no reads of the batch)."""
    ptr = raw if isinstance(raw, int) else raw.ctypes.data
    return int(native().sw_stamp_positions(ptr, pos.ctypes.data, len(pos), int(epoch) & (2 ** 64 - 1),
                                           int(threads)))


def pack_messages(messages):
    """Concatenate a list of payload byte strings into (raw, offs)."""
    offs = np.zeros(len(messages) + 1, np.uint32)
    offs[1:] = np.cumsum([len(m) for m in messages])
    raw = np.frombuffer(b"".join(messages) + b"\0" * 64, np.uint8).copy()
    return raw, offs
