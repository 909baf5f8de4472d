"""Span reporters: ship sampled spans to Jaeger the way the reference does, or to an OTLP collector.

Reference: the Jaeger tracer bean reports to the agent named by ``sitewhere.tracer.server``
(``MicroserviceConfiguration.java:51-58``, ``InstanceSettings.java:57-59``) -- jaeger-client's UDP
sender, i.e. ``Agent.emitBatch(jaeger.Batch)`` as a one-way Thrift *compact* message in one
datagram to port 6831.  This module writes that encoding directly (no Thrift dependency):

* :class:`JaegerUdpReporter` -- batches spans on a background thread (flush every ``interval_s``
  or when a datagram would exceed ``max_packet`` bytes) and sends ``emitBatch`` datagrams;
* :class:`OtlpHttpReporter` -- OTLP/HTTP JSON (``POST /v1/traces``) for OpenTelemetry collectors and
  Jaeger >= 1.35;
* :func:`decode_emit_batch` + :class:`MiniJaegerAgent` -- the inverse, for tests and local use.

``configure_tracing(settings, service)`` installs a reporter on the global tracer from
``InstanceSettings.tracer_server`` (``host[:port]`` -> Jaeger UDP, ``http(s)://...`` -> OTLP).
"""
from __future__ import annotations

import json
import socket
import struct
import threading
import urllib.request

from .tracing import Span, global_tracer

# ------------------------------------------------------------------------- thrift compact writer
T_STOP, T_TRUE, T_FALSE, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE, T_BINARY, T_LIST, T_SET, T_MAP, T_STRUCT = range(13)
# jaeger.thrift TagType
TAG_STRING, TAG_DOUBLE, TAG_BOOL, TAG_LONG, TAG_BINARY = range(5)


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(n: int, bits: int = 64) -> int:
    return ((n << 1) ^ (n >> (bits - 1))) & ((1 << bits) - 1)


def _signed64(u: int) -> int:
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >> 63 else u


class _W:
    """Compact-protocol struct writer: fields must be written in ascending id order."""

    def __init__(self):
        self.b = bytearray()
        self._last = [0]

    def _field(self, fid: int, t: int):
        delta = fid - self._last[-1]
        if 0 < delta <= 15:
            self.b.append((delta << 4) | t)
        else:
            self.b.append(t)
            self.b += _varint(_zz(fid, 16))
        self._last[-1] = fid

    def i32(self, fid, v):
        self._field(fid, T_I32)
        self.b += _varint(_zz(v, 32))
        return self

    def i64(self, fid, v):
        self._field(fid, T_I64)
        self.b += _varint(_zz(v))
        return self

    def double(self, fid, v):
        self._field(fid, T_DOUBLE)
        self.b += struct.pack("<d", v)
        return self

    def boolean(self, fid, v):
        self._field(fid, T_TRUE if v else T_FALSE)
        return self

    def string(self, fid, v):
        raw = v.encode() if isinstance(v, str) else bytes(v)
        self._field(fid, T_BINARY)
        self.b += _varint(len(raw)) + raw
        return self

    def struct(self, fid, fill):
        self._field(fid, T_STRUCT)
        self._last.append(0)
        fill(self)
        self.b.append(T_STOP)
        self._last.pop()
        return self

    def struct_list(self, fid, items, fill):
        self._field(fid, T_LIST)
        n = len(items)
        self.b.append((n << 4) | T_STRUCT if n < 15 else 0xF0 | T_STRUCT)
        if n >= 15:
            self.b += _varint(n)
        for it in items:
            self._last.append(0)
            fill(self, it)
            self.b.append(T_STOP)
            self._last.pop()
        return self


def _tag(w: _W, kv):
    k, v = kv
    w.string(1, str(k))
    if isinstance(v, bool):
        w.i32(2, TAG_BOOL).boolean(5, v)
    elif isinstance(v, int):
        w.i32(2, TAG_LONG).i64(6, v)
    elif isinstance(v, float):
        w.i32(2, TAG_DOUBLE).double(4, v)
    elif isinstance(v, (bytes, bytearray)):
        w.i32(2, TAG_BINARY).string(7, v)
    else:
        w.i32(2, TAG_STRING).string(3, str(v))


def _id64(h: str | None) -> int:
    return _signed64(int(h, 16)) if h else 0


def _span(w: _W, s: Span):
    tid = int(s.trace_id, 16)
    w.i64(1, _signed64(tid)).i64(2, _signed64(tid >> 64)).i64(3, _id64(s.span_id)).i64(4, _id64(s.parent_id))
    w.string(5, s.name)
    w.i32(7, 1 if s.sampled else 0)
    start_us = int(s.start * 1e6)
    w.i64(8, start_us).i64(9, int(((s.end or s.start) - s.start) * 1e6))
    if s.tags:
        w.struct_list(10, list(s.tags.items()), _tag)
    if s.logs:
        def _log(w2, lg):
            w2.i64(1, int(lg.get("ts", s.start) * 1e6))
            w2.struct_list(2, [(k, v) for k, v in lg.items() if k != "ts"], _tag)
        w.struct_list(11, s.logs, _log)


def encode_emit_batch(service: str, spans: list[Span], seq: int = 0, process_tags: dict | None = None) -> bytes:
    """``Agent.emitBatch(batch)`` as a one-way compact-protocol message (one UDP datagram)."""
    w = _W()

    def batch(wb: _W):
        def process(wp: _W):
            wp.string(1, service)
            if process_tags:
                wp.struct_list(2, list(process_tags.items()), _tag)
        wb.struct(1, process)
        wb.struct_list(2, spans, _span)
        wb.i64(3, seq)
    w.struct(1, batch)
    w.b.append(T_STOP)
    name = b"emitBatch"
    return bytes([0x82, 0x81]) + _varint(seq) + _varint(len(name)) + name + bytes(w.b)


# ------------------------------------------------------------------------- thrift compact reader
class _R:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def byte(self):
        v = self.b[self.p]
        self.p += 1
        return v

    def varint(self):
        shift = out = 0
        while True:
            c = self.byte()
            out |= (c & 0x7F) << shift
            if not c & 0x80:
                return out
            shift += 7

    def zz(self):
        n = self.varint()
        return (n >> 1) ^ -(n & 1)

    def value(self, t):
        if t in (T_TRUE, T_FALSE):
            return t == T_TRUE
        if t == T_BYTE:
            return self.byte()
        if t in (T_I16, T_I32, T_I64):
            return self.zz()
        if t == T_DOUBLE:
            v = struct.unpack_from("<d", self.b, self.p)[0]
            self.p += 8
            return v
        if t == T_BINARY:
            n = self.varint()
            v = self.b[self.p:self.p + n]
            self.p += n
            return v
        if t in (T_LIST, T_SET):
            h = self.byte()
            n, et = h >> 4, h & 0x0F
            if n == 15:
                n = self.varint()
            if et in (T_TRUE, T_FALSE):
                return [self.byte() == 1 for _ in range(n)]
            return [self.value(et) for _ in range(n)]
        if t == T_STRUCT:
            return self.struct()
        raise ValueError(f"unsupported compact type {t}")

    def struct(self) -> dict:
        out, last = {}, 0
        while True:
            h = self.byte()
            if h == T_STOP:
                return out
            t, delta = h & 0x0F, h >> 4
            fid = last + delta if delta else (lambda n: (n >> 1) ^ -(n & 1))(self.varint())
            out[fid] = self.value(t)
            last = fid


def _tag_value(t: dict):
    return {TAG_STRING: lambda: t.get(3, b"").decode(), TAG_DOUBLE: lambda: t.get(4), TAG_BOOL: lambda: t.get(5),
            TAG_LONG: lambda: t.get(6), TAG_BINARY: lambda: t.get(7)}[t[2]]()


def decode_emit_batch(packet: bytes) -> dict:
    """Inverse of :func:`encode_emit_batch`: ``{"service", "seq", "spans": [{traceId, spanId, ...}]}``."""
    r = _R(packet)
    if r.byte() != 0x82 or (r.byte() >> 5) != 4:
        raise ValueError("not a compact one-way message")
    seq = r.varint()
    name = r.value(T_BINARY).decode()
    if name != "emitBatch":
        raise ValueError(f"unexpected method {name}")
    args = r.struct()
    b = args[1]
    spans = []
    for s in b.get(2, []):
        u = lambda v: v & ((1 << 64) - 1)   # noqa: E731
        spans.append({"traceId": f"{(u(s.get(2, 0)) << 64) | u(s[1]):x}", "spanId": f"{u(s[3]):016x}",
                      "parentId": f"{u(s[4]):016x}" if s.get(4) else None, "name": s[5].decode(),
                      "flags": s.get(7), "startUs": s[8], "durationUs": s[9],
                      "tags": {t[1].decode(): _tag_value(t) for t in s.get(10, [])},
                      "logs": [{"ts": lg[1], **{t[1].decode(): _tag_value(t) for t in lg.get(2, [])}}
                               for lg in s.get(11, [])]})
    return {"service": b[1][1].decode(), "seq": seq, "spans": spans}


# ------------------------------------------------------------------------- reporters
class _BatchingReporter:
    def __init__(self, interval_s: float = 1.0, max_spans: int = 100):
        self.interval_s, self.max_spans = interval_s, max_spans
        self._buf: list[Span] = []
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = threading.Event()
        self.sent_spans = self.sent_batches = self.errors = 0
        self._t = threading.Thread(target=self._run, daemon=True, name=f"{type(self).__name__}")
        self._t.start()

    def __call__(self, span: Span):
        with self._lock:
            self._buf.append(span)
            full = len(self._buf) >= self.max_spans
        if full:
            self._wake.set()

    def _run(self):
        while not self._stop.is_set():
            self._wake.wait(self.interval_s)
            self._wake.clear()
            self.flush()
        self.flush()

    def flush(self):
        with self._lock:
            spans, self._buf = self._buf, []
        if spans:
            try:
                self._send(spans)
                self.sent_spans += len(spans)
            except Exception:
                self.errors += 1

    def _send(self, spans):
        raise NotImplementedError

    def close(self):
        self._stop.set()
        self._wake.set()
        self._t.join(timeout=5)


class JaegerUdpReporter(_BatchingReporter):
    """jaeger-client's UDP sender: ``emitBatch`` datagrams to the agent (default port 6831)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 6831, service: str = "sitewhere",
                 max_packet: int = 65000, **kw):
        self.addr, self.service, self.max_packet = (host, port), service, max_packet
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self._seq = 0
        super().__init__(**kw)

    def _send(self, spans):
        i = 0
        while i < len(spans):
            n = len(spans) - i
            while True:                                   # halve until the datagram fits
                pkt = encode_emit_batch(self.service, spans[i:i + n], self._seq)
                if len(pkt) <= self.max_packet or n == 1:
                    break
                n = max(1, n // 2)
            if len(pkt) <= self.max_packet:
                self.sock.sendto(pkt, self.addr)
                self.sent_batches += 1
            else:
                self.errors += 1                          # a single span larger than a datagram
            self._seq += 1
            i += n

    def close(self):
        super().close()
        self.sock.close()


def otlp_json(service: str, spans: list[Span]) -> dict:
    def attr(k, v):
        if isinstance(v, bool):
            val = {"boolValue": v}
        elif isinstance(v, int):
            val = {"intValue": str(v)}
        elif isinstance(v, float):
            val = {"doubleValue": v}
        else:
            val = {"stringValue": str(v)}
        return {"key": str(k), "value": val}
    out = []
    for s in spans:
        end = s.end or s.start
        d = {"traceId": s.trace_id.rjust(32, "0"), "spanId": s.span_id.rjust(16, "0"), "name": s.name, "kind": 1,
             "startTimeUnixNano": str(int(s.start * 1e9)), "endTimeUnixNano": str(int(end * 1e9)),
             "attributes": [attr(k, v) for k, v in s.tags.items()],
             "events": [{"timeUnixNano": str(int(lg.get("ts", s.start) * 1e9)), "name": str(lg.get("event", "log")),
                         "attributes": [attr(k, v) for k, v in lg.items() if k not in ("ts", "event")]}
                        for lg in s.logs],
             "status": {"code": 2} if s.tags.get("error") else {}}
        if s.parent_id:
            d["parentSpanId"] = s.parent_id.rjust(16, "0")
        out.append(d)
    return {"resourceSpans": [{"resource": {"attributes": [attr("service.name", service)]},
                               "scopeSpans": [{"scope": {"name": "sitewhere_amd"}, "spans": out}]}]}


class OtlpHttpReporter(_BatchingReporter):
    """OTLP/HTTP JSON exporter: ``POST {url}/v1/traces``."""

    def __init__(self, url: str = "http://127.0.0.1:4318", service: str = "sitewhere", timeout_s: float = 5.0, **kw):
        self.url = url.rstrip("/") + ("" if url.rstrip("/").endswith("/v1/traces") else "/v1/traces")
        self.service, self.timeout_s = service, timeout_s
        super().__init__(**kw)

    def _send(self, spans):
        body = json.dumps(otlp_json(self.service, spans)).encode()
        req = urllib.request.Request(self.url, data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=self.timeout_s) as r:
            r.read()
        self.sent_batches += 1


class MiniJaegerAgent:
    """UDP stand-in for jaeger-agent's compact endpoint: decodes and keeps every received batch."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((host, port))
        self.sock.settimeout(0.2)
        self.host, self.port = self.sock.getsockname()
        self.batches: list[dict] = []
        self.bad = 0
        self._stop = threading.Event()

    def start(self):
        threading.Thread(target=self._run, daemon=True, name="mini-jaeger-agent").start()
        return self

    def _run(self):
        while not self._stop.is_set():
            try:
                pkt, _ = self.sock.recvfrom(65536)
            except (socket.timeout, OSError):
                continue
            try:
                self.batches.append(decode_emit_batch(pkt))
            except Exception:
                self.bad += 1

    @property
    def spans(self) -> list[dict]:
        return [s for b in list(self.batches) for s in b["spans"]]

    def stop(self):
        self._stop.set()
        self.sock.close()


_configured: dict = {}


def configure_tracing(server: str, sample_rate: float | None = None, service: str = "sitewhere"):
    """Install a reporter on the global tracer (once per process per server address)."""
    tracer = global_tracer()
    if sample_rate is not None:
        tracer.sample_rate = sample_rate
    if not server or server in _configured:
        return _configured.get(server)
    if server.startswith(("http://", "https://")):
        rep = OtlpHttpReporter(server, service)
    else:
        host, _, port = server.partition(":")
        rep = JaegerUdpReporter(host or "127.0.0.1", int(port or 6831), service)
    prev = tracer.reporter
    if prev is None:
        tracer.reporter = rep
    else:
        def both(span, _a=prev, _b=rep):
            _a(span)
            _b(span)
        tracer.reporter = both
    _configured[server] = rep
    return rep
