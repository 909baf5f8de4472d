"""AMQP 1.0 (OASIS) client: type system, framing, SASL, connection / session / links.

Reference: ``service-event-sources/.../azure/EventHubInboundEventReceiver.java:150-174`` consumes an
Azure Event Hub through the Azure SDK's ``EventProcessorHost`` (AMQP 1.0 over TLS to
``<namespace>.servicebus.windows.net:5671``).  That SDK is not available here, so this module speaks
the protocol itself (OASIS AMQP 1.0, parts 1-5): the type encoding, frames, the SASL layer, and the
performatives a receiving client needs (open, begin, attach, flow, transfer, disposition, detach,
end, close), plus the message sections.  ``edges/eventhub.py`` builds the Event Hubs consumer on it.
"""
from __future__ import annotations

import socket
import ssl
import struct
import threading
import uuid
from dataclasses import dataclass

# ------------------------------------------------------------------------------------ types


class Symbol(str):
    """AMQP symbol (ASCII)."""


class UInt(int):
    pass


class ULong(int):
    pass


class UByte(int):
    pass


class UShort(int):
    pass


class Timestamp(int):
    """Milliseconds since the epoch."""


@dataclass
class Described:
    descriptor: object
    value: object


@dataclass
class Array:
    """Homogeneous array; ``ctor`` is the element constructor byte (e.g. 0xa3 symbols)."""
    ctor: int
    items: list


def _enc(v, out: bytearray):
    if v is None:
        out.append(0x40)
    elif isinstance(v, bool):
        out.append(0x41 if v else 0x42)
    elif isinstance(v, Described):
        out.append(0x00)
        _enc(v.descriptor, out)
        _enc(v.value, out)
    elif isinstance(v, Symbol):
        b = v.encode("ascii")
        out += (bytes([0xa3, len(b)]) if len(b) < 256 else b"\xb3" + struct.pack(">I", len(b))) + b
    elif isinstance(v, str):
        b = v.encode()
        out += (bytes([0xa1, len(b)]) if len(b) < 256 else b"\xb1" + struct.pack(">I", len(b))) + b
    elif isinstance(v, (bytes, bytearray, memoryview)):
        b = bytes(v)
        out += (bytes([0xa0, len(b)]) if len(b) < 256 else b"\xb0" + struct.pack(">I", len(b))) + b
    elif isinstance(v, UByte):
        out += bytes([0x50, int(v)])
    elif isinstance(v, UShort):
        out += b"\x60" + struct.pack(">H", int(v))
    elif isinstance(v, UInt):
        if v == 0:
            out.append(0x43)
        elif v < 256:
            out += bytes([0x52, int(v)])
        else:
            out += b"\x70" + struct.pack(">I", int(v))
    elif isinstance(v, ULong):
        if v == 0:
            out.append(0x44)
        elif v < 256:
            out += bytes([0x53, int(v)])
        else:
            out += b"\x80" + struct.pack(">Q", int(v))
    elif isinstance(v, Timestamp):
        out += b"\x83" + struct.pack(">q", int(v))
    elif isinstance(v, int):
        if -128 <= v <= 127:
            out += b"\x55" + struct.pack(">b", v)
        else:
            out += b"\x81" + struct.pack(">q", v)
    elif isinstance(v, float):
        out += b"\x82" + struct.pack(">d", v)
    elif isinstance(v, uuid.UUID):
        out += b"\x98" + v.bytes
    elif isinstance(v, (list, tuple)):
        body = bytearray()
        for x in v:
            _enc(x, body)
        if not v:
            out.append(0x45)
        elif len(body) < 255 and len(v) < 256:
            out += bytes([0xc0, len(body) + 1, len(v)]) + body
        else:
            out += b"\xd0" + struct.pack(">II", len(body) + 4, len(v)) + body
    elif isinstance(v, dict):
        body = bytearray()
        for k, x in v.items():
            _enc(k, body)
            _enc(x, body)
        n = 2 * len(v)
        if len(body) < 255 and n < 256:
            out += bytes([0xc1, len(body) + 1, n]) + body
        else:
            out += b"\xd1" + struct.pack(">II", len(body) + 4, n) + body
    elif isinstance(v, Array):
        body = bytearray()
        for x in v.items:
            tmp = bytearray()
            _enc(x, tmp)
            body += _strip_ctor(v.ctor, tmp)
        out += b"\xf0" + struct.pack(">II", len(body) + 5, len(v.items)) + bytes([v.ctor]) + body
    else:
        raise TypeError(f"cannot encode {type(v).__name__} as AMQP")


def _strip_ctor(ctor: int, enc: bytearray) -> bytes:
    """Element bytes of an array: the value without its own constructor, widened to ``ctor``."""
    c = enc[0]
    if ctor == 0xb3 and c == 0xa3:
        return struct.pack(">I", enc[1]) + bytes(enc[2:])
    if ctor == 0xb1 and c == 0xa1:
        return struct.pack(">I", enc[1]) + bytes(enc[2:])
    if ctor == c:
        return bytes(enc[1:])
    raise TypeError(f"array element constructor 0x{c:02x} does not fit 0x{ctor:02x}")


def encode(v) -> bytes:
    out = bytearray()
    _enc(v, out)
    return bytes(out)


_FIXED = {0x50: (1, ">B", UByte), 0x51: (1, ">b", int), 0x60: (2, ">H", UShort), 0x61: (2, ">h", int),
          0x70: (4, ">I", UInt), 0x71: (4, ">i", int), 0x80: (8, ">Q", ULong), 0x81: (8, ">q", int),
          0x72: (4, ">f", float), 0x82: (8, ">d", float), 0x83: (8, ">q", Timestamp), 0x73: (4, ">I", int)}


def _dec_value(b: bytes, i: int, c: int):
    if c == 0x40:
        return None, i
    if c == 0x41:
        return True, i
    if c == 0x42:
        return False, i
    if c == 0x56:
        return b[i] != 0, i + 1
    if c == 0x43:
        return UInt(0), i
    if c == 0x44:
        return ULong(0), i
    if c == 0x52:
        return UInt(b[i]), i + 1
    if c == 0x53:
        return ULong(b[i]), i + 1
    if c == 0x54:
        return struct.unpack_from(">b", b, i)[0], i + 1
    if c == 0x55:
        return struct.unpack_from(">b", b, i)[0], i + 1
    if c in _FIXED:
        n, fmt, cls = _FIXED[c]
        return cls(struct.unpack_from(fmt, b, i)[0]), i + n
    if c == 0x98:
        return uuid.UUID(bytes=bytes(b[i:i + 16])), i + 16
    if c in (0xa0, 0xa1, 0xa3, 0xb0, 0xb1, 0xb3):
        if c & 0x10:
            n = struct.unpack_from(">I", b, i)[0]
            i += 4
        else:
            n = b[i]
            i += 1
        raw = bytes(b[i:i + n])
        i += n
        if c in (0xa0, 0xb0):
            return raw, i
        if c in (0xa3, 0xb3):
            return Symbol(raw.decode("ascii")), i
        return raw.decode(), i
    if c == 0x45:
        return [], i
    if c in (0xc0, 0xc1, 0xd0, 0xd1):
        if c & 0x10:
            size, count = struct.unpack_from(">II", b, i)
            i += 8
            end = i + size - 4
        else:
            size, count = b[i], b[i + 1]
            i += 2
            end = i + size - 1
        items = []
        for _ in range(count):
            x, i = _dec(b, i)
            items.append(x)
        i = end
        if c in (0xc1, 0xd1):
            return {items[k]: items[k + 1] for k in range(0, len(items), 2)}, i
        return items, i
    if c in (0xe0, 0xf0):
        if c == 0xf0:
            size, count = struct.unpack_from(">II", b, i)
            i += 8
            end = i + size - 4
        else:
            size, count = b[i], b[i + 1]
            i += 2
            end = i + size - 1
        ec = b[i]
        i += 1
        items = []
        for _ in range(count):
            x, i = _dec_value(b, i, ec)
            items.append(x)
        return Array(ec, items), end
    raise ValueError(f"unknown AMQP constructor 0x{c:02x}")


def _dec(b: bytes, i: int):
    c = b[i]
    i += 1
    if c == 0x00:
        d, i = _dec(b, i)
        v, i = _dec(b, i)
        return Described(d, v), i
    return _dec_value(b, i, c)


def decode(b: bytes, i: int = 0):
    """(value, next index)."""
    return _dec(b, i)


def decode_all(b: bytes) -> list:
    out, i = [], 0
    while i < len(b):
        v, i = _dec(b, i)
        out.append(v)
    return out


# ------------------------------------------------------------------------------------ performatives
OPEN, BEGIN, ATTACH, FLOW, TRANSFER, DISPOSITION, DETACH, END, CLOSE = range(0x10, 0x19)
SASL_MECHANISMS, SASL_INIT, SASL_CHALLENGE, SASL_RESPONSE, SASL_OUTCOME = range(0x40, 0x45)
SOURCE, TARGET = 0x28, 0x29
ACCEPTED = 0x24
# message sections
HEADER, DELIVERY_ANN, MESSAGE_ANN, PROPERTIES, APP_PROPERTIES, DATA, SEQUENCE, VALUE, FOOTER = range(0x70, 0x79)
SELECTOR = Symbol("apache.org:selector-filter:string")

AMQP_HEADER = b"AMQP\x00\x01\x00\x00"
SASL_HEADER = b"AMQP\x03\x01\x00\x00"


def perf(code: int, fields: list) -> Described:
    # trailing nulls may be omitted (OASIS 1.0 part 1, 1.4)
    while fields and fields[-1] is None:
        fields = fields[:-1]
    return Described(ULong(code), list(fields))


def frame(body: bytes, channel: int = 0, ftype: int = 0) -> bytes:
    return struct.pack(">IBBH", 8 + len(body), 2, ftype, channel) + body


@dataclass
class Message:
    body: bytes | None = None          # data section(s) concatenated
    value: object = None               # amqp-value section
    annotations: dict | None = None    # message annotations
    properties: list | None = None
    app_properties: dict | None = None

    def encode(self) -> bytes:
        out = bytearray()
        if self.annotations:
            _enc(Described(ULong(MESSAGE_ANN), self.annotations), out)
        if self.properties:
            _enc(Described(ULong(PROPERTIES), self.properties), out)
        if self.app_properties:
            _enc(Described(ULong(APP_PROPERTIES), self.app_properties), out)
        if self.body is not None:
            _enc(Described(ULong(DATA), bytes(self.body)), out)
        if self.value is not None:
            _enc(Described(ULong(VALUE), self.value), out)
        return bytes(out)

    @classmethod
    def decode(cls, b: bytes) -> "Message":
        m = cls()
        body = bytearray()
        for sec in decode_all(b):
            if not isinstance(sec, Described):
                continue
            code = int(sec.descriptor) if isinstance(sec.descriptor, int) else None
            if code == MESSAGE_ANN:
                m.annotations = sec.value
            elif code == PROPERTIES:
                m.properties = sec.value
            elif code == APP_PROPERTIES:
                m.app_properties = sec.value
            elif code == DATA:
                body += sec.value
            elif code == VALUE:
                m.value = sec.value
        m.body = bytes(body) if body or m.value is None else None
        return m


# ------------------------------------------------------------------------------------ connection
class AmqpError(Exception):
    pass


class Link:
    """One attached link (receiver: deliveries queue in ``messages``)."""

    def __init__(self, conn: "AmqpConnection", handle: int, name: str, role_receiver: bool):
        self.conn, self.handle, self.name, self.receiver = conn, handle, name, role_receiver
        self.attached = threading.Event()
        self.remote_attach = None
        self.detached = threading.Event()
        self.error = None
        self.on_message = None
        self.delivery_count = 0
        self.credit = 0
        self.remote_credit = 0
        self._partial = bytearray()

    def flow(self, credit: int):
        self.credit = credit
        c = self.conn
        with c._lock:
            c._send(perf(FLOW, [UInt(c.next_incoming), UInt(c.incoming_window), UInt(c.next_outgoing),
                                UInt(c.outgoing_window), UInt(self.handle), UInt(self.delivery_count),
                                UInt(credit), None, False]), c.channel)

    def send(self, msg: Message, settled: bool = True):
        c = self.conn
        if not self.attached.wait(c.timeout):
            raise AmqpError("link not attached")
        with c._lock:
            tag = struct.pack(">I", c.next_outgoing)
            c._send(perf(TRANSFER, [UInt(self.handle), UInt(c.next_outgoing), tag, UInt(0), settled]), c.channel,
                    payload=msg.encode())
            c.next_outgoing += 1
            self.delivery_count += 1

    def detach(self):
        c = self.conn
        with c._lock:
            c._send(perf(DETACH, [UInt(self.handle), True]), c.channel)


class AmqpConnection:
    """Client connection with one session.  ``sasl``: (mechanism, user, password) -- PLAIN or
    ANONYMOUS; ``tls``: wrap the socket (Event Hubs: 5671)."""

    def __init__(self, host: str, port: int, sasl=("ANONYMOUS", None, None), tls: bool = False,
                 virtual_host: str | None = None, container_id: str | None = None, timeout: float = 10.0):
        self.host, self.port, self.sasl, self.tls = host, port, sasl, tls
        self.vhost = virtual_host or host
        self.container = container_id or f"sitewhere-{uuid.uuid4().hex[:8]}"
        self.timeout = timeout
        self.sock = None
        self._lock = threading.Lock()
        self.links: dict[int, Link] = {}
        self._by_remote: dict[int, Link] = {}
        self.channel = 0
        self.next_outgoing, self.incoming_window, self.outgoing_window = 0, 65536, 65536
        self.next_incoming = 0
        self._opened, self._begun, self._closed = threading.Event(), threading.Event(), threading.Event()
        self.error = None
        self._reader = None
        self.max_frame = 65536

    # ---- wire
    def _recv_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise AmqpError("connection closed")
            buf += chunk
        return bytes(buf)

    def _read_frame(self):
        size, doff, ftype, ch = struct.unpack(">IBBH", self._recv_exact(8))
        # a peer's frame header is untrusted: the size covers the 8-byte header and fits the
        # negotiated max-frame-size; the data offset (4-byte words) lies inside the frame
        # (AMQP 1.0 section 2.3.1).  Anything else closes the connection instead of buffering it.
        if size < 8 or size > max(self.max_frame, 512) or doff < 2 or doff * 4 > size:
            raise AmqpError(f"invalid frame header (size {size}, data offset {doff})")
        rest = self._recv_exact(size - 8)
        body = rest[doff * 4 - 8:]
        if not body:
            return ftype, ch, None, b""        # heartbeat
        p, i = decode(body)
        return ftype, ch, p, body[i:]

    def _send(self, p: Described, channel: int = 0, ftype: int = 0, payload: bytes = b""):
        self.sock.sendall(frame(encode(p) + payload, channel, ftype))

    # ---- handshake
    def open(self) -> "AmqpConnection":
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        if self.tls:
            ctx = ssl.create_default_context()
            s = ctx.wrap_socket(s, server_hostname=self.host)
        self.sock = s
        mech, user, pw = self.sasl
        s.sendall(SASL_HEADER)
        if self._recv_exact(8) != SASL_HEADER:
            raise AmqpError("peer refused the SASL layer")
        _, _, p, _ = self._read_frame()
        offered = p.value[0] if p and p.value else []
        offered = offered.items if isinstance(offered, Array) else (offered if isinstance(offered, list) else [offered])
        if mech not in offered:
            raise AmqpError(f"SASL mechanism {mech} not offered ({offered})")
        resp = b"\x00" + (user or "").encode() + b"\x00" + (pw or "").encode() if mech == "PLAIN" else b""
        self._send(perf(SASL_INIT, [Symbol(mech), resp, self.vhost]), ftype=1)
        _, _, p, _ = self._read_frame()
        if not p or int(p.descriptor) != SASL_OUTCOME or int(p.value[0]) != 0:
            raise AmqpError(f"SASL authentication failed ({p.value if p else None})")
        s.sendall(AMQP_HEADER)
        if self._recv_exact(8) != AMQP_HEADER:
            raise AmqpError("peer refused AMQP 1.0")
        self._send(perf(OPEN, [self.container, self.vhost, UInt(self.max_frame), UShort(255), UInt(60000)]))
        self._send(perf(BEGIN, [None, UInt(self.next_outgoing), UInt(self.incoming_window),
                                UInt(self.outgoing_window), UInt(255)]))
        s.settimeout(None)
        self._reader = threading.Thread(target=self._read_loop, daemon=True, name="amqp10-reader")
        self._reader.start()
        if not self._opened.wait(self.timeout) or not self._begun.wait(self.timeout):
            raise AmqpError(f"open / begin not answered ({self.error})")
        return self

    def _read_loop(self):
        try:
            while not self._closed.is_set():
                ftype, ch, p, payload = self._read_frame()
                if p is None:
                    continue
                self._dispatch(int(p.descriptor), p.value, payload)
        except Exception as e:  # noqa: BLE001 -- socket closed / protocol error ends the connection
            if not self._closed.is_set():
                self.error = e
        finally:
            self._closed.set()
            for lk in list(self.links.values()):
                lk.detached.set()

    def _dispatch(self, code: int, f: list, payload: bytes):
        f = list(f) + [None] * 14
        if code == OPEN:
            self.max_frame = min(self.max_frame, int(f[2] or self.max_frame))
            self._opened.set()
        elif code == BEGIN:
            self.next_incoming = int(f[1] or 0)
            self._begun.set()
        elif code == ATTACH:
            lk = self._by_name(f[0])
            if lk is not None:
                lk.remote_attach = f
                self._by_remote[int(f[1])] = lk
                lk.attached.set()
        elif code == FLOW:
            if f[4] is not None:
                lk = self._by_remote.get(int(f[4]))
                if lk is not None and not lk.receiver:
                    lk.remote_credit = int(f[6] or 0)
        elif code == TRANSFER:
            self.next_incoming += 1
            lk = self._by_remote.get(int(f[0]))
            if lk is None:
                return
            lk._partial += payload
            if f[5]:                                   # more: wait for the rest of the delivery
                return
            body, lk._partial = bytes(lk._partial), bytearray()
            lk.delivery_count += 1
            lk.credit -= 1
            if lk.on_message is not None:
                lk.on_message(Message.decode(body), f)
        elif code == DETACH:
            lk = self._by_remote.get(int(f[0]))
            if lk is not None:
                lk.error = f[2]
                lk.detached.set()
        elif code in (END, CLOSE):
            self.error = f[0]
            self._closed.set()

    def _by_name(self, name):
        for lk in self.links.values():
            if lk.name == name:
                return lk
        return None

    # ---- links
    def attach_receiver(self, address: str, filters: dict | None = None, credit: int = 100,
                        on_message=None, name: str | None = None) -> Link:
        """Receiving link from ``address``; ``filters``: the source filter set (e.g. an Event Hubs
        offset selector).  Settlement mode "settled" (the sender settles; at-least-once through the
        caller's checkpoints, as EventProcessorHost does)."""
        with self._lock:
            h = len(self.links)
            lk = Link(self, h, name or f"recv-{uuid.uuid4().hex[:8]}", True)
            lk.on_message = on_message
            self.links[h] = lk
            source = Described(ULong(SOURCE), [address, None, None, None, None, None, None,
                                               filters if filters else None])
            self._send(perf(ATTACH, [lk.name, UInt(h), True, UByte(1), UByte(0), source,
                                     Described(ULong(TARGET), [None]), None, None, None]), self.channel)
        if not lk.attached.wait(self.timeout):
            raise AmqpError(f"attach to {address} not answered")
        if lk.remote_attach[5] is None:
            raise AmqpError(f"attach to {address} refused")
        lk.flow(credit)
        return lk

    def attach_sender(self, address: str, name: str | None = None) -> Link:
        with self._lock:
            h = len(self.links)
            lk = Link(self, h, name or f"send-{uuid.uuid4().hex[:8]}", False)
            self.links[h] = lk
            self._send(perf(ATTACH, [lk.name, UInt(h), False, UByte(1), UByte(0), Described(ULong(SOURCE), [None]),
                                     Described(ULong(TARGET), [address]), None, None, UInt(0)]),
                       self.channel)
        if not lk.attached.wait(self.timeout):
            raise AmqpError(f"attach to {address} not answered")
        return lk

    def close(self):
        if self.sock is None:
            return
        try:
            with self._lock:
                self._send(perf(END, []), self.channel)
                self._send(perf(CLOSE, []))
        except OSError:
            pass
        self._closed.set()
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
        self.sock = None

    @property
    def closed(self) -> bool:
        return self._closed.is_set()
