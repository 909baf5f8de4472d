"""MQTT 3.1.1 client and broker (no external dependency).

The reference ingests device events over MQTT (``MqttInboundEventReceiver.java:40-309``: one
subscription thread + a processor pool, QoS configurable, ack after hand-off), delivers commands
by MQTT publish (``MqttCommandDeliveryProvider.java:87-111``) and publishes from outbound
connectors (``MqttOutboundConnector``).  All three sit on ``MqttLifecycleComponent``
(``sitewhere-communication/.../mqtt/MqttLifecycleComponent.java``): ``protocol`` tcp / ssl / tls,
``hostname``, ``port``, ``username`` / ``password``, trust and key stores, ``clientId``,
``cleanSession`` and ``qos`` (AT_MOST_ONCE / AT_LEAST_ONCE / EXACTLY_ONCE); the fusesource client
underneath reconnects by itself.  The image has no paho / mosquitto, so this module implements the
protocol:

* :class:`MqttClient` -- CONNECT with credentials, will and clean-session flag; TLS (CA file for
  the trust store, PEM certificate + key for the key store); PUBLISH at QoS 0/1/2 both ways (the
  QoS 2 four-way handshake, duplicate suppression of inbound QoS 2 ids); inbound QoS 1/2 acks sent
  after the handler returned (the reference's ack-after-hand-off); SUBSCRIBE / UNSUBSCRIBE with
  granted QoS; keep-alive pings; optional automatic reconnect that re-subscribes and retransmits
  unacknowledged publishes with the DUP flag.
* :class:`MqttBroker` -- the in-process stand-in the tests and ``serve --mqtt-port`` use: username /
  password check, TLS, persistent sessions (subscriptions and QoS>0 messages queued while the
  client is away), retained messages, wills on abnormal disconnect, keep-alive enforcement,
  session take-over by client id, ``+``/``#`` wildcards.
"""
from __future__ import annotations

import os
import socket
import ssl
import struct
import threading
import time
from collections import OrderedDict, deque

CONNECT, CONNACK, PUBLISH, PUBACK, PUBREC, PUBREL, PUBCOMP = 1, 2, 3, 4, 5, 6, 7
SUBSCRIBE, SUBACK, UNSUBSCRIBE, UNSUBACK, PINGREQ, PINGRESP, DISCONNECT = 8, 9, 10, 11, 12, 13, 14

CONNACK_CODES = {1: "unacceptable protocol version", 2: "identifier rejected", 3: "server unavailable",
                 4: "bad user name or password", 5: "not authorized"}
QOS_NAMES = {"AT_MOST_ONCE": 0, "AT_LEAST_ONCE": 1, "EXACTLY_ONCE": 2}


def parse_qos(q) -> int:
    """Reference ``QoS`` enum names or numbers -> 0/1/2."""
    if isinstance(q, str) and q.upper() in QOS_NAMES:
        return QOS_NAMES[q.upper()]
    q = int(q)
    if q not in (0, 1, 2):
        raise ValueError(f"invalid MQTT QoS {q}")
    return q


def _enc_len(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n % 128
        n //= 128
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _enc_str(s: str | bytes) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    return struct.pack("!H", len(b)) + b


def _recv_exact(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("closed")
        buf += chunk
    return bytes(buf)


MAX_PACKET = 256 << 20          # the protocol's own limit


def read_packet(sock):
    h = _recv_exact(sock, 1)[0]
    mult, length = 1, 0
    for _ in range(4):
        b = _recv_exact(sock, 1)[0]
        length += (b & 0x7F) * mult
        if not b & 0x80:
            break
        mult *= 128
    else:
        raise ConnectionError("malformed remaining length")
    body = _recv_exact(sock, length) if length else b""
    return h >> 4, h & 0x0F, body


class _Packets:
    """The packets of a QoS 0 PUBLISH-only batch as (type, flags, start, body start, end) on demand:
    the fast paths (a broker forwarding the batch whole, a client handing payloads over by topic)
    read the header array and never build the tuples."""
    __slots__ = ("hdr",)

    def __init__(self, hdr):
        self.hdr = hdr                            # int64 [k, 4]: first byte, start, body start, end

    def __len__(self):
        return len(self.hdr)

    def _row(self, r):
        return (r[0] >> 4, r[0] & 0x0F, r[1], r[2], r[3])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._row(r) for r in self.hdr[i].tolist()]
        return self._row(self.hdr[i].tolist())

    def __iter__(self):
        return iter([self._row(r) for r in self.hdr.tolist()])


class PacketReader:
    """Buffered MQTT packet reader of one connection: one ``recv_into`` per chunk of up to ``CHUNK``
    bytes, the complete packets in it found natively (``swmqtt_scan``) -- ``read_packet`` costs
    three receives and a Python parse per packet."""
    CHUNK = 1 << 20

    def __init__(self, sock):
        import numpy as np
        from .._native import native
        self.sock = sock
        self.a = np.empty(2 * self.CHUNK, np.uint8)
        self.lo = self.hi = 0
        self._lib = native()
        self._hdr = np.empty(4 * 8192, np.int64)
        self._used = np.zeros(1, np.int64)
        self._pending = None                      # (data, packets, next index) of the last batch
        self._first = np.empty(self.QOS0_TOPICS, np.int64)
        self._tix = np.empty(8192, np.int32)
        # the last batch from read_batch when every packet of it is a QoS 0, non-retained PUBLISH:
        # (distinct topics as bytes, topic number per packet) -- else None (swmqtt_qos0_topics)
        self.qos0 = None

    QOS0_TOPICS = 16

    def _fill(self):
        import numpy as np
        if self.hi == len(self.a):
            if self.lo:                           # move the partial packet to the front
                n = self.hi - self.lo
                self.a[:n] = self.a[self.lo:self.hi]
                self.lo, self.hi = 0, n
            else:                                 # one packet larger than the buffer
                b = np.empty(2 * len(self.a), np.uint8)
                b[:self.hi] = self.a[:self.hi]
                self.a = b
        got = self.sock.recv_into(memoryview(self.a)[self.hi:], min(self.CHUNK, len(self.a) - self.hi))
        if not got:
            raise ConnectionError("closed")
        self.hi += got

    def _scan(self):
        while True:
            n = self.hi - self.lo
            if n >= 2:
                k = int(self._lib.swmqtt_scan(self.a.ctypes.data + self.lo, n, self._hdr.ctypes.data,
                                              len(self._hdr) // 4, MAX_PACKET, self._used.ctypes.data))
                if k < 0:
                    raise ConnectionError("malformed remaining length" if k == -1 else "packet too large")
                if k:
                    used = int(self._used[0])
                    nd = int(self._lib.swmqtt_qos0_topics(self.a.ctypes.data + self.lo, self._hdr.ctypes.data, k,
                                                          self._first.ctypes.data, self.QOS0_TOPICS,
                                                          self._tix.ctypes.data))
                    data = self.a[self.lo:self.lo + used].tobytes()
                    self.lo += used
                    if self.lo == self.hi:
                        self.lo = self.hi = 0
                    if nd > 0:
                        hk = self._hdr[:4 * k].reshape(k, 4).copy()
                        tops = []
                        for i in self._first[:nd].tolist():
                            bs = int(hk[i, 2])
                            tl = (data[bs] << 8) | data[bs + 1]
                            tops.append(data[bs + 2:bs + 2 + tl])
                        self.qos0 = (tops, self._tix[:k].copy(), hk)
                        return data, _Packets(hk)
                    self.qos0 = None
                    h = self._hdr[:4 * k].reshape(k, 4).tolist()
                    return data, [(x[0] >> 4, x[0] & 0x0F, x[1], x[2], x[3]) for x in h]
            self._fill()

    def read(self):
        """The next packet: (type, flags, body)."""
        if self._pending is None:
            d, p = self._scan()
            self._pending = (d, p, 0)
        d, p, i = self._pending
        t, f, _a, bs, e = p[i]
        self._pending = (d, p, i + 1) if i + 1 < len(p) else None
        return t, f, d[bs:e]

    def read_batch(self):
        """Every complete packet buffered (blocks for the first): (data, [(type, flags, start, body
        start, end)]) with offsets into ``data``, one bytes object of the packets."""
        if self._pending is not None:
            d, p, i = self._pending
            self._pending = None
            self.qos0 = None
            return d, p[i:]
        return self._scan()


def packet(ptype: int, flags: int, body: bytes) -> bytes:
    return bytes([(ptype << 4) | flags]) + _enc_len(len(body)) + body


def publish_packet(topic: str, payload: bytes, qos: int = 0, pid: int = 0, retain: bool = False,
                   dup: bool = False) -> bytes:
    flags = (qos << 1) | (1 if retain else 0) | (8 if dup and qos else 0)
    return packet(PUBLISH, flags, _enc_str(topic) + (struct.pack("!H", pid) if qos else b"") + bytes(payload))


def parse_publish(flags: int, body: bytes) -> tuple[str, int, int, bool, bool, bytes]:
    """(topic, qos, packet id, retain, dup, payload) of a PUBLISH body."""
    qos = (flags >> 1) & 3
    if qos == 3:
        raise ConnectionError("invalid QoS 3 publish")
    tl = struct.unpack("!H", body[:2])[0]
    topic = body[2:2 + tl].decode()
    pos, pid = 2 + tl, 0
    if qos:
        pid = struct.unpack("!H", body[pos:pos + 2])[0]
        pos += 2
    return topic, qos, pid, bool(flags & 1), bool(flags & 8), body[pos:]


def topic_matches(filt: str, topic: str) -> bool:
    fp, tp = filt.split("/"), topic.split("/")
    if topic.startswith("$") and fp[0] in ("+", "#"):
        return False                    # $SYS-style topics never match a leading wildcard
    for i, f in enumerate(fp):
        if f == "#":
            return True
        if i >= len(tp):
            return False
        if f != "+" and f != tp[i]:
            return False
    return len(fp) == len(tp)


def client_ssl_context(ca_file: str | None = None, cert_file: str | None = None, key_file: str | None = None,
                       check_hostname: bool = True) -> ssl.SSLContext:
    """TLS context of the reference's trust store (``ca_file``: PEM CAs) and key store (PEM
    certificate + key for mutual TLS)."""
    ctx = ssl.create_default_context(cafile=ca_file)
    ctx.check_hostname = check_hostname
    if cert_file:
        ctx.load_cert_chain(cert_file, key_file)
    return ctx


# ------------------------------------------------------------------------------ client
class MqttClient:
    """MQTT 3.1.1 client.  ``on_message(handler)`` registers ``handler(topic, payload)``, called on
    the reader thread; inbound QoS 1/2 messages are acknowledged when every handler has returned."""

    def __init__(self, host: str, port: int, client_id: str | None = None, keepalive: int = 60,
                 username: str | None = None, password: str | None = None, clean_session: bool = True,
                 protocol: str = "tcp", ca_file: str | None = None, cert_file: str | None = None,
                 key_file: str | None = None, ssl_context: ssl.SSLContext | None = None,
                 will: tuple | None = None, reconnect: bool = False, max_backoff_s: float = 5.0):
        self.host, self.port = host, int(port)
        self.client_id = client_id or f"sw-{os.urandom(6).hex()}"
        self.keepalive = int(keepalive)
        self.username, self.password, self.clean_session = username, password, bool(clean_session)
        self.protocol = (protocol or "tcp").lower()
        if self.protocol not in ("tcp", "ssl", "tls"):
            raise ValueError(f"unsupported MQTT protocol {protocol!r}")
        if self.protocol != "tcp" and ssl_context is None:
            ssl_context = client_ssl_context(ca_file, cert_file, key_file)
        self.ssl_context = ssl_context
        self.will = will                    # (topic, payload, qos, retain)
        self.reconnect, self.max_backoff = bool(reconnect), float(max_backoff_s)
        self.sock = None
        self.session_present = False
        self.connected = threading.Event()
        self.reconnects = 0
        self._pid = 0
        self._handlers: list = []
        self._batch_handlers: list = []           # handler(topic, [payloads]): QoS 0 deliveries by batch
        self._lock = threading.RLock()          # send + state
        self._acks: dict[int, tuple[threading.Event, list]] = {}        # SUBACK / UNSUBACK waiters
        self._out: OrderedDict = OrderedDict()  # pid -> [stage, packet, done Event]  (QoS 1/2 in flight)
        self._in_qos2: set[int] = set()         # inbound QoS 2 ids between PUBREC and PUBREL
        self._subs: dict[str, int] = {}
        self._closed = False
        self._reader = None
        self._last_send = self._last_recv = time.monotonic()
        self._ping_out = None

    # -- connection
    def _open(self, timeout: float):
        s = socket.create_connection((self.host, self.port), timeout=timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if self.ssl_context is not None:
            s = self.ssl_context.wrap_socket(s, server_hostname=self.host)
        flags = 0x02 if self.clean_session else 0
        payload = _enc_str(self.client_id)
        if self.will:
            wt, wp, wq, wr = (tuple(self.will) + (0, False))[:4]
            flags |= 0x04 | (parse_qos(wq) << 3) | (0x20 if wr else 0)
            payload += _enc_str(wt) + _enc_str(wp if isinstance(wp, (bytes, bytearray)) else str(wp).encode())
        if self.username is not None:
            flags |= 0x80
            payload += _enc_str(self.username)
            if self.password is not None:
                flags |= 0x40
                payload += _enc_str(self.password)
        s.sendall(packet(CONNECT, 0, _enc_str("MQTT") + bytes([4, flags]) + struct.pack("!H", self.keepalive)
                         + payload))
        t, _, body = read_packet(s)
        if t != CONNACK or len(body) < 2:
            s.close()
            raise ConnectionError("MQTT: no CONNACK")
        if body[1] != 0:
            s.close()
            raise ConnectionError(f"MQTT connect refused: {CONNACK_CODES.get(body[1], body[1])}")
        s.settimeout(None)
        with self._lock:
            self.sock = s
            self.session_present = bool(body[0] & 1)
            self._last_send = self._last_recv = time.monotonic()
            self._ping_out = None
        self.connected.set()

    def connect(self, timeout: float = 5.0):
        self._open(timeout)
        self._reader = threading.Thread(target=self._run, daemon=True, name=f"mqtt-{self.client_id}")
        self._reader.start()
        if self.keepalive > 0:
            threading.Thread(target=self._pinger, daemon=True, name=f"mqtt-ping-{self.client_id}").start()
        return self

    def _after_reconnect(self):
        """Restore subscriptions (unless the broker kept the session) and retransmit in-flight
        publishes (DUP) / releases."""
        with self._lock:
            subs = dict(self._subs) if not self.session_present else {}
            pending = list(self._out.items())
        for filt, q in subs.items():
            pid = self._next_pid()
            self._send(packet(SUBSCRIBE, 2, struct.pack("!H", pid) + _enc_str(filt) + bytes([q])))
        for pid, (stage, pkt, _) in pending:
            if stage == "pubcomp":
                self._send(packet(PUBREL, 2, struct.pack("!H", pid)))
            else:
                self._send(bytes([pkt[0] | 0x08]) + pkt[1:])       # same packet, DUP set

    def _run(self):
        while not self._closed:
            try:
                self._read_loop(self.sock)
            except (ConnectionError, OSError, struct.error, ValueError, IndexError):
                pass
            self.connected.clear()
            try:
                self.sock.close()
            except OSError:
                pass
            if self._closed or not self.reconnect:
                break
            backoff = 0.05
            while not self._closed:
                try:
                    self._open(5.0)
                    self.reconnects += 1
                    self._after_reconnect()
                    break
                except (ConnectionError, OSError, ssl.SSLError):
                    time.sleep(backoff)
                    backoff = min(backoff * 2, self.max_backoff)

    def _read_loop(self, sock):
        reader = PacketReader(sock)
        while not self._closed:
            data, pkts = reader.read_batch()
            self._last_recv = time.monotonic()
            handlers = list(self._handlers)
            batch_handlers = list(self._batch_handlers)
            if reader.qos0 is not None and batch_handlers and not handlers:
                # QoS 0 publishes only: each topic's payloads handed over together, in order
                tops, tix, hk = reader.qos0
                bs_all, end_all = hk[:, 2], hk[:, 3]
                for q in range(len(tops)):
                    sel = slice(None) if len(tops) == 1 else (tix == q)
                    topic = tops[q].decode()
                    skip = 2 + len(tops[q])
                    payloads = [data[b0 + skip:e0] for b0, e0 in zip(bs_all[sel].tolist(), end_all[sel].tolist())]
                    for h in batch_handlers:
                        try:
                            h(topic, payloads)
                        except Exception:  # noqa: BLE001 -- a handler error never kills the connection
                            pass
                continue
            for t, flags, _a, bs, e in pkts:
                if t == PUBLISH and not flags & 0x06:          # QoS 0: straight to the handlers
                    tl = (data[bs] << 8) | data[bs + 1]
                    topic, payload = data[bs + 2:bs + 2 + tl].decode(), data[bs + 2 + tl:e]
                    for h in batch_handlers:
                        try:
                            h(topic, [payload])
                        except Exception:  # noqa: BLE001 -- a handler error never kills the connection
                            pass
                    for h in handlers:
                        try:
                            h(topic, payload)
                        except Exception:  # noqa: BLE001 -- a handler error never kills the connection
                            pass
                    continue
                self._on_packet(t, flags, data[bs:e])

    def _on_packet(self, t: int, flags: int, body: bytes):
        """One packet other than a QoS 0 PUBLISH (acknowledgements, QoS 1 / 2 deliveries)."""
        if t == PUBLISH:
            topic, qos, pid, _retain, _dup, payload = parse_publish(flags, body)
            if qos == 2 and pid in self._in_qos2:
                self._send(packet(PUBREC, 0, struct.pack("!H", pid)))   # duplicate: already delivered
                return
            for h in list(self._handlers):
                try:
                    h(topic, payload)
                except Exception:  # noqa: BLE001 -- a handler error never kills the connection
                    pass
            if qos == 1:
                self._send(packet(PUBACK, 0, struct.pack("!H", pid)))
            elif qos == 2:
                self._in_qos2.add(pid)
                self._send(packet(PUBREC, 0, struct.pack("!H", pid)))
        elif t == PUBREL:
            pid = struct.unpack("!H", body[:2])[0]
            self._in_qos2.discard(pid)
            self._send(packet(PUBCOMP, 0, body[:2]))
        elif t in (PUBACK, PUBCOMP):
            pid = struct.unpack("!H", body[:2])[0]
            with self._lock:
                ent = self._out.pop(pid, None)
            if ent is not None:
                ent[2].set()
        elif t == PUBREC:
            pid = struct.unpack("!H", body[:2])[0]
            with self._lock:
                ent = self._out.get(pid)
                if ent is not None:
                    ent[0] = "pubcomp"
            self._send(packet(PUBREL, 2, body[:2]))
        elif t in (SUBACK, UNSUBACK):
            pid = struct.unpack("!H", body[:2])[0]
            w = self._acks.pop(pid, None)
            if w is not None:
                w[1].append(body[2:])
                w[0].set()
        elif t == PINGRESP:
            self._ping_out = None


    def _pinger(self):
        while not self._closed:
            time.sleep(min(0.5, self.keepalive / 4))
            if not self.connected.is_set():
                continue
            now = time.monotonic()
            if self._ping_out is not None and now - self._ping_out > self.keepalive:
                try:                            # no PINGRESP within a keep-alive: the link is dead
                    self.sock.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                continue
            if now - self._last_send >= self.keepalive / 2 and self._ping_out is None:
                try:
                    self._ping_out = now
                    self._send(packet(PINGREQ, 0, b""))
                except OSError:
                    pass

    def _next_pid(self) -> int:
        with self._lock:
            for _ in range(65535):
                self._pid = self._pid % 65535 + 1
                if self._pid not in self._out and self._pid not in self._acks:
                    return self._pid
        raise RuntimeError("MQTT: no free packet identifier")

    def _send(self, data: bytes):
        with self._lock:
            self.sock.sendall(data)
            self._last_send = time.monotonic()

    # -- API
    def on_message(self, handler):
        self._handlers.append(handler)

    def on_messages(self, handler):
        """``handler(topic, payloads)``: QoS 0 deliveries a topic at a time (a read's messages of one
        topic, in order); QoS 1 / 2 deliveries still go to :meth:`on_message` handlers only."""
        self._batch_handlers.append(handler)

    def subscribe(self, filt: str, qos: int = 1, timeout: float = 5.0) -> int:
        """Subscribe; returns the granted QoS (0x80 = refused)."""
        qos = parse_qos(qos)
        pid = self._next_pid()
        w = self._acks[pid] = (threading.Event(), [])
        with self._lock:
            self._subs[filt] = qos
        self._send(packet(SUBSCRIBE, 2, struct.pack("!H", pid) + _enc_str(filt) + bytes([qos])))
        if not w[0].wait(timeout):
            raise TimeoutError("SUBACK not received")
        granted = w[1][0][0] if w[1] and w[1][0] else 0x80
        if granted == 0x80:
            with self._lock:
                self._subs.pop(filt, None)
        return granted

    def unsubscribe(self, filt: str, timeout: float = 5.0):
        pid = self._next_pid()
        w = self._acks[pid] = (threading.Event(), [])
        with self._lock:
            self._subs.pop(filt, None)
        self._send(packet(UNSUBSCRIBE, 2, struct.pack("!H", pid) + _enc_str(filt)))
        if not w[0].wait(timeout):
            raise TimeoutError("UNSUBACK not received")

    def publish(self, topic: str, payload: bytes, qos: int = 0, retain: bool = False, timeout: float = 5.0):
        """Publish; QoS 1 returns after PUBACK, QoS 2 after PUBCOMP (TimeoutError otherwise; with
        ``reconnect`` the message stays in flight and is retransmitted on the next connection)."""
        qos = parse_qos(qos)
        if not qos:
            self._send(publish_packet(topic, payload, 0, retain=retain))
            return
        pid = self._next_pid()
        pkt = publish_packet(topic, payload, qos, pid, retain)
        done = threading.Event()
        with self._lock:
            self._out[pid] = ["puback" if qos == 1 else "pubrec", pkt, done]
        try:
            self._send(pkt)
        except OSError:
            if not self.reconnect:
                with self._lock:
                    self._out.pop(pid, None)
                raise
        if not done.wait(timeout):
            raise TimeoutError("PUBACK not received" if qos == 1 else "PUBCOMP not received")

    def publish_many(self, msgs, qos: int = 0, retain: bool = False, timeout: float = 5.0):
        """Publish [(topic, payload)]: QoS 0 packets go out in one write; QoS 1 / 2 are all put
        in flight before any acknowledgement is awaited (a batch costs one round trip, not one
        per message)."""
        qos = parse_qos(qos)
        if not qos:
            self._send(b"".join(publish_packet(t, p, 0, retain=retain) for t, p in msgs))
            return
        waits, pkts = [], []
        with self._lock:
            for t, p in msgs:
                pid = self._next_pid()
                pkt = publish_packet(t, p, qos, pid, retain)
                done = threading.Event()
                self._out[pid] = ["puback" if qos == 1 else "pubrec", pkt, done]
                waits.append(done)
                pkts.append(pkt)
        try:
            self._send(b"".join(pkts))
        except OSError:
            if not self.reconnect:
                raise
        end = time.monotonic() + timeout
        for w in waits:
            if not w.wait(max(0.0, end - time.monotonic())):
                raise TimeoutError("PUBACK not received" if qos == 1 else "PUBCOMP not received")

    def publish_framed_qos0(self, packets):
        """Already framed QoS 0 PUBLISH packets (``swmqtt_publish_qos0``), in one write (any buffer;
        sent before this returns)."""
        self._send(packets)

    @property
    def inflight(self) -> int:
        return len(self._out)

    def ping(self):
        self._send(packet(PINGREQ, 0, b""))

    def disconnect(self):
        self._closed = True
        try:
            self._send(packet(DISCONNECT, 0, b""))
        except (OSError, AttributeError):
            pass
        try:      # shutdown first: the reader thread blocked in recv returns now, before the fd can be reused
            self.sock.shutdown(socket.SHUT_RDWR)
        except (OSError, AttributeError):
            pass
        try:
            self.sock.close()
        except (OSError, AttributeError):
            pass
        self.connected.clear()


MQTT_OPTIONS = ("protocol", "username", "password", "trustStorePath", "keyStorePath", "keyPath", "clientId",
                "cleanSession")


def client_from_config(cfg: dict, **kw) -> MqttClient:
    """An :class:`MqttClient` from the reference's MQTT attributes (``MqttLifecycleComponent``):
    protocol, hostname/host, port, username, password, trustStorePath (PEM CA file),
    keyStorePath (PEM certificate, key in ``keyPath`` or the same file), clientId, cleanSession."""
    cert = cfg.get("keyStorePath")
    return MqttClient(cfg.get("hostname") or cfg.get("host", "127.0.0.1"), int(cfg.get("port", 1883)),
                      client_id=cfg.get("clientId"), username=cfg.get("username"), password=cfg.get("password"),
                      clean_session=str(cfg.get("cleanSession", True)).lower() not in ("false", "0"),
                      protocol=cfg.get("protocol", "tcp"), ca_file=cfg.get("trustStorePath"),
                      cert_file=cert, key_file=cfg.get("keyPath") or cert, **kw)


# ------------------------------------------------------------------------------ broker
class _Session:
    __slots__ = ("client_id", "clean", "subs", "queue", "out", "in_qos2", "conn", "wlock", "pid", "will")

    def __init__(self, client_id: str, clean: bool):
        self.client_id, self.clean = client_id, clean
        self.subs: dict[str, int] = {}
        self.queue: deque = deque(maxlen=100_000)      # (topic, payload, qos, retain) while offline
        self.out: OrderedDict = OrderedDict()          # pid -> [stage, packet]
        self.in_qos2: set[int] = set()
        self.conn = None
        self.wlock = threading.Lock()
        self.pid = 0
        self.will = None

    def next_pid(self) -> int:
        for _ in range(65535):
            self.pid = self.pid % 65535 + 1
            if self.pid not in self.out:
                return self.pid
        raise RuntimeError("session out of packet identifiers")


class MqttBroker:
    """Threaded MQTT 3.1.1 broker (one thread per connection).  ``users``: {username: password}
    enables authentication; ``ssl_context``: a server TLS context."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, users: dict | None = None,
                 ssl_context: ssl.SSLContext | None = None):
        self.host = host
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self.port = self._srv.getsockname()[1]
        self.users = users
        self.ssl_context = ssl_context
        self._sessions: dict[str, _Session] = {}
        self._retained: dict[str, tuple[bytes, int]] = {}
        self._conns: set = set()
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._t = None
        self.published = 0
        self._route_cache: dict[bytes, tuple] = {}     # topic -> subscribed sessions (QoS 0 forwarding)

    def start(self):
        self._srv.listen(128)
        self._t = threading.Thread(target=self._accept, daemon=True, name="mqtt-broker")
        self._t.start()
        return self

    def _accept(self):
        self._srv.settimeout(0.2)
        while not self._stop.is_set():
            try:
                c, _ = self._srv.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._serve, args=(c,), daemon=True, name="mqtt-conn").start()

    @staticmethod
    def _send(sess: _Session, c, data: bytes) -> bool:
        with sess.wlock:
            try:
                c.sendall(data)
                return True
            except OSError:
                return False

    def _connect(self, c, body: bytes):
        """Parse CONNECT; returns (session, keepalive, session_present) or None after a refusal."""
        pl = struct.unpack("!H", body[:2])[0]
        name, pos = body[2:2 + pl], 2 + pl
        level, flags = body[pos], body[pos + 1]
        keepalive = struct.unpack("!H", body[pos + 2:pos + 4])[0]
        pos += 4

        def s():
            nonlocal pos
            n = struct.unpack("!H", body[pos:pos + 2])[0]
            v = body[pos + 2:pos + 2 + n]
            pos += 2 + n
            return v
        cid = s().decode()
        will = None
        if flags & 0x04:
            wt = s().decode()
            will = (wt, s(), (flags >> 3) & 3, bool(flags & 0x20))
        user = s().decode() if flags & 0x80 else None
        pw = s().decode() if flags & 0x40 else None
        clean = bool(flags & 0x02)

        def refuse(code):
            c.sendall(packet(CONNACK, 0, bytes([0, code])))
            return None
        if (name, level) not in ((b"MQTT", 4), (b"MQIsdp", 3)):
            return refuse(1)
        if not cid:
            if not clean:
                return refuse(2)
            cid = f"auto-{os.urandom(6).hex()}"
        if self.users is not None and (user is None or self.users.get(user) != pw):
            return refuse(4)
        with self._lock:
            old = self._sessions.get(cid)
            if old is not None and old.conn is not None:        # take-over: drop the older connection
                try:
                    old.conn.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                old.will = None
            present = old is not None and not clean and not old.clean
            sess = old if present else _Session(cid, clean)
            sess.clean = clean
            sess.will = will
            sess.conn = c
            self._sessions[cid] = sess
            self._route_cache.clear()
        c.sendall(packet(CONNACK, 0, bytes([1 if present else 0, 0])))
        return sess, keepalive, present

    def _serve(self, c):
        sess, graceful = None, False
        try:
            if self.ssl_context is not None:
                c.settimeout(10)
                c = self.ssl_context.wrap_socket(c, server_side=True)
            with self._lock:
                self._conns.add(c)
            c.settimeout(10)
            reader = PacketReader(c)
            t, _, body = reader.read()
            if t != CONNECT:
                return
            r = self._connect(c, body)
            if r is None:
                return
            sess, keepalive, _present = r
            c.settimeout(keepalive * 1.5 if keepalive else None)
            with sess.wlock:
                pending = [(pid, ent[0], ent[1]) for pid, ent in sess.out.items()]
                queued = list(sess.queue)
                sess.queue.clear()
            for pid, stage, pkt in pending:                 # retransmit what the client never acked
                self._send(sess, c, packet(PUBREL, 2, struct.pack("!H", pid)) if stage == "pubcomp"
                           else bytes([pkt[0] | 0x08]) + pkt[1:])
            for q in queued:                                # then what arrived while it was offline
                self._deliver(sess, *q)
            while not self._stop.is_set():
                data, pkts = reader.read_batch()
                if reader.qos0 is not None and self._forward_batch(data, pkts, reader.qos0[0]):
                    continue
                k = 0
                while k < len(pkts):
                    t, flags, a0, bs, e = pkts[k]
                    if t == PUBLISH and not flags & 0x07:
                        # a run of QoS 0, non-retained publishes: forwarded as they came, one send of
                        # the run per subscriber when every topic of it has the same subscribers
                        k = self._forward_run(data, pkts, k)
                        continue
                    k += 1
                    if not self._handle(sess, c, t, flags, data[bs:e]):
                        graceful = True
                        break
                else:
                    continue
                break
        except (ConnectionError, OSError, IndexError, struct.error, UnicodeDecodeError, ssl.SSLError):
            pass
        finally:
            with self._lock:
                self._conns.discard(c)
            if sess is not None:
                with self._lock:
                    mine = sess.conn is c
                    if mine:
                        sess.conn = None
                        if sess.clean and self._sessions.get(sess.client_id) is sess:
                            del self._sessions[sess.client_id]
                            self._route_cache.clear()
                if mine and not graceful and sess.will is not None and not self._stop.is_set():
                    wt, wp, wq, wr = sess.will
                    self.route(wt, wp, wq, wr)
                sess.will = None
            try:
                c.close()
            except OSError:
                pass

    def _handle(self, sess: "_Session", c, t: int, flags: int, body: bytes) -> bool:
        """One packet of a connected session (everything but forwarded QoS 0 runs); False on
        DISCONNECT."""
        if t == PUBLISH:
            topic, qos, pid, retain, _dup, payload = parse_publish(flags, body)
            if qos == 2:
                if pid not in sess.in_qos2:
                    sess.in_qos2.add(pid)
                    self.route(topic, payload, qos, retain)
                self._send(sess, c, packet(PUBREC, 0, struct.pack("!H", pid)))
                return True
            self.route(topic, payload, qos, retain)
            if qos == 1:
                self._send(sess, c, packet(PUBACK, 0, struct.pack("!H", pid)))
        elif t == PUBREL:
            sess.in_qos2.discard(struct.unpack("!H", body[:2])[0])
            self._send(sess, c, packet(PUBCOMP, 0, body[:2]))
        elif t in (PUBACK, PUBCOMP):
            with sess.wlock:
                sess.out.pop(struct.unpack("!H", body[:2])[0], None)
        elif t == PUBREC:
            pid = struct.unpack("!H", body[:2])[0]
            rel = packet(PUBREL, 2, body[:2])
            with sess.wlock:
                if pid in sess.out:
                    sess.out[pid] = ["pubcomp", rel]
            self._send(sess, c, rel)
        elif t == SUBSCRIBE:
            pid, pos, granted, new = body[:2], 2, bytearray(), []
            while pos < len(body):
                ln = struct.unpack("!H", body[pos:pos + 2])[0]
                filt = body[pos + 2:pos + 2 + ln].decode()
                q = body[pos + 2 + ln] & 3
                pos += 3 + ln
                if q == 3 or not filt:
                    granted.append(0x80)
                    continue
                with self._lock:
                    sess.subs[filt] = q
                    self._route_cache.clear()
                granted.append(q)
                new.append((filt, q))
            self._send(sess, c, packet(SUBACK, 0, pid + bytes(granted)))
            with self._lock:
                retained = [(tp, p, rq) for tp, (p, rq) in self._retained.items()]
            for filt, q in new:                     # retained messages of the new filters
                for tp, p, rq in retained:
                    if topic_matches(filt, tp):
                        self._deliver(sess, tp, p, min(q, rq), True)
        elif t == UNSUBSCRIBE:
            pid, pos = body[:2], 2
            while pos < len(body):
                ln = struct.unpack("!H", body[pos:pos + 2])[0]
                with self._lock:
                    sess.subs.pop(body[pos + 2:pos + 2 + ln].decode(), None)
                    self._route_cache.clear()
                pos += 2 + ln
            self._send(sess, c, packet(UNSUBACK, 0, pid))
        elif t == PINGREQ:
            self._send(sess, c, packet(PINGRESP, 0, b""))
        elif t == DISCONNECT:
            return False
        return True

    def _targets(self, topic: bytes) -> tuple:
        """Sessions subscribed to ``topic`` (cached per topic until a subscription or session
        changes); a session granted QoS 0 or more receives a QoS 0 publish at QoS 0."""
        t = self._route_cache.get(topic)
        if t is None:
            ts = topic.decode()
            with self._lock:
                t = tuple(s for s in self._sessions.values() if any(topic_matches(f, ts) for f in s.subs))
                if len(self._route_cache) > 65536:
                    self._route_cache.clear()
                self._route_cache[topic] = t
        return t

    def _forward_batch(self, data: bytes, pkts: list, topics: list) -> bool:
        """A batch of QoS 0, non-retained publishes only, whose topics (``topics``: the distinct
        ones) all have the same subscribers: forwarded whole, one send per subscriber, without a
        per-packet step (what ``_forward_run`` does packet by packet).  False: not applicable."""
        tg = None
        for t in topics:
            x = self._targets(t)
            if tg is None:
                tg = x
            elif x is not tg and x != tg:
                return False
        self.published += len(pkts)
        if tg:
            for s in tg:
                with s.wlock:
                    conn = s.conn
                if conn is not None:
                    self._send(s, conn, data)
        return True

    def _forward_run(self, data: bytes, pkts: list, k: int) -> int:
        """Forward the QoS 0 / non-retained PUBLISH packets from ``pkts[k]`` on while their topics
        have the same subscribers (byte-identical to what ``route`` would send them); returns the
        index after the run."""
        n = len(pkts)
        start = k
        tg = None
        while k < n:
            t, flags, a0, bs, e = pkts[k]
            if t != PUBLISH or flags & 0x07:
                break
            tl = (data[bs] << 8) | data[bs + 1]
            x = self._targets(data[bs + 2:bs + 2 + tl])
            if tg is None:
                tg = x
            elif x is not tg and x != tg:
                break
            k += 1
        self.published += k - start
        if tg:
            chunk = data[pkts[start][2]:pkts[k - 1][4]]
            for s in tg:
                with s.wlock:
                    conn = s.conn
                if conn is not None:
                    self._send(s, conn, chunk)
        return k

    def _deliver(self, sess: _Session, topic: str, payload: bytes, qos: int, retain: bool = False):
        # the connection check and the in-flight / offline bookkeeping happen under the session's
        # write lock, the lock a (re)connecting session drains both under: a message racing a
        # reconnect is either retransmitted or queued there, never parked on the old connection
        with sess.wlock:
            c = sess.conn
            if c is None:
                if qos and not sess.clean:
                    sess.queue.append((topic, payload, qos, retain))
                return
            if qos:
                pid = sess.next_pid()
                pkt = publish_packet(topic, payload, qos, pid, retain)
                sess.out[pid] = ["puback" if qos == 1 else "pubrec", pkt]
            else:
                pkt = publish_packet(topic, payload, 0, retain=retain)
        self._send(sess, c, pkt)

    def route(self, topic: str, payload: bytes, qos: int = 0, retain: bool = False):
        """Publish ``payload`` to every matching subscription at min(publish QoS, granted QoS)."""
        self.published += 1
        payload = bytes(payload)
        with self._lock:
            if retain:
                if payload:
                    self._retained[topic] = (payload, qos)
                else:
                    self._retained.pop(topic, None)
            targets = []
            for s in self._sessions.values():
                q = max((sq for f, sq in s.subs.items() if topic_matches(f, topic)), default=-1)
                if q >= 0:
                    targets.append((s, min(q, qos)))
        for s, q in targets:
            self._deliver(s, topic, payload, q)

    def session(self, client_id: str) -> _Session | None:
        return self._sessions.get(client_id)

    def stop(self):
        self._stop.set()
        try:
            self._srv.shutdown(socket.SHUT_RDWR)        # wakes the accept thread (close alone does not)
        except OSError:
            pass
        if self._t is not None and self._t is not threading.current_thread():
            self._t.join(2)                             # the port is free once stop() returns
        try:
            self._srv.close()
        except OSError:
            pass
        with self._lock:
            conns = list(self._conns)
        for c in conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass
