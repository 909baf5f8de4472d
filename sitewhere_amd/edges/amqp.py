"""AMQP 0-9-1 (RabbitMQ) client, embedded broker, receiver and outbound connector.

Reference: ``service-event-sources/.../sources/rabbitmq/RabbitMqInboundEventReceiver.java`` (consume a
queue, hand bodies to the event source), ``service-outbound-connectors/.../rabbitmq/
RabbitMqOutboundConnector.java`` (publish enriched events to an exchange / routing key) and the
reference's embedded ActiveMQ ``BrokerService`` used by ``EventSourceTests.java:82-111``.  No AMQP
library is available, so the wire protocol is implemented here: frames, field tables, the
connection/channel handshake, queue.declare, basic.publish (method + content header + body
frames), basic.consume / deliver / ack and connection.close.  :class:`AmqpBroker` is a small
in-process broker (default exchange routing: routing key = queue name; named exchanges route by
bindings of exact routing keys) for tests and single-node deployments.
"""
from __future__ import annotations

import itertools
import queue
import socket
import struct
import threading
from collections import defaultdict

from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent

PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"
FRAME_METHOD, FRAME_HEADER, FRAME_BODY, FRAME_HEARTBEAT = 1, 2, 3, 8
FRAME_END = 0xCE

CONNECTION_START, CONNECTION_START_OK = (10, 10), (10, 11)
CONNECTION_TUNE, CONNECTION_TUNE_OK = (10, 30), (10, 31)
CONNECTION_OPEN, CONNECTION_OPEN_OK = (10, 40), (10, 41)
CONNECTION_CLOSE, CONNECTION_CLOSE_OK = (10, 50), (10, 51)
CHANNEL_OPEN, CHANNEL_OPEN_OK = (20, 10), (20, 11)
CHANNEL_CLOSE, CHANNEL_CLOSE_OK = (20, 40), (20, 41)
EXCHANGE_DECLARE, EXCHANGE_DECLARE_OK = (40, 10), (40, 11)
QUEUE_DECLARE, QUEUE_DECLARE_OK = (50, 10), (50, 11)
QUEUE_BIND, QUEUE_BIND_OK = (50, 20), (50, 21)
BASIC_QOS, BASIC_QOS_OK = (60, 10), (60, 11)
BASIC_CONSUME, BASIC_CONSUME_OK = (60, 20), (60, 21)
BASIC_PUBLISH, BASIC_DELIVER, BASIC_ACK = (60, 40), (60, 60), (60, 80)


# ------------------------------------------------------------------------------------ codec
class W:
    def __init__(self):
        self.b = bytearray()
        self._bits: list | None = None

    def _flush_bits(self):
        if self._bits is not None:
            v = 0
            for i, bit in enumerate(self._bits):
                v |= (1 << i) if bit else 0
            self.b.append(v)
            self._bits = None

    def octet(self, v):
        self._flush_bits()
        self.b.append(v & 0xFF)
        return self

    def short(self, v):
        self._flush_bits()
        self.b += struct.pack(">H", v)
        return self

    def long(self, v):
        self._flush_bits()
        self.b += struct.pack(">I", v)
        return self

    def longlong(self, v):
        self._flush_bits()
        self.b += struct.pack(">Q", v)
        return self

    def shortstr(self, s):
        self._flush_bits()
        d = s.encode() if isinstance(s, str) else s
        self.b.append(len(d))
        self.b += d
        return self

    def longstr(self, s):
        self._flush_bits()
        d = s.encode() if isinstance(s, str) else s
        self.b += struct.pack(">I", len(d)) + d
        return self

    def bit(self, v):
        if self._bits is None or len(self._bits) == 8:
            self._flush_bits()
            self._bits = []
        self._bits.append(bool(v))
        return self

    def table(self, d: dict | None):
        self._flush_bits()
        t = W()
        for k, v in (d or {}).items():
            t.shortstr(k)
            if isinstance(v, bool):
                t.b += b"t" + bytes([1 if v else 0])
            elif isinstance(v, int):
                t.b += b"I" + struct.pack(">i", v)
            elif isinstance(v, dict):
                t.b += b"F"
                t.table(v)
            else:
                t.b += b"S"
                t.longstr(str(v))
        self.b += struct.pack(">I", len(t.b)) + t.b
        return self

    def done(self) -> bytes:
        self._flush_bits()
        return bytes(self.b)


class R:
    def __init__(self, b: bytes, pos: int = 0):
        self.b, self.p = b, pos
        self._bits = None
        self._bitn = 8

    def _reset(self):
        self._bits = None

    def octet(self):
        self._reset()
        v = self.b[self.p]
        self.p += 1
        return v

    def short(self):
        self._reset()
        v = struct.unpack_from(">H", self.b, self.p)[0]
        self.p += 2
        return v

    def long(self):
        self._reset()
        v = struct.unpack_from(">I", self.b, self.p)[0]
        self.p += 4
        return v

    def longlong(self):
        self._reset()
        v = struct.unpack_from(">Q", self.b, self.p)[0]
        self.p += 8
        return v

    def shortstr(self) -> str:
        self._reset()
        n = self.b[self.p]
        s = self.b[self.p + 1:self.p + 1 + n].decode()
        self.p += 1 + n
        return s

    def longstr(self) -> bytes:
        self._reset()
        n = struct.unpack_from(">I", self.b, self.p)[0]
        s = self.b[self.p + 4:self.p + 4 + n]
        self.p += 4 + n
        return s

    def bit(self) -> bool:
        if self._bits is None or self._bitn == 8:
            self._bits = self.b[self.p]
            self.p += 1
            self._bitn = 0
        v = bool(self._bits & (1 << self._bitn))
        self._bitn += 1
        return v

    def table(self) -> dict:
        self._reset()
        n = struct.unpack_from(">I", self.b, self.p)[0]
        end = self.p + 4 + n
        self.p += 4
        out = {}
        while self.p < end:
            k = self.shortstr()
            t = chr(self.b[self.p])
            self.p += 1
            if t == "t":
                out[k] = bool(self.b[self.p])
                self.p += 1
            elif t == "I":
                out[k] = struct.unpack_from(">i", self.b, self.p)[0]
                self.p += 4
            elif t == "S":
                out[k] = self.longstr().decode(errors="replace")
            elif t == "F":
                out[k] = self.table()
            elif t == "l":
                out[k] = struct.unpack_from(">q", self.b, self.p)[0]
                self.p += 8
            else:
                raise ValueError(f"unsupported field type {t!r}")
        return out


def frame(ftype: int, channel: int, payload: bytes) -> bytes:
    return struct.pack(">BHI", ftype, channel, len(payload)) + payload + bytes([FRAME_END])


def method_frame(channel: int, cm: tuple, args: bytes = b"") -> bytes:
    return frame(FRAME_METHOD, channel, struct.pack(">HH", *cm) + args)


def content_frames(channel: int, body: bytes, frame_max: int, content_type: str | None = None) -> bytes:
    props = W()
    flags = 0
    if content_type:
        flags |= 0x8000
        props.shortstr(content_type)
    hdr = struct.pack(">HHQH", 60, 0, len(body), flags) + props.done()
    out = frame(FRAME_HEADER, channel, hdr)
    step = max(1, frame_max - 8)
    for i in range(0, len(body), step):
        out += frame(FRAME_BODY, channel, body[i:i + step])
    return out


def read_frame(sock) -> tuple[int, int, bytes]:
    hdr = _recvn(sock, 7)
    ftype, ch, size = struct.unpack(">BHI", hdr)
    payload = _recvn(sock, size)
    if _recvn(sock, 1)[0] != FRAME_END:
        raise ConnectionError("bad AMQP frame end")
    return ftype, ch, payload


def _recvn(sock, n):
    buf = b""
    while len(buf) < n:
        c = sock.recv(n - len(buf))
        if not c:
            raise ConnectionError("connection closed")
        buf += c
    return buf


# ------------------------------------------------------------------------------------ client
class AmqpClient:
    def __init__(self, host="127.0.0.1", port=5672, username="guest", password="guest", vhost="/", timeout=10.0):
        self.host, self.port, self.username, self.password, self.vhost = host, port, username, password, vhost
        self.timeout = timeout
        self.sock = None
        self.frame_max = 131072
        self.channel = 1
        self._lock = threading.Lock()
        self._replies: queue.Queue = queue.Queue()
        self._deliveries: queue.Queue = queue.Queue()
        self._on_message = None
        self._reader = None
        self._closed = False

    def connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.sendall(PROTOCOL_HEADER)
        self.sock = s
        cm, r = self._expect_sync(CONNECTION_START)
        s.sendall(method_frame(0, CONNECTION_START_OK, W().table({"product": "sitewhere_amd", "platform": "python"})
                               .shortstr("PLAIN").longstr(f"\0{self.username}\0{self.password}").shortstr("en_US").done()))
        cm, r = self._expect_sync(CONNECTION_TUNE)
        ch_max, fmax, hb = r.short(), r.long(), r.short()
        self.frame_max = min(fmax or self.frame_max, self.frame_max)
        s.sendall(method_frame(0, CONNECTION_TUNE_OK, W().short(ch_max).long(self.frame_max).short(0).done()))
        s.sendall(method_frame(0, CONNECTION_OPEN, W().shortstr(self.vhost).shortstr("").bit(0).done()))
        self._expect_sync(CONNECTION_OPEN_OK)
        s.sendall(method_frame(self.channel, CHANNEL_OPEN, W().shortstr("").done()))
        self._expect_sync(CHANNEL_OPEN_OK)
        s.settimeout(None)
        self._reader = threading.Thread(target=self._read_loop, daemon=True, name="amqp-reader")
        self._reader.start()
        return self

    def _expect_sync(self, want):
        while True:
            ftype, ch, payload = read_frame(self.sock)
            if ftype == FRAME_HEARTBEAT:
                continue
            cm = struct.unpack_from(">HH", payload)
            if cm == CONNECTION_CLOSE:
                r = R(payload, 4)
                raise ConnectionError(f"broker closed connection: {r.short()} {r.shortstr()}")
            if cm == want:
                return cm, R(payload, 4)
            raise ConnectionError(f"unexpected AMQP method {cm}, wanted {want}")

    def _read_loop(self):
        pending = None
        try:
            while not self._closed:
                ftype, ch, payload = read_frame(self.sock)
                if ftype == FRAME_HEARTBEAT:
                    continue
                if ftype == FRAME_METHOD:
                    cm = struct.unpack_from(">HH", payload)
                    r = R(payload, 4)
                    if cm == BASIC_DELIVER:
                        tag = r.shortstr()
                        dtag = r.longlong()
                        redelivered = r.bit()
                        exch, rkey = r.shortstr(), r.shortstr()
                        pending = {"consumer_tag": tag, "delivery_tag": dtag, "redelivered": redelivered,
                                   "exchange": exch, "routing_key": rkey, "size": None, "body": b""}
                    else:
                        self._replies.put((cm, r))
                elif ftype == FRAME_HEADER and pending is not None:
                    pending["size"] = struct.unpack_from(">Q", payload, 4)[0]
                    if pending["size"] == 0:
                        self._dispatch(pending)
                        pending = None
                elif ftype == FRAME_BODY and pending is not None:
                    pending["body"] += payload
                    if len(pending["body"]) >= pending["size"]:
                        self._dispatch(pending)
                        pending = None
        except (ConnectionError, OSError):
            pass

    def _dispatch(self, d):
        if self._on_message:
            self._on_message(d)
        else:
            self._deliveries.put(d)

    def _rpc(self, cm, args: bytes, want):
        with self._lock:
            self.sock.sendall(method_frame(self.channel, cm, args))
        got, r = self._replies.get(timeout=self.timeout)
        if got != want:
            raise ConnectionError(f"unexpected AMQP reply {got}, wanted {want}")
        return r

    def queue_declare(self, name: str, durable: bool = False) -> str:
        r = self._rpc(QUEUE_DECLARE, W().short(0).shortstr(name).bit(0).bit(durable).bit(0).bit(0).bit(0)
                      .table({}).done(), QUEUE_DECLARE_OK)
        return r.shortstr()

    def queue_bind(self, queue_name: str, exchange: str, routing_key: str):
        self._rpc(QUEUE_BIND, W().short(0).shortstr(queue_name).shortstr(exchange).shortstr(routing_key).bit(0)
                  .table({}).done(), QUEUE_BIND_OK)

    def publish(self, exchange: str, routing_key: str, body: bytes, content_type: str | None = None):
        data = method_frame(self.channel, BASIC_PUBLISH, W().short(0).shortstr(exchange).shortstr(routing_key)
                            .bit(0).bit(0).done()) + content_frames(self.channel, body, self.frame_max, content_type)
        with self._lock:
            self.sock.sendall(data)

    def consume(self, queue_name: str, on_message=None, no_ack: bool = False) -> str:
        self._on_message = on_message
        r = self._rpc(BASIC_CONSUME, W().short(0).shortstr(queue_name).shortstr("").bit(0).bit(no_ack).bit(0).bit(0)
                      .table({}).done(), BASIC_CONSUME_OK)
        return r.shortstr()

    def ack(self, delivery_tag: int):
        with self._lock:
            self.sock.sendall(method_frame(self.channel, BASIC_ACK, W().longlong(delivery_tag).bit(0).done()))

    def get_delivery(self, timeout: float = 5.0):
        return self._deliveries.get(timeout=timeout)

    def close(self):
        if self.sock is None or self._closed:
            return
        try:
            with self._lock:
                self.sock.sendall(method_frame(0, CONNECTION_CLOSE, W().short(200).shortstr("bye").short(0).short(0)
                                               .done()))
        except OSError:
            pass
        self._closed = True
        try:
            self.sock.close()
        except OSError:
            pass


# ------------------------------------------------------------------------------------ broker
class AmqpBroker:
    """Minimal AMQP 0-9-1 broker: default + direct exchanges, queues, round-robin consumers, acks."""

    def __init__(self, host="127.0.0.1", port=0, frame_max=131072):
        self.host, self.port, self.frame_max = host, port, frame_max
        self.queues: dict[str, list] = defaultdict(list)           # name -> [(body, exchange, rkey)]
        self.bindings: dict[tuple, set] = defaultdict(set)         # (exchange, rkey) -> queues
        self.consumers: dict[str, list] = defaultdict(list)        # queue -> [(conn, channel, tag)]
        self._rr = defaultdict(itertools.count)
        self._lock = threading.RLock()
        self._srv = None
        self._stop = threading.Event()
        self.published = 0
        self.acked = 0

    def start(self):
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((self.host, self.port))
        self.port = s.getsockname()[1]
        s.listen(64)
        s.settimeout(0.2)
        self._srv = s
        threading.Thread(target=self._accept, daemon=True, name="amqp-broker").start()
        return self

    def stop(self):
        self._stop.set()
        if self._srv:
            self._srv.close()

    def _accept(self):
        while not self._stop.is_set():
            try:
                c, _ = self._srv.accept()
            except (socket.timeout, OSError):
                continue
            threading.Thread(target=self._serve, args=(c,), daemon=True, name="amqp-conn").start()

    def _send(self, conn, data: bytes):
        with conn[1]:
            conn[0].sendall(data)

    def _serve(self, sock):
        conn = (sock, threading.Lock())
        tags = itertools.count(1)
        dtag = itertools.count(1)
        try:
            if _recvn(sock, 8) != PROTOCOL_HEADER:
                sock.close()
                return
            self._send(conn, method_frame(0, CONNECTION_START, W().octet(0).octet(9).table({"product": "sitewhere-amqp"})
                                          .longstr("PLAIN").longstr("en_US").done()))
            pub = None
            while not self._stop.is_set():
                ftype, ch, payload = read_frame(sock)
                if ftype == FRAME_HEARTBEAT:
                    continue
                if ftype == FRAME_METHOD:
                    cm = struct.unpack_from(">HH", payload)
                    r = R(payload, 4)
                    if cm == CONNECTION_START_OK:
                        self._send(conn, method_frame(0, CONNECTION_TUNE, W().short(2047).long(self.frame_max).short(0).done()))
                    elif cm in (CONNECTION_TUNE_OK,):
                        pass
                    elif cm == CONNECTION_OPEN:
                        self._send(conn, method_frame(0, CONNECTION_OPEN_OK, W().shortstr("").done()))
                    elif cm == CHANNEL_OPEN:
                        self._send(conn, method_frame(ch, CHANNEL_OPEN_OK, W().longstr("").done()))
                    elif cm == EXCHANGE_DECLARE:
                        self._send(conn, method_frame(ch, EXCHANGE_DECLARE_OK))
                    elif cm == QUEUE_DECLARE:
                        r.short()
                        q = r.shortstr() or f"amq.gen-{next(tags)}"
                        with self._lock:
                            self.queues.setdefault(q, [])
                            n = len(self.queues[q])
                        self._send(conn, method_frame(ch, QUEUE_DECLARE_OK, W().shortstr(q).long(n).long(0).done()))
                    elif cm == QUEUE_BIND:
                        r.short()
                        q, ex, rk = r.shortstr(), r.shortstr(), r.shortstr()
                        with self._lock:
                            self.bindings[(ex, rk)].add(q)
                        self._send(conn, method_frame(ch, QUEUE_BIND_OK))
                    elif cm == BASIC_QOS:
                        self._send(conn, method_frame(ch, BASIC_QOS_OK))
                    elif cm == BASIC_CONSUME:
                        r.short()
                        q = r.shortstr()
                        tag = r.shortstr() or f"ctag-{next(tags)}"
                        self._send(conn, method_frame(ch, BASIC_CONSUME_OK, W().shortstr(tag).done()))
                        with self._lock:
                            self.consumers[q].append((conn, ch, tag, dtag))
                            backlog, self.queues[q] = self.queues[q], []
                        for m in backlog:
                            self._route_to_queue(q, *m)
                    elif cm == BASIC_PUBLISH:
                        r.short()
                        pub = {"exchange": r.shortstr(), "rkey": r.shortstr(), "size": None, "body": b""}
                    elif cm == BASIC_ACK:
                        self.acked += 1
                    elif cm == CHANNEL_CLOSE:
                        self._send(conn, method_frame(ch, CHANNEL_CLOSE_OK))
                    elif cm == CONNECTION_CLOSE:
                        self._send(conn, method_frame(0, CONNECTION_CLOSE_OK))
                        break
                elif ftype == FRAME_HEADER and pub is not None:
                    pub["size"] = struct.unpack_from(">Q", payload, 4)[0]
                    if pub["size"] == 0:
                        self._publish(pub)
                        pub = None
                elif ftype == FRAME_BODY and pub is not None:
                    pub["body"] += payload
                    if len(pub["body"]) >= pub["size"]:
                        self._publish(pub)
                        pub = None
        except (ConnectionError, OSError):
            pass
        finally:
            with self._lock:
                for q in self.consumers:
                    self.consumers[q] = [c for c in self.consumers[q] if c[0] is not conn]
            try:
                sock.close()
            except OSError:
                pass

    def _publish(self, pub):
        self.published += 1
        ex, rk = pub["exchange"], pub["rkey"]
        with self._lock:
            targets = {rk} if ex == "" else set(self.bindings.get((ex, rk), ()))
        for q in targets:
            self._route_to_queue(q, pub["body"], ex, rk)

    def _route_to_queue(self, q, body, ex, rk):
        with self._lock:
            cons = self.consumers.get(q) or []
            if not cons:
                self.queues[q].append((body, ex, rk))
                return
            conn, ch, tag, dtag = cons[next(self._rr[q]) % len(cons)]
        data = method_frame(ch, BASIC_DELIVER, W().shortstr(tag).longlong(next(dtag)).bit(0).shortstr(ex).shortstr(rk)
                            .done()) + content_frames(ch, body, self.frame_max)
        try:
            self._send(conn, data)
        except OSError:
            with self._lock:
                self.queues[q].append((body, ex, rk))


# ------------------------------------------------------------------------------------ edges
class RabbitMqReceiver(TenantEngineLifecycleComponent):
    """Consume a queue; each message body is one encoded device payload (acked after hand-off)."""

    component_type = LifecycleComponentType.InboundEventReceiver

    def __init__(self, host="127.0.0.1", port=5672, queue_name="sitewhere.input", username="guest", password="guest",
                 vhost="/", durable=False):
        super().__init__(f"rabbitmq-receiver:{queue_name}")
        self.host, self.port, self.queue_name = host, port, queue_name
        self.username, self.password, self.vhost, self.durable = username, password, vhost, durable
        self.source = None
        self.received = 0
        self.client = None

    def start(self, monitor):
        self.client = AmqpClient(self.host, self.port, self.username, self.password, self.vhost).connect()
        self.client.queue_declare(self.queue_name, self.durable)
        self.client.consume(self.queue_name, self._on)

    def _on(self, d):
        self.received += 1
        if self.source is not None:
            self.source.on_encoded_event_received(self, d["body"], {"queue": self.queue_name,
                                                                     "routingKey": d["routing_key"]})
        self.client.ack(d["delivery_tag"])

    def stop(self, monitor):
        if self.client:
            self.client.close()
