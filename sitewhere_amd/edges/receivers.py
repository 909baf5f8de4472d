"""Inbound event receivers (protocol edges of service-event-sources).

Reference ``service-event-sources/.../sources/*``:
  * ``mqtt/MqttInboundEventReceiver.java`` -- subscription thread + ``numThreads`` processor pool
  * ``socket/*`` -- TCP server with interaction handlers (read-all, HTTP, scripted)
  * ``websocket/*`` -- WebSocket client/server receivers (string / binary)
  * ``coap/*`` -- CoAP server
  * ``rest/PollingRestInboundEventReceiver.java`` -- periodic HTTP poll
  * ``activemq/*`` -- STOMP client receiver (:mod:`.stomp`); ``rabbitmq/*`` -- AMQP 0-9-1 (:mod:`.amqp`);
    ``azure/*`` -- gated (AMQP 1.0 not implemented)
All receivers hand raw bytes to ``source.on_encoded_event_received(receiver, payload, metadata)``.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import socket
import struct
import threading
import time
import urllib.parse
import urllib.request
from collections import OrderedDict
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ..core.errors import SiteWhereException
from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from .mqtt import MQTT_OPTIONS


class Receiver(TenantEngineLifecycleComponent):
    component_type = LifecycleComponentType.InboundEventReceiver

    def __init__(self, name: str):
        super().__init__(name)
        self.source = None
        self.received = 0

    def deliver(self, payload: bytes, metadata: dict | None = None):
        self.received += 1
        if self.source is not None:
            self.source.on_encoded_event_received(self, payload, metadata or {})


class MqttReceiver(Receiver):
    """MQTT subscription receiver (reference ``mqtt/MqttInboundEventReceiver.java``): one client
    subscription, payloads handed to a pool of ``num_threads`` processors; a QoS 1/2 message is
    acknowledged once it has been handed off.  ``mqtt`` carries the ``MqttLifecycleComponent``
    attributes (protocol, username, password, trustStorePath, keyStorePath, clientId,
    cleanSession); the client reconnects and re-subscribes by itself."""

    def __init__(self, host: str, port: int, topic: str = "SiteWhere/default/input/json", qos=1,
                 num_threads: int = 4, **mqtt):
        super().__init__(f"mqtt-receiver:{topic}")
        from .mqtt import parse_qos
        self.host, self.port, self.topic, self.qos, self.num_threads = host, port, topic, parse_qos(qos), num_threads
        self.mqtt = {k: v for k, v in mqtt.items() if v is not None}
        self.client = None
        self.pool = None

    def start(self, monitor):
        from .mqtt import client_from_config
        self.pool = ThreadPoolExecutor(max_workers=self.num_threads, thread_name_prefix="mqtt-proc")
        self.client = client_from_config(dict(self.mqtt, host=self.host, port=self.port), reconnect=True)
        self.client.on_message(lambda t, p: self.pool.submit(self.deliver, p, {"topic": t}))
        self.client.connect()
        self.client.subscribe(self.topic, self.qos)

    def stop(self, monitor):
        if self.client:
            self.client.disconnect()
        if self.pool:
            self.pool.shutdown(wait=True)


class SocketStream:
    """What a scripted socket interaction handler sees as ``socket`` (reference
    ``GroovySocketInteractionHandler`` binds the raw ``java.net.Socket``): blocking reads with a
    per-connection buffer, writes, and the peer address."""

    def __init__(self, conn, addr):
        self._c, self.remote = conn, addr
        self._buf = bytearray()

    def _fill(self) -> bool:
        chunk = self._c.recv(65536)
        if not chunk:
            return False
        self._buf += chunk
        return True

    def read(self, n: int = -1) -> bytes:
        """Up to ``n`` bytes (``-1``: everything until the peer closes)."""
        while (n < 0 or len(self._buf) < n) and self._fill():
            pass
        n = len(self._buf) if n < 0 else min(n, len(self._buf))
        out = bytes(self._buf[:n])
        del self._buf[:n]
        return out

    def read_exactly(self, n: int) -> bytes:
        out = self.read(n)
        if len(out) < n:
            raise ConnectionError(f"peer closed after {len(out)} of {n} bytes")
        return out

    def readline(self) -> bytes:
        """One ``\\n``-terminated line without the terminator (``b""`` at end of stream)."""
        while b"\n" not in self._buf and self._fill():
            pass
        i = self._buf.find(b"\n")
        if i < 0:
            return self.read()
        out = bytes(self._buf[:i]).rstrip(b"\r")
        del self._buf[:i + 1]
        return out

    def write(self, data: bytes):
        self._c.sendall(data)


class SocketReceiver(Receiver):
    """TCP server with a per-connection interaction handler (reference ``socket/*``:
    ``SocketInboundEventReceiver`` + ``ReadAllInteractionHandler`` / ``HttpInteractionHandler`` /
    ``GroovySocketInteractionHandler``):

    * ``read-all`` -- the payload is every byte until the peer closes;
    * ``line`` -- newline-framed payloads on a long-lived connection;
    * ``http`` -- one HTTP/1.1 request per connection; a POST/PUT body (``Content-Length`` or
      chunked) is the payload; replies ``200 Information received by SiteWhere.``;
    * ``script`` -- ``interact(socket, receiver)`` from a user script drives the conversation and
      calls ``receiver.deliver(payload)`` per event (the Groovy handler's contract).
    Connections are served on a pool of ``num_threads`` (reference: a cached executor)."""

    HANDLERS = ("read-all", "line", "http", "script")

    def __init__(self, host: str = "127.0.0.1", port: int = 0, handler: str = "read-all", num_threads: int = 4,
                 script: str | None = None, runner=None):
        super().__init__(f"socket-receiver:{port}")
        if handler not in self.HANDLERS:
            raise ValueError(f"unknown socket interaction handler {handler!r}")
        if handler == "script" and not script:
            raise ValueError("script interaction handler needs a script")
        self.host, self.port, self.handler, self.num_threads = host, port, handler, num_threads
        self.script, self.runner = script, runner
        self._srv = None
        self._pool = None
        self._stop = threading.Event()
        self._conns: set = set()
        self._conns_lock = threading.Lock()

    def start(self, monitor):
        if self.handler == "script":
            if self.runner is None:
                from ..runtime.scripting import ScriptRunner
                self.runner = ScriptRunner()
            fn = self.runner.compile(self.script, f"{self.component_name}.interact").get("interact")
            if not callable(fn):
                raise SiteWhereException("socket interaction script must define interact(socket, receiver)")
            self._interact = fn
        self._srv = socket.socket()
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((self.host, self.port))
        self.port = self._srv.getsockname()[1]
        self._srv.listen(64)
        self._srv.settimeout(0.2)
        self._pool = ThreadPoolExecutor(max_workers=self.num_threads, thread_name_prefix="socket-recv")
        self._stop.clear()
        threading.Thread(target=self._accept, daemon=True, name="socket-accept").start()

    def _accept(self):
        while not self._stop.is_set():
            try:
                c, addr = self._srv.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            self._pool.submit(self._handle, c, addr)

    def _handle(self, c, addr):
        md = {"remote": f"{addr[0]}:{addr[1]}"}
        with self._conns_lock:
            self._conns.add(c)
        try:
            c.settimeout(30)
            st = SocketStream(c, md["remote"])
            if self.handler == "line":
                while True:
                    line = st.readline()
                    if not line and not st._buf and not st._fill():
                        break
                    if line.strip():
                        self.deliver(line, md)
            elif self.handler == "http":
                self._http(st, md)
            elif self.handler == "script":
                self._interact(st, self)
            else:
                body = st.read()
                if body:
                    self.deliver(body, md)
        except Exception as e:  # noqa: BLE001 -- one bad connection never stops the receiver
            if not self._stop.is_set():
                self.logger.warning("socket interaction with %s failed: %s", md["remote"], e)
        finally:
            with self._conns_lock:
                self._conns.discard(c)
            c.close()

    def _http(self, st: SocketStream, md: dict):
        request_line = st.readline().decode("latin-1")
        method = request_line.split(" ", 1)[0].upper()
        headers = {}
        while True:
            ln = st.readline()
            if not ln:
                break
            k, _, v = ln.decode("latin-1").partition(":")
            headers[k.strip().lower()] = v.strip()
        body = b""
        if headers.get("transfer-encoding", "").lower() == "chunked":
            while True:
                size = int(st.readline().split(b";", 1)[0] or b"0", 16)
                if size == 0:
                    while st.readline():        # trailers up to the blank line
                        pass
                    break
                body += st.read_exactly(size)
                st.readline()
        elif "content-length" in headers:
            body = st.read_exactly(int(headers["content-length"]))
        msg = b"Information received by SiteWhere."
        if method in ("POST", "PUT") and body:
            self.deliver(body, dict(md, method=method, path=request_line.split(" ")[1] if " " in request_line else "/"))
        st.write(b"HTTP/1.1 200 OK\r\nContent-Type: text/plain\r\nConnection: close\r\nContent-Length: "
                 + str(len(msg)).encode() + b"\r\n\r\n" + msg)

    def stop(self, monitor):
        self._stop.set()
        if self._srv:
            self._srv.close()
        _shutdown_all(self._conns, self._conns_lock)     # open conversations end with the receiver
        if self._pool:
            self._pool.shutdown(wait=False)


# ------------------------------------------------------------------------------ WebSocket (RFC 6455)
WS_GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"


def ws_accept_key(key: bytes) -> bytes:
    return base64.b64encode(hashlib.sha1(key.strip() + WS_GUID).digest())


def _unmask(data: bytes, mask: bytes) -> bytes:
    """XOR-unmask a frame payload word-at-a-time (numpy; a per-byte loop costs ~100 ns/byte)."""
    if not data:
        return b""
    n = len(data)
    m = np.frombuffer((mask * ((n + 3) // 4))[:n], np.uint8)
    return (np.frombuffer(data, np.uint8) ^ m).tobytes()


def ws_frame(opcode: int, payload: bytes, mask: bool) -> bytes:
    """One FIN frame; clients mask (RFC 6455 §5.3), servers do not."""
    n = len(payload)
    hdr = bytes([0x80 | opcode])
    mbit = 0x80 if mask else 0
    if n < 126:
        hdr += bytes([mbit | n])
    elif n < 65536:
        hdr += bytes([mbit | 126]) + struct.pack("!H", n)
    else:
        hdr += bytes([mbit | 127]) + struct.pack("!Q", n)
    if not mask:
        return hdr + payload
    key = os.urandom(4)
    return hdr + key + _unmask(payload, key)


class WsConnection:
    """Message-level reader over one WebSocket connection: reassembles fragmented messages,
    answers pings and closes; ``next_message()`` returns ``(opcode, payload)`` or None at close."""

    MAX_MESSAGE = 64 << 20

    def __init__(self, sock, is_client: bool, prefix: bytes = b""):
        self.sock, self.is_client = sock, is_client
        self._pre = bytearray(prefix)
        self._lock = threading.Lock()

    def _recv(self, n: int) -> bytes:
        if self._pre:
            take = bytes(self._pre[:n])
            del self._pre[:n]
            if len(take) == n:
                return take
            return take + _recv(self.sock, n - len(take))
        return _recv(self.sock, n)

    def send(self, opcode: int, payload: bytes):
        with self._lock:
            self.sock.sendall(ws_frame(opcode, payload, mask=self.is_client))

    def next_message(self):
        parts, op0 = [], None
        total = 0
        while True:
            h = self._recv(2)
            fin, op, ln = h[0] & 0x80, h[0] & 0x0F, h[1] & 0x7F
            if ln == 126:
                ln = struct.unpack("!H", self._recv(2))[0]
            elif ln == 127:
                ln = struct.unpack("!Q", self._recv(8))[0]
            mask = self._recv(4) if h[1] & 0x80 else None
            data = self._recv(ln) if ln else b""
            if mask:
                data = _unmask(data, mask)
            if op == 0x8:                                   # close: echo the status, then stop
                try:
                    self.send(0x8, data[:2])
                except OSError:
                    pass
                return None
            if op == 0x9:                                   # ping -> pong with the same payload
                self.send(0xA, data)
                continue
            if op == 0xA:
                continue
            if op in (0x1, 0x2):
                op0, parts, total = op, [data], len(data)
            elif op == 0x0 and op0 is not None:
                parts.append(data)
                total += len(data)
            else:
                raise ConnectionError(f"unexpected websocket opcode {op}")
            if total > self.MAX_MESSAGE:
                raise ConnectionError("websocket message too large")
            if fin:
                return op0, b"".join(parts)


class WebSocketReceiver(Receiver):
    """WebSocket receiver.  With ``url`` it is the reference's client receiver
    (``websocket/WebSocketEventReceiver.java``: connects to ``webSocketUrl`` with extra handshake
    ``headers``; ``String``/``BinaryWebSocketEventReceiver`` pick the payload type) and reconnects
    with backoff when the server drops it.  Without ``url`` it listens as a server (devices connect
    to it).  Every complete text/binary message is one payload; fragmented messages are reassembled."""

    GUID = WS_GUID

    def __init__(self, host: str = "127.0.0.1", port: int = 0, url: str | None = None,
                 headers: dict | None = None, payload_type: str = "binary"):
        super().__init__(f"websocket-receiver:{url or port}")
        self.host, self.port, self.url, self.headers = host, port, url, dict(headers or {})
        if payload_type not in ("binary", "string"):
            raise ValueError("payload_type is 'binary' or 'string'")
        self.payload_type = payload_type
        self._stop = threading.Event()
        self._srv = None
        self._client_sock = None
        self.connected = threading.Event()
        self._conns: set = set()
        self._conns_lock = threading.Lock()

    def start(self, monitor):
        self._stop.clear()
        if self.url:
            threading.Thread(target=self._client_loop, daemon=True, name="ws-client").start()
            return
        self._srv = socket.socket()
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((self.host, self.port))
        self.port = self._srv.getsockname()[1]
        self._srv.listen(16)
        self._srv.settimeout(0.2)
        threading.Thread(target=self._accept, daemon=True, name="ws-accept").start()

    # -- client mode (reference behaviour)
    def _client_loop(self):
        backoff = 0.1
        while not self._stop.is_set():
            try:
                conn = ws_connect(self.url, self.headers)
                self._client_sock = conn.sock
                self.connected.set()
                backoff = 0.1
                self._pump(conn)
            except (OSError, ConnectionError, ValueError) as e:
                if not self._stop.is_set():
                    self.logger.warning("websocket %s: %s (retry in %.1fs)", self.url, e, backoff)
            finally:
                self.connected.clear()
                if self._client_sock is not None:
                    try:
                        self._client_sock.close()
                    except OSError:
                        pass
                    self._client_sock = None
            if self._stop.wait(backoff):
                return
            backoff = min(backoff * 2, 5.0)

    # -- server mode
    def _accept(self):
        while not self._stop.is_set():
            try:
                c, _ = self._srv.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        with self._conns_lock:
            self._conns.add(c)
        try:
            data = b""
            while b"\r\n\r\n" not in data:
                chunk = c.recv(4096)
                if not chunk:
                    return
                data += chunk
            head, rest = data.split(b"\r\n\r\n", 1)
            keys = [ln.split(b":", 1)[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"sec-websocket-key")]
            if not keys:
                c.sendall(b"HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\n\r\n")
                return
            c.sendall(b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                      b"Sec-WebSocket-Accept: " + ws_accept_key(keys[0]) + b"\r\n\r\n")
            self._pump(WsConnection(c, is_client=False, prefix=rest))
        except (OSError, ConnectionError, ValueError):
            pass
        finally:
            with self._conns_lock:
                self._conns.discard(c)
            c.close()

    def _pump(self, conn: WsConnection):
        while not self._stop.is_set():
            msg = conn.next_message()
            if msg is None:
                return
            op, payload = msg
            if self.payload_type == "string" and op == 0x2:
                payload = payload.decode("utf-8", errors="replace").encode()
            self.deliver(payload, {"websocket": True, "text": op == 0x1})

    def stop(self, monitor):
        self._stop.set()
        if self._srv is not None:
            self._srv.close()
        _shutdown_all(self._conns, self._conns_lock)
        if self._client_sock is not None:
            try:
                self._client_sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass


def _shutdown_all(conns: set, lock):
    with lock:
        live = list(conns)
    for c in live:
        try:
            c.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass


def _recv(c, n):
    buf = b""
    while len(buf) < n:
        chunk = c.recv(n - len(buf))
        if not chunk:
            raise ConnectionError
        buf += chunk
    return buf


def ws_connect(url: str, headers: dict | None = None, timeout: float = 10.0) -> WsConnection:
    """Open a ``ws://host:port/path`` connection (client handshake, accept key verified)."""
    u = urllib.parse.urlsplit(url)
    if u.scheme != "ws":
        raise ValueError(f"unsupported websocket url {url!r} (ws:// only)")
    s = socket.create_connection((u.hostname, u.port or 80), timeout=timeout)
    key = base64.b64encode(os.urandom(16))
    extra = "".join(f"{k}: {v}\r\n" for k, v in (headers or {}).items()).encode()
    s.sendall(f"GET {u.path or '/'}{'?' + u.query if u.query else ''} HTTP/1.1\r\nHost: {u.netloc}\r\n".encode()
              + b"Upgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Key: " + key
              + b"\r\nSec-WebSocket-Version: 13\r\n" + extra + b"\r\n")
    resp = b""
    while b"\r\n\r\n" not in resp:
        chunk = s.recv(4096)
        if not chunk:
            s.close()
            raise ConnectionError("websocket handshake: connection closed")
        resp += chunk
    head, rest = resp.split(b"\r\n\r\n", 1)
    lines = head.split(b"\r\n")
    acc = [ln.split(b":", 1)[1].strip() for ln in lines[1:] if ln.lower().startswith(b"sec-websocket-accept")]
    if b" 101 " not in lines[0] + b" " or not acc or acc[0] != ws_accept_key(key):
        s.close()
        raise ConnectionError(f"websocket handshake refused: {lines[0]!r}")
    s.settimeout(None)
    return WsConnection(s, is_client=True, prefix=rest)


def ws_client_send(host: str, port: int, messages: list[bytes], text: bool = False):
    """Tiny WebSocket client (tests / device simulators): send messages, then close."""
    conn = ws_connect(f"ws://{host}:{port}/")
    for m in messages:
        conn.send(0x1 if text else 0x2, m)
    conn.send(0x8, struct.pack("!H", 1000))
    try:
        conn.sock.settimeout(2.0)
        while conn.next_message() is not None:
            pass
    except (OSError, ConnectionError):
        pass
    conn.sock.close()


# ------------------------------------------------------------------------------ CoAP (RFC 7252)
COAP_CON, COAP_NON, COAP_ACK, COAP_RST = 0, 1, 2, 3
COAP_POST, COAP_PUT = 2, 3
COAP_CREATED, COAP_CHANGED, COAP_CONTENT = 0x41, 0x44, 0x45
COAP_BAD_REQUEST, COAP_NOT_FOUND = 0x80, 0x84
OPT_URI_PATH, OPT_CONTENT_FORMAT = 11, 12

# reference CoapMessageDeliverer: devices/{token}[/measurements|alerts|locations|acks]
_COAP_OPS = {"measurements": "DeviceMeasurement", "alerts": "DeviceAlert", "locations": "DeviceLocation",
             "acks": "Acknowledge"}


def coap_parse(data: bytes) -> dict:
    """Decode one CoAP message (header, token, options with extended deltas/lengths, payload)."""
    if len(data) < 4 or data[0] >> 6 != 1:
        raise ValueError("not a CoAP v1 message")
    t, tkl = (data[0] >> 4) & 3, data[0] & 0x0F
    if tkl > 8:
        raise ValueError("bad token length")
    msg = {"type": t, "code": data[1], "mid": struct.unpack("!H", data[2:4])[0], "token": data[4:4 + tkl],
           "options": [], "payload": b""}
    pos, opt = 4 + tkl, 0
    while pos < len(data):
        if data[pos] == 0xFF:
            msg["payload"] = data[pos + 1:]
            break
        delta, ln = data[pos] >> 4, data[pos] & 0x0F
        pos += 1
        ext = []
        for v in (delta, ln):
            if v == 13:
                v = data[pos] + 13
                pos += 1
            elif v == 14:
                v = struct.unpack("!H", data[pos:pos + 2])[0] + 269
                pos += 2
            elif v == 15:
                raise ValueError("reserved option nibble")
            ext.append(v)
        opt += ext[0]
        val = data[pos:pos + ext[1]]
        if len(val) != ext[1]:
            raise ValueError("truncated option")
        msg["options"].append((opt, val))
        pos += ext[1]
    msg["path"] = [v.decode() for o, v in msg["options"] if o == OPT_URI_PATH]
    return msg


def _coap_nibble(v: int) -> tuple[int, bytes]:
    if v < 13:
        return v, b""
    if v < 269:
        return 13, bytes([v - 13])
    return 14, struct.pack("!H", v - 269)


def coap_build(t: int, code: int, mid: int, token: bytes = b"", options=(), payload: bytes = b"") -> bytes:
    out = bytearray([0x40 | (t << 4) | len(token), code]) + struct.pack("!H", mid & 0xFFFF) + token
    last = 0
    for num, val in sorted(options, key=lambda o: o[0]):
        d, dx = _coap_nibble(num - last)
        ln, lx = _coap_nibble(len(val))
        out += bytes([(d << 4) | ln]) + dx + lx + val
        last = num
    if payload:
        out += b"\xff" + payload
    return bytes(out)


class CoapReceiver(Receiver):
    """CoAP server (reference ``coap/CoapServerEventReceiver`` + ``CoapMessageDeliverer``).

    ``POST devices/{token}`` registers, ``POST devices/{token}/{measurements|alerts|locations|acks}``
    submits an event; the receiver hands the body on with ``eventType`` / ``token`` metadata for the
    ``coap-json`` decoder (reference ``CoapJsonDecoder``) and answers 2.05 Content, or 4.00 Bad
    Request for an unknown resource / operation.  CON requests get a piggybacked ACK; a retransmitted
    CON (same peer + message id within the exchange lifetime) is answered from the cache and *not*
    delivered again.  ``paths="any"`` delivers every POST/PUT body with its path instead."""

    EXCHANGE_LIFETIME_S = 247.0          # RFC 7252 §4.8.2 defaults
    DEDUP_CAP = 65536

    def __init__(self, host: str = "127.0.0.1", port: int = 0, paths: str = "reference"):
        super().__init__(f"coap-receiver:{port}")
        self.host, self.port, self.paths = host, port, paths
        self._stop = threading.Event()
        self._seen: OrderedDict = OrderedDict()
        self._mid = int.from_bytes(os.urandom(2), "big")
        self.duplicates = 0

    def start(self, monitor):
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self._sock.bind((self.host, self.port))
        self.port = self._sock.getsockname()[1]
        self._sock.settimeout(0.2)
        self._stop.clear()
        threading.Thread(target=self._run, daemon=True, name="coap").start()

    def _route(self, msg) -> tuple[int, bytes, dict | None]:
        """(response code, message, metadata to deliver with) for one request."""
        path = list(msg["path"])
        if self.paths == "any":
            if msg["code"] in (COAP_POST, COAP_PUT):
                return COAP_CHANGED, b"", {"path": "/".join(path)}
            return COAP_BAD_REQUEST, b"Operation not available.", None
        if not path or path[0] != "devices":
            return COAP_BAD_REQUEST, f"Unknown tenant resource type: {path[0] if path else ''}".encode(), None
        if len(path) < 2:
            return COAP_BAD_REQUEST, b"No device token specified.", None
        if msg["code"] != COAP_POST:
            return COAP_BAD_REQUEST, b"Operation not available for device.", None
        token = path[1]
        if len(path) == 2:
            return COAP_CONTENT, b"Device registration submitted successfully.", {"eventType": "RegisterDevice",
                                                                                 "token": token}
        et = _COAP_OPS.get(path[2])
        if et is None:
            return COAP_BAD_REQUEST, f"Unknown device operation: {path[2]}".encode(), None
        what = {"DeviceMeasurement": "measurement", "DeviceAlert": "alert", "DeviceLocation": "location",
                "Acknowledge": "ack"}[et]
        return COAP_CONTENT, f"Device {what} submitted successfully.".encode(), {"eventType": et, "token": token}

    def _next_mid(self) -> int:
        self._mid = (self._mid + 1) & 0xFFFF
        return self._mid

    def _run(self):
        while not self._stop.is_set():
            try:
                data, addr = self._sock.recvfrom(65536)
            except socket.timeout:
                continue
            except OSError:
                return
            try:
                msg = coap_parse(data)
            except (ValueError, IndexError, UnicodeDecodeError):
                continue
            if msg["type"] in (COAP_ACK, COAP_RST) or not 1 <= msg["code"] <= 31:
                continue                                   # not a request
            key = (addr, msg["mid"])
            now = time.monotonic()
            hit = self._seen.get(key)
            if hit is not None and now - hit[0] < self.EXCHANGE_LIFETIME_S:
                self.duplicates += 1
                self._sock.sendto(hit[1], addr)            # retransmission: same answer, no redelivery
                continue
            code, text, md = self._route(msg)
            if md is not None:
                md["remote"] = f"{addr[0]}:{addr[1]}"
                try:
                    self.deliver(msg["payload"], md)
                except Exception as e:  # noqa: BLE001
                    code, text = 0xA0, str(e).encode()[:200]      # 5.00 Internal Server Error
            if msg["type"] == COAP_CON:
                resp = coap_build(COAP_ACK, code, msg["mid"], msg["token"], payload=text)
            else:
                resp = coap_build(COAP_NON, code, self._next_mid(), msg["token"], payload=text)
            self._sock.sendto(resp, addr)
            self._seen[key] = (now, resp)
            while len(self._seen) > self.DEDUP_CAP or (self._seen and now - next(iter(self._seen.values()))[0]
                                                       > self.EXCHANGE_LIFETIME_S):
                self._seen.popitem(last=False)

    def stop(self, monitor):
        self._stop.set()
        self._sock.close()


def coap_request(host: str, port: int, path: str, payload: bytes = b"", code: int = COAP_POST,
                 confirmable: bool = True, timeout: float = 2.0, mid: int | None = None,
                 retries: int = 2) -> dict | None:
    """Send one CoAP request; returns the parsed response (None for NON with no answer / timeout).
    CON requests are retransmitted with the same message id on timeout (RFC 7252 §4.2)."""
    segs = [s.encode() for s in path.strip("/").split("/") if s]
    mid = int.from_bytes(os.urandom(2), "big") if mid is None else mid
    token = os.urandom(4)
    msg = coap_build(COAP_CON if confirmable else COAP_NON, code, mid, token,
                     [(OPT_URI_PATH, s) for s in segs], payload)
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.settimeout(timeout)
    try:
        for _ in range(retries + 1 if confirmable else 1):
            s.sendto(msg, (host, port))
            try:
                while True:
                    resp, _ = s.recvfrom(65536)
                    r = coap_parse(resp)
                    if r["token"] == token:
                        return r
            except socket.timeout:
                continue
        return None
    finally:
        s.close()


def coap_post(host: str, port: int, path: str, payload: bytes, confirmable: bool = True, timeout: float = 2.0) -> bool:
    """POST ``payload``; True when a CON request got a 2.xx answer (NON: sent)."""
    r = coap_request(host, port, path, payload, COAP_POST, confirmable, timeout)
    if not confirmable:
        return True
    return r is not None and (r["code"] >> 5) == 2


class RestHelper:
    """What a polling script gets as ``rest`` (reference ``rest/RestHelper.java``): ``get``/``post``
    relative to ``base_url`` with optional basic auth; JSON bodies in, bytes out."""

    def __init__(self, base_url: str, username: str | None = None, password: str | None = None, timeout: float = 10.0):
        self.base_url, self.timeout = base_url.rstrip("/"), timeout
        self._auth = None
        if username:
            self._auth = "Basic " + base64.b64encode(f"{username}:{password or ''}".encode()).decode()

    def _req(self, method: str, path: str, body=None, headers: dict | None = None) -> bytes:
        url = path if "://" in path else f"{self.base_url}/{path.lstrip('/')}"
        h = dict(headers or {})
        if self._auth:
            h["Authorization"] = self._auth
        data = None
        if body is not None:
            data = body if isinstance(body, (bytes, bytearray)) else json.dumps(body).encode()
            h.setdefault("Content-Type", "application/json")
        req = urllib.request.Request(url, data=data, headers=h, method=method)
        with urllib.request.urlopen(req, timeout=self.timeout) as r:
            return r.read()

    def get(self, path: str = "", headers: dict | None = None) -> bytes:
        return self._req("GET", path, headers=headers)

    def get_json(self, path: str = "", headers: dict | None = None):
        return json.loads(self.get(path, headers) or b"null")

    def post(self, path: str, body=None, headers: dict | None = None) -> bytes:
        return self._req("POST", path, body, headers)


class PollingRestReceiver(Receiver):
    """Periodic REST poll (reference ``rest/PollingRestInboundEventReceiver.java``).

    With a ``script`` (the reference's only mode) each poll runs ``poll(rest, payloads, logger)``:
    the script queries the remote API through :class:`RestHelper` (``baseUrl``, basic auth) and
    appends one ``bytes`` payload per event to ``payloads``.  Without a script the body of
    ``GET url`` is one payload.  A failed poll is logged and retried at the next interval."""

    def __init__(self, url: str | None = None, interval_s: float = 10.0, headers: dict | None = None,
                 script: str | None = None, runner=None, username: str | None = None, password: str | None = None):
        super().__init__(f"rest-poll:{url}")
        if not url:
            raise ValueError("rest-poll receiver needs a url / baseUrl")
        self.url, self.interval, self.headers = url, interval_s, headers or {}
        self.script, self.runner = script, runner
        self.rest = RestHelper(url, username, password)
        self.polls = self.failures = 0
        self._stop = threading.Event()

    def poll_once(self) -> list[bytes]:
        self.polls += 1
        if self.script:
            if self.runner is None:
                from ..runtime.scripting import ScriptRunner
                self.runner = ScriptRunner()
            payloads: list = []
            self.runner.call(self.script, "poll", self.rest, payloads, self.logger, name=f"{self.component_name}.poll")
        else:
            body = self.rest.get("", self.headers)
            payloads = [body] if body else []
        for p in payloads:
            self.deliver(p if isinstance(p, (bytes, bytearray)) else str(p).encode(), {"url": self.url})
        return payloads

    def start(self, monitor):
        self._stop.clear()

        def run():
            while not self._stop.wait(self.interval):
                try:
                    self.poll_once()
                except Exception as e:  # noqa: BLE001
                    self.failures += 1
                    self.logger.warning("poll failed: %s", e)
        threading.Thread(target=run, daemon=True, name="rest-poll").start()

    def stop(self, monitor):
        self._stop.set()


class KafkaReceiver(Receiver):
    """Consume payloads from a Kafka topic (one record value = one encoded device payload) in a
    consumer group, committing after hand-off (at-least-once).  Also the Azure Event Hubs receiver
    (reference ``sources/azure/EventHubInboundEventReceiver``): Event Hubs exposes the Kafka protocol
    on ``<namespace>.servicebus.windows.net:9093`` with TLS and SASL/PLAIN (user ``$ConnectionString``,
    password = the namespace connection string); the event hub is the topic."""

    def __init__(self, bootstrap: str, topic: str, group: str = "sitewhere", tls: bool = False,
                 sasl_plain: tuple[str, str] | None = None, kind: str = "kafka"):
        super().__init__(f"{kind}-receiver:{topic}")
        self.bootstrap, self.topic, self.group = bootstrap, topic, group
        self.tls, self.sasl_plain, self.kind = tls, sasl_plain, kind
        self._stop = threading.Event()
        self._t = None
        self.bus = None

    def start(self, monitor):
        from ..bus.kafka_client import KafkaEventBus
        self.bus = KafkaEventBus(self.bootstrap, client_id=f"sitewhere-{self.kind}", tls=self.tls,
                                 sasl_plain=self.sasl_plain)
        consumer = self.bus.consumer(self.group, [self.topic])
        self._stop.clear()

        def run():
            while not self._stop.is_set():
                try:
                    batch = consumer.poll(500)
                except Exception as e:  # noqa: BLE001
                    self.logger.warning("%s poll failed: %s", self.kind, e)
                    time.sleep(1.0)
                    continue
                for recs in batch.values():
                    for r in recs:
                        self.deliver(r.value, {"topic": r.topic, "partition": r.partition, "offset": r.offset,
                                               "key": r.key.decode(errors="replace") if r.key else None})
                if batch:
                    consumer.commit()
            consumer.close()
        self._t = threading.Thread(target=run, daemon=True, name=f"{self.kind}-receiver")
        self._t.start()

    def stop(self, monitor):
        self._stop.set()
        if self._t:
            self._t.join(5)
        if self.bus:
            self.bus.client.close()


def event_hub_receiver(rc: dict) -> KafkaReceiver:
    """Event Hubs over its Kafka endpoint: ``namespace`` (or ``bootstrap``), ``eventHub``,
    ``connectionString``, ``consumerGroup``."""
    ns = rc.get("namespace")
    bootstrap = rc.get("bootstrap") or f"{ns}.servicebus.windows.net:9093"
    return KafkaReceiver(bootstrap, rc["eventHub"], rc.get("consumerGroup", "$Default"), bool(rc.get("tls", True)),
                         ("$ConnectionString", rc["connectionString"]), kind="eventhub")


def build_receiver(rc: dict, scripts=None) -> Receiver:
    """Receiver from its tenant-configuration entry (``scripts``: the tenant's script runner, for
    scripted socket handlers and polling scripts)."""
    t = rc.get("type")
    if t == "mqtt":
        return MqttReceiver(rc.get("hostname") or rc.get("host", "127.0.0.1"), int(rc.get("port", 1883)),
                            rc.get("topic", "SiteWhere/input"), rc.get("qos", 1), int(rc.get("numThreads", 4)),
                            **{k: rc.get(k) for k in MQTT_OPTIONS})
    if t == "socket":
        return SocketReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)), rc.get("handler", "read-all"),
                              int(rc.get("numThreads", 4)), rc.get("script"), scripts)
    if t == "websocket":
        return WebSocketReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)),
                                 rc.get("webSocketUrl") or rc.get("url"), rc.get("headers"),
                                 rc.get("payloadType", "binary"))
    if t == "coap":
        return CoapReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)), rc.get("paths", "reference"))
    if t == "rest-poll":
        return PollingRestReceiver(rc.get("baseUrl") or rc.get("url"), float(rc.get("interval", 10.0)),
                                   rc.get("headers"), rc.get("script"), scripts, rc.get("username"),
                                   rc.get("password"))
    if t == "activemq-broker" or (t in ("activemq", "stomp") and rc.get("transportUri")):
        from .stomp import StompBrokerReceiver
        return StompBrokerReceiver(rc.get("transportUri", "stomp://127.0.0.1:61613"),
                                   rc.get("queueName", "SITEWHERE.IN"), int(rc.get("numConsumers", 3)),
                                   rc.get("brokerName"))
    if t in ("activemq", "stomp"):
        from .stomp import StompReceiver
        return StompReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 61613)),
                             rc.get("destination", "/queue/SITEWHERE.IN"), rc.get("login"), rc.get("passcode"),
                             int(rc.get("numThreads", 2)))
    if t in ("rabbitmq", "amqp"):
        from .amqp import RabbitMqReceiver
        return RabbitMqReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 5672)), rc.get("queue", "sitewhere.input"),
                                rc.get("username", "guest"), rc.get("password", "guest"), rc.get("vhost", "/"),
                                bool(rc.get("durable", False)))
    if t == "kafka":
        sasl = (rc["username"], rc["password"]) if rc.get("username") else None
        return KafkaReceiver(rc.get("bootstrap", "127.0.0.1:9092"), rc["topic"], rc.get("group", "sitewhere"),
                             bool(rc.get("tls", False)), sasl)
    if t in ("eventhub", "azure-eventhub"):
        # AMQP 1.0 (the reference's EventProcessorHost path) unless the Kafka endpoint is asked for
        if rc.get("protocol") == "kafka" or (rc.get("connectionString") and not rc.get("sasKeyName")):
            return event_hub_receiver(rc)
        from .eventhub import EventHubAmqpReceiver
        return EventHubAmqpReceiver(rc.get("namespace"), rc["eventHub"], rc["sasKeyName"], rc["sasKey"],
                                    rc.get("consumerGroup", "$Default"), rc.get("host"), int(rc.get("port", 5671)),
                                    bool(rc.get("tls", True)), rc.get("hostNamePrefix", "sitewhere"),
                                    rc.get("partitionCount"), checkpoint_every=int(rc.get("checkpointEvery", 100)))
    raise ValueError(f"unknown receiver type {t!r}")
