"""Minimal MQTT 3.1.1 broker and client (no external dependency).

The reference ingests device events over MQTT (``MqttInboundEventReceiver.java:40-309``: one
subscription thread + a processor pool, QoS configurable, ack after hand-off) and delivers commands
by MQTT publish at QoS 1 (``MqttCommandDeliveryProvider.java:87-111``), with outbound connectors
publishing too (``MqttOutboundConnector``).  The image has no paho/mosquitto, so this module
implements the protocol subset those paths need: CONNECT/CONNACK, PUBLISH (QoS 0/1) + PUBACK,
SUBSCRIBE/SUBACK (``+``/``#`` wildcards), UNSUBSCRIBE, PINGREQ/PINGRESP, DISCONNECT.
"""
from __future__ import annotations

import socket
import struct
import threading
import time
from collections import defaultdict

CONNECT, CONNACK, PUBLISH, PUBACK, SUBSCRIBE, SUBACK, UNSUBSCRIBE, UNSUBACK = 1, 2, 3, 4, 8, 9, 10, 11
PINGREQ, PINGRESP, DISCONNECT = 12, 13, 14


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


def read_packet(sock):
    h = _recv_exact(sock, 1)[0]
    mult, length = 1, 0
    while True:
        b = _recv_exact(sock, 1)[0]
        length += (b & 0x7F) * mult
        if not b & 0x80:
            break
        mult *= 128
    body = _recv_exact(sock, length) if length else b""
    return h >> 4, h & 0x0F, body


def packet(ptype: int, flags: int, body: bytes) -> bytes:
    return bytes([(ptype << 4) | flags]) + _enc_len(len(body)) + body


def topic_matches(filt: str, topic: str) -> bool:
    fp, tp = filt.split("/"), topic.split("/")
    for i, f in enumerate(fp):
        if f == "#":
            return True
        if i >= len(tp):
            return False
        if f != "+" and f != tp[i]:
            return False
    return len(fp) == len(tp)


class MqttBroker:
    """Threaded broker; one thread per client connection."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.host = host
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((host, port))
        self.port = self._srv.getsockname()[1]
        self._subs: dict = defaultdict(set)     # conn -> set(filters)
        self._conns: dict = {}
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self._t = None
        self.published = 0

    def start(self):
        self._srv.listen(64)
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

    def _send(self, c, data):
        lock = self._conns.get(c)
        if lock is None:
            return
        with lock:
            try:
                c.sendall(data)
            except OSError:
                pass

    def _serve(self, c):
        with self._lock:
            self._conns[c] = threading.Lock()
        try:
            while not self._stop.is_set():
                t, flags, body = read_packet(c)
                if t == CONNECT:
                    self._send(c, packet(CONNACK, 0, b"\x00\x00"))
                elif t == PUBLISH:
                    qos = (flags >> 1) & 3
                    tl = struct.unpack("!H", body[:2])[0]
                    topic = body[2:2 + tl].decode()
                    pos = 2 + tl
                    if qos:
                        pid = body[pos:pos + 2]
                        pos += 2
                        self._send(c, packet(PUBACK, 0, pid))
                    self.route(topic, body[pos:])
                elif t == SUBSCRIBE:
                    pid = body[:2]
                    pos, granted = 2, bytearray()
                    while pos < len(body):
                        ln = struct.unpack("!H", body[pos:pos + 2])[0]
                        filt = body[pos + 2:pos + 2 + ln].decode()
                        q = body[pos + 2 + ln]
                        pos += 3 + ln
                        with self._lock:
                            self._subs[c].add(filt)
                        granted.append(min(q, 1))
                    self._send(c, packet(SUBACK, 0, pid + bytes(granted)))
                elif t == UNSUBSCRIBE:
                    pid = body[:2]
                    pos = 2
                    while pos < len(body):
                        ln = struct.unpack("!H", body[pos:pos + 2])[0]
                        with self._lock:
                            self._subs[c].discard(body[pos + 2:pos + 2 + ln].decode())
                        pos += 2 + ln
                    self._send(c, packet(UNSUBACK, 0, pid))
                elif t == PINGREQ:
                    self._send(c, packet(PINGRESP, 0, b""))
                elif t == DISCONNECT:
                    break
        except (ConnectionError, OSError, IndexError, struct.error):
            pass
        finally:
            with self._lock:
                self._subs.pop(c, None)
                self._conns.pop(c, None)
            try:
                c.close()
            except OSError:
                pass

    def route(self, topic: str, payload: bytes):
        self.published += 1
        with self._lock:
            targets = [c for c, fs in self._subs.items() if any(topic_matches(f, topic) for f in fs)]
        pkt = packet(PUBLISH, 0, _enc_str(topic) + payload)  # deliver at QoS 0
        for c in targets:
            self._send(c, pkt)

    def stop(self):
        self._stop.set()
        try:
            self._srv.close()
        except OSError:
            pass
        with self._lock:
            for c in list(self._conns):
                try:
                    c.close()
                except OSError:
                    pass


class MqttClient:
    def __init__(self, host: str, port: int, client_id: str | None = None, keepalive: int = 60):
        self.host, self.port = host, port
        self.client_id = client_id or f"sw-{int(time.time() * 1000) % 10**9}-{id(self) % 10000}"
        self.keepalive = keepalive
        self.sock = None
        self._pid = 0
        self._acks: dict[int, threading.Event] = {}
        self._handlers: list = []
        self._lock = threading.Lock()
        self._reader = None
        self._closed = False

    def connect(self, timeout: float = 5.0):
        self.sock = socket.create_connection((self.host, self.port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        vh = _enc_str("MQTT") + bytes([4, 0x02]) + struct.pack("!H", self.keepalive)
        self.sock.sendall(packet(CONNECT, 0, vh + _enc_str(self.client_id)))
        t, _, body = read_packet(self.sock)
        if t != CONNACK or body[1] != 0:
            raise ConnectionError("MQTT connect refused")
        self.sock.settimeout(None)
        self._suback = threading.Event()
        self._reader = threading.Thread(target=self._read, daemon=True, name=f"mqtt-{self.client_id}")
        self._reader.start()
        return self

    def _next_pid(self) -> int:
        with self._lock:
            self._pid = self._pid % 65535 + 1
            return self._pid

    def _read(self):
        try:
            while not self._closed:
                t, flags, body = read_packet(self.sock)
                if t == PUBLISH:
                    tl = struct.unpack("!H", body[:2])[0]
                    topic = body[2:2 + tl].decode()
                    pos = 2 + tl + (2 if (flags >> 1) & 3 else 0)
                    for h in list(self._handlers):
                        try:
                            h(topic, body[pos:])
                        except Exception:
                            pass
                elif t in (PUBACK, SUBACK, UNSUBACK):
                    pid = struct.unpack("!H", body[:2])[0]
                    ev = self._acks.pop(pid, None)
                    if ev:
                        ev.set()
        except (ConnectionError, OSError, struct.error):
            pass

    def on_message(self, handler):
        self._handlers.append(handler)

    def _send(self, data: bytes):
        with self._lock:
            self.sock.sendall(data)

    def subscribe(self, filt: str, qos: int = 1, timeout: float = 5.0):
        pid = self._next_pid()
        ev = self._acks[pid] = threading.Event()
        self._send(packet(SUBSCRIBE, 2, struct.pack("!H", pid) + _enc_str(filt) + bytes([qos])))
        if not ev.wait(timeout):
            raise TimeoutError("SUBACK not received")

    def publish(self, topic: str, payload: bytes, qos: int = 0, timeout: float = 5.0):
        if qos:
            pid = self._next_pid()
            ev = self._acks[pid] = threading.Event()
            self._send(packet(PUBLISH, qos << 1, _enc_str(topic) + struct.pack("!H", pid) + payload))
            if not ev.wait(timeout):
                raise TimeoutError("PUBACK not received")
        else:
            self._send(packet(PUBLISH, 0, _enc_str(topic) + payload))

    def ping(self):
        self._send(packet(PINGREQ, 0, b""))

    def disconnect(self):
        self._closed = True
        try:
            self._send(packet(DISCONNECT, 0, b""))
            self.sock.close()
        except OSError:
            pass
