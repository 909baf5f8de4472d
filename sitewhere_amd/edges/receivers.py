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
import socket
import struct
import threading
import time
import urllib.request
from concurrent.futures import ThreadPoolExecutor

from ..core.errors import SiteWhereException
from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent
from .mqtt import MqttClient


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
    def __init__(self, host: str, port: int, topic: str = "SiteWhere/default/input/json", qos: int = 1,
                 num_threads: int = 4):
        super().__init__(f"mqtt-receiver:{topic}")
        self.host, self.port, self.topic, self.qos, self.num_threads = host, port, topic, qos, num_threads
        self.client = None
        self.pool = None

    def start(self, monitor):
        self.pool = ThreadPoolExecutor(max_workers=self.num_threads, thread_name_prefix="mqtt-proc")
        self.client = MqttClient(self.host, self.port).connect()
        self.client.on_message(lambda t, p: self.pool.submit(self.deliver, p, {"topic": t}))
        self.client.subscribe(self.topic, self.qos)

    def stop(self, monitor):
        if self.client:
            self.client.disconnect()
        if self.pool:
            self.pool.shutdown(wait=True)


class SocketReceiver(Receiver):
    """TCP server; handler ``read-all`` (payload = bytes until close), ``line`` (newline framed) or
    ``http`` (POST body; replies 200)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, handler: str = "read-all", num_threads: int = 4):
        super().__init__(f"socket-receiver:{port}")
        self.host, self.port, self.handler, self.num_threads = host, port, handler, num_threads
        self._srv = None
        self._stop = threading.Event()

    def start(self, monitor):
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
        try:
            c.settimeout(10)
            if self.handler == "line":
                buf = b""
                while True:
                    chunk = c.recv(65536)
                    if not chunk:
                        break
                    buf += chunk
                    while b"\n" in buf:
                        line, buf = buf.split(b"\n", 1)
                        if line.strip():
                            self.deliver(line, {"remote": str(addr)})
            elif self.handler == "http":
                data = b""
                while b"\r\n\r\n" not in data:
                    data += c.recv(65536)
                head, body = data.split(b"\r\n\r\n", 1)
                clen = 0
                for ln in head.split(b"\r\n"):
                    if ln.lower().startswith(b"content-length:"):
                        clen = int(ln.split(b":")[1])
                while len(body) < clen:
                    body += c.recv(65536)
                self.deliver(body, {"remote": str(addr)})
                c.sendall(b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n")
            else:
                chunks = []
                while True:
                    chunk = c.recv(65536)
                    if not chunk:
                        break
                    chunks.append(chunk)
                if chunks:
                    self.deliver(b"".join(chunks), {"remote": str(addr)})
        except OSError:
            pass
        finally:
            c.close()

    def stop(self, monitor):
        self._stop.set()
        if self._srv:
            self._srv.close()


class WebSocketReceiver(Receiver):
    """Minimal RFC 6455 server: every text or binary frame is one payload."""

    GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        super().__init__(f"websocket-receiver:{port}")
        self.host, self.port = host, port
        self._stop = threading.Event()

    def start(self, monitor):
        self._srv = socket.socket()
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._srv.bind((self.host, self.port))
        self.port = self._srv.getsockname()[1]
        self._srv.listen(16)
        self._srv.settimeout(0.2)
        threading.Thread(target=self._accept, daemon=True, name="ws-accept").start()

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
        try:
            data = b""
            while b"\r\n\r\n" not in data:
                data += c.recv(4096)
            key = [ln.split(b":", 1)[1].strip() for ln in data.split(b"\r\n") if ln.lower().startswith(b"sec-websocket-key")][0]
            acc = base64.b64encode(hashlib.sha1(key + self.GUID).digest())
            c.sendall(b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                      b"Sec-WebSocket-Accept: " + acc + b"\r\n\r\n")
            while True:
                h = _recv(c, 2)
                op, ln = h[0] & 0x0F, h[1] & 0x7F
                masked = h[1] & 0x80
                if ln == 126:
                    ln = struct.unpack("!H", _recv(c, 2))[0]
                elif ln == 127:
                    ln = struct.unpack("!Q", _recv(c, 8))[0]
                mask = _recv(c, 4) if masked else b"\0\0\0\0"
                payload = bytes(b ^ mask[i % 4] for i, b in enumerate(_recv(c, ln)))
                if op == 8:
                    break
                if op in (1, 2):
                    self.deliver(payload, {"websocket": True})
        except (OSError, IndexError, ConnectionError):
            pass
        finally:
            c.close()

    def stop(self, monitor):
        self._stop.set()
        self._srv.close()


def _recv(c, n):
    buf = b""
    while len(buf) < n:
        chunk = c.recv(n - len(buf))
        if not chunk:
            raise ConnectionError
        buf += chunk
    return buf


def ws_client_send(host: str, port: int, messages: list[bytes]):
    """Tiny masked-frame WebSocket client (tests / device simulators)."""
    s = socket.create_connection((host, port))
    key = base64.b64encode(b"sitewhere-amd-ws1")
    s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\nSec-WebSocket-Key: " + key +
              b"\r\nSec-WebSocket-Version: 13\r\n\r\n")
    resp = b""
    while b"\r\n\r\n" not in resp:
        resp += s.recv(4096)
    for m in messages:
        mask = b"\x01\x02\x03\x04"
        hdr = bytes([0x82])
        hdr += bytes([0x80 | len(m)]) if len(m) < 126 else bytes([0x80 | 126]) + struct.pack("!H", len(m))
        s.sendall(hdr + mask + bytes(b ^ mask[i % 4] for i, b in enumerate(m)))
    s.sendall(b"\x88\x80" + b"\0\0\0\0")
    time.sleep(0.05)
    s.close()


class CoapReceiver(Receiver):
    """CoAP (RFC 7252) over UDP: CON/NON POST/PUT payloads are events; CON gets a 2.04 ACK."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        super().__init__(f"coap-receiver:{port}")
        self.host, self.port = host, port
        self._stop = threading.Event()

    def start(self, monitor):
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self._sock.bind((self.host, self.port))
        self.port = self._sock.getsockname()[1]
        self._sock.settimeout(0.2)
        threading.Thread(target=self._run, daemon=True, name="coap").start()

    def _run(self):
        while not self._stop.is_set():
            try:
                data, addr = self._sock.recvfrom(65536)
            except socket.timeout:
                continue
            except OSError:
                return
            try:
                ver_t_tkl, code, mid = data[0], data[1], data[2:4]
                t, tkl = (ver_t_tkl >> 4) & 3, ver_t_tkl & 0x0F
                token = data[4:4 + tkl]
                pos, path = 4 + tkl, []
                opt = 0
                while pos < len(data) and data[pos] != 0xFF:
                    delta, ln = data[pos] >> 4, data[pos] & 0x0F
                    pos += 1
                    if delta == 13:
                        delta = data[pos] + 13
                        pos += 1
                    if ln == 13:
                        ln = data[pos] + 13
                        pos += 1
                    opt += delta
                    if opt == 11:
                        path.append(data[pos:pos + ln].decode())
                    pos += ln
                payload = data[pos + 1:] if pos < len(data) else b""
                if code in (2, 3) and payload:   # POST / PUT
                    self.deliver(payload, {"path": "/".join(path), "remote": str(addr)})
                if t == 0:  # CON -> piggybacked ACK 2.04 Changed
                    self._sock.sendto(bytes([0x60 | tkl, 0x44]) + mid + token, addr)
            except (IndexError, UnicodeDecodeError):
                continue

    def stop(self, monitor):
        self._stop.set()
        self._sock.close()


def coap_post(host: str, port: int, path: str, payload: bytes, confirmable: bool = True, timeout: float = 2.0) -> bool:
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.settimeout(timeout)
    opts = b""
    for seg in path.strip("/").split("/"):
        b = seg.encode()
        first = not opts
        delta = 11 if first else 0
        opts += bytes([(delta << 4) | len(b)]) + b
    msg = bytes([0x40 if confirmable else 0x50, 0x02, 0x12, 0x34]) + opts + b"\xff" + payload
    s.sendto(msg, (host, port))
    if not confirmable:
        s.close()
        return True
    try:
        resp, _ = s.recvfrom(1024)
        return resp[1] == 0x44
    finally:
        s.close()


class PollingRestReceiver(Receiver):
    """GET ``url`` every ``interval_s``; a non-empty body is one payload (PollingRestInboundEventReceiver)."""

    def __init__(self, url: str, interval_s: float = 10.0, headers: dict | None = None):
        super().__init__(f"rest-poll:{url}")
        self.url, self.interval, self.headers = url, interval_s, headers or {}
        self._stop = threading.Event()

    def poll_once(self):
        req = urllib.request.Request(self.url, headers=self.headers)
        with urllib.request.urlopen(req, timeout=10) as r:
            body = r.read()
        if body:
            self.deliver(body, {"url": self.url})
        return body

    def start(self, monitor):
        def run():
            while not self._stop.wait(self.interval):
                try:
                    self.poll_once()
                except Exception as e:  # noqa: BLE001
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


def build_receiver(rc: dict) -> Receiver:
    t = rc.get("type")
    if t == "mqtt":
        return MqttReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 1883)), rc.get("topic", "SiteWhere/input"),
                            int(rc.get("qos", 1)), int(rc.get("numThreads", 4)))
    if t == "socket":
        return SocketReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)), rc.get("handler", "read-all"))
    if t == "websocket":
        return WebSocketReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)))
    if t == "coap":
        return CoapReceiver(rc.get("host", "127.0.0.1"), int(rc.get("port", 0)))
    if t == "rest-poll":
        return PollingRestReceiver(rc["url"], float(rc.get("interval", 10.0)), rc.get("headers"))
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
        return event_hub_receiver(rc)
    raise ValueError(f"unknown receiver type {t!r}")
