"""STOMP 1.2 client, embedded broker and receiver (the ActiveMQ edge).

Reference: ``service-event-sources/.../sources/activemq/ActiveMqClientEventReceiver.java`` (consume
a JMS queue on a remote broker), ``ActiveMqBrokerEventReceiver`` (embedded ``BrokerService``), the
STOMP tenant template and ``StompTest.java``.  ActiveMQ speaks STOMP natively; JMS client libraries
are not available here, so the STOMP wire protocol is implemented directly:
``COMMAND\\nheader:value\\n...\\n\\nbody\\0`` frames with ``content-length`` for binary bodies,
CONNECT/CONNECTED, SUBSCRIBE (ack auto | client-individual), SEND, MESSAGE, ACK, RECEIPT,
DISCONNECT.  :class:`StompBroker` routes ``/queue/*`` round-robin to subscribers and ``/topic/*``
to all subscribers.
"""
from __future__ import annotations

import itertools
import queue
import socket
import threading
from collections import defaultdict

from ..core.lifecycle import LifecycleComponentType, TenantEngineLifecycleComponent

_ESC = {"\\": "\\\\", "\n": "\\n", "\r": "\\r", ":": "\\c"}
_UNESC = {"\\\\": "\\", "\\n": "\n", "\\r": "\r", "\\c": ":"}


def _esc(s: str) -> str:
    return "".join(_ESC.get(c, c) for c in s)


def _unesc(s: str) -> str:
    out, i = [], 0
    while i < len(s):
        if s[i] == "\\" and i + 1 < len(s):
            out.append(_UNESC.get(s[i:i + 2], s[i + 1]))
            i += 2
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def encode_frame(command: str, headers: dict | None = None, body: bytes = b"") -> bytes:
    h = dict(headers or {})
    if body:
        h["content-length"] = str(len(body))
    head = command + "\n" + "".join(f"{_esc(str(k))}:{_esc(str(v))}\n" for k, v in h.items()) + "\n"
    return head.encode() + body + b"\0"


class FrameReader:
    def __init__(self, sock):
        self.sock = sock
        self.buf = b""

    def _fill(self):
        c = self.sock.recv(65536)
        if not c:
            raise ConnectionError("connection closed")
        self.buf += c

    def read(self) -> tuple[str, dict, bytes]:
        while True:
            while self.buf.startswith(b"\n") or self.buf.startswith(b"\r\n"):   # heart-beats
                self.buf = self.buf[1:] if self.buf.startswith(b"\n") else self.buf[2:]
            i = self.buf.find(b"\n\n")
            if i < 0:
                self._fill()
                continue
            lines = self.buf[:i].decode().replace("\r", "").split("\n")
            cmd, headers = lines[0], {}
            for ln in lines[1:]:
                k, _, v = ln.partition(":")
                headers.setdefault(_unesc(k), _unesc(v))
            start = i + 2
            if "content-length" in headers:
                n = int(headers["content-length"])
                while len(self.buf) < start + n + 1:
                    self._fill()
                body = self.buf[start:start + n]
                self.buf = self.buf[start + n + 1:]
            else:
                j = self.buf.find(b"\0", start)
                while j < 0:
                    self._fill()
                    j = self.buf.find(b"\0", start)
                body = self.buf[start:j]
                self.buf = self.buf[j + 1:]
            return cmd, headers, body


# ------------------------------------------------------------------------------------ client
class StompClient:
    def __init__(self, host="127.0.0.1", port=61613, login=None, passcode=None, vhost="/", timeout=10.0):
        self.host, self.port, self.login, self.passcode, self.vhost, self.timeout = host, port, login, passcode, vhost, timeout
        self.sock = None
        self._lock = threading.Lock()
        self._subs: dict[str, callable] = {}
        self._ids = itertools.count(1)
        self._receipts: dict[str, threading.Event] = {}
        self._closed = False

    def connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        self.sock = s
        h = {"accept-version": "1.2", "host": self.vhost, "heart-beat": "0,0"}
        if self.login:
            h.update(login=self.login, passcode=self.passcode or "")
        s.sendall(encode_frame("CONNECT", h))
        self.reader = FrameReader(s)
        cmd, hdr, body = self.reader.read()
        if cmd != "CONNECTED":
            raise ConnectionError(f"STOMP connect failed: {cmd} {hdr.get('message', '')}")
        s.settimeout(None)
        threading.Thread(target=self._loop, daemon=True, name="stomp-reader").start()
        return self

    def _send(self, data: bytes):
        with self._lock:
            self.sock.sendall(data)

    def _loop(self):
        try:
            while not self._closed:
                cmd, hdr, body = self.reader.read()
                if cmd == "MESSAGE":
                    cb = self._subs.get(hdr.get("subscription"))
                    if cb:
                        cb(hdr, body)
                elif cmd == "RECEIPT":
                    ev = self._receipts.pop(hdr.get("receipt-id"), None)
                    if ev:
                        ev.set()
        except (ConnectionError, OSError):
            pass

    def send(self, destination: str, body: bytes, headers: dict | None = None, receipt: bool = False):
        h = {"destination": destination, **(headers or {})}
        ev = None
        if receipt:
            rid = f"r{next(self._ids)}"
            ev = self._receipts[rid] = threading.Event()
            h["receipt"] = rid
        self._send(encode_frame("SEND", h, body))
        if ev is not None and not ev.wait(self.timeout):
            raise TimeoutError("no STOMP receipt")

    def subscribe(self, destination: str, callback, ack: str = "auto") -> str:
        sid = f"s{next(self._ids)}"
        self._subs[sid] = callback
        rid = f"r{next(self._ids)}"
        ev = self._receipts[rid] = threading.Event()
        self._send(encode_frame("SUBSCRIBE", {"destination": destination, "id": sid, "ack": ack, "receipt": rid}))
        ev.wait(self.timeout)
        return sid

    def ack(self, ack_id: str):
        self._send(encode_frame("ACK", {"id": ack_id}))

    def close(self):
        if self.sock and not self._closed:
            try:
                self._send(encode_frame("DISCONNECT"))
            except OSError:
                pass
            self._closed = True
            self.sock.close()


# ------------------------------------------------------------------------------------ broker
class StompBroker:
    def __init__(self, host="127.0.0.1", port=0):
        self.host, self.port = host, port
        self.subs: dict[str, list] = defaultdict(list)     # destination -> [(conn, sub_id, ack_mode)]
        self.pending: dict[str, list] = defaultdict(list)  # queue backlog without subscribers
        self._rr = defaultdict(itertools.count)
        self._mid = itertools.count(1)
        self._lock = threading.RLock()
        self._stop = threading.Event()
        self.sent = 0

    def start(self):
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        s.bind((self.host, self.port))
        self.port = s.getsockname()[1]
        s.listen(64)
        s.settimeout(0.2)
        self._srv = s
        threading.Thread(target=self._accept, daemon=True, name="stomp-broker").start()
        return self

    def stop(self):
        self._stop.set()
        self._srv.close()

    def _accept(self):
        while not self._stop.is_set():
            try:
                c, _ = self._srv.accept()
            except (socket.timeout, OSError):
                continue
            threading.Thread(target=self._serve, args=(c,), daemon=True, name="stomp-conn").start()

    def _serve(self, sock):
        conn = (sock, threading.Lock())
        rd = FrameReader(sock)

        def send(data):
            with conn[1]:
                sock.sendall(data)
        try:
            while not self._stop.is_set():
                cmd, hdr, body = rd.read()
                if cmd in ("CONNECT", "STOMP"):
                    send(encode_frame("CONNECTED", {"version": "1.2", "heart-beat": "0,0", "server": "sitewhere-stomp"}))
                elif cmd == "SUBSCRIBE":
                    dest = hdr["destination"]
                    with self._lock:
                        self.subs[dest].append((conn, hdr["id"], hdr.get("ack", "auto")))
                        backlog, self.pending[dest] = self.pending[dest], []
                    if "receipt" in hdr:
                        send(encode_frame("RECEIPT", {"receipt-id": hdr["receipt"]}))
                    for b, h in backlog:
                        self._route(dest, b, h)
                elif cmd == "SEND":
                    self.sent += 1
                    self._route(hdr["destination"], body, {k: v for k, v in hdr.items()
                                                          if k not in ("destination", "content-length", "receipt")})
                    if "receipt" in hdr:
                        send(encode_frame("RECEIPT", {"receipt-id": hdr["receipt"]}))
                elif cmd == "UNSUBSCRIBE":
                    with self._lock:
                        for d in self.subs:
                            self.subs[d] = [x for x in self.subs[d] if not (x[0] is conn and x[1] == hdr.get("id"))]
                elif cmd == "DISCONNECT":
                    if "receipt" in hdr:
                        send(encode_frame("RECEIPT", {"receipt-id": hdr["receipt"]}))
                    break
        except (ConnectionError, OSError):
            pass
        finally:
            with self._lock:
                for d in self.subs:
                    self.subs[d] = [x for x in self.subs[d] if x[0] is not conn]
            sock.close()

    def _route(self, dest, body, headers):
        with self._lock:
            subs = list(self.subs.get(dest, ()))
            if not subs:
                if not dest.startswith("/topic/"):
                    self.pending[dest].append((body, headers))
                return
            targets = subs if dest.startswith("/topic/") else [subs[next(self._rr[dest]) % len(subs)]]
        for conn, sid, ack in targets:
            mid = f"m{next(self._mid)}"
            h = {"destination": dest, "message-id": mid, "subscription": sid, **headers}
            if ack != "auto":
                h["ack"] = mid
            try:
                with conn[1]:
                    conn[0].sendall(encode_frame("MESSAGE", h, body))
            except OSError:
                pass


# ------------------------------------------------------------------------------------ receiver
class StompReceiver(TenantEngineLifecycleComponent):
    """ActiveMQ/STOMP client receiver: each message body is one encoded device payload."""

    component_type = LifecycleComponentType.InboundEventReceiver

    def __init__(self, host="127.0.0.1", port=61613, destination="/queue/SITEWHERE.IN", login=None, passcode=None,
                 num_threads: int = 2):
        super().__init__(f"stomp-receiver:{destination}")
        self.host, self.port, self.destination, self.login, self.passcode = host, port, destination, login, passcode
        self.source = None
        self.received = 0
        self.client = None
        self._q: queue.Queue = queue.Queue()
        self.num_threads = num_threads
        self._workers = []
        self._stop = threading.Event()

    def start(self, monitor):
        self._stop.clear()
        self._workers = [threading.Thread(target=self._work, daemon=True, name="stomp-proc")
                         for _ in range(self.num_threads)]
        for w in self._workers:
            w.start()
        self.client = StompClient(self.host, self.port, self.login, self.passcode).connect()
        self.client.subscribe(self.destination, lambda h, b: self._q.put((h, b)), ack="client-individual")

    def _work(self):
        while not self._stop.is_set():
            try:
                h, b = self._q.get(timeout=0.2)
            except queue.Empty:
                continue
            self.received += 1
            if self.source is not None:
                self.source.on_encoded_event_received(self, b, {"destination": h.get("destination")})
            if "ack" in h:
                self.client.ack(h["ack"])

    def stop(self, monitor):
        self._stop.set()
        if self.client:
            self.client.close()


def parse_transport_uri(uri: str, default_port: int = 61613) -> tuple[str, int]:
    """``stomp://host:port?opts`` (or ``tcp://``) -> (host, port); query options are ignored."""
    rest = uri.split("://", 1)[-1].split("?", 1)[0].rstrip("/")
    host, _, port = rest.rpartition(":")
    if not host:
        return rest or "127.0.0.1", default_port
    return host, int(port)


class StompBrokerReceiver(StompReceiver):
    """Embedded-broker receiver (reference ``ActiveMQBrokerEventReceiver.java:60-120``, selected by
    ``transportUri`` in ``EventSourcesParser.java:481-491``): the receiver itself hosts the message
    broker on ``transportUri`` so devices connect straight to the event source, then consumes the
    configured queue with ``numConsumers`` workers."""

    def __init__(self, transport_uri: str = "stomp://127.0.0.1:61613", queue_name: str = "SITEWHERE.IN",
                 num_consumers: int = 3, broker_name: str | None = None):
        host, port = parse_transport_uri(transport_uri)
        dest = queue_name if queue_name.startswith("/") else f"/queue/{queue_name}"
        super().__init__("127.0.0.1" if host in ("0.0.0.0", "") else host, port, dest, num_threads=num_consumers)
        self.bind_host, self.transport_uri, self.broker_name = host, transport_uri, broker_name
        self.broker = None

    def start(self, monitor):
        self.broker = StompBroker(self.bind_host, self.port).start()
        self.port = self.broker.port                  # port 0: the broker picked one
        super().start(monitor)

    def stop(self, monitor):
        super().stop(monitor)
        if self.broker is not None:
            self.broker.stop()
