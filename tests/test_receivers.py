"""Device-protocol receivers of service-event-sources: TCP socket (read-all / line / HTTP / scripted
interaction handlers), WebSocket (server and the reference's client receiver), CoAP (the reference's
``devices/{token}/...`` resource tree, CON retransmission dedup) and REST polling (scripted).

Reference: ``service-event-sources/.../sources/{socket,websocket,coap,rest}/*`` and
``decoder/coap/CoapJsonDecoder.java``.  The reference only had manual harnesses for these
(``SocketTests.java``, ``websocket/*``, ``CoapTests.java``); here every receiver runs
against a client in the same process.
"""
from __future__ import annotations

import json
import socket
import struct
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from sitewhere_amd.edges.receivers import (COAP_BAD_REQUEST, COAP_CONTENT, COAP_PUT, CoapReceiver, PollingRestReceiver,
                                           SocketReceiver, WebSocketReceiver, WsConnection, build_receiver,
                                           coap_build, coap_parse, coap_request, ws_accept_key, ws_client_send,
                                           ws_connect, ws_frame)
from sitewhere_amd.services.event_sources import CoapJsonDecoder


class _Src:
    def __init__(self):
        self.got = []
        self.lock = threading.Lock()

    def on_encoded_event_received(self, recv, payload, md):
        with self.lock:
            self.got.append((bytes(payload), dict(md)))


def wait(cond, t=30.0):          # returns as soon as cond holds; the bound only catches a real failure
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.01)
    return cond()


def _started(r):
    src = _Src()
    r.source = src
    r.start(None)
    return src


# ------------------------------------------------------------------------------ socket
def test_socket_read_all_and_line_handlers():
    r = SocketReceiver(handler="read-all")
    src = _started(r)
    try:
        for i in range(3):
            with socket.create_connection(("127.0.0.1", r.port)) as s:
                s.sendall(b"x" * 70000 + bytes([i]))          # several recv() chunks
        assert wait(lambda: len(src.got) == 3)
        assert sorted(p[-1] for p, _ in src.got) == [0, 1, 2] and all(len(p) == 70001 for p, _ in src.got)
    finally:
        r.stop(None)
    r = SocketReceiver(handler="line")
    src = _started(r)
    try:
        with socket.create_connection(("127.0.0.1", r.port)) as s:
            s.sendall(b'{"a":1}\n\n{"a"')
            time.sleep(0.05)
            s.sendall(b':2}\r\n{"a":3}')                   # last line unterminated at close
        assert wait(lambda: len(src.got) == 3)
        assert [p for p, _ in src.got] == [b'{"a":1}', b'{"a":2}', b'{"a":3}']
    finally:
        r.stop(None)


def _http_post(port, body: bytes, chunked=False):
    with socket.create_connection(("127.0.0.1", port)) as s:
        if chunked:
            parts = [body[:5], body[5:]]
            wire = b"".join(b"%x\r\n%s\r\n" % (len(p), p) for p in parts if p) + b"0\r\n\r\n"
            s.sendall(b"POST /events HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + wire)
        else:
            s.sendall(b"POST /events HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
        resp = b""
        while True:
            c = s.recv(4096)
            if not c:
                break
            resp += c
    return resp


def test_socket_http_handler_content_length_and_chunked():
    r = SocketReceiver(handler="http")
    src = _started(r)
    try:
        resp = _http_post(r.port, b'{"deviceToken":"d1"}')
        assert resp.startswith(b"HTTP/1.1 200 OK") and resp.endswith(b"Information received by SiteWhere.")
        _http_post(r.port, b"0123456789abcdef", chunked=True)
        with socket.create_connection(("127.0.0.1", r.port)) as s:   # GET: answered, nothing delivered
            s.sendall(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
            assert s.recv(4096).startswith(b"HTTP/1.1 200")
        assert wait(lambda: len(src.got) == 2)
        assert sorted(p for p, _ in src.got) == [b"0123456789abcdef", b'{"deviceToken":"d1"}']
        assert all(md["method"] == "POST" and md["path"] == "/events" for _, md in src.got)
    finally:
        r.stop(None)


def test_socket_script_interaction_handler():
    """GroovySocketInteractionHandler: the script owns the conversation (here a 2-byte length
    prefix framing + a per-message ack) and delivers payloads through the receiver."""
    script = (
        "def interact(socket, receiver):\n"
        "    while True:\n"
        "        hdr = socket.read(2)\n"
        "        if len(hdr) < 2:\n"
        "            return\n"
        "        n = hdr[0] * 256 + hdr[1]\n"
        "        receiver.deliver(socket.read_exactly(n), {'framing': 'len16'})\n"
        "        socket.write(b'K')\n")
    r = build_receiver({"type": "socket", "handler": "script", "script": script})
    src = _started(r)
    try:
        with socket.create_connection(("127.0.0.1", r.port)) as s:
            for m in (b"alpha", b"b" * 1000, b"gamma"):
                s.sendall(struct.pack("!H", len(m)) + m)
                assert s.recv(1) == b"K"
        assert wait(lambda: len(src.got) == 3)
        assert [p for p, _ in src.got] == [b"alpha", b"b" * 1000, b"gamma"]
        assert src.got[0][1]["framing"] == "len16"
    finally:
        r.stop(None)
    with pytest.raises(ValueError):
        SocketReceiver(handler="script")


# ------------------------------------------------------------------------------ websocket
def test_websocket_server_fragments_ping_and_large_frames():
    r = WebSocketReceiver()
    src = _started(r)
    try:
        ws_client_send("127.0.0.1", r.port, [b"small", b"L" * 70000], text=False)
        assert wait(lambda: len(src.got) == 2)
        conn = ws_connect(f"ws://127.0.0.1:{r.port}/")
        # a fragmented text message with a ping in the middle (RFC 6455 §5.4 allows control frames there)
        frag = lambda fin, op, p: bytes([(0x80 if fin else 0) | op]) + ws_frame(op, p, mask=True)[1:]  # noqa: E731
        conn.sock.sendall(frag(False, 0x1, b"hel") + ws_frame(0x9, b"pp", mask=True) + frag(False, 0x0, b"lo ")
                          + frag(True, 0x0, b"world"))
        conn.sock.settimeout(2.0)
        h = conn.sock.recv(2)
        assert h[0] == 0x8A and h[1] == 2 and conn.sock.recv(2) == b"pp"       # pong, unmasked
        assert wait(lambda: len(src.got) == 3)
        conn.send(0x8, struct.pack("!H", 1000))
        assert conn.next_message() is None                                   # server echoes the close
        conn.sock.close()
        assert src.got[2] == (b"hello world", {"websocket": True, "text": True})
        assert src.got[1][0] == b"L" * 70000 and src.got[1][1]["text"] is False
    finally:
        r.stop(None)


class _WsPushServer:
    """A remote WebSocket server that pushes messages to whoever connects (what the reference's
    client receiver connects to), dropping the first connection after one message."""

    def __init__(self, messages):
        self.messages, self.headers_seen, self.connections = messages, [], 0
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(4)
        self.port = self.srv.getsockname()[1]
        threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        while True:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            self.connections += 1
            data = b""
            while b"\r\n\r\n" not in data:
                data += c.recv(4096)
            lines = data.split(b"\r\n")
            self.headers_seen.append(lines)
            key = [ln.split(b":", 1)[1] for ln in lines if ln.lower().startswith(b"sec-websocket-key")][0]
            c.sendall(b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                      b"Sec-WebSocket-Accept: " + ws_accept_key(key) + b"\r\n\r\n")
            if self.connections == 1:
                c.sendall(ws_frame(0x2, self.messages[0], mask=False))
                time.sleep(0.05)
                c.close()                                   # drop: the receiver must reconnect
                continue
            for m in self.messages[1:]:
                c.sendall(ws_frame(0x2, m, mask=False))
            conn = WsConnection(c, is_client=False)
            try:
                conn.next_message()                         # until the receiver closes
            except (OSError, ConnectionError):
                pass
            c.close()


def test_websocket_client_receiver_connects_with_headers_and_reconnects():
    srv = _WsPushServer([b"m0", b"m1", "ü".encode()])
    r = build_receiver({"type": "websocket", "webSocketUrl": f"ws://127.0.0.1:{srv.port}/events",
                        "headers": {"X-SiteWhere-Tenant": "t1"}, "payloadType": "string"})
    src = _started(r)
    try:
        assert wait(lambda: len(src.got) == 3, 10)
        assert [p for p, _ in src.got] == [b"m0", b"m1", "ü".encode()]
        assert srv.connections == 2
        first = srv.headers_seen[0]
        assert first[0] == b"GET /events HTTP/1.1" and b"X-SiteWhere-Tenant: t1" in first
    finally:
        r.stop(None)
        srv.srv.close()


# ------------------------------------------------------------------------------ CoAP
def test_coap_codec_extended_options_roundtrip():
    long_seg = b"t" * 300                                       # 2-byte extended length (nibble 14)
    msg = coap_build(0, 2, 0xBEEF, b"\x01\x02", [(11, b"devices"), (11, b"x" * 20), (11, long_seg), (12, b"\x32")],
                     b"{}")
    p = coap_parse(msg)
    assert (p["type"], p["code"], p["mid"], p["token"]) == (0, 2, 0xBEEF, b"\x01\x02")
    assert p["path"] == ["devices", "x" * 20, long_seg.decode()] and p["payload"] == b"{}"
    assert (12, b"\x32") in p["options"]
    with pytest.raises(ValueError):
        coap_parse(b"\x00\x00")


def test_coap_reference_resource_tree_and_retransmission_dedup():
    r = CoapReceiver()
    src = _started(r)
    try:
        body = json.dumps({"name": "temp", "value": 21.5}).encode()
        resp = coap_request("127.0.0.1", r.port, "devices/dev-1/measurements", body)
        assert resp["code"] == COAP_CONTENT and resp["type"] == 2 and resp["payload"] == \
            b"Device measurement submitted successfully."
        resp = coap_request("127.0.0.1", r.port, "devices/dev-2", json.dumps({"deviceTypeToken": "dt"}).encode())
        assert resp["code"] == COAP_CONTENT
        for bad in ("things/dev-1", "devices", "devices/dev-1/bogus"):
            assert coap_request("127.0.0.1", r.port, bad, b"{}")["code"] == COAP_BAD_REQUEST
        assert coap_request("127.0.0.1", r.port, "devices/dev-1", b"{}", code=COAP_PUT)["code"] == COAP_BAD_REQUEST
        # a CON retransmission (same message id) is answered again but delivered once
        # (RFC 7252 §4.5: same endpoint + message id)
        msg = coap_build(0, 2, 77, b"tk", [(11, b"devices"), (11, b"dev-3"), (11, b"alerts")],
                         b'{"type":"x","message":"m"}')
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.settimeout(2.0)
            for _ in range(3):
                s.sendto(msg, ("127.0.0.1", r.port))
                resp = coap_parse(s.recvfrom(4096)[0])
                assert (resp["code"], resp["mid"], resp["token"]) == (COAP_CONTENT, 77, b"tk")
        # NON request: a NON response
        resp = coap_request("127.0.0.1", r.port, "devices/dev-4/locations", b'{"latitude":1,"longitude":2}',
                            confirmable=False)
        assert resp is not None and resp["type"] == 1 and resp["code"] == COAP_CONTENT
        assert wait(lambda: len(src.got) == 4)
        assert r.duplicates == 2
        mds = [(md["eventType"], md["token"]) for _, md in src.got]
        assert mds == [("DeviceMeasurement", "dev-1"), ("RegisterDevice", "dev-2"), ("DeviceAlert", "dev-3"),
                       ("DeviceLocation", "dev-4")]
        dec = CoapJsonDecoder()
        reqs = [dec.decode(p, md)[0] for p, md in src.got]
        assert reqs[0] == {"deviceToken": "dev-1", "type": "DeviceMeasurement",
                           "request": {"name": "temp", "value": 21.5}, "originator": None}
        assert reqs[1]["request"] == {"deviceTypeToken": "dt"}
    finally:
        r.stop(None)


# ------------------------------------------------------------------------------ REST polling
class _Api(BaseHTTPRequestHandler):
    page = 0

    def do_GET(self):  # noqa: N802
        if self.headers.get("Authorization") != "Basic dXNlcjpwdw==":
            self.send_response(401)
            self.end_headers()
            return
        _Api.page += 1
        body = json.dumps({"readings": [{"id": f"s{_Api.page}", "v": _Api.page},
                                        {"id": f"s{_Api.page}b", "v": -_Api.page}]}).encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def log_message(self, *a):
        pass


def test_polling_rest_receiver_runs_the_script_against_the_api():
    httpd = ThreadingHTTPServer(("127.0.0.1", 0), _Api)
    threading.Thread(target=httpd.serve_forever, daemon=True).start()
    script = ("import json\n"
              "def poll(rest, payloads, logger):\n"
              "    doc = rest.get_json('readings')\n"
              "    for r in doc['readings']:\n"
              "        payloads.append(json.dumps({'deviceToken': r['id'], 'type': 'DeviceMeasurement',\n"
              "                                    'request': {'name': 'v', 'value': r['v']}}).encode())\n")
    r = build_receiver({"type": "rest-poll", "baseUrl": f"http://127.0.0.1:{httpd.server_port}/api",
                        "username": "user", "password": "pw", "interval": 0.05, "script": script})
    src = _started(r)
    try:
        assert wait(lambda: len(src.got) >= 4)
        docs = [json.loads(p) for p, _ in src.got[:4]]
        assert [d["deviceToken"] for d in docs] == ["s1", "s1b", "s2", "s2b"]
        assert docs[3]["request"]["value"] == -2
    finally:
        r.stop(None)
    bad = PollingRestReceiver(f"http://127.0.0.1:{httpd.server_port}/api", 0.05)     # no auth: 401
    bad.source = _Src()
    with pytest.raises(Exception):
        bad.poll_once()
    httpd.shutdown()


# ------------------------------------------------------------------------------ whole tenant
def test_tenant_receivers_after_hot_reconfiguration():
    """A tenant's event-sources configuration is updated live: the engine restarts
    with a CoAP source (coap-json decoder), a WebSocket source and an HTTP socket source, and events
    sent over each protocol are stored."""
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.runtime.config import dump_document
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        es_ms = sw["event-sources"]
        before = es_ms.get_tenant_engine("default")
        doc = json.loads(json.dumps(es_ms.tenant_configuration("default")))
        doc["sources"] += [
            {"id": "coap", "decoder": "coap-json", "receivers": [{"type": "coap"}]},
            {"id": "ws", "decoder": "json", "receivers": [{"type": "websocket"}]},
            {"id": "http", "decoder": "json-batch", "receivers": [{"type": "socket", "handler": "http"}]}]
        sw.instance.coord.put(es_ms.tenant_config_path("default"), dump_document(doc))
        assert wait(lambda: (e := es_ms.get_tenant_engine("default")) is not None and e is not before
                    and e.status.value == "Started" and "coap" in e.manager.sources, 30)
        eng = es_ms.get_tenant_engine("default")
        port = lambda sid: eng.manager.sources[sid].receivers[1].port  # noqa: E731
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        tok = run(lambda: dm.list_devices({"pageSize": 1})).results[0].token
        aid = run(lambda: dm.get_device_by_token(tok)).device_assignment_id
        assert coap_request("127.0.0.1", port("coap"), f"devices/{tok}/measurements",
                            json.dumps({"name": "edge.coap", "value": 1.0}).encode())["code"] == COAP_CONTENT
        ws_client_send("127.0.0.1", port("ws"), [json.dumps({
            "deviceToken": tok, "type": "DeviceMeasurement", "request": {"name": "edge.ws", "value": 2.0}}).encode()],
            text=True)
        assert _http_post(port("http"), json.dumps({"deviceToken": tok, "measurements": [
            {"name": "edge.http", "value": 3.0}]}).encode()).startswith(b"HTTP/1.1 200")
        end, got = time.time() + 30, []
        while len(got) < 3 and time.time() < end:
            got = sorted((e.name, e.value) for e in run(
                lambda: em.list_measurements_for_index("Assignment", [aid], {"pageSize": 1000})).results
                if e.name.startswith("edge."))
            time.sleep(0.1)
        assert got == [("edge.coap", 1.0), ("edge.http", 3.0), ("edge.ws", 2.0)]
    finally:
        sw.stop()


def test_composite_decoder_with_scripted_metadata_extractor():
    """Reference BinaryCompositeDeviceEventDecoder + GroovyMessageMetadataExtractor: a script pulls
    the device token out of a binary frame, the device's type picks the inner decoder, and a device
    type with no choice decodes to nothing."""
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.runtime.config import dump_document
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        run = lambda f: sw.instance.system_user.run(f, "default")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "default"), sw.api("DeviceEventManagement", "default")
        tab = run(lambda: dm.get_device_by_token("galaxytab-001"))
        hab = run(lambda: dm.get_device_by_token("openhab-001"))
        tab_type = run(lambda: dm.get_device_type(tab.device_type_id)).token
        extractor = ("def extract(payload, metadata):\n"
                     "    n = payload[0]\n"
                     "    return payload[1:1 + n].decode(), payload[1 + n:]\n")
        inner = ("import json\n"
                 "def decode(payload, metadata):\n"
                 "    v = json.loads(payload)\n"
                 "    return [{'deviceToken': metadata['deviceToken'], 'type': 'DeviceMeasurement',\n"
                 "             'request': {'name': 'composite.' + metadata['deviceTypeToken'], 'value': v}}]\n")
        es_ms = sw["event-sources"]
        before = es_ms.get_tenant_engine("default")
        doc = json.loads(json.dumps(es_ms.tenant_configuration("default")))
        doc["sources"].append({"id": "binary", "receivers": [], "decoder": {
            "type": "composite", "extractorScript": extractor,
            "choices": {tab_type: {"type": "script", "script": inner}}}})
        sw.instance.coord.put(es_ms.tenant_config_path("default"), dump_document(doc))
        assert wait(lambda: (e := es_ms.get_tenant_engine("default")) is not None and e is not before
                    and e.status.value == "Started" and "binary" in e.manager.sources, 30)
        es = es_ms.get_tenant_engine("default")
        frame = lambda tok, body: bytes([len(tok)]) + tok.encode() + body  # noqa: E731
        assert es.inject("binary", frame("galaxytab-001", b"42.5")) == 1
        assert es.inject("binary", frame("openhab-001", b"1.0")) == 0          # no choice for its type
        end, got = time.time() + 20, []
        while not got and time.time() < end:
            got = [m for m in run(lambda: em.list_measurements_for_index(
                "Assignment", [tab.device_assignment_id], {"pageSize": 0})).results if m.name.startswith("composite.")]
            time.sleep(0.05)
        assert [(m.name, m.value) for m in got] == [(f"composite.{tab_type}", 42.5)]
        assert not [m for m in run(lambda: em.list_measurements_for_index(
            "Assignment", [hab.device_assignment_id], {"pageSize": 0})).results if m.name.startswith("composite.")]
    finally:
        sw.stop()
