"""MQTT 3.1.1: the client behind the MQTT receiver / outbound connector / command provider
(reference ``MqttLifecycleComponent``, ``MqttInboundEventReceiver``, ``MqttCommandDeliveryProvider``)
and the in-process broker, over real sockets.

The reference only had ``MqttTests.java`` (a manual load harness against a LAN broker).
"""
from __future__ import annotations

import shutil
import socket
import ssl
import struct
import subprocess
import threading
import time

import pytest

from sitewhere_amd.edges.mqtt import (CONNECT, PUBLISH, MqttBroker, MqttClient, client_from_config, packet,
                                      parse_qos, publish_packet, read_packet, topic_matches, _enc_str)
from sitewhere_amd.edges.receivers import build_receiver


def wait(cond, t=30.0):          # returns as soon as cond holds; the bound only catches a real failure
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.01)
    return cond()


class _Inbox:
    def __init__(self, client):
        self.got = []
        client.on_message(lambda t, p: self.got.append((t, bytes(p))))


@pytest.fixture
def broker():
    b = MqttBroker().start()
    yield b
    b.stop()


def test_topic_filters_and_qos_names():
    assert topic_matches("a/+/c", "a/b/c") and not topic_matches("a/+/c", "a/b/d")
    assert topic_matches("a/#", "a") and topic_matches("a/#", "a/b/c")      # "#" also matches the parent level
    assert topic_matches("#", "x/y") and not topic_matches("#", "$SYS/x") and not topic_matches("+/x", "$SYS/x")
    assert [parse_qos(q) for q in ("AT_MOST_ONCE", "AT_LEAST_ONCE", "EXACTLY_ONCE", 2)] == [0, 1, 2, 2]
    with pytest.raises(ValueError):
        parse_qos(3)


def test_qos_0_1_2_round_trips_and_granted_qos(broker):
    sub = MqttClient("127.0.0.1", broker.port).connect()
    inbox = _Inbox(sub)
    assert sub.subscribe("dev/+/m", 2) == 2
    assert sub.subscribe("low/#", 0) == 0
    pub = MqttClient("127.0.0.1", broker.port).connect()
    for q in (0, 1, 2):
        pub.publish(f"dev/{q}/m", b"q%d" % q, qos=q)
    pub.publish("low/x", b"downgraded", qos=2)               # delivered at min(2, granted 0)
    assert wait(lambda: len(inbox.got) == 4)
    assert sorted(inbox.got) == [("dev/0/m", b"q0"), ("dev/1/m", b"q1"), ("dev/2/m", b"q2"), ("low/x", b"downgraded")]
    assert pub.inflight == 0
    sub.unsubscribe("dev/+/m")
    pub.publish("dev/9/m", b"after", qos=1)
    time.sleep(0.2)
    assert len(inbox.got) == 4
    pub.disconnect()
    sub.disconnect()


def test_inbound_qos2_duplicate_is_delivered_once(broker):
    """A QoS 2 PUBLISH retransmitted with DUP before PUBREL reaches subscribers once (exactly once)."""
    sub = MqttClient("127.0.0.1", broker.port).connect()
    inbox = _Inbox(sub)
    sub.subscribe("x", 1)
    s = socket.create_connection(("127.0.0.1", broker.port))
    s.sendall(packet(CONNECT, 0, _enc_str("MQTT") + bytes([4, 2]) + struct.pack("!H", 30) + _enc_str("raw")))
    assert read_packet(s)[0] == 2
    for dup in (False, True):
        s.sendall(publish_packet("x", b"once", 2, pid=7, dup=dup))
        t, _, body = read_packet(s)
        assert t == 5 and body == struct.pack("!H", 7)          # PUBREC both times
    s.sendall(packet(6, 2, struct.pack("!H", 7)))                # PUBREL
    assert read_packet(s)[0] == 7                                # PUBCOMP
    assert wait(lambda: len(inbox.got) == 1)
    time.sleep(0.1)
    assert inbox.got == [("x", b"once")]
    s.close()
    sub.disconnect()


def test_authentication_and_client_from_reference_attributes():
    b = MqttBroker(users={"sitewhere": "s3cret"}).start()
    try:
        with pytest.raises(ConnectionError, match="bad user name or password"):
            MqttClient("127.0.0.1", b.port, username="sitewhere", password="wrong").connect()
        with pytest.raises(ConnectionError):
            MqttClient("127.0.0.1", b.port).connect()
        c = client_from_config({"hostname": "127.0.0.1", "port": str(b.port), "username": "sitewhere",
                                "password": "s3cret", "clientId": "sw-ref", "cleanSession": "false"}).connect()
        assert c.client_id == "sw-ref" and c.clean_session is False
        assert b.session("sw-ref") is not None
        c.disconnect()
    finally:
        b.stop()


def test_retained_messages(broker):
    pub = MqttClient("127.0.0.1", broker.port).connect()
    pub.publish("cfg/a", b"v1", qos=1, retain=True)
    pub.publish("cfg/a", b"v2", qos=1, retain=True)              # replaces
    pub.publish("cfg/b", b"b1", qos=0, retain=True)
    late = MqttClient("127.0.0.1", broker.port).connect()
    inbox = _Inbox(late)
    late.subscribe("cfg/#", 1)
    assert wait(lambda: len(inbox.got) == 2)
    assert sorted(inbox.got) == [("cfg/a", b"v2"), ("cfg/b", b"b1")]
    pub.publish("cfg/a", b"", qos=1, retain=True)                # empty retained payload clears it
    late2 = MqttClient("127.0.0.1", broker.port).connect()
    inbox2 = _Inbox(late2)
    late2.subscribe("cfg/#", 1)
    assert wait(lambda: len(inbox2.got) == 1) and inbox2.got == [("cfg/b", b"b1")]
    for c in (pub, late, late2):
        c.disconnect()


def test_persistent_session_queues_while_offline(broker):
    c = MqttClient("127.0.0.1", broker.port, client_id="dev-7", clean_session=False).connect()
    c.subscribe("cmd/dev-7", 1)
    c.disconnect()
    assert wait(lambda: broker.session("dev-7").conn is None)    # the broker saw it go offline
    pub = MqttClient("127.0.0.1", broker.port).connect()
    for i in range(5):
        pub.publish("cmd/dev-7", b"c%d" % i, qos=1)
    pub.publish("cmd/dev-7", b"qos0-dropped", qos=0)
    c2 = MqttClient("127.0.0.1", broker.port, client_id="dev-7", clean_session=False)
    inbox = _Inbox(c2)
    c2.connect()
    assert c2.session_present
    assert wait(lambda: len(inbox.got) == 5)
    assert [p for _, p in inbox.got] == [b"c%d" % i for i in range(5)]
    c2.disconnect()
    c3 = MqttClient("127.0.0.1", broker.port, client_id="dev-7", clean_session=True).connect()
    assert not c3.session_present                                # a clean session discards the old one
    c3.disconnect()
    pub.disconnect()


def test_will_on_abnormal_disconnect_only(broker):
    watcher = MqttClient("127.0.0.1", broker.port).connect()
    inbox = _Inbox(watcher)
    watcher.subscribe("status/#", 1)
    a = MqttClient("127.0.0.1", broker.port, client_id="gw-a", will=("status/gw-a", b"offline", 1, False)).connect()
    a.disconnect()                                               # graceful: no will
    b = MqttClient("127.0.0.1", broker.port, client_id="gw-b", will=("status/gw-b", b"offline", 1, False)).connect()
    b._closed = True
    b.sock.shutdown(socket.SHUT_RDWR)                            # connection lost: the will fires
    assert wait(lambda: inbox.got == [("status/gw-b", b"offline")])
    time.sleep(0.1)
    assert inbox.got == [("status/gw-b", b"offline")]
    watcher.disconnect()


def test_keepalive_enforced_by_broker(broker):
    s = socket.create_connection(("127.0.0.1", broker.port))
    s.sendall(packet(CONNECT, 0, _enc_str("MQTT") + bytes([4, 2]) + struct.pack("!H", 1) + _enc_str("silent")))
    assert read_packet(s)[0] == 2
    s.settimeout(5)
    t0 = time.time()
    assert s.recv(1) == b""                                      # closed after 1.5 x keep-alive
    assert 1.0 <= time.time() - t0 < 4.0
    s.close()


def test_client_reconnects_resubscribes_and_retransmits():
    b = MqttBroker().start()
    port = b.port
    c = MqttClient("127.0.0.1", port, reconnect=True)
    inbox = _Inbox(c)
    c.connect()
    c.subscribe("in/#", 1)
    b.stop()
    assert wait(lambda: not c.connected.is_set())
    got = []

    def publish_while_down():                                    # QoS 1 stays in flight until a broker is back
        c.publish("in/late", b"retransmitted", qos=1, timeout=10)
        got.append(True)
    t = threading.Thread(target=publish_while_down)
    t.start()
    time.sleep(0.3)
    b2 = MqttBroker(port=port).start()
    try:
        assert wait(lambda: c.connected.is_set(), 10)
        t.join(10)
        assert got == [True] and c.reconnects >= 1
        assert wait(lambda: ("in/late", b"retransmitted") in inbox.got)   # resubscribed, then redelivered
        p = MqttClient("127.0.0.1", port).connect()
        p.publish("in/x", b"fresh", qos=1)
        assert wait(lambda: ("in/x", b"fresh") in inbox.got)
        p.disconnect()
    finally:
        c.disconnect()
        b2.stop()


def test_session_takeover_by_client_id(broker):
    first = MqttClient("127.0.0.1", broker.port, client_id="same").connect()
    second = MqttClient("127.0.0.1", broker.port, client_id="same").connect()
    assert wait(lambda: not first._reader.is_alive())            # the broker dropped the older link
    inbox = _Inbox(second)
    second.subscribe("t", 0)
    MqttClient("127.0.0.1", broker.port).connect().publish("t", b"to-second")
    assert wait(lambda: inbox.got == [("t", b"to-second")])
    second.disconnect()


def _openssl_cert(tmp_path):
    if shutil.which("openssl") is None:
        pytest.skip("openssl not available to create a test certificate")
    key, cert = tmp_path / "key.pem", tmp_path / "cert.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                    str(cert), "-days", "1", "-subj", "/CN=localhost",
                    "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost"],
                   check=True, capture_output=True, timeout=60)
    return str(cert), str(key)


def test_tls_and_mutual_tls(tmp_path):
    cert, key = _openssl_cert(tmp_path)
    sctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    sctx.load_cert_chain(cert, key)
    sctx.load_verify_locations(cert)
    sctx.verify_mode = ssl.CERT_REQUIRED                         # key store required on the client too
    b = MqttBroker(ssl_context=sctx).start()
    try:
        c = client_from_config({"protocol": "tls", "hostname": "127.0.0.1", "port": b.port,
                                "trustStorePath": cert, "keyStorePath": cert, "keyPath": key}).connect()
        inbox = _Inbox(c)
        c.subscribe("secure/#", 2)
        c.publish("secure/t", b"over-tls", qos=2)
        assert wait(lambda: inbox.got == [("secure/t", b"over-tls")])
        c.disconnect()
        with pytest.raises((ssl.SSLError, ConnectionError, OSError)):   # no client certificate
            MqttClient("127.0.0.1", b.port, protocol="ssl", ca_file=cert).connect()
        with pytest.raises(ssl.SSLError):                               # untrusted server
            MqttClient("127.0.0.1", b.port, protocol="tls").connect()
    finally:
        b.stop()


def test_receiver_hands_off_then_acks_and_survives_broker_restart():
    b = MqttBroker(users={"u": "p"}).start()
    port = b.port
    got = []

    class Src:
        def on_encoded_event_received(self, recv, payload, md):
            got.append((bytes(payload), md["topic"]))
    r = build_receiver({"type": "mqtt", "hostname": "127.0.0.1", "port": port, "topic": "SiteWhere/t/input/#",
                        "qos": "EXACTLY_ONCE", "username": "u", "password": "p", "numThreads": 2})
    r.source = Src()
    r.start(None)
    try:
        dev = MqttClient("127.0.0.1", port, username="u", password="p").connect()
        dev.publish("SiteWhere/t/input/json", b'{"m":1}', qos=2)
        assert wait(lambda: got == [(b'{"m":1}', "SiteWhere/t/input/json")])
        dev.disconnect()
        b.stop()
        b = MqttBroker(port=port, users={"u": "p"}).start()
        assert wait(lambda: r.client.connected.is_set() and r.client.reconnects >= 1, 10)
        dev = MqttClient("127.0.0.1", port, username="u", password="p").connect()
        end = time.time() + 10
        while len(got) < 2 and time.time() < end:                # until the resubscription is in place
            dev.publish("SiteWhere/t/input/json", b'{"m":2}', qos=1)
            time.sleep(0.1)
        assert (b'{"m":2}', "SiteWhere/t/input/json") in got
        dev.disconnect()
    finally:
        r.stop(None)
        b.stop()


def test_qos0_batches_forwarded_whole_and_delivered_by_topic(broker):
    """A publisher's burst of QoS 0 publishes on two topics reaches the broker in large reads: the
    broker forwards a read whole when its topics share the subscribers (``_forward_batch``), and an
    ``on_messages`` subscriber gets each topic's payloads together, in order; a plain ``on_message``
    subscriber still sees every message; a retained publish in the stream takes the per-packet path."""
    got, single = {}, []
    lock = threading.Lock()
    sub = MqttClient("127.0.0.1", broker.port).connect()

    def batch(topic, payloads):
        with lock:
            got.setdefault(topic, []).extend(payloads)
    sub.on_messages(batch)
    sub.subscribe("fan/#", 0)
    sub2 = MqttClient("127.0.0.1", broker.port).connect()
    sub2.on_message(lambda t, p: single.append((t, p)))
    sub2.subscribe("fan/#", 0)
    pub = MqttClient("127.0.0.1", broker.port).connect()
    n = 3000
    msgs = [(f"fan/{i % 2}", f"m{i}".encode()) for i in range(n)]
    pub.publish_many(msgs, qos=0)
    pub.publish("fan/0", b"retained", qos=0, retain=True)
    end = time.time() + 20
    while time.time() < end and (sum(len(v) for v in got.values()) < n + 1 or len(single) < n + 1):
        time.sleep(0.05)
    assert got["fan/0"] == [p for t, p in msgs if t == "fan/0"] + [b"retained"]
    assert got["fan/1"] == [p for t, p in msgs if t == "fan/1"]
    assert sorted(single) == sorted(msgs + [("fan/0", b"retained")])
    for c in (pub, sub, sub2):
        c.disconnect()
