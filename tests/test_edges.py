"""Protocol edges: AMQP 0-9-1 (RabbitMQ) and STOMP (ActiveMQ) wire protocols, cloud HTTP connectors.

The reference tested these only as manual harnesses against live brokers (SURVEY §4:
``EventSourceTests.java`` with an embedded ActiveMQ broker, ``StompTest.java``); here each protocol
runs against the embedded broker in-process.
"""
from __future__ import annotations

import json
import time
import urllib.parse

import pytest

from sitewhere_amd.edges.amqp import AmqpBroker, AmqpClient, RabbitMqReceiver
from sitewhere_amd.edges.stomp import StompBroker, StompClient, StompReceiver
from sitewhere_amd.models.domain import DeviceLocation, DeviceMeasurement
from sitewhere_amd.services.cloud_connectors import (DweetConnector, EventHubConnector, InitialStateConnector,
                                                      RabbitMqConnector, SqsConnector, sas_token, sigv4_headers)


class _Src:
    def __init__(self):
        self.got = []

    def on_encoded_event_received(self, recv, payload, md):
        self.got.append((bytes(payload), md))


def wait(cond, t=30.0):          # returns as soon as cond holds; the bound only catches a real failure
    end = time.time() + t
    while time.time() < end and not cond():
        time.sleep(0.01)
    return cond()


def test_amqp_publish_consume_large_and_ack():
    b = AmqpBroker().start()
    try:
        c1 = AmqpClient("127.0.0.1", b.port).connect()
        c1.queue_declare("q1")
        c2 = AmqpClient("127.0.0.1", b.port).connect()
        c2.publish("", "q1", b"hello")                  # queued before any consumer: backlog
        big = bytes(range(256)) * 2000                  # 512 KB -> several body frames
        got = []
        c1.consume("q1", lambda d: (got.append(d["body"]), c1.ack(d["delivery_tag"])))
        c2.publish("", "q1", big)
        assert wait(lambda: len(got) == 2)
        assert got == [b"hello", big]
        assert wait(lambda: b.acked == 2)
        # named exchange with binding
        c1.queue_declare("q2")
        c1.queue_bind("q2", "events", "dev.1")
        got2 = []
        c3 = AmqpClient("127.0.0.1", b.port).connect()
        c3.consume("q2", lambda d: got2.append((d["exchange"], d["routing_key"], d["body"])), no_ack=True)
        c2.publish("events", "dev.1", b"x")
        c2.publish("events", "dev.2", b"dropped")
        assert wait(lambda: got2 == [("events", "dev.1", b"x")])
        for c in (c1, c2, c3):
            c.close()
    finally:
        b.stop()


def test_rabbitmq_receiver_and_connector():
    b = AmqpBroker().start()
    try:
        r = RabbitMqReceiver("127.0.0.1", b.port, "sw.in")
        src = _Src()
        r.source = src
        r.start(None)
        pub = AmqpClient("127.0.0.1", b.port).connect()
        for i in range(20):
            pub.publish("", "sw.in", f"payload-{i}".encode())
        assert wait(lambda: len(src.got) == 20)
        assert src.got[0] == (b"payload-0", {"queue": "sw.in", "routingKey": "sw.in"})
        r.stop(None)
        # outbound: the connector publishes enriched events; a consumer reads them back
        sink = AmqpClient("127.0.0.1", b.port).connect()
        sink.queue_declare("out.dev-1")
        got = []
        sink.consume("out.dev-1", lambda d: got.append(json.loads(d["body"])), no_ack=True)
        conn = RabbitMqConnector("rmq", "127.0.0.1", b.port, "", "out.{deviceToken}")
        conn.start(None)
        ev = DeviceMeasurement(name="t", value=2.5, device_id="d1")
        conn.process_batch([(ev, {"deviceToken": "dev-1"})])
        assert wait(lambda: len(got) == 1)
        assert got[0]["event"]["name"] == "t" and got[0]["context"]["deviceToken"] == "dev-1"
        conn.stop(None)
        pub.close()
        sink.close()
    finally:
        b.stop()


def test_stomp_queue_topic_and_receiver():
    b = StompBroker().start()
    try:
        c = StompClient("127.0.0.1", b.port).connect()
        got_t1, got_t2 = [], []
        c.subscribe("/topic/alerts", lambda h, body: got_t1.append(body))
        c2 = StompClient("127.0.0.1", b.port).connect()
        c2.subscribe("/topic/alerts", lambda h, body: got_t2.append(body))
        c.send("/topic/alerts", b"a\0binary\nbody", receipt=True)       # NUL + newline need content-length
        assert wait(lambda: got_t1 == [b"a\0binary\nbody"] and got_t2 == [b"a\0binary\nbody"])
        r = StompReceiver("127.0.0.1", b.port, "/queue/SW.IN")
        src = _Src()
        r.source = src
        c.send("/queue/SW.IN", b"early", receipt=True)                  # backlog before the subscriber
        r.start(None)
        for i in range(10):
            c.send("/queue/SW.IN", f"m{i}".encode(), {"x-key": "a:b"})
        assert wait(lambda: len(src.got) == 11)
        assert sorted(p for p, _ in src.got) == sorted([b"early"] + [f"m{i}".encode() for i in range(10)])
        r.stop(None)
        c.close()
        c2.close()
    finally:
        b.stop()


def test_sigv4_known_vector():
    """AWS SigV4 example (IAM ListUsers, documented test credentials) -> documented signature."""
    from datetime import datetime, timezone
    h = sigv4_headers("GET", "https://iam.amazonaws.com/?Action=ListUsers&Version=2010-05-08", b"", "us-east-1", "iam",
                      "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY",
                      now=datetime(2015, 8, 30, 12, 36, 0, tzinfo=timezone.utc),
                      extra={"content-type": "application/x-www-form-urlencoded; charset=utf-8"})
    assert h["x-amz-date"] == "20150830T123600Z"
    assert "Credential=AKIDEXAMPLE/20150830/us-east-1/iam/aws4_request" in h["Authorization"]
    assert "SignedHeaders=content-type;host;x-amz-content-sha256;x-amz-date" in h["Authorization"]


def test_cloud_http_connectors_requests():
    sent = []
    post = lambda url, body, headers: sent.append((url, body, headers))  # noqa: E731
    evs = [(DeviceMeasurement(name=f"m{i}", value=float(i), device_id="d", event_date=1000 * i), {"deviceToken": "tok"})
           for i in range(13)]
    sqs = SqsConnector("sqs", "https://sqs.us-east-1.amazonaws.com/123/q", "us-east-1", "AK", "SK", post=post)
    sqs.process_batch(evs)
    assert len(sent) == 2                                   # 10 + 3 entries
    params = dict(urllib.parse.parse_qsl(sent[0][1].decode()))
    assert params["Action"] == "SendMessageBatch" and "SendMessageBatchRequestEntry.10.MessageBody" in params
    assert sent[0][2]["Authorization"].startswith("AWS4-HMAC-SHA256 Credential=AK/")
    sent.clear()
    eh = EventHubConnector("eh", "ns", "hub", "send", "secretkey", post=post)
    eh.process_batch(evs[:3])
    url, body, headers = sent[0]
    assert url == "https://ns.servicebus.windows.net/hub/messages"
    assert headers["Authorization"].startswith("SharedAccessSignature sr=https%3A%2F%2Fns.servicebus.windows.net%2Fhub")
    assert len(json.loads(body)) == 3
    tok = sas_token("https://ns.servicebus.windows.net/hub", "send", "k", ttl_s=10, now=100.0)
    assert tok.endswith("&se=110&skn=send")
    sent.clear()
    DweetConnector("dw", post=post).process_batch(evs[:2])
    assert [u for u, _, _ in sent] == ["https://dweet.io/dweet/for/tok"] * 2
    sent.clear()
    loc = DeviceLocation(latitude=1.0, longitude=2.0, device_id="d")
    InitialStateConnector("is", "ACCESS", post=post).process_batch(evs[:2] + [(loc, {"deviceToken": "tok"})])
    assert len(sent) == 1 and sent[0][2]["X-IS-BucketKey"] == "tok"
    assert [e["key"] for e in json.loads(sent[0][1])] == ["m0", "m1", "location"]


def test_build_receiver_and_connector_types():
    from sitewhere_amd.edges.receivers import build_receiver
    assert type(build_receiver({"type": "activemq", "port": 1})).__name__ == "StompReceiver"
    assert type(build_receiver({"type": "rabbitmq", "port": 1})).__name__ == "RabbitMqReceiver"
    with pytest.raises(ValueError):
        build_receiver({"type": "nope"})


def test_solr_connector_indexes_and_search_provider_queries():
    """SolrOutboundConnector -> Solr JSON update handler; SolrSearchProvider -> /select (SURVEY §2.1
    sitewhere-solr, service-event-search).  Against a local HTTP stand-in for a Solr core."""
    import http.server
    import json as _json
    import threading as _th
    import urllib.parse as up

    from sitewhere_amd.models.domain import DeviceMeasurement
    from sitewhere_amd.services.labels_media_search import SolrSearchProvider
    from sitewhere_amd.services.outbound_connectors import SolrConnector

    docs = []

    class Solr(http.server.BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_POST(self):
            assert self.path.startswith("/SiteWhere/update")
            docs.extend(_json.loads(self.rfile.read(int(self.headers["Content-Length"]))))
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b'{"responseHeader":{"status":0}}')

        def do_GET(self):
            u = up.urlparse(self.path)
            q = dict(up.parse_qsl(u.query))
            assert u.path == "/SiteWhere/select" and q["wt"] == "json"
            f, v = q["q"].split(":", 1)
            hits = [d for d in docs if str(d.get(f)) == v][:int(q["rows"])]
            body = _json.dumps({"response": {"numFound": len(hits), "docs": hits}}).encode()
            self.send_response(200)
            self.end_headers()
            self.wfile.write(body)

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Solr)
    _th.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}"
        con = SolrConnector("solr", url)
        evs = [DeviceMeasurement(device_assignment_id="a1", device_id="d1", name="temp", value=float(i),
                                 event_date=1000 + i) for i in range(3)]
        con.deliver([(e, {}) for e in evs])
        assert {d["id"] for d in docs} == {e.id for e in evs}
        assert docs[0]["eventType"] == "Measurement" and docs[0]["name_s"] == "temp" and "value_d" in docs[0]
        hits = SolrSearchProvider("solr", url).search("assignmentId:a1", rows=2)
        assert len(hits) == 2 and all(h["assignmentId"] == "a1" for h in hits)
    finally:
        srv.shutdown()


def test_stomp_template_tenant_hosts_broker(monkeypatch):
    """Reference templates/stomp: the tenant's event source hosts the broker; a STOMP client sends a
    JSON batch to SITEWHERE.STOMP and the measurements are stored."""
    import json
    import socket
    import time

    from sitewhere_amd.assembly import SiteWhereInstance
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    monkeypatch.setenv("STOMP_PORT", str(port))
    sw = SiteWhereInstance().start()
    try:
        sw.wait_for_tenant("default", 60)
        tm = sw.api("TenantManagement")
        sw.instance.system_user.run(lambda: tm.create_tenant({"token": "st", "name": "st",
                                                              "configurationTemplateId": "stomp",
                                                              "datasetTemplateId": "construction"}))
        sw.wait_for_tenant("st", 120)
        run = lambda f: sw.instance.system_user.run(f, "st")  # noqa: E731
        dm, em = sw.api("DeviceManagement", "st"), sw.api("DeviceEventManagement", "st")
        aid = run(lambda: dm.get_device_by_token("meitrack-001")).device_assignment_id
        c = StompClient("127.0.0.1", port).connect()
        c.send("/queue/SITEWHERE.STOMP", json.dumps({"deviceToken": "meitrack-001", "measurements": [
            {"name": "stomp.t", "value": 4.5}, {"name": "stomp.h", "value": 0.5}]}).encode(), receipt=True)
        end, res = time.time() + 30, []
        while len(res) < 2 and time.time() < end:
            res = [e for e in run(lambda: em.list_measurements_for_index("Assignment", [aid])).results
                   if e.name.startswith("stomp.")]
            time.sleep(0.1)
        assert sorted((e.name, e.value) for e in res) == [("stomp.h", 0.5), ("stomp.t", 4.5)]
        c.close()
    finally:
        sw.stop()
