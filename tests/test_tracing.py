"""Span export: Jaeger agent UDP compact ``emitBatch`` and OTLP/HTTP JSON reporters."""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

from sitewhere_amd.core import tracing
from sitewhere_amd.core.trace_export import (JaegerUdpReporter, MiniJaegerAgent, OtlpHttpReporter, decode_emit_batch,
                                             encode_emit_batch)
from sitewhere_amd.core.tracing import Tracer


def _wait(cond, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end and not cond():
        time.sleep(0.02)
    return cond()


def _spans(tr: Tracer, n: int):
    out = []
    for i in range(n):
        with tr.start_span(f"op-{i}", force_sample=True) as root:
            root.set_tag("i", i).set_tag("ratio", 0.5).set_tag("ok", True).set_tag("who", "me")
            with tr.start_span("child") as ch:
                ch.log(event="step", detail="x" * 10)
                try:
                    raise ValueError("boom")
                except ValueError as e:
                    ch.set_error(e)
            out += [ch, root]
    return out


def test_emit_batch_roundtrip():
    tr = Tracer(sample_rate=0.0)
    spans = _spans(tr, 10)                         # 20 spans: list header uses the long form (>= 15)
    spans[1].span_id = "f" * 16                    # ids with the top bit set survive the signed i64 mapping
    pkt = encode_emit_batch("svc", spans, seq=7, process_tags={"host": "h1", "pid": 42})
    d = decode_emit_batch(pkt)
    assert d["service"] == "svc" and d["seq"] == 7 and len(d["spans"]) == 20
    for s, got in zip(spans, d["spans"]):
        assert int(got["traceId"], 16) == int(s.trace_id, 16) and got["spanId"] == s.span_id
        assert got["name"] == s.name and got["flags"] == 1
        assert (got["parentId"] is None) == (s.parent_id is None)
        assert abs(got["durationUs"] - (s.end - s.start) * 1e6) <= 1
    root = d["spans"][1]
    assert root["tags"] == {"service": "sitewhere", "i": 0, "ratio": 0.5, "ok": True, "who": "me"}
    child = d["spans"][0]
    assert child["parentId"] == spans[1].parent_id or child["parentId"] is not None
    assert child["tags"]["error"] is True
    assert [lg["event"] for lg in child["logs"]] == ["step", "error"] and child["logs"][1]["message"] == "boom"


def test_jaeger_udp_reporter_to_agent_splits_datagrams():
    agent = MiniJaegerAgent().start()
    rep = JaegerUdpReporter("127.0.0.1", agent.port, "sw-test", max_packet=2000, interval_s=0.05)
    tr = Tracer(sample_rate=0.0, reporter=rep)
    spans = _spans(tr, 30)
    try:
        assert _wait(lambda: len(agent.spans) == 60)
        assert rep.sent_batches > 1 and rep.errors == 0 and agent.bad == 0
        assert {s["spanId"] for s in agent.spans} == {s.span_id for s in spans}
        assert all(b["service"] == "sw-test" for b in agent.batches)
    finally:
        rep.close()
        agent.stop()


def test_otlp_http_reporter():
    got = []

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            got.append((self.path, json.loads(self.rfile.read(int(self.headers["Content-Length"])))))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass
    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    rep = OtlpHttpReporter(f"http://127.0.0.1:{srv.server_address[1]}", "sw-otlp", interval_s=0.05)
    tr = Tracer(sample_rate=0.0, reporter=rep)
    spans = _spans(tr, 3)
    try:
        assert _wait(lambda: sum(len(b["resourceSpans"][0]["scopeSpans"][0]["spans"]) for _, b in got) == 6)
        assert all(p == "/v1/traces" for p, _ in got)
        rs = got[0][1]["resourceSpans"][0]
        assert rs["resource"]["attributes"][0] == {"key": "service.name", "value": {"stringValue": "sw-otlp"}}
        out = {s["spanId"]: s for _, b in got for s in b["resourceSpans"][0]["scopeSpans"][0]["spans"]}
        child = out[spans[0].span_id.rjust(16, "0")]
        assert child["status"] == {"code": 2} and child["parentSpanId"] == spans[1].span_id.rjust(16, "0")
        assert len(child["traceId"]) == 32 and child["events"][0]["name"] == "step"
    finally:
        rep.close()
        srv.shutdown()


def test_instance_reports_lifecycle_spans_to_jaeger_agent():
    from sitewhere_amd.assembly import SiteWhereInstance
    from sitewhere_amd.runtime.config import InstanceSettings
    agent = MiniJaegerAgent().start()
    saved = tracing.global_tracer()
    tracing.set_global_tracer(Tracer())
    sw = None
    try:
        settings = InstanceSettings(tracer_server=f"127.0.0.1:{agent.port}", tracer_sample_rate=1.0)
        sw = SiteWhereInstance(settings).start()
        sw.wait_for_tenant("default", 60)
        assert _wait(lambda: any(s["name"].startswith("Start microservice") for s in agent.spans), 20)
        names = {s["name"] for s in agent.spans}
        assert any(n.startswith("Initialize tenant engine") for n in names)
        assert agent.batches[0]["service"] == "sitewhere"
    finally:
        if sw is not None:
            sw.stop()
        tracing.set_global_tracer(saved)
        agent.stop()
