"""Native outbound JSON: the connectors' {"event", "context"} documents written by
``swjson_rows`` from a decoded block equal ``json.dumps(event_json(event, context))`` of the Python
path byte for byte -- every event type, engine-generated alerts and presence changes, metadata,
elevation, missing dictionary entries, non-ASCII and malformed UTF-8 strings, float repr edge
values -- and the MQTT QoS 0 framing parses back into the same (topic, payload) pairs."""
from __future__ import annotations

import json

import numpy as np

from sitewhere_amd.models import wire
from sitewhere_amd.persistence import segments as sg
from sitewhere_amd.pipeline.config import EngineConfig
from sitewhere_amd.pipeline.engine_base import Zone, ZoneTest
from sitewhere_amd.pipeline.fleet import FleetSpec, fingerprints, gen_payloads, gen_tokens, pack_messages
from sitewhere_amd.pipeline.native_engine import NativeCpuEngine
from sitewhere_amd.services.enriched_batches import EnrichedBatchReader
from sitewhere_amd.services.outbound_connectors import event_json

N_DEV = 3000
NOW = 1_700_000_100_000


def _block():
    e = NativeCpuEngine(EngineConfig.small(max_msgs=8192, max_devices=8192, max_assignments=8192))
    heap, offs = gen_tokens("dev-", 0, N_DEV)
    lo, hi = fingerprints(heap, offs)
    d = e.register_devices(lo, hi)
    e.set_assignments(d, d)
    sq = [(33.0, -85.0), (33.0, -84.0), (34.0, -84.0), (34.0, -85.0)]
    e.set_zone_rules([Zone("z", sq)], [ZoneTest("z", "inside", "zone.enter", 2, "entered the zone")])
    spec = FleetSpec(prefix="dev-", n_devices=N_DEV, p_location=0.3, p_alert=0.1, mx_per_msg=2, with_alternate_id=True,
                     lat0=33.0, lon0=-85.0, span_deg=2.0, p_meta=0.3)
    raw, off = gen_payloads(spec, 3000, NOW - 60_000, seed=5)
    msgs = [bytes(raw[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    # strings the generator does not make: non-ASCII, escapes, malformed UTF-8, float edge values
    odd = [wire.measurements("dev-0000000007", {"témp": 1e16, "q": 1.5e-05, "z": -0.0, "big": 12345678901234567.0},
                             event_date=NOW - 5, alternate_id="alt-☃-\"q\"\\", metadata={"nöte": "a\tb\n\u0001"}),
           wire.alert("dev-0000000008", "dooré", "msg \U0001F600 \x7f", event_date=NOW - 4, alternate_id="x\xff"),
           wire.location("dev-0000000009", 33.5, -84.5, elevation=0.0001, event_date=NOW - 3)]
    raw2, off2 = pack_messages(msgs + odd)
    res = e.step(raw2, off2, NOW, presence=True)
    blk = e.encode_block(NOW, res, boot=0x5eed)
    # nine hours later: the presence scan's state changes (DevicePresenceManager), in a block of their own
    later = NOW + 9 * 3600 * 1000
    res2 = e.step(np.zeros(64, np.uint8), np.zeros(1, np.uint32), later, presence=True)
    blk2 = e.encode_block(later, res2, boot=0x5eed)
    names = {i: e.names.get(h, str(h)) for h, i in e.intern_table().items()}
    return [np.asarray(blk), np.asarray(blk2)], names, e


def test_native_outbound_json_equals_python():
    blks, names, e = _block()
    # the malformed id bytes: patch one alternate id in the raw stream is not possible through the
    # wire encoder (it writes UTF-8); the block keeps what the device sent, so feed the reader a
    # dictionary with missing and non-ASCII entries instead
    r = EnrichedBatchReader(None)
    asg = {i: [f"asg-{i}", f"dev-id-{i}", f"cust-ç{i % 3}", None, f"asset-{i % 5}", f"dev-{i:010d}",
               "type-\U0001F697"] for i in range(N_DEV) if i % 11}
    asg.update({i: [f"asg-{i}", f"dev-id-{i}", None, None, None] for i in range(0, N_DEV, 22)})   # 5-entry contexts
    rules = {"zone.enter": "entered the zone"}
    r._apply(0x5eed, {"asg": asg, "names": names, "rules": rules})
    kinds = set()
    for blk in blks:
        cols = sg.decode_block(blk)
        cols["asg_ctx"], cols["names"], cols["rules"] = r._asg[0x5eed], r._names[0x5eed], r._rules
        n = len(cols["date"])
        rows = np.arange(n)
        got = r.outbound_json(cols, rows, topic="out/{deviceToken}/{eventType}")
        assert got is not None
        buf, off, tbuf, toff = got
        for i in range(n):
            ev, ctx = r.event(cols, i), r.context(cols, i)
            want = json.dumps(event_json(ev, ctx)).encode()
            assert bytes(buf[off[i]:off[i + 1]]) == want, (i, bytes(buf[off[i]:off[i + 1]])[:400], want[:400])
            topic = f"out/{ctx.get('deviceToken')}/{ev.event_type.value}".encode()
            assert bytes(tbuf[toff[i]:toff[i + 1]]) == topic
            kinds.add((ev.event_type.value, bool(ev.metadata), getattr(ev, "source", None)))
    cols = sg.decode_block(blks[0])
    cols["asg_ctx"], cols["names"], cols["rules"] = r._asg[0x5eed], r._names[0x5eed], r._rules
    n = len(cols["date"])
    buf, off, _, _ = r.outbound_json(cols, np.arange(n))
    assert {k[0] for k in kinds} >= {"Measurement", "Location", "Alert", "StateChange"}
    assert any(k[1] for k in kinds)
    assert any(k[0] == "Alert" and k[2].value == "System" for k in kinds)           # rule-generated alerts
    assert any(k[0] == "Alert" and k[2].value == "Device" for k in kinds)
    # a subset, in any order
    sel = np.array([n - 1, 3, 0, n // 2])
    buf2, off2, _, _ = r.outbound_json(cols, sel)
    for j, i in enumerate(sel):
        assert bytes(buf2[off2[j]:off2[j + 1]]) == bytes(buf[off[i]:off[i + 1]])


def test_malformed_utf8_is_replaced_like_python():
    """Strings the native writer escapes from raw bytes: decode("utf-8", "replace") then ensure_ascii."""
    from sitewhere_amd._native import native
    cases = [b"ok", b"\xff", b"a\xc3", b"\xe0\x80x", b"\xed\xa0\x80", b"\xf0\x9f\x98", b"\xf4\x90\x80\x80",
             b"\xc0\xaf", b"\xe2\x82\xac\xe2\x82", "☃\U0001F600".encode(), b"\x00\x1f\x7f\"\\"]
    for s in cases:
        blk_cols = _cols_with_alt(s)
        r = EnrichedBatchReader(None)
        buf, off, _, _ = r.outbound_json(blk_cols, np.array([0]))
        doc = json.loads(bytes(buf).decode())
        assert doc["event"]["alternateId"] == s.decode("utf-8", "replace"), s
        want = json.dumps(s.decode("utf-8", "replace"))
        assert want.encode() in bytes(buf), (s, bytes(buf))
    assert native() is not None


def _cols_with_alt(alt: bytes) -> dict:
    """Decoded-column stand-in of one measurement row whose alternate id is ``alt`` (raw bytes)."""
    heap = np.frombuffer(alt + b"\0" * 8, np.uint8).copy()
    return {"etype": np.zeros(1, np.uint8), "level": np.zeros(1, np.uint8), "date": np.array([5], np.int64),
            "asg": np.array([-1], np.int32), "name": np.array([0xFFFF], np.uint16), "v0": np.array([1.0]),
            "v1": np.zeros(1), "v2": np.zeros(1), "flags": np.array([0x8], np.uint8), "str_heap": heap,
            "str_off": np.array([0, len(alt), len(alt), len(alt)], np.int64),
            "header": {"boot": 1, "first_seq": 0, "world": 1, "rank": 0, "recv_ms": 9}, "row0": 0}


def test_mqtt_qos0_framing():
    from sitewhere_amd._native import native
    topics = [b"a/b", b"t" * 200, b""]
    payloads = [b"x", b"y" * 20000, b"{}"]
    tb, pb = b"".join(topics), b"".join(payloads)
    to = np.concatenate([[0], np.cumsum([len(t) for t in topics])]).astype(np.int64)
    po = np.concatenate([[0], np.cumsum([len(p) for p in payloads])]).astype(np.int64)
    tba, pba = np.frombuffer(tb, np.uint8), np.frombuffer(pb, np.uint8)
    out = np.empty(1 << 16, np.uint8)
    k = int(native().swmqtt_publish_qos0(tba.ctypes.data, to.ctypes.data, pba.ctypes.data, po.ctypes.data, 3, 0,
                                         out.ctypes.data, len(out)))
    assert k > 0
    data, pos, got = bytes(out[:k]), 0, []
    while pos < len(data):
        assert data[pos] == 0x30
        pos += 1
        rl, mul = 0, 1
        while True:
            b = data[pos]
            pos += 1
            rl += (b & 0x7F) * mul
            mul *= 128
            if not b & 0x80:
                break
        tl = int.from_bytes(data[pos:pos + 2], "big")
        got.append((data[pos + 2:pos + 2 + tl], data[pos + 2 + tl:pos + rl]))
        pos += rl
    assert got == list(zip(topics, payloads))


class _StubEM:
    """Event management of a consumer that started late: the store holds no entry it lacks."""
    def __init__(self):
        self.calls = 0

    def durable_dictionary(self, boot, asg_ids, name_ids):
        self.calls += 1
        return {"asg": {}, "names": {}}


class _StubEngine:
    def __init__(self):
        self.em = _StubEM()
        self.tenant = type("T", (), {"token": "t"})()
        self.ms = type("M", (), {"api": lambda _s, *a: self.em})()


def test_native_block_selection_equals_column_filters():
    """``select_json`` (native selection + JSON straight from the durable block) keeps exactly the
    rows the column filters keep, in block order, with the same documents and topics; assignments
    the consumer never saw a dictionary entry for are resolved (here: to no context) once."""
    from sitewhere_amd.services.outbound_connectors import EventTypeFilter, _Filter, combined_selector
    blks, names, e = _block()
    asg = {i: [f"asg-{i}", f"dev-id-{i}", f"cust-{i % 3}", f"area-{i % 4}", None, f"dev-{i:010d}", f"type-{i % 2}"]
           for i in range(N_DEV) if i % 13}

    class Area(_Filter):
        def __init__(self, op):
            self.op = op

        def exclude(self, cols, reader):
            return self._out(reader.attr_mask(cols, 3, "area-1"))

        def select(self, reader, boot):
            return self._select_attr(reader, boot, 3, "area-1")

    for filters in ([], [Area("include")], [Area("exclude"), EventTypeFilter(["Measurement", "Alert"])],
                    [EventTypeFilter(["Location"])]):
        for threads in (1, 3):
            rec = sg.encode_durable_batch(blks[0], 0x5eed, asg=asg, names=names, rules={"zone.enter": "entered the zone"})
            r = EnrichedBatchReader(_StubEngine())
            got = r.select_json(rec, combined_selector(filters, r), topic="o/{deviceToken}/{eventType}", threads=threads)
            assert got is not None
            buf, off, tbuf, toff, kept, total = got
            r2 = EnrichedBatchReader(_StubEngine())
            cols = r2.columns(rec)
            n = len(cols["date"])
            excl = np.zeros(n, bool)
            for f in filters:
                excl |= f.exclude(cols, r2)
            rows = np.nonzero(~excl)[0]
            assert total == n and kept == len(rows), (filters, kept, len(rows))
            wb, wo, wt, wto = r2.outbound_json(cols, rows, topic="o/{deviceToken}/{eventType}")
            assert bytes(buf) == bytes(wb) and np.array_equal(off, wo)
            assert bytes(tbuf) == bytes(wt) and np.array_equal(toff, wto)
            assert r.engine.em.calls == 1


def test_native_threshold_rows_equal_column_rule():
    """``ThresholdRuleProcessor`` over a durable block natively (``swseg_threshold_rows``) raises the
    same alerts, in the same order, as its column form over the decoded block -- min, max and both
    bounds, a name the batch lacks, and exception-coded (non-decimal) values."""
    from sitewhere_amd.services.rule_processing import ThresholdRuleProcessor
    blks, names, e = _block()
    asg = {i: [f"asg-{i}", f"dev-id-{i}", None, None, None, f"dev-{i:010d}", None] for i in range(N_DEV)}
    rec = sg.encode_durable_batch(blks[0], 0x5eed, asg=asg, names=names)
    mx = sorted({v for v in names.values() if v.startswith("mx.")} | {"témp"})
    rules = [{"measurement": mx[0], "max": 500.0, "alertType": "hi"}, {"measurement": mx[-1], "min": 100.0},
             {"measurement": mx[1 % len(mx)], "min": 200.0, "max": 800.0}, {"measurement": "absent", "max": 1.0}]
    got = {}
    for mode in ("native", "columns"):
        p = ThresholdRuleProcessor("t", rules)
        seen = []
        p.raise_alerts = lambda pairs, seen=seen: seen.extend(pairs)
        r = EnrichedBatchReader(_StubEngine())
        if mode == "native":
            p.process_records(r, [type("R", (), {"value": rec, "key": None})()])
        else:
            p.process_columns(r, r.columns(rec, strings=False))
        got[mode] = seen
    assert got["native"] == got["columns"]
    assert len(got["native"]) > 50
