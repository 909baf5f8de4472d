"""Native JSON -> protobuf transcoding of device requests (``csrc/native/swjson.cpp``,
``pipeline/json_transcode.py``): what a JSON device sends reaches the fused engine as exactly the
payload a protobuf device would send, and everything the engine path cannot represent stays on the
reference's per-event path (``JsonDeviceRequestDecoder``)."""
from __future__ import annotations

import json
import random

import pytest

from sitewhere_amd.models import wire
from sitewhere_amd.pipeline.json_transcode import batch_to_protobuf, to_protobuf
from sitewhere_amd.services.event_sources import JsonDeviceRequestDecoder, ProtobufDecoder


def _j(token, typ, req, originator=None):
    d = {"deviceToken": token, "type": typ, "request": req}
    if originator is not None:
        d["originator"] = originator
    return json.dumps(d).encode()


CASES = [
    (_j("dev-1", "DeviceMeasurement", {"name": "t", "value": 21.5}),
     wire.measurements("dev-1", {"t": 21.5})),
    (_j("dev-1", "DeviceMeasurement", {"name": "t", "value": 7, "eventDate": 1_700_000_000_001,
                                       "alternateId": "m-1", "updateState": False}, originator="o"),
     wire.measurements("dev-1", {"t": 7.0}, event_date=1_700_000_000_001, alternate_id="m-1",
                       update_state=False, originator="o")),
    (_j("dév-ü", "DeviceLocation", {"latitude": 33.75, "longitude": -84.39, "elevation": 312.5,
                                    "eventDate": 1_700_000_000_002, "alternateId": "l\\u00e9-1"}),
     wire.location("dév-ü", 33.75, -84.39, elevation=312.5, event_date=1_700_000_000_002, alternate_id="l\\u00e9-1")),
    (_j("dev-2", "DeviceAlert", {"type": "engine.hot", "message": "too hot \n \"x\"", "level": "Info",
                                 "source": "Device", "eventDate": 5}),
     wire.alert("dev-2", "engine.hot", "too hot \n \"x\"", event_date=5)),
    (_j("d", "DeviceMeasurement", {"name": "t", "value": 1, "metadata": {"unit": "C", "s\u00e9": "x\"y"},
                                   "alternateId": "jm-1", "updateState": True}),
     wire.measurements("d", {"t": 1.0}, alternate_id="jm-1", metadata={"unit": "C", "s\u00e9": "x\"y"},
                       update_state=True)),
    (_j("d", "DeviceLocation", {"latitude": 1.5, "longitude": 2.5, "metadata": {"a": "1", "b": ""}}),
     wire.location("d", 1.5, 2.5, metadata={"a": "1", "b": ""})),
    (_j("d", "DeviceAlert", {"type": "x", "message": "m", "metadata": {"k": "v"}, "eventDate": 9, "alternateId": "ja"}),
     wire.alert("d", "x", "m", event_date=9, alternate_id="ja", metadata={"k": "v"})),
    (_j("d", "DeviceMeasurement", {"name": "t", "value": 2, "metadata": {}}), wire.measurements("d", {"t": 2.0})),
    (b'{ "type" : "DeviceMeasurement" ,\n "request": {"name": "\\ud83d\\ude00", "value": -1.5e3, "extra": [1, {"a": null}]},'
     b' "deviceToken": "dev-3", "unused": {"k": [true, false]} }',
     wire.measurements("dev-3", {"\U0001F600": -1500.0})),
]


@pytest.mark.parametrize("j,pb", CASES)
def test_transcode_equals_the_protobuf_a_device_sends(j, pb):
    assert to_protobuf(j) == pb
    js = JsonDeviceRequestDecoder().decode(j, {})[0]
    pr = ProtobufDecoder().decode(pb, {})[0]
    assert (js["deviceToken"], js["type"]) == (pr["deviceToken"], pr["type"])
    for k, v in js["request"].items():
        if k in ("name", "value", "latitude", "longitude", "elevation", "eventDate", "alternateId", "type",
                 "message", "metadata", "updateState"):
            assert pr["request"].get(k) == (float(v) if k == "value" else v), k


STAYS = [
    b"not json",
    b"{}",
    _j("d", "RegisterDevice", {"deviceTypeToken": "t"}),
    _j("d", "Acknowledge", {"response": "ok"}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": 1, "metadata": {"unit": 5}}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": 1, "metadata": {"unit": None}}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": 1, "metadata": ["unit"]}),
    _j("d", "DeviceAlert", {"type": "x", "message": "m", "metadata": {"a": "b", "c": {"d": "e"}}}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": "12.5"}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": 1, "eventDate": "2024-01-01T00:00:00Z"}),
    _j("d", "DeviceMeasurement", {"name": "t", "value": 1, "eventDate": 1.5}),
    _j("d", "DeviceMeasurement", {"name": "t"}),
    _j("d", "DeviceLocation", {"latitude": 1.0}),
    _j("d", "DeviceAlert", {"type": "x", "message": "m", "level": "Critical"}),
    _j("d", "DeviceAlert", {"type": "x", "message": "m", "source": "System"}),
    _j("", "DeviceMeasurement", {"name": "t", "value": 1}),
    json.dumps({"hardwareId": "d", "type": "DeviceMeasurement", "request": {"name": "t", "value": 1}}).encode(),
    json.dumps({"deviceToken": "d", "type": "DeviceMeasurement"}).encode(),
    b'{"deviceToken": "d", "type": "DeviceMeasurement", "request": {"name": "t", "value": NaN}}',
    b'{"deviceToken": "d\xff", "type": "DeviceMeasurement", "request": {"name": "t", "value": 1}}',
    b'{"deviceToken": "d", "type": "DeviceMeasurement", "request": {"name": "t", "value": 1}} trailing',
]


@pytest.mark.parametrize("j", STAYS)
def test_what_the_engine_cannot_represent_stays_per_event(j):
    assert to_protobuf(j) is None


def test_batch_form_and_fuzzed_inputs():
    good = [c[0] for c in CASES]
    res, st = batch_to_protobuf(good + STAYS)
    assert [r is not None for r in res] == [True] * len(good) + [False] * len(STAYS)
    assert res[:len(good)] == [c[1] for c in CASES]
    rnd = random.Random(5)
    base = good + [_j(f"dev-{i}", "DeviceMeasurement", {"name": f"n{i}", "value": i * 0.25,
                                                         "eventDate": 1_700_000_000_000 + i}) for i in range(20)]
    n_ok = 0
    for k in range(3000):
        b = bytearray(rnd.choice(base))
        for _ in range(rnd.randint(1, 4)):
            op = rnd.random()
            i = rnd.randrange(len(b))
            if op < 0.4:
                b[i] = rnd.randrange(256)
            elif op < 0.7:
                del b[i]
            else:
                b.insert(i, rnd.choice(b'{}[]",:\\0123456789.eE-+ aeflnrstu'))
        out = to_protobuf(bytes(b))
        if out is None:
            continue
        n_ok += 1
        # whatever is transcoded is valid JSON whose request the protobuf form carries exactly
        js = JsonDeviceRequestDecoder().decode(bytes(b), {})[0]
        pr = ProtobufDecoder().decode(out, {})[0]
        assert (js["deviceToken"], js["type"]) == (pr["deviceToken"], pr["type"])
        if js["type"] == "DeviceMeasurement":
            assert pr["request"]["name"] == js["request"]["name"]
            assert pr["request"]["value"] == float(js["request"]["value"])
    assert n_ok > 50
