"""Decoder parity: protobuf runtime encoding -> shared C++/HIP decoder (CPU build here).

Reference: ProtobufDeviceEventDecoder.java:79-281 (delimited Header + body, measurement expansion,
default eventDate = receive time).
"""
import numpy as np

from sitewhere_amd.models import wire
from sitewhere_amd.models.columnar import (EV_ALERT, EV_LOCATION, EV_MEASUREMENT, EV_REGISTRATION, EV_ACK,
                                           EV_DECODE_ERROR, F_HAS_DATE, EVENT_REC)
from sitewhere_amd.pipeline.fleet import (pack_messages, cpu_decode, fingerprint_str, hash64, gen_payloads,
                                          FleetSpec)

NOW = 1_700_000_000_000


def test_record_layout():
    assert EVENT_REC.itemsize == 80
    assert EVENT_REC.fields["etype"][1] == 76


def test_measurements_expand_per_entry():
    p = wire.measurements("dev-1", {"temp": 21.5, "hum": 40.0}, event_date=NOW - 5)
    raw, offs = pack_messages([p])
    r = cpu_decode(raw, offs, NOW)
    assert len(r) == 2
    assert set(r["etype"]) == {EV_MEASUREMENT}
    lo, hi = fingerprint_str("dev-1")
    assert (r["fp_lo"] == lo).all() and (r["fp_hi"] == hi).all()
    assert r[0]["name_hash"] == hash64("temp") and r[0]["v0"] == 21.5
    assert r[1]["name_hash"] == hash64("hum") and r[1]["v0"] == 40.0
    assert (r["event_date"] == NOW - 5).all()
    assert (r["flags"] & F_HAS_DATE).all()
    # aux reference points at the name bytes inside the raw batch
    b = raw.tobytes()
    assert b[r[0]["aux_off"]:r[0]["aux_off"] + r[0]["aux_len"]] == b"temp"


def test_location_alert_and_default_date():
    msgs = [wire.location("d2", 33.7, -84.4, elevation=300.0), wire.alert("d3", "fire", "smoke detected", NOW - 1)]
    raw, offs = pack_messages(msgs)
    r = cpu_decode(raw, offs, NOW)
    assert list(r["etype"]) == [EV_LOCATION, EV_ALERT]
    assert r[0]["v0"] == 33.7 and r[0]["v1"] == -84.4 and r[0]["v2"] == 300.0
    assert r[0]["event_date"] == NOW  # missing eventDate -> receive time
    assert r[1]["name_hash"] == hash64("fire")
    b = raw.tobytes()
    assert b[r[1]["aux2_off"]:r[1]["aux2_off"] + r[1]["aux2_len"]] == b"smoke detected"


def test_control_and_errors():
    msgs = [wire.registration("new-1", "thermostat"), wire.acknowledge("d4", "ok"), b"\x05garbage!!", b""]
    raw, offs = pack_messages(msgs)
    r = cpu_decode(raw, offs, NOW)
    assert list(r["etype"]) == [EV_REGISTRATION, EV_ACK, EV_DECODE_ERROR, EV_DECODE_ERROR]
    assert r[0]["fp_lo"] == fingerprint_str("new-1")[0]
    # control records carry the payload span for the host path
    assert r[0]["aux_off"] == offs[0] and r[0]["aux2_off"] == offs[1]


def test_alternate_id_hashing():
    msgs = [wire.location("d", 1, 2, alternate_id="x1"), wire.location("d", 1, 2, alternate_id="x1"),
            wire.location("d", 1, 2)]
    raw, offs = pack_messages(msgs)
    r = cpu_decode(raw, offs, NOW)
    assert r[0]["alt_hash"] == r[1]["alt_hash"] != 0
    assert r[2]["alt_hash"] == 0


def test_generator_round_trips_through_protobuf_runtime():
    spec = FleetSpec(prefix="g-", n_devices=100, mx_per_msg=2, with_alternate_id=True)
    raw, offs = gen_payloads(spec, 500, NOW, seed=7)
    b = raw.tobytes()
    n_expected = 0
    for i in range(500):
        cmd, _, body = wire.decode(b[offs[i]:offs[i + 1]])
        assert body.hardwareId.startswith("g-")
        n_expected += len(body.measurement) if cmd == wire.SEND_DEVICE_MEASUREMENTS else 1
    r = cpu_decode(raw, offs, NOW)
    assert len(r) == n_expected
    assert (r["etype"] != EV_DECODE_ERROR).all()


def test_threaded_decode_is_deterministic():
    spec = FleetSpec(prefix="t-", n_devices=1000, mx_per_msg=3)
    raw, offs = gen_payloads(spec, 5000, NOW, seed=3)
    a = cpu_decode(raw, offs, NOW, threads=1)
    b = cpu_decode(raw, offs, NOW, threads=8)
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


# ---------------------------------------------------------------- independent oracle (decode_oracle.py)
from decode_oracle import decode, decode_batch, edge_payloads, mutated_payloads, runtime_verdict  # noqa: E402
from decode_oracle import fingerprint as py_fingerprint, hash64 as py_hash64  # noqa: E402


def oracle_batch(seed=11):
    """Generator payloads (alternate ids, control messages, multi-measurement) + edge cases +
    random corruptions, and one payload larger than a workgroup's 32 KB LDS window."""
    spec = FleetSpec(prefix="o-", n_devices=500, mx_per_msg=3, with_alternate_id=True, p_register=0.02,
                     p_ack=0.02)
    raw, offs = gen_payloads(spec, 3000, NOW, seed=seed)
    b = raw.tobytes()
    msgs = [b[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    msgs += edge_payloads(NOW) + mutated_payloads(seed, 3000, NOW)
    msgs.append(wire.measurements("big-1", {f"m{i:05d}": float(i) for i in range(3000)}, alternate_id="big"))
    # strings the durable record keeps: metadata on every event type, updateState, messages
    for i in range(40):
        md = {f"k{j}": f"v{i}-{j}" for j in range(i % 4)}
        msgs.append(wire.alert(f"o-{i}", f"t{i % 3}", f"message {i}", alternate_id=f"al-{i}", metadata=md,
                               update_state=bool(i % 2)))
        msgs.append(wire.location(f"o-{i}", 1.5 + i, 2.5, elevation=None if i % 2 else float(i),
                                  alternate_id=None if i % 3 else f"lo-{i}", metadata=md))
        msgs.append(wire.measurements(f"o-{i}", {"a": i, "b": -i}, alternate_id=f"mx-{i}", metadata=md))
    return pack_messages(msgs)


def test_hashes_match_the_independent_implementation():
    for s in ["", "a", "dev-0000000001", "x" * 300, "ünïcode"]:
        assert fingerprint_str(s) == py_fingerprint(s.encode())
        assert hash64(s) == py_hash64(s.encode())


def test_host_decoder_matches_independent_oracle_bitwise():
    raw, offs = oracle_batch()
    want, why = decode_batch(raw, offs, NOW)
    got = cpu_decode(raw, offs, NOW, cap=len(want) + 16)
    assert len(got) == len(want)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    assert sum(w is not None for w in why) > 1000        # the corruptions do reach the error paths


def test_oracle_agrees_with_the_protobuf_runtime_on_validity():
    """Event payloads are valid exactly when the protobuf runtime parses them with every required
    field (protobuf-java's rule); the one deliberate divergence is refusing groups."""
    for seed in (1, 2):
        for p in edge_payloads(NOW) + mutated_payloads(seed, 2000, NOW):
            cmd, ok = runtime_verdict(p)
            if cmd is not None and cmd not in (3, 4, 5):
                continue                       # control bodies: decoded in full on the host
            recs, why = decode(p, 0, len(p), NOW)
            if ok and why is not None:
                assert why.startswith("group"), (p, why)
            else:
                assert ok == (why is None), (p, why)


def test_oracle_fields_match_the_protobuf_runtime():
    spec = FleetSpec(prefix="f-", n_devices=50, mx_per_msg=2, with_alternate_id=True)
    raw, offs = gen_payloads(spec, 300, NOW, seed=5)
    b = raw.tobytes()
    for i in range(300):
        p = b[offs[i]:offs[i + 1]]
        cmd, _, body = wire.decode(p)
        recs, why = decode(p, 0, len(p), NOW)
        assert why is None
        fp = py_fingerprint(body.hardwareId.encode())
        date = body.eventDate if body.HasField("eventDate") else NOW
        assert all((r["fp_lo"], r["fp_hi"], r["event_date"]) == (*fp, date) for r in recs)
        if cmd == wire.SEND_DEVICE_MEASUREMENTS:
            assert [(r["name_hash"], r["v0"]) for r in recs] == [
                (py_hash64(m.measurementId.encode()), m.measurementValue) for m in body.measurement]
        elif cmd == wire.SEND_DEVICE_LOCATION:
            assert (recs[0]["v0"], recs[0]["v1"]) == (body.latitude, body.longitude)
        else:
            assert recs[0]["name_hash"] == py_hash64(body.alertType.encode())


def test_host_string_refs_match_independent_oracle():
    """Where every record's alternate id and metadata span sit in the batch (the durable record's
    strings), and which measurement of its payload it is: host decoder == oracle, bit for bit."""
    raw, offs = oracle_batch(seed=13)
    want, _, wsp = decode_batch(raw, offs, NOW, spans=True)
    got, gsp = cpu_decode(raw, offs, NOW, cap=len(want) + 16, spans=True)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    assert np.array_equal(gsp.view(np.uint8), wsp.view(np.uint8))
    ev = got["etype"] < 16
    assert (gsp["has"][ev] & 1).sum() > 1000 and (gsp["has"][ev] & 2).sum() > 50 and (gsp["has"][ev] & 4).sum() > 1000
    b = raw.tobytes()
    for i in np.nonzero((gsp["has"] & 1) != 0)[0][:200]:
        o, n = int(gsp["alt_off"][i]), int(gsp["alt_len"][i])
        alt = b[o:o + n] + (b":" + str(int(gsp["k"][i])).encode() if gsp["has"][i] & 4 else b"")
        assert py_hash64(alt) == int(got["alt_hash"][i])


def test_multi_measurement_alternate_ids_hash_like_the_per_event_path():
    """Measurement k of a multi-measurement payload is "<alt>:<k>" on both paths
    (services/event_sources.py names it so), so dedup and the alternate-id index agree."""
    p = wire.measurements("d-1", {"a": 1.0, "b": 2.0, "c": 3.0}, alternate_id="msg-77")
    raw, offs = pack_messages([p])
    recs = cpu_decode(raw, offs, NOW)
    assert [int(h) for h in recs["alt_hash"]] == [hash64(f"msg-77:{k}") for k in range(3)]
    single = cpu_decode(*pack_messages([wire.measurements("d-1", {"a": 1.0}, alternate_id="msg-78")]), NOW)
    assert int(single["alt_hash"][0]) == hash64("msg-78")


def test_oversize_strings_take_the_host_path():
    """An event whose alternate id, alert message or metadata span passes 16-bit lengths is one
    SW_EV_OVERSIZE record (host-routed to the per-event path, stored whole there) -- never truncated."""
    from sitewhere_amd.models.columnar import EV_OVERSIZE
    big = "x" * 70000
    msgs = [wire.alert("d-1", "t", big), wire.measurements("d-2", {"a": 1.0}, alternate_id=big),
            wire.location("d-3", 1.0, 2.0, metadata={"k": big}), wire.measurements("d-4", {big: 1.0}),
            wire.alert("d-5", "t", "fine")]
    raw, offs = pack_messages(msgs)
    recs, sp = cpu_decode(raw, offs, NOW, spans=True)
    want, why, wsp = decode_batch(raw, offs, NOW, spans=True)
    assert np.array_equal(recs.view(np.uint8), want.view(np.uint8))
    assert list(recs["etype"]) == [EV_OVERSIZE] * 4 + [2]
    assert why[:4] == ["oversize"] * 4 and why[4] is None
    assert (recs["fp_lo"][:4] != 0).all()                  # the device is known: routed by its token
