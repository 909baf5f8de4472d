"""Independent decoder of device payloads -> EVENT_REC records (test oracle).

Written from the protobuf wire-format rules and the reference schema
(``sitewhere-communication/src/main/proto/sitewhere.proto``), in plain Python, sharing no code with
``csrc/include/swdecode.h`` (which both the host engine and the gfx950 kernels compile): varints,
tags, fingerprints and string hashes are re-implemented here.  The validity rules are the ones
protobuf-java's ``parseDelimitedFrom`` applies in ``ProtobufDeviceEventDecoder.java:79-95``:

* a payload is a delimited ``SiteWhere.Header`` then a delimited body; bytes after the body are
  ignored;
* a malformed tag or field, field number 0, or a tag key past 32 bits is a decode error;
* the header's ``required Command command`` must carry a known value (an unknown enum value is an
  unknown field in proto2, so a later unknown value does not override an earlier known one);
* event bodies (location, alert, measurements) must hold every ``required`` field, including those
  of each embedded ``Measurement`` / ``Metadata``; control bodies need their ``hardwareId`` (the
  host decodes those payloads in full);
* deprecated groups (wire types 3/4, unused by the schema) are refused -- the one place the device
  decoder is stricter than protobuf-java.

``decode(payload, start, now_ms)`` returns ``(records, reason)``: a list of dicts with the
EVENT_REC fields and ``None`` or the reason the payload is a decode error.
"""
from __future__ import annotations

import struct

import numpy as np

from sitewhere_amd.models.columnar import (EVENT_REC, EV_ACK, EV_ALERT, EV_DECODE_ERROR, EV_LOCATION,
                                           EV_MEASUREMENT, EV_REGISTRATION)

M64 = (1 << 64) - 1
FNV_OFFSET, FNV_PRIME = 0xcbf29ce484222325, 0x100000001b3
POLY_SEED, POLY_MUL = 0x9e3779b97f4a7c15, 0xff51afd7ed558ccd
EV_STREAM_CREATE, EV_STREAM_DATA, EV_STREAM_DATA_REQUEST = 18, 19, 20
F_HAS_UPDATE_STATE, F_UPDATE_STATE, F_HAS_DATE, F_HAS_ELEVATION = 1, 2, 4, 8
EV_OVERSIZE = 21
SR_ALT, SR_META, SR_MULTI = 1, 2, 4
U16 = 0xFFFF
CONTROL_TYPE = {1: EV_REGISTRATION, 2: EV_ACK, 6: EV_STREAM_CREATE, 7: EV_STREAM_DATA, 8: EV_STREAM_DATA_REQUEST}


def mix64(x: int) -> int:
    x &= M64
    x ^= x >> 30
    x = (x * 0xbf58476d1ce4e5b9) & M64
    x ^= x >> 27
    x = (x * 0x94d049bb133111eb) & M64
    return x ^ (x >> 31)


def fingerprint(b: bytes) -> tuple[int, int]:
    a, h = FNV_OFFSET, POLY_SEED ^ len(b)
    for c in b:
        a = ((a ^ c) * FNV_PRIME) & M64
        h = ((h + c + 1) * POLY_MUL) & M64
    a, h = mix64(a), mix64(h ^ (h >> 29))
    return (1 if a == 0 and h == 0 else a), h


def hash64(b: bytes) -> int:
    a = FNV_OFFSET
    for c in b:
        a = ((a ^ c) * FNV_PRIME) & M64
    a = mix64(a ^ ((len(b) << 56) & M64))
    return a or 1


class Bad(Exception):
    pass


def _varint(b: bytes, p: int, e: int) -> tuple[int, int]:
    v = shift = 0
    while p < e and shift < 64:
        c = b[p]
        p += 1
        v |= (c & 0x7f) << shift
        if not c & 0x80:
            return v & M64, p
        shift += 7
    raise Bad("truncated or overlong varint")


def _fields(b: bytes, p: int, e: int, tags: bool = False):
    """Yield (field, wire type, value, value start, next position) over [p, e); ``tags``: the field's
    tag position as a sixth element."""
    while p < e:
        t0 = p
        key, p = _varint(b, p, e)
        if key > 0xffffffff or key >> 3 == 0:
            raise Bad("invalid tag")
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, q = _varint(b, p, e)
            yield (f, wt, v, p, q, t0) if tags else (f, wt, v, p, q)
        elif wt == 1 or wt == 5:
            n = 8 if wt == 1 else 4
            if p + n > e:
                raise Bad("truncated fixed field")
            yield (f, wt, b[p:p + n], p, p + n, t0) if tags else (f, wt, b[p:p + n], p, p + n)
        elif wt == 2:
            n, s = _varint(b, p, e)
            if n > e - s:
                raise Bad("length past the end")
            yield (f, wt, b[s:s + n], s, s + n, t0) if tags else (f, wt, b[s:s + n], s, s + n)
        else:
            raise Bad("group or invalid wire type")
        p = q if wt == 0 else (p + n if wt in (1, 5) else s + n)


def _pair(b: bytes, s: int, e: int, wt2: int):
    """Embedded {required string 1; required <wt2> 2}; returns (name start, name len, field 2)."""
    name, val = None, None
    for f, wt, v, vs, _ in _fields(b, s, e):
        if f == 1 and wt == 2:
            name = (vs, len(v))
        elif f == 2 and wt == wt2:
            val = v
    if name is None or val is None:
        raise Bad("embedded message misses a required field")
    return name, val


def _f64(raw: bytes) -> float:
    return struct.unpack("<d", raw)[0]


def decode(b: bytes, start: int, end: int, now_ms: int, rank: int = 0):
    """Decode payload b[start:end] (offsets in the records are absolute positions in b)."""
    def err(reason):
        return [dict(fp_lo=0, fp_hi=0, event_date=now_ms, name_hash=0, v0=0.0, v1=0.0, v2=0.0, alt_hash=0,
                     aux_off=start, aux2_off=end, aux_len=0, aux2_len=0, etype=EV_DECODE_ERROR, flags=0,
                     src_rank=rank, level=0)], reason
    try:
        hlen, p = _varint(b, start, end)
        if hlen > end - p:
            raise Bad("header past the end")
        cmd = 0
        for f, wt, v, _, _ in _fields(b, p, p + hlen):
            if f == 1 and wt == 0 and 1 <= v <= 8:
                cmd = v
        blen, bs = _varint(b, p + hlen, end)
        if blen > end - bs:
            raise Bad("body past the end")
        if cmd == 0:
            raise Bad("no known command")
        be = bs + blen
        hw = alt = date = None
        us = None
        entries, lat, lon, elev = [], None, None, None
        atype = amsg = None
        meta_f = {5: 4, 3: 6, 4: 5}.get(cmd)
        md = None                                   # [first entry's tag, last entry's end)
        for f, wt, v, vs, fe, t0 in _fields(b, bs, be, tags=True):
            if f == 1 and wt == 2:
                hw = v
            elif f == 15 and wt == 2 and cmd in (3, 4, 5):
                alt = (vs, len(v))
            elif f == meta_f and wt == 2:
                _pair(b, vs, vs + len(v), 2)
                md = (md[0] if md else t0, fe)
            elif cmd == 5:
                if f == 2 and wt == 2:
                    entries.append(_pair(b, vs, vs + len(v), 1))
                elif f == 3 and wt == 1:
                    date = struct.unpack("<q", v)[0]
                elif f == 5 and wt == 0:
                    us = v != 0
            elif cmd == 3:
                if wt == 1 and f in (2, 3, 4):
                    lat, lon, elev = ((_f64(v), lon, elev) if f == 2 else (lat, _f64(v), elev) if f == 3
                                      else (lat, lon, _f64(v)))
                elif f == 5 and wt == 1:
                    date = struct.unpack("<q", v)[0]
                elif f == 7 and wt == 0:
                    us = v != 0
            elif cmd == 4:
                if f == 2 and wt == 2:
                    atype = (vs, len(v))
                elif f == 3 and wt == 2:
                    amsg = (vs, len(v))
                elif f == 4 and wt == 1:
                    date = struct.unpack("<q", v)[0]
                elif f == 6 and wt == 0:
                    us = v != 0
        if cmd == 3 and (lat is None or lon is None):
            raise Bad("location misses latitude/longitude")
        if cmd == 4 and (atype is None or amsg is None):
            raise Bad("alert misses alertType/alertMessage")
        if hw is None:
            raise Bad("no hardwareId")
    except Bad as e:
        return err(str(e))
    lo, hi = fingerprint(hw)
    if cmd in (3, 4, 5):
        # strings past 16-bit lengths: one oversize record, the host routes the payload
        lens = [alt[1] if alt else 0, (md[1] - md[0]) if md else 0]
        lens += [atype[1], amsg[1]] if cmd == 4 else []
        lens += [nl for (_, nl), _ in entries] if cmd == 5 else []
        if max(lens) > U16:
            return [dict(fp_lo=lo, fp_hi=hi, event_date=now_ms, name_hash=0, v0=0.0, v1=0.0, v2=0.0, alt_hash=0,
                         aux_off=start, aux2_off=end, aux_len=0, aux2_len=0, etype=EV_OVERSIZE, flags=0,
                         src_rank=rank, level=0)], "oversize"
    flags = ((F_HAS_UPDATE_STATE if us is not None else 0) | (F_UPDATE_STATE if us else 0) |
             (F_HAS_DATE if date is not None else 0) | (F_HAS_ELEVATION if elev is not None else 0))
    edate = date if date is not None else now_ms
    base = dict(fp_lo=lo, fp_hi=hi, event_date=edate, v0=0.0, v1=0.0, v2=0.0, aux2_off=0, aux2_len=0,
                flags=flags, src_rank=rank, level=0)
    abytes = b[alt[0]:alt[0] + alt[1]] if alt else None
    span = dict(alt_off=alt[0] if alt else start, alt_len=alt[1] if alt else 0,
                meta_off=md[0] if md else start, meta_len=(md[1] - md[0]) if md else 0, k=0,
                has=(SR_ALT if alt else 0) | (SR_META if md else 0))
    if cmd == 5:
        recs = []
        multi = len(entries) > 1
        for k, ((ns, nl), val) in enumerate(entries):
            # measurement k of a multi-measurement payload: alternate id "<alt>:<k>"
            ah = 0 if abytes is None else hash64(abytes + b":" + str(k).encode()) if multi else hash64(abytes)
            recs.append(dict(base, name_hash=hash64(b[ns:ns + nl]) if nl else 0, v0=_f64(val),
                             alt_hash=ah, aux_off=ns, aux_len=nl, etype=EV_MEASUREMENT,
                             _span=dict(span, k=k, has=span["has"] | (SR_MULTI if multi else 0))))
        return recs, None
    ah = hash64(abytes) if abytes is not None else 0
    if cmd == 3:
        return [dict(base, name_hash=0, v0=lat, v1=lon, v2=elev if elev is not None else 0.0, alt_hash=ah,
                     aux_off=start, aux_len=0, etype=EV_LOCATION, _span=span)], None
    if cmd == 4:
        (ts, tl), (ms, ml) = atype, amsg
        return [dict(base, name_hash=hash64(b[ts:ts + tl]) if tl else 0, alt_hash=ah,
                     aux_off=ts, aux_len=tl, aux2_off=ms, aux2_len=ml, etype=EV_ALERT, _span=span)], None
    return [dict(fp_lo=lo, fp_hi=hi, event_date=now_ms, name_hash=0, v0=0.0, v1=0.0, v2=0.0, alt_hash=0,
                 aux_off=start, aux2_off=end, aux_len=0, aux2_len=0, etype=CONTROL_TYPE[cmd], flags=0,
                 src_rank=rank, level=0)], None


def decode_batch(raw: np.ndarray, offs: np.ndarray, now_ms: int, rank: int = 0, spans: bool = False):
    """Oracle records of a packed batch as an EVENT_REC array, plus the per-payload reasons (and,
    with ``spans``, the STR_REF string refs of every record: zero for records without strings)."""
    from sitewhere_amd.models.columnar import STR_REF
    b = raw.tobytes()
    rows, reasons = [], []
    for i in range(len(offs) - 1):
        r, why = decode(b, int(offs[i]), int(offs[i + 1]), now_ms, rank)
        rows.extend(r)
        reasons.append(why)
    out = np.zeros(len(rows), EVENT_REC)
    sp = np.zeros(len(rows), STR_REF)
    for i, r in enumerate(rows):
        for k, v in r.items():
            if k == "_span":
                for k2, v2 in v.items():
                    sp[i][k2] = v2
            else:
                out[i][k] = v
    return (out, reasons, sp) if spans else (out, reasons)


# ------------------------------------------------------------------ malformed / edge-case batches
def _tag(f: int, wt: int) -> bytes:
    return _venc((f << 3) | wt)


def _venc(v: int) -> bytes:
    out = bytearray()
    while True:
        c = v & 0x7f
        v >>= 7
        out.append(c | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _delim(b: bytes) -> bytes:
    return _venc(len(b)) + b


def _s(f: int, s: bytes) -> bytes:
    return _tag(f, 2) + _delim(s)


def _d(f: int, x: float) -> bytes:
    return _tag(f, 1) + struct.pack("<d", x)


def _hdr(cmd: int, *extra: bytes) -> bytes:
    return _delim(_tag(1, 0) + _venc(cmd) + b"".join(extra))


def edge_payloads(now_ms: int) -> list[bytes]:
    """Hand-built payloads on the edges of the validity rules (each named by what it tests)."""
    from sitewhere_amd.models import wire
    m_ok = _s(1, b"temp") + _d(2, 1.5)
    md_ok = _s(1, b"k") + _s(2, b"v")
    loc = _s(1, b"d-1") + _d(2, 1.0) + _d(3, 2.0)
    return [
        wire.measurements("d-1", {"a": 1.0, "b": -0.0}, event_date=now_ms - 7, alternate_id="x",
                          metadata={"k": "v"}, update_state=True),
        wire.location("d-2", 33.7, -84.4, elevation=-0.0, alternate_id="y"),
        wire.alert("d-3", "", "", event_date=(1 << 64) - 5),                         # empty strings, negative date
        _hdr(5) + _delim(_s(1, b"d-1") + _s(2, m_ok) + _s(2, _s(1, b"x"))),          # entry misses its value
        _hdr(5) + _delim(_s(1, b"d-1") + _s(2, _d(2, 3.0))),                         # entry misses its id
        _hdr(5) + _delim(_s(1, b"d-1") + _s(2, m_ok) + _s(4, _s(1, b"k"))),          # metadata misses value
        _hdr(5) + _delim(_s(1, b"d-1") + _s(2, m_ok) + _s(4, md_ok)),                # metadata complete
        _hdr(5) + _delim(_s(1, b"d-1")),                                             # no entries: 0 records
        _hdr(5) + _delim(_s(2, m_ok)),                                               # no hardwareId
        _hdr(3) + _delim(_s(1, b"d-1") + _d(2, 1.0)),                                # location misses longitude
        _hdr(3) + _delim(loc + _s(6, md_ok) + _tag(7, 0) + b"\x00"),                  # updateState false
        _hdr(3) + _delim(loc + _tag(2, 0) + b"\x05"),                                # latitude with a wrong wire type
        _hdr(4) + _delim(_s(1, b"d-1") + _s(2, b"t")),                               # alert misses its message
        _hdr(9) + _delim(loc),                                                       # unknown command
        _hdr(3, _tag(1, 0) + _venc(99)) + _delim(loc),                               # known then unknown command
        _hdr(99, _tag(1, 0) + _venc(3)) + _delim(loc),                               # unknown then known command
        _delim(_s(2, b"orig")) + _delim(loc),                                        # header without a command
        _hdr(3) + _delim(loc + _tag(0, 0) + b"\x01"),                                # field number 0
        _hdr(3) + _delim(loc + _tag(9, 3) + _tag(9, 4)),                             # a group
        _hdr(3) + _delim(loc + _tag(9, 6)),                                          # invalid wire type
        _hdr(3) + _delim(loc + _tag(9, 5) + b"\x00\x00\x00\x00"),                    # fixed32 unknown field
        _hdr(3) + _delim(loc) + b"trailing bytes",                                   # bytes after the body
        _hdr(3) + _delim(loc)[:-3],                                                  # truncated body
        _hdr(3) + _venc(1 << 40),                                                    # body length past the end
        _hdr(3) + b"\xff" * 11,                                                      # overlong varint
        _hdr(3) + _delim(loc + _venc(1 << 36) + b"\x00"),                            # tag key past 32 bits
        b"",
        b"\x00\x00",                                                                 # empty header and body
        _hdr(1) + _delim(_s(1, b"new-1") + _s(2, b"type")),                         # registration
        _hdr(2) + _delim(_s(2, b"no id")),                                          # ack without hardwareId
        _hdr(8) + _delim(_s(1, b"d-9") + _s(2, b"s") + _tag(3, 1) + b"\x01" * 8),   # stream data request
    ]


def mutated_payloads(seed: int, n: int, now_ms: int) -> list[bytes]:
    """Random corruptions of valid payloads: truncation, byte flips, insertions, splices."""
    import random
    from sitewhere_amd.models import wire
    rnd = random.Random(seed)
    base = [wire.measurements("m-1", {"t": 1.0, "h": 2.0}, event_date=now_ms, alternate_id="a1", metadata={"k": "v"}),
            wire.location("l-1", 1.0, 2.0, elevation=3.0, event_date=now_ms, alternate_id="a2"),
            wire.alert("a-1", "fire", "smoke"),
            wire.registration("r-1", "type"), wire.acknowledge("k-1", "ok")]
    out = []
    for _ in range(n):
        p = bytearray(rnd.choice(base))
        op = rnd.randrange(5)
        if op == 0 and p:
            del p[rnd.randrange(len(p)):]
        elif op == 1 and p:
            for _ in range(rnd.randint(1, 3)):
                p[rnd.randrange(len(p))] ^= 1 << rnd.randrange(8)
        elif op == 2:
            i = rnd.randrange(len(p) + 1)
            p[i:i] = bytes(rnd.randrange(256) for _ in range(rnd.randint(1, 4)))
        elif op == 3 and p:
            i = rnd.randrange(len(p))
            p[i] = rnd.randrange(256)
        else:
            p = bytearray(rnd.randrange(256) for _ in range(rnd.randint(0, 40)))
        out.append(bytes(p))
    return out


def runtime_verdict(payload: bytes):
    """The protobuf runtime's view of one payload (python upb, reference schema, required fields
    checked the way protobuf-java checks them): ``(command or None if the header is invalid, valid)``."""
    from google.protobuf.message import DecodeError
    from sitewhere_amd.models import wire
    try:
        hlen, p = _varint(payload, 0, len(payload))
        if hlen > len(payload) - p:
            return None, False
        h = wire.Header()
        h.ParseFromString(payload[p:p + hlen])
        blen, bs = _varint(payload, p + hlen, len(payload))
        if blen > len(payload) - bs or not h.IsInitialized():
            return None, False
    except (Bad, DecodeError):
        return None, False
    try:
        body = wire._BODY[h.command]()
        body.ParseFromString(payload[bs:bs + blen])
        return h.command, body.IsInitialized()
    except DecodeError:
        return h.command, False
