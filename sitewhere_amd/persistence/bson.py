"""BSON (bsonspec.org 1.1) encoder / decoder for the MongoDB wire protocol (``mongo_wire.py``).

Python <-> BSON: float <-> double, str <-> string, dict <-> document (order kept), list/tuple ->
array, bytes <-> binary (subtype 0), :class:`ObjectId`, bool, ``datetime`` <-> UTC datetime,
None <-> null, int -> int32 when it fits else int64 (:class:`Int64` forces int64), int32/int64 ->
int, Timestamp -> (t, i) tuple, Decimal128 -> its 16 raw bytes.
"""
from __future__ import annotations

import datetime as _dt
import os
import struct
import threading
import time

_I32, _I64, _U64, _DBL = struct.Struct("<i"), struct.Struct("<q"), struct.Struct("<Q"), struct.Struct("<d")
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


class Int64(int):
    """An int that always encodes as BSON int64."""


class ObjectId:
    _lock = threading.Lock()
    _inc = int.from_bytes(os.urandom(3), "big")
    _rand = os.urandom(5)

    def __init__(self, oid: bytes | str | None = None):
        if oid is None:
            with ObjectId._lock:
                ObjectId._inc = (ObjectId._inc + 1) & 0xFFFFFF
                inc = ObjectId._inc
            oid = struct.pack(">I", int(time.time())) + ObjectId._rand + inc.to_bytes(3, "big")
        elif isinstance(oid, str):
            oid = bytes.fromhex(oid)
        if len(oid) != 12:
            raise ValueError("ObjectId is 12 bytes")
        self.binary = bytes(oid)

    def __eq__(self, o):
        return isinstance(o, ObjectId) and o.binary == self.binary

    def __hash__(self):
        return hash(self.binary)

    def __repr__(self):
        return f"ObjectId('{self.binary.hex()}')"

    def __str__(self):
        return self.binary.hex()


def _cstring(s: str) -> bytes:
    b = s.encode()
    if b"\0" in b:
        raise ValueError("BSON keys cannot contain NUL")
    return b + b"\0"


def _element(key: str, v, out: bytearray):
    k = _cstring(key)
    if isinstance(v, bool):
        out += b"\x08" + k + (b"\x01" if v else b"\x00")
    elif isinstance(v, Int64):
        out += b"\x12" + k + _I64.pack(v)
    elif isinstance(v, int):
        if -(1 << 31) <= v < (1 << 31):
            out += b"\x10" + k + _I32.pack(v)
        else:
            out += b"\x12" + k + _I64.pack(v)
    elif isinstance(v, float):
        out += b"\x01" + k + _DBL.pack(v)
    elif isinstance(v, str):
        b = v.encode()
        out += b"\x02" + k + _I32.pack(len(b) + 1) + b + b"\0"
    elif isinstance(v, dict):
        out += b"\x03" + k + encode(v)
    elif isinstance(v, (list, tuple)):
        out += b"\x04" + k + encode({str(i): x for i, x in enumerate(v)})
    elif isinstance(v, (bytes, bytearray, memoryview)):
        b = bytes(v)
        out += b"\x05" + k + _I32.pack(len(b)) + b"\x00" + b
    elif isinstance(v, ObjectId):
        out += b"\x07" + k + v.binary
    elif isinstance(v, _dt.datetime):
        if v.tzinfo is None:
            v = v.replace(tzinfo=_dt.timezone.utc)
        out += b"\x09" + k + _I64.pack(int((v - _EPOCH).total_seconds() * 1000))
    elif v is None:
        out += b"\x0a" + k
    else:
        raise TypeError(f"cannot encode {type(v).__name__} as BSON")


def encode(doc: dict) -> bytes:
    out = bytearray(4)
    for k, v in doc.items():
        _element(str(k), v, out)
    out += b"\0"
    out[0:4] = _I32.pack(len(out))
    return bytes(out)


def _read_cstring(buf, pos):
    end = buf.index(0, pos)
    return buf[pos:end].decode(), end + 1


def _decode_doc(buf, pos, as_list=False):
    (n,) = _I32.unpack_from(buf, pos)
    end = pos + n - 1
    pos += 4
    out = [] if as_list else {}
    while pos < end:
        t = buf[pos]
        key, pos = _read_cstring(buf, pos + 1)
        if t == 0x01:
            (v,) = _DBL.unpack_from(buf, pos)
            pos += 8
        elif t == 0x02:
            (ln,) = _I32.unpack_from(buf, pos)
            v = buf[pos + 4:pos + 3 + ln].decode()
            pos += 4 + ln
        elif t in (0x03, 0x04):
            v, pos = _decode_doc(buf, pos, t == 0x04)
        elif t == 0x05:
            (ln,) = _I32.unpack_from(buf, pos)
            v = bytes(buf[pos + 5:pos + 5 + ln])
            pos += 5 + ln
        elif t == 0x07:
            v = ObjectId(bytes(buf[pos:pos + 12]))
            pos += 12
        elif t == 0x08:
            v = buf[pos] == 1
            pos += 1
        elif t == 0x09:
            (ms,) = _I64.unpack_from(buf, pos)
            v = _EPOCH + _dt.timedelta(milliseconds=ms)
            pos += 8
        elif t in (0x0a, 0x06):
            v = None
        elif t == 0x10:
            (v,) = _I32.unpack_from(buf, pos)
            pos += 4
        elif t == 0x11:
            (u,) = _U64.unpack_from(buf, pos)
            v = (u >> 32, u & 0xFFFFFFFF)
            pos += 8
        elif t == 0x12:
            (v,) = _I64.unpack_from(buf, pos)
            pos += 8
        elif t == 0x13:
            v = bytes(buf[pos:pos + 16])
            pos += 16
        elif t in (0x7f, 0xff):
            v = None
        else:
            raise ValueError(f"unsupported BSON type 0x{t:02x}")
        if as_list:
            out.append(v)
        else:
            out[key] = v
    return out, end + 1


def decode(buf, pos: int = 0) -> dict:
    return _decode_doc(buf if isinstance(buf, bytes) else bytes(buf), pos)[0]


def decode_with_end(buf, pos: int = 0) -> tuple[dict, int]:
    return _decode_doc(buf if isinstance(buf, bytes) else bytes(buf), pos)
