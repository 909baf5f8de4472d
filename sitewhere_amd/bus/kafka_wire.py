"""Apache Kafka wire protocol: framing, message schemas and RecordBatch v2.

The reference's data plane *is* Kafka (``MicroserviceKafkaConsumer`` / ``MicroserviceKafkaProducer``,
kafka-clients 0.11).  This module lets the rebuilt bus speak the same protocol in
both directions:

* :mod:`.kafka_broker` serves the native commit log to any Kafka client (the reference's Java
  services, device gateways, Kafka tooling);
* :mod:`.kafka_client` runs our microservices on a real Kafka cluster (``KafkaEventBus``) and reads
  Azure Event Hubs through its Kafka endpoint (SASL PLAIN over TLS).

Only non-flexible API versions are used (no tagged fields), one per API, chosen so that clients from
Kafka 0.11 onwards can negotiate them through ApiVersions:

=============== === ========  =============== === ========
API             key version   API             key version
=============== === ========  =============== === ========
Produce          0     3      JoinGroup        11    1
Fetch            1     4      Heartbeat        12    0
ListOffsets      2     1      LeaveGroup       13    0
Metadata         3     1      SyncGroup        14    0
OffsetCommit     8     2      SaslHandshake    17    1
OffsetFetch      9     1      ApiVersions      18    0
FindCoordinator 10     0      SaslAuthenticate 36    0
=============== === ========  =============== === ========

Records travel as RecordBatch v2 (magic 2, CRC-32C, zig-zag varints); gzip batches are read,
other codecs are refused with UNSUPPORTED_COMPRESSION_TYPE.
"""
from __future__ import annotations

import struct
import zlib

from .._native import native

# ---------------------------------------------------------------------------------- API keys
PRODUCE, FETCH, LIST_OFFSETS, METADATA = 0, 1, 2, 3
OFFSET_COMMIT, OFFSET_FETCH, FIND_COORDINATOR = 8, 9, 10
JOIN_GROUP, HEARTBEAT, LEAVE_GROUP, SYNC_GROUP = 11, 12, 13, 14
SASL_HANDSHAKE, API_VERSIONS, SASL_AUTHENTICATE = 17, 18, 36

# api key -> the one version this implementation speaks
VERSIONS = {PRODUCE: 3, FETCH: 4, LIST_OFFSETS: 1, METADATA: 1, OFFSET_COMMIT: 2, OFFSET_FETCH: 1,
            FIND_COORDINATOR: 0, JOIN_GROUP: 1, HEARTBEAT: 0, LEAVE_GROUP: 0, SYNC_GROUP: 0,
            SASL_HANDSHAKE: 1, API_VERSIONS: 0, SASL_AUTHENTICATE: 0}

# ---------------------------------------------------------------------------------- error codes
NONE = 0
OFFSET_OUT_OF_RANGE = 1
CORRUPT_MESSAGE = 2
UNKNOWN_TOPIC_OR_PARTITION = 3
ILLEGAL_GENERATION = 22
INCONSISTENT_GROUP_PROTOCOL = 23
UNKNOWN_MEMBER_ID = 25
REBALANCE_IN_PROGRESS = 27
UNSUPPORTED_SASL_MECHANISM = 33
ILLEGAL_SASL_STATE = 34
UNSUPPORTED_VERSION = 35
SASL_AUTHENTICATION_FAILED = 58
UNSUPPORTED_COMPRESSION_TYPE = 76


class KafkaError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        super().__init__(f"kafka error {code}{': ' + what if what else ''}")
        self.code = code


# ---------------------------------------------------------------------------------- schemas
# A schema is a list of (field, type); type is a primitive name or ("array", schema | primitive),
# ("narray", ...) for a nullable array.
S, NS, B, NB = "string", "nstring", "bytes", "nbytes"
I8, I16, I32, I64, BOOL = "int8", "int16", "int32", "int64", "bool"


def arr(t):
    return ("array", t)


REQUEST = {
    API_VERSIONS: [],
    METADATA: [("topics", ("narray", S))],
    PRODUCE: [("transactional_id", NS), ("acks", I16), ("timeout_ms", I32),
              ("topics", arr([("name", S), ("partitions", arr([("index", I32), ("records", NB)]))]))],
    FETCH: [("replica_id", I32), ("max_wait_ms", I32), ("min_bytes", I32), ("max_bytes", I32),
            ("isolation_level", I8),
            ("topics", arr([("topic", S), ("partitions", arr([("partition", I32), ("fetch_offset", I64),
                                                            ("partition_max_bytes", I32)]))]))],
    LIST_OFFSETS: [("replica_id", I32),
                   ("topics", arr([("name", S), ("partitions", arr([("partition_index", I32), ("timestamp", I64)]))]))],
    FIND_COORDINATOR: [("key", S)],
    JOIN_GROUP: [("group_id", S), ("session_timeout_ms", I32), ("rebalance_timeout_ms", I32), ("member_id", S),
                 ("protocol_type", S), ("protocols", arr([("name", S), ("metadata", B)]))],
    SYNC_GROUP: [("group_id", S), ("generation_id", I32), ("member_id", S),
                 ("assignments", arr([("member_id", S), ("assignment", B)]))],
    HEARTBEAT: [("group_id", S), ("generation_id", I32), ("member_id", S)],
    LEAVE_GROUP: [("group_id", S), ("member_id", S)],
    OFFSET_COMMIT: [("group_id", S), ("generation_id", I32), ("member_id", S), ("retention_time_ms", I64),
                    ("topics", arr([("name", S), ("partitions", arr([("partition_index", I32),
                                                                     ("committed_offset", I64),
                                                                     ("committed_metadata", NS)]))]))],
    OFFSET_FETCH: [("group_id", S), ("topics", ("narray", [("name", S), ("partition_indexes", arr(I32))]))],
    SASL_HANDSHAKE: [("mechanism", S)],
    SASL_AUTHENTICATE: [("auth_bytes", B)],
}

RESPONSE = {
    API_VERSIONS: [("error_code", I16), ("api_keys", arr([("api_key", I16), ("min_version", I16),
                                                           ("max_version", I16)]))],
    METADATA: [("brokers", arr([("node_id", I32), ("host", S), ("port", I32), ("rack", NS)])),
               ("controller_id", I32),
               ("topics", arr([("error_code", I16), ("name", S), ("is_internal", BOOL),
                               ("partitions", arr([("error_code", I16), ("partition_index", I32), ("leader_id", I32),
                                                   ("replica_nodes", arr(I32)), ("isr_nodes", arr(I32))]))]))],
    PRODUCE: [("responses", arr([("name", S), ("partitions", arr([("index", I32), ("error_code", I16),
                                                                  ("base_offset", I64),
                                                                  ("log_append_time_ms", I64)]))])),
              ("throttle_time_ms", I32)],
    FETCH: [("throttle_time_ms", I32),
            ("responses", arr([("topic", S), ("partitions", arr([
                ("partition_index", I32), ("error_code", I16), ("high_watermark", I64), ("last_stable_offset", I64),
                ("aborted_transactions", ("narray", [("producer_id", I64), ("first_offset", I64)])),
                ("records", NB)]))]))],
    LIST_OFFSETS: [("topics", arr([("name", S), ("partitions", arr([("partition_index", I32), ("error_code", I16),
                                                                     ("timestamp", I64), ("offset", I64)]))]))],
    FIND_COORDINATOR: [("error_code", I16), ("node_id", I32), ("host", S), ("port", I32)],
    JOIN_GROUP: [("error_code", I16), ("generation_id", I32), ("protocol_name", S), ("leader", S),
                 ("member_id", S), ("members", arr([("member_id", S), ("metadata", B)]))],
    SYNC_GROUP: [("error_code", I16), ("assignment", B)],
    HEARTBEAT: [("error_code", I16)],
    LEAVE_GROUP: [("error_code", I16)],
    OFFSET_COMMIT: [("topics", arr([("name", S), ("partitions", arr([("partition_index", I32),
                                                                     ("error_code", I16)]))]))],
    OFFSET_FETCH: [("topics", arr([("name", S), ("partitions", arr([("partition_index", I32),
                                                                     ("committed_offset", I64), ("metadata", NS),
                                                                     ("error_code", I16)]))]))],
    SASL_HANDSHAKE: [("error_code", I16), ("mechanisms", arr(S))],
    SASL_AUTHENTICATE: [("error_code", I16), ("error_message", NS), ("auth_bytes", B)],
}

# consumer protocol payloads (JoinGroup metadata / SyncGroup assignment, protocol type "consumer")
SUBSCRIPTION = [("version", I16), ("topics", arr(S)), ("user_data", NB)]
ASSIGNMENT = [("version", I16), ("partitions", arr([("topic", S), ("partitions", arr(I32))])), ("user_data", NB)]

_FMT = {I8: struct.Struct(">b"), I16: struct.Struct(">h"), I32: struct.Struct(">i"), I64: struct.Struct(">q")}


def _enc(t, v, out: list):
    if isinstance(t, tuple):
        kind, sub = t
        if v is None:
            if kind != "narray":
                raise ValueError("null for a non-nullable array")
            out.append(_FMT[I32].pack(-1))
            return
        out.append(_FMT[I32].pack(len(v)))
        for x in v:
            _enc(sub, x, out)
    elif isinstance(t, list):
        for name, ft in t:
            _enc(ft, v[name], out)
    elif t in _FMT:
        out.append(_FMT[t].pack(int(v)))
    elif t == BOOL:
        out.append(b"\x01" if v else b"\x00")
    elif t in (S, NS):
        if v is None:
            if t == S:
                raise ValueError("null for a non-nullable string")
            out.append(_FMT[I16].pack(-1))
        else:
            b = v.encode() if isinstance(v, str) else bytes(v)
            out.append(_FMT[I16].pack(len(b)))
            out.append(b)
    elif t in (B, NB):
        if v is None:
            if t == B:
                raise ValueError("null for non-nullable bytes")
            out.append(_FMT[I32].pack(-1))
        else:
            out.append(_FMT[I32].pack(len(v)))
            out.append(v)
    else:
        raise ValueError(f"unknown type {t!r}")


def encode(schema, value: dict) -> bytes:
    out: list = []
    _enc(schema, value, out)
    return b"".join(out)


class Reader:
    def __init__(self, buf, pos: int = 0):
        self.buf, self.pos = memoryview(buf), pos

    def take(self, n: int):
        if self.pos + n > len(self.buf):
            raise KafkaError(CORRUPT_MESSAGE, "truncated message")
        v = self.buf[self.pos:self.pos + n]
        self.pos += n
        return v

    def prim(self, t):
        f = _FMT[t]
        if self.pos + f.size > len(self.buf):
            raise KafkaError(CORRUPT_MESSAGE, "truncated message")
        (v,) = f.unpack_from(self.buf, self.pos)
        self.pos += f.size
        return v

    def read(self, t):
        if isinstance(t, tuple):
            kind, sub = t
            n = self.prim(I32)
            if n < 0:
                return None if kind == "narray" else []
            return [self.read(sub) for _ in range(n)]
        if isinstance(t, list):
            return {name: self.read(ft) for name, ft in t}
        if t in _FMT:
            return self.prim(t)
        if t == BOOL:
            return bool(self.take(1)[0])
        if t in (S, NS):
            n = self.prim(I16)
            return None if n < 0 else bytes(self.take(n)).decode()
        if t in (B, NB):
            n = self.prim(I32)
            return None if n < 0 else bytes(self.take(n))
        raise ValueError(f"unknown type {t!r}")


def decode(schema, buf, pos: int = 0) -> dict:
    return Reader(buf, pos).read(schema)


# ---------------------------------------------------------------------------------- framing
_SIZE = struct.Struct(">i")
_REQ_HDR = struct.Struct(">hhi")


def request_frame(api_key: int, version: int, correlation_id: int, client_id: str | None, body: bytes) -> bytes:
    cid = client_id.encode() if client_id is not None else None
    hdr = _REQ_HDR.pack(api_key, version, correlation_id) + (
        _FMT[I16].pack(-1) if cid is None else _FMT[I16].pack(len(cid)) + cid)
    return _SIZE.pack(len(hdr) + len(body)) + hdr + body


def parse_request_header(msg) -> tuple[int, int, int, str | None, int]:
    """-> (api_key, version, correlation_id, client_id, body offset) of a request (size prefix removed)."""
    api_key, version, corr = _REQ_HDR.unpack_from(msg, 0)
    (n,) = _FMT[I16].unpack_from(msg, 8)
    cid = None if n < 0 else bytes(msg[10:10 + n]).decode(errors="replace")
    return api_key, version, corr, cid, 10 + max(n, 0)


def response_frame(correlation_id: int, body: bytes) -> bytes:
    return _SIZE.pack(4 + len(body)) + _FMT[I32].pack(correlation_id) + body


def recv_exact(sock, n: int) -> bytes:
    parts, got = [], 0
    while got < n:
        b = sock.recv(min(n - got, 1 << 20))
        if not b:
            raise ConnectionError("connection closed")
        parts.append(b)
        got += len(b)
    return b"".join(parts)


def recv_frame(sock) -> bytes:
    (n,) = _SIZE.unpack(recv_exact(sock, 4))
    if n < 0 or n > (256 << 20):
        raise KafkaError(CORRUPT_MESSAGE, f"bad frame size {n}")
    return recv_exact(sock, n)


# ---------------------------------------------------------------------------------- varints
def zigzag(v: int) -> int:
    return (v << 1) ^ (v >> 63)


def put_varint(v: int, out: bytearray):
    u = zigzag(v) & 0xFFFFFFFFFFFFFFFF
    while u >= 0x80:
        out.append((u & 0x7F) | 0x80)
        u >>= 7
    out.append(u)


def get_varint(buf, pos: int) -> tuple[int, int]:
    shift = u = 0
    while True:
        if pos >= len(buf):
            raise KafkaError(CORRUPT_MESSAGE, "truncated varint")
        b = buf[pos]
        pos += 1
        u |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
        if shift > 63:
            raise KafkaError(CORRUPT_MESSAGE, "varint too long")
    return (u >> 1) ^ -(u & 1), pos


# ---------------------------------------------------------------------------------- RecordBatch v2
_BATCH_HEAD = struct.Struct(">qiib")          # base offset, batch length, leader epoch, magic
_BATCH_REST = struct.Struct(">Ihiqqqhii")      # crc, attributes, last offset delta, first ts, max ts,
#                                                producer id, producer epoch, base sequence, count


def crc32c(data) -> int:
    b = bytes(data)
    return native().sw_crc32c(b, len(b))


def encode_batch(records, base_offset: int = 0) -> bytes:
    """records: [(key bytes|None, value bytes|None, timestamp ms)] -> one uncompressed RecordBatch v2
    whose offsets run base_offset, base_offset + 1, ..."""
    if not records:
        return b""
    ts0 = min(r[2] for r in records)
    tsmax = max(r[2] for r in records)
    body = bytearray()
    for i, (k, v, ts) in enumerate(records):
        rec = bytearray(b"\x00")                  # record attributes
        put_varint(ts - ts0, rec)
        put_varint(i, rec)
        if k is None:
            put_varint(-1, rec)
        else:
            put_varint(len(k), rec)
            rec += k
        if v is None:
            put_varint(-1, rec)
        else:
            put_varint(len(v), rec)
            rec += v
        put_varint(0, rec)                        # no headers
        put_varint(len(rec), body)
        body += rec
    after_crc = struct.pack(">hiqqqhii", 0, len(records) - 1, ts0, tsmax, -1, -1, -1, len(records)) + bytes(body)
    crc = crc32c(after_crc)
    batch_len = 4 + 1 + 4 + len(after_crc)       # leader epoch + magic + crc + rest
    return _BATCH_HEAD.pack(base_offset, batch_len, -1, 2) + struct.pack(">I", crc) + after_crc


def decode_batches(data, verify_crc: bool = True) -> list[tuple[int, bytes | None, bytes | None, int]]:
    """Every record of a records blob (one or more RecordBatch v2) -> [(offset, key, value, ts)].
    A trailing partial batch (fetch responses may cut one) is ignored; control batches are skipped."""
    out = []
    mv = memoryview(data) if data is not None else memoryview(b"")
    pos = 0
    while pos + _BATCH_HEAD.size <= len(mv):
        base, blen, _epoch, magic = _BATCH_HEAD.unpack_from(mv, pos)
        end = pos + 12 + blen
        if end > len(mv):
            break                                  # partial batch at the end of a fetch
        if magic != 2:
            raise KafkaError(CORRUPT_MESSAGE, f"record batch magic {magic} (only v2 is supported)")
        crc, attrs, _lod, ts0, _tsmax, _pid, _pep, _bseq, count = _BATCH_REST.unpack_from(mv, pos + 17)
        if verify_crc and crc32c(mv[pos + 21:end]) != crc:
            raise KafkaError(CORRUPT_MESSAGE, "record batch CRC mismatch")
        codec = attrs & 0x7
        recs = mv[pos + 17 + _BATCH_REST.size:end]
        if codec == 1:
            recs = memoryview(zlib.decompress(bytes(recs), 16 + zlib.MAX_WBITS))
        elif codec != 0:
            raise KafkaError(UNSUPPORTED_COMPRESSION_TYPE, f"codec {codec}")
        control = bool(attrs & 0x20)
        p = 0
        for _ in range(count):
            ln, p = get_varint(recs, p)
            rend = p + ln
            p += 1                                # record attributes
            tsd, p = get_varint(recs, p)
            od, p = get_varint(recs, p)
            kl, p = get_varint(recs, p)
            key = None if kl < 0 else bytes(recs[p:p + kl])
            p += max(kl, 0)
            vl, p = get_varint(recs, p)
            val = None if vl < 0 else bytes(recs[p:p + vl])
            p = rend                              # headers are skipped
            if not control:
                out.append((base + od, key, val, ts0 + tsd))
        pos = end
    return out
