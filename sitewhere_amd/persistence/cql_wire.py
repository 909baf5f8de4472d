"""Apache Cassandra client over the CQL native protocol v4 -- no driver dependency.

The reference persists events (and stream chunks) in Cassandra through the DataStax driver
(``sitewhere-cassandra/.../CassandraClient.java``, ``CassandraDeviceEventManagement.java``).  This
client implements what the event store needs: STARTUP (+ PasswordAuthenticator), QUERY for DDL,
PREPARE / EXECUTE with typed bind values, and ROWS results decoded by column type (ascii / text /
varchar, int, bigint, tinyint, boolean, double, timestamp, blob, uuid as text).
``persistence/cql_server.py`` serves the same subset in process.
"""
from __future__ import annotations

import datetime as _dt
import itertools
import socket
import struct
import threading
import uuid

VERSION_REQ, VERSION_RESP = 0x04, 0x84
ERROR, STARTUP, READY, AUTHENTICATE, OPTIONS, SUPPORTED = 0x00, 0x01, 0x02, 0x03, 0x05, 0x06
QUERY, RESULT, PREPARE, EXECUTE, AUTH_RESPONSE, AUTH_SUCCESS = 0x07, 0x08, 0x09, 0x0A, 0x0F, 0x10
R_VOID, R_ROWS, R_SET_KEYSPACE, R_PREPARED, R_SCHEMA = 1, 2, 3, 4, 5
ONE, QUORUM, LOCAL_ONE = 0x0001, 0x0004, 0x000A

# CQL type option ids
T_ASCII, T_BIGINT, T_BLOB, T_BOOLEAN, T_DOUBLE, T_INT, T_TIMESTAMP, T_UUID, T_VARCHAR, T_TINYINT = (
    0x01, 0x02, 0x03, 0x04, 0x07, 0x09, 0x0B, 0x0C, 0x0D, 0x14)
TYPE_NAMES = {"ascii": T_ASCII, "bigint": T_BIGINT, "blob": T_BLOB, "boolean": T_BOOLEAN, "double": T_DOUBLE,
              "int": T_INT, "timestamp": T_TIMESTAMP, "uuid": T_UUID, "text": T_VARCHAR, "varchar": T_VARCHAR,
              "tinyint": T_TINYINT, "counter": T_BIGINT}

_HDR = struct.Struct(">BBhBi")


class CqlError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"CQL error 0x{code:04x}: {msg}")
        self.code = code


# ---------------------------------------------------------------------------------- notation
def w_short(v):
    return struct.pack(">H", v)


def w_int(v):
    return struct.pack(">i", v)


def w_string(s: str) -> bytes:
    b = s.encode()
    return w_short(len(b)) + b


def w_long_string(s: str) -> bytes:
    b = s.encode()
    return w_int(len(b)) + b


def w_bytes(b: bytes | None) -> bytes:
    return w_int(-1) if b is None else w_int(len(b)) + b


def w_short_bytes(b: bytes) -> bytes:
    return w_short(len(b)) + b


def w_string_map(m: dict) -> bytes:
    return w_short(len(m)) + b"".join(w_string(k) + w_string(v) for k, v in m.items())


class Buf:
    def __init__(self, b: bytes, pos: int = 0):
        self.b, self.pos = b, pos

    def _u(self, fmt, n):
        (v,) = struct.unpack_from(fmt, self.b, self.pos)
        self.pos += n
        return v

    def byte(self):
        return self._u(">B", 1)

    def short(self):
        return self._u(">H", 2)

    def int(self):
        return self._u(">i", 4)

    def long(self):
        return self._u(">q", 8)

    def raw(self, n):
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return v

    def string(self):
        return self.raw(self.short()).decode()

    def long_string(self):
        return self.raw(self.int()).decode()

    def bytes(self):
        n = self.int()
        return None if n < 0 else self.raw(n)

    def short_bytes(self):
        return self.raw(self.short())

    def string_map(self):
        return {self.string(): self.string() for _ in range(self.short())}

    def string_multimap(self):
        out = {}
        for _ in range(self.short()):
            k = self.string()
            out[k] = [self.string() for _ in range(self.short())]
        return out

    def option(self):
        t = self.short()
        if t in (0x20, 0x22):                   # list / set
            return (t, self.option())
        if t == 0x21:                           # map
            return (t, self.option(), self.option())
        return t


# ---------------------------------------------------------------------------------- values
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def encode_value(t, v) -> bytes | None:
    if v is None:
        return None
    if t in (T_VARCHAR, T_ASCII):
        return str(v).encode()
    if t == T_INT:
        return struct.pack(">i", int(v))
    if t in (T_BIGINT,):
        return struct.pack(">q", int(v))
    if t == T_TIMESTAMP:
        if isinstance(v, _dt.datetime):
            v = int((v - _EPOCH).total_seconds() * 1000)
        return struct.pack(">q", int(v))
    if t == T_TINYINT:
        return struct.pack(">b", int(v))
    if t == T_BOOLEAN:
        return b"\x01" if v else b"\x00"
    if t == T_DOUBLE:
        return struct.pack(">d", float(v))
    if t == T_BLOB:
        return bytes(v)
    if t == T_UUID:
        return uuid.UUID(str(v)).bytes
    raise CqlError(0x2200, f"unsupported bind type {t!r}")


def decode_value(t, b: bytes | None):
    if b is None:
        return None
    if t in (T_VARCHAR, T_ASCII):
        return b.decode()
    if t == T_INT:
        return struct.unpack(">i", b)[0]
    if t in (T_BIGINT, T_TIMESTAMP):
        return struct.unpack(">q", b)[0]                 # timestamps as epoch ms
    if t == T_TINYINT:
        return struct.unpack(">b", b)[0]
    if t == T_BOOLEAN:
        return b != b"\x00"
    if t == T_DOUBLE:
        return struct.unpack(">d", b)[0]
    if t == T_BLOB:
        return bytes(b)
    if t == T_UUID:
        return str(uuid.UUID(bytes=bytes(b)))
    return bytes(b)


def write_option(t) -> bytes:
    if isinstance(t, tuple):
        return w_short(t[0]) + b"".join(write_option(x) for x in t[1:])
    return w_short(t)


def rows_metadata(cols: list[tuple[str, str, str, int]], no_metadata: bool = False) -> bytes:
    """cols: [(keyspace, table, name, type)] with a global table spec."""
    if not cols:
        return w_int(0x0004) + w_int(0)
    flags = 0x0001 | (0x0004 if no_metadata else 0)
    out = w_int(flags) + w_int(len(cols))
    if no_metadata:
        return out
    out += w_string(cols[0][0]) + w_string(cols[0][1])
    for _, _, name, t in cols:
        out += w_string(name) + write_option(t)
    return out


def read_metadata(buf: Buf) -> tuple[int, list[tuple[str, int]]]:
    flags, n = buf.int(), buf.int()
    if flags & 0x0002:
        buf.bytes()                              # paging state
    if flags & 0x0004:
        return flags, [("", 0)] * n
    glob = bool(flags & 0x0001)
    if glob:
        buf.string()
        buf.string()
    cols = []
    for _ in range(n):
        if not glob:
            buf.string()
            buf.string()
        cols.append((buf.string(), buf.option()))
    return flags, cols


# ---------------------------------------------------------------------------------- client
class Prepared:
    def __init__(self, pid: bytes, params: list, result_cols: list, query: str):
        self.id, self.params, self.result_cols, self.query = pid, params, result_cols, query


class CqlSession:
    """One connection (requests serialised, stream ids cycled).  ``CqlSession('host:9042', keyspace,
    username, password)``."""

    def __init__(self, address: str = "127.0.0.1:9042", keyspace: str | None = None, username: str | None = None,
                 password: str | None = None, timeout_s: float = 10.0):
        host, port = address.rsplit(":", 1)
        self.sock = socket.create_connection((host, int(port)), timeout=timeout_s)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._lock = threading.Lock()
        self._streams = itertools.cycle(range(1, 32767))
        self._prepared: dict[str, Prepared] = {}
        op, body = self._request(STARTUP, w_string_map({"CQL_VERSION": "3.0.0"}))
        if op == AUTHENTICATE:
            if username is None:
                raise CqlError(0x0100, f"server requires authentication ({Buf(body).string()})")
            op, body = self._request(AUTH_RESPONSE, w_bytes(b"\0" + username.encode() + b"\0" +
                                                             (password or "").encode()))
            if op != AUTH_SUCCESS:
                raise CqlError(0x0100, "authentication failed")
        elif op != READY:
            raise CqlError(0, f"unexpected startup reply opcode {op}")
        if keyspace:
            self.execute(f"USE {keyspace}")

    def _recv(self, n):
        parts, got = [], 0
        while got < n:
            b = self.sock.recv(min(n - got, 1 << 20))
            if not b:
                raise ConnectionError("connection closed")
            parts.append(b)
            got += len(b)
        return b"".join(parts)

    def _request(self, opcode: int, body: bytes):
        with self._lock:
            sid = next(self._streams)
            self.sock.sendall(_HDR.pack(VERSION_REQ, 0, sid, opcode, len(body)) + body)
            ver, _, rsid, op, ln = _HDR.unpack(self._recv(_HDR.size))
            body = self._recv(ln)
        if rsid != sid:
            raise CqlError(0, f"stream id {rsid} != {sid}")
        if op == ERROR:
            b = Buf(body)
            raise CqlError(b.int(), b.string())
        return op, body

    @staticmethod
    def _parse_result(body: bytes, result_cols=None):
        b = Buf(body)
        kind = b.int()
        if kind == R_ROWS:
            flags, cols = read_metadata(b)
            if flags & 0x0004 and result_cols:
                cols = result_cols
            n = b.int()
            return [{name: decode_value(t, b.bytes()) for name, t in cols} for _ in range(n)]
        if kind == R_PREPARED:
            pid = b.short_bytes()
            flags, n = b.int(), b.int()
            pk = b.int()
            for _ in range(pk):
                b.short()
            glob = bool(flags & 0x0001)
            if glob:
                b.string()
                b.string()
            params = []
            for _ in range(n):
                if not glob:
                    b.string()
                    b.string()
                params.append((b.string(), b.option()))
            _, rcols = read_metadata(b)
            return Prepared(bytes(pid), params, rcols, "")
        return None

    def execute(self, query: str, params: list | tuple | None = None, consistency: int = LOCAL_ONE):
        """DDL / unparameterised statements go as QUERY; with params the statement is prepared once
        (cached) and EXECUTEd with values serialised by the bind-variable types."""
        if params is None:
            _, body = self._request(QUERY, w_long_string(query) + w_short(consistency) + b"\x00")
            return self._parse_result(body)
        p = self.prepare(query)
        if len(params) != len(p.params):
            raise CqlError(0x2200, f"{len(p.params)} bind variables, {len(params)} values")
        vals = b"".join(w_bytes(encode_value(t, v)) for (_, t), v in zip(p.params, params))
        body = w_short_bytes(p.id) + w_short(consistency) + b"\x01" + w_short(len(params)) + vals
        _, rb = self._request(EXECUTE, body)
        return self._parse_result(rb, p.result_cols)

    def prepare(self, query: str) -> Prepared:
        p = self._prepared.get(query)
        if p is None:
            _, body = self._request(PREPARE, w_long_string(query))
            p = self._parse_result(body)
            p.query = query
            self._prepared[query] = p
        return p

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass
