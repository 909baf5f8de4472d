"""In-process Cassandra stand-in: CQL native protocol v4 and the CQL subset the event store uses.

Keyspaces, tables with partition and clustering keys (``WITH CLUSTERING ORDER BY``), upserting
INSERT, SELECT / SELECT COUNT(*) by partition key (``=`` / ``IN``) with clustering-key ranges,
``LIMIT``, ``ALLOW FILTERING`` scans, TRUNCATE; prepared statements with typed bind markers;
optional PasswordAuthenticator.  In memory -- for tests and single-node deployments of the
``cassandra`` tenant template.
"""
from __future__ import annotations

import hashlib
import re
import socket
import socketserver
import struct
import threading

from .cql_wire import (AUTH_RESPONSE, AUTH_SUCCESS, AUTHENTICATE, ERROR, EXECUTE, OPTIONS, PREPARE, QUERY, R_PREPARED,
                       R_ROWS, R_SCHEMA, R_SET_KEYSPACE, R_VOID, READY, RESULT, STARTUP, SUPPORTED, T_BIGINT, T_INT,
                       TYPE_NAMES, VERSION_RESP, Buf, CqlError, decode_value, encode_value, rows_metadata, w_bytes,
                       w_int, w_short, w_short_bytes, w_string, write_option)

_HDR = struct.Struct(">BBhBi")
_TOK = re.compile(r"\s*(?:(?P<str>'(?:''|[^'])*')|(?P<num>-?\d+(?:\.\d+)?)|(?P<id>\"[^\"]+\"|[A-Za-z_][A-Za-z0-9_]*)|"
                  r"(?P<op><=|>=|!=|[(),;=<>.*?{}:\[\]]))")

SYNTAX, INVALID, ALREADY_EXISTS, BAD_CREDENTIALS = 0x2000, 0x2200, 0x2400, 0x0100


class _Lexer:
    def __init__(self, q: str):
        self.t, pos = [], 0
        q = q.strip().rstrip(";")
        while pos < len(q):
            m = _TOK.match(q, pos)
            if not m or m.end() == pos:
                if not q[pos:].strip():
                    break
                raise CqlError(SYNTAX, f"syntax error near {q[pos:pos + 20]!r}")
            pos = m.end()
            if m.group("str") is not None:
                self.t.append(("str", m.group("str")[1:-1].replace("''", "'")))
            elif m.group("num") is not None:
                n = m.group("num")
                self.t.append(("num", float(n) if "." in n else int(n)))
            elif m.group("id") is not None:
                self.t.append(("id", m.group("id")))
            else:
                self.t.append(("op", m.group("op")))
        self.i = 0

    def peek(self, *vals):
        if self.i >= len(self.t):
            return None
        k, v = self.t[self.i]
        if vals and not (isinstance(v, str) and v.upper() in vals):
            return None
        return self.t[self.i]

    def take(self, *vals):
        t = self.peek(*vals)
        if t is None:
            raise CqlError(SYNTAX, f"expected {' or '.join(vals) or 'token'} at {self.t[self.i:self.i + 3]}")
        self.i += 1
        return t

    def ident(self):
        k, v = self.take()
        if k != "id":
            raise CqlError(SYNTAX, f"expected identifier, got {v!r}")
        return v[1:-1] if v.startswith('"') else v.lower()

    def name(self, ks):
        a = self.ident()
        if self.peek(".") and self.t[self.i][0] == "op":
            self.take(".")
            return a, self.ident()
        return ks, a

    def skip_rest(self):
        self.i = len(self.t)


class _Marker:
    def __init__(self, idx):
        self.idx = idx


class _Table:
    def __init__(self, ks, name, cols, pk, ck, desc):
        self.ks, self.name, self.cols, self.pk, self.ck, self.desc = ks, name, cols, pk, ck, desc
        self.types = dict(cols)
        self.parts: dict[tuple, dict[tuple, dict]] = {}

    def sort_rows(self, rows: list[dict]) -> list[dict]:
        for c in reversed(self.ck):
            rows.sort(key=lambda r: (r.get(c) is not None, r.get(c)), reverse=self.desc.get(c, False))
        return rows


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        srv: MiniCassandraServer = self.server.cql        # type: ignore[attr-defined]
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        st = {"ks": None, "authed": not srv.users}
        try:
            while True:
                hdr = self._recv(sock, _HDR.size)
                _, _, sid, op, ln = _HDR.unpack(hdr)
                body = self._recv(sock, ln)
                try:
                    rop, rbody = srv.dispatch(op, body, st)
                except CqlError as e:
                    rop, rbody = ERROR, w_int(e.code) + w_string(str(e).split(": ", 1)[-1])
                sock.sendall(_HDR.pack(VERSION_RESP, 0, sid, rop, len(rbody)) + rbody)
        except (ConnectionError, OSError):
            pass

    @staticmethod
    def _recv(sock, n):
        parts, got = [], 0
        while got < n:
            b = sock.recv(min(n - got, 1 << 20))
            if not b:
                raise ConnectionError("closed")
            parts.append(b)
            got += len(b)
        return b"".join(parts)


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class MiniCassandraServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 9042, users: dict[str, str] | None = None):
        self.users = dict(users or {})
        self._srv = _Server((host, port), _Handler)
        self._srv.cql = self
        self.host, self.port = host, self._srv.server_address[1]
        self._keyspaces: set = set()
        self._tables: dict[tuple[str, str], _Table] = {}
        self._prepared: dict[bytes, tuple] = {}
        self._lock = threading.RLock()

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def start(self):
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="mini-cassandra").start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()

    # ------------------------------------------------------------------ protocol
    def dispatch(self, op, body, st):
        b = Buf(body)
        if op == OPTIONS:
            return SUPPORTED, w_short(1) + w_string("CQL_VERSION") + w_short(1) + w_string("3.4.5")
        if op == STARTUP:
            b.string_map()
            if self.users:
                return AUTHENTICATE, w_string("org.apache.cassandra.auth.PasswordAuthenticator")
            return READY, b""
        if op == AUTH_RESPONSE:
            tok = b.bytes() or b""
            parts = tok.split(b"\0")
            if len(parts) == 3 and self.users.get(parts[1].decode()) == parts[2].decode():
                st["authed"] = True
                return AUTH_SUCCESS, w_bytes(None)
            raise CqlError(BAD_CREDENTIALS, "Provided username and/or password are incorrect")
        if not st["authed"]:
            raise CqlError(0x000A, "not authenticated")
        if op == QUERY:
            q = b.long_string()
            return RESULT, self._run(q, [], st)
        if op == PREPARE:
            q = b.long_string()
            return RESULT, self._prepare(q, st)
        if op == EXECUTE:
            pid = bytes(b.short_bytes())
            b.short()                                     # consistency
            flags = b.byte()
            vals = [b.bytes() for _ in range(b.short())] if flags & 0x01 else []
            q, ks, params = self._prepared.get(pid, (None, None, None))
            if q is None:
                raise CqlError(0x2500, "unprepared statement")
            st2 = dict(st, ks=ks or st["ks"])
            return RESULT, self._run(q, [decode_value(t, v) for (_, t), v in zip(params, vals)], st2)
        raise CqlError(0x000A, f"unsupported opcode {op}")

    def _prepare(self, q, st):
        params, rcols, tbl = self._analyse(q, st)
        pid = hashlib.md5((q + (st["ks"] or "")).encode()).digest()
        self._prepared[pid] = (q, st["ks"], params)
        ks, tn = (tbl.ks, tbl.name) if tbl else ("", "")
        out = w_int(R_PREPARED) + w_short_bytes(pid)
        out += w_int(0x0001) + w_int(len(params)) + w_int(0) + w_string(ks) + w_string(tn)
        for name, t in params:
            out += w_string(name) + write_option(t)
        out += rows_metadata([(ks, tn, n, t) for n, t in rcols])
        return out

    # ------------------------------------------------------------------ statements
    def _table(self, ks, name) -> _Table:
        t = self._tables.get((ks, name))
        if t is None:
            raise CqlError(INVALID, f"unconfigured table {name}" if ks else "no keyspace selected")
        return t

    def _analyse(self, q, st):
        """Bind-variable specs and result columns of a statement (for PREPARE)."""
        lx = _Lexer(q)
        head = lx.take()[1].upper()
        if head == "INSERT":
            lx.take("INTO")
            tbl = self._table(*lx.name(st["ks"]))
            cols = self._paren_idents(lx)
            lx.take("VALUES")
            vals = self._paren_values(lx, [])
            return [(c, tbl.types[c]) for c, v in zip(cols, vals) if isinstance(v, _Marker)], [], tbl
        if head == "SELECT":
            sel, tbl, where, limit = self._parse_select(lx, st, [])
            params = [(c, tbl.types[c]) for c, _, v in where
                      for vv in (v if isinstance(v, list) else [v]) if isinstance(vv, _Marker)]
            if isinstance(limit, _Marker):
                params.append(("[limit]", T_INT))
            return params, self._result_cols(sel, tbl), tbl
        return [], [], None

    def _result_cols(self, sel, tbl):
        if sel == "count":
            return [("count", T_BIGINT)]
        return [(c, tbl.types[c]) for c in (sel if sel != "*" else [c for c, _ in tbl.cols])]

    @staticmethod
    def _paren_idents(lx):
        lx.take("(")
        out = [lx.ident()]
        while lx.peek(","):
            lx.take(",")
            out.append(lx.ident())
        lx.take(")")
        return out

    def _value(self, lx, binds):
        k, v = lx.take()
        if k == "op" and v == "?":
            m = _Marker(len(binds))
            binds.append(m)
            return m
        if k == "id" and v.upper() in ("TRUE", "FALSE", "NULL"):
            return None if v.upper() == "NULL" else v.upper() == "TRUE"
        if k in ("str", "num"):
            return v
        raise CqlError(SYNTAX, f"unexpected {v!r}")

    def _paren_values(self, lx, binds):
        lx.take("(")
        out = [self._value(lx, binds)]
        while lx.peek(","):
            lx.take(",")
            out.append(self._value(lx, binds))
        lx.take(")")
        return out

    def _parse_select(self, lx, st, binds):
        if lx.peek("*"):
            lx.take()
            sel = "*"
        elif lx.peek("COUNT"):
            lx.take()
            lx.take("(")
            lx.take()
            lx.take(")")
            sel = "count"
        else:
            sel = [lx.ident()]
            while lx.peek(","):
                lx.take(",")
                sel.append(lx.ident())
        lx.take("FROM")
        tbl = self._table(*lx.name(st["ks"]))
        where = []
        if lx.peek("WHERE"):
            lx.take()
            while True:
                c = lx.ident()
                if lx.peek("IN"):
                    lx.take()
                    where.append((c, "in", self._paren_values(lx, binds)))
                else:
                    op = lx.take()[1]
                    where.append((c, op, self._value(lx, binds)))
                if not lx.peek("AND"):
                    break
                lx.take()
        limit = None
        while lx.peek() is not None:
            if lx.peek("LIMIT"):
                lx.take()
                limit = self._value(lx, binds)
            elif lx.peek("ALLOW"):
                lx.take()
                lx.take("FILTERING")
            else:
                lx.skip_rest()
        return sel, tbl, where, limit

    def _run(self, q, values, st):
        with self._lock:
            lx = _Lexer(q)
            head = lx.take()[1].upper()
            bind = lambda v: values[v.idx] if isinstance(v, _Marker) else v  # noqa: E731
            if head == "USE":
                st["ks"] = lx.ident()
                if st["ks"] not in self._keyspaces:
                    raise CqlError(INVALID, f"Keyspace '{st['ks']}' does not exist")
                return w_int(R_SET_KEYSPACE) + w_string(st["ks"])
            if head == "CREATE":
                kind = lx.take()[1].upper()
                ine = bool(lx.peek("IF") and (lx.take() and lx.take("NOT") and lx.take("EXISTS")))
                if kind == "KEYSPACE":
                    ks = lx.ident()
                    if ks in self._keyspaces and not ine:
                        raise CqlError(ALREADY_EXISTS, f"keyspace {ks} exists")
                    self._keyspaces.add(ks)
                    return w_int(R_SCHEMA) + w_string("CREATED") + w_string("KEYSPACE") + w_string(ks)
                if kind == "TABLE":
                    return self._create_table(lx, st, ine)
                raise CqlError(SYNTAX, f"CREATE {kind} not supported")
            if head == "INSERT":
                lx.take("INTO")
                tbl = self._table(*lx.name(st["ks"]))
                cols = self._paren_idents(lx)
                lx.take("VALUES")
                vals = [bind(v) for v in self._paren_values(lx, [])]
                row = dict(zip(cols, vals))
                for c in tbl.pk + tbl.ck:
                    if row.get(c) is None:
                        raise CqlError(INVALID, f"missing primary key column {c}")
                part = tbl.parts.setdefault(tuple(row[c] for c in tbl.pk), {})
                ckey = tuple(row[c] for c in tbl.ck)
                part[ckey] = {**part.get(ckey, {}), **row}        # upsert
                return w_int(R_VOID)
            if head == "TRUNCATE":
                lx.peek("TABLE") and lx.take()
                self._table(*lx.name(st["ks"])).parts.clear()
                return w_int(R_VOID)
            if head == "SELECT":
                sel, tbl, where, limit = self._parse_select(lx, st, [])
                return self._select(tbl, sel, [(c, op, [bind(x) for x in v] if isinstance(v, list) else bind(v))
                                               for c, op, v in where], bind(limit))
            raise CqlError(SYNTAX, f"{head} not supported")

    def _create_table(self, lx, st, ine):
        ks, name = lx.name(st["ks"])
        if ks not in self._keyspaces:
            raise CqlError(INVALID, f"Keyspace '{ks}' does not exist")
        lx.take("(")
        cols, pk, ck = [], [], []
        while True:
            if lx.peek("PRIMARY"):
                lx.take()
                lx.take("KEY")
                lx.take("(")
                if lx.peek("("):
                    pk = self._paren_idents(lx)
                else:
                    pk = [lx.ident()]
                while lx.peek(","):
                    lx.take(",")
                    ck.append(lx.ident())
                lx.take(")")
            else:
                c = lx.ident()
                t = lx.ident()
                if t in ("frozen", "list", "set", "map"):
                    raise CqlError(INVALID, f"type {t}<...> not supported by this server")
                cols.append((c, TYPE_NAMES[t]))
                if lx.peek("PRIMARY"):
                    lx.take()
                    lx.take("KEY")
                    pk = [c]
            if lx.peek(","):
                lx.take(",")
                continue
            lx.take(")")
            break
        desc = {}
        if lx.peek("WITH"):
            lx.take()
            if lx.peek("CLUSTERING"):
                lx.take()
                lx.take("ORDER")
                lx.take("BY")
                lx.take("(")
                while True:
                    c = lx.ident()
                    desc[c] = lx.take("ASC", "DESC")[1].upper() == "DESC"
                    if not lx.peek(","):
                        break
                    lx.take(",")
                lx.take(")")
            lx.skip_rest()
        if (ks, name) in self._tables:
            if not ine:
                raise CqlError(ALREADY_EXISTS, f"table {name} exists")
        else:
            self._tables[(ks, name)] = _Table(ks, name, cols, pk, ck, desc)
        return w_int(R_SCHEMA) + w_string("CREATED") + w_string("TABLE") + w_string(ks) + w_string(name)

    def _select(self, tbl: _Table, sel, where, limit):
        eq = {c: v for c, op, v in where if op == "="}
        ins = {c: v for c, op, v in where if op == "in"}
        if all(c in eq or c in ins for c in tbl.pk):
            keys = [()]
            for c in tbl.pk:
                keys = [k + (v,) for k in keys for v in (ins[c] if c in ins else [eq[c]])]
            parts = [tbl.parts.get(k, {}) for k in keys]
        else:
            parts = list(tbl.parts.values())              # ALLOW FILTERING scan
        rows = []
        for p in parts:
            for r in p.values():
                ok = True
                for c, op, v in where:
                    x = r.get(c)
                    if op == "in":
                        ok = x in v
                    elif x is None:
                        ok = False
                    else:
                        ok = {"=": x == v, "<": x < v, "<=": x <= v, ">": x > v, ">=": x >= v, "!=": x != v}[op]
                    if not ok:
                        break
                if ok:
                    rows.append(r)
        rows = tbl.sort_rows(rows)
        if limit:
            rows = rows[:int(limit)]
        rc = self._result_cols(sel, tbl)
        if sel == "count":
            rows = [{"count": len(rows)}]
        out = w_int(R_ROWS) + rows_metadata([(tbl.ks, tbl.name, n, t) for n, t in rc]) + w_int(len(rows))
        for r in rows:
            out += b"".join(w_bytes(encode_value(t, r.get(n))) for n, t in rc)
        return out
