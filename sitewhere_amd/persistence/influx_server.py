"""In-process InfluxDB 1.x HTTP API stand-in: ``/write`` (line protocol) and ``/query`` (the InfluxQL
subset :class:`~sitewhere_amd.persistence.events.InfluxEventStore` issues -- the reference's queries).

Points are keyed like InfluxDB's (measurement, tag set, timestamp): a second write of the same key
merges its fields, as a real series would.  Serves tests and single-node deployments.

    srv = MiniInfluxServer(port=0).start();  InfluxEventStore(srv.url, "tenant")
"""
from __future__ import annotations

import http.server
import json
import re
import threading
import urllib.parse

_TOKEN = re.compile(r"\s*(?:(?P<num>-?\d+(?:\.\d+)?)(?P<unit>ms|s|u|ns)?|(?P<str>'(?:\\.|[^'\\])*')|"
                    r"(?P<op>>=|<=|!=|=|>|<|\(|\)|,|\*)|(?P<id>[A-Za-z_][A-Za-z0-9_.]*|\"[^\"]+\"))")


def _unesc(s: str, chars: str) -> str:
    for c in chars:
        s = s.replace("\\" + c, c)
    return s


def _split_unescaped(s: str, sep: str) -> list[str]:
    out, cur, i, quoted = [], [], 0, False
    while i < len(s):
        ch = s[i]
        if ch == "\\" and i + 1 < len(s):
            cur.append(s[i:i + 2])
            i += 2
            continue
        if ch == '"':
            quoted = not quoted
        if ch == sep and not quoted:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    out.append("".join(cur))
    return out


def parse_line(line: str, precision: str = "ns") -> tuple[str, dict, dict, int]:
    parts = _split_unescaped(line, " ")
    parts = [p for p in parts if p != ""]
    head, fields_s = parts[0], parts[1]
    ts = int(parts[2]) if len(parts) > 2 else 0
    scale = {"ns": 1_000_000, "u": 1000, "ms": 1, "s": 0.001}.get(precision, 1_000_000)
    ts_ms = int(ts / scale) if precision != "ms" else ts
    hp = _split_unescaped(head, ",")
    meas = _unesc(hp[0], ", ")
    tags = {}
    for t in hp[1:]:
        k, v = t.split("=", 1)
        tags[_unesc(k, ", =")] = _unesc(v, ", =")
    fields = {}
    for f in _split_unescaped(fields_s, ","):
        k, v = f.split("=", 1)
        k = _unesc(k, ", =")
        if v.startswith('"'):
            fields[k] = v[1:-1].replace('\\"', '"').replace("\\\\", "\\")
        elif v.endswith("i"):
            fields[k] = int(v[:-1])
        elif v in ("t", "T", "true", "True"):
            fields[k] = True
        elif v in ("f", "F", "false", "False"):
            fields[k] = False
        else:
            fields[k] = float(v)
    return meas, tags, fields, ts_ms


class _Query:
    """Recursive-descent parser/evaluator of the supported InfluxQL statements."""

    def __init__(self, q: str):
        self.toks = []
        pos = 0
        while pos < len(q):
            m = _TOKEN.match(q, pos)
            if not m or m.end() == pos:
                if q[pos:].strip() == "":
                    break
                raise ValueError(f"cannot parse InfluxQL near {q[pos:pos + 20]!r}")
            pos = m.end()
            if m.group("num") is not None:
                v = float(m.group("num")) if "." in m.group("num") else int(m.group("num"))
                if m.group("unit"):
                    v = {"ms": v, "s": v * 1000, "u": v / 1000, "ns": v / 1_000_000}[m.group("unit")]
                self.toks.append(("num", v))
            elif m.group("str") is not None:
                self.toks.append(("str", m.group("str")[1:-1].replace("\\'", "'").replace("\\\\", "\\")))
            elif m.group("op") is not None:
                self.toks.append(("op", m.group("op")))
            else:
                self.toks.append(("id", m.group("id").strip('"')))
        self.i = 0

    def peek(self, kind=None, val=None):
        if self.i >= len(self.toks):
            return None
        t = self.toks[self.i]
        if kind and t[0] != kind:
            return None
        if val is not None and (t[1].upper() if isinstance(t[1], str) else t[1]) != val:
            return None
        return t

    def take(self, kind=None, val=None):
        t = self.peek(kind, val)
        if t is None:
            raise ValueError(f"InfluxQL: expected {val or kind} at token {self.i}")
        self.i += 1
        return t

    def cond(self):
        terms = [self.conj()]
        while self.peek("id", "OR"):
            self.take()
            terms.append(self.conj())
        return lambda p: any(t(p) for t in terms)

    def conj(self):
        terms = [self.atom()]
        while self.peek("id", "AND"):
            self.take()
            terms.append(self.atom())
        return lambda p: all(t(p) for t in terms)

    def atom(self):
        if self.peek("op", "("):
            self.take()
            c = self.cond()
            self.take("op", ")")
            return c
        name = self.take("id")[1]
        op = self.take("op")[1]
        lit = self.take()[1]

        def test(p, name=name, op=op, lit=lit):
            v = p.get(name)
            if v is None:
                return op == "!="
            try:
                return {"=": v == lit, "!=": v != lit, ">=": v >= lit, "<=": v <= lit, ">": v > lit,
                        "<": v < lit}[op]
            except TypeError:
                return False
        return test


class MiniInfluxServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 8086):
        self._dbs: dict[str, dict] = {}
        self._lock = threading.Lock()
        outer = self

        class H(http.server.BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _reply(self, code, obj=None):
                body = b"" if obj is None else json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _handle(self):
                u = urllib.parse.urlparse(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                n = int(self.headers.get("Content-Length") or 0)
                data = self.rfile.read(n) if n else b""
                if u.path == "/write":
                    try:
                        outer.write(q.get("db", ""), data.decode(), q.get("precision", "ns"))
                        self._reply(204)
                    except Exception as e:  # noqa: BLE001
                        self._reply(400, {"error": str(e)})
                elif u.path == "/query":
                    if data and "q" not in q:
                        q.update(urllib.parse.parse_qsl(data.decode()))
                    self._reply(200, {"results": [outer.query(q.get("db", ""), q["q"])]})
                elif u.path == "/ping":
                    self._reply(204)
                else:
                    self._reply(404, {"error": "not found"})

            do_GET = do_POST = _handle

        self._srv = http.server.ThreadingHTTPServer((host, port), H)
        self.host, self.port = host, self._srv.server_address[1]

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def start(self):
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="mini-influx").start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()

    def write(self, db: str, body: str, precision: str):
        with self._lock:
            if db not in self._dbs:
                raise ValueError(f"database not found: {db}")
            pts = self._dbs[db]
            for line in body.splitlines():
                if not line.strip() or line.startswith("#"):
                    continue
                meas, tags, fields, ts = parse_line(line, precision)
                key = (meas, tuple(sorted(tags.items())), ts)
                p = pts.setdefault(key, {"time": ts, **tags})
                p.update(fields)

    def query(self, db: str, q: str) -> dict:
        s = q.strip().rstrip(";")
        m = re.match(r"(?i)CREATE\s+DATABASE\s+\"?([\w-]+)\"?", s)
        if m:
            with self._lock:
                self._dbs.setdefault(m.group(1), {})
            return {"statement_id": 0}
        try:
            return self._select(db, s)
        except ValueError as e:
            return {"statement_id": 0, "error": str(e)}

    def _select(self, db: str, s: str) -> dict:
        p = _Query(s)
        p.take("id", "SELECT")
        agg = None
        if p.peek("op", "*"):
            p.take()
        else:
            fn = p.take("id")[1].lower()
            p.take("op", "(")
            agg = (fn, p.take("id")[1])
            p.take("op", ")")
        p.take("id", "FROM")
        meas = p.take("id")[1]
        cond = (lambda pt: True)
        if p.peek("id", "WHERE"):
            p.take()
            cond = p.cond()
        desc, limit, offset = False, 0, 0
        if p.peek("id", "ORDER"):
            p.take()
            p.take("id", "BY")
            p.take("id", "TIME")
            if p.peek("id", "DESC"):
                p.take()
                desc = True
            elif p.peek("id", "ASC"):
                p.take()
        if p.peek("id", "LIMIT"):
            p.take()
            limit = int(p.take("num")[1])
        if p.peek("id", "OFFSET"):
            p.take()
            offset = int(p.take("num")[1])
        with self._lock:
            pts = [v for (mm, _, _), v in self._dbs.get(db, {}).items() if mm == meas and cond(v)]
        if agg:
            n = sum(1 for x in pts if x.get(agg[1]) is not None)
            return {"statement_id": 0, "series": [{"name": meas, "columns": ["time", agg[0]], "values": [[0, n]]}]}
        pts.sort(key=lambda x: x["time"], reverse=desc)
        pts = pts[offset:offset + limit] if limit else pts[offset:]
        if not pts:
            return {"statement_id": 0}
        cols = ["time"] + sorted({k for x in pts for k in x} - {"time"})
        return {"statement_id": 0, "series": [{"name": meas, "columns": cols,
                                               "values": [[x.get(c) for c in cols] for x in pts]}]}
