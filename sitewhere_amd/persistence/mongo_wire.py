"""MongoDB client over the wire protocol (OP_MSG, BSON) -- no driver dependency.

The reference's default datastore is MongoDB (``sitewhere-mongodb/.../MongoDbClient.java``; nine
services persist through ``persistence/mongodb/*``, events through ``MongoDeviceEventManagement``
with bulk inserts).  This client speaks OP_MSG (MongoDB 3.6+), authenticates with SCRAM-SHA-256 or
SCRAM-SHA-1 (``mongodb://user:pass@host:port/db?authSource=admin&authMechanism=...``) and implements
the command subset the stores need: insert, find / getMore, update (replacement, ``$set``/``$unset``/
``$inc``, upsert), delete, count, createIndexes, drop.  ``persistence/mongo_server.py`` serves the
same subset in process (tests, single-node deployments).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import itertools
import os
import socket
import struct
import threading
import urllib.parse

from . import bson

OP_MSG = 2013
_HDR = struct.Struct("<iiii")


class MongoError(RuntimeError):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


DUPLICATE_KEY = 11000


# ---------------------------------------------------------------------------------- framing
def op_msg(request_id: int, doc: dict, response_to: int = 0) -> bytes:
    body = struct.pack("<I", 0) + b"\x00" + bson.encode(doc)
    return _HDR.pack(16 + len(body), request_id, response_to, OP_MSG) + body


def _recv(sock, n):
    parts, got = [], 0
    while got < n:
        b = sock.recv(min(n - got, 1 << 20))
        if not b:
            raise ConnectionError("connection closed")
        parts.append(b)
        got += len(b)
    return b"".join(parts)


def read_message(sock) -> tuple[int, int, int, bytes]:
    ln, rid, rto, op = _HDR.unpack(_recv(sock, 16))
    if ln < 16 or ln > (48 << 20):
        raise MongoError(f"bad message length {ln}")
    return rid, rto, op, _recv(sock, ln - 16)


def parse_op_msg(body: bytes) -> dict:
    """OP_MSG body -> the command document; kind-1 document sequences become array fields."""
    pos = 4                                   # flag bits
    doc: dict = {}
    seqs: dict = {}
    while pos < len(body):
        kind = body[pos]
        pos += 1
        if kind == 0:
            doc, pos = bson.decode_with_end(body, pos)
        elif kind == 1:
            (size,) = struct.unpack_from("<i", body, pos)
            end = pos + size
            nul = body.index(0, pos + 4)
            ident = body[pos + 4:nul].decode()
            p = nul + 1
            items = []
            while p < end:
                d, p = bson.decode_with_end(body, p)
                items.append(d)
            seqs[ident] = items
            pos = end
        else:
            break                             # checksum (flag bit 0) or unknown section
    doc.update(seqs)
    return doc


# ---------------------------------------------------------------------------------- query semantics
_MISSING = object()


def get_path(doc, path: str):
    cur = doc
    for part in path.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        elif isinstance(cur, list) and part.isdigit() and int(part) < len(cur):
            cur = cur[int(part)]
        else:
            return _MISSING
    return cur


def _cmp_ok(v, op, arg) -> bool:
    if op == "$eq":
        return v == arg or (isinstance(v, list) and arg in v)
    if op == "$ne":
        return not _cmp_ok(v, "$eq", arg)
    if op == "$in":
        return any(_cmp_ok(v, "$eq", a) for a in arg)
    if op == "$nin":
        return not any(_cmp_ok(v, "$eq", a) for a in arg)
    if op == "$exists":
        return (v is not _MISSING) == bool(arg)
    if v is _MISSING or v is None:
        return False
    try:
        if op == "$gt":
            return v > arg
        if op == "$gte":
            return v >= arg
        if op == "$lt":
            return v < arg
        if op == "$lte":
            return v <= arg
    except TypeError:
        return False
    raise MongoError(f"unsupported query operator {op}", 2)


def matches(doc: dict, flt: dict | None) -> bool:
    for k, cond in (flt or {}).items():
        if k == "$and":
            if not all(matches(doc, c) for c in cond):
                return False
            continue
        if k == "$or":
            if not any(matches(doc, c) for c in cond):
                return False
            continue
        v = get_path(doc, k)
        if isinstance(cond, dict) and cond and all(str(x).startswith("$") for x in cond):
            if not all(_cmp_ok(v, op, arg) for op, arg in cond.items()):
                return False
        elif not _cmp_ok(v, "$eq", cond):
            return False
    return True


def _set_path(doc, path, value):
    parts = path.split(".")
    cur = doc
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = value


def apply_update(doc: dict, update: dict) -> dict:
    """Replacement (no ``$`` keys; keeps ``_id``) or ``$set`` / ``$unset`` / ``$inc`` / ``$setOnInsert``."""
    if not any(str(k).startswith("$") for k in update):
        out = dict(update)
        if "_id" in doc:
            out["_id"] = doc["_id"]
        return out
    out = dict(doc)
    for op, fields in update.items():
        for path, v in fields.items():
            if op in ("$set", "$setOnInsert"):
                _set_path(out, path, v)
            elif op == "$unset":
                parts = path.split(".")
                cur = out
                for p in parts[:-1]:
                    cur = cur.get(p, {})
                if isinstance(cur, dict):
                    cur.pop(parts[-1], None)
            elif op == "$inc":
                cur = get_path(out, path)
                _set_path(out, path, (0 if cur is _MISSING else cur) + v)
            else:
                raise MongoError(f"unsupported update operator {op}", 9)
    return out


def sort_docs(docs: list, spec: dict | None) -> list:
    for field, direction in reversed(list((spec or {}).items())):
        docs.sort(key=lambda d: _sort_key(get_path(d, field)), reverse=direction < 0)
    return docs


def _sort_key(v):
    # BSON comparison order, simplified: missing/null < numbers < strings < everything else
    if v is _MISSING or v is None:
        return (0, 0)
    if isinstance(v, bool):
        return (4, int(v))
    if isinstance(v, (int, float)):
        return (1, v)
    if isinstance(v, str):
        return (2, v)
    return (3, repr(v))


# ---------------------------------------------------------------------------------- SCRAM
def _xor(a: bytes, b: bytes) -> bytes:
    return bytes(x ^ y for x, y in zip(a, b))


def scram_salted_password(mechanism: str, user: str, password: str, salt: bytes, iterations: int) -> bytes:
    if mechanism == "SCRAM-SHA-1":
        pw = hashlib.md5(f"{user}:mongo:{password}".encode()).hexdigest().encode()
        return hashlib.pbkdf2_hmac("sha1", pw, salt, iterations)
    return hashlib.pbkdf2_hmac("sha256", password.encode(), salt, iterations)


def _hash(mechanism):
    return hashlib.sha1 if mechanism == "SCRAM-SHA-1" else hashlib.sha256


def scram_parse(payload: bytes) -> dict:
    return dict(kv.split("=", 1) for kv in payload.decode().split(","))


# ---------------------------------------------------------------------------------- client
class _Conn:
    def __init__(self, host, port, timeout_s):
        self.sock = socket.create_connection((host, port), timeout=timeout_s)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.ids = itertools.count(1)

    def command(self, db: str, cmd: dict) -> dict:
        cmd = dict(cmd)
        cmd["$db"] = db
        rid = next(self.ids)
        self.sock.sendall(op_msg(rid, cmd))
        _, rto, op, body = read_message(self.sock)
        if op != OP_MSG or rto != rid:
            raise MongoError(f"unexpected reply (op {op}, responseTo {rto})")
        r = parse_op_msg(body)
        if r.get("ok") != 1 and r.get("ok") != 1.0:
            raise MongoError(r.get("errmsg", "command failed"), int(r.get("code", 0)))
        for we in r.get("writeErrors") or []:
            raise MongoError(we.get("errmsg", "write error"), int(we.get("code", 0)))
        return r


class MongoClient:
    """``MongoClient("mongodb://[user:pass@]host:port[/db][?authSource=..&authMechanism=..]")``;
    one connection per calling thread."""

    def __init__(self, uri: str = "mongodb://localhost:27017", timeout_s: float = 10.0):
        u = urllib.parse.urlparse(uri)
        if u.scheme != "mongodb":
            raise ValueError("only mongodb:// URIs are supported")
        self.host, self.port = u.hostname or "localhost", u.port or 27017
        self.user = urllib.parse.unquote(u.username) if u.username else None
        self.password = urllib.parse.unquote(u.password) if u.password else None
        q = dict(urllib.parse.parse_qsl(u.query))
        self.default_db = (u.path or "/").lstrip("/") or "test"
        self.auth_source = q.get("authSource", self.default_db if self.user else "admin")
        self.mechanism = q.get("authMechanism", "SCRAM-SHA-256")
        self.timeout_s = timeout_s
        self._tls = threading.local()
        self._all: list = []
        self._lock = threading.Lock()
        self.server_info: dict = {}
        self._conn()                            # connect, handshake and authenticate eagerly

    def _conn(self) -> _Conn:
        c = getattr(self._tls, "c", None)
        if c is None:
            c = _Conn(self.host, self.port, self.timeout_s)
            self.server_info = c.command("admin", {"hello": 1, "client": {"driver": {"name": "sitewhere-amd",
                                                                                    "version": "1"}}})
            if self.user:
                self._authenticate(c)
            self._tls.c = c
            with self._lock:
                self._all.append(c)
        return c

    def _authenticate(self, c: _Conn):
        mech, H = self.mechanism, _hash(self.mechanism)
        nonce = base64.b64encode(os.urandom(24)).decode()
        user = self.user.replace("=", "=3D").replace(",", "=2C")
        bare = f"n={user},r={nonce}"
        r = c.command(self.auth_source, {"saslStart": 1, "mechanism": mech, "payload": b"n,," + bare.encode(),
                                          "autoAuthorize": 1, "options": {"skipEmptyExchange": True}})
        server_first = r["payload"].decode()
        sf = scram_parse(r["payload"])
        if not sf["r"].startswith(nonce):
            raise MongoError("SCRAM: server nonce does not extend the client nonce")
        salted = scram_salted_password(mech, self.user, self.password or "", base64.b64decode(sf["s"]), int(sf["i"]))
        client_key = hmac.new(salted, b"Client Key", H).digest()
        stored_key = H(client_key).digest()
        without_proof = f"c=biws,r={sf['r']}"
        auth_msg = f"{bare},{server_first},{without_proof}".encode()
        proof = _xor(client_key, hmac.new(stored_key, auth_msg, H).digest())
        r2 = c.command(self.auth_source, {"saslContinue": 1, "conversationId": r["conversationId"],
                                          "payload": f"{without_proof},p={base64.b64encode(proof).decode()}".encode()})
        server_sig = hmac.new(hmac.new(salted, b"Server Key", H).digest(), auth_msg, H).digest()
        if scram_parse(r2["payload"]).get("v") != base64.b64encode(server_sig).decode():
            raise MongoError("SCRAM: server signature mismatch")
        while not r2.get("done"):
            r2 = c.command(self.auth_source, {"saslContinue": 1, "conversationId": r["conversationId"],
                                              "payload": b""})

    def command(self, db: str, cmd: dict) -> dict:
        return self._conn().command(db, cmd)

    def __getitem__(self, name: str) -> "Database":
        return Database(self, name)

    def close(self):
        with self._lock:
            for c in self._all:
                try:
                    c.sock.close()
                except OSError:
                    pass
            self._all.clear()


class Database:
    def __init__(self, client: MongoClient, name: str):
        self.client, self.name = client, name

    def command(self, cmd: dict) -> dict:
        return self.client.command(self.name, cmd)

    def __getitem__(self, coll: str) -> "Collection":
        return Collection(self, coll)

    def drop(self):
        self.command({"dropDatabase": 1})


class Collection:
    def __init__(self, db: Database, name: str):
        self.db, self.name = db, name

    def insert_many(self, docs: list, ordered: bool = True) -> int:
        n = 0
        for i in range(0, len(docs), 1000):
            n += self.db.command({"insert": self.name, "documents": docs[i:i + 1000], "ordered": ordered}).get("n", 0)
        return n

    def insert_one(self, doc: dict):
        self.insert_many([doc])

    def find(self, flt: dict | None = None, sort: dict | None = None, skip: int = 0, limit: int = 0,
             batch_size: int = 1000) -> list:
        cmd = {"find": self.name, "filter": flt or {}, "batchSize": batch_size}
        if sort:
            cmd["sort"] = sort
        if skip:
            cmd["skip"] = int(skip)
        if limit:
            cmd["limit"] = int(limit)
        r = self.db.command(cmd)
        cur = r["cursor"]
        out = list(cur["firstBatch"])
        while cur.get("id"):
            cur = self.db.command({"getMore": bson.Int64(cur["id"]), "collection": self.name,
                                   "batchSize": batch_size})["cursor"]
            out += cur["nextBatch"]
        return out

    def find_one(self, flt: dict | None = None, sort: dict | None = None):
        r = self.find(flt, sort, limit=1)
        return r[0] if r else None

    def count_documents(self, flt: dict | None = None) -> int:
        return int(self.db.command({"count": self.name, "query": flt or {}})["n"])

    def _update(self, updates: list) -> dict:
        return self.db.command({"update": self.name, "updates": updates, "ordered": True})

    def replace_one(self, flt: dict, doc: dict, upsert: bool = False):
        return self._update([{"q": flt, "u": doc, "upsert": upsert, "multi": False}])

    def update_one(self, flt: dict, update: dict, upsert: bool = False):
        return self._update([{"q": flt, "u": update, "upsert": upsert, "multi": False}])

    def update_many(self, flt: dict, update: dict):
        return self._update([{"q": flt, "u": update, "upsert": False, "multi": True}])

    def bulk_replace(self, docs: list, key: str = "_id"):
        """Upsert-by-key in one round trip per 1000 documents (the reference's bulk writes)."""
        for i in range(0, len(docs), 1000):
            self._update([{"q": {key: d[key]}, "u": d, "upsert": True, "multi": False} for d in docs[i:i + 1000]])

    def delete_one(self, flt: dict) -> int:
        return int(self.db.command({"delete": self.name, "deletes": [{"q": flt, "limit": 1}]}).get("n", 0))

    def delete_many(self, flt: dict) -> int:
        return int(self.db.command({"delete": self.name, "deletes": [{"q": flt, "limit": 0}]}).get("n", 0))

    def create_index(self, keys: dict, unique: bool = False, sparse: bool = False, name: str | None = None):
        name = name or "_".join(f"{k}_{v}" for k, v in keys.items())
        self.db.command({"createIndexes": self.name, "indexes": [{"key": keys, "name": name, "unique": unique,
                                                                   "sparse": sparse}]})
        return name

    def drop(self):
        try:
            self.db.command({"drop": self.name})
        except MongoError as e:
            if e.code != 26:                   # NamespaceNotFound
                raise
