"""In-process MongoDB-protocol server (OP_MSG): the command subset of ``mongo_wire.MongoClient``.

Serves tests and single-node deployments that want the reference's MongoDB datastore layout
without a mongod: databases -> collections -> documents by ``_id``, unique (optionally sparse)
indexes with E11000 duplicate-key errors, cursors with getMore, and SCRAM-SHA-256 / SCRAM-SHA-1
authentication when ``users`` is given.  Storage is in memory.

    srv = MiniMongoServer(port=0, users={"sw": "secret"}).start()
    MongoClient(f"mongodb://sw:secret@{srv.address}/tenant?authSource=admin")
"""
from __future__ import annotations

import base64
import hmac
import itertools
import os
import socket
import socketserver
import threading

from . import bson
from .mongo_wire import (DUPLICATE_KEY, OP_MSG, MongoError, _hash, _xor, apply_update, get_path, matches,
                         op_msg, parse_op_msg, read_message, scram_parse, scram_salted_password, sort_docs,
                         _MISSING)


class _Coll:
    def __init__(self):
        self.docs: dict = {}                      # _id key -> document
        self.indexes: dict[str, dict] = {"_id_": {"key": {"_id": 1}, "unique": True, "sparse": False}}
        self.uniq: dict[str, dict] = {}           # unique index name -> value tuple -> _id key

    @staticmethod
    def idkey(v):
        return v.binary if isinstance(v, bson.ObjectId) else (type(v).__name__, v)

    @staticmethod
    def _ukey(doc: dict, ix: dict):
        """Hashable key of ``doc`` in unique index ``ix`` (None: not indexed, sparse and absent)."""
        vals = tuple(get_path(doc, f) for f in ix["key"])
        if ix["sparse"] and all(v is _MISSING for v in vals):
            return None
        vals = tuple(None if v is _MISSING else v for v in vals)
        try:
            hash(vals)
            return vals
        except TypeError:
            return repr(vals)

    def _unique_indexes(self):
        return [(n, ix) for n, ix in self.indexes.items() if ix["unique"] and n != "_id_"]

    def check_unique(self, doc: dict, ignore_id=None):
        """Hash lookups per unique index (a duplicate raises E11000)."""
        for name, ix in self._unique_indexes():
            key = self._ukey(doc, ix)
            if key is None:
                continue
            other = self.uniq.get(name, {}).get(key)
            if other is not None and other != ignore_id:
                raise MongoError(f"E11000 duplicate key error index: {name} dup key: {key}", DUPLICATE_KEY)

    def index_add(self, doc: dict, k):
        for name, ix in self._unique_indexes():
            key = self._ukey(doc, ix)
            if key is not None:
                self.uniq.setdefault(name, {})[key] = k

    def index_remove(self, doc: dict, k):
        for name, ix in self._unique_indexes():
            key = self._ukey(doc, ix)
            m = self.uniq.get(name)
            if key is not None and m is not None and m.get(key) == k:
                del m[key]


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        srv: MiniMongoServer = self.server.mongo       # type: ignore[attr-defined]
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        state = {"authed": not srv.users, "scram": None}
        try:
            while True:
                rid, _, op, body = read_message(sock)
                if op != OP_MSG:
                    return                         # legacy opcodes are not served
                cmd = parse_op_msg(body)
                try:
                    reply = srv.execute(cmd, state)
                except MongoError as e:
                    reply = {"ok": 0.0, "errmsg": str(e), "code": e.code}
                sock.sendall(op_msg(next(srv._ids), reply, rid))
        except (ConnectionError, OSError):
            pass


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class MiniMongoServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 27017, users: dict[str, str] | None = None):
        self.users = dict(users or {})
        self._srv = _Server((host, port), _Handler)
        self._srv.mongo = self
        self.host, self.port = host, self._srv.server_address[1]
        self._dbs: dict[str, dict[str, _Coll]] = {}
        self._cursors: dict[int, list] = {}
        self._cursor_ids = itertools.count(1)
        self._ids = itertools.count(1)
        self._lock = threading.RLock()
        self._salt = {u: os.urandom(16) for u in self.users}

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def start(self):
        threading.Thread(target=self._srv.serve_forever, daemon=True, name="mini-mongo").start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()

    def _coll(self, db: str, name: str, create: bool = True) -> _Coll | None:
        d = self._dbs.setdefault(db, {}) if create else self._dbs.get(db, {})
        c = d.get(name)
        if c is None and create:
            c = d[name] = _Coll()
        return c

    # ------------------------------------------------------------------ commands
    def execute(self, cmd: dict, state: dict) -> dict:
        name = next(iter(cmd))
        db = cmd.get("$db", "test")
        if name in ("hello", "isMaster", "ismaster"):
            return {"isWritablePrimary": True, "ismaster": True, "maxBsonObjectSize": 16 << 20,
                    "maxMessageSizeBytes": 48 << 20, "maxWriteBatchSize": 100000, "minWireVersion": 0,
                    "maxWireVersion": 17, "logicalSessionTimeoutMinutes": 30, "ok": 1.0}
        if name in ("ping", "endSessions", "buildInfo", "buildinfo"):
            return {"ok": 1.0, "version": "6.0.0-sitewhere-amd"} if name.startswith("build") else {"ok": 1.0}
        if name == "saslStart":
            return self._sasl_start(cmd, state)
        if name == "saslContinue":
            return self._sasl_continue(cmd, state)
        if not state["authed"]:
            raise MongoError(f"command {name} requires authentication", 13)
        with self._lock:
            return getattr(self, "_cmd_" + name, self._unknown)(db, cmd)

    def _unknown(self, db, cmd):
        raise MongoError(f"no such command: '{next(iter(cmd))}'", 59)

    def _cmd_insert(self, db, cmd):
        c = self._coll(db, cmd["insert"])
        n = 0
        for d in cmd.get("documents", []):
            d = dict(d)
            if "_id" not in d:
                d["_id"] = bson.ObjectId()
            k = c.idkey(d["_id"])
            if k in c.docs:
                raise MongoError(f"E11000 duplicate key error index: _id_ dup key: {d['_id']}", DUPLICATE_KEY)
            c.check_unique(d)
            c.docs[k] = d
            c.index_add(d, k)
            n += 1
        return {"n": n, "ok": 1.0}

    def _select(self, c: _Coll | None, flt, sort=None, skip=0, limit=0):
        if c is not None and flt and set(flt) == {"_id"} and not isinstance(flt["_id"], dict):
            d = c.docs.get(c.idkey(flt["_id"]))          # by primary key: no scan
            return [d] if d is not None and not skip else []
        docs = [d for d in (c.docs.values() if c else ()) if matches(d, flt)]
        docs = sort_docs(docs, sort)
        if skip:
            docs = docs[skip:]
        if limit:
            docs = docs[:abs(limit)]
        return docs

    def _cmd_find(self, db, cmd):
        c = self._coll(db, cmd["find"], create=False)
        docs = self._select(c, cmd.get("filter"), cmd.get("sort"), int(cmd.get("skip", 0)), int(cmd.get("limit", 0)))
        bs = int(cmd.get("batchSize", 101)) or len(docs)
        return self._cursor_reply(f"{db}.{cmd['find']}", docs, bs, "firstBatch")

    def _cursor_reply(self, ns, docs, bs, key):
        first, rest = docs[:bs], docs[bs:]
        cid = 0
        if rest:
            cid = next(self._cursor_ids)
            self._cursors[cid] = rest
        return {"cursor": {"id": bson.Int64(cid), "ns": ns, key: first}, "ok": 1.0}

    def _cmd_getMore(self, db, cmd):
        cid = int(cmd["getMore"])
        rest = self._cursors.pop(cid, None)
        if rest is None:
            raise MongoError(f"cursor id {cid} not found", 43)
        bs = int(cmd.get("batchSize", 101)) or len(rest)
        reply = self._cursor_reply(f"{db}.{cmd['collection']}", rest, bs, "nextBatch")
        if reply["cursor"]["id"]:                     # keep the same id for the remainder
            self._cursors[cid] = self._cursors.pop(int(reply["cursor"]["id"]))
            reply["cursor"]["id"] = bson.Int64(cid)
        return reply

    def _cmd_killCursors(self, db, cmd):
        for cid in cmd.get("cursors", []):
            self._cursors.pop(int(cid), None)
        return {"ok": 1.0}

    def _cmd_count(self, db, cmd):
        return {"n": len(self._select(self._coll(db, cmd["count"], create=False), cmd.get("query"))), "ok": 1.0}

    def _cmd_update(self, db, cmd):
        c = self._coll(db, cmd["update"])
        n = nmod = 0
        upserted = []
        for i, u in enumerate(cmd.get("updates", [])):
            hits = self._select(c, u.get("q"), limit=0 if u.get("multi") else 1)
            if hits:
                for d in hits:
                    new = apply_update(d, u["u"])
                    k = c.idkey(d["_id"])
                    c.check_unique(new, ignore_id=k)
                    c.index_remove(d, k)
                    c.docs[k] = new
                    c.index_add(new, k)
                    n += 1
                    nmod += 1
            elif u.get("upsert"):
                base = {k: v for k, v in (u.get("q") or {}).items() if not k.startswith("$") and not isinstance(v, dict)}
                new = apply_update(base, u["u"])
                if not any(str(k).startswith("$") for k in u["u"]) and "_id" in base:
                    new["_id"] = base["_id"]
                new.setdefault("_id", bson.ObjectId())
                c.check_unique(new)
                c.docs[c.idkey(new["_id"])] = new
                c.index_add(new, c.idkey(new["_id"]))
                n += 1
                upserted.append({"index": i, "_id": new["_id"]})
        out = {"n": n, "nModified": nmod, "ok": 1.0}
        if upserted:
            out["upserted"] = upserted
        return out

    def _cmd_delete(self, db, cmd):
        c = self._coll(db, cmd["delete"], create=False)
        n = 0
        for d in cmd.get("deletes", []):
            for doc in self._select(c, d.get("q"), limit=int(d.get("limit", 0))):
                k = c.idkey(doc["_id"])
                del c.docs[k]
                c.index_remove(doc, k)
                n += 1
        return {"n": n, "ok": 1.0}

    def _cmd_createIndexes(self, db, cmd):
        c = self._coll(db, cmd["createIndexes"])
        before = len(c.indexes)
        for ix in cmd.get("indexes", []):
            spec = {"key": dict(ix["key"]), "unique": bool(ix.get("unique")), "sparse": bool(ix.get("sparse"))}
            if spec["unique"] and ix["name"] not in c.uniq:
                m: dict = {}
                for k, d in c.docs.items():
                    key = c._ukey(d, spec)
                    if key is None:
                        continue
                    if key in m:
                        raise MongoError(f"E11000 duplicate key error index: {ix['name']} dup key: {key}",
                                         DUPLICATE_KEY)
                    m[key] = k
                c.uniq[ix["name"]] = m
            c.indexes[ix["name"]] = spec
        return {"numIndexesBefore": before, "numIndexesAfter": len(c.indexes), "ok": 1.0}

    def _cmd_listIndexes(self, db, cmd):
        c = self._coll(db, cmd["listIndexes"], create=False)
        items = [{"v": 2, "key": ix["key"], "name": n, **({"unique": True} if ix["unique"] else {})}
                 for n, ix in (c.indexes.items() if c else [])]
        return {"cursor": {"id": bson.Int64(0), "ns": f"{db}.{cmd['listIndexes']}", "firstBatch": items}, "ok": 1.0}

    def _cmd_listCollections(self, db, cmd):
        items = [{"name": n, "type": "collection"} for n in self._dbs.get(db, {})]
        return {"cursor": {"id": bson.Int64(0), "ns": f"{db}.$cmd.listCollections", "firstBatch": items}, "ok": 1.0}

    def _cmd_drop(self, db, cmd):
        if self._dbs.get(db, {}).pop(cmd["drop"], None) is None:
            raise MongoError("ns not found", 26)
        return {"ok": 1.0}

    def _cmd_dropDatabase(self, db, cmd):
        self._dbs.pop(db, None)
        return {"ok": 1.0}

    # ------------------------------------------------------------------ SCRAM (server side)
    def _sasl_start(self, cmd, state):
        mech = cmd.get("mechanism", "")
        if mech not in ("SCRAM-SHA-256", "SCRAM-SHA-1"):
            raise MongoError(f"unsupported mechanism {mech}", 2)
        payload = cmd["payload"]
        if not payload.startswith(b"n,,"):
            raise MongoError("SCRAM: channel binding not supported", 18)
        bare = payload[3:].decode()
        cf = scram_parse(bare.encode())
        user = cf["n"].replace("=2C", ",").replace("=3D", "=")
        if user not in self.users:
            raise MongoError("Authentication failed.", 18)
        nonce = cf["r"] + base64.b64encode(os.urandom(18)).decode()
        salt, iters = self._salt[user], 4096
        server_first = f"r={nonce},s={base64.b64encode(salt).decode()},i={iters}"
        state["scram"] = {"mech": mech, "user": user, "bare": bare, "server_first": server_first, "nonce": nonce,
                          "salt": salt, "iters": iters}
        return {"conversationId": 1, "done": False, "payload": server_first.encode(), "ok": 1.0}

    def _sasl_continue(self, cmd, state):
        sc = state.get("scram")
        if sc is None:
            raise MongoError("no SASL conversation", 17)
        final = cmd["payload"].decode()
        fields = scram_parse(final.encode())
        without_proof = final[:final.rindex(",p=")]
        if fields.get("r") != sc["nonce"]:
            raise MongoError("Authentication failed.", 18)
        H = _hash(sc["mech"])
        salted = scram_salted_password(sc["mech"], sc["user"], self.users[sc["user"]], sc["salt"], sc["iters"])
        stored_key = H(hmac.new(salted, b"Client Key", H).digest()).digest()
        auth_msg = f"{sc['bare']},{sc['server_first']},{without_proof}".encode()
        client_key = _xor(base64.b64decode(fields["p"]), hmac.new(stored_key, auth_msg, H).digest())
        if not hmac.compare_digest(H(client_key).digest(), stored_key):
            raise MongoError("Authentication failed.", 18)
        server_sig = hmac.new(hmac.new(salted, b"Server Key", H).digest(), auth_msg, H).digest()
        state["authed"] = True
        state["scram"] = None                     # clients send skipEmptyExchange: done in one step
        return {"conversationId": 1, "done": True, "payload": f"v={base64.b64encode(server_sig).decode()}".encode(),
                "ok": 1.0}
