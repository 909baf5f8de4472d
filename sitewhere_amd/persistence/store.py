"""Entity persistence: one document-store interface with in-memory and SQLite backends.

Reference: the per-service ``persistence/mongodb/*`` implementations over ``sitewhere-mongodb``
(``MongoDbClient``, ``MongoPersistence``) and the datastore selection of
``DatastoreConfigurationType.java:18-33``.  :class:`MongoEntityStore` talks to MongoDB through the
native wire-protocol client (``mongo_wire.py``, SCRAM auth, no driver dependency); the in-memory
store backs tests and single-process deployments, SQLite gives a durable zero-dependency store.
"""
from __future__ import annotations

import copy
import enum
import dataclasses
import json
import sqlite3
import threading
from typing import Callable, Iterable

from ..models.domain import Model, camel
from .query import Query, norm


_ATOMIC = (str, int, float, bool, bytes, type(None), enum.Enum)


def _clone(v):
    """Isolation copy of a stored entity: dataclass models, dicts and lists are copied, everything
    else is immutable.  ~10x cheaper than ``copy.deepcopy`` (no memo, no reduce protocol) -- it runs
    on every read and write of the in-memory store."""
    if isinstance(v, _ATOMIC):
        return v
    if isinstance(v, dict):
        return {k: _clone(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_clone(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_clone(x) for x in v)
    d = getattr(v, "__dict__", None)
    if d is not None and dataclasses.is_dataclass(v):
        o = object.__new__(type(v))
        o.__dict__.update({k: _clone(x) for k, x in d.items()})
        return o
    return copy.deepcopy(v)


class EntityStore:
    """Collections of :class:`Model` documents addressed by id and (optionally) unique token.

    ``indexed`` fields (``register``) are the ones :meth:`find` filters and sorts on where the data
    lives; ``loads`` counts the documents a store materialised (deserialised / copied) for callers."""

    loads = 0

    def register(self, collection: str, cls: type[Model], unique_fields: Iterable[str] = ("token",),
                 indexed: Iterable[str] = ()):
        raise NotImplementedError

    def find(self, collection: str, q: Query) -> tuple[int, list]:
        """(total matches, the page of ``q``): filtered, sorted and paged by the store."""
        items = self.query(collection, q.match)
        q.sort_items(items)
        return len(items), q.window(items)

    def put_many(self, collection: str, entities: list):
        for e in entities:
            self.put(collection, e)

    def put(self, collection: str, entity: Model) -> Model:
        raise NotImplementedError

    def get(self, collection: str, id: str) -> Model | None:
        raise NotImplementedError

    def get_by(self, collection: str, field: str, value) -> Model | None:
        raise NotImplementedError

    def get_by_token(self, collection: str, token: str) -> Model | None:
        return self.get_by(collection, "token", token)

    def delete(self, collection: str, id: str) -> Model | None:
        raise NotImplementedError

    def query(self, collection: str, predicate: Callable[[Model], bool] | None = None,
              sort_key: Callable[[Model], object] | None = None, reverse: bool = False) -> list:
        raise NotImplementedError

    def count(self, collection: str) -> int:
        return len(self.query(collection))

    def clear(self):
        raise NotImplementedError


class MemoryEntityStore(EntityStore):
    def __init__(self):
        self._lock = threading.RLock()
        self._data: dict[str, dict[str, Model]] = {}
        self._idx: dict[str, dict[str, dict]] = {}
        self._unique: dict[str, tuple] = {}
        self._sec: dict[str, dict[str, dict]] = {}      # collection -> field -> value -> {ids}
        self.loads = 0

    def register(self, collection, cls, unique_fields=("token",), indexed=()):
        with self._lock:
            self._data.setdefault(collection, {})
            self._unique[collection] = tuple(unique_fields)
            self._idx.setdefault(collection, {f: {} for f in unique_fields})
            sec = self._sec.setdefault(collection, {})
            for f in indexed:
                if f not in sec:
                    ix = sec[f] = {}
                    for e in self._data[collection].values():
                        ix.setdefault(norm(getattr(e, f, None)), set()).add(e.id)

    def _sec_update(self, collection, old, new):
        for f, ix in self._sec.get(collection, {}).items():
            if old is not None:
                s_ = ix.get(norm(getattr(old, f, None)))
                if s_ is not None:
                    s_.discard(old.id)
            if new is not None:
                ix.setdefault(norm(getattr(new, f, None)), set()).add(new.id)

    def _coll(self, c):
        if c not in self._data:
            self.register(c, Model)
        return self._data[c]

    def put(self, collection, entity):
        with self._lock:
            data = self._coll(collection)
            old = data.get(entity.id)
            for f in self._unique.get(collection, ()):
                idx = self._idx[collection][f]
                if old is not None:
                    ov = getattr(old, f, None)
                    if ov is not None and idx.get(ov) == old.id:
                        del idx[ov]
                v = getattr(entity, f, None)
                if v is not None:
                    other = idx.get(v)
                    if other is not None and other != entity.id:
                        from ..core.errors import ErrorCode, SiteWhereSystemException
                        raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"{collection}.{f}={v} exists")
                    idx[v] = entity.id
            data[entity.id] = _clone(entity)
            self._sec_update(collection, old, data[entity.id])
            return _clone(entity)

    def get(self, collection, id):
        with self._lock:
            e = self._coll(collection).get(id)
            return _clone(e) if e is not None else None

    def get_by(self, collection, field, value):
        with self._lock:
            self._coll(collection)
            idx = self._idx.get(collection, {}).get(field)
            if idx is not None:
                i = idx.get(value)
                return self.get(collection, i) if i is not None else None
            for e in self._data[collection].values():
                if getattr(e, field, None) == value:
                    return _clone(e)
            return None

    def delete(self, collection, id):
        with self._lock:
            e = self._coll(collection).pop(id, None)
            if e is not None:
                for f in self._unique.get(collection, ()):
                    v = getattr(e, f, None)
                    if v is not None:
                        self._idx[collection][f].pop(v, None)
                self._sec_update(collection, e, None)
            return e

    def put_many(self, collection, entities):
        """Bulk insert of entities handed over by the caller (kept without a copy)."""
        with self._lock:
            data = self._coll(collection)
            uniq = self._unique.get(collection, ())
            for e in entities:
                for f in uniq:
                    v = getattr(e, f, None)
                    if v is not None:
                        other = self._idx[collection][f].get(v)
                        if other is not None and other != e.id:
                            from ..core.errors import ErrorCode, SiteWhereSystemException
                            raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"{collection}.{f}={v} exists")
                old = data.get(e.id)
                if old is not None:
                    for f in uniq:
                        ov = getattr(old, f, None)
                        if ov is not None and self._idx[collection][f].get(ov) == old.id:
                            del self._idx[collection][f][ov]
                for f in uniq:
                    v = getattr(e, f, None)
                    if v is not None:
                        self._idx[collection][f][v] = e.id
                data[e.id] = e
                self._sec_update(collection, old, e)

    def find(self, collection, q):
        if q.empty:
            return 0, []
        with self._lock:
            data = self._coll(collection)
            sec = self._sec.get(collection, {})
            cand = None
            for f in q.filters:                 # intersect the indexed equality / membership sets
                ix = sec.get(f.field)
                if ix is None or f.op not in ("eq", "in", "null"):
                    continue
                vals = [f.value] if f.op == "eq" else (f.value if f.op == "in" else [None])
                ids = set().union(*(ix.get(v, ()) for v in vals)) if vals else set()
                cand = ids if cand is None else cand & ids
            items = [data[i] for i in cand] if cand is not None else list(data.values())
            matched = [e for e in items if q.match(e)]
            q.sort_items(matched)
            page = q.window(matched)
            self.loads += len(page)
            return len(matched), [_clone(e) for e in page]

    def query(self, collection, predicate=None, sort_key=None, reverse=False):
        with self._lock:
            items = [e for e in self._coll(collection).values() if predicate is None or predicate(e)]
            items = [_clone(e) for e in items]
        if sort_key is not None:
            items.sort(key=sort_key, reverse=reverse)
        return items

    def count(self, collection):
        with self._lock:
            return len(self._coll(collection))

    def clear(self):
        with self._lock:
            for c in self._data:
                self._data[c].clear()
                for f in self._idx[c]:
                    self._idx[c][f].clear()
                for ix in self._sec.get(c, {}).values():
                    ix.clear()


class SQLiteEntityStore(EntityStore):
    """Durable JSON-document store (one table per collection, unique-field indexes)."""

    def __init__(self, path: str = ":memory:"):
        self.path = path
        self._lock = threading.RLock()
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._cls: dict[str, type] = {}
        self._unique: dict[str, tuple] = {}
        self._indexed: dict[str, tuple] = {}
        self.loads = 0

    def _t(self, c):
        return "c_" + "".join(ch if ch.isalnum() else "_" for ch in c)

    def register(self, collection, cls, unique_fields=("token",), indexed=()):
        with self._lock:
            self._cls[collection] = cls
            self._unique[collection] = tuple(unique_fields)
            t = self._t(collection)
            cols = "".join(f", u_{f} TEXT" for f in unique_fields)
            self._db.execute(f"CREATE TABLE IF NOT EXISTS {t} (id TEXT PRIMARY KEY, doc TEXT NOT NULL{cols})")
            for f in unique_fields:
                self._db.execute(f"CREATE UNIQUE INDEX IF NOT EXISTS {t}_u_{f} ON {t}(u_{f})")
            # indexed fields: a column each (filled on put), so WHERE / ORDER BY run on B-trees
            have = {r[1] for r in self._db.execute(f"PRAGMA table_info({t})")}
            new = [f for f in indexed if f"x_{f}" not in have]
            for f in new:
                self._db.execute(f"ALTER TABLE {t} ADD COLUMN x_{f}")
            for f in indexed:
                self._db.execute(f"CREATE INDEX IF NOT EXISTS {t}_x_{f} ON {t}(x_{f})")
            prev = self._indexed.get(collection, ())
            self._indexed[collection] = tuple(dict.fromkeys(tuple(prev) + tuple(indexed)))
            if new:                     # backfill documents written before the column existed
                for rid, doc in self._db.execute(f"SELECT id, doc FROM {t}").fetchall():
                    e = cls.from_dict(json.loads(doc))
                    self._db.execute(f"UPDATE {t} SET " + ", ".join(f"x_{f}=?" for f in new) + " WHERE id=?",
                                     [norm(getattr(e, f, None)) for f in new] + [rid])

    def _row(self, collection, entity):
        uf, xf = self._unique[collection], self._indexed.get(collection, ())
        cols = "".join(f", u_{f}" for f in uf) + "".join(f", x_{f}" for f in xf)
        vals = [getattr(entity, f, None) for f in uf] + [norm(getattr(entity, f, None)) for f in xf]
        return cols, vals

    def _ensure(self, c):
        if c not in self._cls:
            raise KeyError(f"collection {c!r} not registered")

    def put(self, collection, entity):
        self._ensure(collection)
        with self._lock:
            t = self._t(collection)
            uf = self._unique[collection]
            vals = [getattr(entity, f, None) for f in uf]
            cols = "".join(f", u_{f}" for f in uf)
            qs = "".join(", ?" for _ in uf)
            for f, v in zip(uf, vals):
                if v is None:
                    continue
                r = self._db.execute(f"SELECT id FROM {t} WHERE u_{f}=?", (v,)).fetchone()
                if r and r[0] != entity.id:
                    from ..core.errors import ErrorCode, SiteWhereSystemException
                    raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"{collection}.{f}={v} exists")
            cols, vals = self._row(collection, entity)
            qs = "".join(", ?" for _ in vals)
            try:
                self._db.execute(f"INSERT OR REPLACE INTO {t} (id, doc{cols}) VALUES (?, ?{qs})",
                                 [entity.id, json.dumps(entity.to_dict())] + vals)
            except sqlite3.IntegrityError as e:
                from ..core.errors import ErrorCode, SiteWhereSystemException
                raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=str(e)) from e
        return entity

    def _load(self, collection, doc):
        self.loads += 1
        return self._cls[collection].from_dict(json.loads(doc))

    def put_many(self, collection, entities):
        """Bulk insert/replace in one transaction (no per-row uniqueness pre-check: the unique
        indexes still reject duplicates)."""
        self._ensure(collection)
        t = self._t(collection)
        with self._lock:
            rows = []
            for e in entities:
                cols, vals = self._row(collection, e)
                rows.append([e.id, json.dumps(e.to_dict())] + vals)
            if not rows:
                return
            qs = "".join(", ?" for _ in rows[0][2:])
            self._db.execute("BEGIN")
            try:
                self._db.executemany(f"INSERT OR REPLACE INTO {t} (id, doc{cols}) VALUES (?, ?{qs})", rows)
                self._db.execute("COMMIT")
            except Exception:
                self._db.execute("ROLLBACK")
                raise

    def _col(self, collection, f):
        if f in self._indexed.get(collection, ()):
            return f"x_{f}"
        if f in self._unique.get(collection, ()):
            return f"u_{f}"
        if f == "id":
            return "id"
        return f"json_extract(doc, '$.{camel(f)}')"

    def find(self, collection, q):
        self._ensure(collection)
        if q.empty:
            return 0, []
        t = self._t(collection)
        where, params = [], []
        for f in q.filters:
            col = self._col(collection, f.field)
            if f.op == "eq":
                where.append(f"{col} = ?")
                params.append(f.value)
            elif f.op == "in":
                where.append(f"{col} IN ({', '.join('?' for _ in f.value)})")
                params.extend(f.value)
            elif f.op == "gte":
                where.append(f"{col} >= ?")
                params.append(f.value)
            elif f.op == "lte":
                where.append(f"{col} <= ?")
                params.append(f.value)
            elif f.op == "null":
                where.append(f"{col} IS NULL")
            elif f.op == "notnull":
                where.append(f"{col} IS NOT NULL")
        w = (" WHERE " + " AND ".join(where)) if where else ""
        order = ", ".join(f"{self._col(collection, f)} {'DESC' if d else 'ASC'}" for f, d in q.sort)
        sql = f"SELECT doc FROM {t}{w}" + (f" ORDER BY {order}" if order else "")
        if q.limit or q.skip:
            sql += f" LIMIT {int(q.limit) if q.limit else -1} OFFSET {int(q.skip)}"
        with self._lock:
            total = self._db.execute(f"SELECT COUNT(*) FROM {t}{w}", params).fetchone()[0]
            rows = self._db.execute(sql, params).fetchall()
        return total, [self._load(collection, r[0]) for r in rows]

    def get(self, collection, id):
        self._ensure(collection)
        with self._lock:
            r = self._db.execute(f"SELECT doc FROM {self._t(collection)} WHERE id=?", (id,)).fetchone()
        return self._load(collection, r[0]) if r else None

    def get_by(self, collection, field, value):
        self._ensure(collection)
        if field in self._unique[collection]:
            with self._lock:
                r = self._db.execute(f"SELECT doc FROM {self._t(collection)} WHERE u_{field}=?", (value,)).fetchone()
            return self._load(collection, r[0]) if r else None
        for e in self.query(collection):
            if getattr(e, field, None) == value:
                return e
        return None

    def delete(self, collection, id):
        e = self.get(collection, id)
        if e is not None:
            with self._lock:
                self._db.execute(f"DELETE FROM {self._t(collection)} WHERE id=?", (id,))
        return e

    def query(self, collection, predicate=None, sort_key=None, reverse=False):
        self._ensure(collection)
        with self._lock:
            rows = self._db.execute(f"SELECT doc FROM {self._t(collection)}").fetchall()
        items = [self._load(collection, r[0]) for r in rows]
        if predicate is not None:
            items = [e for e in items if predicate(e)]
        if sort_key is not None:
            items.sort(key=sort_key, reverse=reverse)
        return items

    def count(self, collection):
        self._ensure(collection)
        with self._lock:
            return self._db.execute(f"SELECT COUNT(*) FROM {self._t(collection)}").fetchone()[0]

    def clear(self):
        with self._lock:
            for c in self._cls:
                self._db.execute(f"DELETE FROM {self._t(c)}")


class MongoEntityStore(EntityStore):
    """MongoDB backend (the reference default) over the native wire-protocol client
    (``persistence/mongo_wire.py``; no driver dependency).  One collection per entity type, ``_id`` =
    entity id, unique sparse indexes on the unique fields (E11000 -> DuplicateToken)."""

    def __init__(self, uri: str = "mongodb://localhost:27017", database: str = "sitewhere", timeout_ms: int = 3000):
        from .mongo_wire import MongoClient
        self._client = MongoClient(uri, timeout_s=timeout_ms / 1000.0)
        self._db = self._client[database]
        self._cls: dict[str, type] = {}
        self._unique: dict[str, tuple] = {}
        self.loads = 0

    def register(self, collection, cls, unique_fields=("token",), indexed=()):
        self._cls[collection] = cls
        self._unique[collection] = tuple(unique_fields)
        for f in unique_fields:
            self._db[collection].create_index({camel(f): 1}, unique=True, sparse=True)
        for f in indexed:
            self._db[collection].create_index({camel(f): 1})

    def put_many(self, collection, entities):
        docs = []
        for e in entities:
            d = e.to_dict()
            d["_id"] = e.id
            docs.append(d)
        for i in range(0, len(docs), 5000):       # new entities (bulk load): plain inserts
            self._db[collection].insert_many(docs[i:i + 5000])

    @staticmethod
    def _filter(q) -> dict:
        flt: dict = {}
        for f in q.filters:
            key = "_id" if f.field == "id" else camel(f.field)
            cond = flt.setdefault(key, {})
            if f.op == "eq":
                cond["$eq"] = f.value
            elif f.op == "in":
                cond["$in"] = list(f.value)
            elif f.op == "gte":
                cond["$gte"] = f.value
            elif f.op == "lte":
                cond["$lte"] = f.value
            elif f.op == "null":
                cond["$eq"] = None
            elif f.op == "notnull":
                cond["$ne"] = None
        return flt

    def find(self, collection, q):
        if q.empty:
            return 0, []
        flt = self._filter(q)
        sort = {("_id" if f == "id" else camel(f)): (-1 if d else 1) for f, d in q.sort} or None
        c = self._db[collection]
        total = c.count_documents(flt)
        docs = c.find(flt, sort, skip=q.skip, limit=q.limit)
        return total, [self._load(collection, d) for d in docs]

    def put(self, collection, entity):
        from .mongo_wire import DUPLICATE_KEY, MongoError
        d = entity.to_dict()
        d["_id"] = entity.id
        try:
            self._db[collection].replace_one({"_id": entity.id}, d, upsert=True)
        except MongoError as e:
            if e.code == DUPLICATE_KEY:
                from ..core.errors import ErrorCode, SiteWhereSystemException
                raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=str(e)) from e
            raise
        return entity

    def _load(self, collection, d):
        if d is None:
            return None
        self.loads += 1
        d = dict(d)
        d.pop("_id", None)
        return self._cls[collection].from_dict(d)

    def get(self, collection, id):
        return self._load(collection, self._db[collection].find_one({"_id": id}))

    def get_by(self, collection, field, value):
        return self._load(collection, self._db[collection].find_one({camel(field): value}))

    def delete(self, collection, id):
        e = self.get(collection, id)
        self._db[collection].delete_one({"_id": id})
        return e

    def query(self, collection, predicate=None, sort_key=None, reverse=False):
        items = [self._load(collection, d) for d in self._db[collection].find({})]
        if predicate is not None:
            items = [e for e in items if predicate(e)]
        if sort_key is not None:
            items.sort(key=sort_key, reverse=reverse)
        return items

    def count(self, collection):
        return self._db[collection].count_documents({})

    def clear(self):
        for c in self._cls:
            self._db[c].delete_many({})


def create_store(kind: str = "memory", **kw) -> EntityStore:
    """Datastore factory (reference DatastoreConfigurationParser): memory | sqlite | mongodb."""
    kind = (kind or "memory").lower()
    if kind == "memory":
        return MemoryEntityStore()
    if kind == "sqlite":
        return SQLiteEntityStore(kw.get("path", ":memory:"))
    if kind in ("mongo", "mongodb"):
        return MongoEntityStore(kw.get("uri", "mongodb://localhost:27017"), kw.get("database", "sitewhere"))
    raise ValueError(f"unknown datastore type {kind!r}")
