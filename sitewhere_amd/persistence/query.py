"""Structured entity queries pushed down into the datastore.

Reference: ``MongoPersistence.search`` (``sitewhere-mongodb/.../MongoPersistence.java:157``:
``collection.find(query).skip(offset).limit(pageSize).sort(sort)`` plus a count) built by the
services' ``Mongo*Management.list*`` methods (e.g. ``MongoDeviceManagement.java:758-773``).

A :class:`Query` is filters (equality, membership, ranges, null tests) over entity fields, a sort
and a page.  Each store executes it where the data lives -- an indexed candidate set in memory, a
``WHERE ... ORDER BY ... LIMIT/OFFSET`` over indexed columns in SQLite, ``find(filter).sort().skip()
.limit()`` + ``count_documents`` in MongoDB -- so a page costs the page, not the collection.
Field names are the model's attribute names (snake_case)."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field


def norm(v):
    """Stored form of a value (enums by value)."""
    return v.value if isinstance(v, enum.Enum) else v


@dataclass
class Filter:
    field: str
    op: str            # eq | in | gte | lte | null | notnull
    value: object = None

    def test(self, v) -> bool:
        v = norm(v)
        op = self.op
        if op == "eq":
            return v == self.value
        if op == "in":
            return v in self.value
        if op == "null":
            return v is None
        if op == "notnull":
            return v is not None
        if v is None:
            return False
        if op == "gte":
            return v >= self.value
        if op == "lte":
            return v <= self.value
        raise ValueError(f"unknown filter op {op!r}")


@dataclass
class Query:
    filters: list = field(default_factory=list)
    sort: list = field(default_factory=list)        # [(field, descending)]
    skip: int = 0
    limit: int = 0                                  # 0 = everything after skip

    # builders ---------------------------------------------------------------------------
    def eq(self, f: str, v) -> "Query":
        if v is not None:
            self.filters.append(Filter(f, "eq", norm(v)))
        return self

    def in_(self, f: str, values) -> "Query":
        if values is not None:
            self.filters.append(Filter(f, "in", [norm(x) for x in values]))
        return self

    def gte(self, f: str, v) -> "Query":
        if v is not None:
            self.filters.append(Filter(f, "gte", v))
        return self

    def lte(self, f: str, v) -> "Query":
        if v is not None:
            self.filters.append(Filter(f, "lte", v))
        return self

    def null(self, f: str) -> "Query":
        self.filters.append(Filter(f, "null"))
        return self

    def order(self, f: str, descending: bool = False) -> "Query":
        self.sort.append((f, descending))
        return self

    def page(self, page_number: int, page_size: int) -> "Query":
        """1-based page of ``page_size`` (0 = all)."""
        if page_size and page_size > 0:
            self.skip = (max(1, int(page_number or 1)) - 1) * int(page_size)
            self.limit = int(page_size)
        return self

    # evaluation (memory / fallback) ----------------------------------------------------
    def match(self, e) -> bool:
        return all(f.test(getattr(e, f.field, None)) for f in self.filters)

    def sort_items(self, items: list) -> list:
        for f, desc in reversed(self.sort):     # stable multi-key sort, last key first
            items.sort(key=lambda e, f=f: _key(norm(getattr(e, f, None))), reverse=desc)
        return items

    def window(self, items: list) -> list:
        return items[self.skip:self.skip + self.limit] if self.limit else items[self.skip:]

    @property
    def empty(self) -> bool:
        """A membership filter over no values matches nothing."""
        return any(f.op == "in" and not f.value for f in self.filters)


def _key(v):
    # None sorts below every value, like MongoDB / SQLite; mixed types by type name
    return (0, "", 0) if v is None else (1, type(v).__name__, v)
