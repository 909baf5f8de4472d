"""Shared helpers for service implementations: generic CRUD over an EntityStore, request mapping."""
from __future__ import annotations

import dataclasses

from ..core.errors import ErrorCode, NotFoundException, SiteWhereSystemException
from ..core.security import current_authentication
from ..models.domain import Model, SearchCriteria, SearchResults, snake, stamp_created, stamp_updated
from ..utils import fast_uuid4


def _user():
    a = current_authentication()
    return a.username if a else None


def apply_request(entity: Model, request: dict, skip: tuple = ()) -> Model:
    """Copy camelCase request fields onto a dataclass entity (only keys that are present)."""
    hints = {f.name: f for f in dataclasses.fields(entity)}
    for k, v in (request or {}).items():
        n = snake(k)
        if n in skip or n not in hints or n in ("id", "created_date", "created_by"):
            continue
        cur = getattr(entity, n)
        if isinstance(cur, Model) and isinstance(v, dict):
            v = type(cur).from_dict(v)
        elif dataclasses.is_dataclass(entity):
            from ..models.domain import _deser, _hints
            v = _deser(_hints(type(entity)).get(n), v)
        setattr(entity, n, v)
    return entity


def criteria_of(c) -> SearchCriteria:
    if c is None:
        return SearchCriteria(page_size=0)
    if isinstance(c, dict):
        return SearchCriteria(c.get("pageNumber", 1), c.get("pageSize", 100))
    return c


class Crud:
    """Entity CRUD with token uniqueness and not-found error codes."""

    def __init__(self, store, collection: str, cls: type, not_found: ErrorCode, unique=("token",), indexed=()):
        self.s, self.c, self.cls, self.nf = store, collection, cls, not_found
        store.register(collection, cls, unique, indexed=indexed)

    def create(self, request: dict, **fixed) -> Model:
        e = self.cls()
        apply_request(e, request)
        for k, v in fixed.items():
            setattr(e, k, v)
        if not getattr(e, "token", None):
            e.token = fast_uuid4()
        if self.s.get_by_token(self.c, e.token) is not None:
            raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=f"{self.c} token {e.token} in use")
        stamp_created(e, _user())
        return self.s.put(self.c, e)

    def put(self, e: Model) -> Model:
        return self.s.put(self.c, e)

    def get(self, id: str):
        return self.s.get(self.c, id) if id else None

    def get_by_token(self, token: str):
        return self.s.get_by_token(self.c, token) if token else None

    def require(self, id: str):
        e = self.get(id)
        if e is None:
            raise NotFoundException(self.nf, f"{self.c} id {id}")
        return e

    def require_token(self, token: str):
        e = self.get_by_token(token)
        if e is None:
            raise NotFoundException(self.nf, f"{self.c} token {token}")
        return e

    def update(self, id: str, request: dict, **fixed):
        e = self.require(id)
        new_token = (request or {}).get("token")
        if new_token and new_token != e.token and self.s.get_by_token(self.c, new_token) is not None:
            raise SiteWhereSystemException(ErrorCode.DuplicateToken, detail=new_token)
        apply_request(e, request)
        for k, v in fixed.items():
            setattr(e, k, v)
        stamp_updated(e, _user())
        return self.s.put(self.c, e)

    def delete(self, id: str):
        e = self.require(id)
        self.s.delete(self.c, id)
        return e

    def query(self, pred=None, sort=None, reverse=False):
        return self.s.query(self.c, pred, sort_key=sort or (lambda e: (getattr(e, "created_date", None) or 0, e.id)), reverse=reverse)

    def search(self, q, criteria=None) -> SearchResults:
        """Filter / sort / page pushed down into the store (``persistence/query.py``); the page of
        ``criteria`` (pageNumber / pageSize) is applied there too."""
        c = criteria_of(criteria)
        q.page(c.page_number, c.page_size)
        total, items = self.s.find(self.c, q)
        return SearchResults(total, items)

    def list(self, criteria=None, pred=None, sort=None, reverse=False) -> SearchResults:
        c = criteria_of(criteria)
        items = self.query(pred, sort, reverse)
        return SearchResults(len(items), c.slice(items))
