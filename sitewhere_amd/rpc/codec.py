"""Wire codec for the RPC plane and bus payloads: JSON with tagged domain models.

Every :class:`~sitewhere_amd.models.domain.Model` travels as ``{"__t": "<ClassName>", ...camelCase}``
and is rebuilt on the other side, so service APIs exchange the same typed objects in-process and
over gRPC.  (The reference used generated protobuf ``G*`` messages + hand-written ``*ModelConverter``
classes per service; one generic codec replaces ~20k lines of converters.)
"""
from __future__ import annotations

import base64
import copy
import dataclasses
import enum
import json

from ..models import domain

_REGISTRY: dict[str, type] = {}


def register_models(module=domain):
    for name in dir(module):
        obj = getattr(module, name)
        if isinstance(obj, type) and issubclass(obj, domain.Model) and obj is not domain.Model:
            _REGISTRY[obj.__name__] = obj


register_models()


def to_wire(obj):
    if isinstance(obj, domain.SearchResults):
        return {"__t": "SearchResults", "numResults": obj.num_results, "results": [to_wire(r) for r in obj.results]}
    if isinstance(obj, domain.Model):
        d = {"__t": type(obj).__name__}
        # one pass over the (cached) fields; nested models keep their own tags (polymorphic fields)
        for name, key in domain._fields(type(obj)):
            v = getattr(obj, name)
            if isinstance(v, domain.Model):
                d[key] = to_wire(v)
            elif isinstance(v, list) and v and isinstance(v[0], domain.Model):
                d[key] = [to_wire(x) for x in v]
            elif isinstance(v, bytes):
                d[key] = {"__b": base64.b64encode(v).decode()}
            else:
                d[key] = domain._ser(v)
        return d
    if isinstance(obj, bytes):
        return {"__b": base64.b64encode(obj).decode()}
    if type(obj).__name__ == "ndarray":         # buffers travel as bytes over the network
        return {"__b": base64.b64encode(obj.tobytes()).decode()}
    if isinstance(obj, enum.Enum):
        return obj.value
    if isinstance(obj, (list, tuple)):
        return [to_wire(x) for x in obj]
    if isinstance(obj, dict):
        return {k: to_wire(v) for k, v in obj.items()}
    return obj


_camel_cache: dict = {}


def _camel_names(cls) -> dict:
    n = _camel_cache.get(cls)
    if n is None:
        n = _camel_cache[cls] = {c: f for f, c in domain._fields(cls)}
    return n


def from_wire(obj):
    if isinstance(obj, list):
        return [from_wire(x) for x in obj]
    if isinstance(obj, dict):
        if "__b" in obj and len(obj) == 1:
            return base64.b64decode(obj["__b"])
        t = obj.get("__t")
        if t == "SearchResults":
            return domain.SearchResults(obj.get("numResults", 0), [from_wire(r) for r in obj.get("results", [])])
        if t is not None and t in _REGISTRY:
            body = {k: (from_wire(v) if isinstance(v, (dict, list)) else v) for k, v in obj.items() if k != "__t"}
            cls = _REGISTRY[t]
            m = cls.from_dict({k: v for k, v in body.items() if not isinstance(v, domain.Model)})
            names = _camel_names(cls)
            for k, v in body.items():
                if k in names and (isinstance(v, (domain.Model, bytes)) or
                                   (isinstance(v, list) and v and isinstance(v[0], domain.Model))):
                    setattr(m, names[k], v)
            return m
        return {k: from_wire(v) for k, v in obj.items()}
    return obj


def dumps(obj) -> bytes:
    return json.dumps(to_wire(obj), separators=(",", ":")).encode()


def loads(b: bytes):
    return from_wire(json.loads(b)) if b else None


_ATOMIC_TYPES = {str, int, float, bool, bytes, type(None)}


def clone(v):
    """Isolation copy with the result of ``loads(dumps(v))`` but no text round trip: models, dicts,
    lists and tuples are copied, scalars / enums / bytes shared.  Co-located services exchange RPC
    arguments and results through this (``LocalChannel`` in ``clone`` mode)."""
    t = type(v)
    if t in _ATOMIC_TYPES or isinstance(v, enum.Enum):
        return v
    if t.__name__ == "ndarray" and not v.flags.writeable:
        return v            # read-only arrays are shared like bytes (zero-copy columnar payloads)
    if t is dict:
        return {k: clone(x) for k, x in v.items()}
    if t is list or t is tuple:
        return [clone(x) for x in v]
    d = getattr(v, "__dict__", None)
    if d is not None and dataclasses.is_dataclass(v):
        o = object.__new__(t)
        o.__dict__.update({k: clone(x) for k, x in d.items()})
        return o
    return copy.deepcopy(v)
