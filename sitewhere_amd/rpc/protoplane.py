"""The RPC plane on the reference's wire schemas: ``/com.sitewhere.grpc.service.<Service>/<Rpc>``
carrying the ``G*Request`` / ``G*Response`` protobuf messages of ``sitewhere-grpc-*/src/main/proto``
(``rpc/schema/*.proto``, loaded at run time by ``models/protoschema.py`` -- no protoc, no generated
code).  A reference Java client or service can call this framework's services, and its clients can
call a reference service (:class:`ReferenceClient`).

Reference: ``sitewhere-grpc-device-management/src/main/proto/device-management.proto:3-13,136``
(package / service / rpc layout) and the per-service ``*ModelConverter`` classes
(``sitewhere-grpc-device-management/.../DeviceModelConverter.java``: ~20K lines over all services),
which convert every ``G*`` message to the API model and back, field by field.

Here one schema-driven converter does that for all 178 RPCs, from the naming regularities of the
schemas (the same ones the Java converters encode by hand):

* ``GUUID`` <-> id string (a UUID; engine event ids ``<boot hex>-<sequence>`` travel in a UUID
  with version nibble 0xE, see :func:`uuid_of`),
* ``GOptional*`` wrappers <-> plain values (unset wrapper = absent key),
* ``GEntityInformation`` / ``GBrandingInformation`` / ``GDeviceEvent`` /
  ``GDeviceEventCreateRequest`` / ``GPaging`` are flattened into the owning object (the API model
  carries their fields directly: ``PersistentEntity`` / ``BrandedEntity`` / ``DeviceEvent``),
* ``G*Reference { token }`` fields <-> ``<field>Token`` keys (``{ id }`` -> ``<field>Id``;
  username / authority references <-> the plain value),
* enums <-> the API's enum values (``EVENT_INDEX_ASSIGNMENT`` <-> ``"Assignment"``: the common
  value prefix dropped, CamelCase),
* ``G*SearchResults { count, repeated X }`` <-> :class:`~sitewhere_amd.models.domain.SearchResults`.

A request's fields, in declaration order, are the arguments of the snake_case API method (the
transport's mapping); a response's single field receives the result."""
from __future__ import annotations

import functools
import os
import re
import uuid

from google.protobuf import descriptor as _d
from google.protobuf import message_factory

from ..models import domain

SCHEMA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schema")
SERVICE_PKG = "com.sitewhere.grpc.service"
MODEL_PKG = "com.sitewhere.grpc.model"
PATH_PREFIX = SERVICE_PKG + "."

# reference service name -> the name this framework registers it under
SERVICE_ALIASES = {"DeviceState": "DeviceStateManagement"}

_FLATTEN = {f"{MODEL_PKG}.{n}" for n in ("GEntityInformation", "GBrandingInformation", "GDeviceEvent",
                                          "GDeviceEventCreateRequest", "GPaging")}
_UUID = f"{MODEL_PKG}.GUUID"
_ENGINE_ID = re.compile(r"^([0-9a-f]{1,12})-(\d+)$")


@functools.lru_cache(maxsize=1)
def pool():
    from ..models.protoschema import load_proto_files
    files = {}
    for name in sorted(os.listdir(SCHEMA_DIR)):
        if name.endswith(".proto"):
            with open(os.path.join(SCHEMA_DIR, name)) as f:
                files[name] = f.read()
    return load_proto_files(files)


@functools.lru_cache(maxsize=None)
def message_class(full_name: str):
    return message_factory.GetMessageClass(pool().FindMessageTypeByName(full_name))


def services() -> dict:
    """``{service name: ServiceDescriptor}`` of every reference service."""
    out = {}
    p = pool()
    for name in sorted(os.listdir(SCHEMA_DIR)):
        if name.endswith(".proto"):
            for sv in p.FindFileByName(name).services_by_name.values():
                out[sv.name] = sv
    return out


def method(service: str, rpc: str):
    sv = services().get(service)
    return None if sv is None else sv.methods_by_name.get(rpc)


# ---------------------------------------------------------------------------------------- ids
def uuid_of(id_str: str | None) -> tuple[int, int] | None:
    """(msb, lsb) of an id.  UUIDs map directly; an engine event id ``<boot>-<seq>`` becomes a
    UUID with version nibble 0xE (boot in the 48 high bits, sequence in the low half)."""
    if not id_str:
        return None
    try:
        v = uuid.UUID(id_str).int
        return v >> 64, v & ((1 << 64) - 1)
    except (ValueError, AttributeError, TypeError):
        pass
    m = _ENGINE_ID.match(str(id_str))
    if m:
        return (int(m.group(1), 16) << 16) | 0xE000, int(m.group(2))
    raise ValueError(f"id {id_str!r} has no GUUID form")


def id_of(msb: int, lsb: int) -> str | None:
    if not msb and not lsb:
        return None
    if (msb & 0xF000) == 0xE000 and not (msb & 0x0FFF):
        return f"{msb >> 16:x}-{lsb}"
    return str(uuid.UUID(int=(msb << 64) | lsb))


# ---------------------------------------------------------------------------------------- enums
@functools.lru_cache(maxsize=None)
def _enum_maps(full_name: str):
    e = pool().FindEnumTypeByName(full_name)
    names = [v.name for v in e.values]
    prefix = os.path.commonprefix(names) if len(names) > 1 else ""
    prefix = prefix[:prefix.rfind("_") + 1] if "_" in prefix else ""
    to_py, from_py = {}, {}
    for v in e.values:
        rest = v.name[len(prefix):] if prefix and len(v.name) > len(prefix) else v.name
        camel = "".join(p[:1] + p[1:].lower() for p in rest.split("_"))
        to_py[v.number] = None if rest == "UNSPECIFIED" else camel     # proto3 default: "not set"
        from_py[camel.lower()] = v.number
        from_py[rest.lower().replace("_", "")] = v.number
        from_py[v.name.lower()] = v.number
    return to_py, from_py


def enum_to_py(ed, number: int) -> str | None:
    m = _enum_maps(ed.full_name)[0]
    return m[number] if number in m else str(number)


def enum_from_py(ed, value) -> int:
    if isinstance(value, int):
        return value
    if hasattr(value, "value"):
        value = value.value
    key = str(value).lower().replace("_", "")
    n = _enum_maps(ed.full_name)[1].get(key)
    if n is None:
        raise ValueError(f"{value!r} is not a {ed.name}")
    return n


# ---------------------------------------------------------------------------------------- G* -> python
def _is_optional(md) -> bool:
    return md.name.startswith("GOptional") and len(md.fields) == 1 and md.fields[0].name == "value"


def _reference_key(f) -> tuple[str, str] | None:
    """(API key, inner field) of a ``G*Reference`` field."""
    md = f.message_type
    if not md.name.endswith("Reference") or len(md.fields) != 1:
        return None
    inner = md.fields[0].name
    if inner in ("token", "id"):
        return f.name + inner[:1].upper() + inner[1:], inner
    return f.name, inner


def _value_to_py(f, v):
    if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
        md = f.message_type
        if md.full_name == _UUID:
            return id_of(v.msb, v.lsb)
        if _is_optional(md):
            return v.value
        return to_py(v)
    if f.type == _d.FieldDescriptor.TYPE_ENUM:
        return enum_to_py(f.enum_type, v)
    return v


def _rep(f) -> bool:
    return f.is_repeated


def _is_map(f) -> bool:
    return f.type == _d.FieldDescriptor.TYPE_MESSAGE and f.message_type.GetOptions().map_entry


def to_py(msg) -> dict:
    """A ``G*`` message -> the API's camelCase dict (see the module docstring for the rules)."""
    d: dict = {}
    for f in msg.DESCRIPTOR.fields:
        name = f.name
        if _is_map(f):
            vf = f.message_type.fields_by_name["value"]
            m = getattr(msg, name)
            if len(m):
                d[name] = {k: _value_to_py(vf, m[k]) for k in m}
            continue
        if _rep(f):
            vals = getattr(msg, name)
            if len(vals):
                d[name] = [_value_to_py(f, x) for x in vals]
            continue
        if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
            if not msg.HasField(name):
                continue
            sub = getattr(msg, name)
            md = f.message_type
            if md.full_name in _FLATTEN:
                d.update(to_py(sub))
                continue
            ref = _reference_key(f)
            if ref is not None:
                d[ref[0]] = getattr(sub, ref[1])
                continue
            d[name] = _value_to_py(f, sub)
            continue
        if f.type == _d.FieldDescriptor.TYPE_ENUM:
            v = enum_to_py(f.enum_type, getattr(msg, name))
            if v is not None:
                d[name] = v
            continue
        v = getattr(msg, name)
        if v or (f.containing_oneof is not None and msg.HasField(name)):
            d[name] = v
    return d


def arg_of(msg, f):
    """A top-level request field -> the API argument (every field, defaults included)."""
    if _is_map(f):
        vf = f.message_type.fields_by_name["value"]
        return {k: _value_to_py(vf, v) for k, v in getattr(msg, f.name).items()}
    if _rep(f):
        return [_value_to_py(f, x) for x in getattr(msg, f.name)]
    if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
        if not msg.HasField(f.name):
            md = f.message_type
            # an unset request / criteria message is an empty one; ids, wrappers and references
            # are absent values
            plain = md.full_name != _UUID and not _is_optional(md) and _reference_key(f) is None
            return {} if plain else None
        sub = getattr(msg, f.name)
        ref = _reference_key(f)
        if ref is not None:
            return getattr(sub, ref[1])
        return _value_to_py(f, sub)
    if f.type == _d.FieldDescriptor.TYPE_ENUM:
        return enum_to_py(f.enum_type, getattr(msg, f.name))
    return getattr(msg, f.name)


# ---------------------------------------------------------------------------------------- python -> G*
def _plain(obj):
    if isinstance(obj, domain.SearchResults):
        return obj
    if isinstance(obj, domain.Model):
        return obj.to_dict()
    return obj


def _scalar(f, v):
    t = f.type
    if t in (_d.FieldDescriptor.TYPE_DOUBLE, _d.FieldDescriptor.TYPE_FLOAT):
        return float(v)
    if t == _d.FieldDescriptor.TYPE_BOOL:
        return bool(v)
    if t == _d.FieldDescriptor.TYPE_STRING:
        return v if isinstance(v, str) else str(v)
    if t == _d.FieldDescriptor.TYPE_BYTES:
        return bytes(v) if not isinstance(v, str) else v.encode()
    return int(v)


def _set_value(msg, f, v):
    """Set non-repeated field ``f`` of ``msg`` from the API value ``v`` (not None)."""
    if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
        md = f.message_type
        sub = getattr(msg, f.name)
        if md.full_name == _UUID:
            u = uuid_of(v)
            if u is not None:
                sub.msb, sub.lsb = u
        elif _is_optional(md):
            sub.value = _scalar(md.fields[0], v)
        else:
            fill(sub, v)
    elif f.type == _d.FieldDescriptor.TYPE_ENUM:
        setattr(msg, f.name, enum_from_py(f.enum_type, v))
    else:
        setattr(msg, f.name, _scalar(f, v))


def _add_value(container, f, v):
    if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
        md = f.message_type
        sub = container.add()
        if md.full_name == _UUID:
            u = uuid_of(v)
            if u is not None:
                sub.msb, sub.lsb = u
        elif _is_optional(md):
            sub.value = _scalar(md.fields[0], v)
        else:
            fill(sub, v)
    elif f.type == _d.FieldDescriptor.TYPE_ENUM:
        container.append(enum_from_py(f.enum_type, v))
    else:
        container.append(_scalar(f, v))


def fill(msg, obj):
    """Fill a ``G*`` message from an API object (model, dict, SearchResults); returns ``msg``."""
    obj = _plain(obj)
    if obj is None:
        return msg
    if isinstance(obj, domain.SearchResults):
        fields = msg.DESCRIPTOR.fields_by_name
        if "count" in fields:
            msg.count = int(obj.num_results)
        rep = [f for f in msg.DESCRIPTOR.fields if _rep(f)]
        if rep:
            for r in obj.results:
                _add_value(getattr(msg, rep[0].name), rep[0], _plain(r))
        return msg
    if not isinstance(obj, dict):
        fs = msg.DESCRIPTOR.fields
        if len(fs) == 1:                    # a single-valued message (e.g. a reference by token)
            _set_value(msg, fs[0], obj)
            return msg
        raise TypeError(f"cannot convert {type(obj).__name__} to {msg.DESCRIPTOR.name}")
    for f in msg.DESCRIPTOR.fields:
        name = f.name
        if _is_map(f):
            v = obj.get(name)
            if v:
                vf = f.message_type.fields_by_name["value"]
                m = getattr(msg, name)
                for k, x in v.items():
                    if x is None:
                        continue
                    if vf.type == _d.FieldDescriptor.TYPE_MESSAGE:
                        fill(m[str(k)], x)
                    else:
                        m[str(k)] = _scalar(vf, x) if vf.type != _d.FieldDescriptor.TYPE_STRING else str(x)
            continue
        if _rep(f):
            for x in obj.get(name) or []:
                if x is not None:
                    _add_value(getattr(msg, name), f, _plain(x))
            continue
        if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
            md = f.message_type
            if md.full_name in _FLATTEN:
                sub = md.fields
                if any(obj.get(s.name) is not None for s in sub):
                    fill(getattr(msg, name), obj)
                continue
            ref = _reference_key(f)
            if ref is not None:
                v = obj.get(ref[0], obj.get(name) if ref[0] != name else None)
                if isinstance(v, dict):
                    v = v.get(ref[1])
                if v is not None:
                    setattr(getattr(msg, name), ref[1], str(v))
                continue
        v = obj.get(name)
        if v is None:
            continue
        _set_value(msg, f, _plain(v))
    return msg


def request_from_args(md, args: tuple, kwargs: dict):
    """Build a request message of descriptor ``md`` from API call arguments (client side)."""
    msg = message_class(md.full_name)()
    fields = list(md.fields)
    vals = dict(zip([f.name for f in fields], args))
    vals.update(kwargs)
    if len(args) > len(fields) and fields and _rep(fields[-1]):
        vals[fields[-1].name] = list(args[len(fields) - 1:])
    for f in fields:
        v = vals.get(f.name)
        if v is None:
            continue
        if _rep(f) and not _is_map(f):
            for x in (v if isinstance(v, (list, tuple)) else [v]):
                _add_value(getattr(msg, f.name), f, _plain(x))
        elif _is_map(f):
            fill(msg, {f.name: v})
        elif f.type == _d.FieldDescriptor.TYPE_MESSAGE and _reference_key(f) is not None:
            setattr(getattr(msg, f.name), _reference_key(f)[1], str(v))
        else:
            _set_value(msg, f, _plain(v))
    return msg


def set_response(resp, result):
    """Put an API result into a response message (its single field, or its fields)."""
    fields = resp.DESCRIPTOR.fields
    if result is None or not fields:
        return resp
    if len(fields) == 1:
        f = fields[0]
        if _rep(f) and not _is_map(f):
            items = result.results if isinstance(result, domain.SearchResults) else result
            for x in items if isinstance(items, (list, tuple)) else [items]:
                _add_value(getattr(resp, f.name), f, _plain(x))
        else:
            _set_value(resp, f, _plain(result))
        return resp
    return fill(resp, result)


# ---------------------------------------------------------------------------------------- python results
def _model_class(md):
    name = md.name[1:] if md.name.startswith("G") else md.name
    return getattr(domain, name, None)


def result_from_response(resp):
    """Response message -> API result (domain model / SearchResults / list / scalar)."""
    fields = resp.DESCRIPTOR.fields
    if not fields:
        return None
    f = fields[0]
    if len(fields) > 1:
        return to_py(resp)
    if _rep(f) and not _is_map(f):
        if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
            cls = _model_class(f.message_type)
            return [cls.from_dict(to_py(x)) if cls is not None else to_py(x) for x in getattr(resp, f.name)]
        return list(getattr(resp, f.name))
    if f.type == _d.FieldDescriptor.TYPE_MESSAGE:
        if not resp.HasField(f.name):
            return None
        sub = getattr(resp, f.name)
        md = f.message_type
        if md.full_name == _UUID:
            return id_of(sub.msb, sub.lsb)
        if _is_optional(md):
            return sub.value
        if md.name.endswith("SearchResults"):
            rep = [x for x in md.fields if _rep(x)]
            items = []
            if rep:
                cls = _model_class(rep[0].message_type) if rep[0].type == _d.FieldDescriptor.TYPE_MESSAGE else None
                for x in getattr(sub, rep[0].name):
                    if rep[0].type != _d.FieldDescriptor.TYPE_MESSAGE:
                        items.append(x)
                    else:
                        items.append(cls.from_dict(to_py(x)) if cls is not None else to_py(x))
            return domain.SearchResults(int(getattr(sub, "count", len(items))), items)
        cls = _model_class(md)
        d = to_py(sub)
        return cls.from_dict(d) if cls is not None else d
    return arg_of(resp, f)


# ---------------------------------------------------------------------------------------- client
class ReferenceClient:
    """gRPC client on the reference schemas (talks to this framework or to a reference service).

    ``call(service, rpc, request)`` sends a ``G*Request`` and returns the ``G*Response``;
    ``api(service)`` returns a proxy whose snake_case methods take and return API objects, e.g.
    ``api("DeviceManagement").create_device_type({"token": "t", "name": "T"})``."""

    def __init__(self, address: str, jwt: str | None = None, tenant: str | None = None):
        import grpc
        self._grpc = grpc
        self.channel = grpc.insecure_channel(address)
        self.jwt, self.tenant = jwt, tenant
        self._stubs: dict = {}

    def _metadata(self, tenant):
        md = []
        if self.jwt:
            md.append(("authorization", f"Bearer {self.jwt}"))
        if tenant or self.tenant:
            md.append(("tenant", tenant or self.tenant))
        return md

    def call(self, service: str, rpc: str, request, tenant: str | None = None, timeout: float = 30.0):
        md = method(service, rpc)
        if md is None:
            raise KeyError(f"{service}.{rpc} is not a reference rpc")
        key = (service, rpc)
        stub = self._stubs.get(key)
        if stub is None:
            resp_cls = message_class(md.output_type.full_name)
            stub = self._stubs[key] = self.channel.unary_unary(
                f"/{SERVICE_PKG}.{service}/{rpc}", request_serializer=lambda m: m.SerializeToString(),
                response_deserializer=resp_cls.FromString)
        return stub(request, metadata=self._metadata(tenant), timeout=timeout)

    def api(self, service: str, tenant: str | None = None):
        client = self

        class _Proxy:
            def __getattr__(self, name):
                rpc = "".join(p[:1].upper() + p[1:] for p in name.split("_"))
                md = method(service, rpc)
                if md is None:
                    raise AttributeError(f"{service} has no rpc {rpc}")

                def call(*args, **kwargs):
                    req = request_from_args(md.input_type, args, kwargs)
                    return result_from_response(client.call(service, rpc, req, tenant))
                return call
        return _Proxy()

    def close(self):
        self.channel.close()
