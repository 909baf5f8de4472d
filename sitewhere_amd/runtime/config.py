"""Configuration: templated JSON/YAML documents, instance/tenant templates, UI configuration model.

Reference tiers:
  1. process flags: ``instance/InstanceSettings.java:21-63`` (``sitewhere.instance.id``, ports, ...)
  2. instance configuration in ZooKeeper ``/<product>/<instance>/conf/*.xml`` with ``${prop:default}``
     placeholders, copied from a template on first boot (``InstanceManagementMicroservice.java:309-325``)
  3. tenant configuration ``/conf/tenants/<id>/<service>.xml`` from a tenant template, ``[[tenant.id]]``
     substitution (``TenantBootstrapModelConsumer.java:40-225``)
Spring XML + 22 XSDs are replaced by typed JSON documents; the ``*ModelProvider`` role/element
trees the admin UI consumes are kept as :class:`ConfigurationModel`.
"""
from __future__ import annotations

import copy
import json
import os
import re
from dataclasses import dataclass, field

import yaml

_PROP = re.compile(r"\$\{([^}:]+)(?::([^}]*))?\}")
_TENANT = re.compile(r"\[\[([a-zA-Z0-9_.]+)\]\]")


def substitute(value, props: dict | None = None, tenant: dict | None = None):
    """Recursively resolve ``${name:default}`` (props, then env) and ``[[tenant.x]]`` placeholders."""
    props = props or {}
    tenant = tenant or {}
    if isinstance(value, str):
        def rp(m):
            name, default = m.group(1), m.group(2)
            if name in props:
                return str(props[name])
            env = os.environ.get(name.upper().replace(".", "_"))
            if env is not None:
                return env
            return default if default is not None else m.group(0)

        def rt(m):
            key = m.group(1)
            return str(tenant.get(key, tenant.get(key.split(".", 1)[-1], m.group(0))))

        out = _TENANT.sub(rt, _PROP.sub(rp, value))
        # typed scalars when the whole string was a placeholder
        if out != value and _PROP.fullmatch(value or "") is not None:
            for cast in (int, float):
                try:
                    return cast(out)
                except ValueError:
                    pass
            if out in ("true", "false"):
                return out == "true"
        return out
    if isinstance(value, list):
        return [substitute(v, props, tenant) for v in value]
    if isinstance(value, dict):
        return {k: substitute(v, props, tenant) for k, v in value.items()}
    return value


def parse_document(data: bytes | str) -> dict:
    if isinstance(data, bytes):
        data = data.decode()
    data = data.strip()
    if not data:
        return {}
    if data[0] in "{[":
        return json.loads(data)
    return yaml.safe_load(data) or {}


def dump_document(doc: dict) -> bytes:
    return json.dumps(doc, indent=2, sort_keys=True).encode()


@dataclass
class InstanceSettings:
    """Process-level settings (env ``SITEWHERE_*`` overrides; reference defaults)."""
    product_id: str = "sitewhere"
    instance_id: str = "sitewhere1"
    grpc_port: int = 0
    management_grpc_port: int = 0
    # gRPC bind address, and the address other processes are told to dial (topology apiAddress);
    # an empty advertise address means the bind address, or this host's name when binding 0.0.0.0
    # (one container / pod per service, as the reference deploys)
    grpc_host: str = "127.0.0.1"
    grpc_advertise_host: str = ""
    heartbeat_s: float = 20.0
    topology_eviction_s: float = 60.0
    log_metrics: bool = False
    metrics_period_s: float = 20.0
    tracer_sample_rate: float = 0.01
    # reference sitewhere.tracer.server: "host[:port]" -> Jaeger agent (UDP compact emitBatch, 6831);
    # "http(s)://host:4318" -> OTLP/HTTP JSON; empty -> spans stay in the in-process ring only
    tracer_server: str = ""
    # co-located RPC isolation: "clone" (structural copy) or "codec" (full JSON wire round trip)
    local_rpc: str = "clone"
    filesystem_storage_root: str = "/tmp/sitewhere"
    tenant_ops_threads: int = 5
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls, **over):
        s = cls(**over)
        for f in ("product_id", "instance_id", "filesystem_storage_root", "tracer_server", "local_rpc", "grpc_host",
                  "grpc_advertise_host"):
            v = os.environ.get("SITEWHERE_" + f.upper())
            if v:
                setattr(s, f, v)
        for f in ("grpc_port", "management_grpc_port"):
            v = os.environ.get("SITEWHERE_" + f.upper())
            if v:
                setattr(s, f, int(v))
        v = os.environ.get("SITEWHERE_TRACER_SAMPLE_RATE")
        if v:
            s.tracer_sample_rate = float(v)
        return s


# ------------------------------------------------------------------------------ configuration model
@dataclass
class AttributeNode:
    name: str
    type: str = "String"        # String | Integer | Decimal | Boolean | Script | DeviceTypeReference ...
    description: str = ""
    required: bool = False
    default: object = None
    choices: list = field(default_factory=list)


@dataclass
class ElementNode:
    name: str
    role: str
    description: str = ""
    attributes: list[AttributeNode] = field(default_factory=list)
    children: list["ElementNode"] = field(default_factory=list)


@dataclass
class ConfigurationModel:
    microservice: str
    name: str
    root: ElementNode
    roles: dict = field(default_factory=dict)

    def to_dict(self) -> dict:
        def el(e: ElementNode):
            return {"name": e.name, "role": e.role, "description": e.description,
                    "attributes": [a.__dict__ for a in e.attributes], "children": [el(c) for c in e.children]}
        return {"microservice": self.microservice, "name": self.name, "root": el(self.root), "roles": self.roles}

    def validate(self, doc: dict) -> list[str]:
        """Check required attributes of the root element against a configuration document."""
        errs = []
        for a in self.root.attributes:
            if a.required and a.name not in doc:
                errs.append(f"missing required attribute {a.name}")
        return errs


def simple_model(identifier: str, title: str, attrs: list[tuple], children: list[ElementNode] | None = None):
    return ConfigurationModel(identifier, title, ElementNode(title, identifier, attributes=[
        AttributeNode(*a) if isinstance(a, tuple) else a for a in attrs], children=children or []))


def deep_merge(base: dict, over: dict) -> dict:
    out = copy.deepcopy(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out
