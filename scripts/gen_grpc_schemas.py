"""Regenerate ``sitewhere_amd/rpc/schema/*.proto`` -- the RPC plane's wire schemas -- from the
reference's gRPC interface definitions (``sitewhere-grpc-*/src/main/proto``).

The schemas are the wire contract (package ``com.sitewhere.grpc.model`` / ``.service``, message
names, field numbers and types): they must equal the reference's for a reference client or service
to talk to this one.  This script parses them (``models/protoschema.py``) and prints every file
back in one canonical layout (no comments or options), so the copies here carry the contract and
nothing else.

    python scripts/gen_grpc_schemas.py /root/reference
"""
from __future__ import annotations

import glob
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from google.protobuf import descriptor_pb2  # noqa: E402

from sitewhere_amd.models.protoschema import _Parser  # noqa: E402

_F = descriptor_pb2.FieldDescriptorProto
_SCALAR = {v: k for k, v in {
    "double": _F.TYPE_DOUBLE, "float": _F.TYPE_FLOAT, "int64": _F.TYPE_INT64, "uint64": _F.TYPE_UINT64,
    "int32": _F.TYPE_INT32, "fixed64": _F.TYPE_FIXED64, "fixed32": _F.TYPE_FIXED32, "bool": _F.TYPE_BOOL,
    "string": _F.TYPE_STRING, "bytes": _F.TYPE_BYTES, "uint32": _F.TYPE_UINT32, "sfixed32": _F.TYPE_SFIXED32,
    "sfixed64": _F.TYPE_SFIXED64, "sint32": _F.TYPE_SINT32, "sint64": _F.TYPE_SINT64}.items()}


def _tname(f, pkg: str) -> str:
    if f.type in _SCALAR:
        return _SCALAR[f.type]
    full = f.type_name.lstrip(".")
    return full[len(pkg) + 1:] if full.startswith(pkg + ".") else full


def _message(m, pkg: str, ind: str, out: list):
    out.append(f"{ind}message {m.name} {{")
    maps = {n.name: n for n in m.nested_type if n.options.map_entry}
    for n in m.nested_type:
        if not n.options.map_entry:
            _message(n, pkg, ind + "  ", out)
    for e in m.enum_type:
        _enum(e, ind + "  ", out)
    oneofs: dict[int, list] = {}
    for f in m.field:
        if f.HasField("oneof_index"):
            oneofs.setdefault(f.oneof_index, []).append(f)
    done = set()
    for f in m.field:
        if f.HasField("oneof_index"):
            if f.oneof_index in done:
                continue
            done.add(f.oneof_index)
            out.append(f"{ind}  oneof {m.oneof_decl[f.oneof_index].name} {{")
            for g in oneofs[f.oneof_index]:
                out.append(f"{ind}    {_tname(g, pkg)} {g.name} = {g.number};")
            out.append(f"{ind}  }}")
            continue
        entry = maps.get(f.type_name.rsplit(".", 1)[-1]) if f.type == _F.TYPE_MESSAGE else None
        if entry is not None:
            k, v = entry.field
            out.append(f"{ind}  map<{_tname(k, pkg)}, {_tname(v, pkg)}> {f.name} = {f.number};")
            continue
        rep = "repeated " if f.label == _F.LABEL_REPEATED else ""
        out.append(f"{ind}  {rep}{_tname(f, pkg)} {f.name} = {f.number};")
    out.append(f"{ind}}}")


def _enum(e, ind: str, out: list):
    out.append(f"{ind}enum {e.name} {{")
    for v in e.value:
        out.append(f"{ind}  {v.name} = {v.number};")
    out.append(f"{ind}}}")


def render(fd, source: str) -> str:
    pkg = fd.package
    out = [f"// Wire schema of the SiteWhere gRPC plane (generated from {source} by",
           "// scripts/gen_grpc_schemas.py: the reference's contract, re-printed without comments).",
           'syntax = "proto3";', "", f"package {pkg};", ""]
    out += [f'import "{d.replace("-", "_")}";' for d in fd.dependency]
    if fd.dependency:
        out.append("")
    for e in fd.enum_type:
        _enum(e, "", out)
    for m in fd.message_type:
        _message(m, pkg, "", out)
    for sv in fd.service:
        out.append(f"service {sv.name} {{")
        for m in sv.method:
            out.append(f"  rpc {m.name} ({_tname_s(m.input_type, pkg)}) returns ({_tname_s(m.output_type, pkg)});")
        out.append("}")
    return "\n".join(out) + "\n"


def _tname_s(full: str, pkg: str) -> str:
    full = full.lstrip(".")
    return full[len(pkg) + 1:] if full.startswith(pkg + ".") else full


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    paths = sorted(set(glob.glob(os.path.join(ref, "sitewhere-grpc-*/src/main/proto/*.proto"))))
    paths = [p for p in paths if os.path.basename(p) != "sitewhere-kafka.proto"]   # models/proto/kafka_payloads.proto
    parsers = {os.path.basename(p): (_Parser(open(p).read(), os.path.basename(p)).parse(), p) for p in paths}
    enums = set().union(*(pp._enums for pp, _ in parsers.values()))
    msgs = set().union(*(pp._messages for pp, _ in parsers.values()))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sitewhere_amd", "rpc", "schema")
    os.makedirs(dst, exist_ok=True)
    for name, (pp, path) in parsers.items():
        fd = pp.resolve_all(enums, msgs)
        with open(os.path.join(dst, name.replace("-", "_")), "w") as f:
            f.write(render(fd, os.path.relpath(path, ref)))
    print(f"wrote {len(parsers)} schemas to {os.path.normpath(dst)}")


if __name__ == "__main__":
    main()
