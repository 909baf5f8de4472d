"""Load a ``.proto`` (proto3 subset) into protobuf message classes at run time -- no protoc.

Supports what this framework's interface schemas use: ``syntax``, ``package``, top-level and
nested ``message`` / ``enum``, scalar / message / enum fields, ``repeated``, ``map<k, v>``,
``oneof`` and ``service`` / ``rpc`` (unary).  :func:`load_proto` takes one self-contained file;
:func:`load_proto_files` a set of files that ``import`` each other (names resolve across files,
innermost scope first, as protoc does).
"""
from __future__ import annotations

import re

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto
_SCALARS = {
    "double": _F.TYPE_DOUBLE, "float": _F.TYPE_FLOAT, "int64": _F.TYPE_INT64, "uint64": _F.TYPE_UINT64,
    "int32": _F.TYPE_INT32, "fixed64": _F.TYPE_FIXED64, "fixed32": _F.TYPE_FIXED32, "bool": _F.TYPE_BOOL,
    "string": _F.TYPE_STRING, "bytes": _F.TYPE_BYTES, "uint32": _F.TYPE_UINT32, "sfixed32": _F.TYPE_SFIXED32,
    "sfixed64": _F.TYPE_SFIXED64, "sint32": _F.TYPE_SINT32, "sint64": _F.TYPE_SINT64,
}
_TOKEN = re.compile(r'\s*(?:(//[^\n]*)|(/\*.*?\*/)|("(?:[^"\\]|\\.)*")|([A-Za-z_][\w.]*)|(-?\d+)|(.))', re.S)


def _tokens(text: str) -> list[str]:
    out = []
    for m in _TOKEN.finditer(text):
        if m.group(1) or m.group(2):
            continue
        tok = m.group(3) or m.group(4) or m.group(5) or m.group(6)
        if tok and not tok.isspace():
            out.append(tok)
    return out


class _Parser:
    def __init__(self, text: str, name: str):
        self.t, self.i = _tokens(text), 0
        self.fd = descriptor_pb2.FileDescriptorProto(name=name, syntax="proto3")
        self._enums: set[str] = set()        # fully qualified enum names
        self._messages: set[str] = set()     # fully qualified message names
        self._fields: list = []              # (field proto, type name, scope) resolved at the end
        self._methods: list = []             # (method proto, input name, output name, scope)

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, want: str | None = None) -> str:
        tok = self.t[self.i]
        if want is not None and tok != want:
            raise SyntaxError(f"expected {want!r}, got {tok!r} at token {self.i}")
        self.i += 1
        return tok

    def parse(self):
        while self.peek() is not None:
            tok = self.take()
            if tok == "syntax":
                self.take("=")
                if self.take().strip('"') != "proto3":
                    raise SyntaxError("only proto3 schemas are supported")
                self.take(";")
            elif tok == "package":
                self.fd.package = self.take()
                self.take(";")
            elif tok == "import":
                dep = self.take().strip('"')
                while self.take() != ";":
                    pass
                if not dep.startswith("google/"):
                    self.fd.dependency.append(dep)
            elif tok == "option":
                while self.take() != ";":
                    pass
            elif tok == "message":
                self.message(self.fd.message_type.add(), self.fd.package)
            elif tok == "enum":
                self.enum(self.fd.enum_type.add(), self.fd.package)
            elif tok == "service":
                self.service(self.fd.service.add())
            else:
                raise SyntaxError(f"unexpected {tok!r}")
        return self

    def resolve_all(self, enums: set, messages: set):
        """Resolve field / method types against the symbols of every file loaded together."""
        self._enums_all, self._messages_all = enums, messages
        for f, tname, scope in self._fields:
            self._resolve(f, tname, scope)
        for m, tin, tout, scope in self._methods:
            m.input_type = self._resolve_message(tin, scope)
            m.output_type = self._resolve_message(tout, scope)
        return self.fd

    def service(self, sv):
        sv.name = self.take()
        self.take("{")
        while self.peek() != "}":
            tok = self.take()
            if tok == "option":
                while self.take() != ";":
                    pass
                continue
            if tok != "rpc":
                raise SyntaxError(f"unexpected {tok!r} in service {sv.name}")
            m = sv.method.add()
            m.name = self.take()
            self.take("(")
            tin = self.take()
            if tin == "stream":
                raise SyntaxError("streaming rpcs are not supported")
            self.take(")")
            self.take("returns")
            self.take("(")
            tout = self.take()
            self.take(")")
            if self.peek() == "{":
                depth = 0
                while True:
                    t = self.take()
                    depth += (t == "{") - (t == "}")
                    if depth == 0:
                        break
            if self.peek() == ";":
                self.take()
            self._methods.append((m, tin, tout, self.fd.package))
        self.take("}")

    def enum(self, e, scope):
        e.name = self.take()
        self._enums.add(f"{scope}.{e.name}".lstrip("."))
        self.take("{")
        while self.peek() != "}":
            if self.peek() == "option":
                while self.take() != ";":
                    pass
                continue
            v = e.value.add()
            v.name = self.take()
            self.take("=")
            v.number = int(self.take())
            self.take(";")
        self.take("}")

    def message(self, m, scope):
        m.name = self.take()
        here = f"{scope}.{m.name}"
        self._messages.add(here.lstrip("."))
        self.take("{")
        while self.peek() != "}":
            tok = self.peek()
            if tok == "message":
                self.take()
                self.message(m.nested_type.add(), here)
            elif tok == "enum":
                self.take()
                self.enum(m.enum_type.add(), here)
            elif tok == "oneof":
                self.take()
                idx = len(m.oneof_decl)
                m.oneof_decl.add().name = self.take()
                self.take("{")
                while self.peek() != "}":
                    self.field(m, here, oneof=idx)
                self.take("}")
            elif tok in ("option", "reserved"):
                while self.take() != ";":
                    pass
            else:
                self.field(m, here)
        self.take("}")

    def field(self, m, scope, oneof: int | None = None):
        label = _F.LABEL_OPTIONAL
        tok = self.take()
        if tok == "repeated":
            label, tok = _F.LABEL_REPEATED, self.take()
        if tok == "map":
            self.take("<")
            kt = self.take()
            self.take(",")
            vt = self.take()
            self.take(">")
            name = self.take()
            self.take("=")
            num = int(self.take())
            self.take(";")
            entry = m.nested_type.add()
            entry.name = "".join(p[:1].upper() + p[1:] for p in name.split("_")) + "Entry"
            entry.options.map_entry = True
            for n, (fname, t) in enumerate((("key", kt), ("value", vt)), 1):
                ef = entry.field.add(name=fname, number=n, label=_F.LABEL_OPTIONAL)
                self._typed(ef, t, f"{scope}.{entry.name}")
            f = m.field.add(name=name, number=num, label=_F.LABEL_REPEATED, type=_F.TYPE_MESSAGE)
            f.type_name = f".{scope}.{entry.name}"
            f.json_name = name
            return
        name = self.take()
        self.take("=")
        num = int(self.take())
        self.take(";")
        f = m.field.add(name=name, number=num, label=label)
        f.json_name = name
        if oneof is not None:
            f.oneof_index = oneof
        self._typed(f, tok, scope)

    def _typed(self, f, tname: str, scope: str):
        if tname in _SCALARS:
            f.type = _SCALARS[tname]
        else:
            self._fields.append((f, tname, scope))

    def _resolve(self, f, tname: str, scope: str):
        """Innermost-scope-first lookup, as protoc does."""
        parts = scope.split(".")
        for k in range(len(parts), -1, -1):
            cand = ".".join(parts[:k] + [tname]) if k else tname
            cand = cand.lstrip(".")
            if cand in getattr(self, "_enums_all", self._enums):
                f.type, f.type_name = _F.TYPE_ENUM, f".{cand}"
                return
            if self._has_message(cand):
                f.type, f.type_name = _F.TYPE_MESSAGE, f".{cand}"
                return
        raise SyntaxError(f"unknown type {tname!r} in {scope}")

    def _resolve_message(self, tname: str, scope: str) -> str:
        parts = scope.split(".")
        for k in range(len(parts), -1, -1):
            cand = (".".join(parts[:k] + [tname]) if k else tname).lstrip(".")
            if self._has_message(cand):
                return f".{cand}"
        raise SyntaxError(f"unknown message {tname!r} in {scope}")

    def _has_message(self, full: str) -> bool:
        if hasattr(self, "_messages_all"):
            return full in self._messages_all
        pkg = self.fd.package
        if pkg and not full.startswith(pkg + "."):
            return False
        rest = full[len(pkg) + 1:].split(".") if pkg else full.split(".")
        msgs = self.fd.message_type
        for i, n in enumerate(rest):
            m = next((x for x in msgs if x.name == n), None)
            if m is None:
                return False
            msgs = m.nested_type
        return True


def load_proto(text: str, name: str, pool: descriptor_pool.DescriptorPool | None = None) -> dict:
    """Parse ``text`` and return ``{message name: class}`` for its top-level messages (nested ones
    are attributes of their parents) plus ``{enum name: EnumTypeWrapper}`` entries."""
    from google.protobuf.internal.enum_type_wrapper import EnumTypeWrapper
    p = _Parser(text, name).parse()
    fd = p.resolve_all(p._enums, p._messages)
    pool = pool or descriptor_pool.DescriptorPool()
    pool.Add(fd)
    fdesc = pool.FindFileByName(name)
    out: dict = {}
    for m in fd.message_type:
        out[m.name] = message_factory.GetMessageClass(fdesc.message_types_by_name[m.name])
    for e in fd.enum_type:
        out[e.name] = EnumTypeWrapper(fdesc.enum_types_by_name[e.name])
    return out


def load_proto_files(files: dict, pool: descriptor_pool.DescriptorPool | None = None):
    """Parse ``{file name: text}`` (files that import each other) into one descriptor pool; returns
    the pool.  Message classes: ``message_factory.GetMessageClass(pool.FindMessageTypeByName(...))``."""
    parsers = {name: _Parser(text, name).parse() for name, text in files.items()}
    enums = set().union(*(p._enums for p in parsers.values()))
    messages = set().union(*(p._messages for p in parsers.values()))
    fds = {name: p.resolve_all(enums, messages) for name, p in parsers.items()}
    pool = pool or descriptor_pool.DescriptorPool()
    added: set = set()

    def add(name):
        if name in added:
            return
        added.add(name)
        for dep in fds[name].dependency:
            if dep in fds:
                add(dep)
        fd = fds[name]
        # keep only the dependencies actually loaded here (e.g. google/*.proto are dropped)
        keep = [d for d in fd.dependency if d in fds]
        del fd.dependency[:]
        fd.dependency.extend(keep)
        pool.Add(fd)
    for name in fds:
        add(name)
    return pool
