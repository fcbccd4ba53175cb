"""Runtime protobuf loader: parses the ``.proto`` schema files in ``schema/``
into ``FileDescriptorProto``s and registers them in the default descriptor
pool -- no ``protoc`` / ``grpc_tools`` needed (neither exists in the image),
and no generated ``*_pb2.py`` to go stale (the reference's checked-in stubs
use an API removed from protobuf>=4).

Supported proto3 subset: ``syntax``/``package``/``import``, (nested)
messages and enums, scalar / message / enum fields, ``repeated``,
``optional`` (synthetic oneofs), ``oneof``, ``map<K, V>``, ``service`` /
``rpc``.  The ``.proto`` files are the single source of truth of the wire
format.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

from google.protobuf import descriptor_pb2, descriptor_pool
from google.protobuf import timestamp_pb2  # noqa: F401  (registers the WKT file)

SCHEMA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "schema")

FDP = descriptor_pb2.FieldDescriptorProto
SCALARS = {
    "double": FDP.TYPE_DOUBLE, "float": FDP.TYPE_FLOAT, "int64": FDP.TYPE_INT64,
    "uint64": FDP.TYPE_UINT64, "int32": FDP.TYPE_INT32, "fixed64": FDP.TYPE_FIXED64,
    "fixed32": FDP.TYPE_FIXED32, "bool": FDP.TYPE_BOOL, "string": FDP.TYPE_STRING,
    "bytes": FDP.TYPE_BYTES, "uint32": FDP.TYPE_UINT32, "sfixed32": FDP.TYPE_SFIXED32,
    "sfixed64": FDP.TYPE_SFIXED64, "sint32": FDP.TYPE_SINT32, "sint64": FDP.TYPE_SINT64,
}

_TOKEN = re.compile(r'\s*(?:(//[^\n]*)|(/\*.*?\*/)|("(?:[^"\\]|\\.)*")|([A-Za-z_][\w.]*)|(-?\d+)|(.))',
                    re.S)


def tokenize(text: str) -> list[str]:
    out = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            break
        pos = m.end()
        if m.group(1) or m.group(2):
            continue
        tok = m.group(3) or m.group(4) or m.group(5) or m.group(6)
        if tok and not tok.isspace():
            out.append(tok)
    return out


class _Stream:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else None

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, tok):
        got = self.next()
        if got != tok:
            raise SyntaxError(f"expected {tok!r}, got {got!r} near token {self.i}")
        return got

    def skip_options(self):
        # [ ... ] field options or `option x = y;`
        if self.peek() == "[":
            depth = 0
            while True:
                t = self.next()
                depth += t == "["
                depth -= t == "]"
                if depth == 0:
                    break


def _camel(name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


@dataclass
class _Pending:
    field: object
    type_name: str
    scope: str
    is_map_value: bool = False


@dataclass
class _FileCtx:
    proto: descriptor_pb2.FileDescriptorProto
    package: str
    pending: list = field(default_factory=list)


def _parse_enum(s: _Stream, enum: descriptor_pb2.EnumDescriptorProto):
    enum.name = s.next()
    s.expect("{")
    while s.peek() != "}":
        if s.peek() == "option":
            while s.next() != ";":
                pass
            continue
        v = enum.value.add()
        v.name = s.next()
        s.expect("=")
        v.number = int(s.next())
        s.skip_options()
        s.expect(";")
    s.expect("}")


def _parse_field(s: _Stream, msg, ctx: _FileCtx, scope: str, label=None, oneof_index=None):
    tok = s.next()
    proto3_optional = False
    if tok in ("repeated", "optional"):
        label = tok
        proto3_optional = tok == "optional"
        tok = s.next()
    f = msg.field.add()
    if tok == "map":
        s.expect("<")
        ktype = s.next()
        s.expect(",")
        vtype = s.next()
        s.expect(">")
        f.name = s.next()
        s.expect("=")
        f.number = int(s.next())
        s.skip_options()
        s.expect(";")
        entry = msg.nested_type.add()
        entry.name = _camel(f.name) + "Entry"
        entry.options.map_entry = True
        k = entry.field.add()
        k.name, k.number, k.label, k.type = "key", 1, FDP.LABEL_OPTIONAL, SCALARS[ktype]
        v = entry.field.add()
        v.name, v.number, v.label = "value", 2, FDP.LABEL_OPTIONAL
        if vtype in SCALARS:
            v.type = SCALARS[vtype]
        else:
            ctx.pending.append(_Pending(v, vtype, scope))
        f.label = FDP.LABEL_REPEATED
        f.type = FDP.TYPE_MESSAGE
        f.type_name = f".{scope}.{entry.name}"
        return
    f.name = s.next()
    s.expect("=")
    f.number = int(s.next())
    s.skip_options()
    s.expect(";")
    f.label = FDP.LABEL_REPEATED if label == "repeated" else FDP.LABEL_OPTIONAL
    if tok in SCALARS:
        f.type = SCALARS[tok]
    else:
        ctx.pending.append(_Pending(f, tok, scope))
    if oneof_index is not None:
        f.oneof_index = oneof_index
    if proto3_optional:
        f.proto3_optional = True
        od = msg.oneof_decl.add()
        od.name = "_" + f.name
        f.oneof_index = len(msg.oneof_decl) - 1


def _parse_message(s: _Stream, msg, ctx: _FileCtx, outer: str):
    msg.name = s.next()
    scope = f"{outer}.{msg.name}"
    s.expect("{")
    synthetic = []  # proto3 optional oneofs must come after real ones
    while s.peek() != "}":
        t = s.peek()
        if t == "message":
            s.next()
            _parse_message(s, msg.nested_type.add(), ctx, scope)
        elif t == "enum":
            s.next()
            _parse_enum(s, msg.enum_type.add())
        elif t == "oneof":
            s.next()
            od = msg.oneof_decl.add()
            od.name = s.next()
            idx = len(msg.oneof_decl) - 1
            s.expect("{")
            while s.peek() != "}":
                _parse_field(s, msg, ctx, scope, oneof_index=idx)
            s.expect("}")
        elif t in ("option", "reserved"):
            while s.next() != ";":
                pass
        elif t == ";":
            s.next()
        else:
            _parse_field(s, msg, ctx, scope)
    s.expect("}")
    del synthetic
    _reorder_synthetic_oneofs(msg)


def _reorder_synthetic_oneofs(msg):
    """protobuf requires synthetic (proto3 optional) oneofs after real ones."""
    real = [i for i, od in enumerate(msg.oneof_decl) if not od.name.startswith("_")
            or not any(f.proto3_optional and f.oneof_index == i for f in msg.field)]
    synth = [i for i in range(len(msg.oneof_decl)) if i not in real]
    order = real + synth
    if order == list(range(len(msg.oneof_decl))):
        return
    remap = {old: new for new, old in enumerate(order)}
    decls = [descriptor_pb2.OneofDescriptorProto() for _ in order]
    for new, old in enumerate(order):
        decls[new].CopyFrom(msg.oneof_decl[old])
    del msg.oneof_decl[:]
    for d in decls:
        msg.oneof_decl.add().CopyFrom(d)
    for f in msg.field:
        if f.HasField("oneof_index"):
            f.oneof_index = remap[f.oneof_index]


def _parse_service(s: _Stream, svc):
    svc.name = s.next()
    s.expect("{")
    while s.peek() != "}":
        t = s.next()
        if t == "option":
            while s.next() != ";":
                pass
            continue
        if t != "rpc":
            raise SyntaxError(f"unexpected {t!r} in service")
        m = svc.method.add()
        m.name = s.next()
        s.expect("(")
        m.input_type = s.next()
        s.expect(")")
        s.expect("returns")
        s.expect("(")
        m.output_type = s.next()
        s.expect(")")
        if s.peek() == "{":
            s.next()
            s.expect("}")
        else:
            s.expect(";")
    s.expect("}")


def parse_proto(text: str, filename: str) -> _FileCtx:
    s = _Stream(tokenize(text))
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = filename
    ctx = _FileCtx(fdp, "")
    while s.peek() is not None:
        t = s.next()
        if t == "syntax":
            s.expect("=")
            fdp.syntax = s.next().strip('"')
            s.expect(";")
        elif t == "package":
            ctx.package = fdp.package = s.next()
            s.expect(";")
        elif t == "import":
            fdp.dependency.append(s.next().strip('"'))
            s.expect(";")
        elif t == "option":
            while s.next() != ";":
                pass
        elif t == "message":
            _parse_message(s, fdp.message_type.add(), ctx, ctx.package)
        elif t == "enum":
            _parse_enum(s, fdp.enum_type.add())
        elif t == "service":
            _parse_service(s, fdp.service.add())
        elif t == ";":
            continue
        else:
            raise SyntaxError(f"unexpected top-level token {t!r} in {filename}")
    return ctx


def _collect_types(fdp, symbols: dict):
    pkg = fdp.package

    def walk(msg, prefix):
        full = f"{prefix}.{msg.name}"
        symbols[full] = "message"
        for e in msg.enum_type:
            symbols[f"{full}.{e.name}"] = "enum"
        for n in msg.nested_type:
            walk(n, full)

    for m in fdp.message_type:
        walk(m, pkg)
    for e in fdp.enum_type:
        symbols[f"{pkg}.{e.name}"] = "enum"


def _resolve(name: str, scope: str, symbols: dict) -> str:
    if name.startswith("."):
        return name[1:]
    parts = scope.split(".")
    while True:
        cand = ".".join(parts + [name]) if parts else name
        if cand in symbols:
            return cand
        if not parts:
            break
        parts.pop()
    raise KeyError(f"unresolved type {name!r} in scope {scope!r}")


def _wkt_symbols(symbols: dict):
    pool = descriptor_pool.Default()
    ts = pool.FindMessageTypeByName("google.protobuf.Timestamp")
    symbols[ts.full_name] = "message"


SCHEMA_FILES = ["model.proto", "service_common.proto", "metis.proto", "controller.proto",
                "learner.proto"]


# Non-metisfl schemas read or written by the framework (registered under their
# upstream file names): tf.train.Example for TFRecord datasets.
EXTRA_FILES = {"tf_example.proto": "tensorflow/core/example/example.proto"}


def build_file_protos(schema_dir: str = SCHEMA_DIR, files=None) -> list[descriptor_pb2.FileDescriptorProto]:
    ctxs = []
    symbols: dict[str, str] = {}
    _wkt_symbols(symbols)
    files = files or {fn: f"metisfl/proto/{fn}" for fn in SCHEMA_FILES}
    for fn, registered in files.items():
        with open(os.path.join(schema_dir, fn)) as f:
            ctx = parse_proto(f.read(), registered)
        _collect_types(ctx.proto, symbols)
        ctxs.append(ctx)
    for ctx in ctxs:
        for p in ctx.pending:
            full = _resolve(p.type_name, p.scope, symbols)
            p.field.type_name = "." + full
            p.field.type = FDP.TYPE_MESSAGE if symbols[full] == "message" else FDP.TYPE_ENUM
        for svc in ctx.proto.service:
            for m in svc.method:
                m.input_type = "." + _resolve(m.input_type, ctx.package, symbols)
                m.output_type = "." + _resolve(m.output_type, ctx.package, symbols)
    return [c.proto for c in ctxs]


_LOADED = False


def load() -> descriptor_pool.DescriptorPool:
    """Register the metisfl schema in the default pool (idempotent)."""
    global _LOADED
    pool = descriptor_pool.Default()
    if _LOADED:
        return pool
    for fdp in build_file_protos() + build_file_protos(files=EXTRA_FILES):
        try:
            pool.FindFileByName(fdp.name)
        except KeyError:
            pool.Add(fdp)
    _LOADED = True
    return pool
