"""Runtime ``.proto`` (proto3) parser -> ``FileDescriptorProto``.

There is no ``protoc`` / ``grpc_tools`` in the image, so the wire schema is
compiled at import time: ``.proto`` text is tokenised, parsed into
``google.protobuf.descriptor_pb2.FileDescriptorProto`` objects, type references
are resolved with protobuf's scoping rules, and the result is loaded into a
private ``DescriptorPool`` (see ``rust_tensorflow_serving2_amd/schema.py``).

This replaces the reference's build-time codegen step (``build.rs:1-10``,
``tonic_build::configure().compile``) which turns the vendored schema into Rust
types.  Supported grammar: the subset used by TF / TF-Serving schemas —
``syntax``, ``package``, ``import``, ``option`` (ignored except field options
``packed``/``json_name``/``deprecated``/``lazy``), nested ``message``/``enum``,
``oneof``, ``map<,>``, ``repeated``/``optional``, ``reserved`` ranges/names and
``service``/``rpc`` definitions.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple

from google.protobuf import descriptor_pb2 as dpb

FDP = dpb.FieldDescriptorProto

SCALAR_TYPES = {
    "double": FDP.TYPE_DOUBLE, "float": FDP.TYPE_FLOAT, "int64": FDP.TYPE_INT64,
    "uint64": FDP.TYPE_UINT64, "int32": FDP.TYPE_INT32, "fixed64": FDP.TYPE_FIXED64,
    "fixed32": FDP.TYPE_FIXED32, "bool": FDP.TYPE_BOOL, "string": FDP.TYPE_STRING,
    "bytes": FDP.TYPE_BYTES, "uint32": FDP.TYPE_UINT32, "sfixed32": FDP.TYPE_SFIXED32,
    "sfixed64": FDP.TYPE_SFIXED64, "sint32": FDP.TYPE_SINT32, "sint64": FDP.TYPE_SINT64,
}
_MAP_KEY_OK = {"int64", "uint64", "int32", "fixed64", "fixed32", "bool", "string",
               "uint32", "sfixed32", "sfixed64", "sint32", "sint64"}

_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+)
  | (?P<lcomment>//[^\n]*)
  | (?P<bcomment>/\*.*?\*/)
  | (?P<string>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<number>-?(?:0[xX][0-9a-fA-F]+|\d+\.\d*(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?|inf|nan))
  | (?P<ident>\.?[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z_][A-Za-z0-9_]*)*)
  | (?P<sym>[{}\[\]()<>;=,:.\-+])
""", re.X | re.S)


class ProtoSyntaxError(ValueError):
    pass


def tokenize(text: str, filename: str = "<proto>") -> List[Tuple[str, str, int]]:
    out = []
    pos, line = 0, 1
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m:
            raise ProtoSyntaxError(f"{filename}:{line}: unexpected character {text[pos]!r}")
        kind = m.lastgroup
        val = m.group(kind)
        if kind not in ("ws", "lcomment", "bcomment"):
            out.append((kind, val, line))
        line += val.count("\n")
        pos = m.end()
    return out


def _unquote(s: str) -> str:
    body = s[1:-1]
    return bytes(body, "utf-8").decode("unicode_escape")


def _camel(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


@dataclass
class _PendingRef:
    field: FDP
    type_name: str
    scope: str          # fully qualified scope, no leading dot


class _Parser:
    def __init__(self, text: str, filename: str):
        self.toks = tokenize(text, filename)
        self.i = 0
        self.filename = filename
        self.fd = dpb.FileDescriptorProto(name=filename)
        self.refs: List[_PendingRef] = []
        self.defined: List[Tuple[str, str]] = []   # (fqname, 'message'|'enum')

    # -- token helpers -------------------------------------------------
    def peek(self, k: int = 0) -> Optional[str]:
        j = self.i + k
        return self.toks[j][1] if j < len(self.toks) else None

    def next(self) -> str:
        if self.i >= len(self.toks):
            raise ProtoSyntaxError(f"{self.filename}: unexpected end of file")
        v = self.toks[self.i][1]
        self.i += 1
        return v

    def expect(self, val: str) -> None:
        got = self.next()
        if got != val:
            line = self.toks[self.i - 1][2]
            raise ProtoSyntaxError(f"{self.filename}:{line}: expected {val!r}, got {got!r}")

    def accept(self, val: str) -> bool:
        if self.peek() == val:
            self.i += 1
            return True
        return False

    def skip_statement(self) -> None:
        depth = 0
        while True:
            t = self.next()
            if t == "{":
                depth += 1
            elif t == "}":
                depth -= 1
                if depth == 0:
                    return
            elif t == ";" and depth == 0:
                return

    def constant(self) -> str:
        t = self.next()
        if t in ("-", "+"):
            t = t + self.next()
        return t

    # -- grammar -------------------------------------------------------
    def parse(self) -> dpb.FileDescriptorProto:
        pkg = ""
        while self.peek() is not None:
            t = self.peek()
            if t == "syntax":
                self.next(); self.expect("="); s = _unquote(self.next()); self.expect(";")
                self.fd.syntax = s
            elif t == "package":
                self.next(); pkg = self.next(); self.expect(";")
                self.fd.package = pkg
            elif t == "import":
                self.next()
                if self.peek() in ("public", "weak"):
                    self.next()
                self.fd.dependency.append(_unquote(self.next())); self.expect(";")
            elif t == "option":
                self.skip_statement()
            elif t == "message":
                self.message(pkg, self.fd.message_type)
            elif t == "enum":
                self.enum(pkg, self.fd.enum_type)
            elif t == "service":
                self.service(pkg, self.fd.service)
            elif t == ";":
                self.next()
            else:
                raise ProtoSyntaxError(f"{self.filename}: unexpected top-level token {t!r}")
        if not self.fd.syntax:
            self.fd.syntax = "proto2"
        return self.fd

    def field_options(self, f: FDP) -> None:
        if not self.accept("["):
            return
        while True:
            name = self.next()
            if name == "(":   # custom option: skip "(x.y)"
                while self.next() != ")":
                    pass
                name = "custom"
            self.expect("=")
            val = self.constant()
            if name == "packed":
                f.options.packed = (val == "true")
            elif name == "json_name":
                f.json_name = _unquote(val)
            elif name == "deprecated":
                f.options.deprecated = (val == "true")
            elif name == "lazy":
                f.options.lazy = (val == "true")
            if self.accept("]"):
                return
            self.expect(",")

    def reserved(self, msg) -> None:
        self.expect("reserved")
        while True:
            t = self.next()
            if t[0] in "\"'":
                msg.reserved_name.append(_unquote(t))
            else:
                start = int(t, 0)
                end = start
                if self.accept("to"):
                    e = self.next()
                    end = 536870911 if e == "max" else int(e, 0)
                r = msg.reserved_range.add()
                r.start, r.end = start, end + 1
            if self.accept(";"):
                return
            self.expect(",")

    def add_field(self, msg, scope: str, label: int, type_name: str, name: str,
                  number: int, oneof_index: Optional[int] = None) -> FDP:
        f = msg.field.add(name=name, number=number, label=label)
        if type_name in SCALAR_TYPES:
            f.type = SCALAR_TYPES[type_name]
        else:
            self.refs.append(_PendingRef(f, type_name, scope))
        if oneof_index is not None:
            f.oneof_index = oneof_index
        f.json_name = _camel(name)
        return f

    def map_field(self, msg, scope: str) -> None:
        self.expect("map"); self.expect("<")
        ktype = self.next(); self.expect(",")
        vtype = self.next(); self.expect(">")
        name = self.next(); self.expect("="); number = int(self.next(), 0)
        if ktype not in _MAP_KEY_OK:
            raise ProtoSyntaxError(f"{self.filename}: invalid map key type {ktype}")
        entry_name = "".join(p[:1].upper() + p[1:] for p in name.split("_")) + "Entry"
        entry = msg.nested_type.add(name=entry_name)
        entry.options.map_entry = True
        escope = f"{scope}.{entry_name}"
        self.add_field(entry, escope, FDP.LABEL_OPTIONAL, ktype, "key", 1)
        self.add_field(entry, escope, FDP.LABEL_OPTIONAL, vtype, "value", 2)
        f = msg.field.add(name=name, number=number, label=FDP.LABEL_REPEATED,
                          type=FDP.TYPE_MESSAGE, type_name=f".{escope}")
        f.json_name = _camel(name)
        self.field_options(f)
        self.expect(";")

    def plain_field(self, msg, scope: str, oneof_index: Optional[int] = None) -> None:
        label = FDP.LABEL_OPTIONAL
        proto3_optional = False
        if self.peek() == "repeated":
            self.next(); label = FDP.LABEL_REPEATED
        elif self.peek() == "optional":
            self.next(); proto3_optional = self.fd.syntax == "proto3"
        elif self.peek() == "required":
            self.next(); label = FDP.LABEL_REQUIRED
        type_name = self.next()
        name = self.next()
        self.expect("=")
        number = int(self.next(), 0)
        if proto3_optional:
            # synthetic oneof, as protoc emits for proto3 `optional`
            oi = len(msg.oneof_decl)
            msg.oneof_decl.add(name=f"_{name}")
            f = self.add_field(msg, scope, label, type_name, name, number, oi)
            f.proto3_optional = True
        else:
            f = self.add_field(msg, scope, label, type_name, name, number, oneof_index)
        self.field_options(f)
        self.expect(";")

    def message(self, scope: str, container):
        # objects are created in place (container.add) so pending type refs
        # keep pointing at the live field messages
        self.expect("message")
        name = self.next()
        fq = f"{scope}.{name}" if scope else name
        self.defined.append((fq, "message"))
        msg = container.add(name=name)
        self.expect("{")
        while not self.accept("}"):
            t = self.peek()
            if t == "message":
                self.message(fq, msg.nested_type)
            elif t == "enum":
                self.enum(fq, msg.enum_type)
            elif t == "oneof":
                self.next()
                oname = self.next()
                oi = len(msg.oneof_decl)
                msg.oneof_decl.add(name=oname)
                self.expect("{")
                while not self.accept("}"):
                    if self.peek() == "option":
                        self.skip_statement()
                        continue
                    self.plain_field(msg, fq, oi)
            elif t == "map":
                self.map_field(msg, fq)
            elif t == "reserved":
                self.reserved(msg)
            elif t in ("option", "extensions", "extend"):
                self.skip_statement()
            elif t == ";":
                self.next()
            else:
                self.plain_field(msg, fq)
        self.accept(";")
        # proto3 synthetic oneofs must come after real ones (descriptor rule)
        return msg

    def enum(self, scope: str, container):
        self.expect("enum")
        name = self.next()
        fq = f"{scope}.{name}" if scope else name
        self.defined.append((fq, "enum"))
        en = container.add(name=name)
        self.expect("{")
        while not self.accept("}"):
            t = self.peek()
            if t in ("option",):
                self.skip_statement()
                continue
            if t == "reserved":
                self.next()
                while not self.accept(";"):
                    self.next()
                continue
            if t == ";":
                self.next(); continue
            vname = self.next()
            self.expect("=")
            num = int(self.constant(), 0)
            v = en.value.add(name=vname, number=num)
            if self.accept("["):
                while not self.accept("]"):
                    o = self.next()
                    if o == "deprecated":
                        self.expect("="); v.options.deprecated = self.next() == "true"
            self.expect(";")
        self.accept(";")
        return en

    def service(self, scope: str, container):
        self.expect("service")
        svc = container.add(name=self.next())
        self.expect("{")
        while not self.accept("}"):
            t = self.peek()
            if t == "option":
                self.skip_statement(); continue
            if t == ";":
                self.next(); continue
            self.expect("rpc")
            m = svc.method.add(name=self.next())
            self.expect("(")
            if self.accept("stream"):
                m.client_streaming = True
            req = self.next(); self.expect(")")
            self.expect("returns"); self.expect("(")
            if self.accept("stream"):
                m.server_streaming = True
            resp = self.next(); self.expect(")")
            self.refs.append(_PendingRef(m, req, scope))     # type: ignore[arg-type]
            self.refs.append(_PendingRef(m, "@out:" + resp, scope))  # type: ignore[arg-type]
            if self.peek() == "{":
                self.skip_statement()
            else:
                self.expect(";")
        self.accept(";")
        return svc


@dataclass
class ParsedFile:
    fd: dpb.FileDescriptorProto
    refs: List[_PendingRef]
    defined: List[Tuple[str, str]]


def parse_proto(text: str, filename: str) -> ParsedFile:
    p = _Parser(text, filename)
    fd = p.parse()
    return ParsedFile(fd, p.refs, p.defined)


def _resolve(name: str, scope: str, symbols: Dict[str, str]) -> Optional[str]:
    if name.startswith("."):
        return name[1:] if name[1:] in symbols else None
    parts = scope.split(".") if scope else []
    while True:
        cand = ".".join(parts + [name])
        if cand in symbols:
            return cand
        if not parts:
            return None
        parts.pop()


def link(files: Iterable[ParsedFile], extra_symbols: Dict[str, str]) -> List[dpb.FileDescriptorProto]:
    """Resolve every symbolic type reference to a fully-qualified one.

    ``extra_symbols`` maps fq-name -> 'message'|'enum' for types defined outside
    ``files`` (e.g. google.protobuf well-known types already in the pool).
    """
    files = list(files)
    symbols: Dict[str, str] = dict(extra_symbols)
    for pf in files:
        for fq, kind in pf.defined:
            symbols[fq] = kind
    for pf in files:
        for ref in pf.refs:
            tn = ref.type_name
            is_out = tn.startswith("@out:")
            if is_out:
                tn = tn[5:]
            fq = _resolve(tn, ref.scope, symbols)
            if fq is None:
                raise ProtoSyntaxError(f"{pf.fd.name}: unresolved type {tn!r} in scope {ref.scope!r}")
            f = ref.field
            if isinstance(f, dpb.MethodDescriptorProto):
                if is_out:
                    f.output_type = "." + fq
                else:
                    f.input_type = "." + fq
                continue
            f.type_name = "." + fq
            f.type = FDP.TYPE_MESSAGE if symbols[fq] == "message" else FDP.TYPE_ENUM
    return [pf.fd for pf in files]
