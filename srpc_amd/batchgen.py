"""srpc_amd.batchgen -- batch (SoA) companions for sRPC contracts.

The reference generator (``include/srpc/generator.hpp:100-134``,
``handle_message``) emits one C++ struct per ``message`` with ``name``,
``fields`` (the STRUCT_MEMBER tuple) and ``unpack``.  This tool reads the same
``.contract`` language (``include/srpc/token.hpp`` keywords, the field-type
table of ``parser.hpp:253-290``) and emits, next to each struct, what the
GPU batch path needs:

* ``<Msg>_batch``: the SoA device view of N records -- one column per
  flattened field (nested messages inlined in declaration order, as
  ``pack_struct`` does, ``packer.hpp:172-178,183-186``), strings as a chars
  column plus n+1 u64 offsets -- with the schema descriptor (``kinds``,
  ``paths``, ``fixed_bytes``) as compile-time constants;
* ``<Svc>_batch``: per method, the method name the stubs use
  (``generator.hpp:84``: ``<Svc>_servicer::<method>``) and factories for the
  request / response ``srpc::gpu::batch_packer`` of its message types.

    python -m srpc_amd.batchgen calculator.contract -o calculator_batch.hpp [--messages]

Without ``--messages`` the header is included after the generated stubs
(``<name>_srpc.cpp``), which define the message structs.  With it the message
structs are emitted too (same shape as the reference generator's, with a
working nested-message ``unpack``: the reference's ``*(p->getv())`` at
``generator.hpp:127`` does not compile for nested fields).
"""
from __future__ import annotations

import argparse
import re
import sys
from dataclasses import dataclass, field

# contract type -> (C++ type, srpc_kind macro, wire bytes or 0 for string)
PRIMITIVES = {
    "bool": ("bool", "SRPC_KIND_BOOL", 1),
    "int8": ("int8_t", "SRPC_KIND_INT8", 1),
    "char": ("char", "SRPC_KIND_CHAR", 1),
    "int16": ("int16_t", "SRPC_KIND_INT16", 2),
    "int32": ("int32_t", "SRPC_KIND_INT32", 4),
    "int64": ("int64_t", "SRPC_KIND_INT64", 8),
    "string": ("std::string", "SRPC_KIND_STRING", 0),
}
KEYWORDS = {"message", "service", "method", "returns"} | set(PRIMITIVES)
# members every generated message struct has (generator.hpp:103-130)
RESERVED_FIELDS = {"name", "fields", "unpack"}

_TOKEN = re.compile(r"\s*(?:(//[^\n]*)|([A-Za-z_][A-Za-z0-9_]*)|([0-9]+)|(\S))")


class ContractError(ValueError):
    pass


@dataclass
class Field:
    type: str        # contract type: a primitive or a message name
    name: str


@dataclass
class Message:
    name: str
    fields: list[Field] = field(default_factory=list)


@dataclass
class Method:
    name: str
    input_t: str
    output_t: str


@dataclass
class Service:
    name: str
    methods: list[Method] = field(default_factory=list)


@dataclass
class Contract:
    messages: list[Message] = field(default_factory=list)
    services: list[Service] = field(default_factory=list)

    def message(self, name: str) -> Message:
        for m in self.messages:
            if m.name == name:
                return m
        raise KeyError(name)


def tokenize(text: str) -> list[str]:
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            break
        pos = m.end()
        if m.group(1):  # comment
            continue
        tok = m.group(2) or m.group(3) or m.group(4)
        if tok:
            toks.append(tok)
    return toks


def parse(text: str) -> Contract:
    """Parse a contract.  Element names must be defined before use as a
    field type, as in the reference parser (contract::element_index_map)."""
    toks = tokenize(text)
    i = 0
    c = Contract()
    defined: set[str] = set()

    def expect(want: str) -> str:
        nonlocal i
        if i >= len(toks) or (want != "IDENT" and toks[i] != want):
            got = toks[i] if i < len(toks) else "EOF"
            raise ContractError(f"expected {want!r}, got {got!r}")
        if want == "IDENT" and (not re.fullmatch(r"[A-Za-z_][A-Za-z0-9_]*", toks[i]) or toks[i] in KEYWORDS):
            raise ContractError(f"expected an identifier, got {toks[i]!r}")
        i += 1
        return toks[i - 1]

    while i < len(toks):
        kw = toks[i]
        if kw == "message":
            i += 1
            msg = Message(expect("IDENT"))
            if msg.name in defined:
                raise ContractError(f"element {msg.name!r} defined twice")
            expect("{")
            while i < len(toks) and toks[i] != "}":
                t = toks[i]
                if t not in PRIMITIVES:
                    if t not in defined or t == msg.name:
                        raise ContractError(f"Undefined identifier in field type: {t!r}")
                    if not any(m.name == t for m in c.messages):
                        raise ContractError(f"field type {t!r} is not a message")
                i += 1
                fname = expect("IDENT")
                if fname in RESERVED_FIELDS:
                    raise ContractError(f"field name {fname!r} collides with a generated member of {msg.name!r}")
                if any(f.name == fname for f in msg.fields):
                    raise ContractError(f"field {fname!r} repeated in message {msg.name!r}")
                expect(";")
                msg.fields.append(Field(t, fname))
            expect("}")
            defined.add(msg.name)
            c.messages.append(msg)
        elif kw == "service":
            i += 1
            svc = Service(expect("IDENT"))
            expect("{")
            while i < len(toks) and toks[i] != "}":
                expect("method")
                mname = expect("IDENT")
                expect("(")
                it = expect("IDENT")
                expect(")")
                expect("returns")
                expect("(")
                ot = expect("IDENT")
                expect(")")
                expect(";")
                for t in (it, ot):
                    if not any(m.name == t for m in c.messages):
                        raise ContractError(f"Undefined message type in method {mname!r}: {t!r}")
                svc.methods.append(Method(mname, it, ot))
            expect("}")
            defined.add(svc.name)
            c.services.append(svc)
        else:
            raise ContractError(f"expected 'message' or 'service', got {kw!r}")
    return c


def flatten(c: Contract, msg: Message, prefix: str = "") -> list[tuple[str, str]]:
    """(path, contract primitive type) per leaf field, in wire order."""
    out = []
    for f in msg.fields:
        path = f"{prefix}{f.name}"
        if f.type in PRIMITIVES:
            out.append((path, f.type))
        else:
            out.extend(flatten(c, c.message(f.type), path + "_"))
    return out


def _message_struct(c: Contract, msg: Message) -> str:
    """The message struct in the reference generator's shape (generator.hpp:100-134)."""
    lines = [f"struct {msg.name} : public srpc::message_base {{"]
    for f in msg.fields:
        ctype = PRIMITIVES[f.type][0] if f.type in PRIMITIVES else f.type
        lines.append(f"    {ctype} {f.name};")
    lines.append("")
    lines.append(f'    static constexpr const char* name = "{msg.name}";')
    lines.append("    static constexpr auto fields = std::make_tuple(")
    members = [f'        STRUCT_MEMBER({msg.name}, {f.name}, "{msg.name}::{f.name}")' for f in msg.fields]
    lines.append(",\n".join(members))
    lines.append("    );")
    lines.append("    void unpack(srpc::buffer::ptr bp) override {")
    lines.append("        srpc::packer srpc_p(bp);")
    for f in msg.fields:
        if f.type in PRIMITIVES:
            lines.append(f"        srpc_p >> {f.name};")
        else:
            lines.append(f"        {f.name}.unpack(bp);  // nested: same buffer, same cursor")
    lines.append("    }")
    lines.append("};")
    return "\n".join(lines) + "\n"


def _batch_struct(c: Contract, msg: Message) -> str:
    leaves = flatten(c, msg)
    nf = len(leaves)
    if nf == 0:
        return f"// {msg.name}: no fields, no batch view (an empty body packs to zero bytes)\n"
    fixed = sum(8 if t == "string" else PRIMITIVES[t][2] for _, t in leaves)
    has_str = any(t == "string" for _, t in leaves)
    kinds = ", ".join(PRIMITIVES[t][1] for _, t in leaves)
    paths = ", ".join(f'"{p}"' for p, _ in leaves)
    body = [
        f"// {msg.name}: {nf} flattened field{'s' if nf != 1 else ''}, "
        + (f"{fixed} wire bytes per record" if not has_str else f"{fixed} fixed wire bytes per record + string contents"),
        f"struct {msg.name}_batch {{",
        f"    using message_type = {msg.name};",
        f"    static constexpr uint32_t nfields = {nf};",
        f"    static constexpr int32_t kinds[{nf}] = {{{kinds}}};",
        f"    static constexpr const char* paths[{nf}] = {{{paths}}};",
        f"    static constexpr uint64_t fixed_bytes = {fixed};  // body bytes per record without string contents",
        f"    static constexpr bool has_strings = {'true' if has_str else 'false'};",
        "",
        "    uint64_t n = 0;          // records",
        f"    void* cols[{nf}] = {{}};      // device columns: values, or a string field's chars",
        f"    uint64_t* offs[{nf}] = {{}};  // string fields: n + 1 char offsets (device); else null",
        "",
    ]
    for k, (p, t) in enumerate(leaves):
        if t == "string":
            body.append(f"    char* {p}_chars() const {{ return static_cast<char*>(cols[{k}]); }}")
            body.append(f"    uint64_t* {p}_offs() const {{ return offs[{k}]; }}")
        else:
            ctype = PRIMITIVES[t][0]
            body.append(f"    {ctype}* {p}() const {{ return static_cast<{ctype}*>(cols[{k}]); }}")
    body += [
        "",
        "    static srpc_schema_desc schema(const uint8_t* prefix = nullptr, uint32_t prefix_len = 0) {",
        "        return srpc_schema_desc{nfields, kinds, prefix, prefix_len};",
        "    }",
        "    const void* const* columns() const { return cols; }",
        "    void* const* columns() { return cols; }",
        "    const uint64_t* const* str_offsets() const { return offs; }",
        "    uint64_t* const* str_offsets() { return offs; }",
        "};",
        "",
    ]
    return "\n".join(body) + "\n"


def _service_struct(svc: Service) -> str:
    lines = [f"struct {svc.name}_batch {{"]
    for m in svc.methods:
        lines.append(f'    static constexpr const char* {m.name}_method = "{svc.name}_servicer::{m.name}";')
    for m in svc.methods:
        lines += [
            f"    static srpc::gpu::batch_packer<{m.input_t}> {m.name}_request(int device = 0) {{",
            f"        return srpc::gpu::batch_packer<{m.input_t}>::request({m.name}_method, device);",
            "    }",
            f"    static srpc::gpu::batch_packer<{m.output_t}> {m.name}_response(",
            "        srpc::rpc_status_code code = srpc::RPC_SUCCESS, int device = 0) {",
            f"        return srpc::gpu::batch_packer<{m.output_t}>::response(code, device);",
            "    }",
        ]
    lines.append("};")
    return "\n".join(lines) + "\n\n"


def generate(c: Contract, source: str, messages: bool = False) -> str:
    out = [
        f"// generated by srpc_amd.batchgen from {source}; do not edit.",
        "// Batch (SoA) companions of the contract's messages for the GPU batch path",
        "// (include/srpc/gpu.hpp)."
        + ("" if messages else "  Include after the generated stubs, which define the messages."),
        "#pragma once",
        "",
        "#include <cstdint>",
        "#include <string>",
        "#include <tuple>",
        "",
        "#include <srpc/gpu.hpp>",
        "",
    ]
    if messages:
        out += ["#include <srpc/core.hpp>", "#include <srpc/packer.hpp>", ""]
        for m in c.messages:
            out.append(_message_struct(c, m))
    for m in c.messages:
        out.append(_batch_struct(c, m))
    for s in c.services:
        out.append(_service_struct(s))
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("contract")
    ap.add_argument("-o", "--out", default=None, help="output header (default: <contract>_batch.hpp)")
    ap.add_argument("--messages", action="store_true", help="also emit the message structs")
    args = ap.parse_args(argv)
    try:
        c = parse(open(args.contract).read())
    except ContractError as e:
        print(f"parser error: {e}", file=sys.stderr)
        return 1
    out = args.out or re.sub(r"\.[^./]*$", "", args.contract) + "_batch.hpp"
    src = args.contract.rsplit("/", 1)[-1]
    with open(out, "w") as f:
        f.write(generate(c, src, args.messages))
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
