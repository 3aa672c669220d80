"""The JVM shim's JNA binding (jvm/.../CapsmiLib.scala) against the C header it binds (include/capsmi.h).

There is no JVM in this image, so the Scala sources cannot be compiled here; this checks, as text,
what a layout drift would break at run time: every Scala constant equals the header's enum value,
every JNA Structure lists the C struct's fields in the C order with matching widths, and every
declared entry point exists in the header with the same number of parameters.  CPU only."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "capsmi.h")
SCALA = os.path.join(ROOT, "jvm", "src", "main", "scala", "org", "opencypher", "capsmi", "CapsmiLib.scala")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", re.sub(r"//[^\n]*", "", s, flags=re.S), flags=re.S)


def _header():
    return _strip_c_comments(open(HEADER).read())


def _scala():
    return open(SCALA).read()


def _c_enums():
    out = {}
    for body in re.findall(r"enum\s*\{(.*?)\}", _header(), re.S):
        for name, val in re.findall(r"(CAPSMI_[A-Z0-9_]+)\s*=\s*(-?\d+)", body):
            out[name] = int(val)
    return out


def _c_structs():
    out = {}
    for body, name in re.findall(r"typedef\s+struct\s*\{(.*?)\}\s*(capsmi_[a-z_]+)\s*;", _header(), re.S):
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            m = re.match(r"(.*?)([A-Za-z_][A-Za-z0-9_]*)\s*$", decl, re.S)
            ctype, fname = m.group(1).strip(), m.group(2)
            fields.append((fname, ctype))
        out[name] = fields
    return out


def _c_functions():
    out = {}
    for ret, name, args in re.findall(r"^\s*(capsmi_status|size_t|const char\*)\s+(capsmi_[a-z0-9_]+)\s*\((.*?)\)\s*;",
                                      _header(), re.S | re.M):
        args = " ".join(args.split())
        out[name] = 0 if args in ("", "void") else args.count(",") + 1
    return out


SCALA_STRUCTS = {"ColDesc": "capsmi_col_desc", "CapsmiExpr": "capsmi_expr", "CapsmiExprColumn": "capsmi_expr_column",
                 "CapsmiAgg": "capsmi_agg", "CapsmiValue": "capsmi_value", "CapsmiParam": "capsmi_param",
                 "CapsmiCollVec": "capsmi_coll_vec"}


def test_constants_match_header():
    enums = _c_enums()
    consts = re.findall(r"final val ([A-Z0-9_]+)\s*=\s*(-?\d+)", _scala())
    assert len(consts) > 50
    for name, val in consts:
        assert "CAPSMI_" + name in enums, f"Capsmi.{name} has no CAPSMI_{name} in capsmi.h"
        assert enums["CAPSMI_" + name] == int(val), f"Capsmi.{name} = {val}, header {enums['CAPSMI_' + name]}"


def _width(ctype):
    if "*" in ctype:
        return "ptr"
    if ctype.endswith("int64_t") or ctype == "int64_t":
        return 8
    if ctype.endswith("int32_t"):
        return 4
    raise AssertionError(f"unexpected C field type {ctype!r}")


@pytest.mark.parametrize("cls", sorted(SCALA_STRUCTS))
def test_structure_layout_matches_header(cls):
    src = _scala()
    m = re.search(r"@Structure\.FieldOrder\(Array\(([^)]*)\)\)\s*class " + cls + r" extends Structure \{(.*?)\n\}",
                  src, re.S)
    assert m, f"no JNA Structure {cls}"
    order = re.findall(r'"([a-z_]+)"', m.group(1))
    c_fields = _c_structs()[SCALA_STRUCTS[cls]]
    assert order == [f for f, _ in c_fields], (cls, order, c_fields)
    scala_types = {name.strip("`"): ty for name, ty in re.findall(r"var (`?[a-z_]+`?): ([A-Za-z]+)", m.group(2))}
    for fname, ctype in c_fields:
        want = {"ptr": ("Pointer", "String"), 8: ("Long",), 4: ("Int",)}[_width(ctype)]
        assert scala_types[fname] in want, (cls, fname, ctype, scala_types[fname])


def test_entry_points_match_header():
    funcs = _c_functions()
    decls = re.findall(r"def (capsmi_[a-z0-9_]+)\((.*?)\):\s*(Int|Long)", _scala(), re.S)
    assert len(decls) > 40
    for name, params, _ in decls:
        assert name in funcs, f"{name} declared in CapsmiLib.scala but not in capsmi.h"
        n = 0 if not params.strip() else params.count(",") + 1
        assert n == funcs[name], f"{name}: {n} JNA parameters, {funcs[name]} in capsmi.h"
