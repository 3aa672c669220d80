"""Static check of the JVM shim against the reference's Table contract.

jvm/src/main/scala/org/opencypher/capsmi/GpuTable.scala is never compiled here (no JVM in this image).  This
test reads the reference's trait sources as text -- okapi-relational/.../api/table/Table.scala:43-176 and
okapi-api/.../api/table/CypherTable.scala:41-68 -- extracts every member's name, parameter lists (types,
implicit-ness, varargs; parameter names and default values ignored) and result type with `T` read as
GpuTable, and checks that GpuTable overrides every abstract member with the same lists and result, and that
every member it does override matches the trait's.  It runs in the build container only: /root/reference is
not on the GPU box (the test is then skipped)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
TABLE = os.path.join(REF, "okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala")
CYPHER_TABLE = os.path.join(REF, "okapi-api/src/main/scala/org/opencypher/okapi/api/table/CypherTable.scala")
SHIM = os.path.join(ROOT, "jvm/src/main/scala/org/opencypher/capsmi/GpuTable.scala")


def _strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _split_top(s, sep=","):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _norm_type(t, self_type):
    t = re.sub(r"\s+", "", t)
    return re.sub(r"\bT\b", "GpuTable", t) if self_type else t


def _params(group, self_type):
    body = group[1:-1].strip()
    implicit = body.startswith("implicit ")
    if implicit:
        body = body[len("implicit "):]
    types = []
    for p in _split_top(body):
        p = p.split("=", 1)[0]  # default value
        name, _, ty = p.partition(":")
        types.append(_norm_type(ty, self_type))
    return ("implicit " if implicit else "") + ",".join(types)


def members(path, trait=None, overrides_only=False, self_type=True):
    """{(name, (param lists...)): (result type, abstract)} of the members of `trait` (or of the file)"""
    src = _strip_comments(open(path).read())
    if trait:
        i = src.index(f"trait {trait}")
        j = src.index("{", i)
        depth, k = 0, j
        while True:  # the trait body
            depth += {"{": 1, "}": -1}.get(src[k], 0)
            if depth == 0:
                break
            k += 1
        src = src[j + 1:k]
    out = {}
    pat = r"\boverride\s+def\s+(\w+)" if overrides_only else r"(?<![\w.])def\s+(\w+)"
    for m in re.finditer(pat, src):
        if trait and src[:m.start()].count("{") - src[:m.start()].count("}") != 0:
            continue  # a member of a nested object / class, not of the trait
        k = m.end()
        groups = []
        while True:
            while k < len(src) and src[k] in " \t\n":
                k += 1
            if k >= len(src) or src[k] != "(":
                break
            depth, j = 0, k
            while True:
                depth += {"(": 1, ")": -1}.get(src[j], 0)
                if depth == 0:
                    break
                j += 1
            groups.append(_params(src[k:j + 1], self_type))
            k = j + 1
        rest = src[k:]
        result, after = None, rest
        mm = re.match(r"\s*:", rest)
        if mm:  # the result type runs to a top-level '=' (not '=>'), '{' or the line's end
            j, depth = mm.end(), 0
            while j < len(rest):
                ch = rest[j]
                depth += 1 if ch in "([" else -1 if ch in ")]" else 0
                if depth == 0 and (ch in "{\n" or (ch == "=" and rest[j + 1:j + 2] != ">")):
                    break
                j += 1
            result, after = _norm_type(rest[mm.end():j], self_type), rest[j:]
        abstract = not re.match(r"[ \t]*=", after)
        out[(m.group(1), tuple(groups))] = (result, abstract)
    return out


@pytest.mark.skipif(not os.path.exists(TABLE), reason="the reference is only in the build container")
def test_gpu_table_overrides_every_table_member():
    trait = members(TABLE, "Table")
    trait.update(members(CYPHER_TABLE, "CypherTable"))
    shim = members(SHIM, overrides_only=True, self_type=False)
    assert ("join", ("GpuTable,JoinType,(String,String)*",)) in trait  # the parser read Table.scala:88
    missing = [k for k, (_, abstract) in trait.items() if abstract and k not in shim]
    assert not missing, f"GpuTable does not override {missing}"
    by_name = {}
    for k in trait:
        by_name.setdefault(k[0], []).append(k)
    for k, (res, _) in shim.items():
        if k[0] not in by_name:
            continue  # not a Table / CypherTable member (e.g. a records-level override)
        assert k in trait, f"GpuTable.{k[0]}{k[1]} matches no parameter lists of {by_name[k[0]]}"
        assert res == trait[k][0], f"GpuTable.{k[0]} returns {res}, the trait {trait[k][0]}"
