"""CREATE-query -> property graph, restating the reference's test-graph factory -- TEST INFRASTRUCTURE.

Follows okapi-testing/src/main/scala/org/opencypher/okapi/testing/propertygraph/CreateQueryParser.scala:
  - one id counter shared by nodes and relationships, starting at 0 (ParsingContext.fromParams,
    :278-283 `new AtomicLong()`; nextId :262)
  - clauses and comma-separated pattern parts are processed in order (:106-120, :148-153)
  - a relationship chain is left-nested: for `(n0)-[r1]->(n1)-[r2]->(n2)` the order is
    n0, n1, r1, n2, r2 -- each relationship takes its id after its right-hand node (:180-205)
  - the start of a chained relationship is the previous element's id, or for a previous
    relationship its *end* id (:182-185)
  - OUTGOING: (left -> right); INCOMING `<-[]-`: (right -> left) (:197-201)
  - a variable seen before is reused (labels/properties of the repeat are ignored, :165-171)
Supported literal syntax: 'str' / "str", integers (optional L suffix), floats, true/false, null.
"""
from __future__ import annotations

import re
from typing import Dict, List, Tuple

_TOKEN = re.compile(r"""\s*(?:
    (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<num>-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?[LDF]?)
  | (?P<arrow><-|->)
  | (?P<punct>[()\[\]{}:,\-])
  | (?P<word>[A-Za-z_][A-Za-z_0-9]*)
)""", re.X)


def _tokens(text: str) -> List[Tuple[str, str]]:
    out = []
    pos = 0
    text = text.strip()
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"cannot tokenize CREATE at {text[pos:pos + 30]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


class _Parser:
    def __init__(self, text: str):
        self.t = _tokens(text)
        self.i = 0
        self.next_id = 0
        self.vars: Dict[str, Tuple[str, int]] = {}
        self.nodes: List[dict] = []
        self.rels: List[dict] = []
        self._anon = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def eat(self, val=None, kind=None):
        k, v = self.peek()
        if (val is not None and v != val) or (kind is not None and k != kind):
            raise ValueError(f"expected {val or kind}, got {v!r}")
        self.i += 1
        return v

    def parse(self):
        while self.i < len(self.t):
            w = self.eat(kind="word")
            if w.upper() != "CREATE":
                raise ValueError(f"only CREATE is supported, got {w}")
            self.pattern_part()
            while self.peek()[1] == ",":
                self.eat(",")
                self.pattern_part()
        return {"nodes": self.nodes, "rels": self.rels}

    def value(self):
        k, v = self.peek()
        if k == "str":
            self.i += 1
            return v[1:-1].encode().decode("unicode_escape")
        if k == "num":
            self.i += 1
            is_float = v[-1] in "DF" or any(c in v for c in ".eE")
            v = v.rstrip("LDF")
            return float(v) if is_float else int(v)
        if k == "word" and v.lower() in ("true", "false", "null"):
            self.i += 1
            return {"true": True, "false": False, "null": None}[v.lower()]
        if v == "[":
            self.eat("[")
            out = []
            while self.peek()[1] != "]":
                out.append(self.value())
                if self.peek()[1] == ",":
                    self.eat(",")
            self.eat("]")
            return out
        raise ValueError(f"unsupported literal {v!r}")

    def props(self):
        out = {}
        if self.peek()[1] != "{":
            return out
        self.eat("{")
        while self.peek()[1] != "}":
            key = self.eat(kind="word")
            self.eat(":")
            out[key] = self.value()
            if self.peek()[1] == ",":
                self.eat(",")
        self.eat("}")
        return out

    def node(self) -> int:
        self.eat("(")
        var = None
        if self.peek()[0] == "word":
            var = self.eat(kind="word")
        labels = []
        while self.peek()[1] == ":":
            self.eat(":")
            labels.append(self.eat(kind="word"))
        props = self.props()
        self.eat(")")
        if var is not None and var in self.vars:
            kind, ident = self.vars[var]
            if kind != "node":
                raise ValueError(f"{var} is not a node")
            return ident
        ident = self.next_id
        self.next_id += 1
        self.nodes.append({"id": ident, "labels": sorted(labels), "props": props})
        if var is not None:
            self.vars[var] = ("node", ident)
        return ident

    def rel_pattern(self):
        incoming = False
        if self.peek()[1] == "<-":
            self.eat("<-")
            incoming = True
        else:
            self.eat("-")
        self.eat("[")
        var = None
        if self.peek()[0] == "word":
            var = self.eat(kind="word")
        self.eat(":")
        rtype = self.eat(kind="word")
        props = self.props()
        self.eat("]")
        if incoming:
            self.eat("-")
        else:
            self.eat("->")
        return var, rtype, props, incoming

    def pattern_part(self):
        left_end = self.node()   # id of the current chain head (node, or previous relationship's end)
        while self.peek()[1] in ("-", "<-"):
            var, rtype, props, incoming = self.rel_pattern()
            right = self.node()
            ident = self.next_id
            self.next_id += 1
            src, dst = (right, left_end) if incoming else (left_end, right)
            self.rels.append({"id": ident, "src": src, "dst": dst, "type": rtype, "props": props})
            if var is not None:
                self.vars[var] = ("rel", ident)
            left_end = dst  # CreateQueryParser: a chained relationship starts at the previous one's end id


def create_graph(text: str) -> dict:
    """{"nodes": [{"id", "labels", "props"}], "rels": [{"id", "src", "dst", "type", "props"}]}"""
    return _Parser(text).parse()
