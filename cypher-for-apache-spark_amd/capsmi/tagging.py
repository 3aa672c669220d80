"""Multi-graph id tagging: the upper 10 bits of a 64-bit entity id name the graph it came from.

Restates okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/tagging/Tags.scala:33-123
(constants, pickFreeTag, setTag / getTag / replaceTag on Longs and on expressions) and
TagSupport.scala:31-86 (computeRetaggings, replacementsFor).  Retagging runs on the device as
ordinary ``withColumns`` expressions (BitwiseAnd / BitwiseOr / ShiftLeft / ShiftRightUnsigned /
CaseExpr, the same trees Tags.ExprTagging builds), so a UNION of graphs never leaves HBM.

Set iteration order: Scala's small immutable sets keep insertion order and its hash sets order
small Ints by value; the reference tests use ascending tags, so conflicts are renumbered here in
ascending order (TagSupportTest.scala:33-41 pins the results).
"""
from __future__ import annotations

from typing import Dict, Iterable, Mapping, Set

from .expr import BinOp, Case, Expr, Lit

TOTAL_BITS = 64
ID_BITS = 54                                 # Tags.scala:39
TAG_BITS = TOTAL_BITS - ID_BITS              # 10
MAX_TAG = (1 << TAG_BITS) - 1                # 1023
ALL_TAGS = frozenset(range(MAX_TAG + 1))
TAG_MASK = (-1 << ID_BITS) & ((1 << 64) - 1)  # as an unsigned 64-bit pattern
INVERTED_TAG_MASK = (1 << ID_BITS) - 1


class TagSpaceExhausted(RuntimeError):
    """okapi IllegalStateException("Could not complete this operation, ran out of tag space.")"""


def _signed(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def pick_free_tag(used: Iterable[int]) -> int:
    """Tags.pickFreeTag (Tags.scala:60-76)."""
    used = set(used)
    if not used:
        return 0
    mx = max(used)
    if mx < MAX_TAG:
        return mx + 1
    free = ALL_TAGS - used
    if not free:
        raise TagSpaceExhausted("Could not complete this operation, ran out of tag space.")
    return min(free)


# ---- Long tagging (Tags.LongTagging, :78-97) --------------------------------------------------
def set_tag(i: int, tag: int) -> int:
    return _signed((i & INVERTED_TAG_MASK) | (tag << ID_BITS))


def get_tag(i: int) -> int:
    return (i & ((1 << 64) - 1)) >> ID_BITS


def replace_tag(i: int, frm: int, to: int) -> int:
    return set_tag(i, to) if get_tag(i) == frm else i


def replace_tags(i: int, replacements: Mapping[int, int]) -> int:
    t = get_tag(i)
    return set_tag(i, replacements[t]) if t in replacements else i


# ---- expression tagging (Tags.ExprTagging, :99-123) -------------------------------------------
def expr_get_tag(e: Expr) -> Expr:
    return BinOp(">>>", e, Lit(ID_BITS))


def expr_set_tag(e: Expr, tag: int) -> Expr:
    return BinOp("|", BinOp("&", e, Lit(INVERTED_TAG_MASK)), BinOp("<<", Lit(tag), Lit(ID_BITS)))


def expr_replace_tags(e: Expr, replacements: Mapping[int, int]) -> Expr:
    """CaseExpr(getTag(e) = from -> setTag(e, to) ..., default e); identity pairs are kept, as the
    reference builds them (they are no-ops)."""
    alts = tuple((BinOp("=", expr_get_tag(e), Lit(frm)), expr_set_tag(e, to)) for frm, to in replacements.items())
    return Case(alts, e) if alts else e


def expr_replace_tag(e: Expr, frm: int, to: int) -> Expr:
    return expr_replace_tags(e, {frm: to})


# ---- TagSupport (:31-86) ------------------------------------------------------------------------
def replacements_for(lhs: Set[int], rhs: Set[int]) -> Dict[int, int]:
    """TagSet.replacementsFor: new tags for rhs so that none collides with lhs."""
    lhs, rhs = set(lhs), set(rhs)
    if not lhs and not rhs:
        return {}
    if not lhs:
        return {t: t for t in sorted(rhs)}
    if not rhs:
        return {t: t for t in sorted(lhs)}  # the reference's own (odd) branch, kept as is
    nxt = max(max(lhs), max(rhs)) + 1
    conflicts = sorted(lhs & rhs)
    out = {t: nxt + i for i, t in enumerate(conflicts)}
    for t in sorted(rhs - set(conflicts)):
        out[t] = t
    return out


def compute_retaggings(graphs: Mapping[object, Set[int]],
                       fixed: Mapping[object, Mapping[int, int]] = None) -> Dict[object, Dict[int, int]]:
    """TagSupport.computeRetaggings: per graph key, the tag replacements that make the graphs'
    ids disjoint; ``fixed`` retaggings are applied first and their target tags count as used."""
    fixed = dict(fixed or {})
    result: Dict[object, Dict[int, int]] = {k: dict(v) for k, v in fixed.items()}
    used: Set[int] = set()
    for v in fixed.values():
        used |= set(v.values())
    for key, tags in graphs.items():
        if key in fixed:
            continue
        rep = replacements_for(used, set(tags))
        used |= {rep.get(t, t) for t in tags}
        result[key] = rep
    return result
