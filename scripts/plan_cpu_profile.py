"""Host cost of building the C3 plan in the planner mirror, on the CPU (diagnostic).  libcapsmi is
replaced by a stand-in that only tracks schemas (no device, no data), so what is timed is the Python
planner and the ctypes marshalling of the Table[T] calls -- the part of the routed step that runs
before the first kernel.  Usage: python3 scripts/plan_cpu_profile.py [iterations]"""
import cProfile
import ctypes
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
from capsmi import _lib  # noqa: E402
from capsmi.expr import I64  # noqa: E402
from capsmi.planner import EntityTable, Planner, ScanGraph  # noqa: E402
from capsmi.table import GpuTable  # noqa: E402

import bench  # noqa: E402

SCHEMA = {}
NEXT = [1]


def _new(names, types):
    h = NEXT[0]
    NEXT[0] += 1
    SCHEMA[h] = (list(names), list(types))
    return h


def _h(p):
    return p.value if isinstance(p, ctypes.c_void_p) else p


def _strs(arr, n):
    return [arr[i].decode() for i in range(n)]


def fake_call(name, *a):
    if name == "capsmi_table_schema":
        h, n, buf, _, types = _h(a[0]), a[1], a[2], a[3], a[4]
        names, tys = SCHEMA[h]
        n._obj.value = len(names)
        raw = b"".join(x.encode() + b"\0" for x in names)
        ctypes.memmove(buf, raw, len(raw))
        for i, t in enumerate(tys):
            types[i] = t
        return
    out = a[-1]._obj if hasattr(a[-1], "_obj") else None
    if name == "capsmi_with_columns":
        names, tys = SCHEMA[_h(a[0])]
        names, tys = list(names), list(tys)
        for i in range(a[1]):
            nm = a[2][i].name.decode()
            if nm in names:
                tys[names.index(nm)] = I64
            else:
                names.append(nm)
                tys.append(I64)
        out.value = _new(names, tys)
    elif name == "capsmi_select":
        names, tys = SCHEMA[_h(a[0])]
        sel = _strs(a[2], a[1])
        out.value = _new(sel, [tys[names.index(x)] for x in sel])
    elif name == "capsmi_join":
        l, r = SCHEMA[_h(a[0])], SCHEMA[_h(a[1])]
        out.value = _new(l[0] + r[0], l[1] + r[1])
    elif name in ("capsmi_filter", "capsmi_cache", "capsmi_distinct", "capsmi_skip", "capsmi_limit"):
        out.value = _new(*SCHEMA[_h(a[0])])
    elif name == "capsmi_group":
        names, tys = SCHEMA[_h(a[0])]
        by = _strs(a[2], a[1])
        aggs = [a[4][i].output.decode() for i in range(a[3])]
        out.value = _new(by + aggs, [tys[names.index(x)] for x in by] + [I64] * len(aggs))
    elif name == "capsmi_drop":
        names, tys = SCHEMA[_h(a[0])]
        drop = set(_strs(a[2], a[1]))
        keep = [i for i, x in enumerate(names) if x not in drop]
        out.value = _new([names[i] for i in keep], [tys[i] for i in keep])
    elif name == "capsmi_with_column_renamed":
        names, tys = SCHEMA[_h(a[0])]
        old, new = a[1].decode(), a[2].decode()
        out.value = _new([new if x == old else x for x in names], tys)
    elif name == "capsmi_union_all":
        out.value = _new(*SCHEMA[_h(a[0])])
    elif name == "capsmi_table_column_index":
        names, _ = SCHEMA[_h(a[0])]
        a[2]._obj.value = names.index(a[1].decode())
    elif name in ("capsmi_table_release",):
        pass
    else:
        raise NotImplementedError(name)


class FakeSession:
    handle = None

    def encode_str(self, s):
        return hash(s) & 0xFFFF


_lib.call = fake_call
_lib._lib = None  # GpuTable.__del__ releases nothing
sess = FakeSession()
persons = GpuTable(sess, ctypes.c_void_p(_new(["id"], [I64])))
rels = GpuTable(sess, ctypes.c_void_p(_new(["id", "source", "target"], [I64, I64, I64])))
sg = ScanGraph(sess, [EntityTable("node", frozenset({"Person"}), {}, persons, id_col="id")],
               [EntityTable("rel", frozenset({"FRIEND_OF"}), {}, rels, id_col="id", src_col="source", dst_col="target")])
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
for _ in range(50):
    Planner(sg).run(bench.C3_QUERY)
t0 = time.perf_counter()
for _ in range(N):
    Planner(sg).run(bench.C3_QUERY)
print(f"C3 plan build (stand-in library): {1e6 * (time.perf_counter() - t0) / N:.1f} us per query")
pr = cProfile.Profile()
pr.enable()
for _ in range(N // 4):
    Planner(sg).run(bench.C3_QUERY)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
