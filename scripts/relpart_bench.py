"""Build time of the unfused 2-D layout (capsmi_relpart_build: pass 1 + pass 2, no hop) at C3 size,
per kernel from the library's HIP-event timers (diagnostic; CAPSMI_PAIRS=uint2 for the 8-byte form).
Usage: python3 scripts/relpart_bench.py [scale] [builds]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cypher-for-apache-spark_amd")]
import torch  # noqa: E402
from capsmi import Session, _lib, graph  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
builds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
s = Session(0)
s.set_stream(torch.cuda.current_stream().cuda_stream)
n = 1 << scale
rels = graph.rmat_rels(s, scale, 0, 16 << scale, graph.RMAT_GRAPH500, 42)
for _ in range(2):
    graph.RelPartition(s, [rels], 0, n).release()
s.sync()
_lib.call("capsmi_session_set_profiling", s.handle, 1)


def ktime(name):
    cnt, ms = ctypes.c_int64(), ctypes.c_double()
    _lib.call("capsmi_session_kernel_time", s.handle, name.encode(), ctypes.byref(cnt), ctypes.byref(ms))
    return cnt.value, ms.value


for k in ("part_scatter1", "part_scatter2"):
    ktime(k)
t0 = time.perf_counter()
for _ in range(builds):
    graph.RelPartition(s, [rels], 0, n).release()
s.sync()
dt = (time.perf_counter() - t0) / builds
out = {k: ktime(k) for k in ("part_scatter1", "part_scatter2")}
print(f"pairs={os.environ.get('CAPSMI_PAIRS', 'packed')} build {1e3 * dt:.3f} ms/build; " +
      ", ".join(f"{k} {v[1] / max(v[0], 1):.3f} ms" for k, v in out.items()))
