"""Diagnostic (not product): line reads of the C4 v-mode walks, per center (the current kernel) against
prefix reuse over groups of consecutive hub centers (one walk of out(u)'s prefix per (u, group), tested
against an LDS table of the group's out-lists: 2 bits per (center, w) over [0, v_last)).
Usage: python3 scripts/c4_groups.py 22 [lds_bytes] [gmax]"""
import numpy as np, sys
sys.path.insert(0, '.')
from oracle import cpu

s = int(sys.argv[1]); n = 1 << s
lds = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 17
gmax = int(sys.argv[3]) if len(sys.argv) > 3 else 64
hashes = int(sys.argv[4]) if len(sys.argv) > 4 else 1
VMT = 256
import os
cache = f"/tmp/c4_groups_s{s}.npz"
if os.path.exists(cache):
    z = np.load(cache); u = z["u"]; v = z["v"]
else:
    src, dst = cpu.rmat_edges(s, 0, 16 << s)
    keep = src != dst
    a = np.minimum(src[keep], dst[keep]); b = np.maximum(src[keep], dst[keep])
    del src, dst, keep
    uk = np.unique(a.astype(np.int64) * n + b)
    del a, b
    x = uk // n; y = uk % n
    deg = np.bincount(x, minlength=n) + np.bincount(y, minlength=n)
    rank = np.empty(n, np.int64); rank[np.lexsort((np.arange(n), -deg))] = np.arange(n)
    rx, ry = rank[x], rank[y]
    u = np.maximum(rx, ry); v = np.minimum(rx, ry)   # oriented towards the smaller degree-order id
    o = np.lexsort((v, u)); u = u[o].astype(np.int32); v = v[o].astype(np.int32)
    np.savez(cache, u=u, v=v)
u = u.astype(np.int64); v = v.astype(np.int64)
E = len(u)
od = np.bincount(u, minlength=n)
off = np.zeros(n + 1, np.int64); off[1:] = np.cumsum(od)
p = np.arange(E) - off[u]                          # position of v in out(u)
vm = (od[v] >= VMT) & (p < od[v])
print(f"s={s}: E={E}, v-mode edges {vm.sum()} ({vm.mean():.3f}), centers {np.unique(v[vm]).size}")

def lines(start, length):
    a0 = (4 * start) // 128; a1 = (4 * (start + length) + 127) // 128
    return np.where(length > 0, a1 - a0, 0)

uu, vv, pp = u[vm], v[vm], p[vm]
cur_entries = pp.sum(); cur_lines = lines(off[uu], pp).sum()
print(f"per center: prefix entries {cur_entries:.3e}, lines {cur_lines:.3e}")
# groups of consecutive centers: G * v_last * 2 bits <= lds * 8, G <= gmax
cs = np.unique(vv)
gid = np.empty(cs.size, np.int64); g = 0; first = 0
cost = np.zeros(cs.size, np.int64)
for i in range(cs.size):
    G = i - first + 1
    cost[i] = min((cs[i] + 32) // 32 * 6 + od[cs[i]], 8 * od[cs[i]]) if hashes else (cs[i] + 32) // 32 * 6 + od[cs[i]]
    if G > gmax or cost[first:i + 1].sum() > lds:
        g += 1; first = i
    gid[i] = g
ng = g + 1
cg = gid[np.searchsorted(cs, vv)]
key = uu * ng + cg
ordk = np.argsort(key, kind='stable')
k2 = key[ordk]; p2 = pp[ordk]; u2 = uu[ordk]
st = np.flatnonzero(np.r_[True, k2[1:] != k2[:-1]])
pmax = np.maximum.reduceat(p2, st)
ug = u2[st]
grp_entries = pmax.sum(); grp_lines = lines(off[ug], pmax).sum()
sizes = np.bincount(gid)
print(f"groups {ng} (size mean {sizes.mean():.1f}, max {sizes.max()}), walks {st.size} vs {uu.size}")
print(f"grouped: prefix entries {grp_entries:.3e} (x{cur_entries/grp_entries:.2f}), lines {grp_lines:.3e} (x{cur_lines/grp_lines:.2f})")
# by center range
for lo, hi in [(0, 1 << 12), (1 << 12, 1 << 14), (1 << 14, 1 << 16), (1 << 16, n)]:
    m = (vv >= lo) & (vv < hi)
    print(f"  centers [{lo}, {hi}): per-center lines {lines(off[uu[m]], pp[m]).sum():.3e}")
