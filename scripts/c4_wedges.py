"""Diagnostic (not product): wedge structure of the degree-oriented simple graph of R-MAT s (C4 planning).
Prints payload classes, wedge counts, how the wedges concentrate on high-degree middle vertices, the
u-side cost of a v-stationary walk and of rank-block tiling.  Usage: python3 scripts/c4_wedges.py 22"""
import numpy as np, sys
sys.path.insert(0, '.')
from oracle import cpu
s = int(sys.argv[1]); n = 1 << s
src, dst = cpu.rmat_edges(s, 0, 16 << s)
keep = src != dst
a = np.minimum(src[keep], dst[keep]); b = np.maximum(src[keep], dst[keep])
fwd = (src[keep] < dst[keep])
key = a.astype(np.int64) * n + b
order = np.argsort(key, kind='stable'); key = key[order]; fwd = fwd[order]
uk, idx, cnt = np.unique(key, return_index=True, return_counts=True)
mf = np.add.reduceat(fwd.astype(np.int64), idx); mb = cnt - mf   # m(min,max), m(max,min)
x = uk // n; y = uk % n
deg = np.bincount(x, minlength=n) + np.bincount(y, minlength=n)
# orient from lower (deg, id)
xf = (deg[x] < deg[y]) | ((deg[x] == deg[y]) & (x < y))
u = np.where(xf, x, y); v = np.where(xf, y, x)
F = np.where(xf, mf, mb); B = np.where(xf, mb, mf)   # m(u,v), m(v,u)
od = np.bincount(u, minlength=n)
E = len(u)
print(f"s={s}: undirected simple edges {E}, max od {od.max()}")
print("payload classes: (1,0) %.3f (0,1) %.3f (1,1) %.3f other %.3f" % (np.mean((F==1)&(B==0)), np.mean((F==0)&(B==1)), np.mean((F==1)&(B==1)), np.mean(~(((F==1)&(B==0))|((F==0)&(B==1))|((F==1)&(B==1))))))
# wedges per (u,v): od[v]
w_uv = od[v]
W = w_uv.sum(); print(f"wedges {W:.3e}")
# degree rank (descending deg, id)
rank = np.empty(n, np.int64); rank[np.lexsort((np.arange(n), -deg))] = np.arange(n)
for K in [1 << 12, 1 << 14, 1 << 16]:
    hot = rank[v] < K
    # bitmap bytes per (u,v) = rank(v)/8 (bits below v's rank); list bytes = 4*od(v)
    bm = (rank[v][hot] / 8.0).sum(); lst = (4.0 * w_uv[hot]).sum()
    print(f"K={K}: wedges with v in top-K {w_uv[hot].sum()/W:.3f}; list bytes {lst:.3e} vs bitmap bytes {bm:.3e}; "
          f"hot out-lists total {4*od[rank < K].sum()/1e6:.1f} MB")
usq = (od.astype(np.float64) ** 2).sum()
print(f"sum_u od(u)^2 = {usq:.3e} (u-side reads of a v-stationary walk) vs wedges {W:.3e}: ratio {W/usq:.2f}")
# v-stationary: per v, lists of in(v) read; also count pairs and max in-degree
ind = np.bincount(v, minlength=n)
print(f"max oriented in-degree {ind.max()}, vertices with od>64: {(od>64).sum()}")
# hybrid: per edge (u,v) read min(od(u), od(v)) (iterate the shorter list, probe the other side's hash)
mn = np.minimum(od[u], od[v]).astype(np.float64).sum()
print(f"sum over edges of min(od(u), od(v)) = {mn:.3e}: ratio to wedges {W/mn:.2f}")
for K in [1 << 14, 1 << 15, 1 << 16]:
    hu = rank[u] < K
    core_e = hu.sum()
    print(f"K={K}: wedges with u in top-K (all three in the core) {w_uv[hu].sum()/W:.3f}; core edges {core_e} "
          f"(density {core_e/(K*K/2):.3f}); dense KxK int8 {K*K/1e6:.0f} MB")
for K, bs in [(1 << 16, 64), (1 << 16, 256), (1 << 18, 256)]:
    hot = rank[v] < K
    blk = rank[v] // bs
    # per u: distinct hot blocks among out(u)
    uu = u[hot]; bb = blk[hot]
    pairs = np.unique(uu.astype(np.int64) * (n // bs + 1) + bb)
    ub = np.bincount(pairs // (n // bs + 1), minlength=n)
    tiled = (ub.astype(np.float64) * od).sum()
    stationary = (np.bincount(uu, minlength=n).astype(np.float64) * od).sum()
    cold = w_uv[~hot].sum()
    print(f"K={K} block {bs}: u-list reads tiled {tiled:.3e} vs per-v {stationary:.3e} (x{stationary/max(tiled,1):.1f}); "
          f"cold wedges {cold:.3e} ({cold/W:.2f}); hot bitmaps {K*K/16/1e6:.0f} MB")
