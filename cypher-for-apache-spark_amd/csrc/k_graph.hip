// k_graph.hip -- fused pattern kernels over relationship tables (the hot path).
//
// CAPS lowers `(a)-[r]->(b)` to `a ⋈[a.id = r.source] rels ⋈[r.target = b.id] b`
// (RelationalPlanner.scala:113-124).  When both node scans are base node tables with
// dense Long ids, each node scan + label/property filter collapses to one bit per id,
// and each join against it is a bit test.  The relationship table is then streamed
// once per hop -- the HBM-bound part -- and no binding is ever materialised.
//
// Layout in HBM: a relationship table is three int64 columns (id, source, target),
// 8 B per value, coalesced 16 B per lane per load.  Node predicates are uint32 word
// bitmaps over [lo, hi): 2^26 ids -> 8 MiB, resident in the Infinity Cache.
#include "capsmi_impl.h"

namespace capsmi {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

namespace {

// id-domain predicate view passed to kernels
struct BitView {
    const uint32_t* w;
    int64_t lo, hi;
    int full;  // every id in [lo, hi) set: only a range test is needed
};

__device__ __forceinline__ bool bit_ok(const BitView& b, int64_t id) {
    if (id < b.lo || id >= b.hi) return false;
    if (b.full) return true;
    const uint64_t x = (uint64_t)(id - b.lo);
    return (b.w[x >> 5] >> (x & 31)) & 1u;
}

// Set bit `x` (relative id) in `w` for every active lane, combining lanes that hit the same
// word first (segmented OR over the wave; clustered inputs put runs of equal words in
// adjacent lanes), then one check-before-atomicOr per distinct word run.  A plain read that
// misses a bit set on another XCD only costs a redundant atomic: bits are only ever set.
__device__ __forceinline__ void wave_set_bit(uint32_t* w, int64_t x, bool act) {
    const int lane = threadIdx.x & 63;
    int64_t word = act ? (x >> 5) : -1;
    uint32_t m = act ? (1u << (x & 31)) : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t wo = __shfl_down(word, o, 64);
        const uint32_t mo = __shfl_down(m, o, 64);
        if (lane + o < 64 && wo == word) m |= mo;
    }
    const int64_t prev = __shfl_up(word, 1, 64);
    const bool head = act && (lane == 0 || prev != word);
    if (head) {
        const uint32_t cur = w[word];
        if ((cur & m) != m) atomicOr(&w[word], m);
    }
}

// ---- node-scan bitmaps ----------------------------------------------------------
// A wave takes 256 consecutive rows (4 per lane, two 16-B loads).  Fast path: no row filter, no
// nulls, and the wave's ids are one ascending run id0 .. id0+255 inside [lo, hi) -- a base node
// table -- so 9 lanes OR whole word masks.  Otherwise each of the 4 rows per lane goes through a
// segmented OR over lanes hitting the same word (one atomic per word run, duplicates counted
// exactly), which is cheap for clustered ids and correct for any order.  Counters are reduced
// per block before one atomic each.
__device__ __forceinline__ void bitmap_generic(uint32_t* w, int64_t lo, int64_t hi, int64_t id, bool act, bool valid,
                                               unsigned long long& added, unsigned long long& dups,
                                               unsigned long long& bad) {
    const int lane = threadIdx.x & 63;
    int64_t x = 0;
    if (act) {
        if (!valid || id < lo || id >= hi) {
            ++bad;
            act = false;
        } else {
            x = id - lo;
        }
    }
    int64_t word = act ? (x >> 5) : -1;
    uint32_t m = act ? (1u << (x & 31)) : 0u;
    uint32_t cnt = act ? 1u : 0u;
    // segmented suffix reduction over runs of equal `word` in adjacent lanes: `tail` marks
    // that the lane's current window [lane, lane+o) already contains the end of its run
    const int64_t next = __shfl_down(word, 1, 64);
    bool tail = lane == 63 || next != word;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t mo = __shfl_down(m, o, 64);
        const uint32_t co = __shfl_down(cnt, o, 64);
        const bool to = __shfl_down((int)tail, o, 64) != 0;
        if (!tail) {
            m |= mo;
            cnt += co;
            tail = to;
        }
    }
    const int64_t prev = __shfl_up(word, 1, 64);
    if (act && (lane == 0 || prev != word)) {
        const uint32_t old = atomicOr(&w[word], m);
        added += cnt;
        dups += (cnt - (uint32_t)__popc(m)) + (uint32_t)__popc(old & m);
    }
}

__device__ __forceinline__ bool range_ok(const RangePred& rp, int64_t i) {
    bool ok = true;
    for (int k = 0; k < rp.n; ++k) {
        const int64_t v = rp.col[k][i];
        ok = ok && (!rp.valid[k] || rp.valid[k][i]) && v >= rp.lo[k] && v <= rp.hi[k];
    }
    return ok;
}

__global__ void __launch_bounds__(256) k_bitmap_add(uint32_t* w, int64_t lo, int64_t hi, const int64_t* __restrict__ ids,
                                                    const uint8_t* __restrict__ ids_valid,
                                                    const uint8_t* __restrict__ flags, int64_t n, int aligned,
                                                    unsigned long long* counters /* [0]=added, [1]=dups, [2]=bad */,
                                                    RangePred rp) {
    __shared__ unsigned long long red[3][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long added = 0, dups = 0, bad = 0;
    const int64_t stride = (int64_t)gridDim.x * 1024;
    for (int64_t base = (int64_t)blockIdx.x * 1024 + wave * 256; base < n; base += stride) {
        // row base + 128 * k + 2 * lane + j  (k, j in {0, 1}): two coalesced 16-B loads per lane
        int64_t id[4];
        const bool whole = aligned && base + 256 <= n;
        if (whole) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const longlong2 v = reinterpret_cast<const longlong2*>(ids + base + 128 * k)[lane];
                id[2 * k] = v.x;
                id[2 * k + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t i = base + 128 * (u >> 1) + 2 * lane + (u & 1);
                id[u] = i < n ? ids[i] : 0;
            }
        }
        const int64_t id0 = __shfl(id[0], 0, 64);
        bool run = whole && !flags && !ids_valid && rp.n == 0 && id0 >= lo && id0 + 256 <= hi;
#pragma unroll
        for (int u = 0; u < 4; ++u) run = run && id[u] == id0 + 128 * (u >> 1) + 2 * lane + (u & 1);
        if (__ballot(!run) == 0) {  // wave-uniform: one ascending run of 256 ids
            const int64_t x0 = id0 - lo, w0 = x0 >> 5;
            const int64_t k = lane;  // word w0 + k covers bits [32 (w0 + k), 32 (w0 + k + 1)) - x0 of the run
            if (k <= 8) {
                const int64_t b0 = (w0 + k) * 32 - x0;  // run offset of the word's bit 0
                const int64_t s = b0 < 0 ? 0 : b0, t = b0 + 32 > 256 ? 256 : b0 + 32;
                if (t > s) {
                    const uint32_t m = (uint32_t)((((t - s) == 32) ? 0xFFFFFFFFull : ((1ull << (t - s)) - 1)) << (s - b0));
                    const uint32_t old = atomicOr(&w[w0 + k], m);
                    dups += (uint32_t)__popc(old & m);
                }
            }
            if (lane == 0) added += 256;
            continue;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + 128 * (u >> 1) + 2 * lane + (u & 1);
            const bool act = i < n && (!flags || flags[i]) && range_ok(rp, i);
            const bool valid = act && (!ids_valid || ids_valid[i]);
            bitmap_generic(w, lo, hi, id[u], act, valid, added, dups, bad);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        added += __shfl_down(added, o, 64);
        dups += __shfl_down(dups, o, 64);
        bad += __shfl_down(bad, o, 64);
    }
    if (lane == 0) {
        red[0][wave] = added;
        red[1][wave] = dups;
        red[2][wave] = bad;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (v) atomicAdd(&counters[threadIdx.x], v);
    }
}

// popcount of words [b, e): 16-B loads where aligned, block reduction, one atomic per block
__global__ void __launch_bounds__(256) k_popcount(const uint32_t* __restrict__ w, int64_t b, int64_t e,
                                                  unsigned long long* out) {
    __shared__ unsigned long long red[4];
    unsigned long long c = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = b + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t a = (b + 3) & ~int64_t(3);  // first 16-B aligned word
    if (a <= e) {
        for (int64_t k = b + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a; k += stride) c += __popc(w[k]);
        const int64_t nq = (e - a) >> 2;
        const uint4* q = reinterpret_cast<const uint4*>(w + a);
        for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nq; k += stride) {
            const uint4 v = q[k];
            c += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        }
        for (int64_t k = a + 4 * nq + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < e; k += stride) c += __popc(w[k]);
    } else {
        for (; i < e; i += stride) c += __popc(w[i]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = red[0] + red[1] + red[2] + red[3];
        if (t) atomicAdd(out, t);
    }
}

// ---- C2: 1-hop expand with fused node filters --------------------------------------
// Output rows are reserved per block with one atomic (row order across blocks is
// unspecified: results are multisets, as Spark's).
constexpr int kMaxOut = 4;
struct OutCols {
    const int64_t* src[kMaxOut];
    const uint8_t* srcv[kMaxOut];
    int64_t* dst[kMaxOut];
    uint8_t* dstv[kMaxOut];
    int n;
};

// One 8192-relationship tile per iteration: all loads in flight (16-byte pairs when the columns
// are aligned), bitmap tests, wave-aggregated LDS ranks of the kept rows, ONE global atomic per
// tile for the output run, then the projected columns are gathered in tile order and written as
// one contiguous run (coalesced).  Output order across tiles is unspecified (bag semantics).
constexpr int kEfBlock = 1024, kEfItems = 8, kEfTile = kEfBlock * kEfItems;

__global__ void __launch_bounds__(kEfBlock) k_expand_filter(const int64_t* __restrict__ src,
                                                            const int64_t* __restrict__ dst, int64_t m, int aligned,
                                                            BitView a, BitView b, OutCols oc,
                                                            unsigned long long* __restrict__ out_count) {
    __shared__ unsigned short rows[kEfTile];  // tile-relative offsets of the kept rows
    __shared__ unsigned int nkept;
    __shared__ unsigned long long run;
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane == 0 ? 0ULL : (~0ULL >> (64 - lane));
    for (int64_t t0 = (int64_t)blockIdx.x * kEfTile; t0 < m; t0 += (int64_t)gridDim.x * kEfTile) {
        if (threadIdx.x == 0) nkept = 0;
        int64_t s[kEfItems], t[kEfItems];
        const bool full = t0 + kEfTile <= m;
        if (aligned && full) {
#pragma unroll
            for (int k = 0; k < kEfItems / 2; ++k) {
                const int i = k * kEfBlock + (int)threadIdx.x;
                const longlong2 sv = reinterpret_cast<const longlong2*>(src + t0)[i];
                const longlong2 tv = reinterpret_cast<const longlong2*>(dst + t0)[i];
                s[2 * k] = sv.x; s[2 * k + 1] = sv.y; t[2 * k] = tv.x; t[2 * k + 1] = tv.y;
            }
        } else {
            const int last = (int)(min(m - t0, (int64_t)kEfTile) - 1);
#pragma unroll
            for (int u = 0; u < kEfItems; ++u) {
                const int i = min(2 * ((u >> 1) * kEfBlock + (int)threadIdx.x) + (u & 1), last);
                s[u] = src[t0 + i];
                t[u] = dst[t0 + i];
            }
        }
        __syncthreads();  // nkept reset visible
#pragma unroll
        for (int u = 0; u < kEfItems; ++u) {
            const int off = 2 * ((u >> 1) * kEfBlock + (int)threadIdx.x) + (u & 1);
            const bool keep = t0 + off < m && bit_ok(a, s[u]) && bit_ok(b, t[u]);
            const unsigned long long bal = __ballot(keep);
            unsigned int base = 0;
            if (lane == 0 && bal) base = atomicAdd(&nkept, (unsigned int)__popcll(bal));
            base = __shfl(base, 0, 64);
            if (keep) rows[base + __popcll(bal & lt)] = (unsigned short)off;
        }
        __syncthreads();
        const unsigned int total = nkept;
        if (threadIdx.x == 0) run = total ? atomicAdd(out_count, (unsigned long long)total) : 0ULL;
        __syncthreads();
        const unsigned long long r0 = run;
        for (unsigned int i = threadIdx.x; i < total; i += kEfBlock) {
            const int64_t e = t0 + rows[i];
            for (int c = 0; c < oc.n; ++c) {
                oc.dst[c][r0 + i] = oc.src[c][e];
                if (oc.dstv[c]) oc.dstv[c][r0 + i] = oc.srcv[c] ? oc.srcv[c][e] : 1;
            }
        }
        __syncthreads();  // rows / nkept reused by the next tile
    }
}

// Fast path when every projected column is the relationship's source or target (no nulls): the
// kept values are written straight from registers.  Both bitmap tests are random L2/MALL reads,
// the bound of this kernel; the target test is only issued for rows whose source passed.  Per
// tile: wave ballots rank the kept rows, a 16-entry LDS scan orders the waves, one global atomic
// reserves the tile's output run; item-major output order within the tile.
constexpr int kEpBlock = 512, kEpItems = 8, kEpTile = kEpBlock * kEpItems;  // 2 blocks per CU at 85 VGPRs

template <int NOUT>
__global__ void __launch_bounds__(kEpBlock) k_expand_pairs(const int64_t* __restrict__ src,
                                                           const int64_t* __restrict__ dst, int64_t m, int aligned,
                                                           BitView a, BitView b, uint32_t from_dst,
                                                           int64_t* __restrict__ o0, int64_t* __restrict__ o1,
                                                           int64_t* __restrict__ o2, int64_t* __restrict__ o3,
                                                           unsigned long long* __restrict__ out_count) {
    __shared__ unsigned int woff[kEpBlock / 64 + 1];
    __shared__ unsigned long long run;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long lt = lane == 0 ? 0ULL : (~0ULL >> (64 - lane));
    int64_t* const outs[4] = {o0, o1, o2, o3};
    const uint64_t ar = (uint64_t)(a.hi - a.lo), br = (uint64_t)(b.hi - b.lo);
    typedef long long v2i64 __attribute__((ext_vector_type(2)));
    // tile loads; the next tile's are issued while the current tile's bitmap tests are in flight
    auto load = [&](int64_t t0, int64_t (&s)[kEpItems], int64_t (&t)[kEpItems]) {
        if (t0 >= m) return;
        if (aligned && t0 + kEpTile <= m) {
#pragma unroll
            for (int k = 0; k < kEpItems / 2; ++k) {
                const int i = k * kEpBlock + (int)threadIdx.x;
                // streamed once: non-temporal, so the lines do not displace the bitmaps in L2
                const v2i64 sv = __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(src + t0) + i);
                const v2i64 tv = __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(dst + t0) + i);
                s[2 * k] = sv.x; s[2 * k + 1] = sv.y; t[2 * k] = tv.x; t[2 * k + 1] = tv.y;
            }
        } else {
            const int last = (int)(min(m - t0, (int64_t)kEpTile) - 1);
#pragma unroll
            for (int u = 0; u < kEpItems; ++u) {
                const int i = min(2 * ((u >> 1) * kEpBlock + (int)threadIdx.x) + (u & 1), last);
                s[u] = src[t0 + i];
                t[u] = dst[t0 + i];
            }
        }
    };
    const int64_t stride = (int64_t)gridDim.x * kEpTile;
    int64_t s[kEpItems], t[kEpItems], ns[kEpItems], nt[kEpItems];
    load((int64_t)blockIdx.x * kEpTile, s, t);
    for (int64_t t0 = (int64_t)blockIdx.x * kEpTile; t0 < m; t0 += stride) {
        // source test for all items (loads in flight together), then target test for the survivors
        bool keep[kEpItems];
        uint32_t wv[kEpItems];
#pragma unroll
        for (int u = 0; u < kEpItems; ++u) {
            const int off = 2 * ((u >> 1) * kEpBlock + (int)threadIdx.x) + (u & 1);
            const uint64_t x = (uint64_t)(s[u] - a.lo);
            keep[u] = t0 + off < m && x < ar;
            wv[u] = (keep[u] && !a.full) ? a.w[x >> 5] : ~0u;
        }
        load(t0 + stride, ns, nt);
#pragma unroll
        for (int u = 0; u < kEpItems; ++u) {
            const uint64_t x = (uint64_t)(s[u] - a.lo), y = (uint64_t)(t[u] - b.lo);
            keep[u] = keep[u] && ((wv[u] >> (x & 31)) & 1u) && y < br;
            wv[u] = (keep[u] && !b.full) ? b.w[y >> 5] : ~0u;
        }
        unsigned long long bal[kEpItems];
        unsigned int wcnt = 0;
#pragma unroll
        for (int u = 0; u < kEpItems; ++u) {
            const uint64_t y = (uint64_t)(t[u] - b.lo);
            keep[u] = keep[u] && ((wv[u] >> (y & 31)) & 1u);
            bal[u] = __ballot(keep[u]);
            wcnt += (unsigned int)__popcll(bal[u]);
        }
        if (lane == 0) woff[wave] = wcnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned int acc = 0;
            for (int k = 0; k < kEpBlock / 64; ++k) {
                const unsigned int c = woff[k];
                woff[k] = acc;
                acc += c;
            }
            run = acc ? atomicAdd(out_count, (unsigned long long)acc) : 0ULL;
        }
        __syncthreads();
        unsigned long long pos = run + woff[wave];
#pragma unroll
        for (int u = 0; u < kEpItems; ++u) {
            if (keep[u]) {
                const unsigned long long at = pos + __popcll(bal[u] & lt);
#pragma unroll
                for (int c = 0; c < NOUT; ++c) __builtin_nontemporal_store(((from_dst >> c) & 1u) ? t[u] : s[u], &outs[c][at]);
            }
            pos += __popcll(bal[u]);
        }
#pragma unroll
        for (int u = 0; u < kEpItems; ++u) {
            s[u] = ns[u];
            t[u] = nt[u];
        }
        __syncthreads();  // woff / run reused by the next tile
    }
}

// ---- C3: 2-hop count(DISTINCT c) ------------------------------------------------------
// hop 1: for every rel (s -> t):
//   s != t, a_ok(s), b_ok(t)           -> M(t)  (b has an in-edge that differs from any r2 leaving b
//                                                 towards c != b)
//   s == t, a_ok(s), b_ok(s)           -> S1(s); a second such self-loop -> S2(s)
// combine: X1 = M | S1 (middle for r2 not a self-loop), X2 = M | S2 (middle for a self-loop r2,
//   which needs an a_ok in-edge other than r2 itself).
// hop 2: for every rel (b -> c) with c_ok(c): (b != c ? X1(b) : X2(b)) -> C(c)
// count(DISTINCT c) = popcount(C).  Matches the enumeration in oracle/rmat.c.
// two consecutive rels per lane: one 16-B load per column when the column view is 16-B aligned
__device__ __forceinline__ void load2(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t e0,
                                      int64_t m, int aligned, int64_t (&s)[2], int64_t (&t)[2]) {
    if (aligned && e0 + 1 < m) {
        const longlong2 sv = *reinterpret_cast<const longlong2*>(src + e0);
        const longlong2 tv = *reinterpret_cast<const longlong2*>(dst + e0);
        s[0] = sv.x; s[1] = sv.y; t[0] = tv.x; t[1] = tv.y;
    } else {
        s[0] = e0 < m ? src[e0] : -1;
        t[0] = e0 < m ? dst[e0] : -1;
        s[1] = e0 + 1 < m ? src[e0 + 1] : -1;
        t[1] = e0 + 1 < m ? dst[e0 + 1] : -1;
    }
}

template <bool A_FULL, bool B_FULL>
__global__ void __launch_bounds__(256) k_hop1(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                              int64_t m, int aligned, BitView a, BitView b, uint32_t* __restrict__ M,
                                              uint32_t* __restrict__ S1, uint32_t* __restrict__ S2) {
    // wave-uniform trip count: every lane of a wave runs the same iterations, so the
    // cross-lane bit combining in wave_set_bit never reads an exited lane
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 2;
    const int lane = threadIdx.x & 63;
    for (int64_t wbase = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)) * 2; wbase < m; wbase += stride) {
        const int64_t e0 = wbase + 2 * lane;
        int64_t s[2], t[2];
        load2(src, dst, e0, m, aligned, s, t);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool valid = (e0 + k < m);
            const bool aok = valid && (A_FULL ? (s[k] >= a.lo && s[k] < a.hi) : bit_ok(a, s[k]));
            const bool bok = aok && (B_FULL ? (t[k] >= b.lo && t[k] < b.hi) : bit_ok(b, t[k]));
            const bool loop = s[k] == t[k];
            wave_set_bit(M, t[k] - b.lo, bok && !loop);
            if (bok && loop) {  // rare: self-loops
                const uint64_t x = (uint64_t)(t[k] - b.lo);
                const uint32_t bit = 1u << (x & 31);
                const uint32_t old = atomicOr(&S1[x >> 5], bit);
                if (old & bit) atomicOr(&S2[x >> 5], bit);
            }
        }
    }
}

__global__ void k_mid_combine(uint32_t* __restrict__ X1 /* in: M */, uint32_t* __restrict__ X2 /* in: S2 */,
                              const uint32_t* __restrict__ S1, int64_t nw) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t m = X1[i];
        X1[i] = m | S1[i];
        X2[i] = m | X2[i];
    }
}

template <bool C_FULL>
__global__ void __launch_bounds__(256) k_hop2(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                              int64_t m, int aligned, BitView c, const uint32_t* __restrict__ X1,
                                              const uint32_t* __restrict__ X2, int64_t mid_lo, int64_t mid_hi,
                                              uint32_t* __restrict__ C) {
    // wave-uniform trip count: every lane of a wave runs the same iterations, so the
    // cross-lane bit combining in wave_set_bit never reads an exited lane
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 2;
    const int lane = threadIdx.x & 63;
    for (int64_t wbase = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)) * 2; wbase < m; wbase += stride) {
        const int64_t e0 = wbase + 2 * lane;
        int64_t s[2], t[2];
        load2(src, dst, e0, m, aligned, s, t);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const bool valid = (e0 + k < m);
            const bool cok = valid && (C_FULL ? (t[k] >= c.lo && t[k] < c.hi) : bit_ok(c, t[k]));
            bool hit = false;
            if (cok && s[k] >= mid_lo && s[k] < mid_hi) {
                const uint64_t x = (uint64_t)(s[k] - mid_lo);
                const uint32_t* X = (s[k] == t[k]) ? X2 : X1;
                hit = (X[x >> 5] >> (x & 31)) & 1u;
            }
            wave_set_bit(C, t[k] - c.lo, hit);
        }
    }
}

// ---- closed-form count(*) (matched rows) --------------------------------------------
// inA(b) = #rels x->b with a_ok(x); outC(b) = #rels b->y with c_ok(y)
__global__ void k_degrees(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, BitView a,
                          BitView b, BitView c, unsigned int* __restrict__ inA, unsigned int* __restrict__ outC,
                          unsigned long long* __restrict__ loops) {
    unsigned long long nl = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e], t = dst[e];
        const bool sa = bit_ok(a, s), tc = bit_ok(c, t);
        if (sa && t >= b.lo && t < b.hi) atomicAdd(&inA[t - b.lo], 1u);
        if (tc && s >= b.lo && s < b.hi) atomicAdd(&outC[s - b.lo], 1u);
        if (s == t && sa && tc && bit_ok(b, s)) ++nl;
    }
    if (nl) atomicAdd(loops, nl);
}

__global__ void k_deg_product(const unsigned int* __restrict__ inA, const unsigned int* __restrict__ outC, int64_t n,
                              BitView b, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (bit_ok(b, b.lo + i)) acc += (unsigned long long)inA[i] * (unsigned long long)outC[i];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// ---- synthetic R-MAT (definition: oracle/rmat.c rmat_edge) -----------------------------
__device__ __forceinline__ void rmat_edge(int scale, uint64_t tA, uint64_t tAB, uint64_t tABC, uint64_t seed, uint64_t e,
                                          int64_t* so, int64_t* dout) {
    uint64_t s = 0, d = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
        if ((l & 1) == 0) r = splitmix64((seed << 40) | (e << 5) | (uint64_t)(l >> 1));
        const uint64_t u = (l & 1) == 0 ? (r >> 32) : (r & 0xffffffffULL);
        const uint64_t sb = u >= tAB;                       // quadrants C, D
        const uint64_t db = (u >= tA && u < tAB) || u >= tABC;  // quadrants B, D
        s |= sb << (scale - 1 - l);
        d |= db << (scale - 1 - l);
    }
    const uint64_t mask = (1ULL << scale) - 1;
    *so = (int64_t)((s * 0x9E3779B97F4A7C15ULL) & mask);
    *dout = (int64_t)((d * 0x9E3779B97F4A7C15ULL) & mask);
}

__device__ __forceinline__ int owner_of_word(int64_t word, int64_t nwords, int nparts) {
    int p = (int)((word * nparts) / nwords);
    while (p + 1 < nparts && ((int64_t)(p + 1) * nwords) / nparts <= word) ++p;
    while (p > 0 && ((int64_t)p * nwords) / nparts > word) --p;
    return p;
}

struct RmatArgs {
    int scale;
    uint64_t tA, tAB, tABC, seed;
    int64_t e_begin, e_end;
    int part_col, part, nparts;
    int64_t nwords;
};

__device__ __forceinline__ bool rmat_keep(const RmatArgs& g, int64_t s, int64_t d) {
    if (g.part_col < 0 || g.nparts <= 1) return true;
    const int64_t id = g.part_col == 0 ? s : d;
    return owner_of_word(id >> 5, g.nwords, g.nparts) == g.part;
}

__global__ void k_rmat_count(RmatArgs g, unsigned long long* __restrict__ tile_cnt) {
    const int64_t e = g.e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool keep = false;
    if (e < g.e_end) {
        int64_t s, d;
        rmat_edge(g.scale, g.tA, g.tAB, g.tABC, g.seed, (uint64_t)e, &s, &d);
        keep = rmat_keep(g, s, d);
    }
    const unsigned long long bal = __ballot(keep);
    __shared__ unsigned int ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = (unsigned)__popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void k_rmat_write(RmatArgs g, const int64_t* __restrict__ tile_off, int64_t* __restrict__ id,
                             int64_t* __restrict__ so, int64_t* __restrict__ dout) {
    const int64_t e = g.e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool keep = false;
    int64_t s = 0, d = 0;
    if (e < g.e_end) {
        rmat_edge(g.scale, g.tA, g.tAB, g.tABC, g.seed, (uint64_t)e, &s, &d);
        keep = rmat_keep(g, s, d);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long bal = __ballot(keep);
    __shared__ unsigned int ws[4];
    if (lane == 0) ws[wid] = (unsigned)__popcll(bal);
    __syncthreads();
    if (keep) {
        const unsigned long long lt = lane == 0 ? 0ULL : (~0ULL >> (64 - lane));
        int64_t pos = tile_off[blockIdx.x] + __popcll(bal & lt);
        for (int w = 0; w < wid; ++w) pos += ws[w];
        id[pos] = e;
        so[pos] = s;
        dout[pos] = d;
    }
}

__global__ void k_person_flags(int64_t n, int want_person, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const bool p = (splitmix64((uint64_t)i) & 3ULL) != 0;
        f[i] = (p == (want_person != 0)) ? 1 : 0;
    }
}

__global__ void k_age(const int64_t* __restrict__ ids, int64_t n, uint64_t seed, int64_t* __restrict__ age) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        age[i] = (int64_t)(splitmix64(seed ^ (uint64_t)ids[i]) % 100ULL);
}

// ---- row fingerprint ---------------------------------------------------
constexpr int kMaxFp = 8;
struct FpCols {
    const int64_t* d[kMaxFp];
    const uint8_t* v[kMaxFp];
    int n;
};
__global__ void k_fingerprint(FpCols fc, int64_t n, unsigned long long* __restrict__ out /* sum, xor */) {
    unsigned long long hs = 0, hx = 0;
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = 0x243F6A8885A308D3ULL;
        for (int c = 0; c < fc.n; ++c) {
            const bool ok = fc.v[c] == nullptr || fc.v[c][r];
            const uint64_t v = ok ? (uint64_t)fc.d[c][r] : 0x7FF8DEADBEEF0001ULL;  // NULL sentinel
            h = splitmix64(h ^ v);
        }
        hs += h;
        hx ^= h;
    }
    for (int o = 32; o > 0; o >>= 1) {
        hs += __shfl_down(hs, o, 64);
        hx ^= __shfl_down(hx, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], hs);
        atomicXor(&out[1], hx);
    }
}

// bits [b0, b1) of w set, the other bits of the words they touch kept (a registered node table whose
// ids are exactly one window, capsmi_bitmap_add_scan)
__global__ void k_bits_range(uint32_t* __restrict__ w, int64_t b0, int64_t b1) {
    const int64_t w0 = b0 >> 5, w1 = (b1 + 31) >> 5;
    for (int64_t i = w0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w1; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = i * 32 > b0 ? i * 32 : b0, hi = i * 32 + 32 < b1 ? i * 32 + 32 : b1;
        const uint32_t m = (uint32_t)(((hi - lo) == 32 ? 0xFFFFFFFFull : ((1ull << (hi - lo)) - 1)) << (lo - i * 32));
        w[i] = m == 0xFFFFFFFFu ? m : (w[i] | m);
    }
}

inline int grid_cap(int64_t n, int64_t cap) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

}  // namespace

// ================================ host side =================================================

void bitmap_add_rows(capsmi_bitmap* b, const int64_t* ids, const uint8_t* ids_valid, const uint8_t* flags, int64_t n,
                     int64_t* dev_counters, const RangePred* rp) {
    if (n <= 0) return;
    KernelTimer kt(b->sess, "bitmap_add");
    const int aligned = (((uintptr_t)ids) & 15) == 0;
    const int64_t g = std::min<int64_t>((n + 1023) / 1024, (int64_t)b->sess->num_cus * 8);
    hipLaunchKernelGGL(k_bitmap_add, dim3((unsigned)std::max<int64_t>(g, 1)), dim3(256), 0, b->sess->stream,
                       P<uint32_t>(b->words), b->lo, b->hi, ids, ids_valid, flags, n, aligned,
                       (unsigned long long*)dev_counters, rp ? *rp : RangePred());
    HIP_CHECK(hipGetLastError());
}

void bitmap_set_range(capsmi_bitmap* b, int64_t b0, int64_t b1) {
    if (b1 <= b0) return;
    KernelTimer kt(b->sess, "bitmap_range");
    const int64_t words = ((b1 + 31) >> 5) - (b0 >> 5);
    hipLaunchKernelGGL(k_bits_range, dim3((unsigned)grid_cap(words, (int64_t)b->sess->num_cus * 4)), dim3(256), 0,
                       b->sess->stream, P<uint32_t>(b->words), b0, b1);
    HIP_CHECK(hipGetLastError());
}

// Node predicates of the form the bitmap scan evaluates inline: a conjunction of comparisons between
// a Long column and a Long literal (C2's `a.age >= 18 AND a.age < 65`).  3VL: a null column value
// makes its comparison NULL, so the row is not kept (Filter keeps TRUE rows only).
bool compile_range_pred(const capsmi_table* t, int32_t nn, const capsmi_expr* prog, RangePred& rp) {
    rp = RangePred();
    if (nn <= 0) return false;
    auto arity = [](const capsmi_expr& x) {
        switch (x.op) {
            case CAPSMI_X_COL: case CAPSMI_X_LIT: case CAPSMI_X_NULL: return 0;
            case CAPSMI_X_NOT: case CAPSMI_X_ISNULL: case CAPSMI_X_ISNOTNULL: case CAPSMI_X_NEG: return 1;
            case CAPSMI_X_AND: case CAPSMI_X_OR: case CAPSMI_X_COALESCE: return (int)x.arg;
            case CAPSMI_X_IN: return (int)x.arg + 1;
            case CAPSMI_X_CASE: return 2 * (int)x.arg + 1;
            default: return 2;
        }
    };
    // conjunct spans [lo, hi] of the root AND (or the root itself)
    std::vector<std::pair<int, int>> spans;
    const capsmi_expr& root = prog[nn - 1];
    if (root.op == CAPSMI_X_AND) {
        int end = nn - 2;
        for (int k = 0; k < root.arg; ++k) {
            int want = 1, i = end;
            for (; i >= 0; --i) {
                want += arity(prog[i]) - 1;
                if (want == 0) break;
            }
            if (i < 0) return false;
            spans.push_back({i, end});
            end = i - 1;
        }
        if (end != -1) return false;
    } else {
        spans.push_back({0, nn - 1});
    }
    for (const auto& sp : spans) {
        if (sp.second - sp.first != 2) return false;
        const capsmi_expr &a = prog[sp.first], &b = prog[sp.first + 1], &op = prog[sp.second];
        const bool col_first = a.op == CAPSMI_X_COL && b.op == CAPSMI_X_LIT;
        const bool lit_first = a.op == CAPSMI_X_LIT && b.op == CAPSMI_X_COL;
        if (!col_first && !lit_first) return false;
        const capsmi_expr& c = col_first ? a : b;
        const capsmi_expr& l = col_first ? b : a;
        if (c.arg < 0 || c.arg >= (int)t->cols.size() || t->cols[c.arg].type != CAPSMI_I64 || l.type != CAPSMI_I64)
            return false;
        int o = op.op;
        if (lit_first) {  // v op col  ==  col op' v
            if (o == CAPSMI_X_LT) o = CAPSMI_X_GT;
            else if (o == CAPSMI_X_LE) o = CAPSMI_X_GE;
            else if (o == CAPSMI_X_GT) o = CAPSMI_X_LT;
            else if (o == CAPSMI_X_GE) o = CAPSMI_X_LE;
        }
        const int64_t v = l.ival;
        int64_t lo = INT64_MIN, hi = INT64_MAX;
        switch (o) {
            case CAPSMI_X_EQ: lo = hi = v; break;
            case CAPSMI_X_LT: if (v == INT64_MIN) { lo = 1; hi = 0; } else hi = v - 1; break;
            case CAPSMI_X_LE: hi = v; break;
            case CAPSMI_X_GT: if (v == INT64_MAX) { lo = 1; hi = 0; } else lo = v + 1; break;
            case CAPSMI_X_GE: lo = v; break;
            default: return false;
        }
        const Column& col = t->cols[c.arg];
        int k = 0;
        while (k < rp.n && rp.col[k] != col.d()) ++k;
        if (k == rp.n) {
            if (rp.n == kMaxRangeTerms) return false;
            rp.col[k] = col.d();
            rp.valid[k] = col.v();
            rp.lo[k] = INT64_MIN;
            rp.hi[k] = INT64_MAX;
            ++rp.n;
        }
        rp.lo[k] = std::max(rp.lo[k], lo);
        rp.hi[k] = std::min(rp.hi[k], hi);
    }
    return true;
}

void words_popcount_async(capsmi_session* s, const uint32_t* w, int64_t w_begin, int64_t w_end, int64_t* dev_out) {
    HIP_CHECK(hipMemsetAsync(dev_out, 0, 8, s->stream));
    if (w_end > w_begin)
        hipLaunchKernelGGL(k_popcount, dim3(grid_cap((w_end - w_begin + 3) / 4, (int64_t)s->num_cus * 4)), dim3(256), 0,
                           s->stream, w, w_begin, w_end, reinterpret_cast<unsigned long long*>(dev_out));
    HIP_CHECK(hipGetLastError());
}

int64_t words_popcount(capsmi_session* s, const uint32_t* w, int64_t w_begin, int64_t w_end) {
    Buf out = dev_alloc(8, s);
    words_popcount_async(s, w, w_begin, w_end, P<int64_t>(out));
    return read_scalar(s, P<int64_t>(out));
}

namespace graph {

static BitView view(const capsmi_bitmap* b) {
    BitView v;
    v.w = P<uint32_t>(b->words);
    v.lo = b->lo;
    v.hi = b->hi;
    v.full = b->full ? 1 : 0;
    return v;
}

int hop_grid(capsmi_session* s, int64_t m) {
    // 2 rels per thread per iteration; enough waves to keep ~16 KB in flight per CU
    int64_t g = (m / 2 + 255) / 256;
    const int64_t cap = (int64_t)s->num_cus * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

void expand_filter(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
                   const capsmi_bitmap* b, int nout, const int64_t* const* in_d, const uint8_t* const* in_v,
                   int64_t* const* out_d, uint8_t* const* out_v, int64_t* dev_count) {
    OutCols oc;
    oc.n = nout;
    for (int c = 0; c < kMaxOut; ++c) {
        oc.src[c] = c < nout ? in_d[c] : nullptr;
        oc.srcv[c] = c < nout ? in_v[c] : nullptr;
        oc.dst[c] = c < nout ? out_d[c] : nullptr;
        oc.dstv[c] = c < nout ? out_v[c] : nullptr;
    }
    if (m <= 0) return;
    int64_t g = (m + kEfTile - 1) / kEfTile;
    const int64_t cap = (int64_t)s->num_cus * 2;
    if (g > cap) g = cap;
    const int al = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
    // fast path: every projected column is the source or target column, no nulls involved
    bool pairs = true;
    uint32_t from_dst = 0;
    for (int c = 0; c < nout; ++c) {
        pairs = pairs && (in_d[c] == src || in_d[c] == dst) && !in_v[c] && !out_v[c];
        if (in_d[c] == dst) from_dst |= 1u << c;
    }
    KernelTimer kt(s, "expand_filter");
    if (pairs) {
        auto k = nout == 1 ? k_expand_pairs<1> : nout == 2 ? k_expand_pairs<2> : nout == 3 ? k_expand_pairs<3>
                                                                                     : k_expand_pairs<4>;
        // 16 workgroups per CU: C2 s = 24 expand 2.27 / 2.25 / 2.23 ms at 4 / 8 / 16 -- more workgroups than
        // resident ones balance the tail of the tile loop
        const int64_t gp = std::min<int64_t>((m + kEpTile - 1) / kEpTile, (int64_t)s->num_cus * 16);
        hipLaunchKernelGGL(k, dim3((unsigned)gp), dim3(kEpBlock), 0, s->stream, src, dst, m, al, view(a), view(b),
                           from_dst, out_d[0], nout > 1 ? out_d[1] : nullptr, nout > 2 ? out_d[2] : nullptr,
                           nout > 3 ? out_d[3] : nullptr, (unsigned long long*)dev_count);
    } else {
        hipLaunchKernelGGL(k_expand_filter, dim3((unsigned)g), dim3(kEfBlock), 0, s->stream, src, dst, m, al, view(a),
                           view(b), oc, (unsigned long long*)dev_count);
    }
    HIP_CHECK(hipGetLastError());
}

void hop1(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
          const capsmi_bitmap* b, uint32_t* M, uint32_t* S1, uint32_t* S2) {
    if (m <= 0) return;
    const BitView av = view(a), bv = view(b);
    const int al = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
    const dim3 g(hop_grid(s, m)), blk(256);
    KernelTimer kt(s, "hop1");
    if (a->full && b->full) hipLaunchKernelGGL((k_hop1<true, true>), g, blk, 0, s->stream, src, dst, m, al, av, bv, M, S1, S2);
    else if (a->full) hipLaunchKernelGGL((k_hop1<true, false>), g, blk, 0, s->stream, src, dst, m, al, av, bv, M, S1, S2);
    else if (b->full) hipLaunchKernelGGL((k_hop1<false, true>), g, blk, 0, s->stream, src, dst, m, al, av, bv, M, S1, S2);
    else hipLaunchKernelGGL((k_hop1<false, false>), g, blk, 0, s->stream, src, dst, m, al, av, bv, M, S1, S2);
    HIP_CHECK(hipGetLastError());
}

void mid_combine(capsmi_session* s, uint32_t* X1, uint32_t* X2, const uint32_t* S1, int64_t nw) {
    KernelTimer kt(s, "mid_combine");
    hipLaunchKernelGGL(k_mid_combine, dim3(grid_cap(nw, 4096)), dim3(256), 0, s->stream, X1, X2, S1, nw);
    HIP_CHECK(hipGetLastError());
}

void hop2(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* c,
          const uint32_t* X1, const uint32_t* X2, int64_t mid_lo, int64_t mid_hi, uint32_t* C) {
    if (m <= 0) return;
    const BitView cv = view(c);
    const int al = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
    const dim3 g(hop_grid(s, m)), blk(256);
    KernelTimer kt(s, "hop2");
    if (c->full) hipLaunchKernelGGL((k_hop2<true>), g, blk, 0, s->stream, src, dst, m, al, cv, X1, X2, mid_lo, mid_hi, C);
    else hipLaunchKernelGGL((k_hop2<false>), g, blk, 0, s->stream, src, dst, m, al, cv, X1, X2, mid_lo, mid_hi, C);
    HIP_CHECK(hipGetLastError());
}

void degrees(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
             const capsmi_bitmap* b, const capsmi_bitmap* c, uint32_t* inA, uint32_t* outC, int64_t* loops) {
    if (m <= 0) return;
    KernelTimer kt(s, "degrees");
    hipLaunchKernelGGL(k_degrees, dim3(grid_cap(m, (int64_t)s->num_cus * 16)), dim3(256), 0, s->stream, src, dst, m,
                       view(a), view(b), view(c), inA, outC, (unsigned long long*)loops);
    HIP_CHECK(hipGetLastError());
}

void deg_product(capsmi_session* s, const uint32_t* inA, const uint32_t* outC, int64_t n, const capsmi_bitmap* b,
                 int64_t* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_deg_product, dim3(grid_cap(n, 4096)), dim3(256), 0, s->stream, inA, outC, n, view(b),
                       (unsigned long long*)out);
    HIP_CHECK(hipGetLastError());
}

int64_t rmat(capsmi_session* s, int scale, int64_t e_begin, int64_t e_end, int pa, int pb, int pc, uint64_t seed,
             int part_col, int part, int nparts, Buf& id, Buf& so, Buf& dout) {
    RmatArgs g;
    g.scale = scale;
    g.tA = ((uint64_t)pa << 32) / 100;
    g.tAB = ((uint64_t)(pa + pb) << 32) / 100;
    g.tABC = ((uint64_t)(pa + pb + pc) << 32) / 100;
    g.seed = seed;
    g.e_begin = e_begin;
    g.e_end = e_end;
    g.part_col = part_col;
    g.part = part;
    g.nparts = nparts;
    g.nwords = ((int64_t(1) << scale) + 31) / 32;
    const int64_t m = e_end - e_begin;
    const int64_t nb = (m + 255) / 256;
    hipStream_t st = s->stream;
    Buf cnt = dev_alloc(sizeof(int64_t) * (nb > 0 ? nb : 1), s);
    Buf off = dev_alloc(sizeof(int64_t) * (nb + 1), s);
    if (nb > 0) hipLaunchKernelGGL(k_rmat_count, dim3((unsigned)nb), dim3(256), 0, st, g, P<unsigned long long>(cnt));
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(off), nb, s);
    const int64_t total = read_scalar(s, P<int64_t>(off) + nb);
    id = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    so = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    dout = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    if (nb > 0)
        hipLaunchKernelGGL(k_rmat_write, dim3((unsigned)nb), dim3(256), 0, st, g, P<int64_t>(off), P<int64_t>(id),
                           P<int64_t>(so), P<int64_t>(dout));
    HIP_CHECK(hipGetLastError());
    return total;
}

void person_flags(capsmi_session* s, int64_t n, bool want_person, uint8_t* f) {
    hipLaunchKernelGGL(k_person_flags, dim3(grid_cap(n, 8192)), dim3(256), 0, s->stream, n, want_person ? 1 : 0, f);
    HIP_CHECK(hipGetLastError());
}

void ages(capsmi_session* s, const int64_t* ids, int64_t n, uint64_t seed, int64_t* age) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_age, dim3(grid_cap(n, 8192)), dim3(256), 0, s->stream, ids, n, seed, age);
    HIP_CHECK(hipGetLastError());
}

void fingerprint(capsmi_session* s, int ncols, const int64_t* const* d, const uint8_t* const* v, int64_t n,
                 uint64_t* out_sum, uint64_t* out_xor) {
    REQUIRE(ncols <= kMaxFp, CAPSMI_ERR_NOT_IMPLEMENTED, "fingerprint over more than 8 columns");
    FpCols fc;
    fc.n = ncols;
    for (int c = 0; c < kMaxFp; ++c) {
        fc.d[c] = c < ncols ? d[c] : nullptr;
        fc.v[c] = c < ncols ? v[c] : nullptr;
    }
    Buf out = dev_alloc(16, s);
    HIP_CHECK(hipMemsetAsync(P<void>(out), 0, 16, s->stream));
    if (n > 0)
        hipLaunchKernelGGL(k_fingerprint, dim3(grid_cap(n, 4096)), dim3(256), 0, s->stream, fc, n,
                           P<unsigned long long>(out));
    HIP_CHECK(hipGetLastError());
    uint64_t host[2];
    HIP_CHECK(hipMemcpyAsync(host, P<void>(out), 16, hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    *out_sum = host[0];
    *out_xor = host[1];
}

}  // namespace graph
}  // namespace capsmi
