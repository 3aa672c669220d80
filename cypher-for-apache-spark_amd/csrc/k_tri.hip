// k_tri.hip -- fused cyclic triangle count (C4), ExpandInto closing the cycle.
//
//   MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) WHERE n_ok(a), n_ok(b), n_ok(c) RETURN count(*)
//
// CAPS plans two Expands and an ExpandInto on (source, target) = (c, a) (RelationalPlanner.scala:113-154)
// followed by the pairwise uniqueness filter; every binding is a row.  With m(x,y) the multiplicity of
// x->y and s(x) the number of self-loops at x, the rows split by how many of a, b, c coincide
// (derivation in DESIGN.md; checked against enumeration in oracle/rmat.c):
//   count = 3 * sum_{triangles {u,v,w}} [m(u,v)m(v,w)m(w,u) + m(u,w)m(w,v)m(v,u)]
//         + 3 * sum_{u != x} s(u) m(u,x) m(x,u)
//         + sum_u s(u)(s(u)-1)(s(u)-2)
// Triangles of the underlying simple undirected graph are listed once each by orienting every
// undirected edge from the lower (degree, id) end and intersecting sorted out-lists.  The two
// directed multiplicities of each undirected edge ride along with the oriented adjacency, so the
// intersection loop reads no other table.
#include <algorithm>

#include "capsmi_impl.h"

namespace capsmi {
namespace tri {

constexpr uint64_t kNone = ~0ULL;

// Undirected keys of the kept, non-loop relationships: min << 32 | max in the low word with the
// direction bit beside it (bit 31 when the sorted digits of max end below it, else bit 0 with max
// shifted up: `msh` = 0 / 1).  Self-loops are counted directly.  Dropped relationships get kNone,
// which sorts last: a valid key's min is at most n - 2, below the all-ones digits of kNone.
__global__ void k_pack(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                       int64_t hi, const uint32_t* __restrict__ okw, int full, int msh, uint64_t* __restrict__ key,
                       uint32_t* __restrict__ sl) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e], t = dst[e];
        bool ok = s >= lo && s < hi && t >= lo && t < hi;
        if (ok && !full) {
            const uint64_t xs = (uint64_t)(s - lo), xt = (uint64_t)(t - lo);
            ok = ((okw[xs >> 5] >> (xs & 31)) & 1u) && ((okw[xt >> 5] >> (xt & 31)) & 1u);
        }
        uint64_t k = kNone;
        if (ok) {
            const uint64_t xs = (uint64_t)(s - lo), xt = (uint64_t)(t - lo);
            if (xs == xt) {
                atomicAdd(&sl[xs], 1u);
            } else {
                const uint64_t mn = xs < xt ? xs : xt, mx = xs < xt ? xt : xs, dir = xs > xt;
                k = (mn << 32) | (msh ? (mx << 1) | dir : (dir << 31) | mx);
            }
        }
        key[e] = k;
    }
}

// run heads of the sorted undirected keys (direction bit masked off; valid keys only)
__global__ void k_heads(const uint64_t* __restrict__ k, int64_t n, uint64_t mask, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = (k[i] != kNone && (i == 0 || (k[i] & mask) != (k[i - 1] & mask))) ? 1 : 0;
}

// end of the valid keys: the first kNone of the sorted keys (one lane, O(log m) reads on the device)
__global__ void k_first_none(const uint64_t* __restrict__ k, int64_t m, int64_t* __restrict__ out) {
    int64_t a = 0, b = m;
    while (a < b) {
        const int64_t mid = (a + b) / 2;
        if (k[mid] == kNone) b = mid; else a = mid + 1;
    }
    *out = a;
}

// undirected runs -> (key min<<32|max, payload m(min,max)<<32 | m(max,min)), and the lower ends'
// degrees.  The degree that orders the vertices is the relationship count (multi-edges counted, loops
// not): any total order gives the same count, and this one is a sum over sorted keys on both sides
// (k_deg_max counts the upper ends over the keys sorted by max), where the simple-graph degree needed
// one random atomic per undirected edge at its upper end (~8 of k_und_runs' 11 ms at C4).  The runs
// are sorted by their lower end, so a wave's lanes with the same lower end are contiguous: one atomic
// per such segment (hubs would otherwise serialise hundreds of thousands of adds on one counter).
// A run longer than kShortRun (multi-edges between two hubs, up to ~10^4 at C4) is not walked by
// its lane, which would hold its wave for the whole walk: it goes to a list that k_und_long counts
// with a whole workgroup per run.
constexpr int64_t kShortRun = 32;

__device__ __forceinline__ uint64_t back_bit(uint64_t key, int msh) { return msh ? (key & 1u) : ((key >> 31) & 1u); }

__global__ void k_und_runs(const uint64_t* __restrict__ k, const int64_t* __restrict__ heads, int64_t nruns,
                           const int64_t* __restrict__ nvalid_p, int msh, uint64_t* __restrict__ ek,
                           int64_t* __restrict__ ev, uint32_t* __restrict__ deg, int64_t* __restrict__ longr,
                           unsigned long long* __restrict__ nlong) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t nvalid = *nvalid_p;
    for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); r0 < nruns; r0 += stride) {  // wave-uniform
        const int64_t r = r0 + lane;
        const bool act = r < nruns;  // the active lanes are a prefix of the wave
        uint32_t mn = 0;
        int64_t h = 0, h2 = 0;
        if (act) {
            h = heads[r];
            h2 = r + 1 < nruns ? heads[r + 1] : nvalid;
            const uint64_t key = k[h];
            mn = (uint32_t)(key >> 32);
            const uint32_t mx = msh ? ((uint32_t)key >> 1) : ((uint32_t)key & 0x7FFFFFFFu);
            ek[r] = ((uint64_t)mn << 32) | mx;
            if (h2 - h <= kShortRun) {
                uint64_t back = 0;  // relationships max -> min
                for (int64_t i = h; i < h2; ++i) back += back_bit(k[i], msh);
                ev[r] = (int64_t)((((uint64_t)(h2 - h) - back) << 32) | back);
            } else {
                longr[atomicAdd(nlong, 1ull)] = r;
            }
        }
        const uint32_t prev = __shfl_up(mn, 1, 64);
        const bool head = act && (lane == 0 || prev != mn);
        const unsigned long long hb = __ballot(head), am = __ballot(act);
        const unsigned long long later = lane == 63 ? 0ULL : hb >> (lane + 1);
        const int next = later ? lane + 1 + __builtin_ctzll(later) : __popcll(am);
        const int64_t seg_end = __shfl(h2, head ? next - 1 : lane, 64);  // end of the segment's last run
        if (head && deg) atomicAdd(&deg[mn], (uint32_t)(seg_end - h));
    }
}

// upper-end degrees over the undirected keys sorted by their upper end (the max digits' passes of
// the key sort): consecutive lanes with the same end add once (dropped keys are segments of their own)
__global__ void k_deg_max(const uint64_t* __restrict__ k, int64_t m, int msh, uint32_t* __restrict__ deg) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); i0 < m; i0 += stride) {  // wave-uniform
        const int64_t i = i0 + lane;
        uint32_t mx = 0xFFFFFFFFu;  // no valid key has it (ids < 2^31)
        if (i < m) {
            const uint64_t key = k[i];
            if (key != kNone) mx = msh ? ((uint32_t)key >> 1) : ((uint32_t)key & 0x7FFFFFFFu);
        }
        const uint32_t prev = __shfl_up(mx, 1, 64);
        const bool head = lane == 0 || prev != mx;
        const unsigned long long hb = __ballot(head);
        const unsigned long long later = lane == 63 ? 0ULL : hb >> (lane + 1);
        const int next = later ? lane + 1 + __builtin_ctzll(later) : 64;
        if (head && mx != 0xFFFFFFFFu) atomicAdd(&deg[mx], (uint32_t)(next - lane));
    }
}

// the long runs' payloads: one workgroup per run, a block reduction of the direction bits
__global__ void __launch_bounds__(256) k_und_long(const uint64_t* __restrict__ k, const int64_t* __restrict__ heads,
                                                  int64_t nruns, const int64_t* __restrict__ nvalid_p, int msh,
                                                  const int64_t* __restrict__ longr,
                                                  const unsigned long long* __restrict__ nlong,
                                                  int64_t* __restrict__ ev) {
    __shared__ unsigned long long part[4];
    const int64_t cnt = (int64_t)*nlong, nvalid = *nvalid_p;
    for (int64_t q = blockIdx.x; q < cnt; q += gridDim.x) {  // block-uniform
        const int64_t r = longr[q], h = heads[r], h2 = r + 1 < nruns ? heads[r + 1] : nvalid;
        unsigned long long back = 0;
        for (int64_t i = h + threadIdx.x; i < h2; i += 256) back += back_bit(k[i], msh);
        for (int o = 32; o > 0; o >>= 1) back += __shfl_down(back, o, 64);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = back;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t b = part[0] + part[1] + part[2] + part[3];
            ev[r] = (int64_t)((((uint64_t)(h2 - h) - b) << 32) | b);
        }
        __syncthreads();
    }
}

// (degree, id) sort keys of the vertices
// (degree, id) keys -- the id rides in the low word, so the sort is key-only -- and the maximum degree
// (one atomic per wave: the sort then takes only the degree digits it has)
__global__ void k_deg_keys(const uint32_t* __restrict__ deg, int64_t n, uint64_t* __restrict__ key,
                           unsigned int* __restrict__ dmax) {
    uint32_t best = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        key[i] = ((uint64_t)deg[i] << 32) | (uint64_t)i;
        best = max(best, deg[i]);
    }
    for (int o = 32; o > 0; o >>= 1) best = max(best, (uint32_t)__shfl_down(best, o, 64));
    if ((threadIdx.x & 63) == 0 && best) atomicMax(dmax, best);
}

// degree-order ids: the vertex at position p of the ascending (degree, id) order gets n - 1 - p
__global__ void k_rank_ids(const uint64_t* __restrict__ by_order, int64_t n, uint32_t* __restrict__ rid,
                           int64_t* __restrict__ orig) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = (int64_t)(uint32_t)by_order[p], r = n - 1 - p;
        rid[v] = (uint32_t)r;
        orig[r] = v;
    }
}

struct TgCode {
    uint32_t ib, cb;  // id bits, code bits per direction (0: every payload is an exception)
    __host__ __device__ uint32_t idmask() const { return ib >= 32 ? ~0u : (1u << ib) - 1u; }
    __host__ __device__ uint32_t cmask() const { return (1u << cb) - 1u; }
};

// orient each undirected edge from the lower (degree, id) end -- towards the smaller degree-order id;
// key = rid(from)<<32 | rid(to), payload = m(from,to)<<32 | m(to,from).
// Coded (tc.cb > 0): the key's low word is the coded target word (multiplicities above the id, outside
// every sorted digit, so a key-only sort carries them), and only the exceptions' exact payloads are
// kept, appended as (key, payload) to exc (one atomic per wave) and placed after the sort (k_exc_place).
// Uncoded: the payload goes to ov[i], sorted along as the value.
__global__ void k_orient(const uint64_t* __restrict__ ek, const int64_t* __restrict__ ev, int64_t ne,
                         const uint32_t* __restrict__ rid, TgCode tc, uint64_t* __restrict__ ok_,
                         int64_t* __restrict__ ov, uint64_t* __restrict__ exc, unsigned long long* __restrict__ nexc) {
    // four edges per lane and pass, their loads (and the random rid gathers) issued together
    constexpr int U = 4;
    const int lane = threadIdx.x & 63;
    const uint32_t cm = tc.cmask();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
    for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)) * U; i0 < ne; i0 += stride) {  // wave-uniform
        uint64_t kk[U], vv[U];
        uint32_t rx[U], ry[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = i0 + j * 64 + lane;
            kk[j] = i < ne ? ek[i] : 0;
            vv[j] = i < ne ? (uint64_t)ev[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {  // (rid null: the keys are degree-order ids already)
            rx[j] = rid ? rid[(uint32_t)(kk[j] >> 32)] : (uint32_t)(kk[j] >> 32);
            ry[j] = rid ? rid[(uint32_t)kk[j]] : (uint32_t)kk[j];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = i0 + j * 64 + lane;
            bool ex = false;
            uint64_t key = 0, pay = 0;
            if (i < ne) {
                const uint32_t mxy = (uint32_t)(vv[j] >> 32), myx = (uint32_t)vv[j];
                const bool xf = rx[j] > ry[j];  // x is lower in (degree, id)
                const uint32_t f = xf ? mxy : myx, b = xf ? myx : mxy;
                key = xf ? ((uint64_t)rx[j] << 32) | ry[j] : ((uint64_t)ry[j] << 32) | rx[j];
                pay = ((uint64_t)f << 32) | b;
                if (tc.cb) {
                    key |= (uint64_t)(min(f, cm) << tc.ib | min(b, cm) << (tc.ib + tc.cb));
                    ex = f >= cm || b >= cm;
                } else {
                    ov[i] = (int64_t)pay;
                }
                ok_[i] = key;
            }
            const unsigned long long eb = __ballot(ex);
            if (eb) {  // wave-uniform
                unsigned long long base = 0;
                if (lane == __builtin_ctzll(eb)) base = atomicAdd(nexc, (unsigned long long)__popcll(eb));
                base = __shfl(base, __builtin_ctzll(eb), 64);
                if (ex) {
                    const unsigned long long at = base + __popcll(eb & ((1ULL << lane) - 1));
                    exc[2 * at] = key;
                    exc[2 * at + 1] = pay;
                }
            }
        }
    }
}

// ---- the direct oriented build (ids <= 2^24) --------------------------------------------------------------
// The orientation needs only SOME total order in which hubs come first (any order gives the same count;
// the degree order bounds the out-lists).  So the degrees are estimated from a sample of the relationships
// (one at a hashed offset in every block of `rate`; every one below 2^22), the vertices ranked, and every
// relationship packed
// straight into its oriented key: one sort of the raw oriented keys then groups each pair's relationships
// (multiplicities per direction from the direction bit) in the order the lists need -- instead of a sort
// of undirected keys, the orientation, and a second sort of the oriented ones.
constexpr int kSplitTile = 2048;  // tiled passes: 256 lanes x 8 consecutive keys / edges
constexpr int kDegLds = 1 << 14;  // per-block LDS counters for the lowest ids (R-MAT's hubs: few hot counters)

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    return (uint32_t)x;
}

__global__ void __launch_bounds__(256) k_deg_sample(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                    int64_t m, int64_t e0, int64_t lo, int64_t hi,
                                                    const uint32_t* __restrict__ okw, int full, uint32_t rate,
                                                    uint32_t* __restrict__ deg) {
    // one relationship per block of `rate`, at a hashed offset inside it: only the sampled ones are read
    __shared__ uint32_t h[kDegLds];
    for (int i = threadIdx.x; i < kDegLds; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const int64_t ns = (m + rate - 1) / rate;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ns; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = j * rate + (int64_t)(mix32((uint64_t)(e0 / rate + j)) & (rate - 1));
        if (e >= m) continue;
        const int64_t sv = src[e], tv = dst[e];
        bool ok = sv >= lo && sv < hi && tv >= lo && tv < hi && sv != tv;
        if (!ok) continue;
        const uint64_t xs = (uint64_t)(sv - lo), xt = (uint64_t)(tv - lo);
        if (!full && !(((okw[xs >> 5] >> (xs & 31)) & 1u) && ((okw[xt >> 5] >> (xt & 31)) & 1u))) continue;
        if (xs < kDegLds) atomicAdd(&h[xs], 1u); else atomicAdd(&deg[xs], 1u);
        if (xt < kDegLds) atomicAdd(&h[xt], 1u); else atomicAdd(&deg[xt], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kDegLds; i += blockDim.x)
        if (h[i]) atomicAdd(&deg[i], h[i]);
}

// raw oriented keys: from << 32 | dir << 31 | to in degree-order ids (from = the lower (degree, id) end,
// the larger rid; dir = 1 for a relationship to -> from), kNone for dropped ones; self-loops counted in sl.
// HIST: the block writes whole 4096-key sort tiles and counts their first sort digit (bits hshift..+7) into
// hist[d * ntiles + tile], so the sort's first pass skips its histogram read (radix_sort_keys' hist0)
template <bool HIST>
__global__ void __launch_bounds__(256) k_pack_or(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 int64_t m, int64_t lo, int64_t hi, const uint32_t* __restrict__ okw,
                                                 int full, const uint32_t* __restrict__ rid, uint64_t* __restrict__ key,
                                                 uint32_t* __restrict__ sl, int64_t* __restrict__ hist, int hshift) {
    constexpr int U = 4;  // relationships per lane and round: the random rid gathers of four in flight together
    __shared__ unsigned int h[256];
    auto round = [&](int64_t e0) {  // relationships e0 + j * 256
        uint64_t xs[U], xt[U];
        bool ok[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t e = e0 + (int64_t)j * 256;
            const int64_t sv = e < m ? src[e] : lo - 1, tv = e < m ? dst[e] : lo - 1;
            ok[j] = sv >= lo && sv < hi && tv >= lo && tv < hi;
            xs[j] = ok[j] ? (uint64_t)(sv - lo) : 0;
            xt[j] = ok[j] ? (uint64_t)(tv - lo) : 0;
        }
        if (!full) {
#pragma unroll
            for (int j = 0; j < U; ++j)
                ok[j] = ok[j] && ((okw[xs[j] >> 5] >> (xs[j] & 31)) & 1u) && ((okw[xt[j] >> 5] >> (xt[j] & 31)) & 1u);
        }
        uint32_t rs[U], rt[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            rs[j] = rid[xs[j]];
            rt[j] = rid[xt[j]];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t e = e0 + (int64_t)j * 256;
            if (e >= m) break;
            uint64_t k = kNone;
            if (ok[j]) {
                if (xs[j] == xt[j]) atomicAdd(&sl[xs[j]], 1u);
                else k = rs[j] > rt[j] ? ((uint64_t)rs[j] << 32) | rt[j] : ((uint64_t)rt[j] << 32) | (1u << 31) | rs[j];
            }
            key[e] = k;
            if (HIST) atomicAdd(&h[(uint32_t)(k >> hshift) & 255u], 1u);
        }
    };
    if (!HIST) {
        const int64_t stride = (int64_t)gridDim.x * 256 * U;
        for (int64_t e0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x; e0 < m; e0 += stride) round(e0);
        return;
    }
    const int64_t ntiles = (m + kSortTile - 1) / kSortTile;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // block-uniform
        h[threadIdx.x] = 0;
        __syncthreads();
        for (int r = 0; r < kSortTile / (256 * U); ++r) round(t * kSortTile + (int64_t)r * 256 * U + threadIdx.x);
        __syncthreads();
        hist[(int64_t)threadIdx.x * ntiles + t] = h[threadIdx.x];
        __syncthreads();  // h is cleared for the next tile
    }
}

// ---- the runs of the sorted raw oriented keys (the direct build) ----
// One pass counts the run heads of every 4096-key tile, a scan places the tiles, one pass writes: the head
// lane of a run (one pair's relationships; the direction bit at 31 is not sorted) counts the run's keys and
// direction bits -- inside the tile from LDS, past its end from memory -- and writes the pair's coded
// oriented key and target word, its exception when a multiplicity reaches the code's all-ones, and its pair
// term when both directions occur.  Runs longer than kShortRun go to k_or_long (a workgroup per run).  This
// replaces the head flags and their compaction, k_und_runs, k_orient with the identity order, k_targets and
// k_pair_terms of the direct build.
constexpr int kOrB = 256, kOrIt = 16, kOrTile = kOrB * kOrIt;
constexpr uint64_t kOrMask = ~(1ULL << 31);

struct OrOut {
    uint64_t* ok;               // coded oriented keys
    uint32_t* tg;               // their low words (null: written later, after a distributed build's gather)
    int64_t* ov;                // exact payloads: every one uncoded, the exceptions' when exc is null
    uint64_t* exc;              // (key, payload) of the exceptions (coded; a distributed build, whose keys move)
    unsigned long long* nexc;
    int64_t* longr;             // (run, head index) of the long runs
    unsigned long long* nlong;
    const uint32_t* sl;         // self-loop counts in degree-order ids
    int64_t* pair;              // the pair terms: one partial sum per tile, the long runs' at index ntiles
    int64_t* off;               // CSR offsets: off[from] = the from's first run (null: searched for later)
};

// the pair (from, to) = km's ids with f relationships from -> to and b to -> from: run r's outputs; returns
// whether it is an exception (coded) and its key / payload, adds its pair term to acc
__device__ __forceinline__ bool or_emit(int64_t r, uint64_t km, uint32_t f, uint32_t b, TgCode tc, const OrOut& o,
                                        unsigned long long& acc, uint64_t& key, uint64_t& pay) {
    const uint32_t from = (uint32_t)(km >> 32), to = (uint32_t)km;
    key = ((uint64_t)from << 32) | to;
    pay = ((uint64_t)f << 32) | b;
    bool ex = false;
    if (tc.cb) {
        const uint32_t cm = tc.cmask();
        key |= (uint64_t)(min(f, cm) << tc.ib | min(b, cm) << (tc.ib + tc.cb));
        ex = f >= cm || b >= cm;
    }
    if (!tc.cb || (ex && !o.exc)) o.ov[r] = (int64_t)pay;
    o.ok[r] = key;
    if (o.tg) o.tg[r] = (uint32_t)key;
    if (f && b) acc += 3ULL * ((uint64_t)o.sl[from] + o.sl[to]) * f * b;
    return ex;
}

__global__ void __launch_bounds__(kOrB) k_or_count(const uint64_t* __restrict__ key, int64_t m, int64_t* __restrict__ cnt) {
    __shared__ int ws[kOrB / 64];
    const int64_t base = (int64_t)blockIdx.x * kOrTile;
    uint64_t k[kOrIt], p[kOrIt];
#pragma unroll
    for (int j = 0; j < kOrIt; ++j) {
        const int64_t i = base + j * kOrB + threadIdx.x;
        k[j] = i < m ? key[i] : kNone;
        p[j] = i > 0 && i < m ? key[i - 1] : kNone;
    }
    int c = 0;
#pragma unroll
    for (int j = 0; j < kOrIt; ++j) c += k[j] != kNone && (k[j] & kOrMask) != (p[j] & kOrMask);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void __launch_bounds__(kOrB) k_or_write(const uint64_t* __restrict__ key, int64_t m,
                                                   const int64_t* __restrict__ pre, TgCode tc, OrOut o) {
    __shared__ uint64_t tk[kOrTile];
    __shared__ int wc[kOrIt * (kOrB / 64)];  // heads per (item, wave), then their exclusive prefix in key order
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const unsigned long long lt = lane == 0 ? 0ULL : (~0ULL >> (64 - lane));
    const int64_t base = (int64_t)blockIdx.x * kOrTile;
    const int nt = (int)min((int64_t)kOrTile, m - base);
    uint64_t k[kOrIt];
#pragma unroll
    for (int j = 0; j < kOrIt; ++j) {
        const int i = j * kOrB + (int)threadIdx.x;
        k[j] = i < nt ? key[base + i] : kNone;
        if (i < nt) tk[i] = k[j];
    }
    const uint64_t before = base > 0 ? key[base - 1] : kNone;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kOrIt; ++j) {
        const int i = j * kOrB + (int)threadIdx.x;
        const uint64_t p = i > 0 ? tk[i - 1] : before;
        const unsigned long long hb = __ballot(i < nt && k[j] != kNone && (k[j] & kOrMask) != (p & kOrMask));
        if (lane == 0) wc[j * (kOrB / 64) + wid] = __popcll(hb);
    }
    __syncthreads();
    if (wid == 0) {  // 64 (item, wave) counts in key order: one wave's scan
        const int v = wc[lane];
        int incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        wc[lane] = incl - v;
    }
    __syncthreads();
    const int64_t r0 = pre[blockIdx.x];
    unsigned long long acc = 0;
    // per item: the key and its head bit again from LDS (no register arrays indexed in a rolled loop); the
    // head lane counts its run from the next key on (most runs are one relationship: one LDS read)
#pragma unroll 1
    for (int j = 0; j < kOrIt; ++j) {
        const int i = j * kOrB + (int)threadIdx.x;
        const uint64_t kj = i < nt ? tk[i] : kNone;
        const uint64_t p = i > 0 ? tk[i - 1] : before;
        const bool head = i < nt && kj != kNone && (kj & kOrMask) != (p & kOrMask);
        const unsigned long long hb = __ballot(head);
        bool ex = false;
        uint64_t okey = 0, pay = 0;
        if (head) {
            const int64_t r = r0 + wc[j * (kOrB / 64) + wid] + __popcll(hb & lt);
            const uint64_t km = kj & kOrMask;
            if (o.off && (kj >> 32) != (p >> 32)) o.off[kj >> 32] = r;  // the first run of this from
            uint32_t len = 1, bk = (uint32_t)(kj >> 31) & 1u;
            int q = i + 1;
            bool ended = false;
            for (; q < nt && len < (uint32_t)kShortRun; ++q) {  // inside the tile
                const uint64_t x = tk[q];
                if ((x & kOrMask) != km) {
                    ended = true;
                    break;
                }
                bk += (uint32_t)(x >> 31) & 1u;
                ++len;
            }
            if (!ended && len < (uint32_t)kShortRun) {  // past the tile end (rare)
                for (int64_t gi = base + q;; ++gi) {
                    if (gi >= m) {
                        ended = true;
                        break;
                    }
                    const uint64_t x = key[gi];
                    if ((x & kOrMask) != km) {
                        ended = true;
                        break;
                    }
                    bk += (uint32_t)(x >> 31) & 1u;
                    if (++len >= (uint32_t)kShortRun) break;
                }
            }
            if (ended) {
                ex = or_emit(r, km, len - bk, bk, tc, o, acc, okey, pay);
            } else {
                const unsigned long long at = atomicAdd(o.nlong, 1ull);
                o.longr[2 * at] = r;
                o.longr[2 * at + 1] = base + i;
            }
        }
        if (o.exc) {
            const unsigned long long eb = __ballot(ex);
            if (eb) {  // wave-uniform
                unsigned long long at0 = 0;
                if (lane == __builtin_ctzll(eb)) at0 = atomicAdd(o.nexc, (unsigned long long)__popcll(eb));
                at0 = __shfl(at0, __builtin_ctzll(eb), 64);
                if (ex) {
                    const unsigned long long at = at0 + __popcll(eb & lt);
                    o.exc[2 * at] = okey;
                    o.exc[2 * at + 1] = pay;
                }
            }
        }
    }
    // the tile's pair terms: one partial (no same-address atomics; summed by a scan)
    __shared__ unsigned long long pw[kOrB / 64];
    for (int s = 32; s > 0; s >>= 1) acc += __shfl_down(acc, s, 64);
    if (lane == 0) pw[wid] = acc;
    __syncthreads();
    if (threadIdx.x == 0) o.pair[blockIdx.x] = (int64_t)(pw[0] + pw[1] + pw[2] + pw[3]);
}

// the long runs (multi-edges between hubs): a workgroup walks each run 256 keys at a time
__global__ void __launch_bounds__(256) k_or_long(const uint64_t* __restrict__ key, int64_t m, int64_t ntiles, TgCode tc,
                                                 OrOut o) {
    __shared__ int stop;
    __shared__ unsigned int part[4];
    const int64_t cnt = (int64_t)*o.nlong;
    for (int64_t q = blockIdx.x; q < cnt; q += gridDim.x) {  // block-uniform
        const int64_t r = o.longr[2 * q], h = o.longr[2 * q + 1];
        const uint64_t km = key[h] & kOrMask;
        uint32_t bk = 0;
        int64_t len = 0;
        for (int64_t c0 = h;; c0 += 256) {
            if (threadIdx.x == 0) stop = 256;
            __syncthreads();
            const int64_t i = c0 + threadIdx.x;
            const uint64_t x = i < m ? key[i] : kNone;
            if ((x & kOrMask) != km) atomicMin(&stop, (int)threadIdx.x);
            __syncthreads();
            const int st = stop;
            if ((int)threadIdx.x < st) bk += (uint32_t)(x >> 31) & 1u;
            len += st;
            __syncthreads();  // stop is reset by the next chunk
            if (st < 256) break;
        }
        for (int s = 32; s > 0; s >>= 1) bk += __shfl_down(bk, s, 64);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = bk;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t b = part[0] + part[1] + part[2] + part[3];
            unsigned long long acc = 0;
            uint64_t okey, pay;
            if (or_emit(r, km, (uint32_t)len - b, b, tc, o, acc, okey, pay) && o.exc) {
                const unsigned long long at = atomicAdd(o.nexc, 1ull);
                o.exc[2 * at] = okey;
                o.exc[2 * at + 1] = pay;
            }
            if (acc) atomicAdd(reinterpret_cast<unsigned long long*>(o.pair + ntiles), acc);
        }
        __syncthreads();
    }
}

// The CSR offsets without a search: k_or_write stored off[v] at each from change and the rest hold
// INT64_MAX; a vertex without out-edges starts where the next one does, so off becomes its suffix minimum
// over the n + 1 entries (off[n] = ne), the largest out-degree found on the way (k_sufmin_apply).
constexpr int kSmB = 256, kSmIt = 16, kSmTile = kSmB * kSmIt;

__global__ void __launch_bounds__(kSmB) k_sufmin_tiles(const int64_t* __restrict__ off, int64_t n1,
                                                       int64_t* __restrict__ tmin) {
    __shared__ int64_t ws[kSmB / 64];
    const int64_t base = (int64_t)blockIdx.x * kSmTile + threadIdx.x;
    int64_t v = INT64_MAX;
#pragma unroll
    for (int k = 0; k < kSmIt; ++k)  // coalesced: a plain minimum needs no order
        if (base + k * kSmB < n1) v = min(v, off[base + k * kSmB]);
    for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_down(v, o, 64));
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) tmin[blockIdx.x] = min(min(ws[0], ws[1]), min(ws[2], ws[3]));
}

// one workgroup: tmin[t] becomes the minimum over the tiles after t (INT64_MAX for the last)
__global__ void __launch_bounds__(1024) k_sufmin_carry(int64_t* __restrict__ tmin, int64_t nt) {
    __shared__ int64_t cm[1024];
    const int64_t per = (nt + 1023) / 1024, b = (int64_t)threadIdx.x * per;
    int64_t v = INT64_MAX;
    for (int64_t k = 0; k < per; ++k)
        if (b + k < nt) v = min(v, tmin[b + k]);
    cm[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive suffix minimum over the chunk minima
        const int64_t y = threadIdx.x + o < 1024 ? cm[threadIdx.x + o] : INT64_MAX;
        __syncthreads();
        cm[threadIdx.x] = min(cm[threadIdx.x], y);
        __syncthreads();
    }
    int64_t run = threadIdx.x + 1 < 1024 ? cm[threadIdx.x + 1] : INT64_MAX;  // the chunks after this one
    for (int64_t k = per - 1; k >= 0; --k)
        if (b + k < nt) {
            const int64_t x = tmin[b + k];
            tmin[b + k] = run;
            run = min(run, x);
        }
}

// the tile is staged through LDS (coalesced loads and stores; a lane's 16 consecutive entries at a padded
// stride of 17, so the lanes' reads fall in different banks)
__global__ void __launch_bounds__(kSmB) k_sufmin_apply(int64_t* __restrict__ off, int64_t n1,
                                                       const int64_t* __restrict__ carry,
                                                       unsigned long long* __restrict__ maxod) {
    __shared__ int64_t st[kSmB * (kSmIt + 1)];
    __shared__ int64_t cm[kSmB];
    const int64_t tb = (int64_t)blockIdx.x * kSmTile;
    auto pad = [](int i) { return i + i / kSmIt; };
#pragma unroll
    for (int k = 0; k < kSmIt; ++k) {
        const int i = k * kSmB + (int)threadIdx.x;
        st[pad(i)] = tb + i < n1 ? off[tb + i] : INT64_MAX;
    }
    __syncthreads();
    int64_t x[kSmIt];
    int64_t v = INT64_MAX;
#pragma unroll
    for (int k = 0; k < kSmIt; ++k) {
        x[k] = st[threadIdx.x * (kSmIt + 1) + k];
        v = min(v, x[k]);
    }
    cm[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kSmB; o <<= 1) {  // inclusive suffix minimum over the lanes
        const int64_t y = threadIdx.x + o < kSmB ? cm[threadIdx.x + o] : INT64_MAX;
        __syncthreads();
        cm[threadIdx.x] = min(cm[threadIdx.x], y);
        __syncthreads();
    }
    // the final value right after this lane's entries: the next lanes', then the next tile's (carry)
    const int64_t next_first = min(threadIdx.x + 1 < kSmB ? cm[threadIdx.x + 1] : INT64_MAX, carry[blockIdx.x]);
    int64_t run = next_first;
#pragma unroll
    for (int k = kSmIt - 1; k >= 0; --k) {
        run = min(run, x[k]);
        x[k] = run;
    }
    const int64_t base = tb + (int64_t)threadIdx.x * kSmIt;
    unsigned long long best = 0;
#pragma unroll
    for (int k = 0; k < kSmIt; ++k) {
        st[threadIdx.x * (kSmIt + 1) + k] = x[k];
        const int64_t nx = k + 1 < kSmIt ? x[k + 1] : next_first;
        if (base + k + 1 < n1) best = max(best, (unsigned long long)(nx - x[k]));
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmIt; ++k) {
        const int i = k * kSmB + (int)threadIdx.x;
        if (tb + i < n1) off[tb + i] = st[pad(i)];
    }
    for (int o = 32; o > 0; o >>= 1) best = max(best, (unsigned long long)__shfl_down(best, o, 64));
    if ((threadIdx.x & 63) == 0 && best) atomicMax(maxod, best);
}

// sl in degree-order ids
__global__ void k_perm_u32(const uint32_t* __restrict__ a, const int64_t* __restrict__ orig, int64_t n,
                           uint32_t* __restrict__ b) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        b[r] = a[orig[r]];
}

// the largest out-degree (packed in-keys need positions below 2^16)
__global__ void k_max_od(const int64_t* __restrict__ off, int64_t n, unsigned long long* __restrict__ mx) {
    unsigned long long best = 0;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        best = max(best, (unsigned long long)(off[v + 1] - off[v]));
    for (int o = 32; o > 0; o >>= 1) best = max(best, (unsigned long long)__shfl_down(best, o, 64));
    if ((threadIdx.x & 63) == 0 && best) atomicMax(mx, best);
}

// exceptions' exact payloads into ov at their keys' positions in the sorted oriented keys: (from, to)
// is unique and the keys are in (from, to) order -- not in 64-bit order, the unsorted multiplicity bits
// lying above `to`, so they are masked off for the search
__global__ void k_exc_place(const uint64_t* __restrict__ exc, const unsigned long long* __restrict__ nexc,
                            const uint64_t* __restrict__ ok_, int64_t ne, TgCode tc, int64_t* __restrict__ ov) {
    const int64_t cnt = (int64_t)*nexc;
    const uint64_t km = ~((((uint64_t)1 << (2 * tc.cb)) - 1) << tc.ib);
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = exc[2 * j] & km;
        int64_t lo = 0, hi = ne;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((ok_[mid] & km) < key) lo = mid + 1; else hi = mid;
        }
        ov[lo] = (int64_t)exc[2 * j + 1];
    }
}

// in-lists: the oriented edge's position in out(from) bounds the v-mode walk (and locates its payload).
// Packed (iv == nullptr; ids of <= 24 bits, positions < 2^16): key = to << (ib + 16) | from << 16 | pos,
// sorted on the digits of `to` alone.  Otherwise key = to << 32 | from with the edge index as the value.
__global__ void k_swap_keys(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ off, int64_t ne, TgCode tc,
                            uint64_t* __restrict__ ik, int64_t* __restrict__ iv) {
    const uint32_t idm = tc.idmask();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = ok_[i];
        const uint64_t from = k >> 32, to = (uint32_t)k & idm;
        if (iv) {
            ik[i] = (to << 32) | from;
            iv[i] = i;
        } else {
            ik[i] = (to << (tc.ib + 16)) | (from << 16) | (uint64_t)(i - off[from]);
        }
    }
}

// in-list sources and positions from the sorted in-keys (packed: both from the key; else pos = e - off[from])
__global__ void k_in_split(const uint64_t* __restrict__ ik, const int64_t* __restrict__ iv, const int64_t* __restrict__ off,
                           int64_t ne, TgCode tc, uint32_t* __restrict__ itg, uint32_t* __restrict__ ipos) {
    const uint32_t idm = tc.idmask();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = ik[i];
        if (iv) {
            const uint32_t from = (uint32_t)k;
            itg[i] = from;
            ipos[i] = (uint32_t)(iv[i] - off[from]);
        } else {
            itg[i] = (uint32_t)(k >> 16) & idm;
            ipos[i] = (uint32_t)(k & 0xFFFFu);
        }
    }
}

// ---- direction-split lists ------------------------------------------------------------------------
// A wedge closes a cycle in one direction only: u -> v -> w -> u needs m(v,w) >= 1 and u -> w -> v -> u
// needs m(w,v) >= 1 (the two terms of tri_weight).  Each out-list is therefore also kept as two lists:
// out_f(x) = {w : m(x,w) >= 1} and out_b(x) = {w : m(w,x) >= 1}, both sorted, in one array `tgs` (all
// the f lists, then all the b lists; word = id | m << ib with the one multiplicity that list needs,
// capped at 2^(32 - ib) - 1: read the exact value from out(x) then).  A walk of out(v) for the edge
// u -> v becomes a walk of out_f(v) when m(u,v) >= 1 plus one of out_b(v) when m(v,u) >= 1; R-MAT's
// undirected pairs are single-direction for 97 % (class (1,0) or (0,1)), so a walk reads about half the
// entries.  fbo[2x] / fbo[2x + 1] = start of out_f(x) / out_b(x) (2n + 2 entries, uint32: the lists
// hold < 2^32 entries whenever the packed in-keys are used).  Exclusive ranks: rk[2e] = the f-entries
// before oriented edge e, rk[2e + 1] = nF + the b-entries before it (the in-lists' prefix lengths).

__device__ __forceinline__ void split_flags(uint32_t w, TgCode tc, uint32_t& f, uint32_t& b) {
    f = (w >> tc.ib) & tc.cmask();
    b = (w >> (tc.ib + tc.cb)) & tc.cmask();
}

// a lane's 8 consecutive target words (base a multiple of 8): two 16-byte loads, 0 past ne
__device__ __forceinline__ void load8_words(const uint32_t* __restrict__ tg, int64_t base, int64_t ne, uint32_t (&w)[8]) {
    if (base + 8 <= ne) {
        const uint4 a = reinterpret_cast<const uint4*>(tg + base)[0], b = reinterpret_cast<const uint4*>(tg + base)[1];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
        w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = base + j < ne ? tg[base + j] : 0u;
    }
}

__global__ void __launch_bounds__(256) k_split_count(const uint32_t* __restrict__ tg, int64_t ne, TgCode tc,
                                                     int64_t* __restrict__ cnt, int64_t ntiles) {
    const int64_t base = (int64_t)blockIdx.x * kSplitTile + (int64_t)threadIdx.x * 8;
    int64_t cf = 0, cb = 0;
    uint32_t w[8];
    load8_words(tg, base, ne, w);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (base + j < ne) {
            uint32_t f, b;
            split_flags(w[j], tc, f, b);
            cf += f != 0;
            cb += b != 0;
        }
    for (int o = 32; o > 0; o >>= 1) {
        cf += __shfl_down(cf, o, 64);
        cb += __shfl_down(cb, o, 64);
    }
    __shared__ int64_t s[2][4];
    if ((threadIdx.x & 63) == 0) {
        s[0][threadIdx.x >> 6] = cf;
        s[1][threadIdx.x >> 6] = cb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        cnt[blockIdx.x] = s[0][0] + s[0][1] + s[0][2] + s[0][3];
        cnt[ntiles + 1 + blockIdx.x] = s[1][0] + s[1][1] + s[1][2] + s[1][3];
    }
}

// tile-exclusive ranks, the split words and rk; pre = the tiles' exclusive f / b prefix sums
// (pre[0, ntiles], pre[ntiles + 1, 2 ntiles + 1])
__global__ void __launch_bounds__(256) k_split_write(const uint32_t* __restrict__ tg, const int64_t* __restrict__ ov,
                                                     int64_t ne, TgCode tc, const int64_t* __restrict__ pre,
                                                     int64_t ntiles, uint32_t* __restrict__ tgs,
                                                     uint32_t* __restrict__ rk) {
    const int64_t base = (int64_t)blockIdx.x * kSplitTile + (int64_t)threadIdx.x * 8;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t w[8];
    uint32_t cf = 0, cb = 0;
    load8_words(tg, base, ne, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint32_t f, b;
        split_flags(w[j], tc, f, b);
        cf += f != 0;
        cb += b != 0;
    }
    // block-exclusive scan of the packed (f, b) counts (each < 2^16 per tile)
    const uint32_t mine = cf | cb << 16;
    uint32_t x = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __shared__ uint32_t wt[4];
    if (lane == 63) wt[wave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (int q = 0; q < wave; ++q) wb += wt[q];
    const uint32_t ex = x - mine + wb;
    const int64_t nF = pre[ntiles];
    int64_t rf = pre[blockIdx.x] + (ex & 0xFFFFu), rb = nF + pre[ntiles + 1 + blockIdx.x] + (ex >> 16);
    const uint32_t cap = ~0u >> tc.ib, idm = tc.idmask();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int64_t e = base + j;
        if (e >= ne) break;
        uint32_t f, b;
        split_flags(w[j], tc, f, b);
        reinterpret_cast<uint2*>(rk)[e] = make_uint2((uint32_t)rf, (uint32_t)rb);
        if (f == tc.cmask() || b == tc.cmask()) {  // an exception: the exact multiplicities
            const uint64_t p = (uint64_t)ov[e];
            f = (uint32_t)min<uint64_t>(p >> 32, cap);
            b = (uint32_t)min<uint64_t>(p & 0xffffffffULL, cap);
        }
        const uint32_t id = w[j] & idm;
        if (f) tgs[rf++] = id | f << tc.ib;
        if (b) tgs[rb++] = id | b << tc.ib;
    }
}

// list starts: fbo[2x] = rk_f at off[x] (nF past the last edge), fbo[2x + 1] likewise for the b lists
__global__ void k_split_off(const int64_t* __restrict__ off, int64_t n, int64_t ne, const uint32_t* __restrict__ rk,
                            uint32_t nF, uint32_t nFB, uint32_t* __restrict__ fbo) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x <= n; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = off[x];
        fbo[2 * x] = e < ne ? rk[2 * e] : nF;
        fbo[2 * x + 1] = e < ne ? rk[2 * e + 1] : nFB;
    }
}

// per-vertex list record of the split walks: {start of out_f(x), start of out_b(x), |out_f(x)| | |out_b(x)| << 16,
// od(x)} -- one 16-byte load sets up both lists of an edge u -> x (and the v-mode skip test) instead of the
// offsets' and the list starts' separate lines (lengths < 2^16: the split walks run with packed in-keys)
// (od32: the out-degrees alone, 4 bytes a vertex, for the in-list records' random reads)
__global__ void k_vrec(const int64_t* __restrict__ off, const uint32_t* __restrict__ fbo, int64_t n,
                       uint4* __restrict__ vrec, uint32_t* __restrict__ od32) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t f0 = fbo[2 * x], b0 = fbo[2 * x + 1], od = (uint32_t)(off[x + 1] - off[x]);
        vrec[x] = make_uint4(f0, b0, (fbo[2 * x + 2] - f0) | (fbo[2 * x + 3] - b0) << 16, od);
        od32[x] = od;
    }
}

// in-list records of the split walks, in oriented-edge order (sequential reads; `to` is a hub, its
// offsets cached), 16 bytes: x = from | the edge's multiplicity codes (a coded word whose id is the
// source), y = pf | pb << 16 (the f / b entries of out(from) below `to`; 0 when v-mode does not take the
// edge: p >= od(to), u-mode walks it), z / w = the starts of out_f(from) / out_b(from) -- so a v-mode
// list's setup is one dependent load after its key; the in-key to << 40 | e, sorted on the digits of `to`
// (stable: edge order within a target); the v-mode items read the records through it
// A block writes whole 4096-key sort tiles and counts their first sort digit (bits hshift..+7) into hist
// (radix_sort_keys' hist0: the in-key sort's first pass reads no histogram)
__global__ void __launch_bounds__(256) k_swap_keys_sp(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ off,
                                                      int64_t ne, TgCode tc, const uint32_t* __restrict__ tg,
                                                      const uint32_t* __restrict__ rk, const uint32_t* __restrict__ fbo,
                                                      const uint32_t* __restrict__ od32, uint64_t* __restrict__ ik,
                                                      uint4* __restrict__ rec, int64_t* __restrict__ hist, int hshift) {
    constexpr int U = 4;  // edges per lane and round, loads issued together
    const uint32_t idm = tc.idmask();
    __shared__ unsigned int h[256];
    auto round = [&](int64_t e0) {  // edges e0 + j * 256
        uint64_t k[U];
        uint32_t w[U];
        uint2 r[U], fb[U];
        int64_t of[U];
        uint32_t odt[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t e = min(e0 + (int64_t)j * 256, ne - 1);
            k[j] = ok_[e];
            w[j] = tg[e];
            r[j] = reinterpret_cast<const uint2*>(rk)[e];
        }
        // three lane loads per edge: off(from), the from's list starts (one 8-byte word) and od(to) from the
        // 4-byte degree array (was: the to's 16-byte vertex record, and before that off(to) and off(to + 1))
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t from = (uint32_t)(k[j] >> 32), to = (uint32_t)k[j] & idm;
            of[j] = off[from];
            fb[j] = reinterpret_cast<const uint2*>(fbo)[from];
            odt[j] = od32[to];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t e = e0 + (int64_t)j * 256;
            if (e >= ne) break;
            const uint32_t from = (uint32_t)(k[j] >> 32), to = (uint32_t)k[j] & idm;
            const bool take = e - of[j] < (int64_t)odt[j];
            const uint32_t pfb = take ? (r[j].x - fb[j].x) | (r[j].y - fb[j].y) << 16 : 0u;
            rec[e] = make_uint4(from | (w[j] & ~idm), pfb, fb[j].x, fb[j].y);
            const uint64_t key = (uint64_t)to << 40 | (uint64_t)e;
            ik[e] = key;
            atomicAdd(&h[(uint32_t)(key >> hshift) & 255u], 1u);
        }
    };
    const int64_t ntiles = (ne + kSortTile - 1) / kSortTile;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {  // block-uniform
        h[threadIdx.x] = 0;
        __syncthreads();
        for (int q = 0; q < kSortTile / (256 * U); ++q) round(t * kSortTile + (int64_t)q * 256 * U + threadIdx.x);
        __syncthreads();
        hist[(int64_t)threadIdx.x * ntiles + t] = h[threadIdx.x];
        __syncthreads();  // h is cleared for the next tile
    }
}

// the selected edges' in-keys and records (a distributed build's share; sel in edge order)
__global__ void k_swap_keys_sp_sel(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ off,
                                   const int64_t* __restrict__ sel, int64_t nsel, TgCode tc,
                                   const uint32_t* __restrict__ tg, const uint32_t* __restrict__ rk,
                                   const uint32_t* __restrict__ fbo, uint64_t* __restrict__ ik, uint4* __restrict__ rec) {
    const uint32_t idm = tc.idmask();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsel; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = sel[i];
        const uint64_t k = ok_[e];
        const uint32_t from = (uint32_t)(k >> 32), to = (uint32_t)k & idm;
        const uint32_t f0 = fbo[2 * from], b0 = fbo[2 * from + 1];
        const uint32_t pfb = (rk[2 * e] - f0) | (rk[2 * e + 1] - b0) << 16;  // taken
        rec[i] = make_uint4(from | (tg[e] & ~idm), pfb, f0, b0);
        ik[i] = (uint64_t)to << 40 | (uint64_t)i;
    }
}

constexpr uint64_t kInRecMask = (uint64_t(1) << 40) - 1;  // the record index of a split in-key


// v-mode centers: od(v) >= vmt with at least one in-edge
__global__ void k_tri_vm_bins(const int64_t* __restrict__ off, const int64_t* __restrict__ ioff, int64_t n, int vmt,
                              uint8_t* __restrict__ f) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (int64_t)gridDim.x * blockDim.x)
        f[v] = off[v + 1] - off[v] >= vmt && ioff[v + 1] > ioff[v];
}


// CSR offsets of sorted keys whose group field starts at bit `sh`: off[v] = first key with field >= v
__global__ void k_offsets(const uint64_t* __restrict__ ok_, int64_t ne, int64_t n, int sh, int64_t* __restrict__ off) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = ne;
        const uint64_t target = (uint64_t)v << sh;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ok_[mid] < target) lo = mid + 1; else hi = mid;
        }
        off[v] = lo;
    }
}

// ---- triangles: vertex-centric hashing -----------------------------------------------------
// Every triangle {u, v, w} is found once, from its lowest vertex u in (degree, id) order:
// v, w in out(u) and w in out(v).  For each u the out-list is put in an LDS hash (w -> payload
// m(u,w)<<32 | m(w,u)); the wedges (v, w) for v in out(u), w in out(v) are then walked as one flat
// index range (prefix sums of the out-degrees of the v's, binary-searched in LDS) so the lanes
// read out(v) lists contiguously whatever their lengths, and each wedge costs one 4-byte load and
// an LDS probe (the payload of (v, w) is loaded only on a hit).  Orientation by degree bounds
// every out-degree by O(sqrt(E)).  u with out-degree <= 64 go one per wave, larger ones one per
// 1024-lane workgroup (their lists are taken in chunks when they exceed the LDS hash).
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kSmallDeg = 64;
// (the list walks' target loads in flight per lane, U: 4 since the direction choice moved the long hub
// lists to v-mode -- 126.5 ms against 132.4 with 8; before it, 8 beat 4 by 5 %)
constexpr int kSmallSlots = 512;  // load <= 1/8: a miss (most wedges) ends after ~1.2 probes
constexpr int kTriBlock = 256;  // small: 4 waves

// Multiplicative hashes on the full-rate 24-bit multiplier (a 32-bit v_mul_lo is quarter rate, and
// the walks are VALU-bound): the id's bits above 24 are folded in first, so every bit counts
// (both operands masked to 24 bits, so the compiler selects v_mul_u32_u24 for the low 32 bits)
__device__ __forceinline__ uint32_t fold24(uint32_t w) { return (w ^ (w >> 24)) & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) { return a * b; }
__device__ __forceinline__ uint32_t hslot(uint32_t w, int log2cap) { return mul24(fold24(w), 0x9E3779u) >> (32 - log2cap); }

#ifndef CAPSMI_TRI_IDBLOOM
#define CAPSMI_TRI_IDBLOOM 1
#endif

// One-bit pre-filter in front of each hash: a wave's probe loop runs as long as its longest
// chain, so most wedges (misses) are rejected with one LDS read instead.
constexpr int kSmallBloomBits = 10, kBigBloomBits = 16;

// CAPSMI_TRI_IDBLOOM: the filter bit is the id's low bits.  Ids are in degree order (hubs first): a
// hub list's entries are small ids, exact under 2^bits, and other ids' low bits spread like a
// hash's, so the filter passes no more than before while every probe saves the fold and the
// multiply.  (The hash slot keeps the multiplicative hash: with linear probing, runs of
// consecutive ids would form long clusters.)
__device__ __forceinline__ uint32_t bbit(uint32_t w, int bits) {
    return CAPSMI_TRI_IDBLOOM ? (w & ((1u << bits) - 1)) : mul24(fold24(w), 0xC2B2AFu) >> (32 - bits);
}

__device__ __forceinline__ void bset(uint32_t* bf, int bits, uint32_t w) {
    const uint32_t x = bbit(w, bits);
    atomicOr(&bf[x >> 5], 1u << (x & 31));
}

__device__ __forceinline__ bool btest(const uint32_t* bf, int bits, uint32_t w) {
    const uint32_t x = bbit(w, bits);
    return (bf[x >> 5] >> (x & 31)) & 1u;
}

// Oriented targets carry their edge's multiplicities (`TgCode`): word = to | f << ib | b << (ib + cb),
// f = m(from, to), b = m(to, from), cb bits each; a field at its all-ones value (cmask) marks an
// exception whose exact payload is read from ov.  The wedge walks then resolve a hit from the two words
// alone (a hit used to cost two dependent 8-byte payload loads: 47 of the 116 ms at C4, measured by a
// run with the loads removed).  With 2^24 ids, cb = 4: < 1 % of the hits need an exact payload (R-MAT
// s = 20 / 22, hits whose edges carry a multiplicity >= 15).

__device__ __forceinline__ uint32_t tid(uint32_t word, TgCode c) { return word & c.idmask(); }

// payload (f << 32 | b) of a coded word, or the exact one at ov[pos] for an exception
__device__ __forceinline__ uint64_t tpay(uint32_t word, TgCode c, const int64_t* __restrict__ ov, int64_t pos) {
    if (c.cb == 0) return (uint64_t)ov[pos];
    const uint32_t f = (word >> c.ib) & c.cmask(), b = (word >> (c.ib + c.cb)) & c.cmask();
    if (f == c.cmask() || b == c.cmask()) return (uint64_t)ov[pos];
    return (uint64_t)f << 32 | b;
}

// word (id + code bits; the id is the hash key), and the index of its entry in the hashed list (the
// exact payload of an exception is read through it)
template <class Idx>
__device__ __forceinline__ void hinsert(uint32_t* hk, Idx* hi, int log2cap, uint32_t id, uint32_t word, uint32_t idx) {
    const uint32_t mask = (1u << log2cap) - 1;
    uint32_t sl = hslot(id, log2cap);
    while (true) {
        const uint32_t prev = atomicCAS(&hk[sl], kEmpty, word);
        if (prev == kEmpty) {
            hi[sl] = (Idx)idx;
            return;
        }
        sl = (sl + 1) & mask;
    }
}

// slot of id w (keys compared under idm), or -1
__device__ __forceinline__ int hfind(const uint32_t* hk, int log2cap, uint32_t w, uint32_t idm) {
    const uint32_t mask = (1u << log2cap) - 1;
    uint32_t sl = hslot(w, log2cap);
    while (true) {
        const uint32_t k = hk[sl];
        if (k == kEmpty) return -1;
        if ((k & idm) == w) return (int)sl;
        sl = (sl + 1) & mask;
    }
}

__device__ __forceinline__ unsigned long long tri_weight(uint64_t puv, uint64_t pvw, uint64_t puw) {
    const uint64_t m_uv = puv >> 32, m_vu = puv & 0xffffffffULL;
    const uint64_t m_vw = pvw >> 32, m_wv = pvw & 0xffffffffULL;
    const uint64_t m_uw = puw >> 32, m_wu = puw & 0xffffffffULL;
    return m_uv * m_vw * m_wu + m_uw * m_wv * m_vu;
}

struct SmallWave {
    uint32_t bf[(1 << kSmallBloomBits) / 32];
    uint32_t hk[kSmallSlots];
    uint8_t hi[kSmallSlots];  // lane of the key's entry: payload = vp[hi]
    uint64_t vp[kSmallDeg];
    int64_t voff[kSmallDeg];
    uint32_t vl[kSmallDeg];
    uint32_t dv[kSmallDeg];
};


// a wave-uniform 64-bit value into scalar registers, so addresses built on it take the scalar base +
// 32-bit lane offset form instead of 64-bit vector arithmetic per load
__device__ __forceinline__ int64_t uniform64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// One pass of a wave over U x 64 consecutive entries of a list (this lane: entries j0 + r * 64):
// the loads are unconditional at clamped indexes, which keeps them free of per-load branches.  Then
// the U pre-filter words are read together before any is tested; `keep` marks the entries that pass.
// w[] are the coded words (id + multiplicities).
template <int U>
__device__ __forceinline__ void list_pass(const uint32_t* __restrict__ tg, TgCode tc, int64_t vo, int dv, int j0,
                                          const uint32_t* bf, int bits, uint32_t (&w)[U], uint32_t& keep) {
    // unsigned 32-bit indexes off a scalar base: the loads take the scalar-base + lane-offset form
    const uint32_t last = (uint32_t)dv - 1u, j = (uint32_t)j0;
    const char* __restrict__ p = reinterpret_cast<const char*>(tg + vo);
#pragma unroll
    for (int r = 0; r < U; ++r) w[r] = *reinterpret_cast<const uint32_t*>(p + (min(j + (uint32_t)r * 64u, last) << 2));
    uint32_t word[U], bit[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
        bit[r] = bbit(tid(w[r], tc), bits);
        word[r] = bf[bit[r] >> 5];
    }
    keep = 0;  // branch-free: in range and pre-filter bit set
#pragma unroll
    for (int r = 0; r < U; ++r)
        keep |= ((uint32_t)(j + (uint32_t)r * 64u <= last) & (word[r] >> (bit[r] & 31))) << r;
}

// the wave walks each out(v) with all lanes (as k_tri_big_items)
template <int U>
__global__ void __launch_bounds__(kTriBlock) k_tri_small(const uint32_t* __restrict__ tg, TgCode tc,
                                                         const int64_t* __restrict__ ov,
                                                         const int64_t* __restrict__ off, int vmt,
                                                         const int64_t* __restrict__ us, int64_t nu,
                                                         unsigned long long* __restrict__ out) {
    __shared__ SmallWave sw[kTriBlock / 64];
    SmallWave& W = sw[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    unsigned long long acc = 0;
    const int64_t nwaves = (int64_t)gridDim.x * (kTriBlock / 64);
    for (int64_t q = (int64_t)blockIdx.x * (kTriBlock / 64) + (threadIdx.x >> 6); q < nu; q += nwaves) {
        const int64_t u = us[q];
        const int64_t b = off[u];
        const int d = (int)(off[u + 1] - b);
#pragma unroll
        for (int k = 0; k < kSmallSlots / 64; ++k) W.hk[lane + 64 * k] = kEmpty;
        if (lane < (1 << kSmallBloomBits) / 32) W.bf[lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t dv = 0;
        if (lane < d) {
            const uint32_t v = tid(tg[b + lane], tc);
            const uint64_t pv = tpay(tg[b + lane], tc, ov, b + lane);
            const int64_t vo = off[v];
            dv = (uint32_t)(off[v + 1] - vo);
            if (vmt > 0 && dv >= (uint32_t)vmt && (uint32_t)lane < dv) dv = 0;  // v-mode takes u -> v
            W.vl[lane] = v;
            W.vp[lane] = pv;
            W.voff[lane] = vo;
            W.dv[lane] = dv;
            hinsert(W.hk, W.hi, 9, v, v, (uint32_t)lane);
            bset(W.bf, kSmallBloomBits, v);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lists of <= 64 / <= 128 entries walked four / two per pass (as in k_tri_big_items), the
        // rest one per pass with U loads per lane
        const uint64_t sm = __ballot(dv > 0u && dv <= 64u), mm = __ballot(dv > 64u && dv <= 128u);
        uint64_t lm = __ballot(dv > 128u);
        auto grouped = [&](uint64_t mask, int sgl) {
            const int per = 64 >> sgl, sg = 1 << sgl, g = lane >> sgl, e = lane & (sg - 1);
            while (mask) {  // wave-uniform
                uint64_t m = mask;
                for (int i = 0; i < g; ++i) m &= m - 1;  // this lane group's list: the g-th of the mask
                const bool live = m != 0;
                const int k = __builtin_ctzll(live ? m : mask);
                for (int i = 0; i < per; ++i) mask &= mask - 1;
                const int64_t vo = W.voff[k];
                const uint32_t dvk = live ? W.dv[k] : 0u, last = (dvk ? dvk : 1u) - 1u;
                uint32_t w[4], word[4], bit[4], keep = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) w[t] = tg[vo + (int64_t)min((uint32_t)(e + sg * t), last)];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    bit[t] = bbit(tid(w[t], tc), kSmallBloomBits);
                    word[t] = W.bf[bit[t] >> 5];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    keep |= ((uint32_t)((uint32_t)(e + sg * t) < dvk) & (word[t] >> (bit[t] & 31))) << t;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (!((keep >> t) & 1u)) continue;
                    const int sl = hfind(W.hk, 9, tid(w[t], tc), ~0u);
                    if (sl >= 0) acc += tri_weight(W.vp[k], tpay(w[t], tc, ov, vo + e + sg * t), W.vp[W.hi[sl]]);
                }
            }
        };
        grouped(sm, 4);
        grouped(mm, 5);
        while (lm) {  // wave-uniform
            const int k = __builtin_ctzll(lm);
            lm &= lm - 1;
            const int64_t vo = uniform64(W.voff[k]);
            const uint32_t dvk = __builtin_amdgcn_readfirstlane(W.dv[k]);
            const uint64_t puv = W.vp[k];
            for (int j0 = lane; j0 < (int)dvk; j0 += U * 64) {
                uint32_t w[U], keep;  // U target loads in flight per lane
                list_pass<U>(tg, tc, vo, (int)dvk, j0, W.bf, kSmallBloomBits, w, keep);
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    if (!((keep >> r) & 1u)) continue;
                    const int sl = hfind(W.hk, 9, tid(w[r], tc), ~0u);
                    if (sl >= 0) acc += tri_weight(puv, tpay(w[r], tc, ov, vo + j0 + r * 64), W.vp[W.hi[sl]]);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the wave's LDS is reused for the next u
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (lane == 0 && acc) atomicAdd(out, acc);
}

// Big u are split into work items (hash chunk of out(u), chunk of kVChunk v's of out(u)) so a hub's
// wedges spread over many workgroups; items are taken from a global counter (dynamic balance).
constexpr int kVChunk = 256;
// neighbour chunks per item: the item builds its hash chunk once and walks up to kVGroup chunks of
// lists against it (one chunk per item rebuilt the same hash for every 256 lists: at C4 the items'
// setup without their walks took 12-13 ms of each launch)
constexpr int kVGroup = 8;
// lanes per short list in the item walks (lists of <= 4 kSG entries: 64 / kSG of them per wave pass)
#ifndef CAPSMI_TRI_SG
#define CAPSMI_TRI_SG 16
#endif
constexpr int kSG = CAPSMI_TRI_SG;
static_assert(kSG == 8 || kSG == 16 || kSG == 32, "short-list lanes");

// Items run in B-lane workgroups with hash chunks of 2 B out-list entries (4 slots each): 1024 lanes
// for v-mode (hub centers with long out-lists), 512 for u-mode, whose many small items are bound by
// their setup's load latency -- four 512-lane items in flight per CU instead of two 1024-lane ones.
template <int B>
struct ItemLds {
    static constexpr int kChunk = 2 * B, kSlots = 4 * kChunk;
    uint32_t bf[(1 << kBigBloomBits) / 32];
    uint32_t hk[kSlots];
    uint16_t hi[kSlots];  // position of the key in out(u)'s hash chunk: payload = ov[b + h0 + hi]
    uint64_t vp[kVChunk];
    int64_t voff[kVChunk];
    uint32_t vl[kVChunk];
    uint32_t dv[kVChunk];
    uint32_t pre[kVChunk];  // the long and short lists' indexes (2 x uint16)
    uint16_t mk[kVChunk];   // the medium lists' indexes
    uint32_t ncnt[6];       // [3 (c & 1) + 0/1/2] long / short / medium lists of chunk c
    unsigned long long item;
};

// items of center q: hash chunks of out(c) x chunks of its neighbour list (out(c), or in(c) when
// ioff is set: v-mode)
// (epi: neighbour-list entries per item -- kVChunk * kVGroup, or the split items' EPI)
__global__ void k_tri_items(const int64_t* __restrict__ off, const int64_t* __restrict__ ioff,
                            const int64_t* __restrict__ us, int64_t nu, int chunk, int epi, int64_t* __restrict__ items) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nu) return;
    const int64_t c = us[q], d = off[c + 1] - off[c], nd = ioff ? ioff[c + 1] - ioff[c] : d;
    items[q] = ((d + chunk - 1) / chunk) * ((nd + epi - 1) / epi);
}

// item -> (its center's index q) | (its index among q's items) << 32: one load per item instead of a
// ~20-step dependent binary search over ipre at the start of every item
__global__ void k_tri_item_map(const int64_t* __restrict__ ipre, int64_t nu, uint64_t* __restrict__ item_ql) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nu; q += (int64_t)gridDim.x * blockDim.x)
        for (int64_t it = ipre[q]; it < ipre[q + 1]; ++it) item_ql[it] = (uint64_t)q | ((uint64_t)(it - ipre[q]) << 32);
}

// Each wave walks whole out(v) lists of the item's v chunk (wave q takes v = q, q + 16, ...), its lanes
// striding the list -- coalesced loads, no per-wedge segment search.  The wedges of big u lie in long
// lists (wedge-weighted mean ≈600 at R-MAT s = 22; 99.8 % in lists of ≥ 64), so the lanes stay busy; a
// flat form (one prefix-sum index range over the chunk's wedges, removed in round 6) spent ≈70 VALU
// instructions per wedge on the cursor and the segment search and was issue-bound.
// VM (v-mode): the center c is the middle vertex v; its hash holds out(v) and the walked lists are
// out(u) for the in-neighbours u of v with od(u) <= od(v).  Otherwise (u-mode) c = u and the walked
// lists are out(v) for v in out(u), less the edges v-mode takes (vmt > 0: od(v) >= vmt, od(u) <= od(v)).
// Register budget: two 1024-lane items per CU need 8 waves per SIMD, i.e. an SGPR granule of at most
// 96 (800 per SIMD): .amdhsa_next_free_sgpr <= 74 here.  At 77 the v-mode launch admitted one item
// per CU and took 113 instead of 69 ms (the u-mode 512-lane one 25 instead of 21.6 ms).
template <int U, bool VM, int B>
__global__ void __launch_bounds__(B, 8) k_tri_big_items(const uint32_t* __restrict__ tg, TgCode tc,
                                                             const int64_t* __restrict__ ov,
                                                             const int64_t* __restrict__ off,
                                                             const int64_t* __restrict__ ioff,
                                                             const uint32_t* __restrict__ itg,
                                                             const uint32_t* __restrict__ ipos, int vmt,
                                                             const int64_t* __restrict__ us, int64_t nu,
                                                             const int64_t* __restrict__ ipre,
                                                             const uint64_t* __restrict__ item_ql,
                                                             unsigned long long* __restrict__ ctr,
                                                             unsigned long long* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    ItemLds<B>& L = *reinterpret_cast<ItemLds<B>*>(lds_raw);
    constexpr int CH = ItemLds<B>::kChunk;
    unsigned long long& item = L.item;
    const int64_t total = ipre[nu];
    unsigned long long acc = 0;
    while (true) {
        if (threadIdx.x == 0) item = atomicAdd(ctr, 1ULL);
        __syncthreads();
        const int64_t it = (int64_t)item;
        __syncthreads();  // `item` is rewritten next round
        if (it >= total) break;  // block-uniform
        const uint64_t iw = item_ql[it];
        const int64_t lo = (uint32_t)iw;
        const int64_t u = us[lo], b = uniform64(off[u]);  // the center (u-mode: u; v-mode: v)
        const int d = (int)(off[u + 1] - b);
        const int64_t nb = VM ? uniform64(ioff[u]) : b;   // its neighbour list: in(v) / out(u)
        const int nd = VM ? (int)(ioff[u + 1] - nb) : d;
        const int nvc = (nd + kVChunk - 1) / kVChunk, ngr = (nvc + kVGroup - 1) / kVGroup;
        const int local = (int)(iw >> 32);
        const int h0 = (local / ngr) * CH, c0 = (local % ngr) * kVGroup, c1 = min(nvc, c0 + kVGroup);
        const int hn = min(CH, d - h0);
        int lc = 6;  // hash capacity 2^lc >= 4 hn (load <= 1/4), cleared as far as it is used
        while ((1 << lc) < 4 * hn) ++lc;
        for (int k = threadIdx.x; k < (1 << lc); k += B) L.hk[k] = kEmpty;
        for (int k = threadIdx.x; k < (1 << kBigBloomBits) / 32; k += B) L.bf[k] = 0;
        if (threadIdx.x < 6) L.ncnt[threadIdx.x] = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < hn; k += B) {
            const uint32_t word = tg[b + h0 + k], w = tid(word, tc);
            hinsert(L.hk, L.hi, lc, w, word, (uint32_t)k);
            bset(L.bf, kBigBloomBits, w);
        }
        for (int c = c0; c < c1; ++c) {  // block-uniform
            const int v0 = c * kVChunk, vn = min(kVChunk, nd - v0);
            if (c > c0) __syncthreads();  // the previous chunk's walks are done with the list table
            uint16_t* lk = reinterpret_cast<uint16_t*>(L.pre);  // lists of > 64 entries
            uint16_t* sk = lk + kVChunk;                        // lists of 1..64 entries
            uint32_t* nc = L.ncnt + 3 * (c & 1);
            if (threadIdx.x < 3) L.ncnt[3 * ((c + 1) & 1) + threadIdx.x] = 0;  // read last by chunk c - 1
            for (int k = threadIdx.x; k < vn; k += B) {
                const uint32_t v = VM ? itg[nb + v0 + k] : tid(tg[b + v0 + k], tc);
                const int64_t vo = off[v];
                const uint32_t dv = (uint32_t)(off[v + 1] - vo);
                const int64_t e = VM ? vo + ipos[nb + v0 + k] : b + v0 + k;  // the edge u -> v either way
                L.vl[k] = v;
                L.vp[k] = tpay(tg[e], tc, ov, e);
                L.voff[k] = vo;
                // v-mode walks out(u) below the center: the prefix [0, p) of out(u), p = position of the
                // edge; u-mode skips the edges v-mode takes (od(v) >= vmt and p < od(v))
                const uint32_t p = (uint32_t)(e - (VM ? vo : b));
                const uint32_t dw = VM ? (p < (uint32_t)d ? p : 0u) : (vmt > 0 && dv >= (uint32_t)vmt && p < dv ? 0u : dv);
                L.dv[k] = dw;
                if (dw > 8u * kSG) lk[atomicAdd(&nc[0], 1u)] = (uint16_t)k;
                else if (dw > 4u * kSG) L.mk[atomicAdd(&nc[2], 1u)] = (uint16_t)k;
                else if (dw > 0u) sk[atomicAdd(&nc[1], 1u)] = (uint16_t)k;
            }
            __syncthreads();
            const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
            const int nlong = (int)__builtin_amdgcn_readfirstlane(nc[0]);
            const int nshort = (int)__builtin_amdgcn_readfirstlane(nc[1]);
            // short lists (most of them: the median v-mode prefix is ≈56 entries at s = 20): four per
            // pass of the wave, 16 lanes each, four loads per lane -- four lists' lines in flight at
            // once instead of one list's one or two.  The list index is per lane (vector registers:
            // U uniform list bases would cost the SGPR budget above)
            const int nmed = (int)__builtin_amdgcn_readfirstlane(nc[2]);
            // ks[0, nk): lists of <= 4 << sgl entries, (64 >> sgl) per wave pass, 1 << sgl lanes each
            auto grouped = [&](const uint16_t* ks, int nk, int sgl) {
                const int per = 64 >> sgl, sg = 1 << sgl;
                for (int q0 = wave * per; q0 < nk; q0 += (B / 64) * per) {
                    const int g = lane >> sgl, e = lane & (sg - 1);
                    const bool live = q0 + g < nk;
                    const int k = ks[live ? q0 + g : q0];
                    const int64_t vo = L.voff[k];
                    const uint32_t dvk = live ? L.dv[k] : 0u, last = (dvk ? dvk : 1u) - 1u;
                    uint32_t w[4], word[4], bit[4], keep = 0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) w[t] = tg[vo + (int64_t)min((uint32_t)(e + sg * t), last)];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        bit[t] = bbit(tid(w[t], tc), kBigBloomBits);
                        word[t] = L.bf[bit[t] >> 5];
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        keep |= ((uint32_t)((uint32_t)(e + sg * t) < dvk) & (word[t] >> (bit[t] & 31))) << t;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (!((keep >> t) & 1u)) continue;
                        const int sl = hfind(L.hk, lc, tid(w[t], tc), tc.idmask());
                        if (sl >= 0) {
                            const uint64_t pxw = tpay(w[t], tc, ov, vo + e + sg * t);
                            const uint64_t pcw = tpay(L.hk[sl], tc, ov, b + h0 + L.hi[sl]);
                            const uint64_t puv = L.vp[k];
                            acc += VM ? tri_weight(puv, pcw, pxw) : tri_weight(puv, pxw, pcw);
                        }
                    }
                }
            };
            grouped(sk, nshort, kSG == 8 ? 3 : kSG == 16 ? 4 : 5);
            grouped(L.mk, nmed, kSG == 8 ? 4 : kSG == 16 ? 5 : 6);
            for (int q = wave; q < nlong; q += B / 64) {  // long lists: one per wave, U x 64 entries a pass
                const int k = lk[q];
                const int64_t vo = uniform64(L.voff[k]);
                const int64_t dv = (int64_t)__builtin_amdgcn_readfirstlane(L.dv[k]);
                const uint64_t puv = L.vp[k];
                for (int j0 = lane; j0 < (int)dv; j0 += U * 64) {
                    uint32_t w[U], keep;  // U target loads in flight per lane
                    list_pass<U>(tg, tc, vo, (int)dv, j0, L.bf, kBigBloomBits, w, keep);
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        if (!((keep >> r) & 1u)) continue;
                        const int sl = hfind(L.hk, lc, tid(w[r], tc), tc.idmask());
                        if (sl >= 0) {
                            const uint64_t pxw = tpay(w[r], tc, ov, vo + j0 + r * 64);
                            const uint64_t pcw = tpay(L.hk[sl], tc, ov, b + h0 + L.hi[sl]);
                            acc += VM ? tri_weight(puv, pcw, pxw) : tri_weight(puv, pxw, pcw);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// ---- walks over the direction-split lists (k_split_write) ---------------------------------------------
// The exact multiplicity payload of x -> w (w in out(x)): a search of the sorted out(x) -- only for a
// split word at its cap or an in-list word whose codes are an exception (rare: m >= 2^(32 - ib) - 1 / 15)
__device__ __forceinline__ uint64_t exact_pay(const uint32_t* __restrict__ tg, TgCode tc, const int64_t* __restrict__ ov,
                                           const int64_t* __restrict__ off, uint32_t x, uint32_t w) {
    int64_t lo = off[x], hi = off[x + 1];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (tid(tg[mid], tc) < w) lo = mid + 1; else hi = mid;
    }
    return tpay(tg[lo], tc, ov, lo);
}

// m of a split word: the list's multiplicity (f list of x: m(x,w); b list: m(w,x))
__device__ __forceinline__ uint64_t split_m(uint32_t word, TgCode tc, bool bl, const uint32_t* __restrict__ tg,
                                            const int64_t* __restrict__ ov, const int64_t* __restrict__ off, uint32_t x) {
    const uint32_t m = word >> tc.ib, cap = ~0u >> tc.ib;
    if (m != cap) return m;
    const uint64_t p = exact_pay(tg, tc, ov, off, x, tid(word, tc));
    return bl ? (p & 0xffffffffULL) : (p >> 32);
}

// the hit's third factor from the hashed entry's payload ph = (m(c,w), m(w,c)): an f list closes through
// m(w,c), a b list through m(c,w)
__device__ __forceinline__ uint64_t split_field(uint64_t ph, bool bl) { return bl ? (ph >> 32) : (ph & 0xffffffffULL); }

struct SmallWaveSp {
    uint32_t bf[(1 << kSmallBloomBits) / 32];
    uint32_t hk[kSmallSlots];
    uint8_t hi[kSmallSlots];     // lane of the key's entry: payload = vp[hi]
    uint64_t vp[kSmallDeg];      // payload of u -> v
    uint32_t vl[kSmallDeg];      // v (exact multiplicities)
    uint32_t lo[2 * kSmallDeg];  // list l (f: l < 64, b: l >= 64) of v = l & 63: tgs[lo, lo + ln)
    uint32_t ln[2 * kSmallDeg];
    uint32_t kq[2 * kSmallDeg];  // its constant factor: m(u,v) (f) / m(v,u) (b)
};

// k_tri_small over the split lists: each v of out(u) gives an f and a b list (either may be empty)
template <int U>
__global__ void __launch_bounds__(kTriBlock) k_tri_small_sp(const uint32_t* __restrict__ tg, TgCode tc,
                                                            const int64_t* __restrict__ ov,
                                                            const int64_t* __restrict__ off,
                                                            const uint32_t* __restrict__ tgs,
                                                            const uint4* __restrict__ vrec, int vmt,
                                                            const int64_t* __restrict__ us, int64_t nu,
                                                            unsigned long long* __restrict__ out) {
    __shared__ SmallWaveSp sw[kTriBlock / 64];
    SmallWaveSp& W = sw[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    unsigned long long acc = 0;
    const int64_t nwaves = (int64_t)gridDim.x * (kTriBlock / 64);
    for (int64_t q = (int64_t)blockIdx.x * (kTriBlock / 64) + (threadIdx.x >> 6); q < nu; q += nwaves) {
        const int64_t u = us[q];
        const int64_t b = off[u];
        const int d = (int)(off[u + 1] - b);
#pragma unroll
        for (int k = 0; k < kSmallSlots / 64; ++k) W.hk[lane + 64 * k] = kEmpty;
        if (lane < (1 << kSmallBloomBits) / 32) W.bf[lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t lf = 0, lb = 0;
        if (lane < d) {
            const uint32_t word = tg[b + lane], v = tid(word, tc);
            const uint64_t pv = tpay(word, tc, ov, b + lane);
            const uint4 vr = vrec[v];
            const uint32_t dv = vr.w, f0 = vr.x, b0 = vr.y;
            const bool skip = vmt > 0 && dv >= (uint32_t)vmt && (uint32_t)lane < dv;  // v-mode takes u -> v
            const uint32_t kf = (uint32_t)(pv >> 32), kb = (uint32_t)pv;
            lf = skip || !kf ? 0u : vr.z & 0xFFFFu;
            lb = skip || !kb ? 0u : vr.z >> 16;
            W.vl[lane] = v;
            W.vp[lane] = pv;
            W.lo[lane] = f0;
            W.ln[lane] = lf;
            W.kq[lane] = kf;
            W.lo[64 + lane] = b0;
            W.ln[64 + lane] = lb;
            W.kq[64 + lane] = kb;
            hinsert(W.hk, W.hi, 9, v, v, (uint32_t)lane);
            bset(W.bf, kSmallBloomBits, v);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        auto hit = [&](int l, uint32_t word, int sl) {
            const bool bl = l >= 64;
            const uint64_t m = split_m(word, tc, bl, tg, ov, off, W.vl[l & 63]);
            acc += (unsigned long long)W.kq[l] * m * split_field(W.vp[W.hi[sl]], bl);
        };
        // lists of <= 64 / <= 128 entries four / two per pass (16 / 32 lanes, 4 loads each)
        auto grouped = [&](uint64_t mask, int sgl, int ko) {
            const int per = 64 >> sgl, sg = 1 << sgl, g = lane >> sgl, e = lane & (sg - 1);
            while (mask) {  // wave-uniform
                uint64_t m = mask;
                for (int i = 0; i < g; ++i) m &= m - 1;
                const bool live = m != 0;
                const int l = __builtin_ctzll(live ? m : mask) + ko;
                for (int i = 0; i < per; ++i) mask &= mask - 1;
                const uint32_t lo = W.lo[l];
                const uint32_t dvk = live ? W.ln[l] : 0u, last = (dvk ? dvk : 1u) - 1u;
                uint32_t w[4], word[4], bit[4], keep = 0;
#pragma unroll
                for (int t = 0; t < 4; ++t) w[t] = tgs[(int64_t)lo + min((uint32_t)(e + sg * t), last)];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    bit[t] = bbit(tid(w[t], tc), kSmallBloomBits);
                    word[t] = W.bf[bit[t] >> 5];
                }
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    keep |= ((uint32_t)((uint32_t)(e + sg * t) < dvk) & (word[t] >> (bit[t] & 31))) << t;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (!((keep >> t) & 1u)) continue;
                    const int sl = hfind(W.hk, 9, tid(w[t], tc), ~0u);
                    if (sl >= 0) hit(l, w[t], sl);
                }
            }
        };
        auto longs = [&](uint64_t lm, int ko) {
            while (lm) {  // wave-uniform
                const int l = __builtin_ctzll(lm) + ko;
                lm &= lm - 1;
                const int64_t lo = (int64_t)__builtin_amdgcn_readfirstlane(W.lo[l]);
                const uint32_t dvk = __builtin_amdgcn_readfirstlane(W.ln[l]);
                for (int j0 = lane; j0 < (int)dvk; j0 += U * 64) {
                    uint32_t w[U], keep;
                    list_pass<U>(tgs, tc, lo, (int)dvk, j0, W.bf, kSmallBloomBits, w, keep);
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        if (!((keep >> r) & 1u)) continue;
                        const int sl = hfind(W.hk, 9, tid(w[r], tc), ~0u);
                        if (sl >= 0) hit(l, w[r], sl);
                    }
                }
            }
        };
        grouped(__ballot(lf > 0u && lf <= 64u), 4, 0);
        grouped(__ballot(lb > 0u && lb <= 64u), 4, 64);
        grouped(__ballot(lf > 64u && lf <= 128u), 5, 0);
        grouped(__ballot(lb > 64u && lb <= 128u), 5, 64);
        longs(__ballot(lf > 128u), 0);
        longs(__ballot(lb > 128u), 64);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the wave's LDS is reused for the next u
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (lane == 0 && acc) atomicAdd(out, acc);
}

// Items over the split lists: a chunk holds EC edges, i.e. 2 EC lists (2e: f, 2e + 1: b), and an item
// walks 2048 / EC chunks -- the same kVChunk * kVGroup edges per item as k_tri_big_items.  EC = 256 for
// 1024-lane items (half the chunk setups: each is a dependent key -> record load), 128 for 512-lane ones
// (four per CU: their LDS holds 128-edge tables only)
__host__ __device__ constexpr int sp_edges(int b) { return b == 1024 ? kVChunk : kVChunk / 2; }

template <int B, int EC>
struct ItemLdsSp {
    static constexpr int kChunk = 2 * B, kSlots = 4 * kChunk, NL = 2 * EC;
    uint32_t bf[(1 << kBigBloomBits) / 32];
    uint32_t hk[kSlots];
    uint16_t hi[kSlots];
    uint32_t lo[NL];  // list l: tgs[lo, lo + ln), constant factor kq
    uint32_t ln[NL];
    uint32_t kq[NL];
    uint32_t vl[EC];  // the lists' owner: v (u-mode) / u (v-mode)
    uint16_t lk[NL], sk[NL], mk[NL];  // long / short / medium lists
    uint32_t ncnt[6];
    unsigned long long item;
};

// k_tri_big_items over the split lists.  u-mode: the lists of edge u -> v are out_f(v) (when
// m(u,v) >= 1; factor m(u,v)) and out_b(v) (m(v,u)); v-mode (center c, in-edge u -> c): the prefixes of
// out_f(u) (factor m(c,u)) and out_b(u) (factor m(u,c)) below c, of lengths pf / pb from ipos.
template <int U, bool VM, int B, int EC = sp_edges(B), int EPI = kVChunk * kVGroup, int SG = kSG>
__global__ void __launch_bounds__(B, 8) k_tri_items_sp(const uint32_t* __restrict__ tg, TgCode tc,
                                                        const int64_t* __restrict__ ov,
                                                        const int64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ tgs,
                                                        const uint4* __restrict__ vrec,
                                                        const int64_t* __restrict__ ioff,
                                                        const uint64_t* __restrict__ ikey,
                                                        const uint4* __restrict__ irec, int vmt,
                                                        const int64_t* __restrict__ us, int64_t total,
                                                        const uint64_t* __restrict__ item_ql,
                                                        unsigned long long* __restrict__ ctr,
                                                        unsigned long long* __restrict__ out) {
    constexpr int VG = EPI / EC;  // chunks per item
    extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
    ItemLdsSp<B, EC>& L = *reinterpret_cast<ItemLdsSp<B, EC>*>(lds_raw);
    constexpr int CH = ItemLdsSp<B, EC>::kChunk;
    unsigned long long& item = L.item;
    unsigned long long acc = 0;
    while (true) {
        if (threadIdx.x == 0) item = atomicAdd(ctr, 1ULL);
        __syncthreads();
        const int64_t it = (int64_t)item;
        __syncthreads();  // `item` is rewritten next round
        if (it >= total) break;  // block-uniform
        const uint64_t iw = item_ql[it];
        const int64_t c = us[(uint32_t)iw], b = uniform64(off[c]);  // the center (u-mode: u; v-mode: v)
        const int d = (int)(off[c + 1] - b);
        const int64_t nb = VM ? uniform64(ioff[c]) : b;  // its neighbour list: in(v) / out(u)
        const int nd = VM ? (int)(ioff[c + 1] - nb) : d;
        const int nvc = (nd + EC - 1) / EC, ngr = (nvc + VG - 1) / VG;
        const int local = (int)(iw >> 32);
        const int h0 = (local / ngr) * CH, c0 = (local % ngr) * VG, c1 = min(nvc, c0 + VG);
        const int hn = min(CH, d - h0);
        int lc = 6;  // hash capacity 2^lc >= 4 hn (load <= 1/4), cleared as far as it is used
        while ((1 << lc) < 4 * hn) ++lc;
        for (int k = threadIdx.x; k < (1 << lc); k += B) L.hk[k] = kEmpty;
        for (int k = threadIdx.x; k < (1 << kBigBloomBits) / 32; k += B) L.bf[k] = 0;
        if (threadIdx.x < 6) L.ncnt[threadIdx.x] = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < hn; k += B) {
            const uint32_t word = tg[b + h0 + k], w = tid(word, tc);
            hinsert(L.hk, L.hi, lc, w, word, (uint32_t)k);
            bset(L.bf, kBigBloomBits, w);
        }
        for (int ch = c0; ch < c1; ++ch) {  // block-uniform
            const int v0 = ch * EC, vn = min(EC, nd - v0);
            if (ch > c0) __syncthreads();  // the previous chunk's walks are done with the list table
            uint32_t* nc = L.ncnt + 3 * (ch & 1);
            if (threadIdx.x < 3) L.ncnt[3 * ((ch + 1) & 1) + threadIdx.x] = 0;  // read last by chunk ch - 1
            for (int k = threadIdx.x; k < vn; k += B) {
                uint32_t x, f0, b0, lf, lb, kf, kb;
                if (VM) {  // in-edge x -> c: prefixes of out_f(x) / out_b(x) below c
                    const uint4 r = irec[ikey[nb + v0 + k] & kInRecMask];
                    const uint32_t word = r.x;
                    x = tid(word, tc);
                    const uint32_t fc = (word >> tc.ib) & tc.cmask(), bc = (word >> (tc.ib + tc.cb)) & tc.cmask();
                    uint64_t p = (uint64_t)fc << 32 | bc;
                    if (fc == tc.cmask() || bc == tc.cmask()) p = exact_pay(tg, tc, ov, off, x, (uint32_t)c);
                    kf = (uint32_t)p;           // m(c, x)
                    kb = (uint32_t)(p >> 32);   // m(x, c)
                    const uint32_t ip = r.y;
                    f0 = r.z;
                    b0 = r.w;
                    lf = kf ? ip & 0xFFFFu : 0u;
                    lb = kb ? ip >> 16 : 0u;
                } else {  // out-edge c -> x: out_f(x) / out_b(x) unless v-mode takes the edge
                    const uint32_t word = tg[b + v0 + k];
                    x = tid(word, tc);
                    const uint64_t p = tpay(word, tc, ov, b + v0 + k);
                    kf = (uint32_t)(p >> 32);   // m(c, x)
                    kb = (uint32_t)p;           // m(x, c)
                    const uint4 vr = vrec[x];
                    const uint32_t dv = vr.w;
                    const bool skip = vmt > 0 && dv >= (uint32_t)vmt && (uint32_t)(v0 + k) < dv;
                    f0 = vr.x;
                    b0 = vr.y;
                    lf = skip || !kf ? 0u : vr.z & 0xFFFFu;
                    lb = skip || !kb ? 0u : vr.z >> 16;
                }
                L.vl[k] = x;
                L.lo[2 * k] = f0;
                L.ln[2 * k] = lf;
                L.kq[2 * k] = kf;
                L.lo[2 * k + 1] = b0;
                L.ln[2 * k + 1] = lb;
                L.kq[2 * k + 1] = kb;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const uint32_t dw = t ? lb : lf;
                    const uint16_t l = (uint16_t)(2 * k + t);
                    if (dw > 8u * SG) L.lk[atomicAdd(&nc[0], 1u)] = l;
                    else if (dw > 4u * SG) L.mk[atomicAdd(&nc[2], 1u)] = l;
                    else if (dw > 0u) L.sk[atomicAdd(&nc[1], 1u)] = l;
                }
            }
            __syncthreads();
            const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
            const int nlong = (int)__builtin_amdgcn_readfirstlane(nc[0]);
            const int nshort = (int)__builtin_amdgcn_readfirstlane(nc[1]);
            const int nmed = (int)__builtin_amdgcn_readfirstlane(nc[2]);
            auto hit = [&](int l, uint32_t word, int sl) {
                const bool bl = l & 1;
                const uint64_t m = split_m(word, tc, bl, tg, ov, off, L.vl[l >> 1]);
                const uint64_t pcw = tpay(L.hk[sl], tc, ov, b + h0 + L.hi[sl]);
                acc += (unsigned long long)L.kq[l] * m * split_field(pcw, bl);
            };
            auto grouped = [&](const uint16_t* ks, int nk, int sgl) {
                const int per = 64 >> sgl, sg = 1 << sgl;
                for (int q0 = wave * per; q0 < nk; q0 += (B / 64) * per) {
                    const int g = lane >> sgl, e = lane & (sg - 1);
                    const bool live = q0 + g < nk;
                    const int l = ks[live ? q0 + g : q0];
                    const uint32_t lo = L.lo[l];
                    const uint32_t dvk = live ? L.ln[l] : 0u, last = (dvk ? dvk : 1u) - 1u;
                    uint32_t w[4], word[4], bit[4], keep = 0;
#pragma unroll
                    for (int t = 0; t < 4; ++t) w[t] = tgs[(int64_t)lo + min((uint32_t)(e + sg * t), last)];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        bit[t] = bbit(tid(w[t], tc), kBigBloomBits);
                        word[t] = L.bf[bit[t] >> 5];
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        keep |= ((uint32_t)((uint32_t)(e + sg * t) < dvk) & (word[t] >> (bit[t] & 31))) << t;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        if (!((keep >> t) & 1u)) continue;
                        const int sl = hfind(L.hk, lc, tid(w[t], tc), tc.idmask());
                        if (sl >= 0) hit(l, w[t], sl);
                    }
                }
            };
            grouped(L.sk, nshort, SG == 8 ? 3 : SG == 16 ? 4 : 5);
            grouped(L.mk, nmed, SG == 8 ? 4 : SG == 16 ? 5 : 6);
            for (int q = wave; q < nlong; q += B / 64) {  // long lists: one per wave, U x 64 entries a pass
                const int l = L.lk[q];
                const int64_t lo = (int64_t)__builtin_amdgcn_readfirstlane(L.lo[l]);
                const int dv = (int)__builtin_amdgcn_readfirstlane(L.ln[l]);
                for (int j0 = lane; j0 < dv; j0 += U * 64) {
                    uint32_t w[U], keep;
                    list_pass<U>(tgs, tc, lo, dv, j0, L.bf, kBigBloomBits, w, keep);
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        if (!((keep >> r) & 1u)) continue;
                        const int sl = hfind(L.hk, lc, tid(w[r], tc), tc.idmask());
                        if (sl >= 0) hit(l, w[r], sl);
                    }
                }
            }
        }
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// u with 2 <= out-degree: small (<= 64) and big lists; also the 4-byte target array
__global__ void k_tri_bins(const int64_t* __restrict__ off, int64_t n, uint8_t* __restrict__ fs,
                           uint8_t* __restrict__ fb) {
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n; u += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = off[u + 1] - off[u];
        fs[u] = d >= 2 && d <= kSmallDeg;
        fb[u] = d > kSmallDeg;
    }
}

__global__ void k_targets(const uint64_t* __restrict__ ok_, int64_t ne, uint32_t* __restrict__ tg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x)
        tg[i] = (uint32_t)ok_[i];
}


// pair and self terms
__global__ void k_pair_terms(const uint64_t* __restrict__ ek, const int64_t* __restrict__ ev, int64_t ne,
                             const uint32_t* __restrict__ sl, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = (uint64_t)ev[i];
        if ((v >> 32) == 0 || (v & 0xffffffffULL) == 0) continue;  // one direction only: no term, no gathers
        const uint32_t x = (uint32_t)(ek[i] >> 32), y = (uint32_t)ek[i];
        acc += 3ULL * ((uint64_t)sl[x] + sl[y]) * (v >> 32) * (v & 0xffffffffULL);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

__global__ void k_self_terms(const uint32_t* __restrict__ sl, int64_t n, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s = sl[i];
        if (s >= 3) acc += s * (s - 1) * (s - 2);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// ---- the distributed build (multi-GPU C4) --------------------------------------------------------
// destination of an undirected key: the owner of its lower end, which then holds every relationship of
// the pair (kNone: dropped, not sent)
__global__ void k_tri_dest_min(const uint64_t* __restrict__ key, int64_t m, int64_t span, int world,
                               uint64_t* __restrict__ dest) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[i];
        const int64_t q = k == kNone ? 0xFF : (int64_t)(k >> 32) / span;
        dest[i] = (uint64_t)(k == kNone ? 0xFF : (q < world ? q : world - 1));
    }
}

constexpr int kHistBins = 4096;

// coarse histogram of the oriented keys' sources (degree-order id >> hb)
__global__ void k_tri_from_hist(const uint64_t* __restrict__ ok_, int64_t ne, int hb,
                                unsigned long long* __restrict__ hist) {
    __shared__ unsigned int h[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) h[b] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x)
        if (ok_[i] != kNone) atomicAdd(&h[(uint32_t)(ok_[i] >> 32) >> hb], 1u);  // (kNone: a dropped relationship)
    __syncthreads();
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        if (h[b]) atomicAdd(&hist[b], (unsigned long long)h[b]);
}

// destination of an oriented key: the rank whose range of source bins [bbeg[q], bbeg[q + 1]) holds it
__global__ void k_tri_dest_from(const uint64_t* __restrict__ ok_, int64_t ne, int hb, const int64_t* __restrict__ bbeg,
                                int world, uint64_t* __restrict__ dest) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        if (ok_[i] == kNone) {  // dropped, not sent
            dest[i] = 0xFF;
            continue;
        }
        const int64_t bin = (int64_t)((uint32_t)(ok_[i] >> 32) >> hb);
        int a = 0, b = world - 1;  // the last q with bbeg[q] <= bin
        while (a < b) {
            const int mid = (a + b + 1) >> 1;
            if (bbeg[mid] <= bin) a = mid; else b = mid - 1;
        }
        dest[i] = (uint64_t)a;
    }
}

// ---- v-mode shares without replicated in-lists (distributed build) -----------------------------------
// the edges whose in-list entry this rank's v-mode share walks: v mod world = rank, od(v) >= vmt, p < od(v)
__global__ void k_tri_in_flags(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ off, int64_t ne,
                               uint32_t idm, int vmt, int world, int rank, uint8_t* __restrict__ f) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = ok_[e];
        const uint32_t u = (uint32_t)(k >> 32), v = (uint32_t)k & idm;
        bool take = false;
        if ((int)(v % (uint32_t)world) == rank) {
            const int64_t odv = off[v + 1] - off[v];
            take = odv >= vmt && e - off[u] < odv;
        }
        f[e] = take ? 1 : 0;
    }
}

// packed in-keys (to << (ib + 16) | from << 16 | pos) of the selected edges, in edge order
__global__ void k_swap_keys_sel(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ off,
                                const int64_t* __restrict__ sel, int64_t nsel, TgCode tc, uint64_t* __restrict__ ik) {
    const uint32_t idm = tc.idmask();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nsel; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = sel[i];
        const uint64_t k = ok_[e];
        const uint64_t from = k >> 32, to = (uint32_t)k & idm;
        ik[i] = (to << (tc.ib + 16)) | (from << 16) | (uint64_t)(e - off[from]);
    }
}

// every parts-th center from `part`
__global__ void k_tri_stride(const int64_t* __restrict__ cs, int part, int parts, int64_t cnt, int64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += (int64_t)gridDim.x * blockDim.x)
        out[k] = cs[part + k * (int64_t)parts];
}

inline int grid(const capsmi_session* s, int64_t n) {
    int64_t g = (n + 255) / 256;
    const int64_t cap = (int64_t)s->num_cus * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

inline int bits_for(uint64_t range) {
    int b = 1;
    while (b < 32 && (uint64_t(1) << b) < range) ++b;
    return b;
}

}  // namespace tri

namespace tri {
// A distributed build's exchange of oriented keys (source in bits 32+): each key to the rank of its source's
// degree-order range, the ranges made of coarse source bins balanced by their all-reduced key counts, so a
// source's whole list meets on one rank; returns this rank's keys (*nout of them)
Buf to_source_range_owner(capsmi_session* s, const Buf& keys, int64_t nk, int bits, int64_t n, int W, int64_t* nout) {
    hipStream_t st = s->stream;
    const int hb = bits > 12 ? bits - 12 : 0;
    const int64_t nbins = ((n - 1) >> hb) + 1;
    Buf hist = dev_alloc(sizeof(int64_t) * (kHistBins + W + 1), s);
    HIP_CHECK(hipMemsetAsync(P<void>(hist), 0, sizeof(int64_t) * kHistBins, st));
    if (nk > 0)
        hipLaunchKernelGGL(k_tri_from_hist, dim3(std::min(grid(s, nk), 4 * s->num_cus)), dim3(1024), 0, st,
                           P<uint64_t>(keys), nk, hb, P<unsigned long long>(hist));
    HIP_CHECK(hipGetLastError());
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(hist), P<int64_t>(hist), kHistBins, CAPSMI_I64);
    std::vector<int64_t> h(kHistBins), bb(W + 1);
    HIP_CHECK(hipMemcpyAsync(h.data(), P<int64_t>(hist), sizeof(int64_t) * kHistBins, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t tot = 0;
    for (int64_t b = 0; b < nbins; ++b) tot += h[b];
    int64_t cum = 0, b = 0;
    bb[0] = 0;
    for (int q = 1; q < W; ++q) {
        const int64_t want = tot * q / W;
        while (b < nbins && cum + h[b] <= want) cum += h[b++];
        bb[q] = b;
    }
    bb[W] = nbins;
    int64_t* bbeg = P<int64_t>(hist) + kHistBins;
    HIP_CHECK(hipMemcpyAsync(bbeg, bb.data(), sizeof(int64_t) * (W + 1), hipMemcpyHostToDevice, st));
    Buf dest = dev_alloc(sizeof(uint64_t) * (nk > 0 ? nk : 1), s);
    if (nk > 0)
        hipLaunchKernelGGL(k_tri_dest_from, dim3(grid(s, nk)), dim3(256), 0, st, P<uint64_t>(keys), nk, hb, bbeg, W,
                           P<uint64_t>(dest));
    HIP_CHECK(hipGetLastError());
    return exchange_words(s, P<uint64_t>(dest), P<uint64_t>(keys), nk, nout);
}
}  // namespace tri

// Distributed (dd != null, multi-GPU C4): every rank builds from its 1/world of the
// relationships and ends with the same replicated oriented graph.  The undirected keys go to the owner of
// their lower end (one exchange), so each rank sorts 1/world of them and holds every relationship of its
// pairs (exact multiplicities); degrees and self-loop counts are summed over the ranks; each rank orients
// its pairs, sends the oriented keys to the rank of their source's degree-order range (ranges balanced by
// a coarse all-reduced histogram), sorts its range, and one all-gather in rank order concatenates the
// sorted ranges into the whole sorted key array.  The in-lists and bins are then built from it on every
// rank (replicated), with per-center work estimates for tri_count's balanced shares.
void tri_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
               const capsmi_bitmap* n_ok, TriGraph& g, const TriDist* dd) {
    using namespace tri;
    hipStream_t st = s->stream;
    const int64_t lo = n_ok->lo, hi = n_ok->hi, n = hi - lo;
    REQUIRE(n > 0 && (uint64_t)n <= (uint64_t(1) << 31), CAPSMI_ERR_UNSUPPORTED, "triangle count needs <= 2^31 ids");
    g.lo = lo;
    g.n = n;
    g.dist = dd != nullptr;
    int64_t m = 0;
    for (int i = 0; i < nt; ++i) m += ms[i];
    const int bits = bits_for((uint64_t)n);
    REQUIRE(!dd || (bits + 7) / 8 * 8 <= 24, CAPSMI_ERR_UNSUPPORTED,
            "distributed triangle count: at most 2^24 ids (coded oriented keys)");
    REQUIRE(!dd || dd->world < 255, CAPSMI_ERR_UNSUPPORTED, "distributed triangle count: at most 254 ranks (exchanges)");
    int64_t m_all = m;  // every rank's relationships (bounds the out-degrees below)
    if (dd) {
        Buf t = dev_alloc(sizeof(int64_t), s);
        fill_i64(P<int64_t>(t), m, 1, st);
        collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(t), P<int64_t>(t), 1, CAPSMI_I64);
        m_all = read_scalar(s, P<int64_t>(t));
    }
    // coded targets: the ids' sorted digits end at ib = 8 * ceil(bits / 8); with ib <= 24 the two
    // 4-bit multiplicity fields fit above them
    g.ib = (bits + 7) / 8 * 8;
    g.cb = g.ib <= 24 ? 4 : 0;
    const TgCode tc{(uint32_t)g.ib, (uint32_t)g.cb};
    std::vector<int> od;  // (source, target): grouped and target-sorted lists
    for (int sh = 0; sh < bits; sh += 8) od.push_back(sh);
    for (int sh = 32; sh < 32 + bits; sh += 8) od.push_back(sh);
    Buf nv = dev_alloc(sizeof(int64_t) + sizeof(unsigned long long), s);  // nvalid, long-run count (then nexc)
    HIP_CHECK(hipMemsetAsync(P<void>(nv), 0, sizeof(int64_t) + sizeof(unsigned long long), st));
    int64_t* nvalid_p = P<int64_t>(nv);
    unsigned long long* nlong = reinterpret_cast<unsigned long long*>(nvalid_p + 1);
    Buf exc;
    Buf maxod;  // the largest out-degree (u64), when the offsets pass found it
    int64_t ne = 0;
    std::unique_ptr<KernelTimer> ph;
    // the direct oriented build ("the direct oriented build" above) for ids <= 2^24; config
    // CAPSMI_TRI_BUILD=sorted: the undirected sort, orientation and oriented sort (the build above 2^24 ids)
    const bool direct = bits <= 24 && !s->cfg.tri_sorted_build;
    if (direct) {
        ph.reset(new KernelTimer(s, "tri_deg"));
        Buf deg = dev_alloc(sizeof(uint32_t) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(deg), 0, sizeof(uint32_t) * n, st));
        // sampled degrees: 1 in 32 relationships above 2^22 (config CAPSMI_TRI_DEG_SAMPLE = a power of two, 1 = all).
        // At C4 (2^28): all of them took 20 ms of atomics (hubs' counters) and the walks 53.6 ms; 1 in 16 / 64
        // ≈ 1 ms, walks 54.2 ms
        int rate = s->cfg.tri_deg_sample > 0 ? s->cfg.tri_deg_sample : (m_all > (int64_t(1) << 22) ? 32 : 1);
        while (rate & (rate - 1)) rate &= rate - 1;
        {
            int64_t e0 = 0;
            for (int i = 0; i < nt; ++i) {
                if (ms[i] > 0)
                    hipLaunchKernelGGL(k_deg_sample, dim3(std::min(grid(s, ms[i] / rate + 1), 4 * s->num_cus)), dim3(256),
                                       0, st, srcs[i], dsts[i], ms[i], e0, lo, hi, P<uint32_t>(n_ok->words),
                                       n_ok->full ? 1 : 0, (uint32_t)rate, P<uint32_t>(deg));
                e0 += ms[i];
            }
            HIP_CHECK(hipGetLastError());
        }
        ph.reset();
        if (dd) collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<uint32_t>(deg), P<uint32_t>(deg), n, CAPSMI_COLL_U32);
        ph.reset(new KernelTimer(s, "tri_order"));
        Buf rid = dev_alloc(sizeof(uint32_t) * n, s);
        g.orig = dev_alloc(sizeof(int64_t) * n, s);
        {
            Buf dk = dev_alloc(sizeof(uint64_t) * n, s), dm = dev_alloc(sizeof(int64_t), s);
            HIP_CHECK(hipMemsetAsync(P<void>(dm), 0, sizeof(int64_t), st));
            hipLaunchKernelGGL(k_deg_keys, dim3(grid(s, n)), dim3(256), 0, st, P<uint32_t>(deg), n, P<uint64_t>(dk),
                               reinterpret_cast<unsigned int*>(P<int64_t>(dm)));
            const uint64_t dmax = (uint64_t)read_scalar(s, P<int64_t>(dm));
            std::vector<int> dg;
            for (int sh = 32; sh < 64 && (dmax >> (sh - 32)) != 0; sh += 8) dg.push_back(sh);
            radix_sort_digits(s, P<uint64_t>(dk), nullptr, n, dg);
            hipLaunchKernelGGL(k_rank_ids, dim3(grid(s, n)), dim3(256), 0, st, P<uint64_t>(dk), n, P<uint32_t>(rid),
                               P<int64_t>(g.orig));
        }
        deg.reset();
        ph.reset(new KernelTimer(s, "tri_pack"));
        Buf sl0 = dev_alloc(sizeof(uint32_t) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(sl0), 0, sizeof(uint32_t) * n, st));
        Buf key = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
        Buf h0;  // one table on one device: the sort's first-digit tile counts, written with the keys
        if (nt == 1 && !dd && m > 1) {
            const int64_t ntl = (m + kSortTile - 1) / kSortTile;
            h0 = dev_alloc(sizeof(int64_t) * 256 * ntl, s);
            hipLaunchKernelGGL(k_pack_or<true>, dim3((unsigned)std::min<int64_t>(ntl, (int64_t)s->num_cus * 16)), dim3(256),
                               0, st, srcs[0], dsts[0], m, lo, hi, P<uint32_t>(n_ok->words), n_ok->full ? 1 : 0,
                               P<uint32_t>(rid), P<uint64_t>(key), P<uint32_t>(sl0), P<int64_t>(h0), od[0]);
            HIP_CHECK(hipGetLastError());
        } else {
            int64_t off = 0;
            for (int i = 0; i < nt; ++i) {
                if (ms[i] > 0)
                    hipLaunchKernelGGL(k_pack_or<false>, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i],
                                       lo, hi, P<uint32_t>(n_ok->words), n_ok->full ? 1 : 0, P<uint32_t>(rid),
                                       P<uint64_t>(key) + off, P<uint32_t>(sl0), (int64_t*)nullptr, 0);
                off += ms[i];
            }
            HIP_CHECK(hipGetLastError());
        }
        ph.reset();
        rid.reset();
        if (dd) collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<uint32_t>(sl0), P<uint32_t>(sl0), n, CAPSMI_COLL_U32);
        g.sl = dev_alloc(sizeof(uint32_t) * n, s);  // in degree-order ids, as the pair terms' keys
        hipLaunchKernelGGL(k_perm_u32, dim3(grid(s, n)), dim3(256), 0, st, P<uint32_t>(sl0), P<int64_t>(g.orig), n,
                           P<uint32_t>(g.sl));
        sl0.reset();
        if (dd) {
            // every relationship to the rank of its source's degree-order range (ranges balanced by the
            // all-reduced counts of a coarse source histogram): a pair's relationships meet on one rank
            int64_t mr = 0;
            key = to_source_range_owner(s, key, m, bits, n, dd->world, &mr);
            m = mr;
        }
        // one sort of the raw oriented keys (the direction bit unsorted at bit 31), runs = the pairs
        ph.reset(new KernelTimer(s, "tri_sort_or"));
        radix_sort_keys(s, key, m, od, P<int64_t>(h0));
        h0.reset();
        // the runs: tile head counts, their scan, then every pair's outputs (k_or_write; the fused run passes
        // replaced head flags + compaction + k_und_runs + k_orient + k_targets + k_pair_terms, 6.1 ms at C4)
        const int64_t ntl = (m + kOrTile - 1) / kOrTile;
        int64_t nruns = 0;
        Buf pre = dev_alloc(sizeof(int64_t) * (ntl + 1), s);
        if (ntl > 0) {
            Buf cnt = dev_alloc(sizeof(int64_t) * ntl, s);
            hipLaunchKernelGGL(k_or_count, dim3((unsigned)ntl), dim3(kOrB), 0, st, P<uint64_t>(key), m, P<int64_t>(cnt));
            HIP_CHECK(hipGetLastError());
            exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(pre), ntl, s);
            nruns = read_scalar(s, P<int64_t>(pre) + ntl);
        }
        g.ok = dev_alloc(sizeof(uint64_t) * (nruns > 0 ? nruns : 1), s);
        g.ov = dev_alloc(sizeof(int64_t) * (nruns > 0 ? nruns : 1), s);
        if (!dd) g.tg = dev_alloc(sizeof(uint32_t) * (nruns > 0 ? nruns : 1), s);
        exc = dev_alloc(sizeof(uint64_t) * 2 * (dd && nruns > 0 ? nruns : 1), s);
        g.pair = dev_alloc(sizeof(int64_t), s);
        HIP_CHECK(hipMemsetAsync(P<void>(g.pair), 0, sizeof(int64_t), st));
        HIP_CHECK(hipMemsetAsync(P<void>(nv), 0, sizeof(int64_t) + sizeof(unsigned long long), st));  // nexc, nlong
        if (!dd) {  // one device: the CSR offsets from the run heads (k_or_write), see k_sufmin_apply
            g.off = dev_alloc(sizeof(int64_t) * (n + 1), s);
            fill_i64(P<int64_t>(g.off), INT64_MAX, n, st);
            fill_i64(P<int64_t>(g.off) + n, nruns, 1, st);
        }
        if (nruns > 0) {
            Buf longr = dev_alloc(sizeof(int64_t) * 2 * (m / kShortRun + 1), s);
            Buf pp = dev_alloc(sizeof(int64_t) * (ntl + 1), s), ps = dev_alloc(sizeof(int64_t) * (ntl + 2), s);
            HIP_CHECK(hipMemsetAsync(P<int64_t>(pp) + ntl, 0, sizeof(int64_t), st));
            // one device: the exceptions' payloads go straight to ov (the keys stay where they are written)
            OrOut o{P<uint64_t>(g.ok), P<uint32_t>(g.tg), P<int64_t>(g.ov), dd ? P<uint64_t>(exc) : nullptr, nlong,
                    P<int64_t>(longr), reinterpret_cast<unsigned long long*>(nvalid_p), P<uint32_t>(g.sl), P<int64_t>(pp),
                    P<int64_t>(g.off)};
            hipLaunchKernelGGL(k_or_write, dim3((unsigned)ntl), dim3(kOrB), 0, st, P<uint64_t>(key), m, P<int64_t>(pre),
                               tc, o);
            hipLaunchKernelGGL(k_or_long, dim3(4 * s->num_cus), dim3(256), 0, st, P<uint64_t>(key), m, ntl, tc, o);
            HIP_CHECK(hipGetLastError());
            exclusive_scan_i64(P<int64_t>(pp), P<int64_t>(ps), ntl + 1, s);
            HIP_CHECK(hipMemcpyAsync(P<void>(g.pair), P<int64_t>(ps) + ntl + 1, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
        }
        if (!dd) {
            const int64_t n1 = n + 1, nst = (n1 + kSmTile - 1) / kSmTile;
            Buf tm = dev_alloc(sizeof(int64_t) * nst, s);
            maxod = dev_alloc(sizeof(unsigned long long), s);
            HIP_CHECK(hipMemsetAsync(P<void>(maxod), 0, sizeof(unsigned long long), st));
            hipLaunchKernelGGL(k_sufmin_tiles, dim3((unsigned)nst), dim3(kSmB), 0, st, P<int64_t>(g.off), n1, P<int64_t>(tm));
            hipLaunchKernelGGL(k_sufmin_carry, dim3(1), dim3(1024), 0, st, P<int64_t>(tm), nst);
            hipLaunchKernelGGL(k_sufmin_apply, dim3((unsigned)nst), dim3(kSmB), 0, st, P<int64_t>(g.off), n1, P<int64_t>(tm),
                               P<unsigned long long>(maxod));
            HIP_CHECK(hipGetLastError());
        }
        key.reset();
        g.nek = 0;  // the pair terms are in g.pair
        ne = nruns;
        ph.reset();
        if (dd) {  // the ranges in rank order (sorted), every rank's exceptions
            const int64_t nexc = (int64_t)read_scalar(s, reinterpret_cast<const int64_t*>(nlong));
            int64_t nexc_all = 0;
            exc = gather_words(s, P<uint64_t>(exc), 2 * nexc, &nexc_all);
            fill_i64(reinterpret_cast<int64_t*>(nlong), nexc_all / 2, 1, st);
            g.ok = gather_words(s, P<uint64_t>(g.ok), nruns, &ne);
            g.ov = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), s);
        }
    } else {
        // the direction bit rides unsorted at bit 31 when max's digits end at or below bit 24
        const int msh = bits > 24 ? 1 : 0;
        g.sl = dev_alloc(sizeof(uint32_t) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(g.sl), 0, sizeof(uint32_t) * n, st));
        Buf key = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
        {
            KernelTimer kt(s, "tri_pack");
            int64_t off = 0;
            for (int i = 0; i < nt; ++i) {
                if (ms[i] > 0)
                    hipLaunchKernelGGL(k_pack, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, hi,
                                       P<uint32_t>(n_ok->words), n_ok->full ? 1 : 0, msh, P<uint64_t>(key) + off,
                                       P<uint32_t>(g.sl));
                off += ms[i];
            }
        }
        if (dd) {  // every relationship of a pair to the owner of the pair's lower end
            Buf dest = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
            if (m > 0)
                hipLaunchKernelGGL(k_tri_dest_min, dim3(grid(s, m)), dim3(256), 0, st, P<uint64_t>(key), m, dd->span,
                                   dd->world, P<uint64_t>(dest));
            HIP_CHECK(hipGetLastError());
            int64_t mr = 0;
            key = exchange_words(s, P<uint64_t>(dest), P<uint64_t>(key), m, &mr);
            m = mr;
        }
        // build phases timed on the device (pure device work between the exchanges; bench kernel_ms)
        ph.reset(new KernelTimer(s, "tri_sort_und"));
        // one sort of the undirected keys: digits of max (and the direction bit when msh) then of min; the
        // upper ends' degrees are counted between the two halves, while the keys are in max order
        Buf deg = dev_alloc(sizeof(uint32_t) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(deg), 0, sizeof(uint32_t) * n, st));
        std::vector<int> kd;
        for (int sh = 0; sh < bits + msh; sh += 8) kd.push_back(sh);
        const int nmax = (int)kd.size();
        for (int sh = 32; sh < 32 + bits; sh += 8) kd.push_back(sh);
        radix_sort_digits(s, P<uint64_t>(key), nullptr, m, kd, nmax, [&](const uint64_t* kmax) {
            if (m > 0)
                hipLaunchKernelGGL(k_deg_max, dim3(grid(s, m)), dim3(256), 0, st, kmax, m, msh, P<uint32_t>(deg));
        });
        const uint64_t dmask = msh ? ~1ULL : ~(1ULL << 31);
        Buf f = dev_alloc(m > 0 ? m : 1, s), heads;
        hipLaunchKernelGGL(k_heads, dim3(grid(s, m)), dim3(256), 0, st, P<uint64_t>(key), m, dmask, P<uint8_t>(f));
        ne = flags_to_indices(s, P<uint8_t>(f), m, heads);
        hipLaunchKernelGGL(k_first_none, dim3(1), dim3(1), 0, st, P<uint64_t>(key), m, nvalid_p);
        g.ne = ne;
        g.ek = dev_alloc(sizeof(uint64_t) * (ne > 0 ? ne : 1), s);
        g.ev = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), s);
        if (ne > 0) {
            Buf longr = dev_alloc(sizeof(int64_t) * (m / kShortRun + 1), s);
            hipLaunchKernelGGL(k_und_runs, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(key), P<int64_t>(heads), ne,
                               nvalid_p, msh, P<uint64_t>(g.ek), P<int64_t>(g.ev), P<uint32_t>(deg), P<int64_t>(longr), nlong);
            hipLaunchKernelGGL(k_und_long, dim3(4 * s->num_cus), dim3(256), 0, st, P<uint64_t>(key), P<int64_t>(heads), ne,
                               nvalid_p, msh, P<int64_t>(longr), nlong, P<int64_t>(g.ev));
            HIP_CHECK(hipGetLastError());
        }
        key.reset();
        f.reset();
        heads.reset();
        g.nek = ne;
        ph.reset();
        if (dd) {  // a pair's relationships are all on one rank: the sums over the ranks are exact
            collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<uint32_t>(deg), P<uint32_t>(deg), n, CAPSMI_COLL_U32);
            collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<uint32_t>(g.sl), P<uint32_t>(g.sl), n, CAPSMI_COLL_U32);
        }
        // degree-order ids (hubs first): sort the vertices by (degree, id)
        ph.reset(new KernelTimer(s, "tri_order"));
        Buf rid = dev_alloc(sizeof(uint32_t) * n, s);
        g.orig = dev_alloc(sizeof(int64_t) * n, s);
        {
            Buf dk = dev_alloc(sizeof(uint64_t) * n, s), dm = dev_alloc(sizeof(int64_t), s);
            HIP_CHECK(hipMemsetAsync(P<void>(dm), 0, sizeof(int64_t), st));
            hipLaunchKernelGGL(k_deg_keys, dim3(grid(s, n)), dim3(256), 0, st, P<uint32_t>(deg), n, P<uint64_t>(dk),
                               reinterpret_cast<unsigned int*>(P<int64_t>(dm)));
            const uint64_t dmax = (uint64_t)read_scalar(s, P<int64_t>(dm));
            // the keys are written in id order and the LSD sort is stable: the degree digits alone give
            // the (degree, id) order
            std::vector<int> dd;
            for (int sh = 32; sh < 64 && (dmax >> (sh - 32)) != 0; sh += 8) dd.push_back(sh);
            radix_sort_digits(s, P<uint64_t>(dk), nullptr, n, dd);
            hipLaunchKernelGGL(k_rank_ids, dim3(grid(s, n)), dim3(256), 0, st, P<uint64_t>(dk), n, P<uint32_t>(rid),
                               P<int64_t>(g.orig));
        }
        g.ok = dev_alloc(sizeof(uint64_t) * (ne > 0 ? ne : 1), s);
        g.ov = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), s);  // coded: written at the exceptions only
        exc = dev_alloc(tc.cb ? sizeof(uint64_t) * 2 * (ne > 0 ? ne : 1) : 8, s);
        HIP_CHECK(hipMemsetAsync(P<void>(nv), 0, sizeof(int64_t) + sizeof(unsigned long long), st));  // nlong reused: nexc
        if (ne > 0)
            hipLaunchKernelGGL(k_orient, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(g.ek), P<int64_t>(g.ev), ne,
                               P<uint32_t>(rid), tc, P<uint64_t>(g.ok), P<int64_t>(g.ov), P<uint64_t>(exc), nlong);
        ph.reset();
        if (dd) {
            // the exceptions' exact payloads (rare): every rank's list, for the placement in the whole key array
            const int64_t nexc = (int64_t)read_scalar(s, reinterpret_cast<const int64_t*>(nlong));
            int64_t nexc_all = 0;
            exc = gather_words(s, P<uint64_t>(exc), 2 * nexc, &nexc_all);
            fill_i64(reinterpret_cast<int64_t*>(nlong), nexc_all / 2, 1, st);
            // source ranges of coarse degree-order bins, balanced by the all-reduced bin counts
            int64_t nr = 0;
            Buf mine = to_source_range_owner(s, g.ok, ne, bits, n, dd->world, &nr);
            {
                KernelTimer kt(s, "tri_sort_or");
                radix_sort_digits(s, P<uint64_t>(mine), nullptr, nr, od);  // this rank's source range, sorted
            }
            g.ok = gather_words(s, P<uint64_t>(mine), nr, &ne);          // the ranges in rank order: all sorted
            g.ov = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), s);
        } else {
            // no kNone among the oriented keys; coded: key-only (the payloads ride in the key)
            KernelTimer kt(s, "tri_sort_or");
            radix_sort_digits(s, P<uint64_t>(g.ok), tc.cb ? nullptr : P<int64_t>(g.ov), ne, od);
        }
    }
    g.ne = ne;
    ph.reset(new KernelTimer(s, "tri_post"));
    if (tc.cb && ne > 0)
        hipLaunchKernelGGL(k_exc_place, dim3(grid(s, ne / 64 + 1)), dim3(256), 0, st, P<uint64_t>(exc), nlong,
                           P<uint64_t>(g.ok), ne, tc, P<int64_t>(g.ov));
    exc.reset();
    if (!g.off) {  // (the direct build on one device has them from the run heads)
        g.off = dev_alloc(sizeof(int64_t) * (n + 1), s);
        hipLaunchKernelGGL(k_offsets, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(g.ok), ne, n, 32,
                           P<int64_t>(g.off));
    }
    if (!g.tg) {  // (the direct build on one device wrote them with the keys)
        g.tg = dev_alloc(sizeof(uint32_t) * (ne > 0 ? ne : 1), s);
        if (ne > 0)
            hipLaunchKernelGGL(k_targets, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(g.ok), ne, P<uint32_t>(g.tg));
    }
    // packed in-keys (key-only sort) when ids and positions fit: od(u) <= sqrt(2m) under a degree
    // order (every out-neighbour has at least u's degree), so m < 2^31 relationships bound it by 2^16
    bool packed = g.ib <= 24 && m_all < (int64_t(1) << 31);
    if (packed && ne > 0) {  // (an estimated degree order does not carry the sqrt(2m) bound: check it)
        if (!maxod) {
            maxod = dev_alloc(sizeof(unsigned long long), s);
            HIP_CHECK(hipMemsetAsync(P<void>(maxod), 0, sizeof(unsigned long long), st));
            hipLaunchKernelGGL(k_max_od, dim3(grid(s, n)), dim3(256), 0, st, P<int64_t>(g.off), n,
                               P<unsigned long long>(maxod));
        }
        packed = read_scalar(s, reinterpret_cast<const int64_t*>(P<unsigned long long>(maxod))) < 65536;
    }
    // direction-split lists (coded targets); the combined walks when the codes or packed keys do not fit
    // (config tri_split = 0 forces them: tests cover that path at small sizes)
    g.split = tc.cb > 0 && packed && ne > 0 && s->cfg.tri_split;
    Buf rk;  // per oriented edge: f / b ranks (the in-lists' prefix lengths)
    Buf od32;  // split: the out-degrees, 4 bytes a vertex (k_vrec)
    if (g.split) {
        const int64_t ntiles = (ne + kSplitTile - 1) / kSplitTile;
        Buf cnt = dev_alloc(sizeof(int64_t) * 2 * (ntiles + 1), s), pre = dev_alloc(sizeof(int64_t) * 2 * (ntiles + 1), s);
        hipLaunchKernelGGL(k_split_count, dim3((unsigned)ntiles), dim3(256), 0, st, P<uint32_t>(g.tg), ne, tc,
                           P<int64_t>(cnt), ntiles);
        HIP_CHECK(hipGetLastError());
        exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(pre), ntiles, s);
        exclusive_scan_i64(P<int64_t>(cnt) + ntiles + 1, P<int64_t>(pre) + ntiles + 1, ntiles, s);
        const int64_t nF = read_scalar(s, P<int64_t>(pre) + ntiles);
        const int64_t nB = read_scalar(s, P<int64_t>(pre) + 2 * ntiles + 1);
        REQUIRE(nF + nB < (int64_t(1) << 32), CAPSMI_ERR_INTERNAL, "split lists exceed 2^32 entries");
        g.tgs = dev_alloc(sizeof(uint32_t) * (nF + nB > 0 ? nF + nB : 1), s);
        rk = dev_alloc(sizeof(uint32_t) * 2 * ne, s);
        hipLaunchKernelGGL(k_split_write, dim3((unsigned)ntiles), dim3(256), 0, st, P<uint32_t>(g.tg), P<int64_t>(g.ov),
                           ne, tc, P<int64_t>(pre), ntiles, P<uint32_t>(g.tgs), P<uint32_t>(rk));
        g.fbo = dev_alloc(sizeof(uint32_t) * (2 * n + 2), s);
        hipLaunchKernelGGL(k_split_off, dim3(grid(s, n + 1)), dim3(256), 0, st, P<int64_t>(g.off), n, ne,
                           P<uint32_t>(rk), (uint32_t)nF, (uint32_t)(nF + nB), P<uint32_t>(g.fbo));
        g.vrec = dev_alloc(sizeof(uint4) * n, s);
        od32 = dev_alloc(sizeof(uint32_t) * n, s);
        hipLaunchKernelGGL(k_vrec, dim3(grid(s, n)), dim3(256), 0, st, P<int64_t>(g.off), P<uint32_t>(g.fbo), n,
                           P<uint4>(g.vrec), P<uint32_t>(od32));
        HIP_CHECK(hipGetLastError());
    }
    // in-lists and v-mode centers (config CAPSMI_TRI_VMODE_T: the od(v) threshold; 0 = every edge from u)
    g.vmt = s->cfg.tri_vmode_t;
    if (g.vmt > 0 && ne > 0) {
        const int tsh = packed ? g.ib + 16 : 32;
        std::vector<int> td;  // by (to, from): the input is in (from, to) order and the LSD sort is stable, so
        for (int sh = tsh; sh < tsh + bits; sh += 8) td.push_back(sh);  // the digits of `to` alone give that order
        std::vector<int> tds;  // split: in-key to << 40 | edge index
        for (int sh = 40; sh < 40 + bits; sh += 8) tds.push_back(sh);
        if (dd && packed && dd->world > 1) {
            // A rank walks only its v-mode share, so it builds only that share's in-lists (the whole in-list sort
            // was ≈6 ms of every rank's replicated post-processing at s = 24): the centers v with v mod W = rank,
            // interleaved so every rank gets hubs and small centers alike
            Buf f = dev_alloc(ne, s), sel;
            hipLaunchKernelGGL(k_tri_in_flags, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(g.ok), P<int64_t>(g.off),
                               ne, tc.idmask(), g.vmt, dd->world, dd->rank, P<uint8_t>(f));
            HIP_CHECK(hipGetLastError());
            const int64_t nsel = flags_to_indices(s, P<uint8_t>(f), ne, sel);
            f.reset();
            Buf ik = dev_alloc(sizeof(uint64_t) * (nsel > 0 ? nsel : 1), s), rec;
            if (g.split) rec = dev_alloc(sizeof(uint4) * (nsel > 0 ? nsel : 1), s);
            if (nsel > 0 && g.split)
                hipLaunchKernelGGL(k_swap_keys_sp_sel, dim3(grid(s, nsel)), dim3(256), 0, st, P<uint64_t>(g.ok),
                                   P<int64_t>(g.off), P<int64_t>(sel), nsel, tc, P<uint32_t>(g.tg), P<uint32_t>(rk),
                                   P<uint32_t>(g.fbo), P<uint64_t>(ik), P<uint4>(rec));
            else if (nsel > 0)
                hipLaunchKernelGGL(k_swap_keys_sel, dim3(grid(s, nsel)), dim3(256), 0, st, P<uint64_t>(g.ok),
                                   P<int64_t>(g.off), P<int64_t>(sel), nsel, tc, P<uint64_t>(ik));
            sel.reset();
            radix_sort_keys(s, ik, nsel, g.split ? tds : td);
            g.ioff = dev_alloc(sizeof(int64_t) * (n + 1), s);
            hipLaunchKernelGGL(k_offsets, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(ik), nsel, n,
                               g.split ? 40 : tsh, P<int64_t>(g.ioff));
            if (g.split) {
                g.ikey = std::move(ik);
                g.irec = std::move(rec);
            } else {
                g.itg = dev_alloc(sizeof(uint32_t) * (nsel > 0 ? nsel : 1), s);
                g.ipos = dev_alloc(sizeof(uint32_t) * (nsel > 0 ? nsel : 1), s);
            }
            if (nsel > 0 && !g.split)
                hipLaunchKernelGGL(k_in_split, dim3(grid(s, nsel)), dim3(256), 0, st, P<uint64_t>(ik), nullptr,
                                   P<int64_t>(g.off), nsel, tc, P<uint32_t>(g.itg), P<uint32_t>(g.ipos));
            g.vm_own = true;
        } else {
            Buf ik = dev_alloc(sizeof(uint64_t) * ne, s);
            Buf iv = g.split ? dev_alloc(sizeof(uint4) * ne, s) : packed ? Buf() : dev_alloc(sizeof(int64_t) * ne, s);
            Buf h0;  // split: the in-key sort's first-digit tile counts, written with the keys
            if (g.split) {  // iv: the records (k_swap_keys_sp)
                const int64_t ntl = (ne + kSortTile - 1) / kSortTile;
                h0 = dev_alloc(sizeof(int64_t) * 256 * ntl, s);
                hipLaunchKernelGGL(k_swap_keys_sp, dim3((unsigned)std::min<int64_t>(ntl, (int64_t)s->num_cus * 16)),
                                   dim3(256), 0, st, P<uint64_t>(g.ok), P<int64_t>(g.off), ne, tc, P<uint32_t>(g.tg),
                                   P<uint32_t>(rk), P<uint32_t>(g.fbo), P<uint32_t>(od32), P<uint64_t>(ik), P<uint4>(iv),
                                   P<int64_t>(h0), tds[0]);
            } else
                hipLaunchKernelGGL(k_swap_keys, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(g.ok), P<int64_t>(g.off), ne,
                                   tc, P<uint64_t>(ik), packed ? nullptr : P<int64_t>(iv));
            rk.reset();
            if (packed || g.split) radix_sort_keys(s, ik, ne, g.split ? tds : td, P<int64_t>(h0));  // (no copy back)
            else radix_sort_digits(s, P<uint64_t>(ik), P<int64_t>(iv), ne, td);
            g.ioff = dev_alloc(sizeof(int64_t) * (n + 1), s);
            hipLaunchKernelGGL(k_offsets, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(ik), ne, n,
                               g.split ? 40 : tsh, P<int64_t>(g.ioff));
            if (g.split) {
                g.ikey = std::move(ik);
                g.irec = std::move(iv);
            } else {
                g.itg = dev_alloc(sizeof(uint32_t) * ne, s);
                g.ipos = dev_alloc(sizeof(uint32_t) * ne, s);
            }
            if (!g.split)
                hipLaunchKernelGGL(k_in_split, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(ik),
                                   packed ? nullptr : P<int64_t>(iv), P<int64_t>(g.off), ne, tc, P<uint32_t>(g.itg),
                                   P<uint32_t>(g.ipos));
        }
        Buf fvm = dev_alloc(n, s);
        hipLaunchKernelGGL(k_tri_vm_bins, dim3(grid(s, n)), dim3(256), 0, st, P<int64_t>(g.off), P<int64_t>(g.ioff), n,
                           g.vmt, P<uint8_t>(fvm));
        g.nvm = flags_to_indices(s, P<uint8_t>(fvm), n, g.vm_c);
    } else {
        g.vmt = 0;
    }
    Buf fsm = dev_alloc(n, s), fbg = dev_alloc(n, s);
    hipLaunchKernelGGL(k_tri_bins, dim3(grid(s, n)), dim3(256), 0, st, P<int64_t>(g.off), n, P<uint8_t>(fsm),
                       P<uint8_t>(fbg));
    g.nsmall = flags_to_indices(s, P<uint8_t>(fsm), n, g.small_u);
    g.nbig = flags_to_indices(s, P<uint8_t>(fbg), n, g.big_u);
    HIP_CHECK(hipGetLastError());
    ph.reset();
    REQUIRE(!dd || dd->world < 255, CAPSMI_ERR_UNSUPPORTED, "distributed triangle count: at most 254 ranks");
}

namespace {
void set_lds_attr(const void* k, size_t bytes) { lds_attr(k, bytes); }
}  // namespace

// count for vertex share `part` of `nparts` (interleaved center lists); pair/self terms with part 0
uint64_t tri_count(capsmi_session* s, const TriGraph& g, int part, int nparts) {
    using namespace tri;
    hipStream_t st = s->stream;
    Buf out = dev_alloc(24, s);
    HIP_CHECK(hipMemsetAsync(P<void>(out), 0, 24, st));
    {
        KernelTimer kt(s, "triangles");
        // this part's share of each center list: every nparts-th center from `part` (interleaved, so each part
        // gets hubs and small centers alike -- the contiguous work-estimated cuts of round 4 left the shares of
        // a single trigraph at max / mean 1.41); a distributed build's in-lists hold its own v-mode centers only
        std::vector<Buf> keep;
        auto share = [&](const Buf& cs, int64_t nc, bool own, const int64_t*& p, int64_t& cnt) {
            p = P<int64_t>(cs);
            cnt = nc;
            if (nparts <= 1 || own || nc == 0) return;
            cnt = nc > part ? (nc - part + nparts - 1) / nparts : 0;
            if (cnt == 0) return;
            keep.emplace_back(dev_alloc(sizeof(int64_t) * cnt, s));
            hipLaunchKernelGGL(k_tri_stride, dim3(grid(s, cnt)), dim3(256), 0, st, P<int64_t>(cs), part, nparts, cnt,
                               P<int64_t>(keep.back()));
            HIP_CHECK(hipGetLastError());
            p = P<int64_t>(keep.back());
        };
        const int64_t *sp, *bp, *vp;
        int64_t sn, bn, vn;
        share(g.small_u, g.nsmall, false, sp, sn);
        share(g.big_u, g.nbig, false, bp, bn);
        share(g.vm_c, g.nvm, g.vm_own, vp, vn);
        const TgCode tc{(uint32_t)g.ib, (uint32_t)g.cb};
        // items (hash chunk, neighbour chunk) of the centers cs[0, nc), taken from a global counter
        auto run_items = [&](const int64_t* cs, int64_t nc, bool vm) {
            Buf ib = dev_alloc(sizeof(int64_t) * (2 * nc + 2), s);
            int64_t* items = P<int64_t>(ib);
            int64_t* ipre = items + nc;
            // workgroups: v-mode 1024 lanes, u-mode 512 (four items in flight per CU for its many small
            // items; v-mode at 512 lanes re-walks the lists for more hash chunks per hub: 96.0 -> 114 ms).
            // The v-mode split items take 512 edges per chunk (256 -> 512: triangles 55.4 -> 54.0 ms),
            // kVChunk * kVGroup edges per item (4096: the same)
            const int B = vm ? 1024 : 512;
            const int epi = kVChunk * kVGroup;
            hipLaunchKernelGGL(k_tri_items, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, P<int64_t>(g.off),
                               vm ? P<int64_t>(g.ioff) : nullptr, cs, nc, 2 * B, epi, items);
            exclusive_scan_i64(items, ipre, nc, s);
            const int64_t nitems = read_scalar(s, ipre + nc);
            Buf iq = dev_alloc(sizeof(uint64_t) * (nitems > 0 ? nitems : 1), s);
            hipLaunchKernelGGL(k_tri_item_map, dim3(grid(s, nc)), dim3(256), 0, st, ipre, nc, P<uint64_t>(iq));
            Buf ctr = dev_alloc(sizeof(unsigned long long), s);
            HIP_CHECK(hipMemsetAsync(P<void>(ctr), 0, sizeof(unsigned long long), st));
            const size_t lds = B == 1024 ? sizeof(ItemLds<1024>) : sizeof(ItemLds<512>);
            auto kf = vm ? k_tri_big_items<4, true, 1024> : k_tri_big_items<4, false, 512>;
            // resident: two 1024-lane or four 512-lane workgroups per CU (LDS), twice that queued
            const dim3 ig((unsigned)(s->num_cus * (B == 1024 ? 4 : 8)));
            if (g.split) {  // the walks over the direction-split lists
                const size_t ldsp = vm ? sizeof(ItemLdsSp<1024, 512>) : sizeof(ItemLdsSp<512, sp_edges(512)>);
                // (8 lanes per short list instead of 16 -- 8 lists a wave pass for the halved split lists --
                // measured 54.4 -> 55.4 ms)
                auto kp = vm ? k_tri_items_sp<4, true, 1024, 512> : k_tri_items_sp<4, false, 512>;
                set_lds_attr(reinterpret_cast<const void*>(kp), ldsp);
                hipLaunchKernelGGL(kp, ig, dim3(B), ldsp, st, P<uint32_t>(g.tg), tc, P<int64_t>(g.ov), P<int64_t>(g.off),
                                   P<uint32_t>(g.tgs), P<uint4>(g.vrec), P<int64_t>(g.ioff), P<uint64_t>(g.ikey),
                                   P<uint4>(g.irec), g.vmt, cs, nitems, P<uint64_t>(iq), P<unsigned long long>(ctr),
                                   P<unsigned long long>(out));
                return;
            }
            set_lds_attr(reinterpret_cast<const void*>(kf), lds);
            hipLaunchKernelGGL(kf, ig, dim3(B), lds, st,
                               P<uint32_t>(g.tg), tc, P<int64_t>(g.ov), P<int64_t>(g.off),
                               P<int64_t>(g.ioff), P<uint32_t>(g.itg), P<uint32_t>(g.ipos), g.vmt, cs, nc, ipre,
                               P<uint64_t>(iq), P<unsigned long long>(ctr),
                               P<unsigned long long>(out));
        };
        if (bn > 0) run_items(bp, bn, false);
        if (vn > 0) run_items(vp, vn, true);
        if (sn > 0 && g.split) {
            const int64_t gs = std::min<int64_t>((sn + 3) / 4, (int64_t)s->num_cus * 16);
            hipLaunchKernelGGL(k_tri_small_sp<4>, dim3((unsigned)gs), dim3(kTriBlock), 0, st, P<uint32_t>(g.tg), tc,
                               P<int64_t>(g.ov), P<int64_t>(g.off), P<uint32_t>(g.tgs), P<uint4>(g.vrec), g.vmt,
                               sp, sn, P<unsigned long long>(out));
        } else if (sn > 0) {
            const int64_t gs = std::min<int64_t>((sn + 3) / 4, (int64_t)s->num_cus * 16);
            hipLaunchKernelGGL(k_tri_small<4>, dim3((unsigned)gs), dim3(kTriBlock), 0, st,
                               P<uint32_t>(g.tg), tc, P<int64_t>(g.ov), P<int64_t>(g.off), g.vmt,
                               sp, sn, P<unsigned long long>(out));
        }
    }
    // pair terms over this graph's undirected edges (a distributed build's ek holds this rank's pairs, so
    // every part adds its own), self terms once
    if ((part == 0 || g.dist) && g.pair)  // the direct build's sum (a distributed build's: this rank's pairs)
        HIP_CHECK(hipMemcpyAsync(P<unsigned long long>(out) + 1, P<void>(g.pair), sizeof(unsigned long long),
                                 hipMemcpyDeviceToDevice, st));
    if ((part == 0 || g.dist) && g.nek > 0)
        hipLaunchKernelGGL(k_pair_terms, dim3(grid(s, g.nek)), dim3(256), 0, st, P<uint64_t>(g.ek), P<int64_t>(g.ev),
                           g.nek, P<uint32_t>(g.sl), P<unsigned long long>(out) + 1);
    if (part == 0)
        hipLaunchKernelGGL(k_self_terms, dim3(grid(s, g.n)), dim3(256), 0, st, P<uint32_t>(g.sl), g.n,
                           P<unsigned long long>(out) + 2);
    HIP_CHECK(hipGetLastError());
    uint64_t h[3];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(out), 24, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return 3 * h[0] + h[1] + h[2];
}

}  // namespace capsmi
