// k_varlen.hip -- fused BoundedVarLengthExpand + grouped count (C5), never materialising paths.
//
//   MATCH (a)-[r*lower..upper]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), count(*)   (0 <= lower <= upper <= 4,
//   upper >= 1; lower = 0 adds the zero-length path, whose b is a copy of a without b's node scan)
//
// CAPS plans this as `upper` chained joins with an isomorphism filter per hop and a union over the
// lengths (VarLengthExpandPlanner.scala:83-136, 146-171, 247-260): one row per edge-distinct path.
// Per start node a the number of such paths has a closed form in per-node degree sums
// (derivation in DESIGN.md; checked against path enumeration in oracle/rmat.c):
//   od(v)  = #{r: v -> w, b_ok(w)}          s(v) = #self-loops at v
//   W(v)   = sum_{r: v -> w} od(w)          m(v,u) = #rels v -> u
//   len 1: od(a)
//   len 2: sum_{r: a->b} od(b) - s(a) b_ok(a)
//   len 3: sum_{r: a->b} [W(b) - (m(b,a) + s(b)) b_ok(b)] - s(a) (od(a) - 2 b_ok(a))
// Four streaming passes over the relationship table plus one hash probe per relationship for m(b,a).
// Four hops (round 6): var_length4 below.
#include <cstdlib>

#include "part_common.h"

namespace capsmi {
namespace varlen {

struct Dom {
    const uint32_t* a;
    const uint32_t* b;
    int64_t lo, hi;
    int a_full, b_full;
};

__device__ __forceinline__ bool in_dom(const Dom& d, int64_t v) { return v >= d.lo && v < d.hi; }
__device__ __forceinline__ bool bok(const Dom& d, int64_t v) {
    if (!in_dom(d, v)) return false;
    if (d.b_full) return true;
    const uint64_t x = (uint64_t)(v - d.lo);
    return (d.b[x >> 5] >> (x & 31)) & 1u;
}
__device__ __forceinline__ bool aok(const Dom& d, int64_t v) {
    if (!in_dom(d, v)) return false;
    if (d.a_full) return true;
    const uint64_t x = (uint64_t)(v - d.lo);
    return (d.a[x >> 5] >> (x & 31)) & 1u;
}

// pass 1: od(v), s(v)
__global__ void k_deg(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                      unsigned long long* __restrict__ od, unsigned long long* __restrict__ s) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[e], v = dst[e];
        if (!in_dom(d, u)) continue;
        if (bok(d, v)) atomicAdd(&od[u - d.lo], 1ULL);
        if (u == v) atomicAdd(&s[u - d.lo], 1ULL);
    }
}

// pass 2: W(v) = sum_{r: v -> w} od(w)
__global__ void k_w(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                    const unsigned long long* __restrict__ od, unsigned long long* __restrict__ W) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[e], v = dst[e];
        if (!in_dom(d, u) || !in_dom(d, v)) continue;
        const unsigned long long x = od[v - d.lo];
        if (x) atomicAdd(&W[u - d.lo], x);
    }
}

// pass 3: per relationship a -> b: T2(a) += od(b); T3(a) += W(b) - (m(b,a) + s(b)) b_ok(b)
__global__ void k_t(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                    const unsigned long long* __restrict__ od, const unsigned long long* __restrict__ s,
                    const unsigned long long* __restrict__ W, const int64_t* __restrict__ rev_slot,
                    const int64_t* __restrict__ slot_count, int need3, unsigned long long* __restrict__ T2,
                    unsigned long long* __restrict__ T3) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = src[e], b = dst[e];
        if (!in_dom(d, a) || !in_dom(d, b) || !aok(d, a)) continue;
        const int64_t bi = b - d.lo;
        atomicAdd(&T2[a - d.lo], od[bi]);
        if (need3) {
            int64_t t3 = (int64_t)W[bi];
            if (bok(d, b)) {
                const int64_t rs = rev_slot[e];
                const int64_t mba = rs >= 0 ? slot_count[rs] : 0;
                t3 -= mba + (int64_t)s[bi];
            }
            atomicAdd(&T3[a - d.lo], (unsigned long long)t3);  // two's complement sum
        }
    }
}

// pass 4: per node, the count over lengths lower..upper; flags rows with count > 0
__global__ void k_final(int64_t n, Dom d, int lower, int upper, const unsigned long long* __restrict__ od,
                        const unsigned long long* __restrict__ s, const unsigned long long* __restrict__ T2,
                        const unsigned long long* __restrict__ T3, const unsigned long long* __restrict__ L4,
                        int64_t* __restrict__ cnt, uint8_t* __restrict__ f,
                        int64_t own_lo, int64_t own_hi) {  // rows only for the owned a (relative [own_lo, own_hi))
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = d.lo + i;
        int64_t total = 0;
        if (aok(d, a)) {
            const int64_t o = (int64_t)od[i], sl = (int64_t)s[i], ba = bok(d, a) ? 1 : 0;
            const int64_t c1 = o;
            const int64_t c2 = (int64_t)T2[i] - sl * ba;
            const int64_t c3 = (int64_t)T3[i] - sl * (o - 2 * ba);
            if (lower == 0) total += 1;  // the zero-length path: b is a copy of a (VarLengthExpandPlanner.scala:146-153)
            if (lower <= 1 && upper >= 1) total += c1;
            if (lower <= 2 && upper >= 2) total += c2;
            if (lower <= 3 && upper >= 3) total += c3;
            if (L4 && lower <= 4 && upper >= 4) total += (int64_t)L4[i];  // var_length4
        }
        cnt[i] = total;
        f[i] = total > 0 && i >= own_lo && i < own_hi ? 1 : 0;
    }
}

// ---- source-sliced passes (n <= 2^24 ids) ------------------------------------------------------------
// The atomic passes above hit one global counter per relationship; R-MAT hubs make those hot
// addresses.  Here the relationships are first grouped by source slice of 2^kVlBits ids (the
// chunked partition of k_part.hip, buckets by source), so every per-source sum is accumulated in
// LDS by the block that owns the slice segment and flushed once per segment.
// The reverse multiplicity m(b, a) needs, for a in slice j, the relationships *into* slice j: a
// second partition buckets them by target slice, and each slice gets its own open-addressing
// table of (target, source) pair counts sized to the slice, so inserts (walking the target
// partition) and probes (walking the source partition) both stay inside one slice's table,
// small enough for the XCD's L2.
constexpr int kVlBits = 13;  // 8192 ids per slice: two 64 KiB LDS accumulator arrays
constexpr int kVlIds = 1 << kVlBits;
constexpr int kVlBlock = 1024;

__device__ __forceinline__ unsigned long long splitmix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

__device__ __forceinline__ unsigned long long pkey(uint32_t s, uint32_t t) { return ((unsigned long long)s << 32) | t; }

// Exact (source, target) pair counts of the candidate pairs, open addressing, one 64-bit slot per
// pair: bits 0..47 = (s << 24 | t) + 1 (ids < 2^24 - 1, so never 0 = empty), bits 48..63 = count
// mod 2^16; a count that wraps adds 1 to ovf[slot] (units of 2^16) and raises *any_ovf.
constexpr unsigned long long kKeyMask = (1ULL << 48) - 1;
constexpr unsigned long long kCnt1 = 1ULL << 48;

struct PairHash {
    unsigned long long* slot;
    unsigned int* ovf;
    unsigned int* any_ovf;
    unsigned long long mask;
    // sized on the device (the sharded form): the mask lives at *dmask, written by k_vl_hsize from the
    // candidate count, so no host round trip sits between the candidates and the table
    const unsigned long long* dmask = nullptr;
};

__device__ __forceinline__ PairHash sized(PairHash h) {
    if (h.dmask) {
        h.mask = *h.dmask;
        h.any_ovf = h.ovf + h.mask + 1;
    }
    return h;
}

// the table's size from the candidate count: the power of two >= 2 * count (at least 1024) -- as the host
// sizes it in the single-device form -- capped by the allocation (cap_max slots)
__global__ void k_vl_hsize(const unsigned long long* __restrict__ ncand, unsigned long long cap_max,
                           unsigned long long* __restrict__ dmask) {
    unsigned long long cap = 1024;
    while (cap < 2 * *ncand && cap < cap_max) cap <<= 1;
    *dmask = cap - 1;
}

// clears the device-sized table's slots [0, cap) and overflow words [0, cap]
__global__ void k_vl_hclear(PairHash h) {
    h = sized(h);
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i <= h.mask + 1;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        if (i <= h.mask) h.slot[i] = 0;
        h.ovf[i] = 0;  // ovf[cap] is any_ovf
    }
}

__device__ __forceinline__ unsigned long long hkey(uint32_t s, uint32_t t) {
    return (((unsigned long long)s << 24) | t) + 1;
}

__device__ __forceinline__ void pair_insert(const PairHash& h, unsigned long long k) {
    for (unsigned long long i = splitmix(k) & h.mask;; i = (i + 1) & h.mask) {
        unsigned long long cur = h.slot[i];
        if (cur == 0) {
            cur = atomicCAS(&h.slot[i], 0ULL, k | kCnt1);
            if (cur == 0) return;
        }
        if ((cur & kKeyMask) == k) {
            if ((atomicAdd(&h.slot[i], kCnt1) >> 48) == 0xFFFFu) {
                atomicAdd(&h.ovf[i], 1u);
                atomicOr(h.any_ovf, 1u);
            }
            return;
        }
    }
}

__device__ __forceinline__ unsigned long long slot_count(const PairHash& h, unsigned long long i,
                                                         unsigned long long v, bool ovf) {
    return (v >> 48) + (ovf ? (unsigned long long)h.ovf[i] << 16 : 0ULL);
}

__device__ __forceinline__ unsigned long long pair_count(const PairHash& h, unsigned long long k, bool ovf) {
    for (unsigned long long i = splitmix(k) & h.mask;; i = (i + 1) & h.mask) {
        const unsigned long long cur = h.slot[i];
        if ((cur & kKeyMask) == k) return slot_count(h, i, cur, ovf);
        if (cur == 0) return 0;
    }
}

// One-bit filter of the directed pairs present, one region of 2^rshift bits per 2^(kVlBits -
// sublog) TARGET ids (2^sublog regions per slice): the bit of pair (s, t) lives in t's region.
// Walking the target partition sets a slice's regions; the tests ask "does t -> s exist" for an s
// of the slice being walked in the source partition, i.e. inside that slice's regions -- L2-local
// either way.  In every walk the region follows the pair's second (bucket) id.
struct RegionBloom {
    uint32_t* w;
    unsigned long long rmask;  // bits per region - 1 (power of two)
    int rshift;                // log2(bits per region), <= 20 (128 KiB of LDS)
    int sublog;                // log2(regions per slice)
};

// A key sets three bits of ONE 32-bit word of its region (a blocked filter: one load per test).  At 8
// bits per pair that is ~4 % false candidates against 22 % for one bit at 4 bits per pair -- and at
// C5 only 0.3 % of the relationships have a reverse, so the false candidates were nearly all of the
// 7.5·10^6 exact-table inserts.
__device__ __forceinline__ void rb_pos(const RegionBloom& b, unsigned long long k, uint32_t& word, uint32_t& mask) {
    const unsigned long long h = splitmix(k ^ 0x5DEECE66DULL);
    word = (uint32_t)(h & (b.rmask >> 5));
    mask = (1u << ((h >> 40) & 31)) | (1u << ((h >> 46) & 31)) | (1u << ((h >> 52) & 31));
}

__device__ __forceinline__ bool rb_test(const RegionBloom& b, uint32_t y, unsigned long long k) {
    uint32_t word, mask;
    rb_pos(b, k, word, mask);
    const unsigned long long base = (unsigned long long)(y >> (kVlBits - b.sublog)) << (b.rshift - 5);
    return (b.w[base + word] & mask) == mask;
}

// Second-level filter of the candidate pairs (those the RegionBloom passes): one region of
// kF2Words words per source slice, two bits per key inside one word.  Built in LDS by the W walk
// (candidates (s, t) of slice(s)), tested on the reverse key (t, s) in slice(t)'s region: a pair
// whose reverse exists is a candidate both ways, so it always passes.
constexpr int kF2Words = 1 << 14;  // 64 KiB per slice: ~9 bits per candidate at 22 % false positives

__device__ __forceinline__ void f2_pos(unsigned long long key, uint32_t& word, uint32_t& bits) {
    const unsigned long long h = splitmix(key ^ 0x2545F4914F6CDD1DULL);
    word = (uint32_t)h & (kF2Words - 1);
    bits = (1u << ((h >> 40) & 31)) | (1u << ((h >> 50) & 31));
}

__device__ __forceinline__ bool f2_test(const uint32_t* f2, uint32_t x, unsigned long long key) {
    uint32_t word, bits;
    f2_pos(key, word, bits);
    return (f2[((size_t)(x >> kVlBits) * kF2Words) + word] & bits) == bits;
}

using part::ChunkWalk;

template <class Visit, class Flush>
__device__ void walk_chunks(const ChunkWalk& cw, Visit visit, Flush flush) {
    part::walk_chunks<kVlBlock>(cw, visit, flush);
}

__device__ __forceinline__ bool bit_of(const uint32_t* w, int full, uint32_t x) {
    return full || ((w[x >> 5] >> (x & 31)) & 1u);
}

// flush an LDS accumulator array of slice j into the global per-node array, then clear it
__device__ __forceinline__ void flush_acc(unsigned long long* acc, unsigned long long* g, int j, int64_t n) {
    for (int i = threadIdx.x; i < kVlIds; i += kVlBlock) {
        const unsigned long long v = acc[i];
        const int64_t x = (int64_t)j * kVlIds + i;
        if (v && x < n) atomicAdd(&g[x], v);
        acc[i] = 0;
    }
}

// pass 1 (source partition, pair = (target, source)): od(v), s(v)
// With od: od(s) (LDS) and self-loop counts s(v) (global atomics: rare).  With f2part: the
// candidate pairs s -> t (those the first-level filter passes) marked in the block's F2 region for
// slice(s), stored whole per slice segment into partial slot w + j (k_vl_bset's scheme), and
// counted.  One 1024-lane block per CU either way (64 KiB accumulators + 64 KiB F2 region).
// Candidate list (cl set, the single-GPU form): the candidates' exact-table keys hkey(s, t) are
// written to cl (count in *ncand) through a per-wave LDS buffer flushed with one global add per
// kClFlush keys, instead of the F2 region -- the T walk then needs no filter test per relationship.
constexpr int kClWave = 512;   // keys buffered per wave (16 waves: 64 KiB, the F2 region's LDS)
constexpr int kClFlush = 256;  // a wave flushes its buffer at the start of a step once it holds this many

__device__ __forceinline__ void cl_flush(unsigned long long* buf, uint32_t& cnt_lds, unsigned long long* cl,
                                         unsigned long long* ncand) {  // wave-level
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t n = min(__builtin_amdgcn_readfirstlane(cnt_lds), (uint32_t)kClWave);
    if (n == 0) return;
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(ncand, (unsigned long long)n);
    base = __shfl(base, 0, 64);
    for (uint32_t i = lane; i < n; i += 64) cl[base + i] = buf[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) cnt_lds = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__global__ void __launch_bounds__(kVlBlock) k_vl_deg(ChunkWalk cw, const uint32_t* __restrict__ bw, int b_full,
                                                     int64_t n, unsigned long long* __restrict__ od,
                                                     unsigned long long* __restrict__ sl, RegionBloom bl,
                                                     uint4* __restrict__ f2part, unsigned long long* __restrict__ ncand,
                                                     unsigned long long* __restrict__ cl) {
    extern __shared__ unsigned long long vl_lds[];
    unsigned long long* a_od = vl_lds;
    uint32_t* f2 = reinterpret_cast<uint32_t*>(vl_lds + kVlIds);
    const int wave = threadIdx.x >> 6;
    unsigned long long* cbuf = vl_lds + kVlIds + (size_t)wave * kClWave;  // cl: the F2 region's space
    __shared__ unsigned int cand;
    __shared__ uint32_t ccnt[kVlBlock / 64];
    if (threadIdx.x == 0) cand = 0;
    if (threadIdx.x < kVlBlock / 64) ccnt[threadIdx.x] = 0;
    unsigned int mine = 0;  // this lane's candidates (one LDS add per wave at the end)
    const bool cands = f2part || cl;
    for (int i = threadIdx.x; i < kVlIds; i += kVlBlock) a_od[i] = 0;
    if (f2part)
        for (int i = threadIdx.x; i < kF2Words; i += kVlBlock) f2[i] = 0;
    __syncthreads();
    part::walk_chunks_n<kVlBlock>(
        cw,
        [&](const uint2 (&pr)[part::kWalkItems], uint32_t valid, int) {  // pr[k] = (t, s)
            constexpr int K = part::kWalkItems;
            if (cl && __builtin_amdgcn_readfirstlane(ccnt[wave]) >= (uint32_t)kClFlush) cl_flush(cbuf, ccnt[wave], cl, ncand);
            uint32_t bwd[K], rw[K], rm[K];  // every global word of the step loaded before any is used
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t t = pr[k].x, s = pr[k].y;
                bwd[k] = (od && !b_full) ? bw[t >> 5] : 0xFFFFFFFFu;
                if (cands) {
                    uint32_t word;
                    rb_pos(bl, pkey(t, s), word, rm[k]);
                    rw[k] = bl.w[((unsigned long long)(s >> (kVlBits - bl.sublog)) << (bl.rshift - 5)) + word];
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!((valid >> k) & 1u)) continue;
                const uint32_t t = pr[k].x, s = pr[k].y;
                if (od) {
                    if ((bwd[k] >> (t & 31)) & 1u) atomicAdd(&a_od[s & (kVlIds - 1)], 1ULL);
                    if (s == t) atomicAdd(&sl[s], 1ULL);
                }
                if (cands && (rw[k] & rm[k]) == rm[k]) {
                    if (cl) {
                        const uint32_t q = atomicAdd(&ccnt[wave], 1u);
                        if (q < (uint32_t)kClWave) {
                            cbuf[q] = hkey(s, t);
                        } else {  // the step overfilled the buffer: straight to the list (rare)
                            cl[atomicAdd(ncand, 1ULL)] = hkey(s, t);
                        }
                        continue;
                    }
                    uint32_t word, bits;
                    f2_pos(pkey(s, t), word, bits);
                    atomicOr(&f2[word], bits);
                    ++mine;
                }
            }
        },
        [&](int j) {
            if (od) flush_acc(a_od, od, j, n);
            if (f2part) {
                uint4* g = f2part + (((size_t)blockIdx.x + j) * (kF2Words / 4));
                const uint4* l = reinterpret_cast<const uint4*>(f2);
                for (int i = threadIdx.x; i < kF2Words / 4; i += kVlBlock) g[i] = l[i];
                __syncthreads();
                for (int i = threadIdx.x; i < kF2Words; i += kVlBlock) f2[i] = 0;
            }
        });
    if (cl) cl_flush(cbuf, ccnt[wave], cl, ncand);
    if (f2part) {
        for (int o = 32; o > 0; o >>= 1) mine += __shfl_down(mine, o, 64);
        if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&cand, mine);
        __syncthreads();
        if (threadIdx.x == 0 && cand) atomicAdd(ncand, (unsigned long long)cand);
    }
}

// od narrowed to 32 bits for the W walk's gathers: half the bytes, so more of it stays in each XCD's L2
// (an out-degree is below 2^32: relationship counts are)
__global__ void k_vl_narrow(const unsigned long long* __restrict__ od, int64_t n, uint32_t* __restrict__ od32) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        od32[i] = (uint32_t)od[i];
}

// pass 2: W(v) = sum_{v -> w} od(w); 64 KiB of LDS, two blocks per CU for the random od gathers
__global__ void __launch_bounds__(kVlBlock) k_vl_w(ChunkWalk cw, int64_t n, const uint32_t* __restrict__ od,
                                                   unsigned long long* __restrict__ W) {
    extern __shared__ unsigned long long vl_lds[];
    unsigned long long* a_w = vl_lds;
    for (int i = threadIdx.x; i < kVlIds; i += kVlBlock) a_w[i] = 0;
    __syncthreads();
    part::walk_chunks_n<kVlBlock>(
        cw,
        [&](const uint2 (&pr)[part::kWalkItems], uint32_t valid, int) {  // pr[k] = (t, s)
            unsigned long long x[part::kWalkItems];
#pragma unroll
            for (int k = 0; k < part::kWalkItems; ++k) x[k] = od[pr[k].x];  // all gathers first (4 B each)
#pragma unroll
            for (int k = 0; k < part::kWalkItems; ++k)
                if (((valid >> k) & 1u) && x[k]) atomicAdd(&a_w[pr[k].y & (kVlIds - 1)], x[k]);
        },
        [&](int j) { flush_acc(a_w, W, j, n); });
}

// the candidate list into the exact table
__global__ void k_vl_cins(const unsigned long long* __restrict__ cl, const unsigned long long* __restrict__ ncand,
                          PairHash h) {
    h = sized(h);
    const int64_t cnt = (int64_t)*ncand;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * blockDim.x)
        pair_insert(h, cl[i]);
}

// the sharded form's candidates straight from the relationship columns (a shard holds few relationships:
// a flat pass with one filter word per relationship beats partitioning them by source first): the
// relationships s -> t whose reverse may exist, as exact-table keys.  A block takes kFcIt x 256
// relationships per step and claims its candidates' slots with one global add (one add per wave put
// ~5·10^5 adds on the one counter at C5 and took 6.3 ms for 3.4·10^7 relationships).
constexpr int kFcBlock = 256, kFcIt = 16;

__global__ void __launch_bounds__(kFcBlock) k_vl_flatcand(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                          int64_t m, int64_t lo, RegionBloom bl,
                                                          unsigned long long* __restrict__ cl,
                                                          unsigned long long* __restrict__ ncand) {
    constexpr int T = kFcBlock * kFcIt, W = kFcBlock / 64;
    __shared__ uint32_t wsum[W];
    __shared__ unsigned long long base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t t0 = (int64_t)blockIdx.x * T; t0 < m; t0 += (int64_t)gridDim.x * T) {  // block-uniform
        uint32_t ss[kFcIt], tt[kFcIt], mask = 0;
#pragma unroll
        for (int u = 0; u < kFcIt; ++u) {
            const int64_t e = t0 + (int64_t)u * kFcBlock + threadIdx.x;
            ss[u] = tt[u] = 0;
            if (e < m) {
                ss[u] = (uint32_t)(src[e] - lo);
                tt[u] = (uint32_t)(dst[e] - lo);
            }
        }
#pragma unroll
        for (int u = 0; u < kFcIt; ++u) {
            const int64_t e = t0 + (int64_t)u * kFcBlock + threadIdx.x;
            if (e < m && rb_test(bl, ss[u], pkey(tt[u], ss[u]))) mask |= 1u << u;
        }
        const uint32_t c = (uint32_t)__popc(mask);
        uint32_t incl = c;  // block exclusive prefix of the lanes' candidate counts
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            pre += w < wave ? wsum[w] : 0u;
            tot += wsum[w];
        }
        if (threadIdx.x == 0) base = tot ? atomicAdd(ncand, (unsigned long long)tot) : 0ULL;
        __syncthreads();
        unsigned long long pos = base + pre + incl - c;
#pragma unroll
        for (int u = 0; u < kFcIt; ++u)
            if ((mask >> u) & 1u) cl[pos++] = hkey(ss[u], tt[u]);
        __syncthreads();  // wsum and base are rewritten by the next step
    }
}

// target partition (pair = (source, target), j = slice(t)): mark pair (s, t) in t's region.  Each
// region (<= 128 KiB) is built in LDS, one pass over the block's chunks per region of the slice,
// and stored whole into the block's partial slot (w + j) * 2^sublog + sub: the slots of a block are
// distinct from every other block's (a later block's slices start at or after this block's last),
// so no atomics; k_vl_bmerge ORs a region's partials.
__global__ void __launch_bounds__(kVlBlock) k_vl_bset(ChunkWalk cw, RegionBloom bl, uint4* __restrict__ part) {
    extern __shared__ uint32_t rb_lds[];
    const int rwords = 1 << (bl.rshift - 5), nsub = 1 << bl.sublog, rb = kVlBits - bl.sublog;
    for (int i = threadIdx.x; i < rwords; i += kVlBlock) rb_lds[i] = 0;
    __syncthreads();
    for (int sub = 0; sub < nsub; ++sub)
        walk_chunks(
            cw,
            [&](uint2 p, int) {
                if ((int)((p.y >> rb) & (nsub - 1)) != sub) return;
                uint32_t word, mask;
                rb_pos(bl, pkey(p.x, p.y), word, mask);
                atomicOr(&rb_lds[word], mask);
            },
            [&](int j) {
                uint4* g = part + ((((size_t)blockIdx.x + j) * nsub + sub) << (bl.rshift - 7));
                const uint4* l = reinterpret_cast<const uint4*>(rb_lds);
                for (int i = threadIdx.x; i < rwords / 4; i += kVlBlock) g[i] = l[i];
                __syncthreads();
                for (int i = threadIdx.x; i < rwords; i += kVlBlock) rb_lds[i] = 0;
                __syncthreads();  // the next pass's first visits follow the last flush directly
            });
}

// region r = j * 2^sublog + sub = OR of the partials of the blocks whose chunk share meets slice j
__global__ void k_vl_bmerge(const int64_t* __restrict__ jst, int nt, int64_t blocks, const uint4* __restrict__ part,
                            RegionBloom bl) {
    const int64_t q4 = (int64_t)1 << (bl.rshift - 7);  // uint4 per region
    const int64_t total = ((int64_t)nt << bl.sublog) * q4;
    const int64_t per = max((jst[nt] + blocks - 1) / blocks, (int64_t)1);
    uint4* w = reinterpret_cast<uint4*>(bl.w);
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = x / q4, i = x - r * q4, j = r >> bl.sublog, sub = r & ((1 << bl.sublog) - 1);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (jst[j + 1] > jst[j]) {
            const int64_t wl = (jst[j + 1] - 1) / per;
            for (int64_t b = jst[j] / per; b <= wl && b < blocks; ++b) {
                const uint4 u = part[((((size_t)b + j) << bl.sublog) + sub) * q4 + i];
                v.x |= u.x;
                v.y |= u.y;
                v.z |= u.z;
                v.w |= u.w;
            }
        }
        w[x] = v;
    }
}

// (od(b), Y(b) = W(b) - s(b) b_ok(b)) side by side: pass 3 gathers both with one access
// (od, Y) also as one 8-byte word, od << 40 | Y, while od < 2^24 and 0 <= Y < 2^40 everywhere (*misfit set
// otherwise; zeroed with the other accumulators): the T walk then gathers half the bytes
constexpr int kPkShift = 40;
__device__ __forceinline__ void pack8(int64_t i, long long od, long long y, unsigned long long* pk, unsigned int* misfit) {
    const bool ok = od >= 0 && od < (1LL << (64 - kPkShift)) && y >= 0 && y < (1LL << kPkShift);
    pk[i] = ((unsigned long long)od << kPkShift) | (unsigned long long)y;
    if (!ok) atomicOr(misfit, 1u);
}

__global__ void k_vl_y(int64_t n, const uint32_t* __restrict__ bw, int b_full, const unsigned long long* __restrict__ od,
                       const unsigned long long* __restrict__ W, const unsigned long long* __restrict__ sl,
                       longlong2* __restrict__ ody, unsigned long long* __restrict__ pk, unsigned int* __restrict__ misfit) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const long long o = (long long)od[i];
        const long long y = (long long)W[i] - (bit_of(bw, b_full, (uint32_t)i) ? (long long)sl[i] : 0LL);
        ody[i] = make_longlong2(o, y);
        if (pk) pack8(i, o, y, pk, misfit);
    }
}

// sharded form: Y(b) alone (partial: the owner's W), then (od, Y) packed once both are reduced
__global__ void k_vl_yonly(int64_t n, const uint32_t* __restrict__ bw, int b_full,
                           const unsigned long long* __restrict__ W, const unsigned long long* __restrict__ sl,
                           long long* __restrict__ Y) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        Y[i] = (long long)W[i] - (bit_of(bw, b_full, (uint32_t)i) ? (long long)sl[i] : 0LL);
}

__global__ void k_vl_pack(int64_t n, const long long* __restrict__ od, const long long* __restrict__ Y,
                          longlong2* __restrict__ ody, unsigned long long* __restrict__ pk, unsigned int* __restrict__ misfit) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        ody[i] = make_longlong2(od[i], Y[i]);
        if (pk) pack8(i, od[i], Y[i], pk, misfit);
    }
}

// R(a) = sum_b m(a, b) m(b, a) b_ok(b) over the candidate table (every pair with its reverse present
// is in it, both ways): T3(a) -= R(a) for a_ok(a)
__global__ void k_vl_recip(PairHash h, const uint32_t* __restrict__ aw, int a_full, const uint32_t* __restrict__ bw,
                           int b_full, unsigned long long* __restrict__ T3, uint32_t own_lo, uint32_t own_hi) {
    h = sized(h);
    const bool ovf = *h.any_ovf != 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i <= h.mask;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long v = h.slot[i];
        if (!v) continue;
        const unsigned long long key = (v & kKeyMask) - 1;
        const uint32_t a = (uint32_t)(key >> 24), b = (uint32_t)(key & 0xFFFFFF);
        if (a < own_lo || a >= own_hi || !bit_of(aw, a_full, a) || !bit_of(bw, b_full, b)) continue;
        const unsigned long long r = pair_count(h, hkey(b, a), ovf);
        if (r) atomicAdd(&T3[a], (unsigned long long)(-(long long)(slot_count(h, i, v, ovf) * r)));
    }
}

// pass 3 (source partition): per relationship a -> b with a_ok(a): T2(a) += od(b); T3(a) += Y(b)
// (the - m(b, a) b_ok(b) part is k_vl_recip's)
// With the filters (ody set) it also puts the pairs a -> b that pass both (reverse maybe present,
// reverse itself a candidate) into the exact table for k_vl_recip.
__global__ void __launch_bounds__(kVlBlock) k_vl_t(ChunkWalk cw, const uint32_t* __restrict__ aw, int a_full,
                                                   int64_t n, const unsigned long long* __restrict__ od,
                                                   const longlong2* __restrict__ ody, unsigned long long* __restrict__ T2,
                                                   unsigned long long* __restrict__ T3, RegionBloom bl,
                                                   const uint32_t* __restrict__ f2, PairHash h,
                                                   const unsigned long long* __restrict__ pk,
                                                   const unsigned int* __restrict__ misfit) {
    extern __shared__ unsigned long long vl_lds[];
    const bool p8 = ody && pk && *misfit == 0;  // uniform: the 8-byte (od, Y) words
    unsigned long long *a_t2 = vl_lds, *a_t3 = vl_lds + kVlIds;
    for (int i = threadIdx.x; i < kVlIds; i += kVlBlock) a_t2[i] = a_t3[i] = 0;
    __syncthreads();
    part::walk_chunks_n<kVlBlock>(
        cw,
        [&](const uint2 (&pr)[part::kWalkItems], uint32_t valid, int) {
            constexpr int K = part::kWalkItems;
            // every gather of the step issued before any is used: (od, Y) of each target and, with the
            // filters, the second-level word of each reverse key (its table, 64 KiB per slice, passes
            // ~0.3 % of the pairs at C5, so the first-level region is read for those only -- it bounds
            // the inserts by the counted candidates, so it stays)
            longlong2 v[K];
            unsigned long long o1[K];
            uint32_t fw[K], fb[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t b = pr[k].x;  // zero pairs past a chunk's fill: in range
                if (p8) {
                    const unsigned long long w = pk[b];
                    v[k] = make_longlong2((long long)(w >> kPkShift), (long long)(w & ((1ULL << kPkShift) - 1)));
                } else if (ody) {
                    v[k] = ody[b];
                } else {
                    o1[k] = od[b];
                }
                if (h.slot) {
                    uint32_t word;
                    f2_pos(pkey(b, pr[k].y), word, fb[k]);
                    fw[k] = f2[((size_t)(b >> kVlBits) * kF2Words) + word];
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (!((valid >> k) & 1u)) continue;
                const uint32_t b = pr[k].x, a = pr[k].y, i = a & (kVlIds - 1);
                if (h.slot && (fw[k] & fb[k]) == fb[k] && rb_test(bl, a, pkey(b, a))) pair_insert(h, hkey(a, b));
                if (!bit_of(aw, a_full, a)) continue;
                if (ody) {  // T3 also wanted
                    atomicAdd(&a_t2[i], (unsigned long long)v[k].x);
                    atomicAdd(&a_t3[i], (unsigned long long)v[k].y);  // two's complement sum
                } else {
                    atomicAdd(&a_t2[i], o1[k]);
                }
            }
        },
        [&](int j) {
            flush_acc(a_t2, T2, j, n);
            flush_acc(a_t3, T3, j, n);
        });
}

inline int grid(const capsmi_session* s, int64_t n) {
    int64_t g = (n + 255) / 256;
    const int64_t cap = (int64_t)s->num_cus * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

// the accumulators and flags of one query zeroed by one launch (blockIdx.y = buffer) instead of a fill each:
// at 1/8 of C5 a fill is ~2 us of device time behind ~5 us of host launch time
constexpr int kZeroMax = 8;
struct ZeroList {
    unsigned long long* p[kZeroMax];
    int64_t n[kZeroMax];  // 8-byte words
};

__global__ void k_vl_zero(ZeroList z) {
    unsigned long long* p = z.p[blockIdx.y];
    const int64_t n = z.n[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}

void zero_words(capsmi_session* s, std::initializer_list<std::pair<void*, int64_t>> bufs) {
    ZeroList z{};
    int k = 0;
    int64_t nmax = 0;
    for (const auto& b : bufs) {
        if (!b.first || b.second <= 0) continue;
        REQUIRE(k < kZeroMax, CAPSMI_ERR_INTERNAL, "zero_words: too many buffers");
        z.p[k] = static_cast<unsigned long long*>(b.first);
        z.n[k] = b.second;
        nmax = std::max(nmax, b.second);
        ++k;
    }
    if (!k) return;
    hipLaunchKernelGGL(k_vl_zero, dim3(grid(s, nmax), k), dim3(256), 0, s->stream, z);
}

// ---- four hops ----------------------------------------------------------------------------------------
// len 4 (a) = the relationship-distinct 4-hop paths a -> ... -> z with b_ok(z), by inclusion-exclusion over
// the 15 set partitions of the hop positions {1,2,3,4} (Mobius weights prod (-1)^(|B|-1) (|B|-1)!; pinned
// against path enumeration in the oracle, oracle/cpu.py var_length4_closed_form).  A block {i, j} forces
// r_i = r_j, so the walk between them is closed: adjacent positions a self-loop, {1,3} / {2,4} a reciprocal
// pair, {1,4} a 2-walk back along the relationship.  With A the multiplicity matrix, b the end filter,
// s the self-loops, M(x, y) = m(x, y) m(y, x) and od = A b, W = A od (the len-3 vectors):
//   len4 = A^4 b - [s W + A (s od) + A A (s b)] - [M od + A M b + T14] + [2 s^2 b + b M 1]
//          + 2 [s od + 2 s^2 b + A (s b)] - 6 s b,          T14(a) = sum_{r: a -> y} b(y) sum_{r': y -> p} m(p, a)
// Every term but T14 is a product of per-node vectors over the relationships and of the pair multiplicities
// m(y, x), counted in x's sorted in-list; three passes over the (source, target)-sorted relationships (one
// atomic per source run of a wave).  T14 walks the 2-hop wedges a -> y -> p in load-balanced tiles and counts
// each closing p in a's in-list.  Relative ids below 2^24 - 1 (the keys' fields).
struct Vl4 {  // per-node u64 sums (two's complement)
    unsigned long long *X, *Q1, *P, *W4, *Q2, *Rb, *R1, *MAb, *ARb, *T14;
};

// The per-relationship passes run over the (source, target)-sorted keys: the lanes of a wave hold consecutive
// keys, so their sources form contiguous runs and each run's sum takes one atomic (a segmented sum over the
// wave) instead of one per relationship.
__device__ __forceinline__ void seg_add(uint32_t x, unsigned long long v, unsigned long long* __restrict__ arr) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // v = the sum over lanes lane .. min(lane + 2o - 1, the run's end)
        const unsigned long long vv = __shfl_down(v, o, 64);
        const uint32_t xx = __shfl_down(x, o, 64);
        if (lane + o < 64 && xx == x) v += vv;
    }
    const uint32_t xp = __shfl_up(x, 1, 64);
    if ((lane == 0 || xp != x) && x != 0xFFFFFFFFu && v) atomicAdd(&arr[x], v);
}

// the number of p's in x's sorted in-list (m(p, x))
__device__ __forceinline__ unsigned long long in_count(const uint32_t* __restrict__ isrc, int64_t i0, int64_t i1,
                                                       uint32_t p) {
    int64_t l = i0, h = i1;
    while (l < h) {
        const int64_t mid = (l + h) >> 1;
        if (isrc[mid] < p) l = mid + 1; else h = mid;
    }
    unsigned long long c = 0;
    while (l < i1 && isrc[l] == p) {
        ++c;
        ++l;
    }
    return c;
}

// per relationship x -> y: X = A W, Q1 = A (s b), P = A (s od)
__global__ void k_vl4_a(const uint64_t* __restrict__ key, int64_t mv, Dom d, const unsigned long long* __restrict__ od,
                        const unsigned long long* __restrict__ s, const unsigned long long* __restrict__ W, Vl4 v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < mv; e0 += stride) {  // block-uniform
        const int64_t e = e0 + threadIdx.x;
        uint32_t x = 0xFFFFFFFFu;
        unsigned long long wx = 0, q1 = 0, pp = 0;
        if (e < mv) {
            const uint64_t k = key[e];
            x = (uint32_t)(k >> 24);
            const uint32_t y = (uint32_t)(k & 0xFFFFFF);
            wx = W[y];
            const unsigned long long sy = s[y];
            if (sy) {
                if (bok(d, d.lo + y)) q1 = sy;
                pp = sy * od[y];
            }
        }
        seg_add(x, wx, v.X);
        seg_add(x, q1, v.Q1);
        seg_add(x, pp, v.P);
    }
}

// per relationship x -> y: W4 = A X, Q2 = A Q1, and with r = m(y, x): Rb = M b, R1 = M 1, MAb = M od
__global__ void k_vl4_b(const uint64_t* __restrict__ key, int64_t mv, Dom d, const unsigned long long* __restrict__ od,
                        const uint32_t* __restrict__ isrc, const int64_t* __restrict__ ioff, Vl4 v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < mv; e0 += stride) {  // block-uniform
        const int64_t e = e0 + threadIdx.x;
        uint32_t x = 0xFFFFFFFFu;
        unsigned long long w4 = 0, q2 = 0, rb = 0, r1 = 0, mab = 0;
        if (e < mv) {
            const uint64_t k = key[e];
            x = (uint32_t)(k >> 24);
            const uint32_t y = (uint32_t)(k & 0xFFFFFF);
            w4 = v.X[y];
            q2 = v.Q1[y];
            const unsigned long long r = in_count(isrc, ioff[x], ioff[x + 1], y);
            if (r) {
                if (bok(d, d.lo + y)) rb = r;
                r1 = r;
                mab = r * od[y];
            }
        }
        seg_add(x, w4, v.W4);
        seg_add(x, q2, v.Q2);
        seg_add(x, rb, v.Rb);
        seg_add(x, r1, v.R1);
        seg_add(x, mab, v.MAb);
    }
}

// per relationship x -> y: ARb = A Rb
__global__ void k_vl4_c(const uint64_t* __restrict__ key, int64_t mv, Vl4 v) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e0 = (int64_t)blockIdx.x * blockDim.x; e0 < mv; e0 += stride) {  // block-uniform
        const int64_t e = e0 + threadIdx.x;
        uint32_t x = 0xFFFFFFFFu;
        unsigned long long r = 0;
        if (e < mv) {
            const uint64_t k = key[e];
            x = (uint32_t)(k >> 24);
            r = v.Rb[k & 0xFFFFFF];
        }
        seg_add(x, r, v.ARb);
    }
}

// the relationships as (source << 24 | target) keys, relative ids (outside the domain: ~0, sorted last)
__global__ void k_vl4_keys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                           uint64_t* __restrict__ key) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = src[e], y = dst[e];
        key[e] = in_dom(d, x) && in_dom(d, y) ? ((uint64_t)(x - d.lo) << 24) | (uint64_t)(y - d.lo) : ~0ULL;
    }
}

// CSR offsets of the sorted keys (the first key whose source is >= v), and per key its wedge count
// b(y) * od_all(y) (od_all from the same offsets: every relationship out of y)
__global__ void k_vl4_off(const uint64_t* __restrict__ key, int64_t m, int64_t n, int64_t* __restrict__ off) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = m;
        const uint64_t t = (uint64_t)v << 24;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (key[mid] < t) lo = mid + 1; else hi = mid;
        }
        off[v] = lo;
    }
}

__global__ void k_vl4_wcount(const uint64_t* __restrict__ key, int64_t mv, Dom d, const int64_t* __restrict__ off,
                             int64_t* __restrict__ wc) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < mv; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t y = (int64_t)(key[e] & 0xFFFFFF);
        wc[e] = bok(d, d.lo + y) ? off[y + 1] - off[y] : 0;
    }
}

// the in-lists: the (source, target)-sorted keys re-sorted (stably) by target, so each target's sources
// ascend; isrc = the sources, ioff[v] = the first whose target is >= v; tg = the out-list targets (4 bytes)
__global__ void k_vl4_lists(const uint64_t* __restrict__ key, const uint64_t* __restrict__ ik, int64_t mv,
                            uint32_t* __restrict__ tg, uint32_t* __restrict__ isrc) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < mv; e += (int64_t)gridDim.x * blockDim.x) {
        tg[e] = (uint32_t)(key[e] & 0xFFFFFF);
        isrc[e] = (uint32_t)(ik[e] >> 24);
    }
}

__global__ void k_vl4_ioff(const uint64_t* __restrict__ ik, int64_t mv, int64_t n, int64_t* __restrict__ ioff) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = mv;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)(ik[mid] & 0xFFFFFF) < v) lo = mid + 1; else hi = mid;
        }
        ioff[v] = lo;
    }
}

// T14 in load-balanced tiles of kVl4T consecutive wedges (r, r') -- r = a -> y, r' = y -> p -- over the
// relationships with wedges, compacted (cw = the first wedge, coy = off[y], ca = a).  A tile's relationships
// are read once, coalesced, into LDS, each wedge's owner comes from a fill-forward max scan of their start
// positions, and lane t takes the wedges t + 512 j: consecutive lanes read consecutive entries of y's out-list.
// m(p, a) is the number of p's in a's sorted in-list, found by a binary search: in LDS when the whole tile is
// one start's (about half the tiles at C5) and its list fits, else in global memory (the lanes of a wave then
// mostly on one a and its cached lines; loading every start's list of a mixed tile into LDS measured slower,
// 19.5 -> 22.0 ms).  Closing pairs are rare (under 0.1 % of the wedges at C5), each adds one atomic.
constexpr int kVl4B = 512, kVl4I = 4, kVl4T = kVl4B * kVl4I;
constexpr int kVl4L = 4096;  // a single-start tile's in-list, searched in LDS, up to this many sources

// per tile, its first relationship: the last k with cw[k] <= the tile's first wedge (a search per tile here,
// all in flight at once, instead of one dependent search at the head of each tile)
__global__ void k_vl4_tiles(const int64_t* __restrict__ cw, int64_t K, int64_t ntiles, int64_t* __restrict__ tk) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < ntiles; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t W0 = q * kVl4T;
        int64_t lo = 0, hi = K;
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (cw[mid] <= W0) lo = mid; else hi = mid;
        }
        tk[q] = lo;
    }
}

__global__ void k_vl4_nz(const int64_t* __restrict__ wc, int64_t mv, int64_t* __restrict__ fl) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < mv; r += (int64_t)gridDim.x * blockDim.x)
        fl[r] = wc[r] ? 1 : 0;
}

__global__ void k_vl4_compact(const uint64_t* __restrict__ key, const uint32_t* __restrict__ tg, int64_t mv,
                              const int64_t* __restrict__ off, const int64_t* __restrict__ wc,
                              const int64_t* __restrict__ wpre, const int64_t* __restrict__ cpos,
                              int64_t* __restrict__ cw, int64_t* __restrict__ coy, uint32_t* __restrict__ ca) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < mv; r += (int64_t)gridDim.x * blockDim.x) {
        if (!wc[r]) continue;
        const int64_t j = cpos[r];
        cw[j] = wpre[r];
        coy[j] = off[tg[r]];
        ca[j] = (uint32_t)(key[r] >> 24);
    }
}

// inclusive block scan of one value per thread (kVl4B threads), op = sum or max
template <bool MAX>
__device__ __forceinline__ uint32_t vl4_scan(uint32_t v, uint32_t* wtot, uint32_t& excl) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x = MAX ? max(x, y) : x + y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    const uint32_t xp = __shfl_up(x, 1, 64);  // every lane active
    uint32_t pre = lane > 0 ? xp : 0u;
    for (int q = 0; q < wave; ++q) pre = MAX ? max(pre, wtot[q]) : pre + wtot[q];
    excl = pre;
    uint32_t all = 0;
    for (int q = 0; q < kVl4B / 64; ++q) all = MAX ? max(all, wtot[q]) : all + wtot[q];
    __syncthreads();  // wtot is reused by the next scan
    return all;
}

__global__ void __launch_bounds__(kVl4B) k_vl4_wedges(const int64_t* __restrict__ cw, const int64_t* __restrict__ coy,
                                                     const uint32_t* __restrict__ ca, const int64_t* __restrict__ tk,
                                                     int64_t K, int64_t total,
                                                     const uint32_t* __restrict__ tg, const uint32_t* __restrict__ isrc,
                                                     const int64_t* __restrict__ ioff,
                                                     unsigned long long* __restrict__ T14) {
    __shared__ int64_t soy[kVl4T];  // off[y] of the tile's k-th relationship minus its first wedge's tile position
    __shared__ uint32_t sa[kVl4T];
    __shared__ uint16_t own[kVl4T];  // wedge -> its relationship (tile-local k)
    __shared__ uint32_t sl[kVl4L];
    __shared__ uint32_t wtot[kVl4B / 64];
    const int t = threadIdx.x;
    for (int64_t W0 = (int64_t)blockIdx.x * kVl4T; W0 < total; W0 += (int64_t)gridDim.x * kVl4T) {  // block-uniform
        for (int i = t; i < kVl4T; i += kVl4B) own[i] = 0;
        __syncthreads();
        const int64_t k0 = tk[W0 / kVl4T], nt = min((int64_t)kVl4T, total - W0);
        for (int i = t; i < kVl4T && k0 + i < K; i += kVl4B) {
            const int64_t w = cw[k0 + i];
            if (i > 0 && w >= W0 + nt) break;  // past the tile (starts ascend)
            soy[i] = coy[k0 + i] - (w - W0);  // wedge at tile position i: y's out-list entry soy[k] + i
            sa[i] = ca[k0 + i];
            if (i > 0) own[w - W0] = (uint16_t)i;
        }
        __syncthreads();
        // fill forward: own[i] = max(own[0..i]) (the starts ascend with k); thread t holds positions 4t..4t+3
        uint32_t v[kVl4I];
        uint32_t m = 0;
#pragma unroll
        for (int j = 0; j < kVl4I; ++j) {
            m = max(m, (uint32_t)own[t * kVl4I + j]);
            v[j] = m;
        }
        uint32_t pre;
        vl4_scan<true>(m, wtot, pre);
#pragma unroll
        for (int j = 0; j < kVl4I; ++j) own[t * kVl4I + j] = (uint16_t)max(v[j], pre);
        __syncthreads();
        // every wedge's closing source p first (the lane's kVl4I loads in flight together)
        uint32_t pv[kVl4I];
        int kv[kVl4I];
#pragma unroll
        for (int j = 0; j < kVl4I; ++j) {
            const int i = t + j * kVl4B;
            kv[j] = -1;
            pv[j] = 0;
            if (i < nt) {
                const int k = own[i];
                kv[j] = k;
                pv[j] = tg[soy[k] + i];
            }
        }
        // a tile of one start whose in-list fits: the list into LDS, the searches there
        const uint32_t a0 = sa[0];
        const int64_t l0 = ioff[a0], ln = ioff[a0 + 1] - l0;
        if (sa[own[nt - 1]] == a0 && ln <= kVl4L) {  // block-uniform
            for (int i = t; i < ln; i += kVl4B) sl[i] = isrc[l0 + i];
            __syncthreads();
            unsigned long long c = 0;
#pragma unroll
            for (int j = 0; j < kVl4I; ++j) {
                if (kv[j] < 0) continue;
                const uint32_t p = pv[j];
                int l = 0, h = (int)ln;  // the first source >= p
                while (l < h) {
                    const int mid = (l + h) >> 1;
                    if (sl[mid] < p) l = mid + 1; else h = mid;
                }
                while (l < (int)ln && sl[l] == p) {
                    ++c;
                    ++l;
                }
            }
            if (c) atomicAdd(&T14[a0], c);
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int j = 0; j < kVl4I; ++j) {
            if (kv[j] < 0) continue;
            const uint32_t a = sa[kv[j]];
            const unsigned long long c = in_count(isrc, ioff[a], ioff[a + 1], pv[j]);
            if (c) atomicAdd(&T14[a], c);
        }
        __syncthreads();  // the tile's LDS is rewritten by the next
    }
}

__global__ void k_vl4_sum(int64_t n, Dom d, const unsigned long long* __restrict__ od,
                          const unsigned long long* __restrict__ s, const unsigned long long* __restrict__ W, Vl4 v,
                          unsigned long long* __restrict__ L4) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = d.lo + i;
        if (!aok(d, a)) {
            L4[i] = 0;
            continue;
        }
        const unsigned long long b = bok(d, a) ? 1 : 0, si = s[i], o = od[i];
        const unsigned long long pair1 = si * W[i] + v.P[i] + v.Q2[i];
        const unsigned long long pair2 = v.MAb[i] + v.ARb[i] + v.T14[i];
        const unsigned long long two = 2 * si * si * b + b * v.R1[i];
        const unsigned long long three = si * o + 2 * si * si * b + v.Q1[i];
        L4[i] = v.W4[i] - pair1 - pair2 + two + 2 * three - 6 * si * b;  // exact mod 2^64, the count fits
    }
}

// L4 (n u64): the per-node 4-hop counts, from od / s / W of the len-3 passes; ids below 2^24 - 1
void var_length4(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                 const Dom& d, const unsigned long long* od, const unsigned long long* sl, const unsigned long long* W,
                 unsigned long long* L4) {
    hipStream_t st = s->stream;
    const int64_t n = d.hi - d.lo;
    REQUIRE(n < (int64_t(1) << 24) - 1, CAPSMI_ERR_UNSUPPORTED, "fused var-length upper 4: at most 2^24 - 2 ids");
    KernelTimer kt(s, "varlen_4");
    int64_t mtot = 0;
    for (int i = 0; i < nt; ++i) mtot += ms[i] > 0 ? ms[i] : 0;
    const size_t nb = sizeof(unsigned long long) * (n > 0 ? n : 1);
    Buf acc = dev_alloc(nb * 10, s);
    HIP_CHECK(hipMemsetAsync(P<void>(acc), 0, nb * 10, st));
    unsigned long long* base = P<unsigned long long>(acc);
    const int64_t nw = (int64_t)(nb / sizeof(unsigned long long));
    Vl4 v{base, base + nw, base + 2 * nw, base + 3 * nw, base + 4 * nw, base + 5 * nw, base + 6 * nw, base + 7 * nw,
          base + 8 * nw, base + 9 * nw};
    if (mtot > 0) {  // the relationships sorted by (source, target), and the in-lists
        Buf key = dev_alloc(sizeof(uint64_t) * mtot, s);
        int64_t off0 = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_vl4_keys, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<uint64_t>(key) + off0);
            off0 += ms[i] > 0 ? ms[i] : 0;
        }
        std::vector<int> shifts;  // 48 key bits; the out-of-domain keys (~0) sort after every valid one
        for (int sh = 0; sh < 48; sh += 8) shifts.push_back(sh);
        radix_sort_keys(s, key, mtot, shifts);
        Buf off = dev_alloc(sizeof(int64_t) * (n + 2), s);
        hipLaunchKernelGGL(k_vl4_off, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(key), mtot, n, P<int64_t>(off));
        const int64_t mv = read_scalar(s, P<int64_t>(off) + n);  // the keys inside the domain
        if (mv > 0) {
            Buf wc = dev_alloc(sizeof(int64_t) * mv, s), wpre = dev_alloc(sizeof(int64_t) * (mv + 1), s);
            hipLaunchKernelGGL(k_vl4_wcount, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), mv, d, P<int64_t>(off),
                               P<int64_t>(wc));
            exclusive_scan_i64(P<int64_t>(wc), P<int64_t>(wpre), mv, s);
            // the in-lists: a stable sort of the keys by target (3 digits) keeps each target's sources ascending
            Buf ik = dev_alloc(sizeof(uint64_t) * mv, s), tg = dev_alloc(sizeof(uint32_t) * mv, s),
                isrc = dev_alloc(sizeof(uint32_t) * mv, s), ioff = dev_alloc(sizeof(int64_t) * (n + 2), s);
            HIP_CHECK(hipMemcpyAsync(P<void>(ik), P<void>(key), sizeof(uint64_t) * mv, hipMemcpyDeviceToDevice, st));
            radix_sort_keys(s, ik, mv, {0, 8, 16});
            hipLaunchKernelGGL(k_vl4_lists, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), P<uint64_t>(ik), mv,
                               P<uint32_t>(tg), P<uint32_t>(isrc));
            hipLaunchKernelGGL(k_vl4_ioff, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(ik), mv, n, P<int64_t>(ioff));
            ik = Buf();
            hipLaunchKernelGGL(k_vl4_a, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), mv, d, od, sl, W, v);
            hipLaunchKernelGGL(k_vl4_b, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), mv, d, od, P<uint32_t>(isrc),
                               P<int64_t>(ioff), v);
            hipLaunchKernelGGL(k_vl4_c, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), mv, v);
            // T14: the relationships with wedges, compacted
            Buf fl = dev_alloc(sizeof(int64_t) * mv, s), cpos = dev_alloc(sizeof(int64_t) * (mv + 1), s);
            hipLaunchKernelGGL(k_vl4_nz, dim3(grid(s, mv)), dim3(256), 0, st, P<int64_t>(wc), mv, P<int64_t>(fl));
            exclusive_scan_i64(P<int64_t>(fl), P<int64_t>(cpos), mv, s);
            fl = Buf();
            Buf cw = dev_alloc(sizeof(int64_t) * mv, s), coy = dev_alloc(sizeof(int64_t) * mv, s),
                ca = dev_alloc(sizeof(uint32_t) * mv, s);
            hipLaunchKernelGGL(k_vl4_compact, dim3(grid(s, mv)), dim3(256), 0, st, P<uint64_t>(key), P<uint32_t>(tg), mv,
                               P<int64_t>(off), P<int64_t>(wc), P<int64_t>(wpre), P<int64_t>(cpos), P<int64_t>(cw),
                               P<int64_t>(coy), P<uint32_t>(ca));
            int64_t kt[2];
            HIP_CHECK(hipMemcpyAsync(&kt[0], P<int64_t>(cpos) + mv, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(&kt[1], P<int64_t>(wpre) + mv, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            const int64_t K = kt[0], total = kt[1];
            if (total > 0) {
                const int64_t ntiles = (total + kVl4T - 1) / kVl4T;
                Buf tk = dev_alloc(sizeof(int64_t) * ntiles, s);
                hipLaunchKernelGGL(k_vl4_tiles, dim3(grid(s, ntiles)), dim3(256), 0, st, P<int64_t>(cw), K, ntiles,
                                   P<int64_t>(tk));
                hipLaunchKernelGGL(k_vl4_wedges, dim3(grid(s, ntiles * kVl4B)), dim3(kVl4B), 0, st, P<int64_t>(cw),
                                   P<int64_t>(coy), P<uint32_t>(ca), P<int64_t>(tk), K, total, P<uint32_t>(tg),
                                   P<uint32_t>(isrc), P<int64_t>(ioff), v.T14);
            }
        }
    }
    hipLaunchKernelGGL(k_vl4_sum, dim3(grid(s, n)), dim3(256), 0, st, n, d, od, sl, W, v, L4);
    HIP_CHECK(hipGetLastError());
}

}  // namespace varlen

// rows (a, count) of the fused var-length grouped count; returns the table's row count
int64_t var_length_count(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                         int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, int lower, int upper,
                         Buf& out_ids, Buf& out_cnt) {
    using namespace varlen;
    hipStream_t st = s->stream;
    const int64_t n = b_ok->hi - b_ok->lo;
    Dom d{P<uint32_t>(a_ok->words), P<uint32_t>(b_ok->words), b_ok->lo, b_ok->hi, a_ok->full ? 1 : 0,
          b_ok->full ? 1 : 0};
    const size_t nb = sizeof(uint64_t) * (n > 0 ? n : 1);
    Buf od = dev_alloc(nb, s), sl = dev_alloc(nb, s), W = dev_alloc(nb, s), T2 = dev_alloc(nb, s),
        T3 = dev_alloc(nb, s);
    const bool need3 = upper >= 3;
    // the (od, Y) words and their misfit flag (behind them), the candidate count: zeroed with the rest
    Buf pk = need3 ? dev_alloc(nb + sizeof(uint64_t), s) : Buf(), cand = need3 ? dev_alloc(sizeof(int64_t), s) : Buf();
    const int64_t nw = (int64_t)(nb / sizeof(uint64_t));
    zero_words(s, {{P<void>(od), nw}, {P<void>(sl), nw}, {P<void>(W), nw}, {P<void>(T2), nw}, {P<void>(T3), nw},
                   {need3 ? static_cast<void*>(P<unsigned long long>(pk) + nw) : nullptr, 1}, {P<void>(cand), 1}});
    int64_t mtot = 0;
    for (int i = 0; i < nt; ++i) mtot += ms[i] > 0 ? ms[i] : 0;
    if (n > 0 && n < (int64_t(1) << 24) && mtot > 0) {  // hkey: ids < 2^24 - 1
        // source-sliced passes: relationships grouped by source slice, LDS accumulators
        part::Layout L{};
        L.lo = d.lo;
        L.hi = d.hi;
        L.tbits = kVlBits;
        L.nt = (int)((n + kVlIds - 1) / kVlIds);
        L.ns = 1;
        L.sbits = 31;
        L.ncells = L.nt;
        ChunkPart cp, ct;
        {
            KernelTimer kt(s, "varlen_part");
            chunk_partition(s, srcs, dsts, ms, nt, true, L, s->num_cus, cp);
        }
        const ChunkWalk cw{P<uint2>(cp.pool), P<unsigned long long>(cp.meta), cp.order, cp.jst, cp.segbase, cp.ja, L.nt};
        const unsigned g = (unsigned)cp.g2;
        const size_t lds2 = 2 * sizeof(unsigned long long) * kVlIds;
        for (const void* f : {reinterpret_cast<const void*>(k_vl_deg), reinterpret_cast<const void*>(k_vl_w),
                              reinterpret_cast<const void*>(k_vl_t)})
            lds_attr(f, lds2);
        Buf ody, bw, hk, f2;  // hk: the pair table (keys, counts, overflow word)
        unsigned int* misfit = nullptr;
        RegionBloom bl{nullptr, 0, 0, 0};
        PairHash h{nullptr, nullptr, nullptr, 0};
        if (need3) {
            // filter of the directed pairs (RegionBloom): a region holds at most 2^20 bits (128 KiB of
            // LDS while k_vl_bset builds it), so a slice with more pairs gets 2^sublog regions, one
            // more k_vl_bset pass each
            KernelTimer kt(s, "varlen_rev");
            chunk_partition(s, srcs, dsts, ms, nt, false, L, s->num_cus, ct);
            const int64_t per_slice = (mtot + L.nt - 1) / L.nt;
            // 8 bits per pair (config CAPSMI_VL_BITS), in 2^sublog regions of <= 2^20 bits per slice
            const int64_t bits_per = s->cfg.vl_bits;
            int sublog = 0, rshift = 10;
            while (sublog < 3 && (bits_per * per_slice >> sublog) > (int64_t(1) << 20)) ++sublog;
            if (s->cfg.vl_sublog >= 0) sublog = s->cfg.vl_sublog;  // config CAPSMI_VL_SUBLOG
            while ((int64_t(1) << rshift) < (bits_per * per_slice >> sublog) && rshift < 20) ++rshift;
            const int64_t nreg = (int64_t)L.nt << sublog;
            const size_t rbytes = (size_t(1) << rshift) / 8;
            bw = dev_alloc(rbytes * nreg, s);
            bl = RegionBloom{P<uint32_t>(bw), (unsigned long long)((int64_t(1) << rshift) - 1), rshift, sublog};
            {
                Buf part = dev_alloc(rbytes * (((size_t)ct.g2 + L.nt) << sublog), s);
                const ChunkWalk tw{P<uint2>(ct.pool), P<unsigned long long>(ct.meta), ct.order, ct.jst, ct.segbase,
                                   ct.ja, L.nt};
                lds_attr(reinterpret_cast<const void*>(k_vl_bset), rbytes);
                hipLaunchKernelGGL(k_vl_bset, dim3((unsigned)ct.g2), dim3(kVlBlock), rbytes, st, tw, bl, P<uint4>(part));
                hipLaunchKernelGGL(k_vl_bmerge, dim3(grid(s, (int64_t)(rbytes / 16) * nreg)), dim3(256), 0, st, ct.jst,
                                   L.nt, ct.g2, P<uint4>(part), bl);
            }
        }
        // candidates of the reverse-multiplicity count: a list written by the degree walk (default), or
        // the F2 filter tested again in the T walk (config CAPSMI_VL_F2=1, the earlier form; the sharded form's)
        const bool use_f2 = s->cfg.vl_f2;
        Buf clist;
        {
            KernelTimer kt(s, "varlen_deg");
            Buf f2part;
            if (need3 && use_f2) {
                f2 = dev_alloc(sizeof(uint32_t) * kF2Words * (size_t)L.nt, s);
                f2part = dev_alloc(sizeof(uint32_t) * kF2Words * ((size_t)cp.g2 + L.nt), s);
            }
            if (need3 && !use_f2) clist = dev_alloc(sizeof(unsigned long long) * (size_t)mtot, s);
            hipLaunchKernelGGL(k_vl_deg, dim3(g), dim3(kVlBlock), lds2, st, cw, d.b, d.b_full, n, P<unsigned long long>(od),
                               P<unsigned long long>(sl), bl, P<uint4>(f2part), P<unsigned long long>(cand),
                               P<unsigned long long>(clist));
            if (need3 && use_f2) {
                const RegionBloom f2b{P<uint32_t>(f2), 0, 19, 0};  // kF2Words * 32 = 2^19 bits per slice
                hipLaunchKernelGGL(k_vl_bmerge, dim3(grid(s, (int64_t)(kF2Words / 4) * L.nt)), dim3(256), 0, st, cp.jst,
                                   L.nt, cp.g2, P<uint4>(f2part), f2b);
            }
        }
        if (need3) {
            // the candidate count (the pair table's size) is read back while the W walk runs
            read_scalar_async(s, P<int64_t>(cand));
            {
                KernelTimer kt(s, "varlen_w");
                Buf od32 = dev_alloc(sizeof(uint32_t) * (size_t)n, s);
                hipLaunchKernelGGL(k_vl_narrow, dim3(grid(s, n)), dim3(256), 0, st, P<unsigned long long>(od), n,
                                   P<uint32_t>(od32));
                hipLaunchKernelGGL(k_vl_w, dim3(g), dim3(kVlBlock), lds2 / 2, st, cw, n, P<uint32_t>(od32),
                                   P<unsigned long long>(W));
            }
            const int64_t nc = read_scalar_wait(s);
            int64_t cap = 1024;
            while (cap < 2 * nc) cap <<= 1;
            // keys (cap u64), counts (cap u32) and the overflow word in one zeroed block: one fill
            const size_t hbytes = (sizeof(unsigned long long) + sizeof(unsigned int)) * cap + 16;
            hk = dev_alloc(hbytes, s);
            HIP_CHECK(hipMemsetAsync(P<void>(hk), 0, hbytes, st));
            unsigned int* hcw = reinterpret_cast<unsigned int*>(P<unsigned long long>(hk) + cap);
            h = PairHash{P<unsigned long long>(hk), hcw, hcw + cap, (unsigned long long)(cap - 1)};
            if (!use_f2) {
                KernelTimer kt(s, "varlen_cand");
                hipLaunchKernelGGL(k_vl_cins, dim3(grid(s, nc)), dim3(256), 0, st, P<unsigned long long>(clist),
                                   P<unsigned long long>(cand), h);
            }
            ody = dev_alloc(2 * nb, s);
            misfit = reinterpret_cast<unsigned int*>(P<unsigned long long>(pk) + nw);
            hipLaunchKernelGGL(k_vl_y, dim3(grid(s, n)), dim3(256), 0, st, n, d.b, d.b_full, P<unsigned long long>(od),
                               P<unsigned long long>(W), P<unsigned long long>(sl), P<longlong2>(ody),
                               P<unsigned long long>(pk), misfit);
        }
        {
            KernelTimer kt(s, "varlen_t");
            const PairHash ht = use_f2 ? h : PairHash{nullptr, nullptr, nullptr, 0};  // list form: no inserts here
            hipLaunchKernelGGL(k_vl_t, dim3(g), dim3(kVlBlock), lds2, st, cw, d.a, d.a_full, n, P<unsigned long long>(od),
                               need3 ? P<longlong2>(ody) : nullptr, P<unsigned long long>(T2),
                               P<unsigned long long>(T3), bl, P<uint32_t>(f2), ht,
                               need3 ? P<unsigned long long>(pk) : nullptr, misfit);
        }
        if (need3) {
            KernelTimer kt(s, "varlen_recip");
            hipLaunchKernelGGL(k_vl_recip, dim3(grid(s, h.mask + 1)), dim3(256), 0, st, h, d.a, d.a_full, d.b, d.b_full,
                               P<unsigned long long>(T3), 0u, (uint32_t)n);
        }
        HIP_CHECK(hipGetLastError());
    } else {
    {
        KernelTimer kt(s, "varlen_deg");
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_deg, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(sl));
    }
    if (need3) {
        KernelTimer kt(s, "varlen_w");
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_w, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(W));
    }
    // m(b, a): multiplicity of the reverse relationship, from a hash table over (source, target) of all
    // relationship tables (concatenated key columns)
    Buf rev, counts;
    HashTable ht;
    if (need3 && mtot > 0) {
        Buf cs = dev_alloc(sizeof(int64_t) * mtot, s), cd = dev_alloc(sizeof(int64_t) * mtot, s);
        int64_t off = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] <= 0) continue;
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(cs) + off, srcs[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(cd) + off, dsts[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            off += ms[i];
        }
        KeyCols fwd, bwd;
        for (int k = 0; k < kMaxKeys; ++k) { fwd.data[k] = bwd.data[k] = nullptr; fwd.valid[k] = bwd.valid[k] = nullptr; }
        fwd.n = bwd.n = 2;
        fwd.data[0] = P<int64_t>(cs);
        fwd.data[1] = P<int64_t>(cd);
        bwd.data[0] = P<int64_t>(cd);
        bwd.data[1] = P<int64_t>(cs);
        Buf sor;
        KernelTimer kt(s, "varlen_rev");
        hash_build(s, fwd, mtot, false, ht, sor);
        hash_probe(s, bwd, fwd, mtot, ht, rev);
        counts = ht.slot_count;
    }
    {
        KernelTimer kt(s, "varlen_t");
        int64_t off = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_t, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(sl), P<unsigned long long>(W),
                                   need3 ? P<int64_t>(rev) + off : nullptr, need3 ? P<int64_t>(counts) : nullptr,
                                   need3 ? 1 : 0, P<unsigned long long>(T2), P<unsigned long long>(T3));
            off += ms[i];
        }
    }
    }  // atomic passes
    Buf L4;
    if (upper >= 4 && n > 0) {  // four hops: from od / sl / W
        L4 = dev_alloc(nb, s);
        var_length4(s, srcs, dsts, ms, nt, d, P<unsigned long long>(od), P<unsigned long long>(sl),
                    P<unsigned long long>(W), P<unsigned long long>(L4));
    }
    Buf cnt = dev_alloc(nb, s), flags = dev_alloc(n > 0 ? n : 1, s);
    hipLaunchKernelGGL(k_final, dim3(grid(s, n)), dim3(256), 0, st, n, d, lower, upper, P<unsigned long long>(od),
                       P<unsigned long long>(sl), P<unsigned long long>(T2), P<unsigned long long>(T3),
                       P<unsigned long long>(L4), P<int64_t>(cnt), P<uint8_t>(flags), (int64_t)0, n);
    HIP_CHECK(hipGetLastError());
    // rows (lo + i, cnt[i]) of the flagged a, written before the count is read
    return flags_to_rows(s, P<uint8_t>(flags), n, P<int64_t>(cnt), d.lo, out_ids, out_cnt);
}

}  // namespace capsmi

namespace capsmi {

// ---- sharded form (multi-GPU C5) ------------------------------------------------------
// Rank r owns the sources in [own_lo, own_hi) and holds their out-relationships ("out") plus the
// relationships into its owned ids from other ranks' sources ("in", exchanged once at ingest).
//   begin : out by source slice -> od, s of owned ids (0 elsewhere: the caller sums od over ranks);
//           R(a) for owned a from out + in (every reciprocal pair of an owned a is there both ways):
//           filter of out ∪ in by target, candidates by one flat pass (k_vl_flatcand), exact table,
//           k_vl_recip
//   mid   : W(v) of owned v from the summed od -> Y of owned v (0 elsewhere: the caller sums Y)
//   finish: T2, T3 of owned a from the summed od and Y -> rows of owned a
struct VarlenShard {
    capsmi_session* s = nullptr;
    varlen::Dom d{};
    int64_t n = 0, own_lo = 0, own_hi = 0;  // own range relative to d.lo
    int lower = 1, upper = 1;
    bool need3 = false;
    part::Layout L{};
    ChunkPart cp;  // out, by source slice
    Buf sl, W, T2, T3, ody, pk, bw, hk, hc, cand;
    int64_t* od = nullptr;  // caller buffers (n int64 each), summed over ranks by the caller
    int64_t* y = nullptr;
};

VarlenShard* varlen_shard_begin(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts,
                                const int64_t* ms, int nt, const int64_t* const* isrcs, const int64_t* const* idsts,
                                const int64_t* ims, int nin, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                int lower, int upper, int64_t own_lo, int64_t own_hi, int64_t* od) {
    using namespace varlen;
    using namespace part;
    hipStream_t st = s->stream;
    const int64_t n = b_ok->hi - b_ok->lo;
    REQUIRE(n > 0 && n < (int64_t(1) << 24), CAPSMI_ERR_UNSUPPORTED, "sharded var-length count needs < 2^24 ids");
    REQUIRE(own_lo >= b_ok->lo && own_lo <= own_hi && own_hi <= b_ok->hi, CAPSMI_ERR_ILLEGAL_ARGUMENT, "own range");
    auto v = std::make_unique<VarlenShard>();
    v->s = s;
    v->d = Dom{P<uint32_t>(a_ok->words), P<uint32_t>(b_ok->words), b_ok->lo, b_ok->hi, a_ok->full ? 1 : 0,
               b_ok->full ? 1 : 0};
    v->n = n;
    v->own_lo = own_lo - b_ok->lo;
    v->own_hi = own_hi - b_ok->lo;
    v->lower = lower;
    v->upper = upper;
    v->need3 = upper >= 3;
    v->od = od;
    const size_t nb = sizeof(uint64_t) * n;
    v->sl = dev_alloc(nb, s);
    v->W = dev_alloc(nb, s);
    v->T2 = dev_alloc(nb, s);
    v->T3 = dev_alloc(nb, s);
    if (v->need3) {  // finish()'s (od, Y) words + misfit flag, the candidate count: zeroed here with the rest
        v->pk = dev_alloc(nb + sizeof(uint64_t), s);
        v->cand = dev_alloc(sizeof(int64_t), s);
    }
    zero_words(s, {{od, n}, {P<void>(v->sl), n}, {P<void>(v->W), n}, {P<void>(v->T2), n}, {P<void>(v->T3), n},
                   {v->need3 ? static_cast<void*>(P<unsigned long long>(v->pk) + n) : nullptr, 1}, {P<void>(v->cand), 1}});
    Layout& L = v->L;
    L.lo = v->d.lo;
    L.hi = v->d.hi;
    L.tbits = kVlBits;
    L.nt = (int)((n + kVlIds - 1) / kVlIds);
    L.ns = 1;
    L.sbits = 31;
    L.ncells = L.nt;
    int64_t mout = 0, min_ = 0;
    for (int i = 0; i < nt; ++i) mout += ms[i] > 0 ? ms[i] : 0;
    for (int i = 0; i < nin; ++i) min_ += ims[i] > 0 ? ims[i] : 0;
    const size_t lds2 = 2 * sizeof(unsigned long long) * kVlIds;
    for (const void* f : {reinterpret_cast<const void*>(k_vl_deg), reinterpret_cast<const void*>(k_vl_w),
                          reinterpret_cast<const void*>(k_vl_t)})
        lds_attr(f, lds2);
    if (mout > 0) {
        {
            KernelTimer kt(s, "varlen_part");
            chunk_partition(s, srcs, dsts, ms, nt, true, L, s->num_cus, v->cp);
        }
        const ChunkWalk cw{P<uint2>(v->cp.pool), P<unsigned long long>(v->cp.meta), v->cp.order, v->cp.jst,
                           v->cp.segbase, v->cp.ja, L.nt};
        KernelTimer kt(s, "varlen_deg");
        hipLaunchKernelGGL(k_vl_deg, dim3((unsigned)v->cp.g2), dim3(kVlBlock), lds2, st, cw, v->d.b, v->d.b_full, n,
                           reinterpret_cast<unsigned long long*>(od), P<unsigned long long>(v->sl),
                           RegionBloom{nullptr, 0, 0, 0}, nullptr, nullptr, nullptr);
    }
    const int64_t mall = mout + min_;
    if (v->need3 && mall > 0) {
        std::vector<const int64_t*> as(srcs, srcs + nt), ad(dsts, dsts + nt);
        std::vector<int64_t> am(ms, ms + nt);
        for (int i = 0; i < nin; ++i) {
            as.push_back(isrcs[i]);
            ad.push_back(idsts[i]);
            am.push_back(ims[i]);
        }
        const int na = (int)as.size();
        ChunkPart ct;
        KernelTimer kt(s, "varlen_rev");
        std::unique_ptr<KernelTimer> sub(new KernelTimer(s, "vls_rev_part"));
        chunk_partition(s, as.data(), ad.data(), am.data(), na, false, L, s->num_cus, ct);
        sub.reset(new KernelTimer(s, "vls_rev_bloom"));
        const int64_t per_slice = (mall + L.nt - 1) / L.nt;
        int rshift = 10;
        while ((int64_t(1) << rshift) < int64_t(8) * per_slice && rshift < 20) ++rshift;
        const size_t rbytes = (size_t(1) << rshift) / 8;
        v->bw = dev_alloc(rbytes * L.nt, s);
        const RegionBloom bl{P<uint32_t>(v->bw), (unsigned long long)((int64_t(1) << rshift) - 1), rshift, 0};
        {
            Buf part = dev_alloc(rbytes * ((size_t)ct.g2 + L.nt), s);
            const ChunkWalk tw{P<uint2>(ct.pool), P<unsigned long long>(ct.meta), ct.order, ct.jst, ct.segbase, ct.ja,
                               L.nt};
            lds_attr(reinterpret_cast<const void*>(k_vl_bset), rbytes);
            hipLaunchKernelGGL(k_vl_bset, dim3((unsigned)ct.g2), dim3(kVlBlock), rbytes, st, tw, bl, P<uint4>(part));
            hipLaunchKernelGGL(k_vl_bmerge, dim3(grid(s, (int64_t)(rbytes / 16) * L.nt)), dim3(256), 0, st, ct.jst, L.nt,
                               ct.g2, P<uint4>(part), bl);
        }
        sub.reset(new KernelTimer(s, "vls_rev_cand"));
        // candidates (reverse maybe present) of out ∪ in: one flat pass over the columns into a list
        Buf& cand = v->cand;
        Buf clist = dev_alloc(sizeof(unsigned long long) * (size_t)mall, s);
        for (int i = 0; i < na; ++i)
            if (am[i] > 0)
                hipLaunchKernelGGL(k_vl_flatcand,
                                   dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((am[i] + kFcBlock * kFcIt - 1) /
                                                                                             (kFcBlock * kFcIt),
                                                                                         (int64_t)s->num_cus * 8))),
                                   dim3(kFcBlock), 0, st, as[i], ad[i], am[i], v->d.lo, bl,
                                   P<unsigned long long>(clist), P<unsigned long long>(cand));
        // the table sized on the device from the candidates' count (k_vl_hsize): allocated for the upper bound
        // (every relationship a candidate), cleared and scanned only as far as the count needs -- no host
        // round trip (round 4 read the count back: ~40 us of an idle device per rank and query)
        int64_t cap_max = 1024;
        while (cap_max < 2 * mall) cap_max <<= 1;
        v->hk = dev_alloc(sizeof(unsigned long long) * (cap_max + 1), s);  // + the device mask word
        v->hc = dev_alloc(sizeof(unsigned int) * (cap_max + 1), s);
        unsigned long long* dmask = P<unsigned long long>(v->hk) + cap_max;
        hipLaunchKernelGGL(k_vl_hsize, dim3(1), dim3(1), 0, st, P<unsigned long long>(cand), (unsigned long long)cap_max,
                           dmask);
        // any_ovf sits behind the slots' overflow words at ovf[cap]: the device-sized cap, so k_vl_hclear
        // clears it and the kernels find it through the mask (ovf + mask + 1)
        PairHash h{P<unsigned long long>(v->hk), P<unsigned int>(v->hc), nullptr, (unsigned long long)(cap_max - 1),
                   dmask};
        const unsigned gmax = (unsigned)std::min<int64_t>(grid(s, cap_max), (int64_t)s->num_cus * 8);
        hipLaunchKernelGGL(k_vl_hclear, dim3(gmax), dim3(256), 0, st, h);
        hipLaunchKernelGGL(k_vl_cins, dim3(gmax), dim3(256), 0, st, P<unsigned long long>(clist),
                           P<unsigned long long>(cand), h);
        sub.reset(new KernelTimer(s, "vls_rev_recip"));
        hipLaunchKernelGGL(k_vl_recip, dim3(gmax), dim3(256), 0, st, h, v->d.a, v->d.a_full, v->d.b, v->d.b_full,
                           P<unsigned long long>(v->T3), (uint32_t)v->own_lo, (uint32_t)v->own_hi);
    }
    HIP_CHECK(hipGetLastError());
    return v.release();
}

void varlen_shard_mid(VarlenShard* v, int64_t* y) {
    using namespace varlen;
    capsmi_session* s = v->s;
    hipStream_t st = s->stream;
    v->y = y;
    if (!v->need3) {  // no Y: the caller still sums the (zero) vector over the ranks
        HIP_CHECK(hipMemsetAsync(y, 0, sizeof(int64_t) * v->n, st));
        return;
    }  // else k_vl_yonly writes every entry
    if (v->cp.pool) {
        const ChunkWalk cw{P<uint2>(v->cp.pool), P<unsigned long long>(v->cp.meta), v->cp.order, v->cp.jst,
                           v->cp.segbase, v->cp.ja, v->L.nt};
        KernelTimer kt(s, "varlen_w");
        Buf od32 = dev_alloc(sizeof(uint32_t) * (size_t)v->n, s);
        hipLaunchKernelGGL(k_vl_narrow, dim3(grid(s, v->n)), dim3(256), 0, st,
                           reinterpret_cast<const unsigned long long*>(v->od), v->n, P<uint32_t>(od32));
        hipLaunchKernelGGL(k_vl_w, dim3((unsigned)v->cp.g2), dim3(kVlBlock), sizeof(unsigned long long) * kVlIds, st,
                           cw, v->n, P<uint32_t>(od32), P<unsigned long long>(v->W));
    }
    hipLaunchKernelGGL(k_vl_yonly, dim3(grid(s, v->n)), dim3(256), 0, st, v->n, v->d.b, v->d.b_full,
                       P<unsigned long long>(v->W), P<unsigned long long>(v->sl), reinterpret_cast<long long*>(y));
    HIP_CHECK(hipGetLastError());
}

int64_t varlen_shard_finish(VarlenShard* v, Buf& out_ids, Buf& out_cnt) {
    using namespace varlen;
    capsmi_session* s = v->s;
    hipStream_t st = s->stream;
    const int64_t n = v->n;
    unsigned int* misfit = nullptr;
    if (v->need3) {
        REQUIRE(v->y != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, "varlen shard: mid() before finish()");
        v->ody = dev_alloc(2 * sizeof(int64_t) * n, s);
        misfit = reinterpret_cast<unsigned int*>(P<unsigned long long>(v->pk) + n);  // zeroed in begin()
        hipLaunchKernelGGL(k_vl_pack, dim3(grid(s, n)), dim3(256), 0, st, n, reinterpret_cast<const long long*>(v->od),
                           reinterpret_cast<const long long*>(v->y), P<longlong2>(v->ody), P<unsigned long long>(v->pk),
                           misfit);
    }
    if (v->cp.pool) {
        const ChunkWalk cw{P<uint2>(v->cp.pool), P<unsigned long long>(v->cp.meta), v->cp.order, v->cp.jst,
                           v->cp.segbase, v->cp.ja, v->L.nt};
        KernelTimer kt(s, "varlen_t");
        hipLaunchKernelGGL(k_vl_t, dim3((unsigned)v->cp.g2), dim3(kVlBlock), 2 * sizeof(unsigned long long) * kVlIds, st,
                           cw, v->d.a, v->d.a_full, n, reinterpret_cast<const unsigned long long*>(v->od),
                           v->need3 ? P<longlong2>(v->ody) : nullptr, P<unsigned long long>(v->T2),
                           P<unsigned long long>(v->T3), RegionBloom{nullptr, 0, 0, 0}, nullptr,
                           PairHash{nullptr, nullptr, nullptr, 0}, v->need3 ? P<unsigned long long>(v->pk) : nullptr,
                           misfit);
    }
    Buf cnt = dev_alloc(sizeof(int64_t) * n, s), flags = dev_alloc(n, s);
    hipLaunchKernelGGL(k_final, dim3(grid(s, n)), dim3(256), 0, st, n, v->d, v->lower, v->upper,
                       reinterpret_cast<const unsigned long long*>(v->od), P<unsigned long long>(v->sl),
                       P<unsigned long long>(v->T2), P<unsigned long long>(v->T3), (const unsigned long long*)nullptr,
                       P<int64_t>(cnt), P<uint8_t>(flags), v->own_lo, v->own_hi);
    HIP_CHECK(hipGetLastError());
    return flags_to_rows(s, P<uint8_t>(flags), n, P<int64_t>(cnt), v->d.lo, out_ids, out_cnt);
}

void varlen_shard_free(VarlenShard* v) { delete v; }

}  // namespace capsmi
