// k_part.hip -- 2-D radix-partitioned relationship layout and LDS-resident 2-hop kernels.
//
// The 2-hop count(DISTINCT c) touches two id-indexed bitmaps per relationship: the frontier of
// the middle node (indexed by source) and the mark of the end node (indexed by target).  Over
// 2^26 ids each is 8 MiB, twice an XCD's L2, so in ingest order both are random cache traffic
// (the streaming kernels in k_graph.hip run at ~1/8 of HBM bandwidth for that reason).
//
// Layout: relationships are grouped into cells (target slice j, source slice i), j-major.  A
// target slice is 2^19 ids, whose bitmap (64 KiB) a workgroup keeps in LDS while it streams the
// slice's cells, so marks are LDS atomics; a source slice is 2^19 ids too when the domain allows
// (<= 128 x 128 cells), so a workgroup also pulls the frontier slice (64 KiB, from L2/MALL) into
// LDS before a large cell and every frontier test is an LDS read.  Target-side node filters
// (b_ok / c_ok) commute with the OR over relationships and are applied word-wise when a target
// slice is flushed, so the per-relationship work is one 8-byte load and two LDS accesses.
//
// Build: pass 0 counts cells (LDS histogram), pass 1 scatters (source, target) int64 pairs into
// target slices as packed uint32 pairs, pass 2 scatters each target slice into its source cells.
// Both scatters stage an 8192-relationship tile in LDS grouped by bucket, so the HBM writes are
// runs of whole cache lines rather than 8-byte scatters.
#include "capsmi_impl.h"

namespace capsmi {

namespace part {

constexpr int kSliceBits = 19;                   // 2^19 ids per slice = 64 KiB of LDS bitmap
constexpr int kSliceWords = 1 << (kSliceBits - 5);
constexpr int kMaxCells = 16384;                 // cell histogram = 64 KiB of LDS
constexpr int kMaxTSlices = 4096;                // domain <= 2^31 ids
constexpr int kBlock = 1024;
constexpr int kItems = 8;
constexpr int kTile = kBlock * kItems;           // relationships per scatter tile
constexpr int kUnroll = 4;                       // loads in flight per lane in the hops
constexpr int64_t kLoadMin = 8192;               // pull a source slice into LDS for >= this many rels

using Layout = PartLayout;

// Exclusive scan of in[0..n) into out[0..n) by a 1024-lane block; returns the total.
// `wtot` is 16 words of LDS scratch.  Contains barriers: call from block-uniform code.
__device__ uint32_t block_exclusive_scan(const uint32_t* in, uint32_t* out, int n, uint32_t* wtot) {
    const int per = (n + kBlock - 1) / kBlock;
    const int b = threadIdx.x * per;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t sum = 0;
    for (int k = 0; k < per; ++k)
        if (b + k < n) sum += in[b + k];
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint32_t v = lane < kBlock / 64 ? wtot[lane] : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(v, o, 64);
            if (lane >= o) v += y;
        }
        if (lane < kBlock / 64) wtot[lane] = v;
    }
    __syncthreads();
    uint32_t pre = x - sum + (wave > 0 ? wtot[wave - 1] : 0u);
    for (int k = 0; k < per; ++k)
        if (b + k < n) {
            const uint32_t c = in[b + k];
            out[b + k] = pre;
            pre += c;
        }
    const uint32_t total = wtot[kBlock / 64 - 1];
    __syncthreads();
    return total;
}

__device__ __forceinline__ int cell_of(const Layout& L, uint32_t s, uint32_t t) {
    return (int)(t >> kSliceBits) * L.ns + (int)(s >> L.sbits);
}

// Rank of this lane's item among the items of bucket `b` (b < 2^nbits), counted in LDS `cnt`.
// Lanes holding the same bucket are found with nbits ballots (one per key bit), then only the
// lowest such lane touches the LDS counter: a skewed key distribution (R-MAT puts ~15 % of all
// relationships in one target slice) would otherwise serialise up to 64 same-address atomics
// per wave instruction.  Must be called by all lanes of the wave (`act` masks the item).
__device__ __forceinline__ uint32_t wave_rank(int b, bool act, int nbits, uint32_t* cnt) {
    uint64_t mask = __ballot(act);
    for (int k = 0; k < nbits; ++k) {
        const bool bit = (b >> k) & 1;
        const uint64_t bb = __ballot(act && bit);
        mask &= bit ? bb : ~bb;
    }
    const int lane = threadIdx.x & 63;
    const int leader = mask ? __ffsll((unsigned long long)mask) - 1 : 0;
    uint32_t base = 0;
    if (act && lane == leader) base = atomicAdd(&cnt[b], (uint32_t)__popcll(mask));
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(mask & ((uint64_t(1) << lane) - 1));
}

// pass 0: cell sizes (rels with an endpoint outside [lo, hi) can never match a node scan
// over that domain and are dropped here -- an inner join drops them the same way)
__global__ void __launch_bounds__(kBlock) k_part_hist(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      int64_t m, Layout L, unsigned int* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) unsigned int h[];
    for (int i = threadIdx.x; i < L.ncells; i += kBlock) h[i] = 0;
    __syncthreads();
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    const int nbits = L.cbits;
    for (int64_t e0 = (int64_t)blockIdx.x * kBlock + (threadIdx.x & ~63); e0 < m; e0 += stride) {  // wave-uniform
        const int64_t e = e0 + (threadIdx.x & 63);
        bool act = false;
        int c = 0;
        if (e < m) {
            const uint64_t s = (uint64_t)(src[e] - L.lo), t = (uint64_t)(dst[e] - L.lo);
            act = s < range && t < range;
            if (act) c = cell_of(L, (uint32_t)s, (uint32_t)t);
        }
        (void)wave_rank(c, act, nbits, h);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < L.ncells; i += kBlock)
        if (h[i]) atomicAdd(&counts[i], h[i]);
}

// LDS carve-up shared by both scatters: stage[kTile] | base[nb] (u64) | cnt[nb] | loc[nb] | wtot[16]
__host__ __device__ constexpr size_t scatter_lds(int nb) {
    return sizeof(uint2) * kTile + sizeof(unsigned long long) * nb + sizeof(uint32_t) * (2 * nb + 16);
}

// Tile body: items (s, t, bucket) are in registers with their rank within the bucket; reserve
// each bucket's run with one global atomic, regroup the tile in LDS, write the runs out.
__device__ __forceinline__ void scatter_tile(const uint32_t (&sv)[kItems], const uint32_t (&tv)[kItems],
                                             const int (&bk)[kItems], const uint32_t (&rk)[kItems], int nb,
                                             unsigned long long* __restrict__ cursor, uint2* __restrict__ out,
                                             uint2* stage, unsigned long long* base, uint32_t* cnt, uint32_t* loc,
                                             uint32_t* wtot, bool by_target, int sbits) {
    for (int i = threadIdx.x; i < nb; i += kBlock) {
        const uint32_t c = cnt[i];
        base[i] = c ? atomicAdd(&cursor[i], (unsigned long long)c) : 0ULL;
    }
    const uint32_t total = block_exclusive_scan(cnt, loc, nb, wtot);
#pragma unroll
    for (int k = 0; k < kItems; ++k)
        if (bk[k] >= 0) stage[loc[bk[k]] + rk[k]] = make_uint2(sv[k], tv[k]);
    __syncthreads();
    for (uint32_t idx = threadIdx.x; idx < total; idx += kBlock) {
        const uint2 p = stage[idx];
        const int b = by_target ? (int)(p.y >> kSliceBits) : (int)(p.x >> sbits);
        out[base[b] + (idx - loc[b])] = p;
    }
    __syncthreads();
}

// pass 1: int64 (source, target) -> uint32 pairs grouped by target slice
__global__ void __launch_bounds__(kBlock) k_scatter_t(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      int64_t m, Layout L, unsigned long long* __restrict__ cursor,
                                                      uint2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.nt;
    uint2* stage = reinterpret_cast<uint2*>(smem);
    unsigned long long* base = smem + kTile;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + nb);
    uint32_t* loc = cnt + nb;
    uint32_t* wtot = loc + nb;
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    for (int64_t t0 = (int64_t)blockIdx.x * kTile; t0 < m; t0 += (int64_t)gridDim.x * kTile) {
        for (int i = threadIdx.x; i < nb; i += kBlock) cnt[i] = 0;
        __syncthreads();
        uint32_t sv[kItems], tv[kItems], rk[kItems];
        int bk[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            const int64_t e = t0 + (int64_t)k * kBlock + threadIdx.x;
            bk[k] = -1;
            sv[k] = tv[k] = rk[k] = 0;
            if (e < m) {
                const uint64_t s = (uint64_t)(src[e] - L.lo), t = (uint64_t)(dst[e] - L.lo);
                if (s < range && t < range) {
                    sv[k] = (uint32_t)s;
                    tv[k] = (uint32_t)t;
                    bk[k] = (int)(tv[k] >> kSliceBits);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k) rk[k] = wave_rank(bk[k], bk[k] >= 0, L.tbits_n, cnt);
        __syncthreads();
        scatter_tile(sv, tv, bk, rk, nb, cursor, out, stage, base, cnt, loc, wtot, true, L.sbits);
    }
}

// pass 2: each target slice's pairs -> its source cells.  Work unit = one tile of one target
// slice; chunk k of slice j is global chunk cpre[j] + k.
__global__ void __launch_bounds__(kBlock) k_scatter_s(const uint2* __restrict__ in, const int64_t* __restrict__ toff,
                                                      const int64_t* __restrict__ cpre, Layout L,
                                                      unsigned long long* __restrict__ cursor,
                                                      uint2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.ns;
    uint2* stage = reinterpret_cast<uint2*>(smem);
    unsigned long long* base = smem + kTile;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + nb);
    uint32_t* loc = cnt + nb;
    uint32_t* wtot = loc + nb;
    const int64_t nchunks = cpre[L.nt];
    for (int64_t ck = blockIdx.x; ck < nchunks; ck += gridDim.x) {
        int lo = 0, hi = L.nt;  // last j with cpre[j] <= ck
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (cpre[mid] <= ck) lo = mid; else hi = mid;
        }
        const int j = lo;
        const int64_t b0 = toff[j] + (ck - cpre[j]) * kTile;
        const int64_t b1 = min(b0 + (int64_t)kTile, toff[j + 1]);
        for (int i = threadIdx.x; i < nb; i += kBlock) cnt[i] = 0;
        __syncthreads();
        uint32_t sv[kItems], tv[kItems], rk[kItems];
        int bk[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            const int64_t e = b0 + (int64_t)k * kBlock + threadIdx.x;
            bk[k] = -1;
            sv[k] = tv[k] = rk[k] = 0;
            if (e < b1) {
                const uint2 p = in[e];
                sv[k] = p.x;
                tv[k] = p.y;
                bk[k] = (int)(p.x >> L.sbits);
            }
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k) rk[k] = wave_rank(bk[k], bk[k] >= 0, L.sbits_n, cnt);
        __syncthreads();
        scatter_tile(sv, tv, bk, rk, nb, cursor + (int64_t)j * nb, out, stage, base, cnt, loc, wtot, false, L.sbits);
    }
}

struct BitV {
    const uint32_t* w;  // words over [lo, hi) -- same domain as the layout
    int full;
};

__device__ __forceinline__ bool gbit(const uint32_t* w, uint32_t x) { return (w[x >> 5] >> (x & 31)) & 1u; }

__device__ __forceinline__ void lds_set(uint32_t* lds, uint32_t x) {
    const uint32_t bit = 1u << (x & 31);
    uint32_t* p = &lds[x >> 5];
    if (!(*p & bit)) atomicOr(p, bit);
}

// OR the block's target slice j into the global words, masked by the target-side node filter
__device__ __forceinline__ void flush_slice(const uint32_t* tl, uint32_t* g, int j, int64_t gwords, BitV mask) {
    const int64_t w0 = (int64_t)j * kSliceWords;
    for (int i = threadIdx.x; i < kSliceWords; i += kBlock) {
        const int64_t gw = w0 + i;
        if (gw >= gwords) break;
        uint32_t v = tl[i];
        if (v && !mask.full) v &= mask.w[gw];
        if (v) atomicOr(&g[gw], v);
    }
}

// One hop over the 2-D layout.  Block b streams relationships [b*per, (b+1)*per) of the
// j-major cell order.
//   HOP1: M(t) |= a_ok(s) for s != t; self-loops (a_ok(s) and b_ok(t)) -> S1, second one -> S2.
//         Target filter b_ok at flush.
//   HOP2: C(t) |= X1(s) for s != t, X2(s) for s == t.  Target filter c_ok at flush.
// `sb` is the per-relationship source bitmap (a_ok or X1); `tmask` the target filter.
template <bool HOP1, bool SRC_FULL>
__global__ void __launch_bounds__(kBlock) k_hop_2d(const uint2* __restrict__ pairs, const int64_t* __restrict__ coff,
                                                   int64_t kept, int64_t per, Layout L, BitV sb,
                                                   const uint32_t* __restrict__ X2, BitV tmask,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ S1,
                                                   uint32_t* __restrict__ S2, int64_t gwords) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* tl = lds;                // target slice marks
    uint32_t* sl = lds + kSliceWords;  // source slice frontier (when pulled)
    int64_t e0 = (int64_t)blockIdx.x * per;
    const int64_t e1 = min(e0 + per, kept);
    if (e0 >= e1) return;  // block-uniform
    int c = 0;
    {  // last cell with coff[c] <= e0
        int lo = 0, hi = L.ncells;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (coff[mid] <= e0) lo = mid; else hi = mid;
        }
        c = lo;
    }
    int cur_j = -1;
    const bool can_pull = !SRC_FULL && L.sbits == kSliceBits;
    while (e0 < e1) {
        while (coff[c + 1] <= e0) ++c;
        const int j = c / L.ns, i = c % L.ns;
        const int64_t ce = min(e1, coff[c + 1]);
        if (j != cur_j) {
            if (cur_j >= 0) {
                __syncthreads();
                flush_slice(tl, out, cur_j, gwords, tmask);
            }
            __syncthreads();
            for (int k = threadIdx.x; k < kSliceWords; k += kBlock) tl[k] = 0;
            cur_j = j;
        }
        const bool pull = can_pull && ce - e0 >= kLoadMin;
        if (pull) {
            const int64_t w0 = (int64_t)i * kSliceWords;
            for (int k = threadIdx.x; k < kSliceWords; k += kBlock) sl[k] = w0 + k < gwords ? sb.w[w0 + k] : 0u;
        }
        __syncthreads();
        const uint32_t tbase = (uint32_t)j << kSliceBits, sbase = (uint32_t)i << kSliceBits;
        for (int64_t e = e0 + threadIdx.x; e < ce; e += (int64_t)kBlock * kUnroll) {
            uint2 p[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t eu = e + (int64_t)u * kBlock;
                p[u] = eu < ce ? pairs[eu] : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t s = p[u].x, t = p[u].y;
                if (s == 0xFFFFFFFFu && t == 0xFFFFFFFFu) continue;
                if (s != t) {
                    const bool ok = SRC_FULL || (pull ? gbit(sl, s - sbase) : gbit(sb.w, s));
                    if (ok) lds_set(tl, t - tbase);
                } else if (HOP1) {  // rare: self-loops
                    if ((SRC_FULL || gbit(sb.w, s)) && (tmask.full || gbit(tmask.w, t))) {
                        const uint32_t bit = 1u << (t & 31);
                        const uint32_t old = atomicOr(&S1[t >> 5], bit);
                        if (old & bit) atomicOr(&S2[t >> 5], bit);
                    }
                } else {
                    if (gbit(X2, s)) lds_set(tl, t - tbase);
                }
            }
        }
        e0 = ce;
        ++c;
        __syncthreads();  // the next cell may overwrite sl / flush tl
    }
    __syncthreads();
    flush_slice(tl, out, cur_j, gwords, tmask);
}

inline int ceil_log2(uint64_t v) {
    int b = 0;
    while ((uint64_t(1) << b) < v) ++b;
    return b;
}

}  // namespace part

// ================================ host side =====================================================
static part::Layout make_layout(int64_t lo, int64_t hi) {
    part::Layout L;
    L.lo = lo;
    L.hi = hi;
    const uint64_t range = (uint64_t)(hi - lo);
    const uint64_t slice = uint64_t(1) << part::kSliceBits;
    L.nt = (int)((range + slice - 1) / slice);
    if (L.nt < 1) L.nt = 1;
    // source slices: 2^19 ids while nt * ns fits the cell histogram, coarser beyond that
    const uint64_t ns_max = (uint64_t)(part::kMaxCells / L.nt);
    L.sbits = part::kSliceBits;
    while (((range + (uint64_t(1) << L.sbits) - 1) >> L.sbits) > ns_max) ++L.sbits;
    L.ns = (int)((range + (uint64_t(1) << L.sbits) - 1) >> L.sbits);
    if (L.ns < 1) L.ns = 1;
    L.ncells = L.nt * L.ns;
    L.tbits_n = part::ceil_log2((uint64_t)L.nt);
    L.sbits_n = part::ceil_log2((uint64_t)L.ns);
    L.cbits = part::ceil_log2((uint64_t)L.ncells);
    return L;
}

template <typename K>
static void allow_lds(K kernel, size_t bytes) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)bytes));
}

void relpart_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                   int64_t lo, int64_t hi, RelPart& rp) {
    REQUIRE(hi > lo && (uint64_t)(hi - lo) <= (uint64_t(1) << 31), CAPSMI_ERR_UNSUPPORTED,
            "partitioned layout needs an id domain of at most 2^31 ids");
    hipStream_t st = s->stream;
    rp.L = make_layout(lo, hi);
    const part::Layout& L = rp.L;
    REQUIRE(L.nt <= part::kMaxTSlices && L.ncells <= part::kMaxCells, CAPSMI_ERR_INTERNAL, "layout too large");
    Buf counts = dev_alloc(sizeof(unsigned int) * L.ncells, st);
    HIP_CHECK(hipMemsetAsync(P<void>(counts), 0, sizeof(unsigned int) * L.ncells, st));
    const int64_t cap = (int64_t)s->num_cus;
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        int64_t g = (ms[i] + part::kBlock * 16 - 1) / (part::kBlock * 16);
        if (g > cap) g = cap;
        KernelTimer kt(s, "part_hist");
        hipLaunchKernelGGL(part::k_part_hist, dim3((unsigned)g), dim3(part::kBlock),
                           sizeof(unsigned int) * L.ncells, st, srcs[i], dsts[i], ms[i], L, P<unsigned int>(counts));
    }
    // offsets: cells (j-major), target slices, and pass-2 chunks per target slice
    std::vector<unsigned int> hc(L.ncells);
    HIP_CHECK(hipMemcpyAsync(hc.data(), P<void>(counts), sizeof(unsigned int) * L.ncells, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    // host block: [coff (ncells+1) | toff (nt+1) | cpre (nt+1)]
    std::vector<int64_t> hb((size_t)L.ncells + 1 + 2 * ((size_t)L.nt + 1), 0);
    int64_t* coff = hb.data();
    int64_t* toff = coff + L.ncells + 1;
    int64_t* cpre = toff + L.nt + 1;
    for (int c = 0; c < L.ncells; ++c) coff[c + 1] = coff[c] + hc[c];
    for (int j = 0; j <= L.nt; ++j) toff[j] = coff[(int64_t)j * L.ns];
    for (int j = 0; j < L.nt; ++j) cpre[j + 1] = cpre[j] + (toff[j + 1] - toff[j] + part::kTile - 1) / part::kTile;
    rp.kept = coff[L.ncells];
    rp.boff = dev_alloc(sizeof(int64_t) * hb.size(), st);
    HIP_CHECK(hipMemcpyAsync(P<void>(rp.boff), hb.data(), sizeof(int64_t) * hb.size(), hipMemcpyHostToDevice, st));
    // scatter cursors start at the bucket offsets
    Buf cur = dev_alloc(sizeof(int64_t) * ((size_t)L.ncells + L.nt), st);
    HIP_CHECK(hipMemcpyAsync(P<void>(cur), toff, sizeof(int64_t) * L.nt, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(P<int64_t>(cur) + L.nt, coff, sizeof(int64_t) * L.ncells, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));  // host vectors go out of scope
    const size_t bytes = sizeof(uint2) * (rp.kept > 0 ? rp.kept : 1);
    Buf tmp = dev_alloc(bytes, st);
    rp.pairs = dev_alloc(bytes, st);
    if (rp.kept == 0) return;
    const size_t lds1 = part::scatter_lds(L.nt), lds2 = part::scatter_lds(L.ns);
    allow_lds(part::k_scatter_t, lds1);
    allow_lds(part::k_scatter_s, lds2);
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        int64_t g = (ms[i] + part::kTile - 1) / part::kTile;
        if (g > cap * 2) g = cap * 2;
        KernelTimer kt(s, "part_scatter_t");
        hipLaunchKernelGGL(part::k_scatter_t, dim3((unsigned)g), dim3(part::kBlock), lds1, st, srcs[i], dsts[i], ms[i],
                           L, P<unsigned long long>(cur), P<uint2>(tmp));
    }
    {
        int64_t g = cpre[L.nt];
        if (g > cap * 2) g = cap * 2;
        KernelTimer kt(s, "part_scatter_s");
        hipLaunchKernelGGL(part::k_scatter_s, dim3((unsigned)g), dim3(part::kBlock), lds2, st, P<uint2>(tmp),
                           P<int64_t>(rp.boff) + L.ncells + 1, P<int64_t>(rp.boff) + L.ncells + 1 + L.nt + 1, L,
                           P<unsigned long long>(cur) + L.nt, P<uint2>(rp.pairs));
    }
    HIP_CHECK(hipGetLastError());
}

template <bool HOP1, bool SRC_FULL>
static void launch_hop(capsmi_session* s, const RelPart& rp, part::BitV sb, const uint32_t* X2, part::BitV tmask,
                       uint32_t* out, uint32_t* S1, uint32_t* S2, int64_t gwords) {
    const size_t lds = sizeof(uint32_t) * 2 * part::kSliceWords;
    auto k = part::k_hop_2d<HOP1, SRC_FULL>;
    allow_lds(k, lds);
    // one 128 KiB-LDS block per CU at a time; a few rounds of blocks, equal relationship shares
    const int64_t blocks = (int64_t)s->num_cus * 4;
    int64_t per = (rp.kept + blocks - 1) / blocks;
    if (per < part::kBlock * part::kUnroll) per = part::kBlock * part::kUnroll;
    const int64_t g = (rp.kept + per - 1) / per;
    hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(part::kBlock), lds, s->stream, P<uint2>(rp.pairs),
                       P<int64_t>(rp.boff), rp.kept, per, rp.L, sb, X2, tmask, out, S1, S2, gwords);
    HIP_CHECK(hipGetLastError());
}

void relpart_hop1(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* M,
                  uint32_t* S1, uint32_t* S2) {
    REQUIRE(a->lo == rp.L.lo && a->hi == rp.L.hi && b->lo == rp.L.lo && b->hi == rp.L.hi, CAPSMI_ERR_UNSUPPORTED,
            "partitioned 2-hop needs node scans over the layout's id domain");
    if (rp.kept == 0) return;
    const part::BitV av{P<uint32_t>(a->words), a->full ? 1 : 0}, bv{P<uint32_t>(b->words), b->full ? 1 : 0};
    KernelTimer kt(s, "hop1");
    if (a->full)
        launch_hop<true, true>(s, rp, av, nullptr, bv, M, S1, S2, b->nwords);
    else
        launch_hop<true, false>(s, rp, av, nullptr, bv, M, S1, S2, b->nwords);
}

void relpart_hop2(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* c, const uint32_t* X1, const uint32_t* X2,
                  uint32_t* C) {
    REQUIRE(c->lo == rp.L.lo && c->hi == rp.L.hi, CAPSMI_ERR_UNSUPPORTED,
            "partitioned 2-hop needs node scans over the layout's id domain");
    if (rp.kept == 0) return;
    const part::BitV xv{X1, 0}, cv{P<uint32_t>(c->words), c->full ? 1 : 0};
    KernelTimer kt(s, "hop2");
    launch_hop<false, false>(s, rp, xv, X2, cv, C, nullptr, nullptr, c->nwords);
}

}  // namespace capsmi
