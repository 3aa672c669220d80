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
constexpr int kBlock = 1024;                     // histogram and hop workgroups
constexpr int kItems = 8;                        // relationships per lane per tile
constexpr int kRepTile = kBlock * kItems;        // replica assignment unit (8192 rels, see TileWalk)
constexpr int kSBlock = 1024;                    // scatter workgroups (512 lanes x 4096 rels measured slower)
constexpr int kTile = kSBlock * kItems;          // relationships per scatter tile (8192)
constexpr int kUnroll = 8;                       // loads in flight per lane in the hops
constexpr int64_t kLoadMin = 8192;               // pull a source slice into LDS for >= this many rels
constexpr int kPad = 2 * 8192;                   // slack pairs after every pair array (load_pairs)
constexpr int kReps = 32;                        // cursor replicas per bucket (see TileWalk)

using Layout = PartLayout;

// Exclusive scan of in[0..n) into out[0..n) by a B-lane block; returns the total.
// `wtot` is B/64 words of LDS scratch.  Contains barriers: call from block-uniform code.
template <int B>
__device__ uint32_t block_exclusive_scan(const uint32_t* in, uint32_t* out, int n, uint32_t* wtot) {
    const int per = (n + B - 1) / B;
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
        uint32_t v = lane < B / 64 ? wtot[lane] : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(v, o, 64);
            if (lane >= o) v += y;
        }
        if (lane < B / 64) wtot[lane] = v;
    }
    __syncthreads();
    uint32_t pre = x - sum + (wave > 0 ? wtot[wave - 1] : 0u);
    for (int k = 0; k < per; ++k)
        if (b + k < n) {
            const uint32_t c = in[b + k];
            out[b + k] = pre;
            pre += c;
        }
    const uint32_t total = wtot[B / 64 - 1];
    __syncthreads();
    return total;
}

__device__ __forceinline__ int cell_of(const Layout& L, uint32_t s, uint32_t t) {
    return (int)(t >> kSliceBits) * L.ns + (int)(s >> L.sbits);
}

// Input tiles are dealt to kReps replicas (tile t -> replica t % kReps).  Each replica owns a
// contiguous share of every bucket, so a bucket's write cursor is advanced only by the tiles of
// one replica: with one cursor per bucket every tile of the whole input would serialise on the
// hottest bucket's atomic (R-MAT puts ~15 % of all relationships in one target slice).
// Block b works for replica b % kReps and takes that replica's tiles round-robin.
struct TileWalk {
    int r, q, bpr;
    __device__ TileWalk() : r(blockIdx.x % kReps), q(blockIdx.x / kReps), bpr(gridDim.x / kReps) {}
    __device__ int64_t tile(int64_t k) const { return (int64_t)r + (int64_t)kReps * ((int64_t)q + k * bpr); }
};

// Tile item u of this lane is relationship t0 + item_off<B>(u): lanes read 16-byte pairs of
// consecutive relationships (2 int64 per load, the calibrated streaming width), pair k of the
// tile at offset 2 * (k * B + lane).
template <int B>
__device__ __forceinline__ int item_off(int u) {
    return 2 * ((u >> 1) * B + (int)threadIdx.x) + (u & 1);
}

// Issue all of a tile's loads before any test: with a branch around each load the compiler
// waits for every load before issuing the next.  `vec` = both columns 16-byte aligned.
template <int B>
__device__ __forceinline__ void load_tile(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t t0,
                                          int64_t m, bool vec, int64_t (&sr)[kItems], int64_t (&tr)[kItems]) {
    const int64_t* __restrict__ sp = src + t0;  // wave-uniform bases, 32-bit lane offsets
    const int64_t* __restrict__ dp = dst + t0;
    if (vec && t0 + B * kItems <= m) {
        const longlong2* __restrict__ sv = reinterpret_cast<const longlong2*>(sp);
        const longlong2* __restrict__ dv = reinterpret_cast<const longlong2*>(dp);
#pragma unroll
        for (int k = 0; k < kItems / 2; ++k) {
            const longlong2 a = sv[k * B + (int)threadIdx.x], b = dv[k * B + (int)threadIdx.x];
            sr[2 * k] = a.x;
            sr[2 * k + 1] = a.y;
            tr[2 * k] = b.x;
            tr[2 * k + 1] = b.y;
        }
    } else {
        const int last = (int)(min(m - t0, (int64_t)B * kItems) - 1);
#pragma unroll
        for (int u = 0; u < kItems; ++u) {
            const int i = min(item_off<B>(u), last);
            sr[u] = sp[i];
            tr[u] = dp[i];
        }
    }
}

// The B * N pairs of a packed uint2 array starting at the even, wave-uniform index b, as 16-byte
// loads: this lane's item u is b + item_off<B>(u).  Pair arrays are allocated with kPad pairs of
// slack so a tile may run past the last pair; callers mask items outside their range.
template <int B, int N>
__device__ __forceinline__ void load_pairs(const uint2* __restrict__ in, int64_t b, uint2 (&p)[N]) {
    const uint4* __restrict__ v = reinterpret_cast<const uint4*>(in + b);
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
        const uint4 x = v[k * B + (int)threadIdx.x];
        p[2 * k] = make_uint2(x.x, x.y);
        p[2 * k + 1] = make_uint2(x.z, x.w);
    }
}

// pass 0: per-replica cell sizes (rels with an endpoint outside [lo, hi) can never match a node
// scan over that domain and are dropped here -- an inner join drops them the same way)
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8))) k_part_hist(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      int64_t m, Layout L, unsigned int* __restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) unsigned int h[];
    for (int i = threadIdx.x; i < L.ncells; i += kBlock) h[i] = 0;
    __syncthreads();
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const TileWalk w;
    for (int64_t k = 0;; ++k) {
        const int64_t t0 = w.tile(k) * kRepTile;
        if (t0 >= m) break;
        int64_t sr[kItems], tr[kItems];
        load_tile<kBlock>(src, dst, t0, m, vec, sr, tr);
#pragma unroll
        for (int u = 0; u < kItems; ++u) {
            const int64_t e = t0 + item_off<kBlock>(u);
            const uint64_t s = (uint64_t)(sr[u] - L.lo), t = (uint64_t)(tr[u] - L.lo);
            if (e < m && s < range && t < range) atomicAdd(&h[cell_of(L, (uint32_t)s, (uint32_t)t)], 1u);
        }
    }
    __syncthreads();
    unsigned int* out = counts + (size_t)w.r * L.ncells;
    for (int i = threadIdx.x; i < L.ncells; i += kBlock)
        if (h[i]) atomicAdd(&out[i], h[i]);
}

// offsets, one thread per cell: pre[r][c] = sum_{r' < r} cnt[r'][c], tot[c] = sum_r cnt[r][c]
__global__ void k_cell_prefix(const unsigned int* __restrict__ cnt, int ncells, int64_t* __restrict__ pre,
                              int64_t* __restrict__ tot) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    int64_t run = 0;
    for (int r = 0; r < kReps; ++r) {
        pre[(size_t)r * ncells + c] = run;
        run += cnt[(size_t)r * ncells + c];
    }
    tot[c] = run;
}

// one thread per pass-2 unit u = j * kReps + r (the pairs replica r put in target slice j):
// its start (= replica r's pass-1 cursor for slice j), length and tile count
__global__ void k_units(const unsigned int* __restrict__ cnt, const int64_t* __restrict__ pre,
                        const int64_t* __restrict__ coff, Layout L, int64_t* __restrict__ cur1,
                        int64_t* __restrict__ ustart, int64_t* __restrict__ ulen, int64_t* __restrict__ utiles) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= L.nt * kReps) return;
    const int j = u / kReps, r = u % kReps;
    int64_t before = 0, len = 0;
    for (int i = 0; i < L.ns; ++i) {
        const size_t c = (size_t)r * L.ncells + (size_t)j * L.ns + i;
        before += pre[c];
        len += cnt[c];
    }
    const int64_t st = coff[(size_t)j * L.ns] + before;
    cur1[(size_t)r * L.nt + j] = st;
    ustart[u] = st;
    ulen[u] = len;
    utiles[u] = len > 0 ? (st + len - (st & ~int64_t(1)) + kTile - 1) / kTile : 0;  // tiles on an even grid
}

// pass-2 cursors: cur2[r][c] = coff[c] + pre[r][c] (in place)
__global__ void k_add_coff(int64_t* __restrict__ pre, const int64_t* __restrict__ coff, int ncells) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)kReps * ncells) return;
    pre[i] += coff[i % ncells];
}

// tile -> unit map for pass 2, one thread per unit
__global__ void k_tile_unit(const int64_t* __restrict__ upre, int nunits, int* __restrict__ tile_unit) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= nunits) return;
    for (int64_t k = upre[u]; k < upre[u + 1]; ++k) tile_unit[k] = u;
}

// LDS carve-up shared by both scatters: stage[kTile] | base[nb] (u64) | cnt[nb] | loc[nb] | wtot[kSBlock/64]
__host__ __device__ constexpr size_t scatter_lds(int nb) {
    return sizeof(uint2) * kTile + sizeof(unsigned long long) * nb + sizeof(uint32_t) * (2 * nb + kSBlock / 64);
}

// Tile body: items (s, t, bucket) are in registers with their rank within the bucket; reserve
// each bucket's run with one atomic on the replica's cursor, regroup the tile in LDS, write the
// runs out.
__device__ __forceinline__ void scatter_tile(const uint2 (&pr)[kItems], uint32_t valid, const uint32_t (&rk)[kItems], int nb,
                                             unsigned long long* __restrict__ cursor, uint2* __restrict__ out,
                                             uint2* stage, unsigned long long* base, uint32_t* cnt, uint32_t* loc,
                                             uint32_t* wtot, bool by_target, int sbits) {
    for (int i = threadIdx.x; i < nb; i += kSBlock) {
        const uint32_t c = cnt[i];
        base[i] = c ? atomicAdd(&cursor[i], (unsigned long long)c) : 0ULL;
    }
    const uint32_t total = block_exclusive_scan<kSBlock>(cnt, loc, nb, wtot);
#pragma unroll
    for (int k = 0; k < kItems; ++k)
        if ((valid >> k) & 1u) {
            const int b = by_target ? (int)(pr[k].y >> kSliceBits) : (int)(pr[k].x >> sbits);
            stage[loc[b] + rk[k]] = pr[k];
        }
    __syncthreads();
    for (uint32_t idx = threadIdx.x; idx < total; idx += kSBlock) {
        const uint2 p = stage[idx];
        const int b = by_target ? (int)(p.y >> kSliceBits) : (int)(p.x >> sbits);
        out[base[b] + (idx - loc[b])] = p;
    }
    __syncthreads();
}

// pass 1: int64 (source, target) -> uint32 pairs grouped by target slice, replica-major within
// each slice; cursor = cur1[r][j]
__global__ void __launch_bounds__(kSBlock) __attribute__((amdgpu_waves_per_eu(8))) k_scatter_t(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      int64_t m, Layout L, unsigned long long* __restrict__ cur1,
                                                      uint2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.nt;
    uint2* stage = reinterpret_cast<uint2*>(smem);
    unsigned long long* base = smem + kTile;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + nb);
    uint32_t* loc = cnt + nb;
    uint32_t* wtot = loc + nb;
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const TileWalk w;
    unsigned long long* cursor = cur1 + (size_t)w.r * nb;
    for (int64_t k = 0;; ++k) {
      const int64_t r0 = w.tile(k) * kRepTile;
      if (r0 >= m) break;  // block-uniform
      for (int64_t t0 = r0; t0 < min(r0 + (int64_t)kRepTile, m); t0 += kTile) {
        for (int i = threadIdx.x; i < nb; i += kSBlock) cnt[i] = 0;
        __syncthreads();
        uint2 pr[kItems];
        uint32_t rk[kItems];
        uint32_t valid = 0;  // bit u: item u is kept
        {
            int64_t sr[kItems], tr[kItems];
            load_tile<kSBlock>(src, dst, t0, m, vec, sr, tr);
#pragma unroll
            for (int u = 0; u < kItems; ++u) {
                const int64_t e = t0 + item_off<kSBlock>(u);
                const uint64_t s = (uint64_t)(sr[u] - L.lo), t = (uint64_t)(tr[u] - L.lo);
                const bool ok = e < m && s < range && t < range;
                pr[u] = make_uint2((uint32_t)s, (uint32_t)t);
                valid |= (ok ? 1u : 0u) << u;
                rk[u] = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < kItems; ++u)
            if ((valid >> u) & 1u) rk[u] = atomicAdd(&cnt[pr[u].y >> kSliceBits], 1u);
        __syncthreads();
        scatter_tile(pr, valid, rk, nb, cursor, out, stage, base, cnt, loc, wtot, true, L.sbits);
      }
    }
}

// pass 2: unit u = (target slice j, replica r) -> the source cells of slice j; cursor cur2[r][j][*].
// Global tile k belongs to unit tile_unit[k] (upre[u] <= k < upre[u + 1]).
__global__ void __launch_bounds__(kSBlock) __attribute__((amdgpu_waves_per_eu(8))) k_scatter_s(const uint2* __restrict__ in, const int64_t* __restrict__ ustart,
                                                      const int64_t* __restrict__ ulen,
                                                      const int64_t* __restrict__ upre,
                                                      const int* __restrict__ tile_unit, int64_t ntiles, Layout L,
                                                      unsigned long long* __restrict__ cur2,
                                                      uint2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.ns;
    uint2* stage = reinterpret_cast<uint2*>(smem);
    unsigned long long* base = smem + kTile;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(base + nb);
    uint32_t* loc = cnt + nb;
    uint32_t* wtot = loc + nb;
    for (int64_t ck = blockIdx.x; ck < ntiles; ck += gridDim.x) {
        const int u = tile_unit[ck], j = u / kReps, r = u % kReps;
        const int64_t tb = (ustart[u] & ~int64_t(1)) + (ck - upre[u]) * kTile;  // even tile base
        const int64_t b0 = max(tb, ustart[u]), b1 = min(tb + (int64_t)kTile, ustart[u] + ulen[u]);
        for (int i = threadIdx.x; i < nb; i += kSBlock) cnt[i] = 0;
        __syncthreads();
        uint32_t rk[kItems];
        uint32_t valid = 0;
        uint2 pr[kItems];
        load_pairs<kSBlock, kItems>(in, tb, pr);
        const int lo = (int)(b0 - tb), hi = (int)(b1 - tb);  // 32-bit tile-relative bounds
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            const int e = item_off<kSBlock>(k);
            valid |= (e >= lo && e < hi ? 1u : 0u) << k;
            rk[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k)
            if ((valid >> k) & 1u) rk[k] = atomicAdd(&cnt[pr[k].x >> L.sbits], 1u);
        __syncthreads();
        scatter_tile(pr, valid, rk, nb, cur2 + (size_t)r * L.ncells + (size_t)j * nb, out, stage, base, cnt, loc,
                     wtot, false, L.sbits);
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
        auto visit = [&](const uint2 pr) {
            const uint32_t s = pr.x, t = pr.y;
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
        };
        for (int64_t cb = e0 & ~int64_t(1); cb < ce; cb += (int64_t)kBlock * kUnroll) {  // block-uniform, even
            uint2 p[kUnroll];
            load_pairs<kBlock, kUnroll>(pairs, cb, p);
            const int lo = (int)max(e0 - cb, (int64_t)0), hi = (int)min(ce - cb, (int64_t)kBlock * kUnroll);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int e = item_off<kBlock>(u);
                if (e >= lo && e < hi) visit(p[u]);
            }
        }
        e0 = ce;
        ++c;
        __syncthreads();  // the next cell may overwrite sl / flush tl
    }
    __syncthreads();
    flush_slice(tl, out, cur_j, gwords, tmask);
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
    using namespace part;
    hipStream_t st = s->stream;
    rp.L = make_layout(lo, hi);
    const Layout& L = rp.L;
    REQUIRE(L.nt <= kMaxTSlices && L.ncells <= kMaxCells, CAPSMI_ERR_INTERNAL, "layout too large");
    const int nunits = L.nt * kReps;
    // blocks: a multiple of kReps, about two 1024-lane blocks per CU
    const int grid = kReps * (int)std::max<int64_t>(1, (2 * (int64_t)s->num_cus + kReps - 1) / kReps);

    Buf cnt = dev_alloc(sizeof(unsigned int) * kReps * L.ncells, st);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(unsigned int) * kReps * L.ncells, st));
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        KernelTimer kt(s, "part_hist");
        hipLaunchKernelGGL(k_part_hist, dim3(grid), dim3(kBlock), sizeof(unsigned int) * L.ncells, st, srcs[i], dsts[i],
                           ms[i], L, P<unsigned int>(cnt));
    }
    // offsets, all on the device: cells, pass-1 cursors per (replica, slice), pass-2 units
    Buf pre = dev_alloc(sizeof(int64_t) * kReps * L.ncells, st);  // becomes cur2
    Buf tot = dev_alloc(sizeof(int64_t) * L.ncells, st);
    rp.boff = dev_alloc(sizeof(int64_t) * (L.ncells + 1), st);  // coff
    Buf cur1 = dev_alloc(sizeof(int64_t) * nunits, st);
    Buf units = dev_alloc(sizeof(int64_t) * (4 * (size_t)nunits + 1), st);  // ustart | ulen | utiles | upre
    int64_t* ustart = P<int64_t>(units);
    int64_t* ulen = ustart + nunits;
    int64_t* utiles = ulen + nunits;
    int64_t* upre = utiles + nunits;
    hipLaunchKernelGGL(k_cell_prefix, dim3((L.ncells + 255) / 256), dim3(256), 0, st, P<unsigned int>(cnt), L.ncells,
                       P<int64_t>(pre), P<int64_t>(tot));
    exclusive_scan_i64(P<int64_t>(tot), P<int64_t>(rp.boff), L.ncells, st);
    hipLaunchKernelGGL(k_units, dim3((nunits + 255) / 256), dim3(256), 0, st, P<unsigned int>(cnt), P<int64_t>(pre),
                       P<int64_t>(rp.boff), L, P<int64_t>(cur1), ustart, ulen, utiles);
    hipLaunchKernelGGL(k_add_coff, dim3((unsigned)(((int64_t)kReps * L.ncells + 255) / 256)), dim3(256), 0, st,
                       P<int64_t>(pre), P<int64_t>(rp.boff), L.ncells);
    exclusive_scan_i64(utiles, upre, nunits, st);
    HIP_CHECK(hipGetLastError());
    int64_t kept = 0, ntiles = 0;
    HIP_CHECK(hipMemcpyAsync(&kept, P<int64_t>(rp.boff) + L.ncells, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&ntiles, upre + nunits, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    rp.kept = kept;
    const size_t bytes = sizeof(uint2) * ((rp.kept > 0 ? rp.kept : 1) + kPad);
    rp.pairs = dev_alloc(bytes, st);
    if (rp.kept == 0) return;
    Buf tmp = dev_alloc(bytes, st);
    const size_t lds1 = scatter_lds(L.nt), lds2 = scatter_lds(L.ns);
    allow_lds(k_scatter_t, lds1);
    allow_lds(k_scatter_s, lds2);
    Buf tmap = dev_alloc(sizeof(int) * (ntiles > 0 ? ntiles : 1), st);
    hipLaunchKernelGGL(k_tile_unit, dim3((nunits + 255) / 256), dim3(256), 0, st, upre, nunits, P<int>(tmap));
    // scatter blocks: kSBlock lanes, about two per CU, a multiple of kReps
    const int sgrid = kReps * (int)std::max<int64_t>(1, (2 * (int64_t)s->num_cus + kReps - 1) / kReps);
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        KernelTimer kt(s, "part_scatter_t");
        hipLaunchKernelGGL(k_scatter_t, dim3(sgrid), dim3(kSBlock), lds1, st, srcs[i], dsts[i], ms[i], L,
                           P<unsigned long long>(cur1), P<uint2>(tmp));
    }
    {
        KernelTimer kt(s, "part_scatter_s");
        hipLaunchKernelGGL(k_scatter_s, dim3(sgrid), dim3(kSBlock), lds2, st, P<uint2>(tmp), ustart, ulen, upre,
                           P<int>(tmap), ntiles, L, P<unsigned long long>(pre), P<uint2>(rp.pairs));
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
