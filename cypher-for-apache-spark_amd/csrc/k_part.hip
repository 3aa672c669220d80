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
#include <map>
#include <mutex>
#include "part_common.h"

namespace capsmi {

namespace part {
// Cache policies measured at C3 (round 6, alternating libraries on one box; default policy everywhere else):
// non-temporal pass-1 loads 5.23 -> 5.50 ms, non-temporal pass-1 stores 5.23 -> 5.28, non-temporal pass-2 chunk
// loads 3.56 -> 3.60 (hop 2 1.49 -> 1.61), non-temporal pass-2 layout stores 3.56 -> 3.69 with hop 2 1.49 -> 1.36
// (the step unchanged).  The hops' pair loads stay non-temporal.

// ---- pass 1: int64 (source, target) -> packed pairs in per-workgroup chunks of one target slice ------
//
// No counting pass: every workgroup keeps one open chunk (kCh pairs) per target slice and appends
// its tiles' runs to it; a full chunk is retired and the next one taken from the workgroup's own
// range of the pool (a block with T tiles fills at most T chunks and leaves at most one open per
// slice, so T + nt chunks suffice and no global atomic sits in the tile loop).  Chunk metadata
// records (slice, fill); fill 0 = unused.  Each open chunk also counts its pairs per source slice
// (16-bit LDS counters, nt x ns of them = one per 2-D cell), written out as the chunk's cell
// histogram when it is retired; pass 2 derives exact output offsets from those.  The next tile's
// loads are issued before this tile is regrouped and written.



__host__ __device__ constexpr size_t scatter1_lds(int nb, int ns, int block = kP1Block, int tile = kP1Tile) {
    return sizeof(uint2) * tile + sizeof(uint32_t) * ((size_t)nb * hist_words(ns) + 7 * (size_t)nb + block / 64 + 4);
}

// chunks per pass-1 block: tiles of the busiest block + one open chunk per slice
__host__ __device__ inline int64_t chunks_per_block(int64_t m, int64_t grid, int nt, int64_t tile = kP1Tile) {
    return ((m + tile - 1) / tile + grid - 1) / grid + nt;
}

__device__ __forceinline__ void hist_add(uint32_t* H, int hw, int b, uint32_t i) {
    atomicAdd(&H[b * hw + (int)(i >> 1)], 1u << ((i & 1u) * 16u));
}

template <int B, int IT, int MINW, bool NTS>  // MINW: waves per SIMD to fit
__global__ void __launch_bounds__(B, MINW) k_scatter_c(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                       int64_t m, Layout L, int swap, int64_t chunk0, size_t trash,
                                                       uint2* __restrict__ pool, unsigned long long* __restrict__ cmeta,
                                                       uint32_t* __restrict__ chist) {
    constexpr int T = B * IT;
    static_assert(T <= kCh, "a pass-1 run must span at most two chunks");
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.nt, hw = hist_words(L.ns);
    uint2* stage = reinterpret_cast<uint2*>(smem);
    uint32_t* H = reinterpret_cast<uint32_t*>(stage + T);  // nb rows of hw words: open chunks' cell counts
    uint32_t* cnt = H + (size_t)nb * hw;  // this tile's run length per slice
    uint32_t* loc = cnt + nb;             // run start in the stage
    uint32_t* ph = loc + nb;              // open chunk per slice (kNone: none yet) ...
    uint32_t* fl = ph + nb;               // ... and its fill, both as of the start of the tile
    uint32_t* p1 = fl + nb;               // chunk opened by this tile's run (kNone: the run fits)
    uint32_t* opened = p1 + nb;           // slices that opened a chunk in this tile
    uint32_t* wtot = opened + nb;
    uint32_t* misc = wtot + B / 64;  // [0] chunks opened this tile, [1] next free chunk
    for (int i = threadIdx.x; i < nb * hw; i += B) H[i] = 0;
    for (int i = threadIdx.x; i < nb; i += B) {
        ph[i] = kNone;
        fl[i] = 0;
    }
    if (threadIdx.x == 0) {
        misc[0] = 0;
        misc[1] = (uint32_t)(chunk0 + (int64_t)blockIdx.x * chunks_per_block(m, gridDim.x, nb, T));
    }
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const int64_t stride = (int64_t)gridDim.x * T;
    int64_t sr[IT], tr[IT];
    int64_t t0 = (int64_t)blockIdx.x * T;
    if (t0 < m) load_tile<B>(src, dst, t0, m, vec, sr, tr);
    for (; t0 < m; t0 += stride) {  // block-uniform
        for (int i = threadIdx.x; i < nb; i += B) cnt[i] = 0;
        __syncthreads();
        uint2 pr[IT];
        uint32_t rk[IT];
        uint32_t valid = 0;
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int64_t e = t0 + item_off<B>(u);
            const uint64_t s = (uint64_t)(sr[u] - L.lo), t = (uint64_t)(tr[u] - L.lo);
            const bool ok = e < m && s < range && t < range;
            pr[u] = swap ? make_uint2((uint32_t)t, (uint32_t)s) : make_uint2((uint32_t)s, (uint32_t)t);
            valid |= (ok ? 1u : 0u) << u;
            rk[u] = 0;
        }
        if (t0 + stride < m) load_tile<B>(src, dst, t0 + stride, m, vec, sr, tr);  // prefetch
#pragma unroll
        for (int u = 0; u < IT; ++u)
            if ((valid >> u) & 1u) rk[u] = atomicAdd(&cnt[pr[u].y >> L.tbits], 1u);
        __syncthreads();
        const uint32_t total = block_exclusive_scan<B>(cnt, loc, nb, wtot);
        const uint32_t nf = misc[1];
        for (int i = threadIdx.x; i < nb; i += B) {  // a run that does not fit opens a chunk
            const uint32_t c = cnt[i];
            uint32_t np = kNone;
            if (c && (ph[i] == kNone || fl[i] + c > (uint32_t)kCh)) {
                const uint32_t k = atomicAdd(&misc[0], 1u);
                np = nf + k;
                opened[k] = (uint32_t)i;
            }
            p1[i] = np;
        }
#pragma unroll
        for (int u = 0; u < IT; ++u)
            if ((valid >> u) & 1u) stage[loc[pr[u].y >> L.tbits] + rk[u]] = pr[u];
        __syncthreads();
        // run item r of slice b: r < room -> open chunk ph[b] at fl[b] + r, else the opened chunk p1[b]
#pragma unroll
        for (int k = 0; k < IT; ++k) {  // unconditional stores (idx >= total -> trash chunk)
            const uint32_t idx = (uint32_t)(k * B + (int)threadIdx.x);
            const uint2 p = stage[idx];
            const int b = min((int)(p.y >> L.tbits), nb - 1);  // stale stage entries past `total`
            const uint32_t r = idx - loc[b], o = ph[b], room = o == kNone ? 0u : (uint32_t)kCh - fl[b];
            const bool first = r < room;
            if (idx < total && first) hist_add(H, hw, b, p.x >> L.sbits);
            const size_t at = idx >= total ? trash + threadIdx.x
                            : first       ? (size_t)o * kCh + fl[b] + r
                                          : (size_t)p1[b] * kCh + (r - room);
            if (NTS)
                __builtin_nontemporal_store(*reinterpret_cast<const unsigned long long*>(&p),
                                            reinterpret_cast<unsigned long long*>(pool + at));
            else
                pool[at] = p;
        }
        const uint32_t nop = misc[0];
        if (nop) {  // block-uniform: retire the filled chunks (histogram row out), count the runs' tails
            __syncthreads();
            for (uint32_t x = threadIdx.x; x < nop * (uint32_t)hw; x += B) {
                const int b = (int)opened[x / hw], w = (int)(x % hw);
                if (ph[b] != kNone) {
                    chist[(size_t)ph[b] * hw + w] = H[b * hw + w];
                    H[b * hw + w] = 0;
                }
            }
            __syncthreads();
            for (uint32_t k = 0; k < nop; ++k) {
                const int b = (int)opened[k];
                const uint32_t room = ph[b] == kNone ? 0u : (uint32_t)kCh - fl[b];
                for (uint32_t r = room + threadIdx.x; r < cnt[b]; r += B)
                    hist_add(H, hw, b, stage[loc[b] + r].x >> L.sbits);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nb; i += B) {  // advance the open chunks
            const uint32_t c = cnt[i];
            if (!c) continue;
            if (p1[i] == kNone) {
                fl[i] += c;
            } else {
                if (ph[i] != kNone) cmeta[ph[i]] = chunk_meta(i, (uint32_t)kCh);
                fl[i] = ph[i] == kNone ? c : fl[i] + c - (uint32_t)kCh;
                ph[i] = p1[i];
            }
        }
        if (threadIdx.x == 0) {
            misc[1] += misc[0];
            misc[0] = 0;
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += B)
        if (ph[i] != kNone) cmeta[ph[i]] = chunk_meta(i, fl[i]);
    for (int x = threadIdx.x; x < nb * hw; x += B) {
        const uint32_t p = ph[x / hw];
        if (p != kNone) chist[(size_t)p * hw + x % hw] = H[x];
    }
}

// ---- pass 1, whole-line variant (used when its LDS fits: <= 128 target slices at 2^19 ids) -------
// The chunk bookkeeping of a tile (scan of the run lengths, chunks opened) and the deferred part of
// the previous tile (retiring the chunks it filled, the histogram counts of its runs' tails,
// advancing the open chunks) run in wave 0 between the ranking and the regroup; run lengths are
// double-buffered by tile parity, so a tile takes three barriers.

// orders one wave's LDS accesses (wave 0 runs the bookkeeping alone)
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// Pass 1 writing whole 128-byte lines only.  A slice's run is appended behind the items its open
// chunk still holds back (fewer than kLine, kept in LDS): the combined sequence is staged, every
// complete line of it is stored, and the tail is held back again.  A line is then written once,
// by one wave, instead of in two pieces by two tiles, which the L2 may write back separately.
// The chunk contents and histograms equal k_scatter_c's up to the order within a chunk.
constexpr int kLine = 16;  // pairs per 128-byte line

__device__ __forceinline__ uint32_t held(uint32_t o, uint32_t f) { return o == kNone ? 0u : (f & (kLine - 1)); }

// wave 0: retire the chunks the previous tile filled, add its runs' tails to the opened chunks'
// histogram rows, advance the open chunks and clear the previous run lengths `cp`
__device__ __forceinline__ void p1l_settle(const Layout& L, int hw, const uint2* stage, uint32_t* H, uint32_t* cp,
                                           const uint32_t* loc, uint32_t* ph, uint32_t* fl, const uint32_t* p1,
                                           const uint32_t* opened, uint32_t* misc, unsigned long long* cmeta,
                                           uint32_t* chist) {
    const int nb = L.nt, lane = threadIdx.x & 63;
    const uint32_t nop = misc[0];
    for (uint32_t x = lane; x < nop * (uint32_t)hw; x += 64) {
        const int b = (int)opened[x / hw], w = (int)(x % hw);
        if (ph[b] != kNone) {
            chist[(size_t)ph[b] * hw + w] = H[b * hw + w];
            H[b * hw + w] = 0;
        }
    }
    wave_lds_order();
    for (uint32_t k = 0; k < nop; ++k) {  // items past the old chunk's room belong to the opened one
        const int b = (int)opened[k];
        const uint32_t h = held(ph[b], fl[b]);
        const uint32_t room = ph[b] == kNone ? 0u : (uint32_t)kCh - (fl[b] - h);
        for (uint32_t r = room + lane; r < h + cp[b]; r += 64) hist_add(H, hw, b, stage[loc[b] + r].x >> L.sbits);
    }
    wave_lds_order();
    for (int i = lane; i < nb; i += 64) {
        const uint32_t c = cp[i];
        if (!c) continue;
        if (p1[i] == kNone) {
            fl[i] += c;
        } else {
            if (ph[i] != kNone) cmeta[ph[i]] = chunk_meta(i, (uint32_t)kCh);
            fl[i] = ph[i] == kNone ? c : fl[i] + c - (uint32_t)kCh;
            ph[i] = p1[i];
        }
        cp[i] = 0;
    }
    if (lane == 0) {
        misc[1] += nop;
        misc[0] = 0;
    }
    wave_lds_order();
}

// wave 0: run starts `loc` of this tile (exclusive scan over each slice's staged sequence = held
// items + run), the chunks its runs open (p1, opened, misc[0]) and the staged total (misc[2])
__device__ __forceinline__ void p1l_plan(int nb, const uint32_t* cn, uint32_t* loc, const uint32_t* ph,
                                         const uint32_t* fl, uint32_t* p1, uint32_t* opened, uint32_t* misc) {
    const int lane = threadIdx.x & 63;
    const int per = (nb + 63) / 64, b0 = lane * per, b1 = min(b0 + per, nb);
    uint32_t sum = 0, need = 0;
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = cn[i];
        sum += c + held(ph[i], fl[i]);
        need += (c && (ph[i] == kNone || fl[i] + c > (uint32_t)kCh)) ? 1u : 0u;
    }
    const uint32_t is = wave_incl_scan(sum), in = wave_incl_scan(need);
    uint32_t pre = is - sum, k = in - need;
    const uint32_t nf = misc[1];
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = cn[i];
        loc[i] = pre;
        pre += c + held(ph[i], fl[i]);
        uint32_t np = kNone;
        if (c && (ph[i] == kNone || fl[i] + c > (uint32_t)kCh)) {
            np = nf + k;
            opened[k++] = (uint32_t)i;
        }
        p1[i] = np;
    }
    if (lane == 63) {
        misc[0] = in;
        misc[2] = is;
    }
    wave_lds_order();
}

__host__ __device__ constexpr size_t scatter1l_lds(int nb, int ns, int block, int tile) {
    return sizeof(uint2) * ((size_t)tile + (size_t)nb * (2 * kLine)) +
           sizeof(uint32_t) * ((size_t)nb * hist_words(ns) + 7 * (size_t)nb + block / 64 + 4);
}

template <int B, int IT, int MINW, bool NTL = false, bool NTS = false>
__global__ void __launch_bounds__(B, MINW) k_scatter_l(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                      int64_t m, Layout L, int swap, int64_t chunk0, size_t trash,
                                                      uint2* __restrict__ pool, unsigned long long* __restrict__ cmeta,
                                                      uint32_t* __restrict__ chist) {
    constexpr int T = B * IT;
    static_assert(T <= kCh && kCh % kLine == 0, "a pass-1 run must span at most two chunks");
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.nt, hw = hist_words(L.ns);
    uint2* stage = reinterpret_cast<uint2*>(smem);    // T + nb * kLine: runs behind their held items
    uint2* hold = stage + T + (size_t)nb * kLine;      // nb x kLine held items
    uint32_t* H = reinterpret_cast<uint32_t*>(hold + (size_t)nb * kLine);
    uint32_t* cnt = H + (size_t)nb * hw;
    uint32_t* loc = cnt + 2 * nb;
    uint32_t* ph = loc + nb;
    uint32_t* fl = ph + nb;  // logical fill of the open chunk (held items included)
    uint32_t* p1 = fl + nb;
    uint32_t* opened = p1 + nb;
    uint32_t* misc = opened + nb;
    for (int i = threadIdx.x; i < nb * hw; i += B) H[i] = 0;
    for (int i = threadIdx.x; i < nb; i += B) {
        cnt[i] = 0;
        cnt[nb + i] = 0;
        ph[i] = kNone;
        fl[i] = 0;
    }
    if (threadIdx.x == 0) {
        misc[0] = 0;
        misc[1] = (uint32_t)(chunk0 + (int64_t)blockIdx.x * chunks_per_block(m, gridDim.x, nb, T));
    }
    __syncthreads();
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const int64_t stride = (int64_t)gridDim.x * T;
    int64_t sr[IT], tr[IT];
    int64_t t0 = (int64_t)blockIdx.x * T;
    if (t0 < m) load_tile<B, NTL>(src, dst, t0, m, vec, sr, tr);
    int par = 0;
    bool pending = false;
    for (; t0 < m; t0 += stride, par ^= 1) {
        uint32_t* cn = cnt + par * nb;
        uint2 pr[IT];
        uint32_t rk[IT];
        uint32_t valid = 0;
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int64_t e = t0 + item_off<B>(u);
            const uint64_t s = (uint64_t)(sr[u] - L.lo), t = (uint64_t)(tr[u] - L.lo);
            const bool ok = e < m && s < range && t < range;
            pr[u] = swap ? make_uint2((uint32_t)t, (uint32_t)s) : make_uint2((uint32_t)s, (uint32_t)t);
            valid |= (ok ? 1u : 0u) << u;
            rk[u] = 0;
        }
        if (t0 + stride < m) load_tile<B, NTL>(src, dst, t0 + stride, m, vec, sr, tr);  // prefetch
#pragma unroll
        for (int u = 0; u < IT; ++u)
            if ((valid >> u) & 1u) rk[u] = atomicAdd(&cn[pr[u].y >> L.tbits], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {
            if (pending) p1l_settle(L, hw, stage, H, cnt + (par ^ 1) * nb, loc, ph, fl, p1, opened, misc, cmeta, chist);
            p1l_plan(nb, cn, loc, ph, fl, p1, opened, misc);
        }
        __syncthreads();
        pending = true;
        const uint32_t total = misc[2];
        for (int x = threadIdx.x; x < nb * kLine; x += B) {  // held items first
            const int b = x / kLine, k = x % kLine;
            if ((uint32_t)k < held(ph[b], fl[b])) stage[loc[b] + k] = hold[x];
        }
#pragma unroll
        for (int u = 0; u < IT; ++u)
            if ((valid >> u) & 1u) {
                const int b = pr[u].y >> L.tbits;
                stage[loc[b] + held(ph[b], fl[b]) + rk[u]] = pr[u];
            }
        __syncthreads();
        // staged item r of slice b: logical position w + r of chunk ph[b] (w = written prefix) while
        // it fits, else position r - room of the opened chunk p1[b]; positions below the chunk's
        // last complete line are stored, the rest held back
        for (uint32_t idx = threadIdx.x; idx < (uint32_t)(T + nb * kLine); idx += B) {
            const uint2 p = stage[idx];
            const int b = min((int)(p.y >> L.tbits), nb - 1);
            const uint32_t r = idx - loc[b], o = ph[b], f = fl[b], h = held(o, f), c = cn[b];
            const uint32_t w = f - h, room = o == kNone ? 0u : (uint32_t)kCh - w;
            const bool first = r < room;
            if (idx < total && first && r >= h) hist_add(H, hw, b, p.x >> L.sbits);
            // end of the sequence in the chunk it lands in, and that chunk's stored prefix
            const uint32_t end = first ? min(w + h + c, (uint32_t)kCh) : h + c - room;
            const uint32_t pos = first ? w + r : r - room;
            const uint32_t cut = end & ~(uint32_t)(kLine - 1);
            if (idx >= total) {
                break;  // idx only grows
            } else if (pos < cut) {
                uint2* d = pool + (size_t)(first ? o : p1[b]) * kCh + pos;
                if (NTS)
                    __builtin_nontemporal_store(*reinterpret_cast<const unsigned long long*>(&p),
                                                reinterpret_cast<unsigned long long*>(d));
                else
                    *d = p;
            } else {
                hold[b * kLine + (pos - cut)] = p;
            }
        }
    }
    __syncthreads();
    if (pending && threadIdx.x < 64)
        p1l_settle(L, hw, stage, H, cnt + (par ^ 1) * nb, loc, ph, fl, p1, opened, misc, cmeta, chist);
    __syncthreads();
    for (int x = threadIdx.x; x < nb * kLine; x += B) {  // held tails
        const int b = x / kLine, k = x % kLine;
        if ((uint32_t)k < held(ph[b], fl[b])) pool[(size_t)ph[b] * kCh + (fl[b] - held(ph[b], fl[b])) + k] = hold[x];
    }
    for (int i = threadIdx.x; i < nb; i += B)
        if (ph[i] != kNone) cmeta[ph[i]] = chunk_meta(i, fl[i]);
    for (int x = threadIdx.x; x < nb * hw; x += B) {
        const uint32_t p = ph[x / hw];
        if (p != kNone) chist[(size_t)p * hw + x % hw] = H[x];
    }
}

// this lane's item u of a 4-items-per-load walk starting at the 4-aligned index b: item u is
// b + 4 * ((u >> 2) * B + lane) + (u & 3)
template <int B>
__device__ __forceinline__ int item_off4(int u) {
    return 4 * ((u >> 2) * B + (int)threadIdx.x) + (u & 3);
}

// used chunks (fill > 0) grouped by target slice (order within a slice is arbitrary).  Each block
// takes kChunkPer chunks and aggregates per slice in LDS, so a slice counter sees one global atomic
// per block instead of one per chunk (≈10^5 chunks on ≈10^2 counters at C3).
constexpr int kChunkBlock = 1024, kChunkPer = 8192;

__global__ void __launch_bounds__(kChunkBlock) k_chunk_count(const unsigned long long* __restrict__ cmeta,
                                                             int64_t nchunks, int nt, int64_t* __restrict__ jcnt) {
    extern __shared__ uint32_t h[];  // nt
    for (int i = threadIdx.x; i < nt; i += kChunkBlock) h[i] = 0;
    __syncthreads();
    const int64_t q0 = (int64_t)blockIdx.x * kChunkPer, q1 = min(q0 + kChunkPer, nchunks);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += kChunkBlock)
        if (cmeta[q] >> 32) atomicAdd(&h[(uint32_t)cmeta[q]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += kChunkBlock)
        if (h[i]) atomicAdd(reinterpret_cast<unsigned long long*>(&jcnt[i]), (unsigned long long)h[i]);
}

__global__ void __launch_bounds__(kChunkBlock) k_chunk_place(const unsigned long long* __restrict__ cmeta,
                                                             int64_t nchunks, int nt,
                                                             unsigned long long* __restrict__ jcur,
                                                             uint32_t* __restrict__ order) {
    extern __shared__ uint32_t h[];  // nt counts, then nt bases (low 32 bits of the global cursor)
    uint32_t* base = h + nt;
    for (int i = threadIdx.x; i < nt; i += kChunkBlock) h[i] = 0;
    __syncthreads();
    const int64_t q0 = (int64_t)blockIdx.x * kChunkPer, q1 = min(q0 + kChunkPer, nchunks);
    for (int64_t q = q0 + threadIdx.x; q < q1; q += kChunkBlock)
        if (cmeta[q] >> 32) atomicAdd(&h[(uint32_t)cmeta[q]], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < nt; i += kChunkBlock) {
        base[i] = h[i] ? (uint32_t)atomicAdd(&jcur[i], (unsigned long long)h[i]) : 0u;  // order has < 2^32 entries
        h[i] = 0;
    }
    __syncthreads();
    for (int64_t q = q0 + threadIdx.x; q < q1; q += kChunkBlock)
        if (cmeta[q] >> 32) {
            const uint32_t j = (uint32_t)cmeta[q];
            order[base[j] + atomicAdd(&h[j], 1u)] = (uint32_t)q;
        }
}

// block exclusive scan of a[0, n) in place (1024 lanes, each a run of consecutive entries); returns the total
__device__ uint32_t block_scan_inplace(uint32_t* a, int n, uint32_t* wtot) {
    constexpr int B = kChunkBlock;
    const int per = (n + B - 1) / B, b0 = (int)threadIdx.x * per, b1 = min(b0 + per, n);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t sum = 0;
    for (int i = b0; i < b1; ++i) sum += a[i];
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
    for (int i = b0; i < b1; ++i) {
        const uint32_t c = a[i];
        a[i] = pre;
        pre += c;
    }
    const uint32_t total = wtot[B / 64 - 1];
    __syncthreads();
    return total;
}

// chunk_order in ONE launch for small pools (a rank's shard, C5's partitions): one workgroup counts the used
// chunks per slice, scans them (jst), places the chunks (order), and splits them into the g2 consumer blocks'
// segments (kseg -> segbase, ja) -- instead of a fill, two count / place launches, a copy and two scans
// (≈28 µs of launches and gaps per partition at a C5 shard of 2^22 relationships)
constexpr int64_t kOrder1Max = 32768;  // chunks; and nt <= kMaxTSlices, g2 <= 4096 (one workgroup over C3's 160K chunks: +0.13 ms)

__global__ void __launch_bounds__(kChunkBlock) k_chunk_order1(const unsigned long long* __restrict__ cmeta,
                                                              int64_t nchunks, int nt, int64_t g2,
                                                              int64_t* __restrict__ jst_out,
                                                              uint32_t* __restrict__ order,
                                                              int64_t* __restrict__ segbase, int* __restrict__ ja) {
    __shared__ uint32_t h[kMaxTSlices + 1];  // counts -> starts
    __shared__ uint32_t cur[kMaxTSlices];
    __shared__ uint32_t ks[4096 + 1];        // segments per consumer block -> their first index
    __shared__ uint32_t wtot[kChunkBlock / 64];
    for (int i = threadIdx.x; i <= nt; i += kChunkBlock) h[i] = 0;
    __syncthreads();
    for (int64_t q = threadIdx.x; q < nchunks; q += kChunkBlock)
        if (cmeta[q] >> 32) atomicAdd(&h[(uint32_t)cmeta[q]], 1u);
    __syncthreads();
    const uint32_t used = block_scan_inplace(h, nt, wtot);
    if (threadIdx.x == 0) h[nt] = used;
    __syncthreads();
    for (int i = threadIdx.x; i <= nt; i += kChunkBlock) {
        jst_out[i] = (int64_t)h[i];
        if (i < nt) cur[i] = h[i];
    }
    __syncthreads();
    for (int64_t q = threadIdx.x; q < nchunks; q += kChunkBlock)
        if (cmeta[q] >> 32) order[atomicAdd(&cur[(uint32_t)cmeta[q]], 1u)] = (uint32_t)q;
    // the consumers' split (k_seg_count / SegSplit): block w takes chunks [w per, (w + 1) per) of `order`
    const int64_t per = max((int64_t)1, ((int64_t)used + g2 - 1) / g2);
    for (int64_t w = threadIdx.x; w < g2; w += kChunkBlock) {
        const int64_t q0 = w * per, q1 = min(q0 + per, (int64_t)used);
        uint32_t k = 0;
        int a = 0;
        if (q0 < q1) {
            int lo = 0, hi = nt;  // last j with start <= q0, and with start <= q1 - 1
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if ((int64_t)h[mid] <= q0) lo = mid; else hi = mid;
            }
            a = lo;
            hi = nt;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if ((int64_t)h[mid] <= q1 - 1) lo = mid; else hi = mid;
            }
            k = (uint32_t)(lo - a + 1);
        }
        ks[w] = k;
        ja[w] = a;
    }
    __syncthreads();
    const uint32_t nseg = block_scan_inplace(ks, (int)g2, wtot);
    for (int64_t w = threadIdx.x; w < g2; w += kChunkBlock) segbase[w] = (int64_t)ks[w];
    if (threadIdx.x == 0) segbase[g2] = (int64_t)nseg;
}

// segments per block, ja(w)
__global__ void k_seg_count(const int64_t* __restrict__ jst, int nt, int64_t blocks, int64_t* __restrict__ kseg,
                            int* __restrict__ ja) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= blocks) return;
    const SegSplit S(jst, nt, blocks);
    const int64_t q0 = w * S.per, q1 = min(q0 + S.per, S.nch);
    if (q0 >= q1) {
        kseg[w] = 0;
        ja[w] = 0;
        return;
    }
    const int a = slice_of(jst, nt, q0), b = slice_of(jst, nt, q1 - 1);
    kseg[w] = b - a + 1;
    ja[w] = a;
}

// psum[g][i] = pairs of segment g in source slice i (sum of its chunks' histogram rows)
__global__ void __launch_bounds__(1024) k_seg_sum(const uint32_t* __restrict__ chist, const uint32_t* __restrict__ order,
                                                 const int64_t* __restrict__ jst, int nt, int64_t blocks,
                                                 const int64_t* __restrict__ segbase, const int* __restrict__ ja,
                                                 int ns, uint32_t* __restrict__ psum) {
    __shared__ uint32_t acc[1024];
    const int64_t g = blockIdx.x;
    if (g >= segbase[blocks]) return;  // grid sized by an upper bound
    const SegSplit S(jst, nt, blocks);
    const int64_t w = block_of_seg(segbase, blocks, g);
    const Seg sg = seg_of(jst, nt, S, ja, w, g - segbase[w]);
    const int hw = hist_words(ns), rows = 1024 / hw;  // hw <= 64
    const int r = threadIdx.x / hw, x = threadIdx.x % hw;
    uint32_t lo = 0, hi = 0;
    if (r < rows) {
        int64_t q = sg.q0 + r;
        for (; q + 3 * rows < sg.q1; q += 4 * rows) {  // four rows' loads in flight per lane
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = chist[(size_t)order[q + k * rows] * hw + x];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                lo += v[k] & 0xFFFFu;
                hi += v[k] >> 16;
            }
        }
        for (; q < sg.q1; q += rows) {
            const uint32_t v = chist[(size_t)order[q] * hw + x];
            lo += v & 0xFFFFu;
            hi += v >> 16;
        }
    }
    for (int half = 0; half < 2; ++half) {
        acc[threadIdx.x] = half ? hi : lo;
        __syncthreads();
        if (threadIdx.x < hw && 2 * (int)threadIdx.x + half < ns) {
            uint32_t s = 0;
            for (int k = 0; k < rows; ++k) s += acc[k * hw + threadIdx.x];
            psum[(size_t)g * ns + 2 * threadIdx.x + half] = s;
        }
        __syncthreads();
    }
}

// per cell (j, i): exclusive running sum over slice j's segments (in place) and the cell total
__global__ void k_seg_prefix(uint32_t* __restrict__ psum, const int64_t* __restrict__ jst, int64_t blocks,
                             const int64_t* __restrict__ segbase, const int* __restrict__ ja, Layout L,
                             int64_t* __restrict__ tot) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= L.ncells) return;
    const int j = c / L.ns, i = c % L.ns;
    const SegSplit S(jst, L.nt, blocks);
    int64_t run = 0;
    if (jst[j + 1] > jst[j])
        for (int64_t w = jst[j] / S.per; w <= (jst[j + 1] - 1) / S.per; ++w) {
            const size_t at = (size_t)(segbase[w] + (j - ja[w])) * L.ns + i;
            const uint32_t v = psum[at];
            psum[at] = (uint32_t)run;
            run += v;
        }
    tot[c] = run;
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

// hop-1 outputs when it runs inside pass 2 (a_ok covers the whole domain, so no source test)
struct Hop1Out {
    BitV tmask;  // b_ok
    uint32_t* M;
    uint32_t* S1;
    uint32_t* S2;
    int64_t gwords;
};

// The 2-hop layout's pair store.  Packed (L.packed): the cell-relative key
// k = (s mod 2^sbits) << tbits | (t mod 2^tbits), at most 40 bits, split into its low word w[pos]
// and high byte b[pos] -- 5 bytes per relationship instead of 8; the cell gives the slices back.
struct PairOut {
    uint2* p;     // unpacked
    uint32_t* w;  // packed: low words
    uint8_t* b;   // packed: high bytes
};

__device__ __forceinline__ uint64_t cell_key(const Layout& L, uint2 v) {
    return (uint64_t)(v.x & ((1u << L.sbits) - 1u)) << L.tbits | (v.y & ((1u << L.tbits) - 1u));
}

// pair of a cell-relative key in cell (j, i)
__device__ __forceinline__ uint2 key_pair(const Layout& L, uint32_t sbase, uint32_t tbase, uint32_t w, uint32_t b) {
    const uint64_t k = (uint64_t)b << 32 | w;
    return make_uint2(sbase + (uint32_t)(k >> L.tbits), tbase + (w & ((1u << L.tbits) - 1u)));
}

// ---- pass 2: block w's segments (chunks of one target slice each) -> the slices' source cells -----
// Output offsets are exact and precomputed, so the reservation per tile is an LDS cursor bump and the
// layout is deterministic.  The next chunk is loaded (buffer loads clipped at its fill) while this
// one is regrouped.  With HOP1 the block also runs hop 1 on the pairs it moves: M(t) for s != t
// marked in an LDS copy of the current slice (flushed through b_ok when it changes), self-loops
// -> S1 / S2.
// output line in items: 128 bytes of pairs, or of the packed low words
__host__ __device__ constexpr int s2_line(bool pk) { return pk ? 32 : kLine; }

// LDS bytes of the per-cell held items (packed: low word + high byte each)
__host__ __device__ constexpr size_t s2_hold_bytes(int nb, bool pk) {
    return pk ? (((size_t)nb * s2_line(true) * 5 + 15) & ~(size_t)15) : sizeof(uint2) * (size_t)nb * kLine;
}

template <bool HOP1, bool PK>  // PK: without HOP1 (LDS)
__global__ void __launch_bounds__(kSBlock) k_scatter_s2(const void* __restrict__ pool_,
                                                        const unsigned long long* __restrict__ cmeta,
                                                        const uint32_t* __restrict__ order,
                                                        const int64_t* __restrict__ jst,
                                                        const int64_t* __restrict__ segbase,
                                                        const int* __restrict__ ja, const uint32_t* __restrict__ prel,
                                                        const int64_t* __restrict__ coff, Layout L,
                                                        PairOut out, int64_t trash, Hop1Out h1) {
    constexpr int LN = s2_line(PK);
    extern __shared__ __attribute__((aligned(16))) unsigned long long smem[];
    const int nb = L.ns;
    const int64_t w = blockIdx.x, blocks = gridDim.x;
    uint2* stage = reinterpret_cast<uint2*>(smem);
    // per source cell: the items of its unfinished output line, slot = index mod LN
    unsigned char* hbase = reinterpret_cast<unsigned char*>(stage + kTile);
    uint2* hold = reinterpret_cast<uint2*>(hbase);
    uint32_t* holdw = reinterpret_cast<uint32_t*>(hbase);
    uint8_t* holdb = hbase + sizeof(uint32_t) * (size_t)nb * LN;
    uint32_t* cur = reinterpret_cast<uint32_t*>(hbase + s2_hold_bytes(nb, PK));  // next output index per cell (< 2^32)
    uint32_t* cnt = cur + nb;
    uint32_t* loc = cnt + nb;
    uint32_t* hc = loc + nb;  // items held per cell (all in the line of cur)
    uint32_t* wtot = hc + nb;
    uint32_t* tl = wtot + kSBlock / 64;  // HOP1: target slice marks
    const SegSplit S(jst, L.nt, blocks);
    for (int i = threadIdx.x; i < nb; i += kSBlock) hc[i] = 0;
    auto put = [&](uint32_t pos, uint2 v) {
        if (PK) {
            const uint64_t k = cell_key(L, v);
            out.w[pos] = (uint32_t)k;
            out.b[pos] = (uint8_t)(k >> 32);
        } else {
            out.p[pos] = v;
        }
    };
    auto hold_put = [&](int slot, uint2 v) {
        if (PK) {
            const uint64_t k = cell_key(L, v);
            holdw[slot] = (uint32_t)k;
            holdb[slot] = (uint8_t)(k >> 32);
        } else {
            hold[slot] = v;
        }
    };
    auto hold_out = [&](uint32_t pos, int slot) {
        if (PK) {
            out.w[pos] = holdw[slot];
            out.b[pos] = holdb[slot];
        } else {
            out.p[pos] = hold[slot];
        }
    };
    auto flush_held = [&]() {  // the segment's unfinished lines (shared with a neighbouring segment)
        for (int x = threadIdx.x; x < nb * LN; x += kSBlock) {
            const int b = x / LN, k = x % LN;
            if ((uint32_t)k < hc[b]) {
                const uint32_t pos = cur[b] - hc[b] + (uint32_t)k;
                hold_out(pos, b * LN + (int)(pos & (LN - 1)));
            }
        }
    };
    const uint2* pool = static_cast<const uint2*>(pool_);
    auto load_chunk = [&](int64_t q, uint2 (&pr)[kItems]) -> uint32_t {
        const uint32_t phys = order[q];
        const uint32_t fill = (uint32_t)(cmeta[phys] >> 32);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint2*>(pool + (size_t)phys * kCh), (short)0, (int)(fill * sizeof(uint2)), 0x00020000);
#pragma unroll
        for (int k = 0; k < kItems / 2; ++k) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(k * kSBlock + (int)threadIdx.x) * 16u, 0, 0);
            pr[2 * k] = make_uint2(v[0], v[1]);
            pr[2 * k + 1] = make_uint2(v[2], v[3]);
        }
        return fill;
    };
    const int64_t qb = w * S.per, qe = min(qb + S.per, S.nch);
    uint2 nx[kItems];
    uint32_t nfill = qb < qe ? load_chunk(qb, nx) : 0u;
    int64_t g = segbase[w] - 1, seg_end = qb;  // current segment and the end of its chunk range
    int cur_j = -1;
    uint32_t tbase = 0;
    // One flat loop over the block's chunks, so the only vector-memory operations between a
    // chunk's prefetch and its use are the kItems stores of the tile before (unconditional, so the
    // compiler can wait for the loads alone); segment changes are the rare branch.
    for (int64_t q = qb; q < qe; ++q) {  // block-uniform
        if (q == seg_end) {
            __syncthreads();
            flush_held();
            __syncthreads();
            for (int i = threadIdx.x; i < nb; i += kSBlock) hc[i] = 0;
            Seg sg;
            do {
                ++g;
                sg = seg_of(jst, L.nt, S, ja, w, g - segbase[w]);
            } while (sg.q0 >= sg.q1);  // skip empty slices
            seg_end = sg.q1;
            if (HOP1 && sg.j != cur_j) {
                if (cur_j >= 0) {
                    __syncthreads();
                    flush_slice(tl, h1.M, cur_j, h1.gwords, h1.tmask);
                }
                __syncthreads();
                for (int k = threadIdx.x; k < kSliceWords; k += kSBlock) tl[k] = 0;
            }
            cur_j = sg.j;
            tbase = (uint32_t)sg.j << kSliceBits;
            __syncthreads();
            for (int i = threadIdx.x; i < nb; i += kSBlock)
                cur[i] = (uint32_t)(coff[(size_t)sg.j * nb + i] + prel[(size_t)g * nb + i]);
        }
        uint2 pr[kItems];
#pragma unroll
        for (int k = 0; k < kItems; ++k) pr[k] = nx[k];
        const uint32_t fill = nfill;
        if (q + 1 < qe) nfill = load_chunk(q + 1, nx);  // prefetch (may be the next segment's)
        for (int i = threadIdx.x; i < nb; i += kSBlock) cnt[i] = 0;
        __syncthreads();
        uint32_t rk[kItems];
        uint32_t valid = 0;
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            valid |= ((uint32_t)item_off<kSBlock>(k) < fill ? 1u : 0u) << k;
            rk[k] = 0;
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k)
            if ((valid >> k) & 1u) {
                rk[k] = atomicAdd(&cnt[pr[k].x >> L.sbits], 1u);
                if (HOP1) {
                    const uint32_t s = pr[k].x, t = pr[k].y;
                    if (s != t) {
                        lds_set(tl, t - tbase);
                    } else if (h1.tmask.full || gbit(h1.tmask.w, t)) {  // rare: self-loops
                        const uint32_t bit = 1u << (t & 31);
                        const uint32_t old = atomicOr(&h1.S1[t >> 5], bit);
                        if (old & bit) atomicOr(&h1.S2[t >> 5], bit);
                    }
                }
            }
        __syncthreads();
        const uint32_t total = small_exclusive_scan<kSBlock>(cnt, loc, nb, wtot);
        // Whole output lines: a cell's run is stored up to the last line boundary it reaches, the
        // rest held in LDS; held items go out when their line completes, together with the run
        // items that complete it (so a line is written within one tile, not in pieces by two).
        for (int x = threadIdx.x; x < nb * LN; x += kSBlock) {
            const int b = x / LN, k = x % LN;
            if ((uint32_t)k < hc[b]) {
                const uint32_t c = cur[b], pos = c - hc[b] + (uint32_t)k;
                if (((c + cnt[b]) & ~(uint32_t)(LN - 1)) > (c & ~(uint32_t)(LN - 1)))
                    hold_out(pos, b * LN + (int)(pos & (LN - 1)));
            }
        }
#pragma unroll
        for (int k = 0; k < kItems; ++k)
            if ((valid >> k) & 1u) stage[loc[pr[k].x >> L.sbits] + rk[k]] = pr[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kItems; ++k) {
            const uint32_t idx = (uint32_t)(k * kSBlock + (int)threadIdx.x);
            const uint2 v = stage[idx];
            const int b = min((int)(v.x >> L.sbits), nb - 1);  // stale stage entries past `total`
            const uint32_t pos = cur[b] + idx - loc[b];
            const uint32_t cut = (cur[b] + cnt[b]) & ~(uint32_t)(LN - 1);
            if (idx >= total)
                put((uint32_t)trash + threadIdx.x, v);
            else if (pos < cut)
                put(pos, v);
            else
                hold_put(b * LN + (int)(pos & (LN - 1)), v);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nb; i += kSBlock) {
            const uint32_t c = cur[i], n = cnt[i];
            const uint32_t cut = (c + n) & ~(uint32_t)(LN - 1);
            hc[i] = cut > (c & ~(uint32_t)(LN - 1)) ? c + n - cut : hc[i] + n;
            cur[i] = c + n;
        }
    }
    __syncthreads();
    flush_held();
    if (HOP1 && cur_j >= 0) flush_slice(tl, h1.M, cur_j, h1.gwords, h1.tmask);
}

// One hop over the 2-D layout.  Block b streams relationships [b*per, (b+1)*per) of the
// j-major cell order, per = max(ceil(kept / blocks), min_per); kept = coff[ncells] is read on the
// device, so building the layout needs no host round trip.
//   HOP1: M(t) |= a_ok(s) for s != t; self-loops (a_ok(s) and b_ok(t)) -> S1, second one -> S2.
//         Target filter b_ok at flush.
//   HOP2: C(t) |= X1(s) for s != t, X2(s) for s == t.  Target filter c_ok at flush.
// `sb` is the per-relationship source bitmap (a_ok or X1); `tmask` the target filter.
// this lane's kN packed items of the cell walk starting at the 4-aligned index b: item u is
// b + 4 * ((u >> 2) * B + lane) + (u & 3), one 16-byte low-word load and one 4-byte high-byte load
// per four items (streamed once: non-temporal)

template <int B, int N>
__device__ __forceinline__ void load_packed(const uint32_t* __restrict__ w, const uint8_t* __restrict__ hb, int64_t b,
                                            uint32_t (&lw)[N], uint32_t (&hw)[N / 4]) {
    typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
    const v4u32* __restrict__ v = reinterpret_cast<const v4u32*>(w + b);
    const uint32_t* __restrict__ h = reinterpret_cast<const uint32_t*>(hb + b);
#pragma unroll
    for (int k = 0; k < N / 4; ++k) {
        const v4u32 x = __builtin_nontemporal_load(v + k * B + (int)threadIdx.x);
        lw[4 * k] = x.x;
        lw[4 * k + 1] = x.y;
        lw[4 * k + 2] = x.z;
        lw[4 * k + 3] = x.w;
        hw[k] = __builtin_nontemporal_load(h + k * B + (int)threadIdx.x);
    }
}

template <bool HOP1, bool SRC_FULL, bool PK>
__global__ void __launch_bounds__(kBlock) k_hop_2d(PairOut pairs, const int64_t* __restrict__ coff,
                                                   int64_t min_per, Layout L, BitV sb,
                                                   const uint32_t* __restrict__ X2, BitV tmask,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ S1,
                                                   uint32_t* __restrict__ S2, int64_t gwords) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* tl = lds;                // target slice marks
    uint32_t* sl = lds + kSliceWords;  // source slice frontier (when pulled)
    const int64_t kept = coff[L.ncells];
    int64_t per = (kept + gridDim.x - 1) / gridDim.x;
    if (per < min_per) per = min_per;
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
    // The source slice a cell pulls is loaded into registers while the cell before it streams (this lane's
    // kSliceWords / kBlock words, 16-byte loads issued ahead of the cell's pair loads), so the pull no longer
    // waits for its own load latency behind a barrier; `nxt_i` = the slice held (-1: none).
    static_assert(kSliceWords % (4 * kBlock) == 0, "pull prefetch: whole 16-byte words per lane");
    constexpr int kPw = kSliceWords / (4 * kBlock);
    uint4 nsl[kPw];
    int nxt_i = -1;
    auto prefetch_slice = [&](int i2) {
        const uint4* src4 = reinterpret_cast<const uint4*>(sb.w + (int64_t)i2 * kSliceWords);
        const int64_t lim4 = (gwords - (int64_t)i2 * kSliceWords) / 4;  // whole uint4 words inside the bitmap
#pragma unroll
        for (int k = 0; k < kPw; ++k) {
            const int64_t x = (int64_t)k * kBlock + threadIdx.x;
            nsl[k] = x < lim4 ? src4[x] : make_uint4(0u, 0u, 0u, 0u);
        }
        nxt_i = i2;
    };
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
            if (nxt_i == i && (gwords - w0) % 4 == 0) {
                uint4* sl4 = reinterpret_cast<uint4*>(sl);
#pragma unroll
                for (int k = 0; k < kPw; ++k) sl4[k * kBlock + threadIdx.x] = nsl[k];
            } else {
                for (int k = threadIdx.x; k < kSliceWords; k += kBlock) sl[k] = w0 + k < gwords ? sb.w[w0 + k] : 0u;
            }
            nxt_i = -1;
        }
        if (can_pull && ce == coff[c + 1] && ce < e1 && ((uintptr_t)sb.w & 15) == 0) {  // the next cell, if it pulls
            const int c2 = c + 1;
            if (min(e1, coff[c2 + 1]) - ce >= kLoadMin) prefetch_slice(c2 % L.ns);
        }
        __syncthreads();
        const uint32_t tbase = (uint32_t)j << L.tbits, sbase = (uint32_t)i << L.sbits;  // pull: sbits = kSliceBits
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
        if (PK) {  // 5 bytes per item: twice the items per step for the same loads in flight
            constexpr int U = 2 * kUnroll;
            for (int64_t cb = e0 & ~int64_t(3); cb < ce; cb += (int64_t)kBlock * U) {  // block-uniform
                uint32_t lw[U], hw[U / 4];
                load_packed<kBlock, U>(pairs.w, pairs.b, cb, lw, hw);
                const int lo = (int)max(e0 - cb, (int64_t)0), hi = (int)min(ce - cb, (int64_t)kBlock * U);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = item_off4<kBlock>(u);
                    if (e >= lo && e < hi) visit(key_pair(L, sbase, tbase, lw[u], (hw[u >> 2] >> (8 * (u & 3))) & 0xFFu));
                }
            }
        } else {
            for (int64_t cb = e0 & ~int64_t(1); cb < ce; cb += (int64_t)kBlock * kUnroll) {  // block-uniform, even
                uint2 p[kUnroll];
                load_pairs<kBlock, kUnroll>(pairs.p, cb, p);
                const int lo = (int)max(e0 - cb, (int64_t)0), hi = (int)min(ce - cb, (int64_t)kBlock * kUnroll);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const int e = item_off<kBlock>(u);
                    if (e >= lo && e < hi) visit(p[u]);
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


}  // namespace part

// ================================ host side =====================================================
static part::Layout make_layout(int64_t lo, int64_t hi, bool allow_packed) {
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
    L.tbits = part::kSliceBits;
    L.packed = allow_packed && L.sbits + L.tbits <= 40;  // 5-byte cell keys
    return L;
}

static part::PairOut pair_out(const RelPart& rp) {
    part::PairOut o{};
    if (rp.L.packed) {
        o.w = P<uint32_t>(rp.pairs);
        o.b = reinterpret_cast<uint8_t*>(o.w + rp.cap);
    } else {
        o.p = P<uint2>(rp.pairs);
    }
    return o;
}

void lds_attr(const void* kernel, size_t bytes) {
    // set once per (device, kernel) and raised only when a launch needs more: the attribute call
    // costs host time on every query otherwise
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, size_t> done;
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    const auto key = std::make_pair(dev, kernel);
    std::lock_guard<std::mutex> g(mu);
    auto it = done.find(key);
    if (it != done.end() && it->second >= bytes) return;
    HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    done[key] = bytes;
}

template <typename K>
static void allow_lds(K kernel, size_t bytes) {
    lds_attr(reinterpret_cast<const void*>(kernel), bytes);
}

void chunk_partition(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                     int nt, bool swap, const part::Layout& L, int64_t g2_want, ChunkPart& cp) {
    using namespace part;
    hipStream_t st = s->stream;
    cp.L = L;
    // pass 1 grid: one 1024-lane block per CU, fewer for small inputs so the open chunks
    // (blocks x slices) stay within a few times the filled ones
    std::vector<int> g1(nt, 0);
    std::vector<int64_t> c0(nt, 0);
    int64_t pool_chunks = 0, mtot = 0;
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        const int64_t full = (ms[i] + kCh - 1) / kCh;
        // tiles per block: 8 for large inputs; small ones (a rank's 1/8 shard of C5: 2^22 relationships) take
        // 2, so the pass spreads over the CUs instead of 64 blocks walking 8 tiles each (124 us for 2^22
        // relationships at 64 blocks, round-5 kernel trace, profiles/r05_c5_small_trace_stats.csv)
        const int64_t tmin = ms[i] <= (int64_t(1) << 24) ? 2 : 8;
        int64_t g = std::min<int64_t>((int64_t)s->num_cus * (kSBlock / kP1Block),
                                      (ms[i] + tmin * (int64_t)kP1Tile - 1) / (tmin * (int64_t)kP1Tile));
        // (at most ~32 open chunks per filled one -- 64 for small inputs, whose pools are small anyway: a 1/8
        // shard of C5's 2^25 relationships got 32 blocks at the earlier bound of 8, and its three
        // partitions took 1.33 ms against 0.29 ms for the whole table's two)
        g = std::min<int64_t>(g, std::max<int64_t>(1, (tmin == 2 ? 64 : 32) * full / L.nt));
        g1[i] = (int)std::max<int64_t>(1, g);
        c0[i] = pool_chunks;
        pool_chunks += (int64_t)g1[i] * chunks_per_block(ms[i], g1[i], L.nt);
        mtot += ms[i];
    }
    REQUIRE(pool_chunks < (int64_t)INT32_MAX && mtot + 2 * kPad < (int64_t)UINT32_MAX, CAPSMI_ERR_UNSUPPORTED,
            "relationship table too large for the layout");
    const int64_t npool = pool_chunks > 0 ? pool_chunks : 1;
    const int hw = hist_words(L.ns);
    cp.pool = dev_alloc(sizeof(uint2) * kCh * (size_t)(npool + 1), s);  // + a trash chunk
    cp.meta = dev_alloc(sizeof(unsigned long long) * npool, s);
    cp.chist = dev_alloc(sizeof(uint32_t) * hw * (size_t)npool, s);
    // (clearing each block's metadata range inside pass 1 instead measured 5.25 -> 5.39 ms at C3: the fill stays)
    HIP_CHECK(hipMemsetAsync(P<void>(cp.meta), 0, sizeof(unsigned long long) * npool, st));
    const size_t lds1l = scatter1l_lds(L.nt, L.ns, kP1Block, kP1Tile);
    const bool lines = lds1l <= (size_t)160 * 1024;
    const size_t lds1 = lines ? lds1l : scatter1_lds(L.nt, L.ns);
    if (lines)
        allow_lds(k_scatter_l<kP1Block, kItems, 4>, lds1);
    else
        allow_lds(k_scatter_c<kP1Block, kItems, 4, kP1NT>, lds1);
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        KernelTimer kt(s, "part_scatter1");
        if (lines)
            hipLaunchKernelGGL((k_scatter_l<kP1Block, kItems, 4>), dim3(g1[i]), dim3(kP1Block), lds1, st, srcs[i], dsts[i],
                               ms[i], L, swap ? 1 : 0, c0[i], (size_t)npool * kCh, P<uint2>(cp.pool),
                               P<unsigned long long>(cp.meta), P<uint32_t>(cp.chist));
        else
            hipLaunchKernelGGL((k_scatter_c<kP1Block, kItems, 4, kP1NT>), dim3(g1[i]), dim3(kP1Block), lds1, st, srcs[i],
                               dsts[i], ms[i], L, swap ? 1 : 0, c0[i], (size_t)npool * kCh, P<uint2>(cp.pool),
                               P<unsigned long long>(cp.meta), P<uint32_t>(cp.chist));
    }
    HIP_CHECK(hipGetLastError());
    cp.mtot = mtot;
    chunk_order(s, L.nt, pool_chunks, g2_want, cp);
}

// used chunks (cp.meta: slice, fill) ordered by target slice and the block-balanced segment split
// of a consumer grid of g2 blocks; no host round trip
void chunk_order(capsmi_session* s, int nt, int64_t pool_chunks, int64_t g2_want, ChunkPart& cp) {
    using namespace part;
    hipStream_t st = s->stream;
    Layout L = cp.L;
    L.nt = nt;
    const int64_t npool = pool_chunks > 0 ? pool_chunks : 1;
    const int64_t g2 = std::max<int64_t>(1, std::min<int64_t>(g2_want, npool));
    cp.jbuf = dev_alloc(sizeof(int64_t) * (3 * (size_t)L.nt + 2 * (size_t)g2 + 3) + sizeof(uint32_t) * npool +
                             sizeof(int) * g2, s);
    int64_t* jcnt = P<int64_t>(cp.jbuf);
    int64_t* jst = jcnt + L.nt;        // nt + 1
    int64_t* jcur = jst + L.nt + 1;    // nt
    int64_t* kseg = jcur + L.nt;       // g2
    int64_t* segbase = kseg + g2;      // g2 + 1
    uint32_t* order = reinterpret_cast<uint32_t*>(segbase + g2 + 2);
    int* ja = reinterpret_cast<int*>(order + npool);
    if (npool <= kOrder1Max && L.nt <= kMaxTSlices && g2 <= 4096) {  // small pools: one launch
        hipLaunchKernelGGL(k_chunk_order1, dim3(1), dim3(kChunkBlock), 0, st, P<unsigned long long>(cp.meta),
                           pool_chunks, L.nt, g2, jst, order, segbase, ja);
        HIP_CHECK(hipGetLastError());
        cp.pool_chunks = pool_chunks;
        cp.npool = npool;
        cp.g2 = g2;
        cp.jst = jst;
        cp.segbase = segbase;
        cp.ja = ja;
        cp.order = order;
        return;
    }
    HIP_CHECK(hipMemsetAsync(jcnt, 0, sizeof(int64_t) * L.nt, st));
    const unsigned cg = (unsigned)((npool + kChunkPer - 1) / kChunkPer);
    hipLaunchKernelGGL(k_chunk_count, dim3(cg), dim3(kChunkBlock), sizeof(uint32_t) * L.nt, st,
                       P<unsigned long long>(cp.meta), pool_chunks, L.nt, jcnt);
    exclusive_scan_i64(jcnt, jst, L.nt, s);
    HIP_CHECK(hipMemcpyAsync(jcur, jst, sizeof(int64_t) * L.nt, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(k_chunk_place, dim3(cg), dim3(kChunkBlock), sizeof(uint32_t) * 2 * L.nt, st,
                       P<unsigned long long>(cp.meta), pool_chunks, L.nt,
                       reinterpret_cast<unsigned long long*>(jcur), order);
    hipLaunchKernelGGL(k_seg_count, dim3((unsigned)((g2 + 255) / 256)), dim3(256), 0, st, jst, L.nt, g2, kseg, ja);
    exclusive_scan_i64(kseg, segbase, g2, s);
    HIP_CHECK(hipGetLastError());
    cp.pool_chunks = pool_chunks;
    cp.npool = npool;
    cp.g2 = g2;
    cp.jst = jst;
    cp.segbase = segbase;
    cp.ja = ja;
    cp.order = order;
}

void relpart_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                   int64_t lo, int64_t hi, RelPart& rp, const RelPartHop1* h1, bool unpacked) {
    REQUIRE(hi > lo && (uint64_t)(hi - lo) <= (uint64_t(1) << 30), CAPSMI_ERR_UNSUPPORTED,
            "partitioned layout needs an id domain of at most 2^30 ids");
    using namespace part;
    hipStream_t st = s->stream;
    rp.L = make_layout(lo, hi, s->cfg.pairs != 2);  // config CAPSMI_PAIRS=uint2: 8-byte pairs
    // Only a layout kept for later queries (capsmi_relpart_build, the cache() route) is packed: pass 2
    // writing the packed form is slower (C3: 3.45 -> 3.9-4.45 ms unfused, 3.73 -> 4.14 ms with hop 1
    // fused) while each hop over it gains 0.2-0.4 ms (hop 1 1.30 -> 0.90, hop 2 1.57 -> 1.35 ms), so a
    // layout read by one query's two hops is left in 8-byte pairs
    if (h1 || unpacked) rp.L.packed = 0;
    const Layout& L = rp.L;
    REQUIRE(L.nt <= kMaxTSlices && L.ncells <= kMaxCells, CAPSMI_ERR_INTERNAL, "layout too large");
    if (h1)
        REQUIRE(h1->a->lo == lo && h1->a->hi == hi && h1->b->lo == lo && h1->b->hi == hi, CAPSMI_ERR_UNSUPPORTED,
                "partitioned 2-hop needs node scans over the layout's id domain");

    const bool fuse = h1 && h1->a->full;
    ChunkPart cp;
    // (measured and removed in round 6: a 6-byte pass-1 pool, u32 + u16 arrays per chunk -- pass 1 5.26 ->
    // 5.58 ms, pass 2 + hop 1 3.76 -> 4.45 ms at C3; both passes are bound by their LDS / VALU phases)
    chunk_partition(s, srcs, dsts, ms, nt, false, L, (int64_t)s->num_cus * (fuse ? 1 : 2), cp);
    const int64_t g2 = cp.g2, mtot = cp.mtot;
    const int64_t maxg = g2 + L.nt;  // segments <= blocks + slices
    int64_t* jst = cp.jst;
    int64_t* segbase = cp.segbase;
    int* ja = cp.ja;
    uint32_t* order = cp.order;
    Buf& pool = cp.pool;
    Buf& meta = cp.meta;
    Buf& chist = cp.chist;
    Buf pbuf = dev_alloc(sizeof(uint32_t) * (size_t)maxg * L.ns, s);
    uint32_t* psum = P<uint32_t>(pbuf);
    Buf tot = dev_alloc(sizeof(int64_t) * L.ncells, s);
    hipLaunchKernelGGL(k_seg_sum, dim3((unsigned)maxg), dim3(1024), 0, st, P<uint32_t>(chist), order, jst, L.nt, g2,
                       segbase, ja, L.ns, psum);
    hipLaunchKernelGGL(k_seg_prefix, dim3((L.ncells + 255) / 256), dim3(256), 0, st, psum, jst, g2, segbase, ja, L,
                       P<int64_t>(tot));
    rp.boff = dev_alloc(sizeof(int64_t) * (L.ncells + 1), s);  // cell offsets
    exclusive_scan_i64(P<int64_t>(tot), P<int64_t>(rp.boff), L.ncells, s);
    HIP_CHECK(hipGetLastError());
    rp.cap = mtot + kPad;  // kept <= mtot; slack for the hops' whole-step loads and pass 2's trash stores
    rp.pairs = dev_alloc(L.packed ? 5 * (size_t)rp.cap : sizeof(uint2) * (size_t)rp.cap, s);

    Hop1Out ho{};
    if (fuse) ho = Hop1Out{BitV{P<uint32_t>(h1->b->words), h1->b->full ? 1 : 0}, h1->M, h1->S1, h1->S2, h1->b->nwords};
    const size_t lds2 = sizeof(uint2) * (size_t)kTile + s2_hold_bytes(L.ns, L.packed) +
                        sizeof(uint32_t) * (4 * L.ns + kSBlock / 64) + (fuse ? sizeof(uint32_t) * kSliceWords : 0);
    REQUIRE(lds2 <= (size_t)160 * 1024, CAPSMI_ERR_INTERNAL, "pass-2 LDS");
    auto k2 = L.packed ? k_scatter_s2<false, true> : fuse ? k_scatter_s2<true, false> : k_scatter_s2<false, false>;
    allow_lds(k2, lds2);
    {
        KernelTimer kt(s, fuse ? "part_scatter2_hop1" : "part_scatter2");
        hipLaunchKernelGGL(k2, dim3((unsigned)g2), dim3(kSBlock), lds2, st, P<void>(pool), P<unsigned long long>(meta),
                           order, jst, segbase, ja, psum, P<int64_t>(rp.boff), L, pair_out(rp), mtot, ho);
    }
    HIP_CHECK(hipGetLastError());
    rp.kept = -1;  // known on the device (boff[ncells]); read only when asked (relpart_kept)
    rp.rows = mtot;
    if (h1 && !fuse) relpart_hop1(s, rp, h1->a, h1->b, h1->M, h1->S1, h1->S2);
}

template <bool HOP1, bool SRC_FULL>
static void launch_hop(capsmi_session* s, const RelPart& rp, part::BitV sb, const uint32_t* X2, part::BitV tmask,
                       uint32_t* out, uint32_t* S1, uint32_t* S2, int64_t gwords) {
    const size_t lds = sizeof(uint32_t) * 2 * part::kSliceWords;
    auto k = rp.L.packed ? part::k_hop_2d<HOP1, SRC_FULL, true> : part::k_hop_2d<HOP1, SRC_FULL, false>;
    allow_lds(k, lds);
    // one 128 KiB-LDS block per CU at a time; a few rounds of blocks, equal relationship shares
    // (at least kBlock * kUnroll each; blocks past the end exit at once).  Grid sized from the upper
    // bound of the kept count (the table rows), the exact count is read by the kernel.
    const int64_t min_per = (int64_t)part::kBlock * part::kUnroll;
    int64_t blocks = (int64_t)s->num_cus * 4;
    const int64_t bound = rp.kept >= 0 ? rp.kept : rp.rows;
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, (bound + min_per - 1) / min_per));
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(part::kBlock), lds, s->stream, pair_out(rp),
                       P<int64_t>(rp.boff), min_per, rp.L, sb, X2, tmask, out, S1, S2, gwords);
    HIP_CHECK(hipGetLastError());
}

void relpart_hop1(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* M,
                  uint32_t* S1, uint32_t* S2) {
    REQUIRE(a->lo == rp.L.lo && a->hi == rp.L.hi && b->lo == rp.L.lo && b->hi == rp.L.hi, CAPSMI_ERR_UNSUPPORTED,
            "partitioned 2-hop needs node scans over the layout's id domain");
    if (rp.rows == 0) return;
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
    if (rp.rows == 0) return;
    const part::BitV xv{X1, 0}, cv{P<uint32_t>(c->words), c->full ? 1 : 0};
    KernelTimer kt(s, "hop2");
    launch_hop<false, false>(s, rp, xv, X2, cv, C, nullptr, nullptr, c->nwords);
}

// ---- layout digest (test support): per cell, pair count and wrapping sum of a 64-bit mix ----------------
__device__ __forceinline__ uint64_t pair_mix(uint2 p) {
    uint64_t z = ((uint64_t)p.x << 32 | p.y) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_cell_digest(part::PairOut pairs, const int64_t* __restrict__ boff,
                                                    part::Layout L, unsigned long long* __restrict__ sums,
                                                    unsigned long long* __restrict__ bad) {
    const int c = blockIdx.x;
    const uint32_t sbase = (uint32_t)(c % L.ns) << L.sbits, tbase = (uint32_t)(c / L.ns) << L.tbits;
    unsigned long long acc = 0, nb = 0;
    for (int64_t i = boff[c] + threadIdx.x; i < boff[c + 1]; i += 256) {
        // packed: the pair comes back through its cell, so a misplaced one shows as a wrong sum
        const uint2 p = L.packed ? part::key_pair(L, sbase, tbase, pairs.w[i], pairs.b[i]) : pairs.p[i];
        acc += pair_mix(p);
        if (part::cell_of(L, p.x, p.y) != c) ++nb;
    }
    atomicAdd(&sums[c], acc);
    if (nb) atomicAdd(bad, nb);
}

void relpart_digest(capsmi_session* s, const RelPart& rp, int64_t* counts, uint64_t* sums, int64_t* misplaced) {
    hipStream_t st = s->stream;
    const int nc = rp.L.ncells;
    std::vector<int64_t> off(nc + 1, 0);
    Buf d = dev_alloc(sizeof(unsigned long long) * (nc + 1), s);
    HIP_CHECK(hipMemsetAsync(P<void>(d), 0, sizeof(unsigned long long) * (nc + 1), st));
    if (rp.rows > 0) {
        hipLaunchKernelGGL(k_cell_digest, dim3(nc), dim3(256), 0, st, pair_out(rp), P<int64_t>(rp.boff), rp.L,
                           P<unsigned long long>(d), P<unsigned long long>(d) + nc);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(off.data(), P<void>(rp.boff), sizeof(int64_t) * (nc + 1), hipMemcpyDeviceToHost, st));
    }
    std::vector<unsigned long long> h(nc + 1);
    HIP_CHECK(hipMemcpyAsync(h.data(), P<void>(d), sizeof(unsigned long long) * (nc + 1), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    for (int c = 0; c < nc; ++c) {
        counts[c] = off[c + 1] - off[c];
        sums[c] = h[c];
    }
    *misplaced = (int64_t)h[nc];
}

int64_t relpart_kept(capsmi_session* s, RelPart& rp) {
    if (rp.kept < 0) rp.kept = rp.rows > 0 ? read_scalar(s, P<int64_t>(rp.boff) + rp.L.ncells) : 0;
    return rp.kept;
}

}  // namespace capsmi
