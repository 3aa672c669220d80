// part_common.h -- shared pieces of the chunked relationship partition (k_part.hip) and its users
// (C3 2-D layout build, C5 source-sliced var-length passes in k_varlen.hip).  Not part of the ABI.
#pragma once
#include "capsmi_impl.h"

namespace capsmi {
namespace part {

constexpr int kSliceBits = 19;                   // 2^19 ids per slice = 64 KiB of LDS bitmap
constexpr int kSliceWords = 1 << (kSliceBits - 5);
constexpr int kMaxCells = 16384;                 // cell histogram = 32 KiB of 16-bit LDS counters
constexpr int kMaxTSlices = 2048;                // domain <= 2^30 ids (pass-1 LDS: 7 words per slice)
constexpr int kBlock = 1024;                     // hop workgroups
constexpr int kItems = 8;                        // relationships per lane per tile
constexpr int kSBlock = 1024;                    // scatter workgroups
constexpr int kTile = kSBlock * kItems;          // relationships per scatter tile (8192)
constexpr int kCh = kTile;                       // pairs per pass-1 chunk: a tile's run spans <= 2 chunks
constexpr int kP1Block = 1024;                   // pass-1 workgroup (512 x 2 per CU measured slower; 768 lanes
                                                 // with 134 VGPRs, round 6: pass 1 5.25 -> 5.97 ms at C3)
constexpr int kP1Tile = kP1Block * kItems;       // pass-1 tile (<= kCh)
static_assert(kP1Tile <= kCh, "a pass-1 run must span at most two chunks");
constexpr bool kP1NT = false;                    // pass-1 pool stores non-temporal
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kUnroll = 8;                       // loads in flight per lane in the hops
constexpr int64_t kLoadMin = 8192;               // pull a source slice into LDS for >= this many rels
constexpr int kPad = 2 * 8192;                   // slack pairs after every pair array (load_pairs)

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

// The same scan for n <= 128 (the partition passes' per-tile histograms at C3: 128 source slices): wave 0
// alone, two counters per lane, then one barrier -- instead of three; larger n take block_exclusive_scan.
// `wtot` word 0 carries the total to the block.
template <int B>
__device__ uint32_t small_exclusive_scan(const uint32_t* in, uint32_t* out, int n, uint32_t* wtot) {
    if (n > 128) return block_exclusive_scan<B>(in, out, n, wtot);  // block-uniform
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x, i0 = 2 * lane;
        const uint32_t a = i0 < n ? in[i0] : 0u, b = i0 + 1 < n ? in[i0 + 1] : 0u;
        uint32_t x = a + b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        const uint32_t ex = x - a - b;
        if (i0 < n) out[i0] = ex;
        if (i0 + 1 < n) out[i0 + 1] = ex + a;
        if (lane == 63) wtot[0] = x;
    }
    __syncthreads();
    return wtot[0];
}

__device__ __forceinline__ int cell_of(const Layout& L, uint32_t s, uint32_t t) {
    return (int)(t >> L.tbits) * L.ns + (int)(s >> L.sbits);
}

// Tile item u of this lane is relationship t0 + item_off<B>(u): lanes read 16-byte pairs of
// consecutive relationships (2 int64 per load, the calibrated streaming width), pair k of the
// tile at offset 2 * (k * B + lane).
template <int B>
__device__ __forceinline__ int item_off(int u) {
    return 2 * ((u >> 1) * B + (int)threadIdx.x) + (u & 1);
}

// Issue all of a tile's loads before any test: with a branch around each load the compiler
// waits for every load before issuing the next.  `vec` = both columns 16-byte aligned.
template <int B, bool NTL = false, int N>
__device__ __forceinline__ void load_tile(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t t0,
                                          int64_t m, bool vec, int64_t (&sr)[N], int64_t (&tr)[N]) {
    const int64_t* __restrict__ sp = src + t0;  // wave-uniform bases, 32-bit lane offsets
    const int64_t* __restrict__ dp = dst + t0;
    if (vec && t0 + B * N <= m) {
        const longlong2* __restrict__ sv = reinterpret_cast<const longlong2*>(sp);
        const longlong2* __restrict__ dv = reinterpret_cast<const longlong2*>(dp);
#pragma unroll
        for (int k = 0; k < N / 2; ++k) {
            typedef long long v2i64 __attribute__((ext_vector_type(2)));
            longlong2 a, b;
            if (NTL) {  // streamed once: keep the L2 for lines still being written
                const v2i64 x = __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(sv) + k * B + (int)threadIdx.x);
                const v2i64 y = __builtin_nontemporal_load(reinterpret_cast<const v2i64*>(dv) + k * B + (int)threadIdx.x);
                a.x = x.x;
                a.y = x.y;
                b.x = y.x;
                b.y = y.y;
            } else {
                a = sv[k * B + (int)threadIdx.x];
                b = dv[k * B + (int)threadIdx.x];
            }
            sr[2 * k] = a.x;
            sr[2 * k + 1] = a.y;
            tr[2 * k] = b.x;
            tr[2 * k + 1] = b.y;
        }
    } else {
        const int last = (int)(min(m - t0, (int64_t)B * N) - 1);
#pragma unroll
        for (int u = 0; u < N; ++u) {
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
    typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
    const v4u32* __restrict__ v = reinterpret_cast<const v4u32*>(in + b);
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {  // streamed once: non-temporal, keeps the L2 for the bitmaps
        const v4u32 x = __builtin_nontemporal_load(v + k * B + (int)threadIdx.x);
        p[2 * k] = make_uint2(x.x, x.y);
        p[2 * k + 1] = make_uint2(x.z, x.w);
    }
}

__device__ __forceinline__ unsigned long long chunk_meta(int j, uint32_t fill) {
    return (unsigned long long)(uint32_t)j | ((unsigned long long)fill << 32);
}

// per-chunk histogram row: ns 16-bit counters padded to an even count (whole 32-bit words)
__host__ __device__ constexpr int hist_words(int ns) { return (ns + 1) >> 1; }

// ---- pass-2 work split ------------------------------------------------------------------------------
// Block w of pass 2 takes the used chunks [w * per, (w + 1) * per) of the slice-ordered list
// (per = ceil(chunks / blocks), read on the device).  Its range meets slices ja(w) .. jb(w); each
// (block, slice) intersection is a segment, numbered block-major, so the segments of one slice are
// consecutive.  The exact output start of segment g in cell (j, i) is coff[(j, i)] + the pairs the
// slice's earlier segments put there (prefix over the per-chunk histograms).

__device__ __forceinline__ int slice_of(const int64_t* jst, int nt, int64_t q) {  // last j with jst[j] <= q
    int lo = 0, hi = nt;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (jst[mid] <= q) lo = mid; else hi = mid;
    }
    return lo;
}

struct SegSplit {
    int64_t nch, per;
    __device__ SegSplit(const int64_t* jst, int nt, int64_t blocks) : nch(jst[nt]), per((jst[nt] + blocks - 1) / blocks) {
        if (per < 1) per = 1;
    }
};

struct Seg {
    int j;
    int64_t q0, q1;  // chunk range in `order`
};

__device__ __forceinline__ Seg seg_of(const int64_t* jst, int nt, const SegSplit& S, const int* ja, int64_t w,
                                      int64_t k) {
    Seg g;
    g.j = ja[w] + (int)k;
    g.q0 = max(w * S.per, jst[g.j]);
    g.q1 = min(min(w * S.per + S.per, S.nch), jst[g.j + 1]);
    return g;
}

__device__ __forceinline__ int64_t block_of_seg(const int64_t* segbase, int64_t blocks, int64_t g) {
    int64_t lo = 0, hi = blocks;  // last w with segbase[w] <= g
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (segbase[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

struct BitV {
    const uint32_t* w;  // words over [lo, hi) -- same domain as the layout
    int full;
};

__device__ __forceinline__ bool gbit(const uint32_t* w, uint32_t x) { return (w[x >> 5] >> (x & 31)) & 1u; }

// set bit x of an LDS bitmap: a no-return ds_or (a read-then-or measured 0.1 ms slower at C3)
__device__ __forceinline__ void lds_set(uint32_t* lds, uint32_t x) { atomicOr(&lds[x >> 5], 1u << (x & 31)); }

struct ChunkWalk {
    const uint2* pool;
    const unsigned long long* meta;
    const uint32_t* order;
    const int64_t* jst;
    const int64_t* segbase;
    const int* ja;
    int nt;
};

// A chunked partition (chunk_partition below) as its consumers walk it.
// Block w visits the pairs (x, y) (relative ids; the bucket follows y) of its chunk share in
// slice order: visit(pair, j) per pair; at every slice change and at the end flush(j) runs between
// barriers (it must also clear the block's accumulators).  The next chunk is loaded while the
// current one is visited.
struct NoBegin {
    __device__ void operator()(int) const {}
};

// begin(j) runs (between barriers) before the first pair of each slice the block visits.
// Inside a slice visit each wave takes whole chunks from an LDS cursor and walks them 512 pairs at
// a time (four 16-byte loads per lane, all issued before the pairs are visited), with the next
// chunk's ids fetched ahead: a part-full chunk (most of them when the slices are many) costs its own
// pairs, not a pass of the whole block.  Visits must not depend on the order of the pairs.
// (G, the chunks in flight of the former block-per-chunk walk, is kept for the callers.)
constexpr int kWalkItems = 8;  // pairs per lane per walk step (four 16-byte loads)

// The walk below with the visit taking a lane's whole step: visit(pr, valid, j), pr[k] valid where
// bit k of `valid` is set (entries past a chunk's fill read as zero pairs).  Lets a visit issue the
// gathers of all its items before it uses any (a per-item visit waits for each in turn).
template <int BLK, int G = 1, class VisitN, class Flush, class Begin = NoBegin>
__device__ void walk_chunks_n(const ChunkWalk& cw, VisitN visit, Flush flush, Begin begin = Begin()) {
    constexpr int kLd = kWalkItems / 2;    // 16-byte loads per lane per step
    constexpr uint32_t kStep = 64 * kLd * 2;  // pairs per wave step
    __shared__ uint32_t qn;                // next chunk of the slice visit
    const int64_t w = blockIdx.x, blocks = gridDim.x;
    const SegSplit S(cw.jst, cw.nt, blocks);
    const int64_t qb = w * S.per, qe = min(qb + S.per, S.nch);
    if (qb >= qe) return;  // block-uniform
    const int lane = threadIdx.x & 63;
    auto grab = [&]() -> uint32_t {  // wave-uniform
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(&qn, 1u);
        return __shfl(t, 0, 64);
    };
    int cur_j = slice_of(cw.jst, cw.nt, qb);
    for (;;) {  // block-uniform: one visit per slice of the share
        const int64_t c0 = max(qb, cw.jst[cur_j]), c1 = min(qe, cw.jst[cur_j + 1]);
        if (threadIdx.x == 0) qn = 0;
        begin(cur_j);
        __syncthreads();
        const int j = cur_j;
        uint32_t t = grab(), phys = 0, fill = 0;
        if (c0 + t < c1) {
            phys = cw.order[c0 + t];
            fill = (uint32_t)(cw.meta[phys] >> 32);
        }
        while (c0 + t < c1) {  // wave-uniform
            const uint32_t tn = grab();
            uint32_t pn = 0, fn = 0;
            if (c0 + tn < c1) {
                pn = cw.order[c0 + tn];
                fn = (uint32_t)(cw.meta[pn] >> 32);
            }
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint2*>(cw.pool + (size_t)phys * kCh), (short)0, (int)(fill * sizeof(uint2)), 0x00020000);
            for (uint32_t o = 0; o < fill; o += kStep) {  // wave-uniform
                uint2 pr[2 * kLd];
#pragma unroll
                for (int k = 0; k < kLd; ++k) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(
                        rs, (o + 2u * (uint32_t)(k * 64 + lane)) * 8u, 0, 2);  // nt
                    pr[2 * k] = make_uint2(v[0], v[1]);
                    pr[2 * k + 1] = make_uint2(v[2], v[3]);
                }
                uint32_t valid = 0;
#pragma unroll
                for (int k = 0; k < 2 * kLd; ++k)
                    valid |= (o + 2u * (uint32_t)((k >> 1) * 64 + lane) + (uint32_t)(k & 1) < fill ? 1u : 0u) << k;
                visit(pr, valid, j);
            }
            t = tn;
            phys = pn;
            fill = fn;
        }
        __syncthreads();
        flush(cur_j);
        if (c1 >= qe) break;
        do {
            ++cur_j;
        } while (cw.jst[cur_j + 1] <= cw.jst[cur_j]);  // empty slices are skipped
        __syncthreads();
    }
}

template <int BLK, int G = 1, class Visit, class Flush, class Begin = NoBegin>
__device__ void walk_chunks(const ChunkWalk& cw, Visit visit, Flush flush, Begin begin = Begin()) {
    walk_chunks_n<BLK, G>(
        cw,
        [&](const uint2 (&pr)[kWalkItems], uint32_t valid, int j) {
#pragma unroll
            for (int k = 0; k < kWalkItems; ++k)
                if ((valid >> k) & 1u) visit(pr[k], j);
        },
        flush, begin);
}

// whether block w's chunk share holds all of slice j's chunks (then its flush owns the slice)
__device__ __forceinline__ bool owns_slice(const ChunkWalk& cw, int j) {
    const SegSplit S(cw.jst, cw.nt, gridDim.x);
    const int64_t qb = (int64_t)blockIdx.x * S.per, qe = min(qb + S.per, S.nch);
    return qb <= cw.jst[j] && qe >= cw.jst[j + 1];
}

}  // namespace part

// Pass 1 of the partition plus chunk ordering and the block-balanced segment split (k_part.hip):
// relationships grouped by bucket = (y >> L.tbits) of their packed (x, y) = (source - lo, target - lo)
// pair, in chunks of kCh pairs; with `swap` the pair is (target, source) and buckets follow the
// source.  Blocks of a consumer kernel launched with g2 blocks walk segments via part::seg_of.
struct ChunkPart {
    part::Layout L;
    Buf pool, meta, chist, jbuf;
    int64_t pool_chunks = 0, npool = 1, mtot = 0, g2 = 1;
    int64_t* jst = nullptr;      // nt + 1 chunk offsets per bucket in `order`
    int64_t* segbase = nullptr;  // g2 + 1
    int* ja = nullptr;           // first bucket per block
    uint32_t* order = nullptr;   // used chunks grouped by bucket
};
void chunk_partition(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                     int nt, bool swap, const part::Layout& L, int64_t g2, ChunkPart& cp);
// the ordering half of chunk_partition for a pool another kernel filled (cp.meta: bucket | fill << 32)
void chunk_order(capsmi_session* s, int nt, int64_t pool_chunks, int64_t g2, ChunkPart& cp);

// the record form in phases (k_count.hip): begin = partition + in-degree walk, fold = the owned
// ids' in-degrees for an all-gather, finish = the out walk over all ids' in-degrees
struct CountRec {
    capsmi_session* s = nullptr;
    int64_t n = 0, mtot = 0;
    int nb = 0;
    const uint32_t* bw = nullptr;
    int b_full = 0;
    Buf inA, corr, acc;
    ChunkPart cp;
};
void count_rec_begin(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                     const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, CountRec& cr,
                     bool undirected = false);
void count_rec_fold(CountRec& cr, int64_t own_lo, int64_t own_hi, uint32_t* out);
int64_t count_rec_finish(CountRec& cr, const uint32_t* in_all, int64_t* dev_out);


}  // namespace capsmi
