// k_count.hip -- count(*) of the 2-hop Expand chain without per-relationship global atomics.
//
//   MATCH (a)-[r1]->(b)-[r2]->(c) WHERE a_ok(a) AND b_ok(b) AND c_ok(c) RETURN count(*)
//
// CAPS counts the rows of join(join(a, r1), b) ... with the uniqueness filter NOT(r1 = r2)
// (RelationalPlanner.scala:113-177, count(*) AggregationBehaviour); the closed form is
//   count(*) = sum_b b_ok(b) inA(b) outC(b) - #{self-loops b->b with a_ok, b_ok, c_ok}
//   inA(b) = #{r: x -> b, a_ok(x)},  outC(b) = #{r: b -> y, c_ok(y)}
// (oracle/closed.c orc_two_hop_closed_form_mt).  The atomic form (k_graph.hip k_degrees) adds one
// global atomic per relationship to a random counter -- memory-side, uncached, 2^31 of them at C3.
// Here one read of the relationships emits two 2-byte records per relationship into 2 x 1024 buckets of
// 2^16 ids (the record partition below), and two walks count them in LDS.  (Round 2's form -- two 8-byte
// pair partitions of 2^15-id slices with 32-bit LDS counts -- took 23.9 ms against 9.7 at C3 and was
// removed in round 6; a pass 2 over the relationships in table order, gathering inA(source) from HBM,
// measured 19.6 ms.)
#include <mutex>

#include "part_common.h"

namespace capsmi {
namespace cnt {

__device__ __forceinline__ void block_add(unsigned long long v, unsigned long long* out) {
    __shared__ unsigned long long red;
    if (threadIdx.x == 0) red = 0;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&red, v);
    __syncthreads();
    if (threadIdx.x == 0 && red) atomicAdd(out, red);
}

}  // namespace cnt

// ---- count(*) partitions of 2-byte records -----------------------------------------------------------
// A pair partition writes 8 bytes per relationship into 2048 buckets, and at 4 pairs per bucket per
// tile its chunk tails are partial lines (k_scatter_c ran at 2.7 TB/s).  A count needs
// less: the in-pass needs only the target of a relationship whose source passes a_ok, the out-pass
// only the source of one whose target passes c_ok.  So each pass here writes one 2-byte record per
// kept relationship -- the id's low 16 bits, the bucket being the id's high bits (2^16 ids, <= 1024
// buckets) -- and a bucket's records leave the workgroup as whole 64-byte pieces: a tile's run is
// appended behind the < 32 records the bucket holds back in LDS, every complete piece is stored,
// the rest is held for the next tile.  The walks count a bucket in 16-bit LDS counters (128 KiB)
// with exact wrap corrections: 16 + 2 + 2 bytes per relationship and pass, against 16 + 8 + 8 for
// the pair partition.
namespace rec {

constexpr int kBits = 16;        // ids per bucket
constexpr int kB = 1024;         // workgroup
constexpr int kIT = 8;           // relationships per lane per tile
constexpr int kT = kB * kIT;     // relationships per tile
#ifndef CAPSMI_REC_PIECE
#define CAPSMI_REC_PIECE 16
#endif
constexpr int kPiece = CAPSMI_REC_PIECE;  // records per piece store (8 or 16: one or two 16-byte lanes)
static_assert(kPiece == 8 || kPiece == 16, "a piece is one or two 16-byte lane stores");
constexpr int kPieceLanes = kPiece / 8;
constexpr int kCh = 8192;        // records per chunk (16 KiB; one 16-byte load per walk lane)
constexpr int kMaxBuckets = 1024;  // per side
constexpr int kBig = 255;        // OUT walk: values >= 0xFF00 per bucket kept exactly in LDS
constexpr size_t walk_lds() { return sizeof(uint32_t) * ((1 << (kBits - 1)) + kBig + 2); }
constexpr uint32_t kNone = 0xFFFFFFFFu;

// nb2 = buckets of both sides
// pieces of one tile: (held + run records) / kPiece summed over the buckets
__host__ __device__ constexpr int max_pieces(int nb2) { return (2 * kT + nb2 * (kPiece - 1)) / kPiece; }

__host__ __device__ constexpr size_t part_lds(int nb2) {
    return sizeof(uint16_t) * (2 * (size_t)kT + (size_t)nb2 * kPiece) + sizeof(uint16_t) * 2 * (size_t)nb2 +
           sizeof(uint32_t) * (6 * (size_t)nb2 + kB / 64 + 4) + sizeof(uint16_t) * (size_t)max_pieces(nb2);
}

// relationships per lane and per tile: the undirected form emits up to four records per relationship
// (both arcs), so its tiles hold half the relationships and the same 2 kT records
__host__ __device__ constexpr int part_it(bool und) { return und ? kIT / 2 : kIT; }

__host__ __device__ constexpr int64_t chunks_per_block(int64_t m, int64_t grid, int nb2, bool und = false) {
    // full chunks of the block's records (2 kT per tile at most), plus per bucket the open one and one
    // retired part-full by the final flush
    const int64_t T = (int64_t)kB * part_it(und);
    return ((((m + T - 1) / T + grid - 1) / grid) * 2 * kT + kCh - 1) / kCh + 2 * (int64_t)nb2 + 1;
}

__device__ __forceinline__ bool bit(const part::BitV& v, uint64_t x) { return v.full || part::gbit(v.w, (uint32_t)x); }

// FULL: every node filter full (a query without node predicates) -- the tests fold away and the filter views
// leave the kernel's scalar registers (the general form spills them to VGPR lanes).  Taken for the undirected
// form only: C3u's und_count_part 11.50 -> 10.63 ms; the directed form, already at 128 VGPRs, spills 108 bytes
// to scratch when specialised -- the 64-bit addresses of its misaligned / last-tile load path -- and
// count_part goes 6.94 -> 10.85 ms
template <bool FULL>
__device__ __forceinline__ bool fbit(const part::BitV& v, uint64_t x) { return FULL || bit(v, x); }

// One read of the relationships, two record kinds into 2 * nb buckets:
//   bucket t >> 16        (the in side):  t & 0xFFFF for relationships s -> t with a_ok(s);
//   bucket nb + (s >> 16) (the out side): s & 0xFFFF for relationships s -> t with c_ok(t);
// the a_ok, b_ok, c_ok self-loops are counted into `loops`.
// UND (undirected 2-hop, RelationalPlanner.scala:126-136: out ∪ in-without-loops per hop): each relationship
// s -> t is the arc s -> t and, when s != t, the arc t -> s; every arc x -> y gives an in record of y when
// a_ok(x) and an out record of x when c_ok(y), so the walks give sum_b b_ok(b) inU(b) outU(b); `loops`
// gets the bindings with r1 = r2 (a non-loop walked in and back out, [a(s) b(t) c(s)] + [a(t) b(s) c(t)], a
// loop [a b c](s)).
// One block scan for both per-bucket prefixes of a tile (k_rec_part): the record runs (loc, of cnt) and the
// pieces the held + run records complete (pb, of pc = (hc + cnt) / kPiece), as the 16-bit halves of one word
// (a tile holds at most 2 kT = 2^14 records and fewer than 2^12 pieces, so the low half never carries); the
// pre-pass also opens the chunks the pieces need.  Three barriers where two scans and the pass between them
// took seven.  Returns the tile's piece count.
__device__ uint32_t scan_runs_pieces(const uint32_t* cnt, const uint16_t* hc, const uint16_t* fl, uint32_t* loc,
                                     uint32_t* pc, uint32_t* pb, uint32_t* np, uint32_t* misc, int n,
                                     uint32_t* wtot) {
    const int per = (n + kB - 1) / kB;
    const int b = threadIdx.x * per;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t sum = 0;
    for (int k = 0; k < per; ++k)
        if (b + k < n) {
            const int i = b + k;
            const uint32_t c = cnt[i], npc = ((uint32_t)hc[i] + c) / kPiece;
            pc[i] = npc;
            if (npc) {  // pieces take positions [fl, fl + npc * kPiece): chunk index pos / kCh past ph
                const uint32_t nnew = ((uint32_t)fl[i] + npc * kPiece - 1) / kCh;
                if (nnew) np[i] = atomicAdd(&misc[0], nnew);
            }
            sum += c | npc << 16;
        }
    uint32_t x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        uint32_t v = lane < kB / 64 ? wtot[lane] : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(v, o, 64);
            if (lane >= o) v += y;
        }
        if (lane < kB / 64) wtot[lane] = v;
    }
    __syncthreads();
    uint32_t pre = x - sum + (wave > 0 ? wtot[wave - 1] : 0u);
    for (int k = 0; k < per; ++k)
        if (b + k < n) {
            const int i = b + k;
            loc[i] = pre & 0xFFFFu;
            pb[i] = pre >> 16;
            pre += cnt[i] | pc[i] << 16;
        }
    const uint32_t total = wtot[kB / 64 - 1];
    __syncthreads();
    return total >> 16;
}

template <bool UND, bool FULL = false>
__global__ void __launch_bounds__(kB) k_rec_part(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                 int64_t m, int64_t lo, int64_t range, int nb, part::BitV a, part::BitV b,
                                                 part::BitV c, int64_t chunk0, int64_t cpb, uint16_t* __restrict__ pool,
                                                 unsigned long long* __restrict__ cmeta,
                                                 unsigned long long* __restrict__ loops) {
    constexpr int IT = part_it(UND), T = kB * IT;
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    const int nb2 = 2 * nb;
    uint16_t* stage = reinterpret_cast<uint16_t*>(sm);  // 2 kT: this tile's records grouped by bucket
    uint16_t* hold = stage + 2 * kT;                     // nb2 x kPiece: records held back per bucket
    uint16_t* hc = hold + (size_t)nb2 * kPiece;          // records held (< kPiece)
    uint16_t* fl = hc + nb2;                             // records stored in the open chunk (kCh: none open)
    uint32_t* cnt = reinterpret_cast<uint32_t*>(fl + nb2);  // run length this tile
    uint32_t* loc = cnt + nb2;  // run start in the stage
    uint32_t* ph = loc + nb2;   // open chunk
    uint32_t* np = ph + nb2;    // first of the chunks opened for this tile's pieces (consecutive)
    uint32_t* pc = np + nb2;    // pieces stored this tile
    uint32_t* pb = pc + nb2;    // first piece of the bucket this tile
    uint32_t* wtot = pb + nb2;
    uint32_t* misc = wtot + kB / 64;  // [0] next free chunk of this block
    uint16_t* owner = reinterpret_cast<uint16_t*>(misc + 4);  // bucket of each piece of the tile
    for (int i = threadIdx.x; i < nb2; i += kB) {
        cnt[i] = 0;
        hc[i] = 0;
        fl[i] = (uint16_t)kCh;
        ph[i] = kNone;
    }
    if (threadIdx.x == 0) misc[0] = (uint32_t)(chunk0 + (int64_t)blockIdx.x * cpb);
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const int64_t stride = (int64_t)gridDim.x * T;
    unsigned long long nl = 0;
    int64_t sr[IT], tr[IT];
    int64_t t0 = (int64_t)blockIdx.x * T;
    if (t0 < m) part::load_tile<kB>(src, dst, t0, m, vec, sr, tr);
    __syncthreads();
    for (; t0 < m; t0 += stride) {  // block-uniform
        uint32_t xs[IT], ys[IT], rin[IT], rout[IT], rin2[UND ? IT : 1], rout2[UND ? IT : 1];
        uint32_t vin = 0, vout = 0, vin2 = 0, vout2 = 0;
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            const int64_t e = t0 + part::item_off<kB>(u);
            const uint64_t x = (uint64_t)(sr[u] - lo), y = (uint64_t)(tr[u] - lo);
            const bool ok = e < m && x < (uint64_t)range && y < (uint64_t)range;
            const bool ain = ok && fbit<FULL>(a, x), aout = ok && fbit<FULL>(c, y);
            if constexpr (!UND) {
                if (ain && x == y && fbit<FULL>(b, x) && fbit<FULL>(c, x)) ++nl;
            } else if (ok) {  // the reverse arc y -> x of a non-loop, and the r1 = r2 bindings
                const bool ay = fbit<FULL>(a, y), cx = fbit<FULL>(c, x), bx = fbit<FULL>(b, x), by = fbit<FULL>(b, y);
                const bool two = x != y;
                vin2 |= (two && ay ? 1u : 0u) << u;
                vout2 |= (two && cx ? 1u : 0u) << u;
                nl += two ? (ain && by && cx ? 1 : 0) + (ay && bx && aout ? 1 : 0) : (ain && bx && cx ? 1 : 0);
            }
            xs[u] = (uint32_t)x;
            ys[u] = (uint32_t)y;
            vin |= (ain ? 1u : 0u) << u;
            vout |= (aout ? 1u : 0u) << u;
        }
        if (t0 + stride < m) part::load_tile<kB>(src, dst, t0 + stride, m, vec, sr, tr);  // prefetch
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            rin[u] = ((vin >> u) & 1u) ? atomicAdd(&cnt[ys[u] >> kBits], 1u) : 0u;
            rout[u] = ((vout >> u) & 1u) ? atomicAdd(&cnt[nb + (xs[u] >> kBits)], 1u) : 0u;
            if constexpr (UND) {
                rin2[u] = ((vin2 >> u) & 1u) ? atomicAdd(&cnt[xs[u] >> kBits], 1u) : 0u;
                rout2[u] = ((vout2 >> u) & 1u) ? atomicAdd(&cnt[nb + (ys[u] >> kBits)], 1u) : 0u;
            }
        }
        __syncthreads();
        const uint32_t P = scan_runs_pieces(cnt, hc, fl, loc, pc, pb, np, misc, nb2, wtot);
#pragma unroll
        for (int u = 0; u < IT; ++u) {
            if ((vin >> u) & 1u) stage[loc[ys[u] >> kBits] + rin[u]] = (uint16_t)(ys[u] & 0xFFFFu);
            if ((vout >> u) & 1u) stage[loc[nb + (xs[u] >> kBits)] + rout[u]] = (uint16_t)(xs[u] & 0xFFFFu);
            if constexpr (UND) {
                if ((vin2 >> u) & 1u) stage[loc[xs[u] >> kBits] + rin2[u]] = (uint16_t)(xs[u] & 0xFFFFu);
                if ((vout2 >> u) & 1u) stage[loc[nb + (ys[u] >> kBits)] + rout2[u]] = (uint16_t)(ys[u] & 0xFFFFu);
            }
        }
        for (int i = threadIdx.x; i < nb2; i += kB) {  // piece -> bucket; pc becomes the first held rank
            const uint32_t npc = pc[i];
            for (uint32_t k = 0; k < npc; ++k) owner[pb[i] + k] = (uint16_t)i;
            pc[i] = npc * kPiece - (uint32_t)hc[i];  // a run item of rank >= this (signed) is held
        }
        __syncthreads();
        // piece g: kPieceLanes lanes x 8 records; element e < held comes from the hold, the rest from the run
        for (uint32_t x = threadIdx.x; x < P * kPieceLanes; x += kB) {
            const uint32_t g = x / kPieceLanes, r = x % kPieceLanes;
            const int bk = owner[g];
            const uint32_t k = g - pb[bk], h = hc[bk];
            uint16_t v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t e = k * kPiece + r * 8 + (uint32_t)q;
                v[q] = e < h ? hold[bk * kPiece + (int)e] : stage[loc[bk] + e - h];
            }
            const uint32_t pos = (uint32_t)fl[bk] + k * kPiece, ci = pos / kCh;
            const uint32_t ch = ci == 0 ? ph[bk] : np[bk] + ci - 1;
            const uint32_t off = pos - ci * kCh + r * 8;
            uint4 w;
            w.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
            w.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
            w.z = (uint32_t)v[4] | ((uint32_t)v[5] << 16);
            w.w = (uint32_t)v[6] | ((uint32_t)v[7] << 16);
            *reinterpret_cast<uint4*>(pool + (size_t)ch * kCh + off) = w;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < IT; ++u) {  // the new held records: the run's items past its last whole piece
            if ((vin >> u) & 1u) {
                const uint32_t bk = ys[u] >> kBits;
                const int d = (int)rin[u] - (int)pc[bk];
                if (d >= 0) hold[bk * kPiece + d] = (uint16_t)(ys[u] & 0xFFFFu);
            }
            if ((vout >> u) & 1u) {
                const uint32_t bk = nb + (xs[u] >> kBits);
                const int d = (int)rout[u] - (int)pc[bk];
                if (d >= 0) hold[bk * kPiece + d] = (uint16_t)(xs[u] & 0xFFFFu);
            }
            if constexpr (UND) {
                if ((vin2 >> u) & 1u) {
                    const uint32_t bk = xs[u] >> kBits;
                    const int d = (int)rin2[u] - (int)pc[bk];
                    if (d >= 0) hold[bk * kPiece + d] = (uint16_t)(xs[u] & 0xFFFFu);
                }
                if ((vout2 >> u) & 1u) {
                    const uint32_t bk = nb + (ys[u] >> kBits);
                    const int d = (int)rout2[u] - (int)pc[bk];
                    if (d >= 0) hold[bk * kPiece + d] = (uint16_t)(ys[u] & 0xFFFFu);
                }
            }
        }
        // (no barrier: the bookkeeping below reads and writes neither `hold` nor `pc`, the held records above
        // touch nothing else; both only had to follow the piece stores)
        for (int i = threadIdx.x; i < nb2; i += kB) {
            const uint32_t tot = (uint32_t)hc[i] + cnt[i], npc = tot / kPiece;
            if (npc) {
                const uint32_t end = (uint32_t)fl[i] + npc * kPiece, nnew = (end - 1) / kCh;
                if (nnew) {  // the chunks filled by this tile are retired, the last one opened stays open
                    if (ph[i] != kNone) cmeta[ph[i]] = part::chunk_meta(i, (uint32_t)kCh);
                    for (uint32_t t = 0; t + 1 < nnew; ++t) cmeta[np[i] + t] = part::chunk_meta(i, (uint32_t)kCh);
                    ph[i] = np[i] + nnew - 1;
                    fl[i] = (uint16_t)(end - nnew * kCh);
                } else {
                    fl[i] = (uint16_t)end;
                }
            }
            hc[i] = (uint16_t)(tot - npc * kPiece);
            cnt[i] = 0;
        }
        __syncthreads();
    }
    // the held records: into the open chunk, or a new one when there is none or it is full
    for (int i = threadIdx.x; i < nb2; i += kB) {
        if (hc[i] && (ph[i] == kNone || (uint32_t)fl[i] + hc[i] > (uint32_t)kCh)) {
            if (ph[i] != kNone) cmeta[ph[i]] = part::chunk_meta(i, fl[i]);
            ph[i] = atomicAdd(&misc[0], 1u);
            fl[i] = 0;
        }
    }
    __syncthreads();
    for (int x = threadIdx.x; x < nb2 * kPiece; x += kB) {
        const int bk = x / kPiece, e = x % kPiece;
        if ((uint32_t)e < hc[bk]) pool[(size_t)ph[bk] * kCh + fl[bk] + (uint32_t)e] = hold[x];
    }
    for (int i = threadIdx.x; i < nb2; i += kB)
        if (ph[i] != kNone) cmeta[ph[i]] = part::chunk_meta(i, (uint32_t)fl[i] + hc[i]);
    cnt::block_add(nl, loops);
}

// Walk of a record partition in bucket order, one pass per bucket: the bucket's 2^16 ids as 16-bit
// LDS counters, two per word (128 KiB).
//   OUT = false: inA(t) counted with word atomics; a counter that wraps is corrected exactly in
//     `corr` (global, rare: ids with >= 2^16 in-relationships): a low half going 0xFFFF -> 0 adds
//     2^16 to its id and, through the carry, 1 too many to the high id; a high half wrapping (its
//     own add, or a carry into 0xFFFF) adds 2^16 to the high id.  Counts are stored through b_ok
//     at each bucket change.
//   OUT = true: inA + corr of the bucket staged as saturated 16-bit values; 0xFFFF (>= 2^16)
//     reads the exact value from HBM.  sum += inA(s) per record.
template <bool OUT>
__global__ void __launch_bounds__(kB) k_rec_walk(const uint16_t* __restrict__ pool,
                                                 const unsigned long long* __restrict__ meta,
                                                 const uint32_t* __restrict__ order, const int64_t* __restrict__ jst,
                                                 int nb, int64_t n, part::BitV b, uint32_t* __restrict__ inA,
                                                 int32_t* __restrict__ corr, unsigned long long* __restrict__ sum) {
    extern __shared__ uint32_t cl[];  // 2^15 words = 2^16 16-bit counters / staged values
    constexpr int kWords = 1 << (kBits - 1);
    uint32_t* bigv = cl + kWords;  // OUT: exact values behind 0xFF00 + k
    uint32_t* nbig = bigv + kBig;
    uint32_t* qn = nbig + 1;  // next chunk of the bucket visit (waves take chunks from it)
    const int lane = threadIdx.x & 63;
    // jst: nb + 1 bucket starts in `order` (the side's buckets of the two-sided partition, so
    // jst[0] need not be 0); block w takes an equal share of the side's chunks
    const int64_t q00 = jst[0], nch = jst[nb] - q00;
    int64_t per = (nch + gridDim.x - 1) / gridDim.x;
    if (per < 1) per = 1;
    const int64_t qb = q00 + (int64_t)blockIdx.x * per, qe = min(qb + per, q00 + nch);
    unsigned long long acc = 0;
    if (qb < qe) {  // block-uniform
        auto exact = [&](int64_t x) -> uint32_t {  // OUT: the stored count of id x (corr null: folded already)
            if (x >= n) return 0u;
            if (!corr) return inA[x];
            return bit(b, (uint64_t)x) ? (uint32_t)((int64_t)inA[x] + corr[x]) : 0u;
        };
        auto slot16 = [&](uint32_t v) -> uint32_t {  // OUT: a value as its 16-bit slot
            if (v < 0xFF00u) return v;
            const uint32_t k = atomicAdd(nbig, 1u);
            if (k < (uint32_t)kBig) {
                bigv[k] = v;
                return 0xFF00u + k;
            }
            return 0xFFFFu;  // read from HBM
        };
        auto begin = [&](int j) {
            const int64_t base = (int64_t)j << kBits;
            if (threadIdx.x == 0) {
                *qn = 0;
                *nbig = 0;
            }
            __syncthreads();
            for (int i = threadIdx.x; i < kWords; i += kB) {
                uint32_t w = 0;
                if (OUT) w = slot16(exact(base + 2 * i)) | (slot16(exact(base + 2 * i + 1)) << 16);
                cl[i] = w;
            }
        };
        auto flush = [&](int j) {
            if (OUT) return;
            const bool own = qb <= jst[j] && qe >= jst[j + 1];  // else the bucket's other blocks add to it too
            const int64_t base = (int64_t)j << kBits;
            for (int i = threadIdx.x; i < kWords; i += kB) {
                const uint32_t w = cl[i];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int64_t x = base + 2 * i + h;
                    if (x < n) {
                        const uint32_t keep = bit(b, (uint64_t)x) ? (h ? w >> 16 : w & 0xFFFFu) : 0u;
                        if (own) inA[x] = keep;
                        else if (keep) atomicAdd(&inA[x], keep);
                    }
                }
            }
        };
        auto grab = [&]() -> uint32_t {  // the wave's next chunk of the visit (wave-uniform)
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(qn, 1u);
            return __shfl(t, 0, 64);
        };
        // records r of a 16-byte group at [8 * lane-group, + 8): lim = records of it below the fill
        auto walk8 = [&](const uint4 v0, int lim, int64_t base) {
            const uint32_t w[4] = {v0.x, v0.y, v0.z, v0.w};
            // all 8 LDS accesses are issued before any result is used; the wrap test is one
            // compare per record, its (rare) corrections out of line
            uint32_t got[8], rr[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                rr[e] = __builtin_amdgcn_ubfe(w[e >> 1], 16 * (e & 1), 16);
                got[e] = 0u;
                if (e < lim) {
                    uint32_t* word = &cl[rr[e] >> 1];
                    got[e] = OUT ? *word : atomicAdd(word, 1u << ((rr[e] & 1u) << 4));
                }
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (e >= lim) continue;
                const uint32_t v = __builtin_amdgcn_ubfe(got[e], (rr[e] & 1u) << 4, 16);
                if (OUT) {
                    acc += v < 0xFF00u ? v : v != 0xFFFFu ? bigv[v - 0xFF00u] : exact(base + rr[e]);
                } else if (v == 0xFFFFu) {  // this add wrapped its half (rare: ids with >= 2^16 in-relationships)
                    const int64_t xl = base + (rr[e] & ~1u), xh = xl + 1;
                    if (!(rr[e] & 1u)) {  // low half: + 2^16 to it, and the carry went into the high half
                        atomicAdd(&corr[xl], 65536);
                        if (xh < n) atomicAdd(&corr[xh], (got[e] >> 16) == 0xFFFFu ? 65535 : -1);  // carry wrapped high too
                    } else {
                        atomicAdd(&corr[xh], 65536);
                    }
                }
            }
        };
        // One visit per bucket the share touches.  Inside a visit each wave takes whole chunks from
        // an LDS cursor and walks them 512 records (one 16-byte load per lane) at a time, so a
        // part-full chunk costs its own records, not a whole block's pass.
        int cur_j = part::slice_of(jst, nb, qb);
        for (;;) {  // block-uniform
            const int64_t c0 = max(qb, jst[cur_j]), c1 = min(qe, jst[cur_j + 1]);
            begin(cur_j);
            __syncthreads();
            const int64_t base = (int64_t)cur_j << kBits;
            uint32_t t = grab();
            uint32_t phys = 0, fill = 0;
            if (c0 + t < c1) {
                phys = order[c0 + t];
                fill = (uint32_t)(meta[phys] >> 32);
            }
            while (c0 + t < c1) {  // wave-uniform
                const uint32_t tn = grab();  // the next chunk's ids are fetched while this one is walked
                uint32_t pn = 0, fn = 0;
                if (c0 + tn < c1) {
                    pn = order[c0 + tn];
                    fn = (uint32_t)(meta[pn] >> 32);
                }
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint16_t*>(pool + (size_t)phys * kCh), (short)0,
                    (int)((fill * sizeof(uint16_t) + 15) & ~(size_t)15), 0x00020000);  // whole dwords: masked by lim
                // two 512-record groups in flight per wave (one 16-byte load per lane each)
                auto x0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)lane * 16u, 0, 2);
                auto x1 = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024u + (uint32_t)lane * 16u, 0, 2);
                for (uint32_t o = 0; o < fill; o += 1024) {  // wave-uniform
                    const uint4 v0 = make_uint4(x0[0], x0[1], x0[2], x0[3]);
                    const uint4 v1 = make_uint4(x1[0], x1[1], x1[2], x1[3]);
                    if (o + 1024 < fill) {
                        x0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (o + 1024) * 2u + (uint32_t)lane * 16u, 0, 2);
                        x1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (o + 1536) * 2u + (uint32_t)lane * 16u, 0, 2);
                    }
                    walk8(v0, (int)(fill - o) - lane * 8, base);
                    if (o + 512 < fill) walk8(v1, (int)(fill - o) - 512 - lane * 8, base);
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
            } while (jst[cur_j + 1] <= jst[cur_j]);  // empty buckets are skipped
            __syncthreads();
        }
    }
    if (OUT) cnt::block_add(acc, sum);
}

}  // namespace rec

namespace rec {

// owned in-degrees, folded: out[x - own_lo] = b_ok(x) ? inA(x) + corr(x) : 0
__global__ void k_rec_fold(const uint32_t* __restrict__ inA, const int32_t* __restrict__ corr, part::BitV b,
                           int64_t own_lo, int64_t own_hi, uint32_t* __restrict__ out) {
    for (int64_t x = own_lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < own_hi;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x - own_lo] = bit(b, (uint64_t)x) ? (uint32_t)((int64_t)inA[x] + corr[x]) : 0u;
}

__global__ void k_rec_result(const unsigned long long* __restrict__ acc, int64_t* __restrict__ out) {
    *out = (int64_t)(acc[1] - acc[0]);  // sum - self-loops
}

}  // namespace rec

// phase 1: the two-sided record partition and the IN walk (inA of every target this table holds)
void count_rec_begin(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                     const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, CountRec& cr,
                     bool undirected) {
    using namespace rec;
    const int64_t lo = b_ok->lo, n = b_ok->hi - b_ok->lo;
    const part::BitV a{P<uint32_t>(a_ok->words), a_ok->full ? 1 : 0}, b{P<uint32_t>(b_ok->words), b_ok->full ? 1 : 0},
        c{P<uint32_t>(c_ok->words), c_ok->full ? 1 : 0};
    hipStream_t st = s->stream;
    const int nb = (int)((n + (int64_t(1) << kBits) - 1) >> kBits);
    REQUIRE(nb >= 1 && nb <= kMaxBuckets, CAPSMI_ERR_INTERNAL, "count(*) records: domain too large");
    cr.s = s;
    cr.n = n;
    cr.nb = nb;
    cr.bw = b.w;
    cr.b_full = b.full;
    cr.inA = dev_alloc(sizeof(uint32_t) * (size_t)n, s);
    cr.corr = dev_alloc(sizeof(int32_t) * (size_t)n, s);  // wrap corrections of the 16-bit LDS counters
    cr.acc = dev_alloc(2 * sizeof(unsigned long long), s);  // loops, sum
    HIP_CHECK(hipMemsetAsync(P<void>(cr.inA), 0, sizeof(uint32_t) * (size_t)n, st));
    HIP_CHECK(hipMemsetAsync(P<void>(cr.corr), 0, sizeof(int32_t) * (size_t)n, st));
    HIP_CHECK(hipMemsetAsync(P<void>(cr.acc), 0, 2 * sizeof(unsigned long long), st));
    static std::once_flag once;
    std::call_once(once, [] {
        for (const void* f : {reinterpret_cast<const void*>(k_rec_part<false>), reinterpret_cast<const void*>(k_rec_part<true>),
                              reinterpret_cast<const void*>(k_rec_part<true, true>)})
            HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)part_lds(2 * kMaxBuckets)));
        for (const void* f : {reinterpret_cast<const void*>(k_rec_walk<false>), reinterpret_cast<const void*>(k_rec_walk<true>)})
            HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)walk_lds()));
    });
    int64_t mtot = 0;
    std::vector<int> g1(nt, 0);
    std::vector<int64_t> c0(nt, 0), cpb(nt, 0);
    int64_t pool_chunks = 0;
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        mtot += ms[i];
        const int64_t T = (int64_t)kB * part_it(undirected);
        g1[i] = (int)std::max<int64_t>(1, std::min<int64_t>(s->num_cus, (ms[i] + 4 * T - 1) / (4 * T)));
        cpb[i] = chunks_per_block(ms[i], g1[i], 2 * nb, undirected);
        c0[i] = pool_chunks;
        pool_chunks += (int64_t)g1[i] * cpb[i];
    }
    REQUIRE(pool_chunks < (int64_t)INT32_MAX, CAPSMI_ERR_UNSUPPORTED, "relationship table too large for the count");
    cr.mtot = mtot;
    const int64_t npool = pool_chunks > 0 ? pool_chunks : 1;
    ChunkPart& cp = cr.cp;
    cp.L.lo = lo;
    cp.L.hi = lo + n;
    cp.L.nt = 2 * nb;
    {
        // read 2 x int64, write two 2-byte records (undirected: four)
        KernelTimer kt(s, undirected ? "und_count_part" : "count_part", (double)mtot * (undirected ? 24 : 20));
        cp.pool = dev_alloc(sizeof(uint16_t) * kCh * (size_t)npool, s);
        cp.meta = dev_alloc(sizeof(unsigned long long) * npool, s);
        HIP_CHECK(hipMemsetAsync(P<void>(cp.meta), 0, sizeof(unsigned long long) * npool, st));
        for (int i = 0; i < nt; ++i) {
            if (ms[i] <= 0) continue;
            const bool full = a.full && b.full && c.full && s->cfg.rec_full;  // (config CAPSMI_REC_FULL=0: general)
            auto kf = undirected ? (full ? k_rec_part<true, true> : k_rec_part<true>) : k_rec_part<false>;
            hipLaunchKernelGGL(kf, dim3(g1[i]), dim3(kB), part_lds(2 * nb), st,
                               srcs[i], dsts[i], ms[i], lo, n, nb, a, b, c, c0[i], cpb[i], P<uint16_t>(cp.pool),
                               P<unsigned long long>(cp.meta), P<unsigned long long>(cr.acc));
        }
        HIP_CHECK(hipGetLastError());
    }
    chunk_order(s, 2 * nb, pool_chunks, s->num_cus, cp);
    {
        KernelTimer kt(s, "count_in", (double)mtot * 2 + (double)n * 4);
        hipLaunchKernelGGL(k_rec_walk<false>, dim3((unsigned)s->num_cus), dim3(kB), walk_lds(), st, P<uint16_t>(cp.pool),
                           P<unsigned long long>(cp.meta), cp.order, cp.jst, nb, n, b, P<uint32_t>(cr.inA),
                           P<int32_t>(cr.corr), P<unsigned long long>(cr.acc) + 1);
        HIP_CHECK(hipGetLastError());
    }
}

// the folded in-degrees of ids [own_lo, own_hi) (domain-relative) into `out` (device)
void count_rec_fold(CountRec& cr, int64_t own_lo, int64_t own_hi, uint32_t* out) {
    using namespace rec;
    const part::BitV b{cr.bw, cr.b_full};
    if (own_hi > own_lo)
        hipLaunchKernelGGL(k_rec_fold, dim3((unsigned)std::min<int64_t>((own_hi - own_lo + 255) / 256, 4096)), dim3(256), 0,
                           cr.s->stream, P<uint32_t>(cr.inA), P<int32_t>(cr.corr), b, own_lo, own_hi, out);
    HIP_CHECK(hipGetLastError());
}

// phase 2: the OUT walk, sum of inA(source) over the out-records; in_all = every id's folded
// in-degree (null: this table's own, corrections applied on the fly).  The result (sum - the
// counted self-loops) goes to dev_out (device int64) when given, else it is returned.
int64_t count_rec_finish(CountRec& cr, const uint32_t* in_all, int64_t* dev_out) {
    using namespace rec;
    capsmi_session* s = cr.s;
    hipStream_t st = s->stream;
    const part::BitV b{cr.bw, cr.b_full};
    {
        KernelTimer kt(s, "count_out", (double)cr.mtot * 2 + (double)cr.n * 8);
        hipLaunchKernelGGL(k_rec_walk<true>, dim3((unsigned)s->num_cus), dim3(kB), walk_lds(), st, P<uint16_t>(cr.cp.pool),
                           P<unsigned long long>(cr.cp.meta), cr.cp.order, cr.cp.jst + cr.nb, cr.nb, cr.n, b,
                           in_all ? const_cast<uint32_t*>(in_all) : P<uint32_t>(cr.inA),
                           in_all ? nullptr : P<int32_t>(cr.corr), P<unsigned long long>(cr.acc) + 1);
        HIP_CHECK(hipGetLastError());
    }
    if (dev_out) {
        hipLaunchKernelGGL(k_rec_result, dim3(1), dim3(1), 0, st, P<unsigned long long>(cr.acc), dev_out);
        HIP_CHECK(hipGetLastError());
        return 0;
    }
    unsigned long long h[2];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(cr.acc), sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return (int64_t)(h[1] - h[0]);
}

// the same count from two record partitions (rec:: above); one id domain of at most 2^26 ids
int64_t two_hop_count_rec(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                          int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok,
                          bool undirected) {
    CountRec cr;
    count_rec_begin(s, srcs, dsts, ms, nt, a_ok, b_ok, c_ok, cr, undirected);
    return count_rec_finish(cr, nullptr, nullptr);
}

}  // namespace capsmi
