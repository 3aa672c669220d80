// k_undirected.hip -- undirected Expand patterns, fused.
//
// RelationalPlanner lowers an undirected Expand (a)-[r]-(b) to the union of the outgoing branch and
// the incoming branch over the relationships whose start differs from their end
// (okapi-relational/.../planning/RelationalPlanner.scala:126-136).  Viewed from a node, that is one
// step along an *arc* of the symmetrised relationship set: every relationship e = (s, t) gives the arc
// s -> t, and, when s != t, the arc t -> s.  The kernels below stream the relationship table once per
// phase and handle both arcs of a row; nothing is materialised.
//
// 2-hop (a)-[r1]-(b)-[r2]-(c), r1 <> r2 (the front-end's uniqueness predicate):
//   count(*) = sum_b b_ok(b) inU(b) outU(b) - corr, with inU(b) = a_ok arcs into b, outU(b) = c_ok arcs
//     out of b, and corr the bindings with r1 = r2: a non-loop e = (s, t) walked in and back out
//     ([a(s) b(t) c(s)] + [a(t) b(s) c(t)]), a loop walked once in and once out ([a b c](s));
//   count(DISTINCT c): per middle b, K(b) = the a_ok arcs into b, capped at 2, and for K = 1 the arc's
//     other end x(b).  An arc b -> c (e2) extends some binding iff K(b) = 2, or K(b) = 1 and e2 is not
//     the unique arc's relationship -- and since K(b) = 1 means exactly one relationship joins b and
//     x(b), that is c != x(b).  One 32-bit word per b: 0 (no arc), x + 1 (one arc from x), ~0 (two or
//     more), kept with a compare-and-swap and an exchange.
// Every test is against the node-scan bitmaps; relationships with an endpoint outside [lo, hi) have no
// node on that side and are skipped.
#include "capsmi_impl.h"

namespace capsmi {

namespace {


inline unsigned grid_for(int64_t n, int block = 256) {
    const int64_t g = (n + block - 1) / block;
    return (unsigned)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

struct Bits {
    const uint32_t* w;
    int full;
};
__device__ __forceinline__ bool ok(const Bits& b, int64_t x) {
    return b.full || ((b.w[x >> 5] >> (x & 31)) & 1u);
}

__device__ __forceinline__ void block_add(unsigned long long* acc, unsigned long long v) {
    __shared__ unsigned long long part[16];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) part[wave] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += part[i];
        if (t) atomicAdd(acc, t);
    }
    __syncthreads();  // part[] is reused by the next call: thread 0 must have read it first
}

// arcs leaving / entering each id and the r1 = r2 bindings (count(*) of the 2-hop, and the 1-hop arcs)
__global__ void k_und_deg(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                          int64_t n, Bits a, Bits b, Bits c, uint32_t* __restrict__ inU, uint32_t* __restrict__ outU,
                          unsigned long long* __restrict__ acc) {
    unsigned long long corr = 0, arcs = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        if (s < 0 || s >= n || t < 0 || t >= n) continue;
        const bool as = ok(a, s), bs = ok(b, s), cs = ok(c, s), at = ok(a, t), bt = ok(b, t), ct = ok(c, t);
        if (as && bt) {  // s -> t
            if (inU) atomicAdd(&inU[t], 1u);
            ++arcs;
        }
        if (outU && bs && ct) atomicAdd(&outU[s], 1u);
        if (s != t) {  // t -> s
            if (at && bs) {
                if (inU) atomicAdd(&inU[s], 1u);
                ++arcs;
            }
            if (outU && bt && cs) atomicAdd(&outU[t], 1u);
            corr += (as && bt && cs ? 1 : 0) + (at && bs && ct ? 1 : 0);
        } else {
            corr += as && bs && cs ? 1 : 0;
        }
    }
    block_add(&acc[0], corr);
    block_add(&acc[1], arcs);
}

__global__ void k_und_product(const uint32_t* __restrict__ inU, const uint32_t* __restrict__ outU, int64_t n,
                              unsigned long long* __restrict__ acc) {
    unsigned long long sum = 0;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x)
        sum += (unsigned long long)inU[x] * outU[x];
    block_add(&acc[2], sum);
}

// K(b) as two bitmaps (8 MiB each at 2^26 ids, cache-resident where the 4-byte state words were not):
// B1 = at least one a_ok arc into b, B2 = at least two; x(b) (the first arc's other end) is read only
// where K(b) = 1.  An arc reads B2 first -- hubs, which take most arcs, are settled by that one cached
// read -- then sets its B1 bit: the arc that found it clear is the first and stores x(b); one that found
// it set sets B2.
__device__ __forceinline__ bool bit_at(const uint32_t* w, int64_t i) { return (w[i >> 5] >> (i & 31)) & 1u; }

__device__ __forceinline__ void und_note(uint32_t* B1, uint32_t* B2, uint32_t* xb, int64_t b, int64_t x) {
    if (bit_at(B2, b)) return;
    const uint32_t m = 1u << (b & 31);
    if (atomicOr(&B1[b >> 5], m) & m) atomicOr(&B2[b >> 5], m);
    else xb[b] = (uint32_t)x;
}

// hop 1 of the distinct 2-hop: K(b) / x(b) from the a_ok arcs into b_ok ids
__global__ void k_und_hop1(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                           int64_t n, Bits a, Bits b, uint32_t* __restrict__ B1, uint32_t* __restrict__ B2,
                           uint32_t* __restrict__ xb) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        if (s < 0 || s >= n || t < 0 || t >= n) continue;
        if (ok(a, s) && ok(b, t)) und_note(B1, B2, xb, t, s);
        if (s != t && ok(a, t) && ok(b, s)) und_note(B1, B2, xb, s, t);
    }
}

__device__ __forceinline__ bool extends(const uint32_t* B1, const uint32_t* B2, const uint32_t* xb, int64_t b,
                                        int64_t c) {
    return bit_at(B2, b) || (bit_at(B1, b) && (int64_t)xb[b] != c);
}

// hop 2: mark every c_ok end of an arc b -> c that extends a binding
__global__ void k_und_hop2(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                           int64_t n, Bits c, const uint32_t* __restrict__ B1, const uint32_t* __restrict__ B2,
                           const uint32_t* __restrict__ xb, uint32_t* __restrict__ C) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        if (s < 0 || s >= n || t < 0 || t >= n) continue;
        // check, then set: most ends are reached many times, and a set bit needs no atomic
        if (ok(c, t) && !bit_at(C, t) && extends(B1, B2, xb, s, t)) atomicOr(&C[t >> 5], 1u << (t & 31));
        if (s != t && ok(c, s) && !bit_at(C, s) && extends(B1, B2, xb, t, s)) atomicOr(&C[s >> 5], 1u << (s & 31));
    }
}

// 1 hop: the distinct ends (or starts) of the a_ok -> b_ok arcs
__global__ void k_und_mark1(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                            int64_t n, Bits a, Bits b, int mark_start, uint32_t* __restrict__ M) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        if (s < 0 || s >= n || t < 0 || t >= n) continue;
        if (ok(a, s) && ok(b, t)) {  // check, then set (hub ends are marked by many arcs)
            const int64_t x = mark_start ? s : t;
            if (!bit_at(M, x)) atomicOr(&M[x >> 5], 1u << (x & 31));
        }
        if (s != t && ok(a, t) && ok(b, s)) {
            const int64_t x = mark_start ? t : s;
            if (!bit_at(M, x)) atomicOr(&M[x >> 5], 1u << (x & 31));
        }
    }
}

Bits bits_of(const capsmi_bitmap* b) { return Bits{P<uint32_t>(b->words), b->full ? 1 : 0}; }

}  // namespace

int64_t undirected_count(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                         int nt, int hops, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c,
                         int kind, uint32_t* marks) {
    REQUIRE(hops == 1 || hops == 2, CAPSMI_ERR_INTERNAL, "undirected hops");
    REQUIRE(a->lo == b->lo && a->hi == b->hi && (!c || (c->lo == b->lo && c->hi == b->hi)), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "undirected patterns: the node bitmaps must share one id domain");
    const int64_t lo = b->lo, n = b->hi - b->lo;
    REQUIRE(n > 0 && n <= (int64_t(1) << 31), CAPSMI_ERR_UNSUPPORTED, "undirected patterns: domain of 1 .. 2^31 ids");
    hipStream_t st = s->stream;
    const int64_t nw = (n + 31) / 32;
    Buf acc = dev_alloc(4 * sizeof(unsigned long long), s);
    HIP_CHECK(hipMemsetAsync(P<void>(acc), 0, 4 * sizeof(unsigned long long), st));
    if (hops == 1 && kind == 0) {  // count(*): the arcs
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_und_deg, dim3(grid_for(ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, n,
                                   bits_of(a), bits_of(b), bits_of(b), (uint32_t*)nullptr, (uint32_t*)nullptr,
                                   P<unsigned long long>(acc));
        HIP_CHECK(hipGetLastError());
        unsigned long long h[4];
        HIP_CHECK(hipMemcpyAsync(h, P<void>(acc), sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        return (int64_t)h[1];
    }
    if (hops == 1) {  // count(DISTINCT end | start)
        Buf own;
        uint32_t* M = marks;
        if (!M) {
            own = dev_alloc(sizeof(uint32_t) * nw, s);
            M = P<uint32_t>(own);
        }
        HIP_CHECK(hipMemsetAsync(M, 0, sizeof(uint32_t) * nw, st));
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_und_mark1, dim3(grid_for(ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, n,
                                   bits_of(a), bits_of(b), kind == 2 ? 1 : 0, M);
        HIP_CHECK(hipGetLastError());
        return marks ? 0 : words_popcount(s, M, 0, nw);
    }
    // (config CAPSMI_COUNT=atomic: the per-relationship atomic degrees below, the form above 2^26 ids)
    if (kind == 0 && n <= (int64_t(1) << 26) && !s->cfg.count_atomic) {
        // 2-hop count(*): the two-sided record partition of the directed count(*) with both arcs of every
        // relationship (k_count.hip k_rec_part<true>), walks in LDS, no per-relationship global atomics
        return two_hop_count_rec(s, srcs, dsts, ms, nt, a, b, c, true);
    }
    if (kind == 0) {  // 2-hop count(*), atomic degrees (domains above 2^26 ids)
        KernelTimer kt(s, "und_count");
        Buf inU = dev_alloc(sizeof(uint32_t) * n, s), outU = dev_alloc(sizeof(uint32_t) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(inU), 0, sizeof(uint32_t) * n, st));
        HIP_CHECK(hipMemsetAsync(P<void>(outU), 0, sizeof(uint32_t) * n, st));
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_und_deg, dim3(grid_for(ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, n,
                                   bits_of(a), bits_of(b), bits_of(c), P<uint32_t>(inU), P<uint32_t>(outU),
                                   P<unsigned long long>(acc));
        hipLaunchKernelGGL(k_und_product, dim3(grid_for(n)), dim3(256), 0, st, P<uint32_t>(inU), P<uint32_t>(outU), n,
                           P<unsigned long long>(acc));
        HIP_CHECK(hipGetLastError());
        unsigned long long h[4];
        HIP_CHECK(hipMemcpyAsync(h, P<void>(acc), sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        return (int64_t)(h[2] - h[0]);
    }
    // 2-hop count(DISTINCT end); distinct start is the same walk from the other end (the arcs are symmetric)
    const capsmi_bitmap* A = kind == 2 ? c : a;
    const capsmi_bitmap* Cc = kind == 2 ? a : c;
    // (config CAPSMI_UND=stream: the per-arc streaming form below, the form above 2^26 ids)
    if (undirected_distinct_part_ok(n) && !s->cfg.und_stream)
        return undirected_distinct_part(s, srcs, dsts, ms, nt, A, b, Cc, marks);  // the 2-D cell layout
    KernelTimer kt(s, "und_distinct");
    // B1, B2, C: three bitmaps in one buffer (one fill); x(b) needs no clearing (read only where B1 says
    // an arc stored it)
    Buf bm = dev_alloc(sizeof(uint32_t) * 3 * nw, s), xb = dev_alloc(sizeof(uint32_t) * n, s);
    HIP_CHECK(hipMemsetAsync(P<void>(bm), 0, sizeof(uint32_t) * 3 * nw, st));
    uint32_t *B1 = P<uint32_t>(bm), *B2 = B1 + nw, *C = B2 + nw;
    if (marks) {  // the caller's end bitmap (a rank's partial marks, ORed over the ranks by the caller)
        C = marks;
        HIP_CHECK(hipMemsetAsync(C, 0, sizeof(uint32_t) * nw, st));
    }
    for (int i = 0; i < nt; ++i)
        if (ms[i] > 0)
            hipLaunchKernelGGL(k_und_hop1, dim3(grid_for(ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, n,
                               bits_of(A), bits_of(b), B1, B2, P<uint32_t>(xb));
    for (int i = 0; i < nt; ++i)
        if (ms[i] > 0)
            hipLaunchKernelGGL(k_und_hop2, dim3(grid_for(ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, n,
                               bits_of(Cc), B1, B2, P<uint32_t>(xb), C);
    HIP_CHECK(hipGetLastError());
    return marks ? 0 : words_popcount(s, C, 0, nw);
}

}  // namespace capsmi
