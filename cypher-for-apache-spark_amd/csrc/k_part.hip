// k_part.hip -- radix-partitioned relationship layout and LDS-resident 2-hop kernels.
//
// The 2-hop count(DISTINCT c) touches two id-indexed bitmaps per relationship: the frontier of
// the middle node (indexed by source) and the mark of the end node (indexed by target).  Over
// 2^26 ids each is 8 MiB, twice an XCD's L2, so in ingest order both accesses are random L2/MALL
// traffic.  Partitioning removes both:
//   - target slices of 2^kSliceBits ids: a slice's bitmap (64 KiB) lives in LDS while a
//     workgroup streams that slice's relationships, so marks are LDS atomics;
//   - source super-slices, one per XCD (8): workgroups on XCD x only see sources in super-slice
//     x, so the source bitmap they read is 1/8 of the whole (1 MiB) and stays in that XCD's L2.
//     Blocks are dealt round-robin over XCDs (MI355X_MICROARCH.md, dispatch): block b runs on the
//     XCD of b % 8, so bucket (x, j) is given to blocks with b % 8 == x.  A different placement
//     changes only speed, never the result.
// Bucket b = x * nslices + j holds packed (source - lo, target - lo) uint32 pairs.
#include "capsmi_impl.h"

namespace capsmi {

namespace part {

constexpr int kSliceBits = 19;                   // 2^19 ids per target slice = 64 KiB of LDS bitmap
constexpr int kSliceWords = 1 << (kSliceBits - 5);
constexpr int kXcds = 8;
constexpr int kPBlock = 256;
constexpr int kPItems = 16;                      // rels per thread per partition tile
constexpr int kHBlock = 1024;

using Layout = PartLayout;

__device__ __forceinline__ int bucket_of(const Layout& L, uint64_t s, uint64_t t) {
    return (int)(s >> L.sx_shift) * L.nslices + (int)(t >> kSliceBits);
}

// pass 1: bucket sizes (rels with an endpoint outside [lo, hi) can never match a node scan
// over that domain and are dropped here -- an inner join drops them the same way)
__global__ void __launch_bounds__(kPBlock) k_part_hist(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                       int64_t m, Layout L, unsigned int* __restrict__ counts) {
    extern __shared__ unsigned int h[];
    for (int i = threadIdx.x; i < L.nbuckets; i += kPBlock) h[i] = 0;
    __syncthreads();
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const int64_t stride = (int64_t)gridDim.x * kPBlock;
    for (int64_t e = (int64_t)blockIdx.x * kPBlock + threadIdx.x; e < m; e += stride) {
        const uint64_t s = (uint64_t)(src[e] - L.lo), t = (uint64_t)(dst[e] - L.lo);
        if (s < range && t < range) atomicAdd(&h[bucket_of(L, s, t)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < L.nbuckets; i += kPBlock)
        if (h[i]) atomicAdd(&counts[i], h[i]);
}

// pass 2: scatter packed pairs; each tile reserves a run per bucket with one global atomic
__global__ void __launch_bounds__(kPBlock) k_part_scatter(const int64_t* __restrict__ src,
                                                          const int64_t* __restrict__ dst, int64_t m, Layout L,
                                                          unsigned long long* __restrict__ cursor,
                                                          uint2* __restrict__ out) {
    extern __shared__ unsigned long long sm[];
    unsigned int* cnt = reinterpret_cast<unsigned int*>(sm + L.nbuckets);  // after the bases
    unsigned long long* base = sm;
    const uint64_t range = (uint64_t)(L.hi - L.lo);
    const int64_t tile = (int64_t)kPBlock * kPItems;
    for (int64_t t0 = (int64_t)blockIdx.x * tile; t0 < m; t0 += (int64_t)gridDim.x * tile) {
        for (int i = threadIdx.x; i < L.nbuckets; i += kPBlock) cnt[i] = 0;
        __syncthreads();
        uint32_t sv[kPItems], tv[kPItems];
        int bk[kPItems];
#pragma unroll
        for (int k = 0; k < kPItems; ++k) {
            const int64_t e = t0 + (int64_t)k * kPBlock + threadIdx.x;
            bk[k] = -1;
            if (e < m) {
                const uint64_t s = (uint64_t)(src[e] - L.lo), t = (uint64_t)(dst[e] - L.lo);
                if (s < range && t < range) {
                    sv[k] = (uint32_t)s;
                    tv[k] = (uint32_t)t;
                    bk[k] = bucket_of(L, s, t);
                    atomicAdd(&cnt[bk[k]], 1u);
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < L.nbuckets; i += kPBlock) {
            const unsigned int c = cnt[i];
            base[i] = c ? atomicAdd(&cursor[i], (unsigned long long)c) : 0ULL;
            cnt[i] = 0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPItems; ++k) {
            if (bk[k] >= 0) {
                const unsigned int r = atomicAdd(&cnt[bk[k]], 1u);
                out[base[bk[k]] + r] = make_uint2(sv[k], tv[k]);
            }
        }
        __syncthreads();
    }
}

struct BitV {
    const uint32_t* w;  // words over [lo, hi) -- same domain as the layout
    int full;
};

__device__ __forceinline__ bool bv(const BitV& b, uint32_t x) {
    return b.full || ((b.w[x >> 5] >> (x & 31)) & 1u);
}

__device__ __forceinline__ void lds_set(uint32_t* lds, uint32_t x) {
    const uint32_t bit = 1u << (x & 31);
    uint32_t* p = &lds[x >> 5];
    if (!(*p & bit)) atomicOr(p, bit);
}

// OR the block's LDS slice into the global words of slice j (only non-zero words)
__device__ __forceinline__ void flush_slice(const uint32_t* lds, uint32_t* g, int j, int64_t gwords) {
    const int64_t w0 = (int64_t)j * kSliceWords;
    for (int i = threadIdx.x; i < kSliceWords; i += kHBlock) {
        const uint32_t v = lds[i];
        if (v && w0 + i < gwords) atomicOr(&g[w0 + i], v);
    }
}

// hop 1 over one bucket share: M(t) for a_ok(s), b_ok(t), s != t (LDS); self-loops -> S1/S2 (global)
template <bool A_FULL, bool B_FULL>
__global__ void __launch_bounds__(kHBlock) k_hop1_part(const uint2* __restrict__ pairs,
                                                       const int64_t* __restrict__ boff, Layout L, int splits,
                                                       BitV a, BitV b, uint32_t* __restrict__ M,
                                                       uint32_t* __restrict__ S1, uint32_t* __restrict__ S2,
                                                       int64_t gwords) {
    __shared__ uint32_t lds[kSliceWords];
    const int x = blockIdx.x % kXcds;
    const int rest = blockIdx.x / kXcds;
    const int j = rest % L.nslices;
    const int sp = rest / L.nslices;
    const int bucket = x * L.nslices + j;
    const int64_t b0 = boff[bucket], b1 = boff[bucket + 1];
    const int64_t len = b1 - b0;
    if (len == 0) return;  // block-uniform
    for (int i = threadIdx.x; i < kSliceWords; i += kHBlock) lds[i] = 0;
    __syncthreads();
    const int64_t s0 = b0 + len * sp / splits, s1 = b0 + len * (sp + 1) / splits;
    const uint32_t slice_base = (uint32_t)j << kSliceBits;
    for (int64_t e = s0 + threadIdx.x; e < s1; e += kHBlock) {
        const uint2 p = pairs[e];
        if (!(A_FULL || bv(a, p.x))) continue;
        if (!(B_FULL || bv(b, p.y))) continue;
        if (p.x != p.y) {
            lds_set(lds, p.y - slice_base);
        } else {  // rare: self-loops
            const uint32_t bit = 1u << (p.y & 31);
            const uint32_t old = atomicOr(&S1[p.y >> 5], bit);
            if (old & bit) atomicOr(&S2[p.y >> 5], bit);
        }
    }
    __syncthreads();
    flush_slice(lds, M, j, gwords);
}

// hop 2 over one bucket share: C(t) if c_ok(t) and (s != t ? X1(s) : X2(s))
template <bool C_FULL>
__global__ void __launch_bounds__(kHBlock) k_hop2_part(const uint2* __restrict__ pairs,
                                                       const int64_t* __restrict__ boff, Layout L, int splits,
                                                       BitV c, const uint32_t* __restrict__ X1,
                                                       const uint32_t* __restrict__ X2, uint32_t* __restrict__ C,
                                                       int64_t gwords) {
    __shared__ uint32_t lds[kSliceWords];
    const int x = blockIdx.x % kXcds;
    const int rest = blockIdx.x / kXcds;
    const int j = rest % L.nslices;
    const int sp = rest / L.nslices;
    const int bucket = x * L.nslices + j;
    const int64_t b0 = boff[bucket], b1 = boff[bucket + 1];
    const int64_t len = b1 - b0;
    if (len == 0) return;
    for (int i = threadIdx.x; i < kSliceWords; i += kHBlock) lds[i] = 0;
    __syncthreads();
    const int64_t s0 = b0 + len * sp / splits, s1 = b0 + len * (sp + 1) / splits;
    const uint32_t slice_base = (uint32_t)j << kSliceBits;
    for (int64_t e = s0 + threadIdx.x; e < s1; e += kHBlock) {
        const uint2 p = pairs[e];
        if (!(C_FULL || bv(c, p.y))) continue;
        const uint32_t* X = p.x == p.y ? X2 : X1;
        if ((X[p.x >> 5] >> (p.x & 31)) & 1u) lds_set(lds, p.y - slice_base);
    }
    __syncthreads();
    flush_slice(lds, C, j, gwords);
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
    L.nslices = (int)((range + (uint64_t(1) << part::kSliceBits) - 1) >> part::kSliceBits);
    if (L.nslices < 1) L.nslices = 1;
    const int lg = part::ceil_log2(range > 1 ? range : 2);
    L.sx_shift = lg > 3 ? lg - 3 : 0;
    L.nbuckets = part::kXcds * L.nslices;
    return L;
}

void relpart_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                   int64_t lo, int64_t hi, RelPart& rp) {
    REQUIRE(hi > lo && (uint64_t)(hi - lo) <= (uint64_t(1) << 32), CAPSMI_ERR_UNSUPPORTED,
            "partitioned layout needs an id domain of at most 2^32 ids");
    hipStream_t st = s->stream;
    rp.L = make_layout(lo, hi);
    const int nb = rp.L.nbuckets;
    REQUIRE(nb <= 32768, CAPSMI_ERR_UNSUPPORTED, "too many partition buckets");
    Buf counts = dev_alloc(sizeof(unsigned int) * nb, st);
    HIP_CHECK(hipMemsetAsync(P<void>(counts), 0, sizeof(unsigned int) * nb, st));
    int64_t mtot = 0;
    for (int i = 0; i < nt; ++i) {
        mtot += ms[i];
        if (ms[i] <= 0) continue;
        int64_t g = (ms[i] + part::kPBlock * 8 - 1) / (part::kPBlock * 8);
        const int64_t cap = (int64_t)s->num_cus * 8;
        if (g > cap) g = cap;
        KernelTimer kt(s, "part_hist");
        hipLaunchKernelGGL(part::k_part_hist, dim3((unsigned)g), dim3(part::kPBlock), sizeof(unsigned int) * nb, st,
                           srcs[i], dsts[i], ms[i], rp.L, P<unsigned int>(counts));
    }
    // offsets (int64) from the uint32 counts
    Buf c64 = dev_alloc(sizeof(int64_t) * nb, st);
    {
        std::vector<unsigned int> hc(nb);
        HIP_CHECK(hipMemcpyAsync(hc.data(), P<void>(counts), sizeof(unsigned int) * nb, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        std::vector<int64_t> off(nb + 1, 0);
        for (int i = 0; i < nb; ++i) off[i + 1] = off[i] + hc[i];
        rp.kept = off[nb];
        rp.boff = dev_alloc(sizeof(int64_t) * (nb + 1), st);
        HIP_CHECK(hipMemcpyAsync(P<void>(rp.boff), off.data(), sizeof(int64_t) * (nb + 1), hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(P<void>(c64), off.data(), sizeof(int64_t) * nb, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    rp.pairs = dev_alloc(sizeof(uint2) * (rp.kept > 0 ? rp.kept : 1), st);
    const size_t lds = sizeof(unsigned long long) * nb + sizeof(unsigned int) * nb;
    REQUIRE(lds <= 160 * 1024, CAPSMI_ERR_UNSUPPORTED, "partition histogram exceeds LDS");
    for (int i = 0; i < nt; ++i) {
        if (ms[i] <= 0) continue;
        const int64_t tile = (int64_t)part::kPBlock * part::kPItems;
        int64_t g = (ms[i] + tile - 1) / tile;
        const int64_t cap = (int64_t)s->num_cus * 4;
        if (g > cap) g = cap;
        KernelTimer kt(s, "part_scatter");
        hipLaunchKernelGGL(part::k_part_scatter, dim3((unsigned)g), dim3(part::kPBlock), lds, st, srcs[i], dsts[i],
                           ms[i], rp.L, P<unsigned long long>(c64), P<uint2>(rp.pairs));
    }
    HIP_CHECK(hipGetLastError());
    (void)mtot;
}

static int hop_splits(const RelPart& rp, const capsmi_session* s) {
    // enough blocks to cover the chip several times over (2 blocks of 1024 threads per CU fit)
    const int64_t want = (int64_t)s->num_cus * 8;
    int sp = (int)((want + rp.L.nbuckets - 1) / rp.L.nbuckets);
    if (sp < 1) sp = 1;
    if (sp > 64) sp = 64;
    return sp;
}

void relpart_hop1(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* M,
                  uint32_t* S1, uint32_t* S2) {
    REQUIRE(a->lo == rp.L.lo && a->hi == rp.L.hi && b->lo == rp.L.lo && b->hi == rp.L.hi, CAPSMI_ERR_UNSUPPORTED,
            "partitioned 2-hop needs node scans over the layout's id domain");
    if (rp.kept == 0) return;
    const int sp = hop_splits(rp, s);
    const dim3 g((unsigned)(rp.L.nbuckets * sp)), blk(part::kHBlock);
    const part::BitV av{P<uint32_t>(a->words), a->full ? 1 : 0}, bv{P<uint32_t>(b->words), b->full ? 1 : 0};
    const int64_t gw = b->nwords;
    KernelTimer kt(s, "hop1");
    if (a->full && b->full)
        hipLaunchKernelGGL((part::k_hop1_part<true, true>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, av, bv, M, S1, S2, gw);
    else if (a->full)
        hipLaunchKernelGGL((part::k_hop1_part<true, false>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, av, bv, M, S1, S2, gw);
    else if (b->full)
        hipLaunchKernelGGL((part::k_hop1_part<false, true>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, av, bv, M, S1, S2, gw);
    else
        hipLaunchKernelGGL((part::k_hop1_part<false, false>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, av, bv, M, S1, S2, gw);
    HIP_CHECK(hipGetLastError());
}

void relpart_hop2(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* c, const uint32_t* X1, const uint32_t* X2,
                  uint32_t* C) {
    REQUIRE(c->lo == rp.L.lo && c->hi == rp.L.hi, CAPSMI_ERR_UNSUPPORTED,
            "partitioned 2-hop needs node scans over the layout's id domain");
    if (rp.kept == 0) return;
    const int sp = hop_splits(rp, s);
    const dim3 g((unsigned)(rp.L.nbuckets * sp)), blk(part::kHBlock);
    const part::BitV cv{P<uint32_t>(c->words), c->full ? 1 : 0};
    KernelTimer kt(s, "hop2");
    if (c->full)
        hipLaunchKernelGGL((part::k_hop2_part<true>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, cv, X1, X2, C, c->nwords);
    else
        hipLaunchKernelGGL((part::k_hop2_part<false>), g, blk, 0, s->stream, P<uint2>(rp.pairs), P<int64_t>(rp.boff), rp.L, sp, cv, X1, X2, C, c->nwords);
    HIP_CHECK(hipGetLastError());
}

}  // namespace capsmi
