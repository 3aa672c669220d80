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
// Here the relationships are grouped twice by the chunked partition of k_part.hip, in slices of
// 2^15 ids (a slice's 32-bit counters are 128 KiB of LDS):
//   pass 1, by target slice: a block counts inA(t) of its slice segment in LDS and stores the
//           slice's counts once (added atomically only where a slice is split between blocks);
//   pass 2, by source slice: each relationship b -> y with c_ok(y) adds inA(b), read from the
//           block's LDS copy of the slice's inA (128 KiB, staged once per slice segment).
// (Pass 2 over the relationships in table order, gathering inA(source) from HBM instead of a second
// partition, measured 19.6 ms against 8.4 + 5.8 ms at C3.)
#include "part_common.h"

namespace capsmi {
namespace cnt {

constexpr int kBits = 15;
constexpr int kIds = 1 << kBits;
constexpr int kBlock = 1024;
constexpr int kGroup = 2;  // chunks in flight per block (walk_chunks; 4 spills at 1024 lanes)

__device__ __forceinline__ bool bit(const part::BitV& v, uint32_t x) { return v.full || part::gbit(v.w, x); }

__device__ __forceinline__ void block_add(unsigned long long v, unsigned long long* out) {
    __shared__ unsigned long long red;
    if (threadIdx.x == 0) red = 0;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&red, v);
    __syncthreads();
    if (threadIdx.x == 0 && red) atomicAdd(out, red);
}

// target partition: pair = (source, target) relative to the domain
__global__ void __launch_bounds__(kBlock) k_cnt_in(part::ChunkWalk cw, part::BitV a, part::BitV b, part::BitV c,
                                                   int64_t n, uint32_t* __restrict__ inA,
                                                   unsigned long long* __restrict__ loops) {
    extern __shared__ uint32_t cin[];
    for (int i = threadIdx.x; i < kIds; i += kBlock) cin[i] = 0;
    __syncthreads();
    unsigned long long nl = 0;
    part::walk_chunks<kBlock, kGroup>(
        cw,
        [&](uint2 p, int) {
            const uint32_t s = p.x, t = p.y;
            if (bit(a, s)) {
                atomicAdd(&cin[t & (kIds - 1)], 1u);
                if (s == t && bit(b, s) && bit(c, s)) ++nl;
            }
        },
        [&](int j) {
            const bool own = part::owns_slice(cw, j);  // else the slice's other blocks add to it too
            for (int i = threadIdx.x; i < kIds; i += kBlock) {
                const uint32_t v = cin[i];
                const int64_t x = ((int64_t)j << kBits) + i;
                if (x < n) {
                    const uint32_t keep = bit(b, (uint32_t)x) ? v : 0u;
                    if (own) inA[x] = keep;
                    else if (keep) atomicAdd(&inA[x], keep);
                }
                cin[i] = 0;
            }
        });
    block_add(nl, loops);
}

// source partition: pair = (target, source); the slice's inA staged in LDS at each slice start
__global__ void __launch_bounds__(kBlock) k_cnt_out(part::ChunkWalk cw, part::BitV c, int64_t n,
                                                    const uint32_t* __restrict__ inA, unsigned long long* __restrict__ sum) {
    extern __shared__ uint32_t sin[];
    unsigned long long acc = 0;
    part::walk_chunks<kBlock, kGroup>(
        cw,
        [&](uint2 p, int) {
            if (bit(c, p.x)) acc += sin[p.y & (kIds - 1)];
        },
        [&](int) {},
        [&](int j) {
            const int64_t base = (int64_t)j << kBits;
            for (int i = threadIdx.x; i < kIds; i += kBlock) sin[i] = base + i < n ? inA[base + i] : 0u;
        });
    block_add(acc, sum);
}

}  // namespace cnt

// count(*) of the 2-hop chain over relationship tables (srcs[i], dsts[i], ms[i]); the three node
// bitmaps share one id domain of at most 2^26 ids (<= 2048 slices).  Returns the count.
int64_t two_hop_count_part(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                           int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok) {
    using namespace cnt;
    const int64_t lo = b_ok->lo, n = b_ok->hi - b_ok->lo;
    const part::BitV a{P<uint32_t>(a_ok->words), a_ok->full ? 1 : 0}, b{P<uint32_t>(b_ok->words), b_ok->full ? 1 : 0},
        c{P<uint32_t>(c_ok->words), c_ok->full ? 1 : 0};
    hipStream_t st = s->stream;
    part::Layout L{};
    L.lo = lo;
    L.hi = lo + n;
    L.tbits = kBits;
    L.nt = (int)((n + kIds - 1) / kIds);
    L.ns = 1;
    L.sbits = 31;
    L.ncells = L.nt;
    REQUIRE(L.nt >= 1 && L.nt <= part::kMaxTSlices, CAPSMI_ERR_INTERNAL, "count(*) partition: domain too large");
    Buf inA = dev_alloc(sizeof(uint32_t) * (size_t)n, s);
    Buf acc = dev_alloc(2 * sizeof(unsigned long long), s);  // loops, sum
    HIP_CHECK(hipMemsetAsync(P<void>(inA), 0, sizeof(uint32_t) * (size_t)n, st));
    HIP_CHECK(hipMemsetAsync(P<void>(acc), 0, 2 * sizeof(unsigned long long), st));
    const size_t lds = sizeof(uint32_t) * kIds;
    for (const void* f : {reinterpret_cast<const void*>(k_cnt_in), reinterpret_cast<const void*>(k_cnt_out)})
        HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int64_t mtot = 0;
    for (int i = 0; i < nt; ++i) mtot += ms[i] > 0 ? ms[i] : 0;
    {
        ChunkPart cp;
        {
            KernelTimer kt(s, "count_part_in");
            chunk_partition(s, srcs, dsts, ms, nt, false, L, s->num_cus, cp);
        }
        const part::ChunkWalk cw{P<uint2>(cp.pool), P<unsigned long long>(cp.meta), cp.order, cp.jst, cp.segbase, cp.ja,
                                 L.nt};
        KernelTimer kt(s, "count_in", (double)mtot * 8 + (double)n * 4);
        hipLaunchKernelGGL(k_cnt_in, dim3((unsigned)cp.g2), dim3(kBlock), lds, st, cw, a, b, c, n, P<uint32_t>(inA),
                           P<unsigned long long>(acc));
        HIP_CHECK(hipGetLastError());
    }
    {
        ChunkPart cp;
        {
            KernelTimer kt(s, "count_part_out");
            chunk_partition(s, srcs, dsts, ms, nt, true, L, s->num_cus, cp);
        }
        const part::ChunkWalk cw{P<uint2>(cp.pool), P<unsigned long long>(cp.meta), cp.order, cp.jst, cp.segbase, cp.ja,
                                 L.nt};
        KernelTimer kt(s, "count_out", (double)mtot * 8 + (double)n * 4);
        hipLaunchKernelGGL(k_cnt_out, dim3((unsigned)cp.g2), dim3(kBlock), lds, st, cw, c, n, P<uint32_t>(inA),
                           P<unsigned long long>(acc) + 1);
        HIP_CHECK(hipGetLastError());
    }
    unsigned long long h[2];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(acc), sizeof(h), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return (int64_t)(h[1] - h[0]);
}

}  // namespace capsmi
