// k_und_part.hip -- undirected 2-hop count(DISTINCT end) over the 2-D cell layout (k_part.hip).
//
// RelationalPlanner lowers (a)-[r1]-(b)-[r2]-(c) to the union of outgoing and incoming branches per hop,
// the incoming ones over relationships with start <> end (okapi-relational/.../RelationalPlanner.scala:
// 126-136).  Viewed from a node that is a walk along arcs: relationship (s, t) is the arc s -> t and, when
// s != t, the arc t -> s.  The closed form: K(b) = the a_ok arcs into b, capped at 2, and for
// K = 1 the arc's other end x(b); an arc b -> c extends a binding iff K(b) = 2, or K(b) = 1 and c != x(b).
//
// The streaming form (k_undirected.hip) pays one random bitmap access per arc per hop.  Here the
// relationships are laid out once by 2-D cell (target slice j, source slice i) -- the directed C3 build --
// and both hops walk them grouped by the slice of the id the arc goes INTO, q: the cells (q, i) forwards
// (arcs s -> t, t in q) and the cells (j, q) backwards (arcs t -> s, s in q, s != t).  Every relationship is
// read twice per hop, sequentially, and the per-arc state lives in LDS:
//   hop 1: K1 (>= 1 arc) and K2 (>= 2) of slice q in LDS, x(b) stored by the arc that sets K1 locally;
//          flushed per slice with one atomicOr into the global K1 whose old value finds the ids another
//          workgroup also reached (they get K2), b_ok applied at the flush;
//   hop 2: the end marks C of slice q in LDS; every cell has one FROM slice (i forwards, j backwards),
//          whose K2 words are pulled into LDS for large cells; a middle with K2 = 0 reads K1 and x(b) from
//          memory (with a_ok covering the domain, K(b) = 1 means b has one relationship, whose reverse is
//          the only arc out of b).  c_ok applied at the flush.
// The "into" groups need square cells (source slices of 2^19 ids as the targets'): domains of at most
// 2^26 ids (128 x 128 cells); larger ones keep the streaming form.
#include <mutex>
#include <set>

#include "capsmi_impl.h"
#include "part_common.h"

namespace capsmi {

namespace undp {
using namespace part;

// virtual item v of the into-grouped walk: group q = v / (2 nt), k = v % (2 nt); k < nt: cell (q, k)
// forwards, else cell (k - nt, q) backwards.  Sizes of the items (cell sizes), scanned by the host
__global__ void k_und_vsizes(const int64_t* __restrict__ boff, int nt, int64_t* __restrict__ vs) {
    const int64_t nv = 2 * (int64_t)nt * nt;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (int64_t)gridDim.x * blockDim.x) {
        const int q = (int)(v / (2 * nt)), k = (int)(v % (2 * nt));
        const int c = k < nt ? q * nt + k : (k - nt) * nt + q;
        vs[v] = boff[c + 1] - boff[c];
    }
}

template <bool HOP2>
__global__ void __launch_bounds__(kBlock) k_und_2d(const uint2* __restrict__ pairs, const int64_t* __restrict__ boff,
                                                   const int64_t* __restrict__ voff, int nt, int64_t min_per, BitV a,
                                                   BitV tmask, uint32_t* __restrict__ K1, uint32_t* __restrict__ K2,
                                                   uint32_t* __restrict__ xb, uint32_t* __restrict__ C, int64_t gwords) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    // hop 1: l0 = K1, l1 = K2 of the into slice; hop 2: l0 = C of the into slice, l1 = K2 of the from slice
    uint32_t* l0 = lds;
    uint32_t* l1 = lds + kSliceWords;
    const int64_t nv = 2 * (int64_t)nt * nt;
    const int64_t total = voff[nv];
    int64_t per = (total + gridDim.x - 1) / gridDim.x;
    if (per < min_per) per = min_per;
    int64_t e0 = (int64_t)blockIdx.x * per;
    const int64_t e1 = min(e0 + per, total);
    if (e0 >= e1) return;  // block-uniform
    int64_t v = 0;
    {  // last item with voff[v] <= e0
        int64_t lo = 0, hi = nv;
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (voff[mid] <= e0) lo = mid; else hi = mid;
        }
        v = lo;
    }
    int cur_q = -1;
    auto flush = [&](int q) {
        const int64_t w0 = (int64_t)q * kSliceWords;
        for (int i = threadIdx.x; i < kSliceWords; i += kBlock) {
            const int64_t gw = w0 + i;
            if (gw >= gwords) break;
            const uint32_t m = tmask.full ? ~0u : tmask.w[gw];
            if (HOP2) {
                const uint32_t c = l0[i] & m;
                if (c) atomicOr(&C[gw], c);
            } else {
                const uint32_t k1 = l0[i] & m;
                uint32_t k2 = l1[i] & m;
                if (k1) k2 |= atomicOr(&K1[gw], k1) & k1;  // ids another workgroup reached too: >= 2 arcs
                if (k2) atomicOr(&K2[gw], k2);
            }
        }
    };
    while (e0 < e1) {
        while (voff[v + 1] <= e0) ++v;
        const int q = (int)(v / (2 * nt)), k = (int)(v % (2 * nt));
        const bool back = k >= nt;
        const int from = back ? k - nt : k;  // the slice of the arcs' start
        const int c = back ? from * nt + q : q * nt + k;
        const int64_t ce = min(e1, voff[v + 1]);
        if (q != cur_q) {
            if (cur_q >= 0) {
                __syncthreads();
                flush(cur_q);
            }
            __syncthreads();
            for (int i = threadIdx.x; i < kSliceWords; i += kBlock) l0[i] = 0;
            if (!HOP2)
                for (int i = threadIdx.x; i < kSliceWords; i += kBlock) l1[i] = 0;
            cur_q = q;
        }
        const bool pull = HOP2 && ce - e0 >= kLoadMin;
        if (pull) {
            const int64_t w0 = (int64_t)from * kSliceWords;
            for (int i = threadIdx.x; i < kSliceWords; i += kBlock) l1[i] = w0 + i < gwords ? K2[w0 + i] : 0u;
        }
        __syncthreads();
        const uint32_t qbase = (uint32_t)q << kSliceBits, fbase = (uint32_t)from << kSliceBits;
        auto visit = [&](const uint2 pr) {
            uint32_t into = pr.y, frm = pr.x;  // forwards: s -> t
            if (back) {                        // backwards: t -> s, never a self-loop
                if (pr.x == pr.y) return;
                into = pr.x;
                frm = pr.y;
            }
            const uint32_t x = into - qbase, w = x >> 5, bit = 1u << (x & 31);
            if (HOP2) {
                if (l0[w] & bit) return;  // check, then set: most ends are reached many times
                bool ext = pull ? gbit(l1, frm - fbase) : gbit(K2, frm);
                if (!ext && gbit(K1, frm)) ext = xb[frm] != into;
                if (ext) atomicOr(&l0[w], bit);
            } else {
                if (!a.full && !gbit(a.w, frm)) return;
                if (l1[w] & bit) return;  // hubs: settled by one LDS read
                if (atomicOr(&l0[w], bit) & bit) atomicOr(&l1[w], bit);
                else xb[into] = frm;  // the first arc into this id in this workgroup
            }
        };
        const int64_t p0 = boff[c] + (e0 - voff[v]), p1 = p0 + (ce - e0);
        for (int64_t cb = p0 & ~int64_t(1); cb < p1; cb += (int64_t)kBlock * kUnroll) {  // block-uniform, even
            uint2 p[kUnroll];
            load_pairs<kBlock, kUnroll>(pairs, cb, p);
            const int lo = (int)max(p0 - cb, (int64_t)0), hi = (int)min(p1 - cb, (int64_t)kBlock * kUnroll);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int e = item_off<kBlock>(u);
                if (e >= lo && e < hi) visit(p[u]);
            }
        }
        e0 = ce;
        ++v;
        __syncthreads();  // the next item may overwrite l1 / flush
    }
    __syncthreads();
    flush(cur_q);
}

}  // namespace undp

bool undirected_distinct_part_ok(int64_t n) { return n > 0 && n <= (int64_t(1) << 26); }

int64_t undirected_distinct_part(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts,
                                 const int64_t* ms, int nt, const capsmi_bitmap* a, const capsmi_bitmap* b,
                                 const capsmi_bitmap* c, uint32_t* marks) {
    using namespace part;
    const int64_t lo = b->lo, n = b->hi - b->lo, nw = b->nwords;
    REQUIRE(undirected_distinct_part_ok(n), CAPSMI_ERR_INTERNAL, "undirected layout: domain of at most 2^26 ids");
    hipStream_t st = s->stream;
    RelPart rp;
    relpart_build(s, srcs, dsts, ms, nt, lo, b->hi, rp, nullptr, /*unpacked=*/true);
    const Layout& L = rp.L;
    REQUIRE(L.ns == L.nt && L.sbits == kSliceBits && !L.packed, CAPSMI_ERR_INTERNAL, "undirected layout: square cells");
    const int64_t nv = 2 * (int64_t)L.nt * L.nt;
    Buf vb = dev_alloc(sizeof(int64_t) * (2 * nv + 1), s);
    int64_t *vs = P<int64_t>(vb), *voff = vs + nv;
    hipLaunchKernelGGL(undp::k_und_vsizes, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, P<int64_t>(rp.boff),
                       L.nt, vs);
    exclusive_scan_i64(vs, voff, nv, s);
    // K1, K2 and (unless the caller's) C in one buffer, one fill; x(b) needs none (read only where K1 is set
    // and K2 is not, i.e. where exactly one arc stored it)
    Buf kb = dev_alloc(sizeof(uint32_t) * 3 * (size_t)nw, s), xb = dev_alloc(sizeof(uint32_t) * (size_t)n, s);
    HIP_CHECK(hipMemsetAsync(P<void>(kb), 0, sizeof(uint32_t) * 3 * (size_t)nw, st));
    uint32_t *K1 = P<uint32_t>(kb), *K2 = K1 + nw, *C = K2 + nw;
    if (marks) {
        C = marks;
        HIP_CHECK(hipMemsetAsync(C, 0, sizeof(uint32_t) * (size_t)nw, st));
    }
    const size_t lds = sizeof(uint32_t) * 2 * kSliceWords;
    {  // the LDS attribute, once per device (one 128 KiB block per CU)
        static std::mutex mu;
        static std::set<int> done;
        std::lock_guard<std::mutex> g(mu);
        if (!done.count(s->device)) {
            HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(undp::k_und_2d<false>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(undp::k_und_2d<true>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            done.insert(s->device);
        }
    }
    const int64_t min_per = (int64_t)kBlock * kUnroll;
    int64_t blocks = (int64_t)s->num_cus * 4;
    blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, (2 * rp.rows + min_per - 1) / min_per));
    const BitV av{P<uint32_t>(a->words), a->full ? 1 : 0}, bv{P<uint32_t>(b->words), b->full ? 1 : 0},
        cv{P<uint32_t>(c->words), c->full ? 1 : 0};
    // algorithmic bytes per hop: every pair read twice (its row and its column walk), the hop's bitmaps
    const double hop_bytes = 16.0 * (double)rp.rows + 3.0 * 4.0 * (double)nw;
    {
        KernelTimer kt(s, "und_hop1", hop_bytes);
        hipLaunchKernelGGL(undp::k_und_2d<false>, dim3((unsigned)blocks), dim3(kBlock), lds, st, P<uint2>(rp.pairs),
                           P<int64_t>(rp.boff), voff, L.nt, min_per, av, bv, K1, K2, P<uint32_t>(xb), C, nw);
    }
    {
        KernelTimer kt(s, "und_hop2", hop_bytes);
        hipLaunchKernelGGL(undp::k_und_2d<true>, dim3((unsigned)blocks), dim3(kBlock), lds, st, P<uint2>(rp.pairs),
                           P<int64_t>(rp.boff), voff, L.nt, min_per, av, cv, K1, K2, P<uint32_t>(xb), C, nw);
    }
    HIP_CHECK(hipGetLastError());
    return marks ? 0 : words_popcount(s, C, 0, nw);
}

}  // namespace capsmi
