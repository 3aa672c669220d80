// k_tri.hip -- fused cyclic triangle count (C4), ExpandInto closing the cycle.
//
//   MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) WHERE n_ok(a), n_ok(b), n_ok(c) RETURN count(*)
//
// CAPS plans two Expands and an ExpandInto on (source, target) = (c, a) (RelationalPlanner.scala:113-154)
// followed by the pairwise uniqueness filter; every binding is a row.  With m(x,y) the multiplicity of
// x->y and s(x) the number of self-loops at x, the rows split by how many of a, b, c coincide
// (derivation in DESIGN.md; checked against enumeration in oracle/rmat.c):
//   count = 3 * sum_{triangles {u,v,w}} [m(u,v)m(v,w)m(w,u) + m(u,w)m(w,v)m(v,u)]
//         + 3 * sum_{u != x} s(u) m(u,x) m(x,u)
//         + sum_u s(u)(s(u)-1)(s(u)-2)
// Triangles of the underlying simple undirected graph are listed once each by orienting every
// undirected edge from the lower (degree, id) end and intersecting sorted out-lists.  The two
// directed multiplicities of each undirected edge ride along with the oriented adjacency, so the
// intersection loop reads no other table.
#include "capsmi_impl.h"

namespace capsmi {
namespace tri {

constexpr uint64_t kNone = ~0ULL;

__global__ void k_pack(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                       int64_t hi, const uint32_t* __restrict__ okw, int full, uint64_t* __restrict__ key) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e], t = dst[e];
        bool ok = s >= lo && s < hi && t >= lo && t < hi;
        if (ok && !full) {
            const uint64_t xs = (uint64_t)(s - lo), xt = (uint64_t)(t - lo);
            ok = ((okw[xs >> 5] >> (xs & 31)) & 1u) && ((okw[xt >> 5] >> (xt & 31)) & 1u);
        }
        key[e] = ok ? (((uint64_t)(s - lo) << 32) | (uint64_t)(t - lo)) : kNone;
    }
}

// run heads of a sorted key array (valid keys only)
__global__ void k_heads(const uint64_t* __restrict__ k, int64_t n, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = (k[i] != kNone && (i == 0 || k[i] != k[i - 1])) ? 1 : 0;
}

// directed runs -> self-loop counts, and undirected records (key = min<<32|max, val = m(min,max)<<32 | m(max,min))
__global__ void k_dir_runs(const uint64_t* __restrict__ k, const int64_t* __restrict__ heads, int64_t nruns,
                           int64_t nvalid, uint32_t* __restrict__ sl, uint64_t* __restrict__ ukey,
                           int64_t* __restrict__ uval) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t h = heads[r], h2 = r + 1 < nruns ? heads[r + 1] : nvalid;
        const uint64_t c = (uint64_t)(h2 - h);
        const uint64_t key = k[h];
        const uint32_t s = (uint32_t)(key >> 32), t = (uint32_t)key;
        if (s == t) {
            sl[s] = (uint32_t)c;
            ukey[r] = kNone;
            uval[r] = 0;
        } else if (s < t) {
            ukey[r] = ((uint64_t)s << 32) | t;
            uval[r] = (int64_t)(c << 32);
        } else {
            ukey[r] = ((uint64_t)t << 32) | s;
            uval[r] = (int64_t)c;
        }
    }
}

// undirected runs (<= 2 records each) -> combined multiplicities, degrees
__global__ void k_und_runs(const uint64_t* __restrict__ uk, const int64_t* __restrict__ uv,
                           const int64_t* __restrict__ heads, int64_t nruns, int64_t nvalid,
                           uint64_t* __restrict__ ek, int64_t* __restrict__ ev, uint32_t* __restrict__ deg) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nruns; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t h = heads[r], h2 = r + 1 < nruns ? heads[r + 1] : nvalid;
        int64_t v = 0;
        for (int64_t i = h; i < h2; ++i) v += uv[i];
        ek[r] = uk[h];
        ev[r] = v;
        atomicAdd(&deg[(uint32_t)(uk[h] >> 32)], 1u);
        atomicAdd(&deg[(uint32_t)uk[h]], 1u);
    }
}

// orient each undirected edge from the lower (degree, id) end; payload = m(from,to)<<32 | m(to,from)
__global__ void k_orient(const uint64_t* __restrict__ ek, const int64_t* __restrict__ ev, int64_t ne,
                         const uint32_t* __restrict__ deg, uint64_t* __restrict__ ok_, int64_t* __restrict__ ov) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)(ek[i] >> 32), y = (uint32_t)ek[i];
        const uint64_t v = (uint64_t)ev[i];
        const uint32_t mxy = (uint32_t)(v >> 32), myx = (uint32_t)v;
        const bool x_first = deg[x] < deg[y] || (deg[x] == deg[y] && x < y);
        if (x_first) {
            ok_[i] = ((uint64_t)x << 32) | y;
            ov[i] = (int64_t)(((uint64_t)mxy << 32) | myx);
        } else {
            ok_[i] = ((uint64_t)y << 32) | x;
            ov[i] = (int64_t)(((uint64_t)myx << 32) | mxy);
        }
    }
}

// CSR offsets of the oriented (sorted) edges: off[v] = first edge with source >= v
__global__ void k_offsets(const uint64_t* __restrict__ ok_, int64_t ne, int64_t n, int64_t* __restrict__ off) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = ne;
        const uint64_t target = (uint64_t)v << 32;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (ok_[mid] < target) lo = mid + 1; else hi = mid;
        }
        off[v] = lo;
    }
}

// one thread per oriented edge (u -> v): intersect out(u) and out(v); weight of each triangle
__global__ void __launch_bounds__(256) k_triangles(const uint64_t* __restrict__ ok_, const int64_t* __restrict__ ov,
                                                   int64_t e_begin, int64_t e_end, const int64_t* __restrict__ off,
                                                   unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = e_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < e_end;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)(ok_[i] >> 32), v = (uint32_t)ok_[i];
        const uint64_t muv_p = (uint64_t)ov[i];
        const uint64_t m_uv = muv_p >> 32, m_vu = muv_p & 0xffffffffULL;
        int64_t a = off[u], a_end = off[u + 1], b = off[v], b_end = off[v + 1];
        // merge intersection of two sorted lists
        while (a < a_end && b < b_end) {
            const uint32_t wa = (uint32_t)ok_[a], wb = (uint32_t)ok_[b];
            if (wa < wb) { ++a; continue; }
            if (wb < wa) { ++b; continue; }
            const uint64_t pa = (uint64_t)ov[a], pb = (uint64_t)ov[b];
            const uint64_t m_uw = pa >> 32, m_wu = pa & 0xffffffffULL;
            const uint64_t m_vw = pb >> 32, m_wv = pb & 0xffffffffULL;
            acc += m_uv * m_vw * m_wu + m_uw * m_wv * m_vu;
            ++a;
            ++b;
        }
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

// pair and self terms
__global__ void k_pair_terms(const uint64_t* __restrict__ ek, const int64_t* __restrict__ ev, int64_t ne,
                             const uint32_t* __restrict__ sl, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)(ek[i] >> 32), y = (uint32_t)ek[i];
        const uint64_t v = (uint64_t)ev[i];
        acc += 3ULL * ((uint64_t)sl[x] + sl[y]) * (v >> 32) * (v & 0xffffffffULL);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

__global__ void k_self_terms(const uint32_t* __restrict__ sl, int64_t n, unsigned long long* __restrict__ out) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s = sl[i];
        if (s >= 3) acc += s * (s - 1) * (s - 2);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

inline int grid(const capsmi_session* s, int64_t n) {
    int64_t g = (n + 255) / 256;
    const int64_t cap = (int64_t)s->num_cus * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

inline int bits_for(uint64_t range) {
    int b = 1;
    while (b < 32 && (uint64_t(1) << b) < range) ++b;
    return b;
}

}  // namespace tri

void tri_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
               const capsmi_bitmap* n_ok, TriGraph& g) {
    using namespace tri;
    hipStream_t st = s->stream;
    const int64_t lo = n_ok->lo, hi = n_ok->hi, n = hi - lo;
    REQUIRE(n > 0 && (uint64_t)n <= (uint64_t(1) << 32), CAPSMI_ERR_UNSUPPORTED, "triangle count needs <= 2^32 ids");
    g.lo = lo;
    g.n = n;
    int64_t m = 0;
    for (int i = 0; i < nt; ++i) m += ms[i];
    const int bits = bits_for((uint64_t)n);
    Buf key = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), st), val = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), st);
    {
        KernelTimer kt(s, "tri_pack");
        int64_t off = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_pack, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], lo, hi,
                                   P<uint32_t>(n_ok->words), n_ok->full ? 1 : 0, P<uint64_t>(key) + off);
            off += ms[i];
        }
    }
    iota_i64(P<int64_t>(val), 0, m, st);
    radix_sort_pairs(s, P<uint64_t>(key), P<int64_t>(val), m, 0, 64);  // kNone (all ones) sorts last
    // directed runs
    Buf f = dev_alloc(m > 0 ? m : 1, st), heads;
    hipLaunchKernelGGL(k_heads, dim3(grid(s, m)), dim3(256), 0, st, P<uint64_t>(key), m, P<uint8_t>(f));
    const int64_t nruns = flags_to_indices(s, P<uint8_t>(f), m, heads);
    int64_t nvalid = 0;
    {
        // nvalid: binary search for the first kNone in the sorted keys (host-side bisection, O(log m) reads)
        int64_t a = 0, b = m;
        while (a < b) {
            const int64_t mid = (a + b) / 2;
            uint64_t kv;
            HIP_CHECK(hipMemcpyAsync(&kv, P<uint64_t>(key) + mid, 8, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            if (kv == kNone) b = mid; else a = mid + 1;
        }
        nvalid = a;
    }
    g.sl = dev_alloc(sizeof(uint32_t) * n, st);
    HIP_CHECK(hipMemsetAsync(P<void>(g.sl), 0, sizeof(uint32_t) * n, st));
    Buf uk = dev_alloc(sizeof(uint64_t) * (nruns > 0 ? nruns : 1), st), uv = dev_alloc(sizeof(int64_t) * (nruns > 0 ? nruns : 1), st);
    if (nruns > 0)
        hipLaunchKernelGGL(k_dir_runs, dim3(grid(s, nruns)), dim3(256), 0, st, P<uint64_t>(key), P<int64_t>(heads),
                           nruns, nvalid, P<uint32_t>(g.sl), P<uint64_t>(uk), P<int64_t>(uv));
    key.reset();
    val.reset();
    radix_sort_pairs(s, P<uint64_t>(uk), P<int64_t>(uv), nruns, 0, 64);
    Buf f2 = dev_alloc(nruns > 0 ? nruns : 1, st), heads2;
    hipLaunchKernelGGL(k_heads, dim3(grid(s, nruns)), dim3(256), 0, st, P<uint64_t>(uk), nruns, P<uint8_t>(f2));
    const int64_t ne = flags_to_indices(s, P<uint8_t>(f2), nruns, heads2);
    int64_t nuvalid = 0;
    {
        int64_t a = 0, b = nruns;
        while (a < b) {
            const int64_t mid = (a + b) / 2;
            uint64_t kv;
            HIP_CHECK(hipMemcpyAsync(&kv, P<uint64_t>(uk) + mid, 8, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            if (kv == kNone) b = mid; else a = mid + 1;
        }
        nuvalid = a;
    }
    g.ne = ne;
    g.ek = dev_alloc(sizeof(uint64_t) * (ne > 0 ? ne : 1), st);
    g.ev = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), st);
    Buf deg = dev_alloc(sizeof(uint32_t) * n, st);
    HIP_CHECK(hipMemsetAsync(P<void>(deg), 0, sizeof(uint32_t) * n, st));
    if (ne > 0)
        hipLaunchKernelGGL(k_und_runs, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(uk), P<int64_t>(uv),
                           P<int64_t>(heads2), ne, nuvalid, P<uint64_t>(g.ek), P<int64_t>(g.ev), P<uint32_t>(deg));
    g.ok = dev_alloc(sizeof(uint64_t) * (ne > 0 ? ne : 1), st);
    g.ov = dev_alloc(sizeof(int64_t) * (ne > 0 ? ne : 1), st);
    if (ne > 0)
        hipLaunchKernelGGL(k_orient, dim3(grid(s, ne)), dim3(256), 0, st, P<uint64_t>(g.ek), P<int64_t>(g.ev), ne,
                           P<uint32_t>(deg), P<uint64_t>(g.ok), P<int64_t>(g.ov));
    radix_sort_pairs(s, P<uint64_t>(g.ok), P<int64_t>(g.ov), ne, 0, 32 + bits);
    g.off = dev_alloc(sizeof(int64_t) * (n + 1), st);
    hipLaunchKernelGGL(k_offsets, dim3(grid(s, n + 1)), dim3(256), 0, st, P<uint64_t>(g.ok), ne, n, P<int64_t>(g.off));
    HIP_CHECK(hipGetLastError());
}

// count over oriented edges [e_begin, e_end) (+ pair/self terms when with_terms)
uint64_t tri_count(capsmi_session* s, const TriGraph& g, int64_t e_begin, int64_t e_end, bool with_terms) {
    using namespace tri;
    hipStream_t st = s->stream;
    Buf out = dev_alloc(24, st);
    HIP_CHECK(hipMemsetAsync(P<void>(out), 0, 24, st));
    if (e_end > e_begin) {
        KernelTimer kt(s, "triangles");
        hipLaunchKernelGGL(k_triangles, dim3(grid(s, e_end - e_begin)), dim3(256), 0, st, P<uint64_t>(g.ok),
                           P<int64_t>(g.ov), e_begin, e_end, P<int64_t>(g.off), P<unsigned long long>(out));
    }
    if (with_terms) {
        if (g.ne > 0)
            hipLaunchKernelGGL(k_pair_terms, dim3(grid(s, g.ne)), dim3(256), 0, st, P<uint64_t>(g.ek), P<int64_t>(g.ev),
                               g.ne, P<uint32_t>(g.sl), P<unsigned long long>(out) + 1);
        hipLaunchKernelGGL(k_self_terms, dim3(grid(s, g.n)), dim3(256), 0, st, P<uint32_t>(g.sl), g.n,
                           P<unsigned long long>(out) + 2);
    }
    HIP_CHECK(hipGetLastError());
    uint64_t h[3];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(out), 24, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    return 3 * h[0] + h[1] + h[2];
}

}  // namespace capsmi
