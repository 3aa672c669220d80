// k_varlen.hip -- fused BoundedVarLengthExpand + grouped count (C5), never materialising paths.
//
//   MATCH (a)-[r*lower..upper]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), count(*)   (1 <= lower <= upper <= 3)
//
// CAPS plans this as `upper` chained joins with an isomorphism filter per hop and a union over the
// lengths (VarLengthExpandPlanner.scala:83-136, 146-171, 247-260): one row per edge-distinct path.
// Per start node a the number of such paths has a closed form in per-node degree sums
// (derivation in DESIGN.md; checked against path enumeration in oracle/rmat.c):
//   od(v)  = #{r: v -> w, b_ok(w)}          s(v) = #self-loops at v
//   W(v)   = sum_{r: v -> w} od(w)          m(v,u) = #rels v -> u
//   len 1: od(a)
//   len 2: sum_{r: a->b} od(b) - s(a) b_ok(a)
//   len 3: sum_{r: a->b} [W(b) - (m(b,a) + s(b)) b_ok(b)] - s(a) (od(a) - 2 b_ok(a))
// Four streaming passes over the relationship table plus one hash probe per relationship for m(b,a).
#include "capsmi_impl.h"

namespace capsmi {
namespace varlen {

struct Dom {
    const uint32_t* a;
    const uint32_t* b;
    int64_t lo, hi;
    int a_full, b_full;
};

__device__ __forceinline__ bool in_dom(const Dom& d, int64_t v) { return v >= d.lo && v < d.hi; }
__device__ __forceinline__ bool bok(const Dom& d, int64_t v) {
    if (!in_dom(d, v)) return false;
    if (d.b_full) return true;
    const uint64_t x = (uint64_t)(v - d.lo);
    return (d.b[x >> 5] >> (x & 31)) & 1u;
}
__device__ __forceinline__ bool aok(const Dom& d, int64_t v) {
    if (!in_dom(d, v)) return false;
    if (d.a_full) return true;
    const uint64_t x = (uint64_t)(v - d.lo);
    return (d.a[x >> 5] >> (x & 31)) & 1u;
}

// pass 1: od(v), s(v)
__global__ void k_deg(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                      unsigned long long* __restrict__ od, unsigned long long* __restrict__ s) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[e], v = dst[e];
        if (!in_dom(d, u)) continue;
        if (bok(d, v)) atomicAdd(&od[u - d.lo], 1ULL);
        if (u == v) atomicAdd(&s[u - d.lo], 1ULL);
    }
}

// pass 2: W(v) = sum_{r: v -> w} od(w)
__global__ void k_w(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                    const unsigned long long* __restrict__ od, unsigned long long* __restrict__ W) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[e], v = dst[e];
        if (!in_dom(d, u) || !in_dom(d, v)) continue;
        const unsigned long long x = od[v - d.lo];
        if (x) atomicAdd(&W[u - d.lo], x);
    }
}

// pass 3: per relationship a -> b: T2(a) += od(b); T3(a) += W(b) - (m(b,a) + s(b)) b_ok(b)
__global__ void k_t(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, Dom d,
                    const unsigned long long* __restrict__ od, const unsigned long long* __restrict__ s,
                    const unsigned long long* __restrict__ W, const int64_t* __restrict__ rev_slot,
                    const int64_t* __restrict__ slot_count, int need3, unsigned long long* __restrict__ T2,
                    unsigned long long* __restrict__ T3) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = src[e], b = dst[e];
        if (!in_dom(d, a) || !in_dom(d, b) || !aok(d, a)) continue;
        const int64_t bi = b - d.lo;
        atomicAdd(&T2[a - d.lo], od[bi]);
        if (need3) {
            int64_t t3 = (int64_t)W[bi];
            if (bok(d, b)) {
                const int64_t rs = rev_slot[e];
                const int64_t mba = rs >= 0 ? slot_count[rs] : 0;
                t3 -= mba + (int64_t)s[bi];
            }
            atomicAdd(&T3[a - d.lo], (unsigned long long)t3);  // two's complement sum
        }
    }
}

// pass 4: per node, the count over lengths lower..upper; flags rows with count > 0
__global__ void k_final(int64_t n, Dom d, int lower, int upper, const unsigned long long* __restrict__ od,
                        const unsigned long long* __restrict__ s, const unsigned long long* __restrict__ T2,
                        const unsigned long long* __restrict__ T3, int64_t* __restrict__ cnt, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = d.lo + i;
        int64_t total = 0;
        if (aok(d, a)) {
            const int64_t o = (int64_t)od[i], sl = (int64_t)s[i], ba = bok(d, a) ? 1 : 0;
            const int64_t c1 = o;
            const int64_t c2 = (int64_t)T2[i] - sl * ba;
            const int64_t c3 = (int64_t)T3[i] - sl * (o - 2 * ba);
            if (lower <= 1 && upper >= 1) total += c1;
            if (lower <= 2 && upper >= 2) total += c2;
            if (lower <= 3 && upper >= 3) total += c3;
        }
        cnt[i] = total;
        f[i] = total > 0 ? 1 : 0;
    }
}

inline int grid(const capsmi_session* s, int64_t n) {
    int64_t g = (n + 255) / 256;
    const int64_t cap = (int64_t)s->num_cus * 16;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace varlen

// rows (a, count) of the fused var-length grouped count; returns the table's row count
int64_t var_length_count(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                         int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, int lower, int upper,
                         Buf& out_ids, Buf& out_cnt) {
    using namespace varlen;
    hipStream_t st = s->stream;
    const int64_t n = b_ok->hi - b_ok->lo;
    Dom d{P<uint32_t>(a_ok->words), P<uint32_t>(b_ok->words), b_ok->lo, b_ok->hi, a_ok->full ? 1 : 0,
          b_ok->full ? 1 : 0};
    const size_t nb = sizeof(uint64_t) * (n > 0 ? n : 1);
    Buf od = dev_alloc(nb, st), sl = dev_alloc(nb, st), W = dev_alloc(nb, st), T2 = dev_alloc(nb, st),
        T3 = dev_alloc(nb, st);
    for (Buf* b : {&od, &sl, &W, &T2, &T3}) HIP_CHECK(hipMemsetAsync(P<void>(*b), 0, nb, st));
    const bool need3 = upper >= 3;
    {
        KernelTimer kt(s, "varlen_deg");
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_deg, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(sl));
    }
    if (need3) {
        KernelTimer kt(s, "varlen_w");
        for (int i = 0; i < nt; ++i)
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_w, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(W));
    }
    // m(b, a): multiplicity of the reverse relationship, from a hash table over (source, target) of all
    // relationship tables (concatenated key columns)
    Buf rev, counts;
    HashTable ht;
    int64_t mtot = 0;
    for (int i = 0; i < nt; ++i) mtot += ms[i];
    if (need3 && mtot > 0) {
        Buf cs = dev_alloc(sizeof(int64_t) * mtot, st), cd = dev_alloc(sizeof(int64_t) * mtot, st);
        int64_t off = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] <= 0) continue;
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(cs) + off, srcs[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(cd) + off, dsts[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            off += ms[i];
        }
        KeyCols fwd, bwd;
        for (int k = 0; k < kMaxKeys; ++k) { fwd.data[k] = bwd.data[k] = nullptr; fwd.valid[k] = bwd.valid[k] = nullptr; }
        fwd.n = bwd.n = 2;
        fwd.data[0] = P<int64_t>(cs);
        fwd.data[1] = P<int64_t>(cd);
        bwd.data[0] = P<int64_t>(cd);
        bwd.data[1] = P<int64_t>(cs);
        Buf sor;
        KernelTimer kt(s, "varlen_rev");
        hash_build(s, fwd, mtot, false, ht, sor);
        hash_probe(s, bwd, fwd, mtot, ht, rev);
        counts = ht.slot_count;
    }
    {
        KernelTimer kt(s, "varlen_t");
        int64_t off = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] > 0)
                hipLaunchKernelGGL(k_t, dim3(grid(s, ms[i])), dim3(256), 0, st, srcs[i], dsts[i], ms[i], d,
                                   P<unsigned long long>(od), P<unsigned long long>(sl), P<unsigned long long>(W),
                                   need3 ? P<int64_t>(rev) + off : nullptr, need3 ? P<int64_t>(counts) : nullptr,
                                   need3 ? 1 : 0, P<unsigned long long>(T2), P<unsigned long long>(T3));
            off += ms[i];
        }
    }
    Buf cnt = dev_alloc(nb, st), flags = dev_alloc(n > 0 ? n : 1, st);
    hipLaunchKernelGGL(k_final, dim3(grid(s, n)), dim3(256), 0, st, n, d, lower, upper, P<unsigned long long>(od),
                       P<unsigned long long>(sl), P<unsigned long long>(T2), P<unsigned long long>(T3),
                       P<int64_t>(cnt), P<uint8_t>(flags));
    HIP_CHECK(hipGetLastError());
    Buf idx;
    const int64_t rows = flags_to_indices(s, P<uint8_t>(flags), n, idx);
    out_ids = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), st);
    out_cnt = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), st);
    // ids = lo + idx; counts = cnt[idx]
    gather_col(P<int64_t>(cnt), nullptr, P<int64_t>(idx), rows, P<int64_t>(out_cnt), nullptr, st);
    if (rows > 0) {
        HIP_CHECK(hipMemcpyAsync(P<void>(out_ids), P<void>(idx), sizeof(int64_t) * rows, hipMemcpyDeviceToDevice, st));
        add_i64(P<int64_t>(out_ids), d.lo, rows, st);
    }
    return rows;
}

}  // namespace capsmi
