// k_grouped.hip -- the 2-hop chain grouped by its start node (C3's grouped form):
//   MATCH (a)-[r1]->(b)-[r2]->(c) WHERE a_ok(a) AND b_ok(b) AND c_ok(c)   [r1 <> r2]
//   RETURN id(a), count(*)   |   RETURN id(a), count(DISTINCT c)
// The relational plan joins four times and aggregates (RelationalPlanner.scala:113-137,
// SparkTable.scala:121-188); here nothing per binding is materialised for count(*), and only one
// 8-byte (a, c) key per binding for count(DISTINCT c).
//
// r1 = r2 only when r1 is a self-loop at b = a walked twice, so with outC(b) = #{b -> y : c_ok(y)}:
//   count(*)(a) = sum over r1 = (a -> b), a_ok(a), b_ok(b) of outC(b) - [r1 is a loop and c_ok(b)].
// count(DISTINCT c)(a): the relationships b -> y with b_ok(b), c_ok(y) are grouped by b (a stable radix
// sort, so each list keeps relationship order); every r1 emits the key (a << 31 | c) of each r2 of
// out(b) other than itself (a wave per r1, coalesced stores); the keys are sorted, equal keys
// collapse, and the distinct keys of one a are counted.  The keys need 8 bytes per binding: the
// route checks the binding count (the count(*) pass) against the device memory first.
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
__device__ __forceinline__ bool ok(const Bits& b, int64_t x) { return b.full || ((b.w[x >> 5] >> (x & 31)) & 1u); }
Bits bits_of(const capsmi_bitmap* b) { return Bits{P<uint32_t>(b->words), b->full ? 1 : 0}; }

constexpr uint64_t kNone = uint64_t(1) << 62;  // sort key of a relationship outside the hop-2 lists

// hop-2 lists: key = b for relationships b -> y with b_ok(b), c_ok(y), else kNone; value = y; outC(b)
__global__ void k_g_lists(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                          int64_t n, Bits b, Bits c, uint64_t* __restrict__ key, int64_t* __restrict__ val,
                          unsigned long long* __restrict__ outc) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        const bool keep = s >= 0 && s < n && t >= 0 && t < n && ok(b, s) && ok(c, t);
        key[e] = keep ? (uint64_t)s : kNone;
        val[e] = t;
        if (keep) atomicAdd(&outc[s], 1ull);
    }
}

// per r1 = (a -> b): the bindings it starts (count(*)), added to a; and its count for the key expansion
__global__ void k_g_count(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                          int64_t n, Bits a, Bits b, Bits c, const unsigned long long* __restrict__ outc,
                          unsigned long long* __restrict__ per_a, int64_t* __restrict__ per_r1) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        int64_t k = 0;
        if (s >= 0 && s < n && t >= 0 && t < n && ok(a, s) && ok(b, t))
            k = (int64_t)outc[t] - ((s == t && ok(c, t)) ? 1 : 0);
        if (per_r1) per_r1[e] = k;
        if (per_a && k > 0) atomicAdd(&per_a[s], (unsigned long long)k);
    }
}

// keys of the bindings: a wave per r1 (grid-stride over r1 in waves); r1 = row e of the list input,
// list row numbers are the input row numbers of the same (single) relationship array
__global__ void k_g_keys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                         const int64_t* __restrict__ per_r1, const int64_t* __restrict__ start,
                         const int64_t* __restrict__ off, const int64_t* __restrict__ lval,
                         const int64_t* __restrict__ lrow, uint64_t* __restrict__ keys) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t e = wave; e < m; e += nwaves) {
        const int64_t k = per_r1[e];
        if (k <= 0) continue;
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        const int64_t b0 = off[t], b1 = off[t + 1];
        uint64_t* out = keys + start[e];
        // r1 is in out(t) when it is a loop kept in the lists: find its list position (rows in order)
        int64_t skip = -1;
        if (k < b1 - b0) {
            int64_t l = b0, h = b1;
            while (l < h) {
                const int64_t mid = (l + h) >> 1;
                if (lrow[mid] < e) l = mid + 1;
                else h = mid;
            }
            skip = l;
        }
        for (int64_t j = b0 + lane, w = lane; j < b1; j += 64, w += 64) {
            if (j == skip) continue;
            const int64_t pos = (skip >= 0 && j > skip) ? w - 1 : w;
            out[pos] = ((uint64_t)s << 31) | (uint64_t)lval[j];
        }
    }
}

__global__ void k_g_first(const uint64_t* __restrict__ keys, int64_t n, int shift, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = (i == 0 || (keys[i] >> shift) != (keys[i - 1] >> shift)) ? 1 : 0;
}

__global__ void k_g_runs(const int64_t* __restrict__ starts, int64_t g, int64_t total, const uint64_t* __restrict__ keys,
                         const int64_t* __restrict__ key_idx, int64_t* __restrict__ ids, int64_t* __restrict__ cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i + 1 < g ? starts[i + 1] : total;
        cnt[i] = e - starts[i];
        ids[i] = (int64_t)(keys[key_idx[starts[i]]] >> 31);
    }
}

__global__ void k_g_nonzero(const unsigned long long* __restrict__ v, int64_t n, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = v[i] ? 1 : 0;
}

}  // namespace

// rows (relative id of a, value) of the grouped 2-hop; distinct = count(DISTINCT c), else count(*).
// Returns false (nothing produced) when the count(DISTINCT c) keys would not fit `key_budget` bytes.
bool grouped_two_hop(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                     int nt, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c, bool distinct,
                     int64_t key_budget, Buf& out_ids, Buf& out_vals, int64_t* rows) {
    REQUIRE(a->lo == b->lo && a->hi == b->hi && c->lo == b->lo && c->hi == b->hi, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "grouped 2-hop: the node bitmaps must share one id domain");
    const int64_t lo = b->lo, n = b->hi - b->lo;
    REQUIRE(n > 0 && n <= (int64_t(1) << 31), CAPSMI_ERR_UNSUPPORTED, "grouped 2-hop: domain of 1 .. 2^31 ids");
    hipStream_t st = s->stream;
    // one relationship array (the union of the tables), so that row numbers identify relationships
    int64_t m = 0;
    for (int i = 0; i < nt; ++i) m += ms[i] > 0 ? ms[i] : 0;
    Buf S = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s), T = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s);
    {
        int64_t at = 0;
        for (int i = 0; i < nt; ++i) {
            if (ms[i] <= 0) continue;
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(S) + at, srcs[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(T) + at, dsts[i], sizeof(int64_t) * ms[i], hipMemcpyDeviceToDevice, st));
            at += ms[i];
        }
    }
    Buf outc = dev_alloc(sizeof(unsigned long long) * n, s);
    HIP_CHECK(hipMemsetAsync(P<void>(outc), 0, sizeof(unsigned long long) * n, st));
    Buf lkey = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s), lval = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s);
    if (m) hipLaunchKernelGGL(k_g_lists, dim3(grid_for(m)), dim3(256), 0, st, P<int64_t>(S), P<int64_t>(T), m, lo, n,
                              bits_of(b), bits_of(c), P<uint64_t>(lkey), P<int64_t>(lval), P<unsigned long long>(outc));
    HIP_CHECK(hipGetLastError());
    if (!distinct) {
        Buf per_a = dev_alloc(sizeof(unsigned long long) * n, s);
        HIP_CHECK(hipMemsetAsync(P<void>(per_a), 0, sizeof(unsigned long long) * n, st));
        if (m) hipLaunchKernelGGL(k_g_count, dim3(grid_for(m)), dim3(256), 0, st, P<int64_t>(S), P<int64_t>(T), m, lo, n,
                                  bits_of(a), bits_of(b), bits_of(c), P<unsigned long long>(outc),
                                  P<unsigned long long>(per_a), (int64_t*)nullptr);
        Buf f = dev_alloc(n, s);
        hipLaunchKernelGGL(k_g_nonzero, dim3(grid_for(n)), dim3(256), 0, st, P<unsigned long long>(per_a), n, P<uint8_t>(f));
        HIP_CHECK(hipGetLastError());
        Buf idx;
        const int64_t g = flags_to_indices(s, P<uint8_t>(f), n, idx);
        out_ids = idx;
        out_vals = dev_alloc(sizeof(int64_t) * (g > 0 ? g : 1), s);
        gather_col(reinterpret_cast<const int64_t*>(P<unsigned long long>(per_a)), nullptr, P<int64_t>(idx), g,
                   P<int64_t>(out_vals), nullptr, st);
        *rows = g;
        return true;
    }
    // bindings per r1 and their key offsets
    Buf per_r1 = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s), start = dev_alloc(sizeof(int64_t) * (m + 1), s);
    if (m) hipLaunchKernelGGL(k_g_count, dim3(grid_for(m)), dim3(256), 0, st, P<int64_t>(S), P<int64_t>(T), m, lo, n,
                              bits_of(a), bits_of(b), bits_of(c), P<unsigned long long>(outc),
                              (unsigned long long*)nullptr, P<int64_t>(per_r1));
    HIP_CHECK(hipGetLastError());
    exclusive_scan_i64(P<int64_t>(per_r1), P<int64_t>(start), m, s);
    const int64_t total = read_scalar(s, P<int64_t>(start) + m);
    if (total * (int64_t)sizeof(uint64_t) * 2 > key_budget) return false;  // keys + the sort's second buffer
    // the lists: relationships grouped by b, rows in order (stable sort); CSR offsets from outC
    Buf lrow = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s);
    iota_i64(P<int64_t>(lrow), 0, m, st);
    {
        std::vector<int> shifts;
        for (int sh = 0; sh < 32; sh += 8) shifts.push_back(sh);
        shifts.push_back(56);  // kNone's bit 62 lands in this digit
        Buf key2 = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
        HIP_CHECK(hipMemcpyAsync(P<void>(key2), P<void>(lkey), sizeof(uint64_t) * m, hipMemcpyDeviceToDevice, st));
        radix_sort_digits(s, P<uint64_t>(lkey), P<int64_t>(lrow), m, shifts);       // rows by b
        radix_sort_digits(s, P<uint64_t>(key2), P<int64_t>(lval), m, shifts);       // targets by b (same order)
    }
    Buf off = dev_alloc(sizeof(int64_t) * (n + 1), s);
    exclusive_scan_i64(reinterpret_cast<const int64_t*>(P<unsigned long long>(outc)), P<int64_t>(off), n, s);
    Buf keys = dev_alloc(sizeof(uint64_t) * (total > 0 ? total : 1), s);
    if (m) hipLaunchKernelGGL(k_g_keys, dim3(grid_for(m * 64 > (int64_t(1) << 24) ? (int64_t(1) << 24) : m * 64)),
                              dim3(256), 0, st, P<int64_t>(S), P<int64_t>(T), m, lo, P<int64_t>(per_r1),
                              P<int64_t>(start), P<int64_t>(off), P<int64_t>(lval), P<int64_t>(lrow), P<uint64_t>(keys));
    HIP_CHECK(hipGetLastError());
    {
        std::vector<int> shifts;
        for (int sh = 0; sh < 64; sh += 8) shifts.push_back(sh);
        radix_sort_digits(s, P<uint64_t>(keys), nullptr, total, shifts);
    }
    // distinct keys, then runs of one a among them
    Buf f = dev_alloc(total > 0 ? total : 1, s), didx, gidx;
    if (total) hipLaunchKernelGGL(k_g_first, dim3(grid_for(total)), dim3(256), 0, st, P<uint64_t>(keys), total, 0,
                                  P<uint8_t>(f));
    const int64_t d = flags_to_indices(s, P<uint8_t>(f), total, didx);
    Buf dkeys = dev_alloc(sizeof(uint64_t) * (d > 0 ? d : 1), s), f2 = dev_alloc(d > 0 ? d : 1, s);
    gather_col(reinterpret_cast<const int64_t*>(P<uint64_t>(keys)), nullptr, P<int64_t>(didx), d,
               reinterpret_cast<int64_t*>(P<uint64_t>(dkeys)), nullptr, st);
    if (d) hipLaunchKernelGGL(k_g_first, dim3(grid_for(d)), dim3(256), 0, st, P<uint64_t>(dkeys), d, 31, P<uint8_t>(f2));
    const int64_t g = flags_to_indices(s, P<uint8_t>(f2), d, gidx);
    Buf iota = dev_alloc(sizeof(int64_t) * (d > 0 ? d : 1), s);
    iota_i64(P<int64_t>(iota), 0, d, st);
    out_ids = dev_alloc(sizeof(int64_t) * (g > 0 ? g : 1), s);
    out_vals = dev_alloc(sizeof(int64_t) * (g > 0 ? g : 1), s);
    if (g) hipLaunchKernelGGL(k_g_runs, dim3(grid_for(g)), dim3(256), 0, st, P<int64_t>(gidx), g, d, P<uint64_t>(dkeys),
                              P<int64_t>(iota), P<int64_t>(out_ids), P<int64_t>(out_vals));
    HIP_CHECK(hipGetLastError());
    *rows = g;
    return true;
}

}  // namespace capsmi
