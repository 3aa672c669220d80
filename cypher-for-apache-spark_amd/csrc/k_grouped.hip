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
#include <algorithm>
#include <string>

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

// ---- count(DISTINCT c) per a without per-binding keys ---------------------------------------------
// The distinct hop-1 pairs (a, b) (a_ok, b_ok) and hop-2 pairs (b, y) (b_ok, c_ok) as sorted u64 keys
// (hi << 32 | lo), deduplicated: multi-edges collapse, and a's distinct ends are the union of the
// deduplicated out(b) over its deduplicated b's.  r1 <> r2 excludes only c = a reached through b = a by
// the same self-loop, so walking b = a skips c = a unless a carries two loops (loops(a) >= 2).  Each a's
// union is counted in LDS: an open-addressing set per wave (small a), per workgroup (medium), or a bitmap
// over 2^20-id ranges of c per workgroup (large a, the c range walked once per range).
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__global__ void k_gd_keys(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t lo,
                          int64_t n, Bits x, Bits y, uint64_t* __restrict__ key, unsigned int* __restrict__ loops) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e] - lo, t = dst[e] - lo;
        const bool in = s >= 0 && s < n && t >= 0 && t < n;
        key[e] = in && ok(x, s) && ok(y, t) ? ((uint64_t)s << 32 | (uint64_t)t) : ~0ULL;
        if (loops && in && s == t) atomicAdd(&loops[s], 1u);
    }
}

// first occurrence of each valid sorted key
__global__ void k_gd_first(const uint64_t* __restrict__ k, int64_t m, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = k[i] != ~0ULL && (i == 0 || k[i] != k[i - 1]);
}

// CSR offsets of the sorted distinct keys by their high word: off[v] = first key with hi >= v
__global__ void k_gd_off(const uint64_t* __restrict__ k, int64_t ne, int64_t n, int64_t* __restrict__ off) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v <= n; v += (int64_t)gridDim.x * blockDim.x) {
        int64_t l = 0, h = ne;
        const uint64_t target = (uint64_t)v << 32;
        while (l < h) {
            const int64_t mid = (l + h) >> 1;
            if (k[mid] < target) l = mid + 1; else h = mid;
        }
        off[v] = l;
    }
}

// per a: the hop-2 entries its walk reads (sum of |out2(b)| over its b's); one wave per a
__global__ void k_gd_work(const uint64_t* __restrict__ k1, const int64_t* __restrict__ off1,
                          const int64_t* __restrict__ off2, int64_t n, int64_t* __restrict__ w) {
    const int lane = threadIdx.x & 63;
    for (int64_t a = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; a < n;
         a += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        int64_t acc = 0;
        for (int64_t i = off1[a] + lane; i < off1[a + 1]; i += 64) {
            const int64_t b = (int64_t)(uint32_t)k1[i];
            acc += off2[b + 1] - off2[b];
        }
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
        if (lane == 0) w[a] = acc;
    }
}

// the flat walk of one a by one wave, over its b's in chunks of 64: f(c) for every c of every out2(b),
// with c = a from b = a dropped when a carries fewer than two loops
// per-wave LDS of the flat walk: the chunk's list starts (exclusive prefix), bases and b's
struct GdWave {
    uint32_t pre[64];
    uint32_t bv[64];
    int64_t base[64];
};

template <class F>
__device__ __forceinline__ void gd_walk(int64_t a, const uint64_t* __restrict__ k1, const int64_t* __restrict__ off1,
                                        const uint64_t* __restrict__ k2, const int64_t* __restrict__ off2,
                                        const unsigned int* __restrict__ loops, int first_chunk, int chunk_step,
                                        GdWave& L, F f) {
    const int lane = threadIdx.x & 63;
    const int64_t b0 = off1[a], nb = off1[a + 1] - b0;
    const bool drop_self = loops[a] < 2u;
    for (int64_t c0 = (int64_t)first_chunk * 64; c0 < nb; c0 += (int64_t)chunk_step * 64) {
        int64_t lb = 0, len = 0;
        uint32_t bb = 0xFFFFFFFFu;
        if (c0 + lane < nb) {
            bb = (uint32_t)k1[b0 + c0 + lane];
            lb = off2[bb];
            len = off2[bb + 1] - lb;
        }
        uint32_t x = (uint32_t)len;  // inclusive scan over the wave (all lanes active)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        L.pre[lane] = x - (uint32_t)len;
        L.bv[lane] = bb;
        L.base[lane] = lb;
        const uint32_t total = __shfl(x, 63, 64);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t q = lane; q < total; q += 64) {
            int l = 0, h = 63;  // last i with pre[i] <= q (empty lists share their successor's start)
            while (l < h) {
                const int mid = (l + h + 1) >> 1;
                if (L.pre[mid] <= q) l = mid; else h = mid - 1;
            }
            const uint32_t c = (uint32_t)k2[L.base[l] + (q - L.pre[l])];
            if (drop_self && (int64_t)L.bv[l] == a && (int64_t)c == a) continue;
            f(c);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

__device__ __forceinline__ uint32_t gd_slot(uint32_t c, int log2cap) { return (c * 0x9E3779B1u) >> (32 - log2cap); }

// insert c into an LDS set; 1 when it was not there
__device__ __forceinline__ int gd_insert(uint32_t* hk, int log2cap, uint32_t c) {
    const uint32_t mask = (1u << log2cap) - 1;
    uint32_t sl = gd_slot(c, log2cap);
    while (true) {
        const uint32_t prev = hk[sl];
        if (prev == c) return 0;
        if (prev == kEmpty) {
            const uint32_t got = atomicCAS(&hk[sl], kEmpty, c);
            if (got == kEmpty) return 1;
            if (got == c) return 0;
        }
        sl = (sl + 1) & mask;
    }
}

// small a (work <= SLOTS / 2): one wave per a, a private LDS set of SLOTS keys
template <int SLOTS>
__global__ void __launch_bounds__(256) k_gd_small(const int64_t* __restrict__ as, int64_t na,
                                                  const uint64_t* __restrict__ k1, const int64_t* __restrict__ off1,
                                                  const uint64_t* __restrict__ k2, const int64_t* __restrict__ off2,
                                                  const unsigned int* __restrict__ loops, int64_t* __restrict__ out) {
    __shared__ uint32_t hk[4][SLOTS];
    __shared__ GdWave pre[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int log2cap = 0;
    while ((1 << log2cap) < SLOTS) ++log2cap;
    for (int64_t q = (int64_t)blockIdx.x * 4 + wv; q < na; q += (int64_t)gridDim.x * 4) {
        const int64_t a = as[q];
        for (int i = lane; i < SLOTS; i += 64) hk[wv][i] = kEmpty;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int64_t cnt = 0;
        gd_walk(a, k1, off1, k2, off2, loops, 0, 1, pre[wv], [&](uint32_t c) { cnt += gd_insert(hk[wv], log2cap, c); });
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
        if (lane == 0) out[a] = cnt;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// large a: one 1024-lane workgroup per a, a bitmap of the c range [r * 2^20, (r + 1) * 2^20) in LDS per pass
constexpr int kGdRangeBits = 20;
__global__ void __launch_bounds__(1024) k_gd_large(const int64_t* __restrict__ as, int64_t na,
                                                   const uint64_t* __restrict__ k1, const int64_t* __restrict__ off1,
                                                   const uint64_t* __restrict__ k2, const int64_t* __restrict__ off2,
                                                   const unsigned int* __restrict__ loops, int64_t n,
                                                   int64_t* __restrict__ out) {
    extern __shared__ uint32_t bm[];  // 2^20 bits
    __shared__ GdWave pre[16];
    __shared__ unsigned long long tot;
    constexpr int kW = 1 << (kGdRangeBits - 5);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t nr = (n + (int64_t(1) << kGdRangeBits) - 1) >> kGdRangeBits;
    for (int64_t q = blockIdx.x; q < na; q += gridDim.x) {
        const int64_t a = as[q];
        if (threadIdx.x == 0) tot = 0;
        for (int64_t r = 0; r < nr; ++r) {
            for (int i = threadIdx.x; i < kW; i += 1024) bm[i] = 0;
            __syncthreads();
            const uint32_t rlo = (uint32_t)(r << kGdRangeBits);
            unsigned long long cnt = 0;
            gd_walk(a, k1, off1, k2, off2, loops, wv, 16, pre[wv], [&](uint32_t c) {
                const uint32_t x = c - rlo;
                if (x >> kGdRangeBits) return;  // another range
                const uint32_t bit = 1u << (x & 31);
                if (!(bm[x >> 5] & bit) && !(atomicOr(&bm[x >> 5], bit) & bit)) ++cnt;
            });
            for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
            if (lane == 0 && cnt) atomicAdd(&tot, cnt);
            __syncthreads();
        }
        if (threadIdx.x == 0) out[a] = (int64_t)tot;
        __syncthreads();
    }
}

__global__ void k_gd_class(const int64_t* __restrict__ w, int64_t n, int64_t small_max, uint8_t* __restrict__ fs,
                           uint8_t* __restrict__ fl) {
    for (int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; a < n; a += (int64_t)gridDim.x * blockDim.x) {
        fs[a] = w[a] > 0 && w[a] <= small_max;
        fl[a] = w[a] > small_max;
    }
}

__global__ void k_gd_nonzero(const int64_t* __restrict__ v, int64_t n, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = v[i] > 0;
}

}  // namespace

// sorted, deduplicated pair keys (x -> y with x_ok, y_ok) of the relationship array, and their CSR offsets
static int64_t gd_pairs(capsmi_session* s, const int64_t* S, const int64_t* T, int64_t m, int64_t lo, int64_t n,
                        const capsmi_bitmap* x, const capsmi_bitmap* y, unsigned int* loops, Buf& keys, Buf& off) {
    hipStream_t st = s->stream;
    Buf k = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
    if (m) hipLaunchKernelGGL(k_gd_keys, dim3(grid_for(m)), dim3(256), 0, st, S, T, m, lo, n, bits_of(x), bits_of(y),
                              P<uint64_t>(k), loops);
    HIP_CHECK(hipGetLastError());
    int bits = 1;
    while ((int64_t(1) << bits) < n) ++bits;
    std::vector<int> shifts;
    for (int sh = 0; sh < bits; sh += 8) shifts.push_back(sh);
    for (int sh = 32; sh < 32 + bits; sh += 8) shifts.push_back(sh);
    shifts.push_back(56);  // the invalid keys (all ones) sort last
    radix_sort_digits(s, P<uint64_t>(k), nullptr, m, shifts);
    Buf f = dev_alloc(m > 0 ? m : 1, s), idx;
    if (m) hipLaunchKernelGGL(k_gd_first, dim3(grid_for(m)), dim3(256), 0, st, P<uint64_t>(k), m, P<uint8_t>(f));
    const int64_t ne = flags_to_indices(s, P<uint8_t>(f), m, idx);
    keys = dev_alloc(sizeof(uint64_t) * (ne > 0 ? ne : 1), s);
    gather_col(reinterpret_cast<const int64_t*>(P<uint64_t>(k)), nullptr, P<int64_t>(idx), ne,
               reinterpret_cast<int64_t*>(P<uint64_t>(keys)), nullptr, st);
    off = dev_alloc(sizeof(int64_t) * (n + 1), s);
    hipLaunchKernelGGL(k_gd_off, dim3(grid_for(n + 1)), dim3(256), 0, st, P<uint64_t>(keys), ne, n, P<int64_t>(off));
    HIP_CHECK(hipGetLastError());
    return ne;
}

// count(DISTINCT c) per a by LDS sets over the deduplicated lists (above)
// Returns false (nothing produced, on every rank alike) when a distributed run's gathered hop-2 keys would
// not fit `key_budget` bytes.
static bool grouped_distinct_sets(capsmi_session* s, const int64_t* S, const int64_t* T, int64_t m, int64_t lo,
                                  int64_t n, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c,
                                  bool dist, int64_t key_budget, Buf& out_ids, Buf& out_vals, int64_t* rows) {
    hipStream_t st = s->stream;
    KernelTimer kt(s, "grouped_distinct");
    Buf loops = dev_alloc(sizeof(unsigned int) * n, s);
    HIP_CHECK(hipMemsetAsync(P<void>(loops), 0, sizeof(unsigned int) * n, st));
    Buf k1, off1, k2, off2;
    gd_pairs(s, S, T, m, lo, n, a, b, P<unsigned int>(loops), k1, off1);
    const int64_t ne2 = gd_pairs(s, S, T, m, lo, n, b, c, nullptr, k2, off2);
    if (dist) {
        // BY_SOURCE shards: this rank's deduplicated (b, y) keys are those of its owned b's, an id range that
        // grows with the rank, so every rank's keys concatenated in rank order are the whole sorted key set:
        // one all-gather, then the offsets over it (each rank walks the out2(b) of any b its a's reach)
        // (the whole key set on every rank: refused together above the key budget)
        int64_t tot = 0;
        k2 = gather_words(s, P<uint64_t>(k2), ne2, &tot, key_budget > 0 ? key_budget : 0);
        if (tot < 0) return false;
        hipLaunchKernelGGL(k_gd_off, dim3(grid_for(n + 1)), dim3(256), 0, st, P<uint64_t>(k2), tot, n, P<int64_t>(off2));
        HIP_CHECK(hipGetLastError());
    }
    Buf w = dev_alloc(sizeof(int64_t) * n, s), cnt = dev_alloc(sizeof(int64_t) * n, s);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(int64_t) * n, st));
    hipLaunchKernelGGL(k_gd_work, dim3(grid_for(n * 64, 256)), dim3(256), 0, st, P<uint64_t>(k1), P<int64_t>(off1),
                       P<int64_t>(off2), n, P<int64_t>(w));
    constexpr int kSmallSlots = 2048;
    Buf fs = dev_alloc(n, s), fl = dev_alloc(n, s), small, large;
    hipLaunchKernelGGL(k_gd_class, dim3(grid_for(n)), dim3(256), 0, st, P<int64_t>(w), n, (int64_t)kSmallSlots / 2,
                       P<uint8_t>(fs), P<uint8_t>(fl));
    HIP_CHECK(hipGetLastError());
    const int64_t ns = flags_to_indices(s, P<uint8_t>(fs), n, small);
    const int64_t nl = flags_to_indices(s, P<uint8_t>(fl), n, large);
    if (ns)
        hipLaunchKernelGGL(k_gd_small<kSmallSlots>, dim3((unsigned)std::min<int64_t>((ns + 3) / 4, 16 * (int64_t)s->num_cus)),
                           dim3(256), 0, st, P<int64_t>(small), ns, P<uint64_t>(k1), P<int64_t>(off1), P<uint64_t>(k2),
                           P<int64_t>(off2), P<unsigned int>(loops), P<int64_t>(cnt));
    if (nl) {
        const size_t lds = sizeof(uint32_t) << (kGdRangeBits - 5);
        lds_attr(reinterpret_cast<const void*>(k_gd_large), lds);
        hipLaunchKernelGGL(k_gd_large, dim3((unsigned)std::min<int64_t>(nl, 2 * (int64_t)s->num_cus)), dim3(1024), lds, st,
                           P<int64_t>(large), nl, P<uint64_t>(k1), P<int64_t>(off1), P<uint64_t>(k2), P<int64_t>(off2),
                           P<unsigned int>(loops), n, P<int64_t>(cnt));
    }
    HIP_CHECK(hipGetLastError());
    Buf f = dev_alloc(n, s), idx;
    hipLaunchKernelGGL(k_gd_nonzero, dim3(grid_for(n)), dim3(256), 0, st, P<int64_t>(cnt), n, P<uint8_t>(f));
    const int64_t g = flags_to_indices(s, P<uint8_t>(f), n, idx);
    out_ids = idx;
    out_vals = dev_alloc(sizeof(int64_t) * (g > 0 ? g : 1), s);
    gather_col(P<int64_t>(cnt), nullptr, P<int64_t>(idx), g, P<int64_t>(out_vals), nullptr, st);
    *rows = g;
    return true;
}

// rows (relative id of a, value) of the grouped 2-hop; distinct = count(DISTINCT c), else count(*).
// Returns false (nothing produced) when the count(DISTINCT c) keys would not fit `key_budget` bytes.
bool grouped_two_hop(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                     int nt, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c, bool distinct,
                     int64_t key_budget, Buf& out_ids, Buf& out_vals, int64_t* rows, const GroupedDist* dd) {
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
    if (dd && !distinct) {
        // BY_SOURCE shards: outC(b) is complete for the owned b's (their out-relationships are all here); one
        // all-gather of the owned slices gives every rank outC of every id
        REQUIRE(dd->span * dd->world == n, CAPSMI_ERR_INTERNAL, "grouped 2-hop: distributed domain geometry");
        Buf full = dev_alloc(sizeof(unsigned long long) * n, s);
        collective(s, CAPSMI_COLL_ALL_GATHER, P<unsigned long long>(outc) + dd->rank * dd->span, P<void>(full), dd->span,
                   CAPSMI_I64);
        outc = full;
    }
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
    // (config CAPSMI_GROUPED=keys: the per-binding key sort below, bounded by memory)
    if (dd || !s->cfg.grouped_keys)
        return grouped_distinct_sets(s, P<int64_t>(S), P<int64_t>(T), m, lo, n, a, b, c, dd != nullptr, key_budget,
                                     out_ids, out_vals, rows);
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
