// k_hash.hip -- hash tables for equi-joins, Distinct and Aggregate.
//
// Semantics (Spark, as used by DataFrameTable):
//  - join (SparkTable.scala:205-229): `===` never matches a null key;
//  - distinct / dropDuplicates / groupBy (SparkTable.scala:128-136, 231-235): nulls group together.
// One open-addressing table maps each DISTINCT key to a slot (representative row +
// row count); duplicates of a key never extend a probe chain, so skewed keys (R-MAT
// hubs) cost one atomic per row, not a quadratic probe walk.  The join build side is
// then grouped by slot (counting sort), and the probe side is expanded with a
// load-balanced search over the per-row match counts, so one hub row emitting 10^5
// matches is spread over 10^5 threads.
#include "capsmi_impl.h"

namespace capsmi {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ bool key_null(const KeyCols& k, int64_t r) {
    for (int c = 0; c < k.n; ++c)
        if (k.valid[c] && !k.valid[c][r]) return true;
    return false;
}

__device__ __forceinline__ uint64_t key_hash(const KeyCols& k, int64_t r) {
    uint64_t h = 0x9E3779B97F4A7C15ULL;
    for (int c = 0; c < k.n; ++c) {
        const bool nul = k.valid[c] && !k.valid[c][r];
        const uint64_t v = nul ? 0x6A09E667F3BCC909ULL : (uint64_t)k.data[c][r];
        h = mix64(h ^ (v + (nul ? 0x3C6EF372FE94F82BULL : 0) + (uint64_t)c * 0x9E3779B97F4A7C15ULL));
    }
    return h;
}

__device__ __forceinline__ bool key_eq(const KeyCols& a, int64_t ra, const KeyCols& b, int64_t rb) {
    for (int c = 0; c < a.n; ++c) {
        const bool na = a.valid[c] && !a.valid[c][ra];
        const bool nb = b.valid[c] && !b.valid[c][rb];
        if (na || nb) {
            if (na != nb) return false;
            continue;
        }
        if (a.data[c][ra] != b.data[c][rb]) return false;
    }
    return true;
}

__global__ void k_hash_build(KeyCols k, int64_t n, int skip_null, unsigned long long* slot_row,
                             unsigned long long* slot_count, int64_t cap_mask, int64_t* slot_of_row) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (skip_null && key_null(k, i)) {
            slot_of_row[i] = -1;
            continue;
        }
        int64_t pos = (int64_t)(key_hash(k, i) & (uint64_t)cap_mask);
        while (true) {
            unsigned long long cur = __hip_atomic_load(&slot_row[pos], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == ~0ULL) {
                const unsigned long long prev = atomicCAS(&slot_row[pos], ~0ULL, (unsigned long long)i);
                cur = prev == ~0ULL ? (unsigned long long)i : prev;
            }
            if ((int64_t)cur == i || key_eq(k, (int64_t)cur, k, i)) {
                slot_of_row[i] = pos;
                atomicAdd(&slot_count[pos], 1ULL);
                break;
            }
            pos = (pos + 1) & cap_mask;
        }
    }
}

__global__ void k_hash_probe(KeyCols probe, KeyCols build, int64_t n, const int64_t* __restrict__ slot_row,
                             int64_t cap_mask, int64_t* __restrict__ slot_of_probe) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t found = -1;
        if (!key_null(probe, i)) {
            int64_t pos = (int64_t)(key_hash(probe, i) & (uint64_t)cap_mask);
            while (true) {
                const int64_t cur = slot_row[pos];
                if (cur < 0) break;
                if (key_eq(build, cur, probe, i)) {
                    found = pos;
                    break;
                }
                pos = (pos + 1) & cap_mask;
            }
        }
        slot_of_probe[i] = found;
    }
}

__global__ void k_occupied(const int64_t* __restrict__ slot_row, int64_t cap, uint8_t* __restrict__ f) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
        f[i] = slot_row[i] >= 0 ? 1 : 0;
}

__global__ void k_slot_gid(const int64_t* __restrict__ slots, int64_t ng, const int64_t* __restrict__ slot_row,
                           int64_t* __restrict__ slot_gid, int64_t* __restrict__ rep) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = slots[g];
        slot_gid[s] = g;
        rep[g] = slot_row[s];
    }
}

__global__ void k_row_gid(const int64_t* __restrict__ slot_of_row, int64_t n, const int64_t* __restrict__ slot_gid,
                          int64_t* __restrict__ gid) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = slot_of_row[i];
        gid[i] = s >= 0 ? slot_gid[s] : -1;
    }
}

__global__ void k_scatter_rows(const int64_t* __restrict__ slot_of_row, int64_t n, unsigned long long* cursor,
                               int64_t* __restrict__ rows) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = slot_of_row[i];
        if (s < 0) continue;
        const unsigned long long p = atomicAdd(&cursor[s], 1ULL);
        rows[p] = i;
    }
}

__global__ void k_probe_counts(const int64_t* __restrict__ slot_of_probe, int64_t n,
                               const int64_t* __restrict__ slot_count, int outer, int64_t* __restrict__ cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = slot_of_probe[i];
        int64_t c = s >= 0 ? slot_count[s] : 0;
        if (outer && c == 0) c = 1;
        cnt[i] = c;
    }
}

// load-balanced expansion: output o belongs to probe row p = upper_bound(prefix, o) - 1
__global__ void k_join_expand(const int64_t* __restrict__ prefix, int64_t nprobe, int64_t total,
                              const int64_t* __restrict__ slot_of_probe, const int64_t* __restrict__ offsets,
                              const int64_t* __restrict__ rows, int64_t* __restrict__ out_l,
                              int64_t* __restrict__ out_r, uint8_t* __restrict__ matched) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = nprobe;  // find last p with prefix[p] <= o
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (prefix[mid] <= o) lo = mid; else hi = mid;
        }
        const int64_t p = lo;
        const int64_t k = o - prefix[p];
        const int64_t s = slot_of_probe[p];
        int64_t r = -1;
        if (s >= 0) {
            r = rows[offsets[s] + k];
            if (matched) matched[r] = 1;
        }
        out_l[o] = p;
        out_r[o] = r;
    }
}

__global__ void k_cross(int64_t nl, int64_t nr, int64_t* __restrict__ out_l, int64_t* __restrict__ out_r) {
    const int64_t total = nl * nr;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
        out_l[o] = o / nr;
        out_r[o] = o % nr;
    }
}

// ---- aggregates --------------------------------------------------------------
__global__ void k_agg_count(const int64_t* __restrict__ gid, const uint8_t* __restrict__ valid, int64_t n,
                            unsigned long long* out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = gid[i];
        if (g >= 0 && (!valid || valid[i])) atomicAdd(&out[g], 1ULL);
    }
}

__global__ void k_agg_sum_i64(const int64_t* __restrict__ gid, const int64_t* __restrict__ v,
                              const uint8_t* __restrict__ valid, int64_t n, unsigned long long* sum, uint8_t* seen) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = gid[i];
        if (g < 0 || (valid && !valid[i])) continue;
        atomicAdd(&sum[g], (unsigned long long)v[i]);
        seen[g] = 1;
    }
}

__global__ void k_agg_sum_f64(const int64_t* __restrict__ gid, const int64_t* __restrict__ v,
                              const uint8_t* __restrict__ valid, int64_t n, double* sum, uint8_t* seen) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = gid[i];
        if (g < 0 || (valid && !valid[i])) continue;
        atomicAdd(&sum[g], __longlong_as_double(v[i]));
        seen[g] = 1;
    }
}

// doubles are compared through an order-preserving integer image
__device__ __forceinline__ int64_t f64_key(int64_t bits) { return bits ^ ((bits >> 63) & 0x7FFFFFFFFFFFFFFFLL); }

__global__ void k_agg_minmax(const int64_t* __restrict__ gid, const int64_t* __restrict__ v,
                             const uint8_t* __restrict__ valid, int64_t n, int is_f64, int is_max, long long* out,
                             uint8_t* seen) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = gid[i];
        if (g < 0 || (valid && !valid[i])) continue;
        const long long x = is_f64 ? f64_key(v[i]) : v[i];
        if (is_max) atomicMax(&out[g], x); else atomicMin(&out[g], x);
        seen[g] = 1;
    }
}

__global__ void k_minmax_finish(int64_t* v, int64_t ng) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x)
        v[g] = f64_key(v[g]);  // the image is an involution
}

// avg(..).cast(cypherType) (SparkTable.scala:141-146): an integer input's average is cast back to Long
__global__ void k_avg_finish(const double* __restrict__ sum, const int64_t* __restrict__ cnt, int64_t ng,
                             int to_i64, int64_t* __restrict__ out, uint8_t* __restrict__ valid) {
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = cnt[g];
        const double a = c > 0 ? sum[g] / (double)c : 0.0;
        out[g] = to_i64 ? (int64_t)a : __double_as_longlong(a);
        valid[g] = c > 0 ? 1 : 0;
    }
}

inline int grid_for(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 8192) g = 8192;
    return (int)g;
}

}  // namespace

void hash_build(capsmi_session* s, const KeyCols& k, int64_t n, bool skip_null_keys, HashTable& ht,
                Buf& slot_of_row) {
    hipStream_t st = s->stream;
    int64_t cap = 64;
    while (cap < 2 * n) cap <<= 1;
    ht.cap = cap;
    ht.slot_row = dev_alloc(sizeof(int64_t) * cap, s);
    ht.slot_count = dev_alloc(sizeof(int64_t) * cap, s);
    fill_i64(P<int64_t>(ht.slot_row), -1, cap, st);
    HIP_CHECK(hipMemsetAsync(P<void>(ht.slot_count), 0, sizeof(int64_t) * cap, st));
    slot_of_row = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_hash_build, dim3(grid_for(n)), dim3(256), 0, st, k, n, skip_null_keys ? 1 : 0,
                           P<unsigned long long>(ht.slot_row), P<unsigned long long>(ht.slot_count), cap - 1,
                           P<int64_t>(slot_of_row));
    HIP_CHECK(hipGetLastError());
}

void hash_probe(capsmi_session* s, const KeyCols& probe, const KeyCols& build, int64_t n, const HashTable& ht,
                Buf& slot_of_probe) {
    hipStream_t st = s->stream;
    slot_of_probe = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_hash_probe, dim3(grid_for(n)), dim3(256), 0, st, probe, build, n,
                           P<int64_t>(ht.slot_row), ht.cap - 1, P<int64_t>(slot_of_probe));
    HIP_CHECK(hipGetLastError());
}

int64_t hash_group_ids(capsmi_session* s, const HashTable& ht, const Buf& slot_of_row, int64_t n, Buf& gid_of_row,
                       Buf& rep_row_of_gid) {
    hipStream_t st = s->stream;
    Buf occ = dev_alloc(ht.cap, s);
    hipLaunchKernelGGL(k_occupied, dim3(grid_for(ht.cap)), dim3(256), 0, st, P<int64_t>(ht.slot_row), ht.cap,
                       P<uint8_t>(occ));
    Buf slots;
    const int64_t ng = flags_to_indices(s, P<uint8_t>(occ), ht.cap, slots);
    Buf slot_gid = dev_alloc(sizeof(int64_t) * ht.cap, s);
    rep_row_of_gid = dev_alloc(sizeof(int64_t) * (ng > 0 ? ng : 1), s);
    if (ng > 0)
        hipLaunchKernelGGL(k_slot_gid, dim3(grid_for(ng)), dim3(256), 0, st, P<int64_t>(slots), ng,
                           P<int64_t>(ht.slot_row), P<int64_t>(slot_gid), P<int64_t>(rep_row_of_gid));
    gid_of_row = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_row_gid, dim3(grid_for(n)), dim3(256), 0, st, P<int64_t>(slot_of_row), n,
                           P<int64_t>(slot_gid), P<int64_t>(gid_of_row));
    HIP_CHECK(hipGetLastError());
    return ng;
}

void hash_group_rows(capsmi_session* s, const HashTable& ht, const Buf& slot_of_row, int64_t n, Buf& offsets,
                     Buf& rows) {
    hipStream_t st = s->stream;
    offsets = dev_alloc(sizeof(int64_t) * (ht.cap + 1), s);
    exclusive_scan_i64(P<int64_t>(ht.slot_count), P<int64_t>(offsets), ht.cap, s);
    Buf cursor = dev_alloc(sizeof(int64_t) * ht.cap, s);
    HIP_CHECK(hipMemcpyAsync(P<void>(cursor), P<void>(offsets), sizeof(int64_t) * ht.cap, hipMemcpyDeviceToDevice, st));
    rows = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_scatter_rows, dim3(grid_for(n)), dim3(256), 0, st, P<int64_t>(slot_of_row), n,
                           P<unsigned long long>(cursor), P<int64_t>(rows));
    HIP_CHECK(hipGetLastError());
}

int64_t join_expand(capsmi_session* s, const Buf& slot_of_probe, int64_t nprobe, const HashTable& ht,
                    const Buf& offsets, const Buf& rows, bool left_outer, Buf& out_l, Buf& out_r,
                    Buf* matched_build, int64_t nbuild) {
    hipStream_t st = s->stream;
    Buf cnt = dev_alloc(sizeof(int64_t) * (nprobe > 0 ? nprobe : 1), s);
    Buf prefix = dev_alloc(sizeof(int64_t) * (nprobe + 1), s);
    if (nprobe > 0)
        hipLaunchKernelGGL(k_probe_counts, dim3(grid_for(nprobe)), dim3(256), 0, st, P<int64_t>(slot_of_probe),
                           nprobe, P<int64_t>(ht.slot_count), left_outer ? 1 : 0, P<int64_t>(cnt));
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(prefix), nprobe, s);
    const int64_t total = read_scalar(s, P<int64_t>(prefix) + nprobe);
    out_l = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    out_r = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    uint8_t* matched = nullptr;
    if (matched_build) {
        *matched_build = dev_alloc(nbuild > 0 ? nbuild : 1, s);
        matched = P<uint8_t>(*matched_build);
        HIP_CHECK(hipMemsetAsync(matched, 0, nbuild > 0 ? nbuild : 1, st));
    }
    if (total > 0)
        hipLaunchKernelGGL(k_join_expand, dim3(grid_for(total)), dim3(256), 0, st, P<int64_t>(prefix), nprobe, total,
                           P<int64_t>(slot_of_probe), P<int64_t>(offsets), P<int64_t>(rows), P<int64_t>(out_l),
                           P<int64_t>(out_r), matched);
    HIP_CHECK(hipGetLastError());
    return total;
}

void cross_pairs(int64_t nl, int64_t nr, int64_t* out_l, int64_t* out_r, hipStream_t st) {
    const int64_t total = nl * nr;
    if (total <= 0) return;
    hipLaunchKernelGGL(k_cross, dim3(grid_for(total)), dim3(256), 0, st, nl, nr, out_l, out_r);
    HIP_CHECK(hipGetLastError());
}

void agg_count(const int64_t* gid, const uint8_t* valid, int64_t n, int64_t* out, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_agg_count, dim3(grid_for(n)), dim3(256), 0, st, gid, valid, n, (unsigned long long*)out);
    HIP_CHECK(hipGetLastError());
}

void agg_sum_i64(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, int64_t* sum, uint8_t* seen,
                 hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_agg_sum_i64, dim3(grid_for(n)), dim3(256), 0, st, gid, v, valid, n,
                       (unsigned long long*)sum, seen);
    HIP_CHECK(hipGetLastError());
}

void agg_sum_f64(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, double* sum, uint8_t* seen,
                 hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_agg_sum_f64, dim3(grid_for(n)), dim3(256), 0, st, gid, v, valid, n, sum, seen);
    HIP_CHECK(hipGetLastError());
}

void agg_minmax(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, int type, bool is_max,
                int64_t* out, uint8_t* seen, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_agg_minmax, dim3(grid_for(n)), dim3(256), 0, st, gid, v, valid, n,
                       type == CAPSMI_F64 ? 1 : 0, is_max ? 1 : 0, (long long*)out, seen);
    HIP_CHECK(hipGetLastError());
}

void minmax_finish(int64_t* v, int type, bool, int64_t ng, hipStream_t st) {
    if (type != CAPSMI_F64 || ng <= 0) return;
    hipLaunchKernelGGL(k_minmax_finish, dim3(grid_for(ng)), dim3(256), 0, st, v, ng);
    HIP_CHECK(hipGetLastError());
}

void avg_finish(const double* sum, const int64_t* cnt, int64_t ng, bool to_i64, int64_t* out, uint8_t* valid,
                hipStream_t st) {
    if (ng <= 0) return;
    hipLaunchKernelGGL(k_avg_finish, dim3(grid_for(ng)), dim3(256), 0, st, sum, cnt, ng, to_i64 ? 1 : 0, out, valid);
    HIP_CHECK(hipGetLastError());
}

}  // namespace capsmi
