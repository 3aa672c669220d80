// k_sort.hip -- stable LSD radix sort of (uint64 key, int64 value) pairs, 8 bits per pass.
//
// Used by ORDER BY (DataFrameTable.orderBy, SparkTable.scala:94-103) and by the
// Cache-analogue clustering of relationship tables (capsmi_cluster_by).
// Pass = (1) per-tile digit histogram in LDS, (2) digit-major exclusive scan of the
// [digit][tile] counts, (3) stable scatter: each tile is walked in 256-key rounds;
// the rank of a key among equal digits in its wave comes from 8 ballots (wave64),
// ranks across the 4 waves and earlier rounds from LDS counters.
#include "capsmi_impl.h"

namespace capsmi {

namespace {

constexpr int kBlock = 256;
constexpr int kRounds = 16;
constexpr int kTile = kBlock * kRounds;  // 4096 keys per tile

__global__ void __launch_bounds__(kBlock) k_hist(const uint64_t* __restrict__ keys, int64_t n, int shift,
                                                 int64_t ntiles, int64_t* __restrict__ hist) {
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile;
    for (int j = 0; j < kRounds; ++j) {
        const int64_t i = base + j * kBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255], 1u);
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

__global__ void __launch_bounds__(kBlock) k_scatter(const uint64_t* __restrict__ keys, const int64_t* __restrict__ vals,
                                                    int64_t n, int shift, int64_t ntiles,
                                                    const int64_t* __restrict__ offs, uint64_t* __restrict__ okeys,
                                                    int64_t* __restrict__ ovals) {
    __shared__ int64_t base_d[256];           // running output position per digit for this tile
    __shared__ unsigned int wcnt[4][256];     // per-wave digit counts of the current round
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    base_d[threadIdx.x] = offs[(int64_t)threadIdx.x * ntiles + blockIdx.x];
    const int64_t tbase = (int64_t)blockIdx.x * kTile;
    const unsigned long long lt_mask = (lane == 0) ? 0ULL : (~0ULL >> (64 - lane));
    for (int j = 0; j < kRounds; ++j) {
        for (int w = 0; w < 4; ++w) wcnt[w][threadIdx.x] = 0;
        __syncthreads();
        const int64_t i = tbase + j * kBlock + threadIdx.x;
        const bool act = i < n;
        uint64_t k = 0;
        int64_t v = 0;
        int d = 0;
        if (act) {
            k = keys[i];
            if (vals) v = vals[i];
            d = (int)((k >> shift) & 255);
        }
        unsigned long long peers = __ballot(act);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot(act && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const int rank = __popcll(peers & lt_mask);
        const int cnt = __popcll(peers);
        if (act && rank == 0) wcnt[wid][d] = (unsigned)cnt;
        __syncthreads();
        if (act) {
            int64_t pos = base_d[d] + rank;
            for (int w = 0; w < wid; ++w) pos += wcnt[w][d];
            okeys[pos] = k;
            if (vals) ovals[pos] = v;
        }
        __syncthreads();
        base_d[threadIdx.x] += wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] + wcnt[3][threadIdx.x];
        __syncthreads();
    }
}

}  // namespace

void radix_sort_pairs(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, int begin_bit, int end_bit) {
    std::vector<int> shifts;
    for (int shift = begin_bit; shift < end_bit; shift += 8) shifts.push_back(shift);
    radix_sort_digits(s, keys, vals, n, shifts);
}

void radix_sort_digits(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts) {
    if (n <= 1 || shifts.empty()) return;
    hipStream_t st = s->stream;
    const int64_t ntiles = (n + kTile - 1) / kTile;
    Buf hist = dev_alloc(sizeof(int64_t) * 256 * ntiles, s);
    Buf offs = dev_alloc(sizeof(int64_t) * (256 * ntiles + 1), s);
    Buf k2 = dev_alloc(sizeof(uint64_t) * n, s);
    Buf v2 = vals ? dev_alloc(sizeof(int64_t) * n, s) : Buf();
    uint64_t *ki = keys, *ko = P<uint64_t>(k2);
    int64_t *vi = vals, *vo = P<int64_t>(v2);
    int passes = 0;
    for (const int shift : shifts) {
        hipLaunchKernelGGL(k_hist, dim3((unsigned)ntiles), dim3(kBlock), 0, st, ki, n, shift, ntiles, P<int64_t>(hist));
        exclusive_scan_i64(P<int64_t>(hist), P<int64_t>(offs), 256 * ntiles, s);
        hipLaunchKernelGGL(k_scatter, dim3((unsigned)ntiles), dim3(kBlock), 0, st, ki, vi, n, shift, ntiles,
                           P<int64_t>(offs), ko, vo);
        HIP_CHECK(hipGetLastError());
        std::swap(ki, ko);
        std::swap(vi, vo);
        ++passes;
    }
    if (passes & 1) {
        HIP_CHECK(hipMemcpyAsync(keys, ki, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, st));
        if (vals) HIP_CHECK(hipMemcpyAsync(vals, vi, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, st));
    }
}

}  // namespace capsmi

namespace capsmi {
namespace {

// sort key of column value at perm[i]: unsigned-order-preserving image, complemented for DESC;
// null_pass: 1-byte key on the null flag (ASC: nulls first, DESC: nulls last -- Spark defaults)
__global__ void k_order_keys(const int64_t* __restrict__ col, const uint8_t* __restrict__ valid, int is_f64, int desc,
                             int null_pass, const int64_t* __restrict__ perm, int64_t n, uint64_t* __restrict__ key) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = perm[i];
        if (null_pass) {
            const bool ok = valid == nullptr || valid[r];
            key[i] = desc ? (ok ? 0 : 1) : (ok ? 1 : 0);
            continue;
        }
        int64_t b = col[r];
        if (is_f64) b = b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFFLL);
        const uint64_t u = (uint64_t)b ^ 0x8000000000000000ULL;
        key[i] = desc ? ~u : u;
    }
}

}  // namespace

void order_keys(capsmi_session* s, const int64_t* col, const uint8_t* valid, int type, bool desc, bool null_pass,
                const int64_t* perm, int64_t n, uint64_t* key) {
    if (n <= 0) return;
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_order_keys, dim3((unsigned)g), dim3(256), 0, s->stream, col, valid, type == CAPSMI_F64 ? 1 : 0,
                       desc ? 1 : 0, null_pass ? 1 : 0, perm, n, key);
    HIP_CHECK(hipGetLastError());
}

}  // namespace capsmi
