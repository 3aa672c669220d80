// k_sort.hip -- stable LSD radix sort of (uint64 key, int64 value) pairs, 8 bits per pass.
//
// Used by ORDER BY (DataFrameTable.orderBy, SparkTable.scala:94-103), the Cache-analogue
// clustering of relationship tables (capsmi_cluster_by), the radix join's partitioning and the C4
// graph build (k_tri.hip).
// Pass = (1) per-tile digit histogram in LDS, (2) digit-major exclusive scan of the
// [digit][tile] counts, (3) stable scatter of a tile (4096 or 16384 keys):
//   - every lane issues its kItems key (and value) loads up front, so a tile's loads are in flight
//     together (coalesced: item k of lane t is key k*kBlock + t of the tile);
//   - each wave ranks its own consecutive keys item by item: the rank among equal digits in
//     one load comes from 8 ballots (wave64), the rank across the wave's earlier items from its
//     per-digit running count in LDS (wave-local, no barrier); one prefix over the waves' counts
//     then orders the waves (3 barriers per tile);
//   - keys, then values, are staged in LDS in digit order and written out by consecutive lanes, so
//     a digit's run of the tile leaves as contiguous stores (16-64 keys on average) instead of one
//     8-byte store per key per 256-key round (k_scatter at C4: 1.5 -> 2.5-5.7 TB/s).
#include <mutex>
#include <string>

#include "capsmi_impl.h"

#include <functional>

namespace capsmi {

namespace {

// rank of this lane among the active lanes of its wave holding digit d, and their count
__device__ __forceinline__ void wave_digit_rank(bool act, int d, int& rank, int& cnt) {
    const int lane = threadIdx.x & 63;
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    unsigned long long peers = __ballot(act);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const unsigned long long bb = __ballot(act && ((d >> b) & 1));
        peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    rank = __popcll(peers & lt);
    cnt = __popcll(peers);
}

// B lanes x IT keys per tile; item j of lane l of wave w is key w * 64 * IT + j * 64 + l of the tile
template <int B, int IT>
__global__ void __launch_bounds__(B) k_hist(const uint64_t* __restrict__ keys, int64_t n, int shift, int64_t ntiles,
                                            int64_t* __restrict__ hist) {
    constexpr int T = B * IT;
    __shared__ unsigned int h[256];
    for (int i = threadIdx.x; i < 256; i += B) h[i] = 0;
    const int lane = threadIdx.x & 63, wbase = (int)(threadIdx.x >> 6) * 64 * IT;
    const int64_t tbase = (int64_t)blockIdx.x * T;
    const int cnt_tile = (int)min((int64_t)T, n - tbase);
    uint64_t k[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int idx = wbase + j * 64 + lane;
        k[j] = idx < cnt_tile ? keys[tbase + idx] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; ++j) {  // one LDS add per (wave, digit): skewed digits do not serialise
        const bool act = wbase + j * 64 + lane < cnt_tile;
        const int d = (int)((k[j] >> shift) & 255);
        int rank, cnt;
        wave_digit_rank(act, d, rank, cnt);
        if (act && rank == 0) atomicAdd(&h[d], (unsigned)cnt);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += B) hist[(int64_t)i * ntiles + blockIdx.x] = h[i];
}

template <int B>
constexpr size_t scatter_lds(int tile) {
    return sizeof(uint64_t) * tile + sizeof(int64_t) * 256 + sizeof(unsigned short) * (B / 64) * 256 +
           sizeof(unsigned int) * (256 + B / 64 + 1);
}

template <int B, int IT, bool VALS>
__global__ void __launch_bounds__(B) k_scatter(const uint64_t* __restrict__ keys, const int64_t* __restrict__ vals,
                                               int64_t n, int shift, int64_t ntiles, const int64_t* __restrict__ offs,
                                               uint64_t* __restrict__ okeys, int64_t* __restrict__ ovals) {
    constexpr int T = B * IT, W = B / 64;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];  // scatter_lds<B>(T) bytes
    uint64_t* stage = smem;                                              // the tile in digit order (keys, then values)
    int64_t* gbase = reinterpret_cast<int64_t*>(stage + T);              // the digit's first output position
    unsigned short (*wc)[256] = reinterpret_cast<unsigned short (*)[256]>(gbase + 256);  // per-wave digit counts
    unsigned int* tstart = reinterpret_cast<unsigned int*>(&wc[W][0]);  // the digit's first position in the tile
    unsigned int* wsum = tstart + 256;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t tile = blockIdx.x;
    const int64_t tbase = tile * T;
    const int cnt_tile = (int)min((int64_t)T, n - tbase);
    // wave w owns keys [w * 64 * IT, (w + 1) * 64 * IT) of the tile: index order inside a wave is
    // (item, lane), so a wave ranks its own keys alone and one prefix over the waves' per-digit
    // counts orders the waves
    const int wbase = wid * 64 * IT;
    uint64_t k[IT];
    int64_t v[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int idx = wbase + j * 64 + lane;
        k[j] = idx < cnt_tile ? keys[tbase + idx] : 0;
    }
    for (int i = threadIdx.x; i < 256; i += B) gbase[i] = offs[(int64_t)i * ntiles + blockIdx.x];
#pragma unroll
    for (int i = 0; i < 4; ++i) wc[wid][i * 64 + lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    unsigned int lrank[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {  // wave-local: LDS accesses of one wave are ordered
        const bool act = wbase + j * 64 + lane < cnt_tile;
        const int d = (int)((k[j] >> shift) & 255);
        int rank, cnt;
        wave_digit_rank(act, d, rank, cnt);
        const unsigned int before = act ? wc[wid][d] : 0u;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (act && rank == 0) wc[wid][d] = (unsigned short)(before + (unsigned)cnt);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        lrank[j] = before + (unsigned)rank;
    }
    if (VALS) {  // the values are only staged after the keys: their loads overlap the prefix and key phase
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const int idx = wbase + j * 64 + lane;
            v[j] = idx < cnt_tile ? vals[tbase + idx] : 0;
        }
    }
    __syncthreads();
    unsigned int tot = 0;
    if (threadIdx.x < 256) {  // exclusive prefix of each digit's count over the waves
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const unsigned int c = wc[w][threadIdx.x];
            wc[w][threadIdx.x] = (unsigned short)tot;
            tot += c;
        }
    }
    // tile-local digit starts: exclusive scan of the totals (one per lane of waves 0-3)
    unsigned int incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (threadIdx.x < 256) {
        unsigned int pre = 0;
        for (int w = 0; w < wid; ++w) pre += wsum[w];
        tstart[threadIdx.x] = pre + incl - tot;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < IT; ++j) {  // stage position of each key (kept for the values)
        const int d = (int)((k[j] >> shift) & 255);
        lrank[j] += tstart[d] + wc[wid][d];
        if (wbase + j * 64 + lane < cnt_tile) stage[lrank[j]] = k[j];
    }
    __syncthreads();
    // a digit's run of the tile leaves as contiguous stores by consecutive lanes
    int dd[IT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int i = j * B + (int)threadIdx.x;
        dd[j] = 0;
        if (i < cnt_tile) {
            const uint64_t key = stage[i];
            dd[j] = (int)((key >> shift) & 255);
            okeys[gbase[dd[j]] + (i - (int)tstart[dd[j]])] = key;
        }
    }
    if (VALS) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j)
            if (wbase + j * 64 + lane < cnt_tile) stage[lrank[j]] = (uint64_t)v[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const int i = j * B + (int)threadIdx.x;
            if (i < cnt_tile) ovals[gbase[dd[j]] + (i - (int)tstart[dd[j]])] = (int64_t)stage[i];
        }
    }
}

template <int B, int IT>
void sort_passes(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts,
                 int at, const std::function<void(const uint64_t*)>& cb, Buf* kbuf = nullptr,
                 const int64_t* hist0 = nullptr) {
    constexpr int T = B * IT;
    static std::once_flag once;  // the staged tile takes more than 64 KiB of LDS
    std::call_once(once, [] {
        for (const void* k : {reinterpret_cast<const void*>(k_scatter<B, IT, true>),
                              reinterpret_cast<const void*>(k_scatter<B, IT, false>)})
            HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)scatter_lds<B>(T)));
    });
    hipStream_t st = s->stream;
    const int64_t ntiles = (n + T - 1) / T;
    // a histogram kernel and a scan per pass.  (A onesweep form -- every pass's histogram from one read, tiles
    // finding their starts by decoupled look-back -- measured slower at C4 and removed in round 6: tri_sort_und
    // 16.5 -> 20.2 ms, tri_sort_or 11.8 -> 15.2 ms; the look-back's agent-scope polls cross the XCDs' L2s)
    Buf hist = dev_alloc(sizeof(int64_t) * 256 * ntiles, s);
    Buf offs = dev_alloc(sizeof(int64_t) * (256 * ntiles + 1), s);
    Buf k2 = dev_alloc(sizeof(uint64_t) * n, s);
    Buf v2 = vals ? dev_alloc(sizeof(int64_t) * n, s) : Buf();
    uint64_t *ki = keys, *ko = P<uint64_t>(k2);
    int64_t *vi = vals, *vo = P<int64_t>(v2);
    int passes = 0;
    for (const int shift : shifts) {
        {
            if (passes == 0 && hist0)  // the first digit's tile counts came with the keys
                exclusive_scan_i64(hist0, P<int64_t>(offs), 256 * ntiles, s);
            else {
                hipLaunchKernelGGL((k_hist<B, IT>), dim3((unsigned)ntiles), dim3(B), 0, st, ki, n, shift, ntiles,
                                   P<int64_t>(hist));
                exclusive_scan_i64(P<int64_t>(hist), P<int64_t>(offs), 256 * ntiles, s);
            }
            if (vals)
                hipLaunchKernelGGL((k_scatter<B, IT, true>), dim3((unsigned)ntiles), dim3(B), scatter_lds<B>(T), st, ki,
                                   vi, n, shift, ntiles, P<int64_t>(offs), ko, vo);
            else
                hipLaunchKernelGGL((k_scatter<B, IT, false>), dim3((unsigned)ntiles), dim3(B), scatter_lds<B>(T), st,
                                   ki, vi, n, shift, ntiles, P<int64_t>(offs), ko, vo);
        }
        HIP_CHECK(hipGetLastError());
        std::swap(ki, ko);
        std::swap(vi, vo);
        ++passes;
        if (passes == at && cb) cb(ki);
    }
    if ((passes & 1) && kbuf && !vals) {  // the caller takes the other buffer: no copy back
        *kbuf = k2;
    } else if (passes & 1) {
        HIP_CHECK(hipMemcpyAsync(keys, ki, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, st));
        if (vals) HIP_CHECK(hipMemcpyAsync(vals, vi, sizeof(int64_t) * n, hipMemcpyDeviceToDevice, st));
    }
}

}  // namespace

void radix_sort_pairs(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, int begin_bit, int end_bit) {
    std::vector<int> shifts;
    for (int shift = begin_bit; shift < end_bit; shift += 8) shifts.push_back(shift);
    radix_sort_digits(s, keys, vals, n, shifts);
}

// Key-value sorts of >= 1024 tiles use 12288-key tiles (one 1024-lane block per CU): a digit's run
// of a tile then averages 48 keys, so random digits cost fewer partial-line writes in the two
// output arrays (C4 at s=24, 2^28 pairs: 2.4-3.3 -> 1.6-2.5 ms per pass).  Key-only sorts and
// smaller ones use 4096-key tiles (two 512-lane blocks per CU): a 2^28-key pass takes 1.19 ms
// there against 1.4 ms with the larger tile.
void radix_sort_digits(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts,
                       int at, const std::function<void(const uint64_t*)>& cb) {
    if (n <= 1 || shifts.empty()) {
        if (cb) cb(keys);
        return;
    }
    if (vals && n >= (int64_t(1024) * 12288)) sort_passes<1024, 12>(s, keys, vals, n, shifts, at, cb);
    else sort_passes<512, 8>(s, keys, vals, n, shifts, at, cb);
}

void radix_sort_digits(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts) {
    radix_sort_digits(s, keys, vals, n, shifts, 0, nullptr);
}

static_assert(512 * 8 == kSortTile, "key-only sorts: 4096-key tiles");

void radix_sort_keys(capsmi_session* s, Buf& keys, int64_t n, const std::vector<int>& shifts, const int64_t* hist0) {
    if (n <= 1 || shifts.empty()) return;
    sort_passes<512, 8>(s, P<uint64_t>(keys), nullptr, n, shifts, 0, nullptr, &keys, hist0);
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
