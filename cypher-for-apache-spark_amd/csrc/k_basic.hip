// k_basic.hip -- scan, stream compaction, gather: the building blocks every
// Table operator uses (filter = predicate + compaction + gather; join/group =
// hash + scan + gather).  Wave64 throughout: __ballot is 64-bit and the
// per-wave scans run over 64 lanes.
#include <climits>

#include "capsmi_impl.h"

namespace capsmi {

namespace {

constexpr int kBlock = 256;           // 4 waves
constexpr int kItems = 8;             // items per thread in tiled kernels
constexpr int kTile = kBlock * kItems;  // 2048 rows per tile

__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// exclusive block scan of one value per thread; returns prefix, writes block total
__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t* lds4, int64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int64_t inc = wave_incl_scan(x);
    if (lane == 63) lds4[wid] = inc;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const int64_t v = lds4[w];
        if (w < wid) base += v;
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return base + inc - x;
}

__global__ void __launch_bounds__(kBlock) k_tile_sum(const int64_t* __restrict__ in, int64_t n,
                                                     int64_t* __restrict__ sums) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t i = base + j * kBlock + threadIdx.x;
        if (i < n) s += in[i];
    }
    __shared__ int64_t lds[kBlock / 64];
    int64_t tot;
    block_excl_scan(s, lds, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// blocked per-thread scan via an LDS transpose (coalesced global loads)
__global__ void __launch_bounds__(kBlock) k_tile_scan(const int64_t* __restrict__ in, int64_t n,
                                                      const int64_t* __restrict__ tile_off,
                                                      int64_t* __restrict__ out) {
    __shared__ int64_t tile[kTile];
    __shared__ int64_t lds[kBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t i = base + j * kBlock + threadIdx.x;
        tile[j * kBlock + threadIdx.x] = i < n ? in[i] : 0;
    }
    __syncthreads();
    int64_t v[kItems];
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        v[j] = tile[threadIdx.x * kItems + j];
        s += v[j];
    }
    int64_t tot;
    const int64_t toff = tile_off ? tile_off[blockIdx.x] : 0;  // null: a single tile
    int64_t pre = block_excl_scan(s, lds, &tot) + toff;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        tile[threadIdx.x * kItems + j] = pre;
        pre += v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t i = base + j * kBlock + threadIdx.x;
        if (i < n) out[i] = tile[j * kBlock + threadIdx.x];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) out[n] = toff + tot;
}

__global__ void k_fill_i64(int64_t* p, int64_t v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
__global__ void k_fill_u8(uint8_t* p, uint8_t v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
__global__ void k_iota_i64(int64_t* p, int64_t start, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = start + i;
}

// per-tile count of set flags (blocked: thread t owns rows [t*8, t*8+8) of the tile)
__global__ void __launch_bounds__(kBlock) k_flag_count(const uint8_t* __restrict__ f, int64_t n,
                                                       int64_t* __restrict__ cnt) {
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) c += (base + j < n && f[base + j]) ? 1 : 0;
    __shared__ int64_t lds[kBlock / 64];
    int64_t tot;
    block_excl_scan(c, lds, &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// the rows of the set flags as two columns at once: ids[pos] = base + i, vals[pos] = val[i] (flags_to_rows)
__global__ void __launch_bounds__(kBlock) k_flag_rows(const uint8_t* __restrict__ f, int64_t n,
                                                      const int64_t* __restrict__ off, const int64_t* __restrict__ val,
                                                      int64_t id_base, int64_t* __restrict__ ids,
                                                      int64_t* __restrict__ vals) {
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
    uint8_t fl[kItems];
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        fl[j] = (base + j < n && f[base + j]) ? 1 : 0;
        c += fl[j];
    }
    __shared__ int64_t lds[kBlock / 64];
    int64_t tot;
    int64_t pos = block_excl_scan(c, lds, &tot) + off[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kItems; ++j)
        if (fl[j]) {
            ids[pos] = id_base + base + j;
            vals[pos] = val[base + j];
            ++pos;
        }
}

__global__ void __launch_bounds__(kBlock) k_flag_write(const uint8_t* __restrict__ f, int64_t n,
                                                       const int64_t* __restrict__ off,
                                                       int64_t* __restrict__ idx) {
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
    uint8_t fl[kItems];
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        fl[j] = (base + j < n && f[base + j]) ? 1 : 0;
        c += fl[j];
    }
    __shared__ int64_t lds[kBlock / 64];
    int64_t tot;
    int64_t pos = block_excl_scan(c, lds, &tot) + off[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kItems; ++j)
        if (fl[j]) idx[pos++] = base + j;
}

__global__ void k_gather(const int64_t* __restrict__ src, const uint8_t* __restrict__ sv,
                         const int64_t* __restrict__ idx, int64_t n, int64_t* __restrict__ dst,
                         uint8_t* __restrict__ dv) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = idx[i];
        const bool ok = j >= 0 && (sv == nullptr || sv[j]);
        dst[i] = ok ? src[j] : 0;
        if (dv) dv[i] = ok ? 1 : 0;
    }
}

inline int grid_for(int64_t n, int block = 256) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 8192) g = 8192;
    return (int)g;
}

}  // namespace

void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, capsmi_session* s) {
    hipStream_t st = s->stream;
    const int64_t ntiles = (n + kTile - 1) / kTile;
    if (n == 0) {
        HIP_CHECK(hipMemsetAsync(out, 0, sizeof(int64_t), st));
        return;
    }
    if (ntiles == 1) {  // one launch
        hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(kBlock), 0, st, in, n, (const int64_t*)nullptr, out);
        HIP_CHECK(hipGetLastError());
        return;
    }
    Buf sums = dev_alloc(sizeof(int64_t) * ntiles, s);
    Buf offs = dev_alloc(sizeof(int64_t) * (ntiles + 1), s);
    hipLaunchKernelGGL(k_tile_sum, dim3((unsigned)ntiles), dim3(kBlock), 0, st, in, n, P<int64_t>(sums));
    exclusive_scan_i64(P<int64_t>(sums), P<int64_t>(offs), ntiles, s);
    hipLaunchKernelGGL(k_tile_scan, dim3((unsigned)ntiles), dim3(kBlock), 0, st, in, n, P<int64_t>(offs), out);
    HIP_CHECK(hipGetLastError());
}

void fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(n)), dim3(256), 0, st, p, v, n);
}
void fill_u8(uint8_t* p, uint8_t v, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill_u8, dim3(grid_for(n)), dim3(256), 0, st, p, v, n);
}
void iota_i64(int64_t* p, int64_t start, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_iota_i64, dim3(grid_for(n)), dim3(256), 0, st, p, start, n);
}

int64_t read_scalar(capsmi_session* s, const int64_t* dev) {
    HIP_CHECK(hipMemcpyAsync(s->pinned, dev, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    return s->pinned[0];
}

void read_scalar_async(capsmi_session* s, const int64_t* dev) {
    HIP_CHECK(hipMemcpyAsync(s->pinned + 1, dev, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipEventRecord(s->ev_read, s->stream));
}

int64_t read_scalar_wait(capsmi_session* s) {
    HIP_CHECK(hipEventSynchronize(s->ev_read));
    return s->pinned[1];
}

int64_t flags_to_indices(capsmi_session* s, const uint8_t* flags, int64_t n, Buf& out_idx) {
    hipStream_t st = s->stream;
    if (n == 0) {
        out_idx = dev_alloc(8, s);
        return 0;
    }
    const int64_t ntiles = (n + kTile - 1) / kTile;
    Buf cnt = dev_alloc(sizeof(int64_t) * ntiles, s);
    Buf off = dev_alloc(sizeof(int64_t) * (ntiles + 1), s);
    hipLaunchKernelGGL(k_flag_count, dim3((unsigned)ntiles), dim3(kBlock), 0, st, flags, n, P<int64_t>(cnt));
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(off), ntiles, s);
    const int64_t total = read_scalar(s, P<int64_t>(off) + ntiles);
    out_idx = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    hipLaunchKernelGGL(k_flag_write, dim3((unsigned)ntiles), dim3(kBlock), 0, st, flags, n, P<int64_t>(off),
                       P<int64_t>(out_idx));
    HIP_CHECK(hipGetLastError());
    return total;
}

int64_t flags_to_rows(capsmi_session* s, const uint8_t* flags, int64_t n, const int64_t* val, int64_t id_base,
                      Buf& out_ids, Buf& out_vals) {
    hipStream_t st = s->stream;
    out_ids = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    out_vals = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    if (n == 0) return 0;
    const int64_t ntiles = (n + kTile - 1) / kTile;
    Buf cnt = dev_alloc(sizeof(int64_t) * ntiles, s);
    Buf off = dev_alloc(sizeof(int64_t) * (ntiles + 1), s);
    hipLaunchKernelGGL(k_flag_count, dim3((unsigned)ntiles), dim3(kBlock), 0, st, flags, n, P<int64_t>(cnt));
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(off), ntiles, s);
    hipLaunchKernelGGL(k_flag_rows, dim3((unsigned)ntiles), dim3(kBlock), 0, st, flags, n, P<int64_t>(off), val, id_base,
                       P<int64_t>(out_ids), P<int64_t>(out_vals));
    HIP_CHECK(hipGetLastError());
    return read_scalar(s, P<int64_t>(off) + ntiles);  // the one host round trip, behind the writes
}

void gather_col(const int64_t* src, const uint8_t* src_valid, const int64_t* idx, int64_t n, int64_t* dst,
                uint8_t* dst_valid, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_gather, dim3(grid_for(n)), dim3(256), 0, st, src, src_valid, idx, n, dst, dst_valid);
    HIP_CHECK(hipGetLastError());
}

}  // namespace capsmi

namespace capsmi {
namespace {
__global__ void k_invert_u8(const uint8_t* __restrict__ a, uint8_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i] ? 0 : 1;
}
__global__ void k_i64_to_f64(const int64_t* __restrict__ a, int64_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = __double_as_longlong((double)a[i]);
}
}  // namespace

void invert_u8(const uint8_t* a, uint8_t* b, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_invert_u8, dim3(grid_for(n)), dim3(256), 0, st, a, b, n);
    HIP_CHECK(hipGetLastError());
}
namespace {

// block min/max over up to 3 columns, one atomic pair per block
__global__ void k_minmax(const int64_t* __restrict__ c0, const int64_t* __restrict__ c1, const int64_t* __restrict__ c2,
                         int64_t n, long long* out) {
    long long lo = LLONG_MAX, hi = LLONG_MIN;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const long long a = c0[i];
        lo = min(lo, a);
        hi = max(hi, a);
        if (c1) { const long long b = c1[i]; lo = min(lo, b); hi = max(hi, b); }
        if (c2) { const long long c = c2[i]; lo = min(lo, c); hi = max(hi, c); }
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (long long)__shfl_xor(lo, o));
        hi = max(hi, (long long)__shfl_xor(hi, o));
    }
    __shared__ long long slo[4], shi[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { slo[w] = lo; shi[w] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) { lo = min(lo, slo[k]); hi = max(hi, shi[k]); }
        atomicMin(&out[0], lo);
        atomicMax(&out[1], hi);
    }
}

// DataFrameOps.withCypherCompatibleTypes (spark-cypher/.../impl/DataFrameOps.scala:185-198):
// Byte/Short/Integer -> Long, Float -> Double; Boolean bytes -> 0/1 words
__global__ void k_widen(const void* __restrict__ in, int code, int64_t* __restrict__ out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t v;
        switch (code) {
            case CAPSMI_IN_I32: v = ((const int32_t*)in)[i]; break;
            case CAPSMI_IN_I16: v = ((const int16_t*)in)[i]; break;
            case CAPSMI_IN_I8: v = ((const int8_t*)in)[i]; break;
            case CAPSMI_IN_F32: v = __double_as_longlong((double)((const float*)in)[i]); break;
            default: v = ((const uint8_t*)in)[i] != 0; break;  // CAPSMI_IN_BOOL8
        }
        out[i] = v;
    }
}

}  // namespace

void minmax_i64(capsmi_session* s, const int64_t* const* cols, int ncols, int64_t n, int64_t* out) {
    Buf d = dev_alloc(2 * sizeof(long long), s);
    const long long init[2] = {LLONG_MAX, LLONG_MIN};
    HIP_CHECK(hipMemcpyAsync(P<void>(d), init, sizeof(init), hipMemcpyHostToDevice, s->stream));
    if (n > 0) {
        hipLaunchKernelGGL(k_minmax, dim3(grid_for(n)), dim3(256), 0, s->stream, cols[0], ncols > 1 ? cols[1] : nullptr,
                           ncols > 2 ? cols[2] : nullptr, n, P<long long>(d));
        HIP_CHECK(hipGetLastError());
    }
    long long h[2];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(d), sizeof(h), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    out[0] = h[0];
    out[1] = h[1];
}

void widen_words(const void* in, int code, int64_t* out, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_widen, dim3(grid_for(n)), dim3(256), 0, st, in, code, out, n);
    HIP_CHECK(hipGetLastError());
}

void i64_to_f64(const int64_t* a, int64_t* b, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_i64_to_f64, dim3(grid_for(n)), dim3(256), 0, st, a, b, n);
    HIP_CHECK(hipGetLastError());
}
}  // namespace capsmi

namespace capsmi {
namespace {
__global__ void k_add_i64(int64_t* p, int64_t v, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] += v;
}
}  // namespace

void add_i64(int64_t* p, int64_t v, int64_t n, hipStream_t st) {
    if (n <= 0 || v == 0) return;
    hipLaunchKernelGGL(k_add_i64, dim3(grid_for(n)), dim3(256), 0, st, p, v, n);
    HIP_CHECK(hipGetLastError());
}
}  // namespace capsmi
