// k_dist.hip -- multi-GPU shards of a graph: the rank view of a session, hash
// ownership of ids, and the registration of a rank's entity tables as its shard.
//
// Spark partitions every DataFrame and shuffles rows by a hash of the join / grouping key before
// joins and aggregates (Exchange hashpartitioning, SparkTable.scala:133, 226).  Here ownership is
// fixed once per graph: ids are scrambled by a bijection of the graph's id window, and each rank
// owns one contiguous range of scrambled ids, so balance does not depend on how the ids were assigned
// (R-MAT hubs, edge lists whose hubs sit at ids 0..1000).  The fused kernels run on the scrambled ids
// (the dense key columns of capsmi_graph_compact's machinery); the routes in plan.hip exchange
// bitmap slices and counts through the host's collective (capsmi_session_set_ranks).
#include <memory>

#include "capsmi_impl.h"

namespace capsmi {

void set_last_error(const std::string& m);

namespace {

constexpr uint64_t kScrambleMul = 0x9E3779B97F4A7C15ULL;  // odd: a bijection modulo any 2^k

inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

__device__ __forceinline__ int64_t h_of(int64_t x, int64_t lo, uint64_t mul, uint64_t mask) {
    return (int64_t)(((uint64_t)(x - lo) * mul) & mask);
}

__global__ void k_scramble(const int64_t* __restrict__ in, int64_t n, int64_t lo, int64_t hi, uint64_t mul,
                           uint64_t mask, int64_t own_lo, int64_t own_hi, int64_t* __restrict__ out,
                           unsigned long long* __restrict__ bad) {
    unsigned long long outside = 0, foreign = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = in[i];
        const bool ok = x >= lo && x < hi;
        const int64_t d = ok ? h_of(x, lo, mul, mask) : 0;
        out[i] = d;
        outside += ok ? 0 : 1;
        foreign += (own_lo < own_hi && ok && (d < own_lo || d >= own_hi)) ? 1 : 0;
    }
    if (outside) atomicAdd(&bad[0], outside);
    if (foreign) atomicAdd(&bad[1], foreign);
}

__global__ void k_unscramble(int64_t* __restrict__ v, int64_t n, int64_t lo, uint64_t mul_inv, uint64_t mask) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (int64_t)(((uint64_t)v[i] * mul_inv) & mask) + lo;
}

// counts[q] = #{i : low byte of the sorted dest[i] == q}, q < world: one binary search per rank boundary
__global__ void k_dest_counts(const uint64_t* __restrict__ dest, int64_t n, int world, int64_t* __restrict__ counts) {
    const int q = threadIdx.x;  // one block of 256 lanes, world < 255
    __shared__ int64_t at[257];
    if (q <= world) {
        int64_t a = 0, b = n;  // first i with dest[i] >= q
        while (a < b) {
            const int64_t mid = (a + b) >> 1;
            if ((int64_t)(dest[mid] & 0xFF) < q) a = mid + 1; else b = mid;
        }
        at[q] = a;
    }
    __syncthreads();
    if (q < world) counts[q] = at[q + 1] - at[q];
}

// (source, target) rows whose target another rank owns -> one word source << 32 | target to that rank
// the complement exchange of a relationship shard: each row to the owner of its `key` end (dst for BY_SOURCE
// shards: their in-relationships; src for BY_TARGET shards: their out-relationships), 0xFF when that is this rank
__global__ void k_in_words(const int64_t* __restrict__ src, const int64_t* __restrict__ dst, int64_t m, int64_t span,
                           int rank, int world, int key_src, uint64_t* __restrict__ dest, uint64_t* __restrict__ w) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = dst[i];
        int q = (int)((key_src ? src[i] : t) / span);
        q = q < world ? q : world - 1;
        dest[i] = q == rank ? 0xFF : (uint64_t)q;
        w[i] = ((uint64_t)src[i] << 32) | (uint64_t)t;
    }
}

__global__ void k_unpack_words(const uint64_t* __restrict__ w, int64_t n, int64_t* __restrict__ a,
                               int64_t* __restrict__ b) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        a[i] = (int64_t)(w[i] >> 32);
        b[i] = (int64_t)(uint32_t)w[i];
    }
}

// destination of each row: a hash of its key columns mod world (Spark's HashPartitioning); rows with a
// null key go to `null_rank` when it is >= 0 (they match nothing: joins keep them where they are), else
// nulls hash as a tag (grouping: nulls form one group).  as_f64[k]: hash key k as a double (a Long key
// joined with a Double key, widened by the join)
struct KeyHashCols {
    const int64_t* d[8];
    const uint8_t* v[8];
    int as_f64[8];
    int n;
};
__device__ __forceinline__ uint64_t dmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__global__ void k_key_dest(KeyHashCols k, int64_t n, int world, int null_rank, uint64_t* __restrict__ dest) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        uint64_t h = 0x243F6A8885A308D3ULL;
        bool any_null = false;
        for (int c = 0; c < k.n; ++c) {
            const bool nul = k.v[c] && !k.v[c][r];
            any_null = any_null || nul;
            uint64_t v = nul ? 0 : (uint64_t)k.d[c][r];
            if (!nul && k.as_f64[c] == 1) {  // a Long widened to its double
                const double x = (double)(int64_t)v;
                v = __double_as_longlong(x);
            }
            if (!nul && k.as_f64[c] && (v << 1) == 0) v = 0;  // -0.0 == 0.0
            h = dmix64(h ^ (v + (nul ? 0x3C6EF372FE94F82BULL : 0) + (uint64_t)c * 0x9E3779B97F4A7C15ULL));
        }
        dest[r] = (any_null && null_rank >= 0) ? (uint64_t)null_rank : (h % (uint64_t)world);
    }
}

__global__ void k_row_dest_slice(int64_t n, int rank, int world, uint64_t* __restrict__ dest) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        dest[r] = (uint64_t)(r % world == rank ? rank : 0xFF);
}

__global__ void k_valid_to_words(const uint8_t* __restrict__ v, int64_t n, int64_t* __restrict__ w) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        w[r] = v ? v[r] : 1;
}

__global__ void k_words_to_valid(const int64_t* __restrict__ w, int64_t n, uint8_t* __restrict__ v) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x)
        v[r] = (uint8_t)(w[r] != 0);
}

// list columns: each row's list length (0 for a null row) in the order `idx` (or row order when null)
__global__ void k_list_lens(const int64_t* __restrict__ li, const uint8_t* __restrict__ valid,
                            const int64_t* __restrict__ off, const int64_t* __restrict__ idx, int64_t n,
                            int64_t* __restrict__ len) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx ? idx[k] : k;
        len[k] = (valid && !valid[r]) ? 0 : off[li[r] + 1] - off[li[r]];
    }
}

// the rows' list values back to back in the order `idx` (voff: exclusive prefix of their lengths)
__global__ void k_list_pack(const int64_t* __restrict__ li, const uint8_t* __restrict__ valid,
                            const int64_t* __restrict__ off, const int64_t* __restrict__ vals,
                            const int64_t* __restrict__ idx, int64_t n, const int64_t* __restrict__ voff,
                            int64_t* __restrict__ out) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = idx ? idx[k] : k;
        if (valid && !valid[r]) continue;
        const int64_t b = off[li[r]], e = off[li[r] + 1];
        for (int64_t j = b; j < e; ++j) out[voff[k] + (j - b)] = vals[j];
    }
}

// value counts per destination: voff at the row-segment boundaries (rs: W + 1 row starts)
__global__ void k_seg_values(const int64_t* __restrict__ voff, const int64_t* __restrict__ rs, int W,
                             int64_t* __restrict__ out) {
    const int q = threadIdx.x;
    if (q < W) out[q] = voff[rs[q + 1]] - voff[rs[q]];
}

__global__ void k_owned_flags(const int64_t* __restrict__ in, int64_t n, int64_t lo, int64_t hi, uint64_t mul,
                              uint64_t mask, int64_t own_lo, int64_t own_hi, uint8_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = in[i];
        const int64_t d = h_of(x, lo, mul, mask);
        flags[i] = (x >= lo && x < hi && d >= own_lo && d < own_hi) ? 1 : 0;
    }
}

}  // namespace

// Elements one call of the host's collective moves in all (CAPSMI_COLL_CHUNK, default 2^26: 512 MiB of
// int64).  Every call the library makes is cut to this size here, so no host adapter (TorchCollective, the
// JVM CollectiveFn) ever receives a larger one.  Round 4's C4 route at world size 1 faulted
// (hipErrorIllegalAddress) in the first run that handed RCCL 2^28-word (2^31-byte) calls; the same build
// equals its fixture with every call below 2^31 bytes.
int64_t coll_chunk(const capsmi_session* s) { return s->cfg.coll_chunk > 0 ? s->cfg.coll_chunk : (int64_t(1) << 26); }

namespace {
size_t coll_elem_bytes(int dtype) { return dtype == CAPSMI_COLL_U32 ? 4 : 8; }

void coll_call(capsmi_session* s, int op, const void* send, void* recv, int64_t count, int dtype) {
    REQUIRE(s->coll != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "a distributed route needs the session's collective (capsmi_session_set_ranks)");
    const int32_t rc = s->coll(s->coll_ctx, op, send, recv, count, dtype);
    REQUIRE(rc == 0, CAPSMI_ERR_DEVICE, "the host collective failed (op " + std::to_string(op) + ")");
}
}  // namespace

void collective(capsmi_session* s, int op, const void* send, void* recv, int64_t count, int dtype) {
    REQUIRE(op != CAPSMI_COLL_ALL_TO_ALL_V, CAPSMI_ERR_INTERNAL, "ALL_TO_ALL_V goes through collective_a2av");
    const int W = s->world > 0 ? s->world : 1;
    const int64_t chunk = coll_chunk(s);
    const size_t es = coll_elem_bytes(dtype);
    if (op == CAPSMI_COLL_ALL_GATHER) {
        const int64_t per = std::max<int64_t>(1, chunk / W);  // words per rank in one call
        if (count <= per) {
            coll_call(s, op, send, recv, count, dtype);
            return;
        }
        // slices of `per` words per rank gathered into a staging buffer (rank-major W x c), then placed
        // into the rank-major output (W x count) by one strided copy
        Buf tmp = dev_alloc(es * (size_t)W * (size_t)per, s);
        for (int64_t off = 0; off < count; off += per) {
            const int64_t c = std::min(per, count - off);
            coll_call(s, op, static_cast<const char*>(send) + es * off, P<void>(tmp), c, dtype);
            HIP_CHECK(hipMemcpy2DAsync(static_cast<char*>(recv) + es * off, es * count, P<void>(tmp), es * c, es * c, W,
                                       hipMemcpyDeviceToDevice, s->stream));
        }
        return;
    }
    if (count <= chunk) {
        coll_call(s, op, send, recv, count, dtype);
        return;
    }
    for (int64_t off = 0; off < count; off += chunk)  // all-reduces are element-wise: consecutive sub-ranges
        coll_call(s, op, static_cast<const char*>(send) + es * off, static_cast<char*>(recv) + es * off,
                  std::min(chunk, count - off), dtype);
}

// max_pair: the largest entry of the whole W x W count matrix (the same on every rank, which all-gathered
// it): the ranks then agree on the number of rounds without a collective of their own
void collective_a2av(capsmi_session* s, const void* send, const int64_t* send_counts, void* recv,
                     const int64_t* recv_counts, int dtype, int64_t max_pair) {
    const int W = s->world;
    const int64_t per = std::max<int64_t>(1, coll_chunk(s) / std::max(W, 1));  // words per (source, destination)
    const int64_t rounds = std::max<int64_t>(1, (max_pair + per - 1) / per);
    if (rounds == 1) {
        capsmi_coll_vec sv{const_cast<void*>(send), send_counts}, rv{recv, recv_counts};
        coll_call(s, CAPSMI_COLL_ALL_TO_ALL_V, &sv, &rv, W, dtype);
        return;
    }
    // rounds of at most `per` words per pair: round k moves words [k * per, (k + 1) * per) of every segment,
    // packed into / unpacked from staging buffers
    const size_t es = coll_elem_bytes(dtype);
    std::vector<int64_t> so(W + 1, 0), ro(W + 1, 0), ss(W), rr(W);
    for (int q = 0; q < W; ++q) {
        so[q + 1] = so[q] + send_counts[q];
        ro[q + 1] = ro[q] + recv_counts[q];
    }
    Buf ts = dev_alloc(es * (size_t)W * (size_t)per, s), tr = dev_alloc(es * (size_t)W * (size_t)per, s);
    const char* sb = static_cast<const char*>(send);
    char* rb = static_cast<char*>(recv);
    for (int64_t k = 0; k < rounds; ++k) {
        int64_t at = 0;
        for (int q = 0; q < W; ++q) {
            ss[q] = std::min(per, std::max<int64_t>(0, send_counts[q] - k * per));
            rr[q] = std::min(per, std::max<int64_t>(0, recv_counts[q] - k * per));
            if (ss[q] > 0)
                HIP_CHECK(hipMemcpyAsync(P<char>(ts) + es * at, sb + es * (so[q] + k * per), es * ss[q],
                                         hipMemcpyDeviceToDevice, s->stream));
            at += ss[q];
        }
        capsmi_coll_vec sv{P<void>(ts), ss.data()}, rv{P<void>(tr), rr.data()};
        coll_call(s, CAPSMI_COLL_ALL_TO_ALL_V, &sv, &rv, W, dtype);
        at = 0;
        for (int q = 0; q < W; ++q) {
            if (rr[q] > 0)
                HIP_CHECK(hipMemcpyAsync(rb + es * (ro[q] + k * per), P<char>(tr) + es * at, es * rr[q],
                                         hipMemcpyDeviceToDevice, s->stream));
            at += rr[q];
        }
    }
}

int64_t matrix_max(const std::vector<int64_t>& m) {
    int64_t x = 0;
    for (int64_t v : m) x = std::max(x, v);
    return x;
}

// The hash Exchange of u64 words (SparkTable.scala:133, 226 insert one before every join and grouping):
// word i goes to rank dest[i] (its low byte; 0xFF = keep it out of the exchange).  One stable 8-bit radix
// pass groups the words by destination, an ALL_GATHER of the per-rank counts gives every rank the whole
// count matrix, and one ALL_TO_ALL_V moves the words.  dest and words are scratch (reordered).  Returns
// the received words, rank-major by source rank; synchronises (the counts come to the host).
Buf exchange_words(capsmi_session* s, uint64_t* dest, uint64_t* words, int64_t n, int64_t* nrecv) {
    const int W = s->world;
    REQUIRE(W >= 1 && W < 255, CAPSMI_ERR_UNSUPPORTED, "exchange: at most 254 ranks");
    hipStream_t st = s->stream;
    radix_sort_digits(s, dest, reinterpret_cast<int64_t*>(words), n, {0});
    Buf cnt = dev_alloc(sizeof(int64_t) * (W + (size_t)W * W), s);
    int64_t* mine = P<int64_t>(cnt);
    int64_t* all = mine + W;
    if (n > 0) {
        hipLaunchKernelGGL(k_dest_counts, dim3(1), dim3(256), 0, st, dest, n, W, mine);
        HIP_CHECK(hipGetLastError());
    } else {
        HIP_CHECK(hipMemsetAsync(mine, 0, sizeof(int64_t) * W, st));
    }
    collective(s, CAPSMI_COLL_ALL_GATHER, mine, all, W, CAPSMI_I64);
    std::vector<int64_t> m((size_t)W * W);
    HIP_CHECK(hipMemcpyAsync(m.data(), all, sizeof(int64_t) * m.size(), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    std::vector<int64_t> sc(W), rc(W);
    int64_t tot = 0;
    for (int q = 0; q < W; ++q) {
        sc[q] = m[(size_t)s->rank * W + q];  // row r of the matrix: what this rank sends to q
        rc[q] = m[(size_t)q * W + s->rank];
        tot += rc[q];
    }
    Buf out = dev_alloc(sizeof(uint64_t) * (tot > 0 ? tot : 1), s);
    collective_a2av(s, words, sc.data(), P<void>(out), rc.data(), CAPSMI_I64, matrix_max(m));
    *nrecv = tot;
    return out;
}

// every rank's n words, concatenated in rank order (counts first, then one ALL_GATHER padded to the
// largest share, compacted on the device); synchronises
Buf gather_words(capsmi_session* s, const uint64_t* words, int64_t n, int64_t* ntotal, int64_t budget_bytes) {
    const int W = s->world;
    hipStream_t st = s->stream;
    // (count, budget) of every rank: the ranks' budgets may differ (free device memory), so each decides on
    // the smallest -- the same decision everywhere, no rank left waiting inside a collective
    Buf cnt = dev_alloc(sizeof(int64_t) * 2 * (1 + W), s);
    const int64_t mine[2] = {n, budget_bytes > 0 ? budget_bytes : INT64_MAX};
    HIP_CHECK(hipMemcpyAsync(P<int64_t>(cnt), mine, sizeof(mine), hipMemcpyHostToDevice, st));
    collective(s, CAPSMI_COLL_ALL_GATHER, P<int64_t>(cnt), P<int64_t>(cnt) + 2, 2, CAPSMI_I64);
    std::vector<int64_t> cb(2 * W), c(W);
    HIP_CHECK(hipMemcpyAsync(cb.data(), P<int64_t>(cnt) + 2, sizeof(int64_t) * 2 * W, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t mx = 0, tot = 0, budget = INT64_MAX;
    for (int q = 0; q < W; ++q) {
        c[q] = cb[2 * q];
        mx = std::max(mx, c[q]);
        tot += c[q];
        budget = std::min(budget, cb[2 * q + 1]);
    }
    if ((double)sizeof(uint64_t) * ((double)mx * W + (double)mx + (double)tot) > (double)budget) {
        *ntotal = -1;
        return Buf();
    }
    Buf pad = dev_alloc(sizeof(uint64_t) * (mx > 0 ? mx : 1), s);
    if (n > 0) HIP_CHECK(hipMemcpyAsync(P<void>(pad), words, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, st));
    Buf all = dev_alloc(sizeof(uint64_t) * (size_t)(mx > 0 ? mx : 1) * W, s);
    if (mx > 0) collective(s, CAPSMI_COLL_ALL_GATHER, P<void>(pad), P<void>(all), mx, CAPSMI_I64);
    Buf out = dev_alloc(sizeof(uint64_t) * (tot > 0 ? tot : 1), s);
    int64_t at = 0;
    for (int q = 0; q < W; ++q) {
        if (c[q] > 0)
            HIP_CHECK(hipMemcpyAsync(P<uint64_t>(out) + at, P<uint64_t>(all) + (size_t)q * mx, sizeof(uint64_t) * c[q],
                                     hipMemcpyDeviceToDevice, st));
        at += c[q];
    }
    *ntotal = tot;
    return out;
}

// ---- row exchanges of the generic operators over partitioned tables (Spark's Exchange) ------------
namespace {
capsmi_table* new_table(capsmi_session* s, int64_t nrows) {
    auto* t = new capsmi_table();
    t->sess = s;
    t->nrows = nrows;
    return t;
}

}  // namespace

namespace {
// per column of t: whether any rank's rows carry a validity buffer (one MAX all-reduce of the flags)
std::vector<bool> agreed_validity(capsmi_session* s, const capsmi_table* t) {
    const size_t nc = t->cols.size();
    std::vector<bool> out(nc, false);
    if (nc == 0) return out;
    std::vector<int64_t> h(nc);
    for (size_t i = 0; i < nc; ++i) h[i] = t->cols[i].valid ? 1 : 0;
    Buf f = dev_alloc(sizeof(int64_t) * nc, s);
    HIP_CHECK(hipMemcpyAsync(P<int64_t>(f), h.data(), sizeof(int64_t) * nc, hipMemcpyHostToDevice, s->stream));
    collective(s, CAPSMI_COLL_ALL_REDUCE_MAX, P<int64_t>(f), P<int64_t>(f), (int64_t)nc, CAPSMI_I64);
    HIP_CHECK(hipMemcpyAsync(h.data(), P<int64_t>(f), sizeof(int64_t) * nc, hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    for (size_t i = 0; i < nc; ++i) out[i] = h[i] != 0;
    return out;
}

// a list column of n rows over (lengths, values): row r holds list r (null rows: empty lists, valid 0)
Column list_column(capsmi_session* s, const Column& like, const Buf& lens, int64_t n, const Buf& values,
                   int64_t nvalues, const Buf& valid) {
    auto L = std::make_shared<ListStore>();
    L->elem = like.list->elem;
    L->nlists = n;
    L->nvalues = nvalues;
    L->offsets = dev_alloc(sizeof(int64_t) * (n + 1), s);
    exclusive_scan_i64(P<int64_t>(lens), P<int64_t>(L->offsets), n, s);
    L->values = values;
    Column x;
    x.name = like.name;
    x.type = like.type;
    x.data = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    iota_i64(P<int64_t>(x.data), 0, n, s->stream);
    x.valid = valid;
    x.list = L;
    return x;
}
}  // namespace

// Rows of t to the rank dest[r] (low byte; 0xFF: dropped): one stable 8-bit radix pass orders the row
// indices by destination, every column is gathered in that order and exchanged (one ALL_TO_ALL_V per
// column, validity as a word column).  Returns this rank's received rows, rank-major, same schema.
capsmi_table* exchange_rows(capsmi_session* s, const capsmi_table* t, uint64_t* dest) {
    hipStream_t st = s->stream;
    const int W = s->world;
    REQUIRE(W >= 1 && W < 255, CAPSMI_ERR_UNSUPPORTED, "exchange: at most 254 ranks");
    const int64_t n = t->nrows;
    // validity buffers depend on the data (read_csv allocates one only where a rank's rows hold a null):
    // the ranks agree on which columns carry one, so every rank issues the same collectives
    const std::vector<bool> nullable = agreed_validity(s, t);
    Buf idx = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    iota_i64(P<int64_t>(idx), 0, n, st);
    radix_sort_digits(s, dest, P<int64_t>(idx), n, {0});
    Buf cnt = dev_alloc(sizeof(int64_t) * (W + (size_t)W * W), s);
    int64_t* mine = P<int64_t>(cnt);
    if (n > 0) hipLaunchKernelGGL(k_dest_counts, dim3(1), dim3(256), 0, st, dest, n, W, mine);
    else HIP_CHECK(hipMemsetAsync(mine, 0, sizeof(int64_t) * W, st));
    HIP_CHECK(hipGetLastError());
    collective(s, CAPSMI_COLL_ALL_GATHER, mine, mine + W, W, CAPSMI_I64);
    std::vector<int64_t> mat((size_t)W * W);
    int64_t mat_max = 0;
    HIP_CHECK(hipMemcpyAsync(mat.data(), mine + W, sizeof(int64_t) * mat.size(), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    std::vector<int64_t> sc(W), rc(W);
    int64_t nsend = 0, nrecv = 0;
    for (int q = 0; q < W; ++q) {
        sc[q] = mat[(size_t)s->rank * W + q];
        rc[q] = mat[(size_t)q * W + s->rank];
        nsend += sc[q];
        nrecv += rc[q];
    }
    mat_max = matrix_max(mat);
    auto* o = new_table(s, nrecv);
    Buf tmp = dev_alloc(sizeof(int64_t) * (nsend > 0 ? nsend : 1), s);
    Buf rs;  // list columns: the W + 1 starts of the destination segments of the ordered rows
    for (size_t ci = 0; ci < t->cols.size(); ++ci) {
        const Column& c = t->cols[ci];
        if (is_list_type(c.type)) {  // lengths with the rows, then the values with per-rank value counts
            REQUIRE(c.list, CAPSMI_ERR_INTERNAL, "list column without a store");
            if (!rs) {
                rs = dev_alloc(sizeof(int64_t) * (W + 1), s);
                std::vector<int64_t> h(W + 1, 0);
                for (int q = 0; q < W; ++q) h[q + 1] = h[q] + sc[q];
                HIP_CHECK(hipMemcpyAsync(P<int64_t>(rs), h.data(), sizeof(int64_t) * (W + 1), hipMemcpyHostToDevice, st));
            }
            const ListStore& L = *c.list;
            Buf lens = dev_alloc(sizeof(int64_t) * (nsend + 1), s), voff = dev_alloc(sizeof(int64_t) * (nsend + 1), s);
            if (nsend > 0)
                hipLaunchKernelGGL(k_list_lens, dim3(grid_for(nsend)), dim3(256), 0, st, c.d(), c.v(),
                                   P<int64_t>(L.offsets), P<int64_t>(idx), nsend, P<int64_t>(lens));
            exclusive_scan_i64(P<int64_t>(lens), P<int64_t>(voff), nsend, s);
            Buf vc = dev_alloc(sizeof(int64_t) * (W + (size_t)W * W), s);
            hipLaunchKernelGGL(k_seg_values, dim3(1), dim3(256), 0, st, P<int64_t>(voff), P<int64_t>(rs), W, P<int64_t>(vc));
            HIP_CHECK(hipGetLastError());
            collective(s, CAPSMI_COLL_ALL_GATHER, P<int64_t>(vc), P<int64_t>(vc) + W, W, CAPSMI_I64);
            std::vector<int64_t> vm((size_t)W * W), vs(W), vr(W);
            HIP_CHECK(hipMemcpyAsync(vm.data(), P<int64_t>(vc) + W, sizeof(int64_t) * vm.size(), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            int64_t vsend = 0, vrecv = 0;
            for (int q = 0; q < W; ++q) {
                vs[q] = vm[(size_t)s->rank * W + q];
                vr[q] = vm[(size_t)q * W + s->rank];
                vsend += vs[q];
                vrecv += vr[q];
            }
            Buf packed = dev_alloc(sizeof(int64_t) * (vsend > 0 ? vsend : 1), s);
            if (nsend > 0)
                hipLaunchKernelGGL(k_list_pack, dim3(grid_for(nsend)), dim3(256), 0, st, c.d(), c.v(), P<int64_t>(L.offsets),
                                   P<int64_t>(L.values), P<int64_t>(idx), nsend, P<int64_t>(voff), P<int64_t>(packed));
            HIP_CHECK(hipGetLastError());
            Buf rlens = dev_alloc(sizeof(int64_t) * (nrecv + 1), s), rvals = dev_alloc(sizeof(int64_t) * (vrecv > 0 ? vrecv : 1), s);
            collective_a2av(s, P<int64_t>(lens), sc.data(), P<int64_t>(rlens), rc.data(), CAPSMI_I64, mat_max);
            collective_a2av(s, P<int64_t>(packed), vs.data(), P<int64_t>(rvals), vr.data(), CAPSMI_I64, matrix_max(vm));
            Buf valid;
            if (nullable[ci]) {
                Buf vw = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s), rw = dev_alloc(sizeof(int64_t) * (nrecv > 0 ? nrecv : 1), s);
                if (n > 0) hipLaunchKernelGGL(k_valid_to_words, dim3(grid_for(n)), dim3(256), 0, st, c.v(), n, P<int64_t>(vw));
                gather_col(P<int64_t>(vw), nullptr, P<int64_t>(idx), nsend, P<int64_t>(tmp), nullptr, st);
                collective_a2av(s, P<int64_t>(tmp), sc.data(), P<int64_t>(rw), rc.data(), CAPSMI_I64, mat_max);
                valid = dev_alloc(nrecv > 0 ? nrecv : 1, s);
                if (nrecv > 0)
                    hipLaunchKernelGGL(k_words_to_valid, dim3(grid_for(nrecv)), dim3(256), 0, st, P<int64_t>(rw), nrecv,
                                       P<uint8_t>(valid));
                HIP_CHECK(hipGetLastError());
            }
            o->cols.push_back(list_column(s, c, rlens, nrecv, rvals, vrecv, valid));
            continue;
        }
        Column x;
        x.name = c.name;
        x.type = c.type;
        x.data = dev_alloc(sizeof(int64_t) * (nrecv > 0 ? nrecv : 1), s);
        gather_col(c.d(), nullptr, P<int64_t>(idx), nsend, P<int64_t>(tmp), nullptr, st);
        collective_a2av(s, P<int64_t>(tmp), sc.data(), P<int64_t>(x.data), rc.data(), CAPSMI_I64, mat_max);
        if (nullable[ci]) {
            Buf vw = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s), rw = dev_alloc(sizeof(int64_t) * (nrecv > 0 ? nrecv : 1), s);
            if (n > 0)
                hipLaunchKernelGGL(k_valid_to_words, dim3(grid_for(n)), dim3(256), 0, st, c.v(), n, P<int64_t>(vw));
            gather_col(P<int64_t>(vw), nullptr, P<int64_t>(idx), nsend, P<int64_t>(tmp), nullptr, st);
            collective_a2av(s, P<int64_t>(tmp), sc.data(), P<int64_t>(rw), rc.data(), CAPSMI_I64, mat_max);
            x.valid = dev_alloc(nrecv > 0 ? nrecv : 1, s);
            if (nrecv > 0)
                hipLaunchKernelGGL(k_words_to_valid, dim3(grid_for(nrecv)), dim3(256), 0, st, P<int64_t>(rw), nrecv,
                                   P<uint8_t>(x.valid));
            HIP_CHECK(hipGetLastError());
        }
        o->cols.push_back(std::move(x));
    }
    o->partitioned = true;
    return o;
}

// Rows of t hash-partitioned by its key columns `keys` (HashPartitioning): equal keys meet on one rank.
// as_f64 (may be empty): per key 1 = a Long key hashed as the double it widens to, 2 = a Double key.
// null_local: rows with a null key stay on this rank (they match nothing), else nulls hash as one value.
capsmi_table* exchange_by_keys(capsmi_session* s, const capsmi_table* t, const std::vector<int>& keys,
                               const std::vector<int>& as_f64, bool null_local) {
    REQUIRE(keys.size() <= 8, CAPSMI_ERR_UNSUPPORTED, "exchange on more than 8 key columns");
    KeyHashCols k{};
    k.n = (int)keys.size();
    for (size_t i = 0; i < keys.size(); ++i) {
        const Column& c = t->cols.at(keys[i]);
        k.d[i] = c.d();
        k.v[i] = c.v();
        k.as_f64[i] = i < as_f64.size() ? as_f64[i] : (c.type == CAPSMI_F64 ? 2 : 0);
    }
    const int64_t n = t->nrows;
    Buf dest = dev_alloc(sizeof(uint64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_key_dest, dim3(grid_for(n)), dim3(256), 0, s->stream, k, n, s->world,
                           null_local ? s->rank : -1, P<uint64_t>(dest));
    HIP_CHECK(hipGetLastError());
    return exchange_rows(s, t, P<uint64_t>(dest));
}

// this rank's share of a table every rank holds whole (rows r with r mod world = rank)
capsmi_table* slice_rows(capsmi_session* s, const capsmi_table* t) {
    const int64_t n = t->nrows;
    Buf dest = dev_alloc(sizeof(uint64_t) * (n > 0 ? n : 1), s);
    if (n > 0)
        hipLaunchKernelGGL(k_row_dest_slice, dim3(grid_for(n)), dim3(256), 0, s->stream, n, s->rank, s->world,
                           P<uint64_t>(dest));
    HIP_CHECK(hipGetLastError());
    return exchange_rows(s, t, P<uint64_t>(dest));  // keeps its own share (sends to itself only)
}

// every rank's rows of t, concatenated in rank order (the ranks' partitions of a distributed result ->
// the whole result on every rank)
capsmi_table* gather_rows(capsmi_session* s, const capsmi_table* t) {
    hipStream_t st = s->stream;
    const int64_t n = t->nrows;
    const std::vector<bool> nullable = agreed_validity(s, t);  // the same collectives on every rank
    int64_t tot = 0;
    std::vector<std::pair<Buf, Buf>> cols;
    std::vector<std::pair<Buf, int64_t>> lvals(t->cols.size());  // list columns: gathered values
    for (size_t ci = 0; ci < t->cols.size(); ++ci) {
        const Column& c = t->cols[ci];
        Buf d, v;
        if (is_list_type(c.type)) {  // gathered lengths (as the column data for now) and values
            REQUIRE(c.list, CAPSMI_ERR_INTERNAL, "list column without a store");
            const ListStore& L = *c.list;
            Buf lens = dev_alloc(sizeof(int64_t) * (n + 1), s), voff = dev_alloc(sizeof(int64_t) * (n + 1), s);
            if (n > 0)
                hipLaunchKernelGGL(k_list_lens, dim3(grid_for(n)), dim3(256), 0, st, c.d(), c.v(), P<int64_t>(L.offsets),
                                   (const int64_t*)nullptr, n, P<int64_t>(lens));
            exclusive_scan_i64(P<int64_t>(lens), P<int64_t>(voff), n, s);
            const int64_t nv = read_scalar(s, P<int64_t>(voff) + n);
            Buf packed = dev_alloc(sizeof(int64_t) * (nv > 0 ? nv : 1), s);
            if (n > 0)
                hipLaunchKernelGGL(k_list_pack, dim3(grid_for(n)), dim3(256), 0, st, c.d(), c.v(), P<int64_t>(L.offsets),
                                   P<int64_t>(L.values), (const int64_t*)nullptr, n, P<int64_t>(voff), P<int64_t>(packed));
            HIP_CHECK(hipGetLastError());
            int64_t tv = 0;
            lvals[ci] = {gather_words(s, P<uint64_t>(packed), nv, &tv), 0};
            lvals[ci].second = tv;
            d = gather_words(s, P<uint64_t>(lens), n, &tot);
        } else {
            d = gather_words(s, reinterpret_cast<const uint64_t*>(c.d()), n, &tot);
        }
        if (nullable[ci]) {
            Buf vw = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
            if (n > 0) hipLaunchKernelGGL(k_valid_to_words, dim3(grid_for(n)), dim3(256), 0, st, c.v(), n, P<int64_t>(vw));
            HIP_CHECK(hipGetLastError());
            int64_t t2 = 0;
            Buf rw = gather_words(s, P<uint64_t>(vw), n, &t2);
            v = dev_alloc(tot > 0 ? tot : 1, s);
            if (tot > 0)
                hipLaunchKernelGGL(k_words_to_valid, dim3(grid_for(tot)), dim3(256), 0, st, P<int64_t>(rw), tot, P<uint8_t>(v));
            HIP_CHECK(hipGetLastError());
        }
        cols.push_back({d, v});
    }
    if (t->cols.empty()) {  // no columns: the row count alone
        Buf c = dev_alloc(sizeof(int64_t), s);
        fill_i64(P<int64_t>(c), n, 1, st);
        collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(c), P<int64_t>(c), 1, CAPSMI_I64);
        tot = read_scalar(s, P<int64_t>(c));
    }
    auto* o = new_table(s, tot);
    for (size_t i = 0; i < t->cols.size(); ++i) {
        if (is_list_type(t->cols[i].type)) {
            o->cols.push_back(list_column(s, t->cols[i], cols[i].first, tot, lvals[i].first, lvals[i].second,
                                          cols[i].second));
            continue;
        }
        Column x;
        x.name = t->cols[i].name;
        x.type = t->cols[i].type;
        x.data = cols[i].first;
        x.valid = cols[i].second;
        o->cols.push_back(std::move(x));
    }
    o->partitioned = false;
    return o;
}

Scramble make_scramble(int64_t lo, int64_t hi, int world) {
    REQUIRE(hi > lo && (uint64_t)(hi - lo) <= (uint64_t(1) << 30), CAPSMI_ERR_UNSUPPORTED,
            "distributed graph: the id domain must hold 1 .. 2^30 ids");
    REQUIRE(world >= 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "world size");
    Scramble sc;
    sc.kbits = 5;
    while ((int64_t(1) << sc.kbits) < hi - lo) ++sc.kbits;
    sc.mul = kScrambleMul;
    uint64_t inv = kScrambleMul;  // Newton: each step doubles the correct low bits (3 -> 6 -> ... -> 96)
    for (int i = 0; i < 5; ++i) inv *= 2 - kScrambleMul * inv;
    sc.mul_inv = inv;
    sc.lo = lo;
    sc.hi = hi;
    const int64_t words = (int64_t(1) << sc.kbits) / 32;
    sc.slice_words = (words + world - 1) / world;
    sc.n = (int64_t)world * 32 * sc.slice_words;
    return sc;
}

void scramble_ids(capsmi_session* s, const Scramble& sc, const int64_t* in, int64_t n, int64_t* out, int64_t own_lo,
                  int64_t own_hi, unsigned long long* bad) {
    if (n <= 0) return;
    const uint64_t mask = (uint64_t(1) << sc.kbits) - 1;
    hipLaunchKernelGGL(k_scramble, dim3(grid_for(n)), dim3(256), 0, s->stream, in, n, sc.lo, sc.hi, sc.mul, mask,
                       own_lo, own_hi, out, bad);
    HIP_CHECK(hipGetLastError());
}

void unscramble_ids(capsmi_session* s, const DenseIds& d, int64_t* v, int64_t n) {
    REQUIRE(d.scrambled, CAPSMI_ERR_INTERNAL, "unscramble of a non-scrambled domain");
    if (n <= 0) return;
    hipLaunchKernelGGL(k_unscramble, dim3(grid_for(n)), dim3(256), 0, s->stream, v, n, d.lo, d.mul_inv,
                       (uint64_t(1) << d.kbits) - 1);
    HIP_CHECK(hipGetLastError());
}

void owned_flags(capsmi_session* s, const Scramble& sc, const int64_t* in, int64_t n, int64_t own_lo, int64_t own_hi,
                 uint8_t* flags) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_owned_flags, dim3(grid_for(n)), dim3(256), 0, s->stream, in, n, sc.lo, sc.hi, sc.mul,
                       (uint64_t(1) << sc.kbits) - 1, own_lo, own_hi, flags);
    HIP_CHECK(hipGetLastError());
}

}  // namespace capsmi

using namespace capsmi;

namespace {

#define D_BEGIN try {
#define D_END                                                   \
    }                                                           \
    catch (const capsmi::Error& e) {                            \
        set_last_error(e.what());                               \
        return e.code;                                          \
    }                                                           \
    catch (const std::bad_alloc&) {                             \
        set_last_error("host allocation failed");               \
        return CAPSMI_ERR_OUT_OF_MEMORY;                        \
    }                                                           \
    catch (const std::exception& e) {                           \
        set_last_error(e.what());                               \
        return CAPSMI_ERR_INTERNAL;                             \
    }                                                           \
    return CAPSMI_OK;

void need(const void* p, const char* what) {
    REQUIRE(p != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("null argument: ") + what);
}

Column key_column(capsmi_session* s, int64_t rows) {
    Column c;
    c.type = CAPSMI_I64;
    c.data = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), s);
    return c;
}

}  // namespace

extern "C" {

capsmi_status capsmi_session_set_ranks(capsmi_session* s, int32_t rank, int32_t world, capsmi_collective_fn fn,
                                       void* ctx) {
    D_BEGIN
    need(s, "session");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, CAPSMI_ERR_ILLEGAL_ARGUMENT, "rank / world");
    REQUIRE(world == 1 || fn != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, "a multi-rank session needs a collective");
    s->rank = rank;
    s->world = world;
    s->coll = fn;
    s->coll_ctx = ctx;
    D_END
}

capsmi_status capsmi_graph_distribute(capsmi_session* s, int64_t id_lo, int64_t id_hi, int32_t nnodes,
                                      capsmi_table* const* nodes, int32_t node_mode, int32_t nrels,
                                      capsmi_table* const* rels, int32_t rel_mode) {
    D_BEGIN
    need(s, "session");
    REQUIRE(nnodes >= 0 && nrels >= 0 && (nnodes == 0 || nodes) && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "entity table arrays");
    REQUIRE(node_mode == CAPSMI_NODES_REPLICATED || node_mode == CAPSMI_NODES_OWNED, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "node mode");
    REQUIRE(rel_mode == CAPSMI_RELS_BY_SOURCE || rel_mode == CAPSMI_RELS_BY_TARGET, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "relationship mode");
    HIP_CHECK(hipSetDevice(s->device));
    const Scramble sc = make_scramble(id_lo, id_hi, s->world);
    // the routes run on the padded scrambled domain (whole word slices per rank): refuse here, not at
    // every later query, a window whose padding takes it past the 2^30 ids the fused kernels address
    REQUIRE(sc.n <= (int64_t(1) << 30), CAPSMI_ERR_UNSUPPORTED,
            "distributed graph: the id domain padded to " + std::to_string(s->world) + " whole word slices holds " +
                std::to_string(sc.n) + " ids, above 2^30");
    const int64_t own_lo = (int64_t)s->rank * 32 * sc.slice_words, own_hi = own_lo + 32 * sc.slice_words;
    Buf bad = dev_alloc(2 * sizeof(unsigned long long), s);
    HIP_CHECK(hipMemsetAsync(P<void>(bad), 0, 2 * sizeof(unsigned long long), s->stream));
    struct Pending {
        capsmi_table* t;
        Column a, b;  // node: did; relationship: dsrc, ddst
    };
    std::vector<Pending> work;
    auto keys = [&](capsmi_table* t, int kind) {
        need(t, "entity table");
        REQUIRE(t->sess == s, CAPSMI_ERR_ILLEGAL_ARGUMENT, "table of another session");
        materialize(t);
        REQUIRE(t->entity && t->entity->kind == kind, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                kind == 1 ? "capsmi_graph_distribute: nodes must be registered node tables (capsmi_node_table)"
                          : "capsmi_graph_distribute: rels must be registered relationship tables (capsmi_rel_table)");
        REQUIRE(!t->dense || t->shard, CAPSMI_ERR_UNSUPPORTED, "a compacted table cannot also be distributed");
        Pending p{t, key_column(s, t->nrows), key_column(s, t->nrows)};
        const EntityInfo& e = *t->entity;
        if (kind == 1) {
            const bool owned = node_mode == CAPSMI_NODES_OWNED;
            scramble_ids(s, sc, t->cols[e.id].d(), t->nrows, P<int64_t>(p.a.data), owned ? own_lo : 0, owned ? own_hi : 0,
                         P<unsigned long long>(bad));
        } else {
            const bool by_src = rel_mode == CAPSMI_RELS_BY_SOURCE;
            scramble_ids(s, sc, t->cols[e.src].d(), t->nrows, P<int64_t>(p.a.data), by_src ? own_lo : 0,
                         by_src ? own_hi : 0, P<unsigned long long>(bad));
            scramble_ids(s, sc, t->cols[e.dst].d(), t->nrows, P<int64_t>(p.b.data), by_src ? 0 : own_lo,
                         by_src ? 0 : own_hi, P<unsigned long long>(bad));
        }
        work.push_back(std::move(p));
    };
    for (int i = 0; i < nnodes; ++i) keys(nodes[i], 1);
    for (int i = 0; i < nrels; ++i) keys(rels[i], 2);
    unsigned long long h[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(h, P<void>(bad), sizeof(h), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    REQUIRE(h[0] == 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::to_string(h[0]) + " ids outside the distributed graph's domain [" + std::to_string(id_lo) + ", " +
                std::to_string(id_hi) + ")");
    REQUIRE(h[1] == 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::to_string(h[1]) + " rows of this rank's shard are owned by another rank (capsmi_owned_rows)");
    auto dom = std::make_shared<DenseIds>();
    dom->n = sc.n;
    dom->scrambled = true;
    dom->kbits = sc.kbits;
    dom->mul = sc.mul;
    dom->mul_inv = sc.mul_inv;
    dom->lo = id_lo;
    for (Pending& p : work) {
        auto sh = std::make_shared<Shard>();
        sh->kind = p.t->entity->kind;
        sh->mode = sh->kind == 1 ? node_mode : rel_mode;
        sh->rank = s->rank;
        sh->world = s->world;
        sh->slice_words = sc.slice_words;
        p.t->dense = dom;
        if (sh->kind == 1) {
            p.t->did = p.a;
        } else {
            p.t->dsrc = p.a;
            p.t->ddst = p.b;
        }
        if (sh->kind == 1 && id_hi - id_lo == sc.n) {
            // coverage (Shard::covers): this shard's rows and repeated ids over the domain, summed over the
            // ranks for OWNED shards (an id's rows all live on its owner, so repeats are rank-local)
            capsmi_bitmap bm;
            bm.sess = s;
            bm.lo = 0;
            bm.hi = sc.n;
            bm.nwords = sc.n / 32;
            bm.words = dev_alloc(sizeof(uint32_t) * (size_t)bm.nwords, s);
            HIP_CHECK(hipMemsetAsync(P<void>(bm.words), 0, sizeof(uint32_t) * (size_t)bm.nwords, s->stream));
            Buf cnt = dev_alloc(3 * sizeof(int64_t), s);
            HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, 3 * sizeof(int64_t), s->stream));
            bitmap_add_rows(&bm, P<int64_t>(p.a.data), nullptr, nullptr, p.t->nrows, P<int64_t>(cnt));
            fill_i64(P<int64_t>(cnt), p.t->nrows, 1, s->stream);  // (rows, repeats)
            if (node_mode == CAPSMI_NODES_OWNED && (s->world > 1 || s->coll))
                collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(cnt), P<int64_t>(cnt), 2, CAPSMI_I64);
            int64_t rc[2];
            HIP_CHECK(hipMemcpyAsync(rc, P<void>(cnt), sizeof(rc), hipMemcpyDeviceToHost, s->stream));
            HIP_CHECK(hipStreamSynchronize(s->stream));
            sh->covers = rc[0] == sc.n && rc[1] == 0;
        }
        p.t->shard = sh;
        p.t->partitioned = s->world > 1 && !(sh->kind == 1 && node_mode == CAPSMI_NODES_REPLICATED);
        p.t->layouts.clear();
        p.t->in_src = p.t->in_dst = Column();
        p.t->in_rows = 0;
        // The complement shard, by one exchange (every rank takes part, in table order), kept with the shard:
        // BY_SOURCE, the relationships into this rank's owned ids from other ranks' sources; BY_TARGET, the
        // relationships out of its owned ids into other ranks' targets.  With it a rank holds every
        // relationship incident to an owned id exactly once (the owned-middle routes: count(*), undirected,
        // var-length)
        if (sh->kind == 2 && (s->world > 1 || s->coll)) {
            const int64_t m = p.t->nrows;
            Buf dest = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s), w = dev_alloc(sizeof(uint64_t) * (m > 0 ? m : 1), s);
            if (m > 0)
                hipLaunchKernelGGL(k_in_words, dim3(grid_for(m)), dim3(256), 0, s->stream, P<int64_t>(p.a.data),
                                   P<int64_t>(p.b.data), m, 32 * sc.slice_words, s->rank,
                                   s->world, rel_mode == CAPSMI_RELS_BY_TARGET ? 1 : 0, P<uint64_t>(dest),
                                   P<uint64_t>(w));
            HIP_CHECK(hipGetLastError());
            int64_t nin = 0;
            Buf got = exchange_words(s, P<uint64_t>(dest), P<uint64_t>(w), m, &nin);
            p.t->in_src = key_column(s, nin);
            p.t->in_dst = key_column(s, nin);
            if (nin > 0)
                hipLaunchKernelGGL(k_unpack_words, dim3(grid_for(nin)), dim3(256), 0, s->stream, P<uint64_t>(got), nin,
                                   P<int64_t>(p.t->in_src.data), P<int64_t>(p.t->in_dst.data));
            HIP_CHECK(hipGetLastError());
            p.t->in_rows = nin;
        }
    }
    D_END
}

capsmi_status capsmi_owned_rows(capsmi_session* s, capsmi_table* t, const char* col, int64_t id_lo, int64_t id_hi,
                                capsmi_table** out) {
    D_BEGIN
    need(s, "session");
    need(t, "table");
    need(col, "column");
    need(out, "out");
    HIP_CHECK(hipSetDevice(s->device));
    materialize(t);
    const int c = t->find(col);
    REQUIRE(c >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("no column named '") + col + "'");
    REQUIRE(t->cols[c].type == CAPSMI_I64 && !t->cols[c].valid, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string("owner column '") + col + "' must be a non-null Long column");
    const Scramble sc = make_scramble(id_lo, id_hi, s->world);
    const int64_t own_lo = (int64_t)s->rank * 32 * sc.slice_words, own_hi = own_lo + 32 * sc.slice_words;
    Buf flags = dev_alloc(t->nrows > 0 ? t->nrows : 1, s);
    owned_flags(s, sc, t->cols[c].d(), t->nrows, own_lo, own_hi, P<uint8_t>(flags));
    Buf idx;
    const int64_t n = flags_to_indices(s, P<uint8_t>(flags), t->nrows, idx);
    auto* o = new capsmi_table();
    o->sess = s;
    o->nrows = n;
    for (const Column& x : t->cols) {
        Column y;
        y.name = x.name;
        y.type = x.type;
        y.list = x.list;
        y.data = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
        if (x.valid) y.valid = dev_alloc(n > 0 ? n : 1, s);
        gather_col(x.d(), x.v(), P<int64_t>(idx), n, P<int64_t>(y.data), P<uint8_t>(y.valid), s->stream);
        o->cols.push_back(std::move(y));
    }
    *out = o;
    D_END
}

capsmi_status capsmi_id_owner(int64_t id_lo, int64_t id_hi, int32_t world, int64_t id, int32_t* owner,
                              int64_t* dense_id) {
    D_BEGIN
    const Scramble sc = make_scramble(id_lo, id_hi, world);
    REQUIRE(id >= id_lo && id < id_hi, CAPSMI_ERR_ILLEGAL_ARGUMENT, "id outside the domain");
    const int64_t d = (int64_t)(((uint64_t)(id - id_lo) * sc.mul) & ((uint64_t(1) << sc.kbits) - 1));
    if (owner) *owner = (int32_t)(d / (32 * sc.slice_words));
    if (dense_id) *dense_id = d;
    D_END
}

capsmi_status capsmi_table_partitioned(const capsmi_table* t, int32_t* out) {
    D_BEGIN
    need(t, "table");
    need(out, "out");
    materialize(const_cast<capsmi_table*>(t));
    *out = t->partitioned ? 1 : 0;
    D_END
}

}  // extern "C"
