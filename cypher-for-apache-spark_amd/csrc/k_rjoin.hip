// k_rjoin.hip -- equi-join strategies: radix-partitioned with LDS-resident partition hash tables,
// and direct-address tables for unique dense integer keys (strategy choice: api.hip join_impl).
//
// The generic Join of the Table[T] boundary (DataFrameTable.join, SparkTable.scala:205-229): inner
// and probe-side-preserving outer joins on 1..8 key columns, null keys never match.  Both sides are
// hashed to 64 bits and radix-partitioned on the top `pbits` hash bits so that one partition of the
// build side (<= kChunk rows per pass) fits an LDS table; the probe side of a partition is cut into
// tiles, so a hub key's probe rows spread over many workgroups.  A single Long key is hashed with a
// bijective mix, so equal hashes are equal keys and no key column is re-read; several keys keep a
// folded hash and equal hashes are verified against the key columns.
//   count pass: matches per probe row (outer: at least 1) -> exclusive scan -> write pass: pairs.
#include "capsmi_impl.h"

namespace capsmi {
namespace rj {

constexpr int kBlock = 256;
constexpr int kRows = 8;                   // probe rows per lane per tile
constexpr int kTile = kBlock * kRows;      // 2048 probe rows per work item
constexpr int kSlots = 4096;               // LDS table: 4096 x (8-B hash + 4-B row) = 48 KiB
constexpr int kChunk = kSlots / 2;         // build rows per table fill (load <= 1/2)

__device__ __forceinline__ uint64_t mix(uint64_t z) {  // splitmix64 finaliser: a bijection
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// h(row); ok(row) = 1 when every key is non-null
__global__ void k_keys(KeyCols k, int64_t n, uint64_t* __restrict__ h, uint8_t* __restrict__ ok) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool valid = true;
        uint64_t x = 0x243F6A8885A308D3ULL;
        for (int c = 0; c < k.n; ++c) {
            if (k.valid[c] && !k.valid[c][i]) valid = false;
            x = k.n == 1 ? (uint64_t)k.data[c][i] : mix(x ^ (uint64_t)k.data[c][i]);
        }
        if (k.n == 1) x = mix(x);
        h[i] = x;
        if (ok) ok[i] = valid ? 1 : 0;
    }
}

__global__ void k_part_offsets(const uint64_t* __restrict__ h, int64_t n, int pbits, int64_t nparts,
                               int64_t* __restrict__ off) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nparts; p += (int64_t)gridDim.x * blockDim.x) {
        if (p == nparts) { off[p] = n; continue; }
        const uint64_t lo = pbits == 0 ? 0 : (uint64_t)p << (64 - pbits);
        int64_t a = 0, b = n;
        while (a < b) {
            const int64_t mid = (a + b) >> 1;
            if (h[mid] < lo) a = mid + 1; else b = mid;
        }
        off[p] = a;
    }
}

__global__ void k_tiles(const int64_t* __restrict__ poff, const int64_t* __restrict__ boff, int64_t nparts, int outer,
                        int64_t* __restrict__ nt) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t np = poff[p + 1] - poff[p], nb = boff[p + 1] - boff[p];
        nt[p] = (nb > 0 || outer) ? (np + kTile - 1) / kTile : 0;
    }
}

__device__ __forceinline__ bool keys_equal(const KeyCols& pk, const KeyCols& bk, int64_t pr, int64_t br) {
    for (int c = 0; c < pk.n; ++c)
        if (pk.data[c][pr] != bk.data[c][br]) return false;
    return true;
}

// WRITE = false: cnt[q] = matches of probe row q (outer: max(1, .)); true: its pairs at off[q].
// q = the row's partition-sorted position: every access here is sequential and the output is in
// partition order.  (Output in probe-row order -- sequential gathers of the probe side's columns
// afterwards, for a random scatter of counts and pairs here -- measured slower at every size of
// scripts/join_bench.py and was removed in round 6.)
template <bool WRITE>
__global__ void __launch_bounds__(kBlock) k_join(const uint64_t* __restrict__ ph, const int64_t* __restrict__ prow,
                                                 const int64_t* __restrict__ poff, const uint64_t* __restrict__ bh,
                                                 const int64_t* __restrict__ brow, const int64_t* __restrict__ boff,
                                                 const int64_t* __restrict__ ipre, int64_t nparts, int64_t nitems,
                                                 KeyCols pk, KeyCols bk, int verify, int outer,
                                                 int64_t* __restrict__ cnt, const int64_t* __restrict__ off,
                                                 int64_t* __restrict__ out_p, int64_t* __restrict__ out_b) {
    __shared__ uint64_t hk[kSlots];
    __shared__ uint32_t hr[kSlots];  // 1 + build row within the chunk; 0 = empty slot
    for (int64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
        int64_t a = 0, b = nparts;  // partition of item `it`: last p with ipre[p] <= it
        while (b - a > 1) {
            const int64_t mid = (a + b) >> 1;
            if (ipre[mid] <= it) a = mid; else b = mid;
        }
        const int64_t p = a;
        const int64_t t0 = poff[p] + (it - ipre[p]) * kTile, t1 = min(t0 + kTile, poff[p + 1]);
        const int64_t b0 = boff[p], b1 = boff[p + 1];
        int64_t mine[kRows];
        uint64_t hv[kRows];
        int64_t got[kRows];
        int64_t base[kRows];
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            const int64_t i = t0 + r * kBlock + threadIdx.x;
            mine[r] = i < t1 ? i : -1;
            hv[r] = i < t1 ? ph[i] : 0;
            got[r] = 0;
            base[r] = WRITE && i < t1 ? off[i] : 0;
        }
        for (int64_t c0 = b0; c0 < b1; c0 += kChunk) {  // block-uniform
            const int64_t c1 = min(c0 + kChunk, b1);
            __syncthreads();
            for (int s = threadIdx.x; s < kSlots; s += kBlock) hr[s] = 0;
            __syncthreads();
            for (int64_t j = c0 + threadIdx.x; j < c1; j += kBlock) {
                const uint64_t x = bh[j];
                uint32_t s = (uint32_t)x & (kSlots - 1);
                while (atomicCAS(&hr[s], 0u, (uint32_t)(j - c0 + 1)) != 0u) s = (s + 1) & (kSlots - 1);
                hk[s] = x;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < kRows; ++r) {
                if (mine[r] < 0) continue;
                const uint64_t x = hv[r];
                uint32_t s = (uint32_t)x & (kSlots - 1);
                while (true) {
                    const uint32_t hrow = hr[s];
                    if (hrow == 0) break;
                    if (hk[s] == x) {
                        const int64_t bj = c0 + hrow - 1;
                        if (!verify || keys_equal(pk, bk, prow[mine[r]], brow[bj])) {
                            if (WRITE) {
                                const int64_t o = base[r] + got[r];
                                out_p[o] = prow[mine[r]];
                                out_b[o] = brow[bj];
                            }
                            ++got[r];
                        }
                    }
                    s = (s + 1) & (kSlots - 1);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            if (mine[r] < 0) continue;
            if (!WRITE) {
                cnt[mine[r]] = (outer && got[r] == 0) ? 1 : got[r];
            } else if (outer && got[r] == 0) {
                const int64_t o = base[r];
                out_p[o] = prow[mine[r]];
                out_b[o] = -1;
            }
        }
    }
}

// probe rows with a null key in an outer join: one (row, -1) pair each, after the matched pairs
__global__ void k_null_rows(const int64_t* __restrict__ rows, int64_t n, int64_t base, int64_t* __restrict__ out_p,
                            int64_t* __restrict__ out_b) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = base + i;
        out_p[o] = rows[i];
        out_b[o] = -1;
    }
}

// ---- direct-address join: unique integer build keys in a dense range ---------------------------
// slot[key - lo] = build row (int32; -1 empty); a second row for a key raises `dup`
__global__ void k_direct_build(const int64_t* __restrict__ key, const uint8_t* __restrict__ valid, int64_t n,
                               int64_t lo, int32_t* __restrict__ slot, int32_t* __restrict__ dup) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (valid && !valid[i]) continue;
        if (atomicCAS(&slot[(uint64_t)key[i] - (uint64_t)lo], -1, (int32_t)i) != -1) *dup = 1;
    }
}

// m[i] = matching build row or -1; flags[i] = m[i] >= 0 (inner joins)
__global__ void k_direct_probe(const int64_t* __restrict__ key, const uint8_t* __restrict__ valid, int64_t n,
                               int64_t lo, uint64_t range, const int32_t* __restrict__ slot, int64_t* __restrict__ m,
                               uint8_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t off = (uint64_t)key[i] - (uint64_t)lo;
        int64_t r = -1;
        if ((!valid || valid[i]) && off < range) r = slot[off];
        m[i] = r;
        if (flags) flags[i] = r >= 0 ? 1 : 0;
    }
}

inline unsigned grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1 << 16)); }

struct Side {
    Buf h, row;  // hashes sorted by partition, their rows
    int64_t n = 0;
    Buf nulls;   // rows with a null key
    int64_t nnull = 0;
};

void prepare(capsmi_session* s, const KeyCols& k, int64_t n, int pbits, Side& sd) {
    hipStream_t st = s->stream;
    bool nullable = false;
    for (int c = 0; c < k.n; ++c) nullable |= k.valid[c] != nullptr;
    Buf h = dev_alloc(sizeof(uint64_t) * (n > 0 ? n : 1), s);
    Buf ok = nullable ? dev_alloc(n > 0 ? n : 1, s) : Buf();
    if (n > 0)
        hipLaunchKernelGGL(k_keys, dim3(grid(n)), dim3(256), 0, st, k, n, P<uint64_t>(h),
                           nullable ? P<uint8_t>(ok) : nullptr);
    HIP_CHECK(hipGetLastError());
    if (!nullable) {  // every row takes part
        sd.n = n;
        sd.h = h;
        sd.row = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
        iota_i64(P<int64_t>(sd.row), 0, n, st);
    } else {
        sd.n = flags_to_indices(s, P<uint8_t>(ok), n, sd.row);
        sd.h = dev_alloc(sizeof(uint64_t) * (sd.n > 0 ? sd.n : 1), s);
        gather_col(P<int64_t>(h), nullptr, P<int64_t>(sd.row), sd.n, P<int64_t>(sd.h), nullptr, st);
        if (sd.n < n) {  // rows with a null key (outer joins emit them)
            invert_u8(P<uint8_t>(ok), P<uint8_t>(ok), n, st);
            sd.nnull = flags_to_indices(s, P<uint8_t>(ok), n, sd.nulls);
        }
    }
    // group by partition: LSD passes over the top pbits (whole 8-bit digits)
    std::vector<int> shifts;
    for (int b = 64 - ((pbits + 7) / 8) * 8; b < 64; b += 8) shifts.push_back(b);
    radix_sort_digits(s, P<uint64_t>(sd.h), P<int64_t>(sd.row), sd.n, shifts);
}

}  // namespace rj

// (probe row, build row) pairs of an equi-join; build row -1 for an unmatched / null-key probe row
// of an outer join.  Returns the number of pairs.
int64_t radix_join(capsmi_session* s, const KeyCols& bk, int64_t nb, const KeyCols& pk, int64_t np, bool outer,
                   Buf& out_p, Buf& out_b) {
    using namespace rj;
    hipStream_t st = s->stream;
    int pbits = 0;
    while (pbits < 24 && (nb >> pbits) > kChunk / 2) ++pbits;  // ~1k build rows per partition
    const int64_t nparts = int64_t(1) << pbits;
    Side B, Pr;
    prepare(s, bk, nb, pbits, B);
    prepare(s, pk, np, pbits, Pr);
    Buf offs = dev_alloc(sizeof(int64_t) * (4 * (nparts + 1)), s);
    int64_t* boff = P<int64_t>(offs);
    int64_t* poff = boff + nparts + 1;
    int64_t* ntl = poff + nparts + 1;
    int64_t* ipre = ntl + nparts + 1;
    hipLaunchKernelGGL(k_part_offsets, dim3(grid(nparts + 1)), dim3(256), 0, st, P<uint64_t>(B.h), B.n, pbits, nparts,
                       boff);
    hipLaunchKernelGGL(k_part_offsets, dim3(grid(nparts + 1)), dim3(256), 0, st, P<uint64_t>(Pr.h), Pr.n, pbits, nparts,
                       poff);
    hipLaunchKernelGGL(k_tiles, dim3(grid(nparts)), dim3(256), 0, st, poff, boff, nparts, outer ? 1 : 0, ntl);
    exclusive_scan_i64(ntl, ipre, nparts, s);
    HIP_CHECK(hipGetLastError());
    const int64_t nitems = read_scalar(s, ipre + nparts);
    const int verify = pk.n > 1 ? 1 : 0;
    const int64_t nc = Pr.n;  // counts per partition-sorted position
    Buf cnt = dev_alloc(sizeof(int64_t) * (nc > 0 ? nc : 1), s);
    // rows of partitions without build rows get no work item (inner joins): their count stays 0
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(int64_t) * (nc > 0 ? nc : 1), st));
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(nitems, (int64_t)s->num_cus * 8));
    {
        KernelTimer kt(s, "radix_join_count", (double)Pr.n * (16 + 8) + (double)B.n * 16);
        if (nitems > 0)
            hipLaunchKernelGGL(k_join<false>, dim3(g), dim3(kBlock), 0, st, P<uint64_t>(Pr.h), P<int64_t>(Pr.row), poff,
                               P<uint64_t>(B.h), P<int64_t>(B.row), boff, ipre, nparts, nitems, pk, bk, verify,
                               outer ? 1 : 0, P<int64_t>(cnt), nullptr, nullptr, nullptr);
    }
    Buf off = dev_alloc(sizeof(int64_t) * (nc + 1), s);
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(off), nc, s);
    const int64_t matched = read_scalar(s, P<int64_t>(off) + nc);
    const int64_t total = matched + (outer ? Pr.nnull : 0);
    out_p = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    out_b = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
    {
        KernelTimer kt(s, "radix_join_write", (double)Pr.n * (16 + 8) + (double)B.n * 16 + (double)total * 16);
        if (nitems > 0 && matched > 0)
            hipLaunchKernelGGL(k_join<true>, dim3(g), dim3(kBlock), 0, st, P<uint64_t>(Pr.h), P<int64_t>(Pr.row), poff,
                               P<uint64_t>(B.h), P<int64_t>(B.row), boff, ipre, nparts, nitems, pk, bk, verify,
                               outer ? 1 : 0, nullptr, P<int64_t>(off), P<int64_t>(out_p), P<int64_t>(out_b));
    }
    if (outer && Pr.nnull > 0)
        hipLaunchKernelGGL(k_null_rows, dim3(grid(Pr.nnull)), dim3(256), 0, st, P<int64_t>(Pr.nulls), Pr.nnull,
                           matched, P<int64_t>(out_p), P<int64_t>(out_b));
    HIP_CHECK(hipGetLastError());
    return total;
}

// Direct-address join for a single Long key whose build side is unique and spans a dense range
// (node ids joined with relationship endpoints -- the Expand joins): one 4-byte table read per probe
// row, output in probe-row order.  Returns false (nothing done) when the keys are not eligible.
bool direct_join(capsmi_session* s, const KeyCols& bk, int64_t nb, const KeyCols& pk, int64_t np, bool outer,
                 Buf& out_p, Buf& out_b, int64_t* total) {
    using namespace rj;
    if (bk.n != 1 || nb <= 0 || nb >= (int64_t(1) << 31)) return false;
    hipStream_t st = s->stream;
    int64_t mm[2];
    const int64_t* cols[1] = {bk.data[0]};
    minmax_i64(s, cols, 1, nb, mm);
    const uint64_t range = (uint64_t)mm[1] - (uint64_t)mm[0] + 1;
    if (mm[1] < mm[0] || range > (uint64_t)std::max<int64_t>(4 * nb, int64_t(1) << 20) || range > (uint64_t(1) << 31))
        return false;
    Buf slot = dev_alloc(sizeof(int32_t) * range, s);
    Buf dup = dev_alloc(sizeof(int32_t), s);
    HIP_CHECK(hipMemsetAsync(P<void>(slot), 0xff, sizeof(int32_t) * range, st));
    HIP_CHECK(hipMemsetAsync(P<void>(dup), 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(k_direct_build, dim3(grid(nb)), dim3(256), 0, st, bk.data[0], bk.valid[0], nb, mm[0],
                       P<int32_t>(slot), P<int32_t>(dup));
    HIP_CHECK(hipGetLastError());
    int32_t d = 0;
    HIP_CHECK(hipMemcpyAsync(&d, P<void>(dup), sizeof(d), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (d) return false;  // duplicate build keys: a hashed strategy
    Buf m = dev_alloc(sizeof(int64_t) * (np > 0 ? np : 1), s);
    Buf flags = outer ? Buf() : dev_alloc(np > 0 ? np : 1, s);
    {
        // key + match row (+ flag, + validity) per probe row, one 4-byte table entry read per probe row
        KernelTimer kt(s, "direct_join_probe", (double)np * (8 + 8 + 4 + (outer ? 0 : 1) + (pk.valid[0] ? 1 : 0)));
        if (np > 0)
            hipLaunchKernelGGL(k_direct_probe, dim3(grid(np)), dim3(256), 0, st, pk.data[0], pk.valid[0], np, mm[0],
                               range, P<int32_t>(slot), P<int64_t>(m), outer ? nullptr : P<uint8_t>(flags));
        HIP_CHECK(hipGetLastError());
    }
    if (outer) {  // every probe row once, in order
        out_p = dev_alloc(sizeof(int64_t) * (np > 0 ? np : 1), s);
        iota_i64(P<int64_t>(out_p), 0, np, st);
        out_b = m;
        *total = np;
        return true;
    }
    *total = flags_to_indices(s, P<uint8_t>(flags), np, out_p);
    out_b = dev_alloc(sizeof(int64_t) * (*total > 0 ? *total : 1), s);
    gather_col(P<int64_t>(m), nullptr, P<int64_t>(out_p), *total, P<int64_t>(out_b), nullptr, st);
    return true;
}

}  // namespace capsmi
