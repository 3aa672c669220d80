// Pass-1 microbenchmark (not shipped): times k_scatter_c / k_scatter_l against a copy floor with the same
// access pattern (16-B loads of both int64 columns, packed 8-B pairs written linearly) on uniform
// random (source, target) ids over 2^26.  Build: see scripts/p1bench.sh; run on the GPU box.
#include "../cypher-for-apache-spark_amd/csrc/k_part.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace capsmi;
using namespace capsmi::part;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__global__ void k_gen(int64_t* __restrict__ a, int64_t* __restrict__ b, int64_t m, int bits) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        a[i] = (int64_t)(z & ((1ull << bits) - 1));
        b[i] = (int64_t)((z >> 32) & ((1ull << bits) - 1));
    }
}

// copy floor: same loads as pass 1, pairs written linearly with 16-B stores
template <bool NTL, bool NTS>
__global__ void __launch_bounds__(kP1Block) k_floor(const int64_t* __restrict__ src, const int64_t* __restrict__ dst,
                                                   int64_t m, uint2* __restrict__ out) {
    int64_t sr[kItems], tr[kItems];
    const int64_t stride = (int64_t)gridDim.x * kP1Tile;
    int64_t t0 = (int64_t)blockIdx.x * kP1Tile;
    typedef long long v2i64 __attribute__((ext_vector_type(2)));
    auto ld = [&](int64_t b) {
        const v2i64* sv = reinterpret_cast<const v2i64*>(src + b);
        const v2i64* dv = reinterpret_cast<const v2i64*>(dst + b);
#pragma unroll
        for (int k = 0; k < kItems / 2; ++k) {
            v2i64 a, c;
            if (NTL) {
                a = __builtin_nontemporal_load(sv + k * kP1Block + threadIdx.x);
                c = __builtin_nontemporal_load(dv + k * kP1Block + threadIdx.x);
            } else {
                a = sv[k * kP1Block + threadIdx.x];
                c = dv[k * kP1Block + threadIdx.x];
            }
            sr[2 * k] = a.x; sr[2 * k + 1] = a.y; tr[2 * k] = c.x; tr[2 * k + 1] = c.y;
        }
    };
    if (t0 < m) ld(t0);
    for (; t0 < m; t0 += stride) {
        uint4 v[kItems / 2];
#pragma unroll
        for (int k = 0; k < kItems / 2; ++k)
            v[k] = make_uint4((uint32_t)sr[2 * k], (uint32_t)tr[2 * k], (uint32_t)sr[2 * k + 1], (uint32_t)tr[2 * k + 1]);
        if (t0 + stride < m) ld(t0 + stride);
        uint4* o = reinterpret_cast<uint4*>(out + t0);
#pragma unroll
        for (int k = 0; k < kItems / 2; ++k) {
            typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
            v4u32 w = {v[k].x, v[k].y, v[k].z, v[k].w};
            v4u32* q = reinterpret_cast<v4u32*>(o) + k * kP1Block + threadIdx.x;
            if (NTS) __builtin_nontemporal_store(w, q); else *q = w;
        }
    }
}

// validation: every used chunk's pairs lie in its slice and match its histogram row; per-slice
// pair checksums (sum and xor of a mix of the pair) for comparison across kernels
__global__ void k_check(const uint2* __restrict__ pool, const unsigned long long* __restrict__ meta,
                        const uint32_t* __restrict__ chist, int64_t npool, Layout L,
                        unsigned long long* __restrict__ sums, unsigned long long* __restrict__ bad, int cs) {
    __shared__ uint32_t h[2048];
    const int64_t q = blockIdx.x;
    if (q >= npool) return;
    const uint32_t fill = (uint32_t)(meta[q] >> 32), j = (uint32_t)meta[q];
    if (!fill) return;
    for (int i = threadIdx.x; i < L.ns; i += blockDim.x) h[i] = 0;
    __syncthreads();
    unsigned long long sa = 0, sx = 0, nb = 0;
    for (uint32_t i = threadIdx.x; i < fill; i += blockDim.x) {
        const uint2 p = pool[(size_t)q * cs + i];
        if ((p.y >> L.tbits) != j) ++nb;
        atomicAdd(&h[p.x >> L.sbits], 1u);
        uint64_t z = ((uint64_t)p.x << 32 | p.y) * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        sa += z;
        sx ^= z;
    }
    __syncthreads();
    const int hw = hist_words(L.ns);
    for (int i = threadIdx.x; i < L.ns; i += blockDim.x) {
        const uint32_t v = (chist[(size_t)q * hw + (i >> 1)] >> ((i & 1) * 16)) & 0xFFFFu;
        if (v != h[i]) ++nb;
    }
    if (nb) atomicAdd(bad, nb);
    atomicAdd(&sums[2 * j], sa);
    atomicXor(&sums[2 * j + 1], sx);
}

int main(int argc, char** argv) {
    const int bits = 26;
    const int64_t m = argc > 1 ? atoll(argv[1]) : (int64_t(1) << 30);
    int dev_cus = 0;
    CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
    int64_t *src, *dst;
    CK(hipMalloc(&src, 8 * m));
    CK(hipMalloc(&dst, 8 * m));
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, src, dst, m, bits);
    Layout L;
    L.lo = 0;
    L.hi = int64_t(1) << bits;
    L.nt = 128;
    L.ns = 128;
    L.sbits = 19;
    L.tbits = 19;
    L.ncells = L.nt * L.ns;
    struct V {
        const char* name;
        const void* fn;
        int block, tile, gmul, floor;  // floor: 0 k_scatter_c, 1 copy floor, 2 k_scatter_l
    };
    const V vs[] = {
        {"sc_1024x8", (const void*)k_scatter_c<1024, 8, 4, false>, 1024, 8192, 1, 0},
        {"sl_1024x8", (const void*)k_scatter_l<1024, 8, 4>, 1024, 8192, 1, 2},
        {"sl_ntl", (const void*)k_scatter_l<1024, 8, 4, true, false>, 1024, 8192, 1, 2},
        {"sl_nts", (const void*)k_scatter_l<1024, 8, 4, false, true>, 1024, 8192, 1, 2},
        {"sl_ntl_nts", (const void*)k_scatter_l<1024, 8, 4, true, true>, 1024, 8192, 1, 2},
        {"floor", (const void*)k_floor<false, false>, 1024, 8192, 1, 1},
        {"floor_ntls", (const void*)k_floor<true, true>, 1024, 8192, 1, 1},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    int64_t npool = 1;
    for (int v = 0; v < nv; ++v) {
        const int64_t g = (int64_t)dev_cus * vs[v].gmul;
        const int64_t c = g * chunks_per_block(m, g, L.nt, vs[v].tile);
        npool = c > npool ? c : npool;
    }
    const int hw = hist_words(L.ns);
    uint2* pool;
    unsigned long long* meta;
    uint32_t* chist;
    CK(hipMalloc(&pool, sizeof(uint2) * (kCh + 1024) * (size_t)(npool + 1)));
    CK(hipMalloc(&meta, 8 * npool));
    CK(hipMalloc(&chist, 4 * hw * (size_t)npool));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 24.0 * (double)m;
    int64_t* dcount;
    CK(hipMalloc(&dcount, 8));
    for (int v = 0; v < nv; ++v) {
        const int64_t g = (int64_t)dev_cus * vs[v].gmul;
        const size_t lds = vs[v].floor == 1 ? 0 : vs[v].floor == 2 ? scatter1l_lds(L.nt, L.ns, vs[v].block, vs[v].tile) : scatter1_lds(L.nt, L.ns, vs[v].block, vs[v].tile);
        if (lds) CK(hipFuncSetAttribute(vs[v].fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        float best = 1e30f, sum = 0;
        for (int r = 0; r < 6; ++r) {
            CK(hipMemsetAsync(meta, 0, 8 * npool, 0));
            CK(hipEventRecord(e0, 0));
            if (vs[v].floor == 1) {
                void* args[] = {&src, &dst, (void*)&m, &pool};
                CK(hipLaunchKernel(vs[v].fn, dim3(g), dim3(vs[v].block), args, 0, 0));
            } else if (vs[v].floor == 2) {
                int swap = 0;
                int64_t c0 = 0;
                size_t trash = (size_t)npool * kCh;
                void* args[] = {&src, &dst, (void*)&m, &L, &swap, &c0, &trash, &pool, &meta, &chist};
                CK(hipLaunchKernel(vs[v].fn, dim3(g), dim3(vs[v].block), args, lds, 0));
            } else {
                int swap = 0;
                int64_t c0 = 0;
                size_t trash = (size_t)npool * kCh;
                void* args[] = {&src, &dst, (void*)&m, &L, &swap, &c0, &trash, &pool, &meta, &chist};
                CK(hipLaunchKernel(vs[v].fn, dim3(g), dim3(vs[v].block), args, lds, 0));
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) {
                best = ms < best ? ms : best;
                sum += ms;
            }
        }
        // check: total fill over chunk metadata == m; chunks consistent with their histograms
        unsigned long long tot = 0, nbad = 0, sig = 0;
        if (vs[v].floor != 1) {
            unsigned long long* d;
            CK(hipMalloc(&d, 8 * (2 * L.nt + 1)));
            CK(hipMemset(d, 0, 8 * (2 * L.nt + 1)));
            hipLaunchKernelGGL(k_check, dim3(npool), dim3(256), 0, 0, pool, meta, chist, npool, L, d, d + 2 * L.nt, kCh);
            std::vector<unsigned long long> hs(2 * L.nt + 1);
            CK(hipMemcpy(hs.data(), d, 8 * hs.size(), hipMemcpyDeviceToHost));
            nbad = hs[2 * L.nt];
            for (int j = 0; j < 2 * L.nt; ++j) sig = sig * 0x100000001B3ull + hs[j];
            CK(hipFree(d));
            std::vector<unsigned long long> h(npool);
            CK(hipMemcpy(h.data(), meta, 8 * npool, hipMemcpyDeviceToHost));
            for (auto x : h) tot += x >> 32;
        }
        printf("%-14s best %.3f ms avg %.3f ms  %.0f GB/s  filled=%llu bad=%llu sig=%016llx\n", vs[v].name, best,
               sum / 5, bytes / (best * 1e6), tot, nbad, sig);
        fflush(stdout);
    }
    return 0;
}
