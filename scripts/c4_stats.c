// Diagnostic (not product): wedge statistics of the degree-oriented simple graph of R-MAT s (C4).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
void orc_rmat_edges(int scale, int pa, int pb, int pc, uint64_t seed, int64_t e_begin, int64_t e_end, int64_t* src, int64_t* dst);
static int cmpu(const void* a, const void* b) { uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b; return (x > y) - (x < y); }
int main(int argc, char** argv) {
    int s = argc > 1 ? atoi(argv[1]) : 20;
    int64_t n = 1LL << s, m = 16LL << s;
    int64_t *src = malloc(8 * m), *dst = malloc(8 * m);
    orc_rmat_edges(s, 57, 19, 19, 42, 0, m, src, dst);
    uint64_t* k = malloc(8 * m);
    int64_t kk = 0;
    for (int64_t e = 0; e < m; ++e) if (src[e] != dst[e]) {
        uint64_t a = src[e] < dst[e] ? src[e] : dst[e], b = src[e] < dst[e] ? dst[e] : src[e];
        k[kk++] = (a << 32) | b;
    }
    qsort(k, kk, 8, cmpu);
    int64_t ne = 0;
    for (int64_t i = 0; i < kk; ++i) if (i == 0 || k[i] != k[i - 1]) k[ne++] = k[i];
    int64_t* deg = calloc(n, 8);
    for (int64_t i = 0; i < ne; ++i) { deg[k[i] >> 32]++; deg[k[i] & 0xffffffff]++; }
    int64_t* od = calloc(n + 1, 8);
    for (int64_t i = 0; i < ne; ++i) {
        int64_t x = k[i] >> 32, y = k[i] & 0xffffffff;
        int xf = deg[x] < deg[y] || (deg[x] == deg[y] && x < y);
        od[xf ? x : y]++;
    }
    // wedges per u: sum_{v in out(u)} od(v)
    double wbig = 0, wsmall = 0; int64_t nbig = 0, nsmall = 0, dbig = 0;
    int64_t* wv = calloc(n, 8);  // per u
    for (int64_t i = 0; i < ne; ++i) {
        int64_t x = k[i] >> 32, y = k[i] & 0xffffffff;
        int xf = deg[x] < deg[y] || (deg[x] == deg[y] && x < y);
        int64_t u = xf ? x : y, v = xf ? y : x;
        wv[u] += od[v];
    }
    // core: vertices that are the v of a big u
    char* core = calloc(n, 1);
    for (int64_t i = 0; i < ne; ++i) {
        int64_t x = k[i] >> 32, y = k[i] & 0xffffffff;
        int xf = deg[x] < deg[y] || (deg[x] == deg[y] && x < y);
        int64_t u = xf ? x : y, v = xf ? y : x;
        if (od[u] > 64) core[v] = 1;
    }
    int64_t ncore = 0, core_adj = 0, maxod = 0;
    for (int64_t u = 0; u < n; ++u) {
        if (od[u] > maxod) maxod = od[u];
        if (od[u] > 64) { nbig++; wbig += wv[u]; dbig += od[u]; }
        else if (od[u] >= 2) { nsmall++; wsmall += wv[u]; }
        if (core[u]) { ncore++; core_adj += od[u]; }
    }
    printf("s=%d ne=%lld max_out=%lld big_u=%lld (sum d %lld) small_u=%lld wedges big=%.3e small=%.3e core_v=%lld core_adj_entries=%lld (%.1f MB @4B)\n",
           s, (long long)ne, (long long)maxod, (long long)nbig, (long long)dbig, (long long)nsmall, wbig, wsmall,
           (long long)ncore, (long long)core_adj, core_adj * 4 / 1e6);
    return 0;
}
