/* oracle_san.c -- the oracle's C restatement (oracle/rmat.c, oracle/closed.c) under AddressSanitizer and
 * UndefinedBehaviorSanitizer: every closed form against binding enumeration on seeded random
 * multigraphs (self-loops, multi-edges, node filters, empty graphs) and on R-MAT scale 8, single- and
 * multi-threaded.  Test infrastructure: built and run by tests/test_sanitizers.py, exit status 0 = all equal. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void orc_rmat_edges(int scale, int pa, int pb, int pc, uint64_t seed, int64_t e_begin, int64_t e_end, int64_t* src,
                    int64_t* dst);
int orc_two_hop_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                          const uint8_t* b_ok, const uint8_t* c_ok, int64_t* out_rows, int64_t* out_distinct,
                          int64_t* group_rows, int64_t* group_distinct, int nthreads);
int orc_two_hop_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                            const uint8_t* b_ok, const uint8_t* c_ok, int64_t* out_rows, int64_t* out_distinct);
int orc_two_hop_closed_form_mt(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                               const uint8_t* b_ok, const uint8_t* c_ok, int64_t* out_rows, int64_t* out_distinct,
                               int nthreads);
int orc_two_hop_undirected_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                                     const uint8_t* b_ok, const uint8_t* c_ok, int64_t* out_rows,
                                     int64_t* out_distinct_c, int64_t* out_distinct_a, int nthreads);
int orc_two_hop_undirected_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                                       const uint8_t* a_ok, const uint8_t* b_ok, const uint8_t* c_ok,
                                       int64_t* out_rows, int64_t* out_distinct, int nthreads);
int orc_triangle_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, int64_t* out_rows,
                           int nthreads);
int orc_triangle_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* n_ok,
                             int64_t* out_rows, int nthreads);
int orc_var_length_count(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                         const uint8_t* b_ok, int lo, int hi, int64_t* group_rows, int64_t* out_rows, int nthreads);
int orc_var_length_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                               const uint8_t* b_ok, int lo, int hi, int64_t* group_rows, int64_t* out_rows,
                               int nthreads);
void orc_expand_filter(int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok, const uint8_t* b_ok,
                       int64_t* out_rows, uint64_t* out_sum, uint64_t* out_xor);

static uint64_t rng_state = 0x9E3779B97F4A7C15ULL;
static uint64_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}

static int fails = 0;
#define EQ(what, x, y)                                                                                   \
    do {                                                                                                 \
        if ((x) != (y)) {                                                                                \
            fprintf(stderr, "case %d: %s: %lld != %lld\n", cs, what, (long long)(x), (long long)(y));     \
            ++fails;                                                                                     \
        }                                                                                                \
    } while (0)

static void check(int cs, int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a,
                  const uint8_t* b, const uint8_t* c, int threads) {
    int64_t r1 = 0, d1 = 0, r2 = 0, d2 = 0, r3 = 0, d3 = 0;
    int64_t* gr = calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t* gd = calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t* g1 = calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t* g2 = calloc((size_t)(n ? n : 1), sizeof(int64_t));
    EQ("enumerate rc", orc_two_hop_enumerate(n, m, src, dst, a, b, c, &r1, &d1, gr, gd, threads), 0);
    EQ("closed rc", orc_two_hop_closed_form(n, m, src, dst, a, b, c, &r2, &d2), 0);
    EQ("closed_mt rc", orc_two_hop_closed_form_mt(n, m, src, dst, a, b, c, &r3, &d3, threads), 0);
    EQ("2-hop rows", r1, r2);
    EQ("2-hop rows mt", r1, r3);
    EQ("2-hop distinct", d1, d2);
    EQ("2-hop distinct mt", d1, d3);
    int64_t ur = 0, udc = 0, uda = 0, ur2 = 0, ud2 = 0;
    EQ("und enumerate rc", orc_two_hop_undirected_enumerate(n, m, src, dst, a, b, c, &ur, &udc, &uda, threads), 0);
    EQ("und closed rc", orc_two_hop_undirected_closed_form(n, m, src, dst, a, b, c, &ur2, &ud2, threads), 0);
    EQ("undirected rows", ur, ur2);
    EQ("undirected distinct", udc, ud2);
    int64_t t1 = 0, t2 = 0;
    EQ("tri enumerate rc", orc_triangle_enumerate(n, m, src, dst, &t1, threads), 0);
    EQ("tri closed rc", orc_triangle_closed_form(n, m, src, dst, NULL, &t2, threads), 0);
    EQ("triangles", t1, t2);
    for (int lo = 1; lo <= 3; ++lo)
        for (int hi = lo; hi <= 3; ++hi) {
            int64_t v1 = 0, v2 = 0;
            memset(g1, 0, sizeof(int64_t) * (size_t)(n ? n : 1));
            memset(g2, 0, sizeof(int64_t) * (size_t)(n ? n : 1));
            EQ("varlen enumerate rc", orc_var_length_count(n, m, src, dst, a, b, lo, hi, g1, &v1, threads), 0);
            EQ("varlen closed rc", orc_var_length_closed_form(n, m, src, dst, a, b, lo, hi, g2, &v2, threads), 0);
            EQ("varlen rows", v1, v2);
            for (int64_t i = 0; i < n; ++i) EQ("varlen group", g1[i], g2[i]);
        }
    int64_t er = 0;
    uint64_t es = 0, ex = 0;
    orc_expand_filter(m, src, dst, a, b, &er, &es, &ex);
    int64_t want = 0;
    for (int64_t i = 0; i < m; ++i) want += (!a || a[src[i]]) && (!b || b[dst[i]]);
    EQ("expand rows", er, want);
    free(gr);
    free(gd);
    free(g1);
    free(g2);
}

int main(void) {
    int cs = 0;
    for (cs = 0; cs < 60; ++cs) {
        const int64_t n = 1 + (int64_t)(rnd() % 40);
        const int64_t m = (int64_t)(rnd() % 300);
        int64_t* src = malloc(sizeof(int64_t) * (size_t)(m ? m : 1));
        int64_t* dst = malloc(sizeof(int64_t) * (size_t)(m ? m : 1));
        uint8_t* a = malloc((size_t)n);
        uint8_t* b = malloc((size_t)n);
        uint8_t* c = malloc((size_t)n);
        for (int64_t i = 0; i < m; ++i) {
            src[i] = (int64_t)(rnd() % (uint64_t)n);
            dst[i] = (i % 7 == 0) ? src[i] : (int64_t)(rnd() % (uint64_t)n); /* self-loops */
        }
        for (int64_t i = 0; i < n; ++i) {
            a[i] = (uint8_t)(rnd() % 4 != 0);
            b[i] = (uint8_t)(rnd() % 5 != 0);
            c[i] = (uint8_t)(rnd() % 3 != 0);
        }
        const int filt = cs % 2;
        check(cs, n, m, src, dst, filt ? a : NULL, filt ? b : NULL, filt ? c : NULL, 1 + cs % 3);
        free(src);
        free(dst);
        free(a);
        free(b);
        free(c);
    }
    {
        const int scale = 8;
        const int64_t n = (int64_t)1 << scale, m = (int64_t)16 << scale;
        int64_t* src = malloc(sizeof(int64_t) * (size_t)m);
        int64_t* dst = malloc(sizeof(int64_t) * (size_t)m);
        orc_rmat_edges(scale, 57, 19, 19, 42, 0, m, src, dst);
        for (int64_t i = 0; i < m; ++i)
            if (src[i] < 0 || src[i] >= n || dst[i] < 0 || dst[i] >= n) {
                fprintf(stderr, "rmat edge %lld out of range\n", (long long)i);
                ++fails;
                break;
            }
        check(cs, n, m, src, dst, NULL, NULL, NULL, 4);
        free(src);
        free(dst);
    }
    printf("oracle_san: %d cases, %d mismatches\n", cs + 1, fails);
    return fails ? 1 : 0;
}
