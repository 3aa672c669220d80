/*
 * oracle/closed.c -- closed-form CPU restatements (TEST INFRASTRUCTURE ONLY).
 *
 * Loaded only by tests/, bench.py's cpu_baseline leg, __graft_entry__.smoke() and
 * tests/golden/make_rmat_full.py.  libcapsmi.so never links or calls it.
 *
 * rmat.c enumerates bindings the way CAPS's joins emit them; this file derives the same counts
 * without enumeration so that the full BASELINE sizes (where enumeration cannot finish) get exact
 * expected values.  Each closed form is pinned against rmat.c's enumeration AND against
 * oracle/enumerate.py on the reference's golden graphs (tests/test_oracle_pins.py).
 *
 * Semantics followed:
 *   - 2-hop Expand chain, RelationalPlanner.scala:113-137, uniqueness r1 <> r2 (front-end rewrite,
 *     okapi-ir/.../parse/CypherParser.scala:64-76)
 *   - cyclic triangle with the closing ExpandInto, RelationalPlanner.scala:139-154, pairwise
 *     distinct r1, r2, r3
 *   - directed var-length with edge-distinct paths, VarLengthExpandPlanner.scala:83-136,179-180;
 *     intermediate nodes are not scanned (expand(i) joins rel scans directly, :108-136), the target
 *     is (addTargetOps :219-230)
 *   - count(*) / count(DISTINCT x): SparkTable.scala:148-158
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

uint64_t orc_splitmix64(uint64_t x);

#define OK(bm, v) ((bm) == NULL || (bm)[v])

static void set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
}

/* C2 node tables: person[id] = splitmix64(id) & 3 != 0;
 * adult[id] = person && 18 <= age < 65 with age = splitmix64(seed ^ id) % 100. */
void orc_c2_masks(int64_t n, uint64_t seed, uint8_t* person, uint8_t* adult) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int p = (orc_splitmix64((uint64_t)i) & 3ULL) != 0;
        const int64_t age = (int64_t)(orc_splitmix64(seed ^ (uint64_t)i) % 100ULL);
        person[i] = (uint8_t)p;
        adult[i] = (uint8_t)(p && age >= 18 && age < 65);
    }
}

/* C3 closed form, multi-threaded (the same derivation as rmat.c orc_two_hop_closed_form):
 *   count(*) = sum_b [b_ok] inA(b) outC(b) - #{self-loops at b : a_ok b_ok c_ok}
 *   c counted iff c_ok(c) and some r2 = b->c with b_ok(b) has an a_ok in-edge r1 != r2:
 *   inA(b) >= 1 for b != c, inA(b) >= 2 for a self-loop r2 at an a_ok b. */
int orc_two_hop_closed_form_mt(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                               const uint8_t* b_ok, const uint8_t* c_ok, int64_t* out_rows, int64_t* out_distinct,
                               int nthreads) {
    int64_t* in_a = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    int64_t* out_c = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    uint8_t* mark = (uint8_t*)calloc((size_t)n, 1);
    if (!in_a || !out_c || !mark) { free(in_a); free(out_c); free(mark); return -1; }
    set_threads(nthreads);
    int64_t loops = 0, rows = 0, d = 0;
#pragma omp parallel for schedule(static) reduction(+ : loops)
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        if (OK(a_ok, s)) {
#pragma omp atomic
            in_a[t]++;
        }
        if (OK(c_ok, t)) {
#pragma omp atomic
            out_c[s]++;
        }
        if (s == t && OK(a_ok, s) && OK(b_ok, s) && OK(c_ok, s)) loops++;
    }
#pragma omp parallel for schedule(static) reduction(+ : rows)
    for (int64_t b = 0; b < n; ++b)
        if (OK(b_ok, b)) rows += in_a[b] * out_c[b];
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < m; ++e) {
        const int64_t b = src[e], c = dst[e];
        if (!OK(b_ok, b) || !OK(c_ok, c)) continue;
        const int64_t need = (b == c && OK(a_ok, b)) ? 2 : 1;
        if (in_a[b] >= need) mark[c] = 1; /* every writer stores 1 */
    }
#pragma omp parallel for schedule(static) reduction(+ : d)
    for (int64_t i = 0; i < n; ++i) d += mark[i];
    *out_rows = rows - loops;
    *out_distinct = d;
    free(in_a); free(out_c); free(mark);
    return 0;
}

/* Undirected 2-hop (a)-[r1]-(b)-[r2]-(c), r1 <> r2 (RelationalPlanner.scala:126-136: out ∪ in-without-loops per
 * hop; MatchBehaviour.scala:258-279).  Every relationship e = (s, t) is the arc s -> t and, when s != t, the
 * arc t -> s.  With inU(b) = a_ok arcs into b and outU(b) = c_ok arcs out of b:
 *   count(*) = sum_b [b_ok] inU(b) outU(b) - corr, corr = the bindings with r1 = r2 (a non-loop walked in
 *   and back out: [a(s) b(t) c(s)] + [a(t) b(s) c(t)]; a loop: [a b c](s));
 *   count(DISTINCT c): K(b) = a_ok arcs into b capped at 2, x(b) the other end of the only one when K = 1;
 *   an arc b -> c (c_ok, b_ok) extends a binding iff K(b) = 2, or K(b) = 1 and c != x(b).
 * The same derivation as the device path (csrc/k_undirected.hip, csrc/k_count.hip k_rec_part<true>);
 * pinned against rmat.c orc_two_hop_undirected_enumerate (tests/test_oracle_pins.py). */
int orc_two_hop_undirected_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                                       const uint8_t* a_ok, const uint8_t* b_ok, const uint8_t* c_ok,
                                       int64_t* out_rows, int64_t* out_distinct, int nthreads) {
    int64_t* in_u = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t* out_u = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
    int64_t* kx = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t)); /* 0, x + 1, or -1 (two or more) */
    uint8_t* mark = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    if (!in_u || !out_u || !kx || !mark) { free(in_u); free(out_u); free(kx); free(mark); return -1; }
    set_threads(nthreads);
    int64_t corr = 0, rows = 0, d = 0;
#pragma omp parallel for schedule(static) reduction(+ : corr)
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        if (OK(a_ok, s)) {
#pragma omp atomic
            in_u[t]++;
        }
        if (OK(c_ok, t)) {
#pragma omp atomic
            out_u[s]++;
        }
        if (s != t) {
            if (OK(a_ok, t)) {
#pragma omp atomic
                in_u[s]++;
            }
            if (OK(c_ok, s)) {
#pragma omp atomic
                out_u[t]++;
            }
            corr += (OK(a_ok, s) && OK(b_ok, t) && OK(c_ok, s)) + (OK(a_ok, t) && OK(b_ok, s) && OK(c_ok, t));
        } else {
            corr += OK(a_ok, s) && OK(b_ok, s) && OK(c_ok, s);
        }
    }
#pragma omp parallel for schedule(static) reduction(+ : rows)
    for (int64_t b = 0; b < n; ++b)
        if (OK(b_ok, b)) rows += in_u[b] * out_u[b];
    for (int64_t e = 0; e < m; ++e) { /* K(b), x(b): the a_ok arcs into b_ok ids (sequential) */
        const int64_t s = src[e], t = dst[e];
        for (int dir = 0; dir < (s != t ? 2 : 1); ++dir) {
            const int64_t x = dir ? t : s, b = dir ? s : t;
            if (!OK(a_ok, x) || !OK(b_ok, b)) continue;
            kx[b] = kx[b] == 0 ? x + 1 : -1;
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        for (int dir = 0; dir < (s != t ? 2 : 1); ++dir) {
            const int64_t b = dir ? t : s, c = dir ? s : t;
            if (!OK(c_ok, c)) continue;
            const int64_t k = kx[b];
            if (k == -1 || (k != 0 && k - 1 != c)) mark[c] = 1;
        }
    }
#pragma omp parallel for schedule(static) reduction(+ : d)
    for (int64_t i = 0; i < n; ++i) d += mark[i];
    *out_rows = rows - corr;
    *out_distinct = d;
    free(in_u); free(out_u); free(kx); free(mark);
    return 0;
}

/* ---- sorted adjacency helpers ------------------------------------------------------------- */
static int cmp_i64(const void* a, const void* b) {
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return (x > y) - (x < y);
}

/* CSR by source with each vertex's targets sorted (multi-edges adjacent) */
static int sorted_csr(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, int64_t** off_out,
                      int64_t** tgt_out) {
    int64_t* off = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* tgt = (int64_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    int64_t* cur = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!off || !tgt || !cur) { free(off); free(tgt); free(cur); return -1; }
    for (int64_t e = 0; e < m; ++e) off[src[e] + 1]++;
    for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
    memcpy(cur, off, (size_t)n * sizeof(int64_t));
    for (int64_t e = 0; e < m; ++e) tgt[cur[src[e]]++] = dst[e];
    free(cur);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t v = 0; v < n; ++v)
        if (off[v + 1] - off[v] > 1) qsort(tgt + off[v], (size_t)(off[v + 1] - off[v]), sizeof(int64_t), cmp_i64);
    *off_out = off;
    *tgt_out = tgt;
    return 0;
}

/* number of entries equal to x in the sorted range [lo, hi) */
static int64_t count_in(const int64_t* a, int64_t lo, int64_t hi, int64_t x) {
    int64_t l = lo, h = hi;
    while (l < h) { const int64_t mid = (l + h) / 2; if (a[mid] < x) l = mid + 1; else h = mid; }
    int64_t first = l;
    h = hi;
    while (l < h) { const int64_t mid = (l + h) / 2; if (a[mid] <= x) l = mid + 1; else h = mid; }
    return l - first;
}

/* C5 closed form: MATCH (a)-[*lo..hi]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), count(*),
 * 1 <= lo <= hi <= 3, edge-distinct paths.  With od(v) = #{v->w : b_ok(w)}, s(v) = #self-loops at v,
 * W(v) = sum_{v->w} od(w), m(v,u) = multiplicity of v->u, per source a:
 *   len1 = od(a)
 *   len2 = sum_{a->v} od(v) - s(a) b_ok(a)                 (r2 = r1 only for a self-loop at a, ending at a)
 *   len3 = sum_{a->v} W(v) - |A u B u C| where A: r2 = r1 (s(a) od(a)), B: r3 = r2 (sum_{a->v} s(v) b_ok(v)),
 *          C: r3 = r1 (sum_{a->v} m(v,a) b_ok(v)); every pairwise intersection is r1 = r2 = r3, a self-loop at
 *          a used thrice (s(a) b_ok(a)), so |A u B u C| = |A| + |B| + |C| - 2 s(a) b_ok(a).
 * group_rows[a] = sum of len_k(a) for k in [lo, hi] (0 when !a_ok(a)). */
int orc_var_length_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                               const uint8_t* b_ok, int lo, int hi, int64_t* group_rows, int64_t* out_rows,
                               int nthreads) {
    if (lo < 1 || hi < lo || hi > 3) return -2;
    set_threads(nthreads);
    int64_t *off, *tgt;
    if (sorted_csr(n, m, src, dst, &off, &tgt)) return -1;
    int64_t* od = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    int64_t* sl = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    int64_t* W = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    if (!od || !sl || !W) { free(off); free(tgt); free(od); free(sl); free(W); return -1; }
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t v = 0; v < n; ++v) {
        int64_t o = 0, s = 0;
        for (int64_t i = off[v]; i < off[v + 1]; ++i) {
            o += OK(b_ok, tgt[i]);
            s += tgt[i] == v;
        }
        od[v] = o;
        sl[v] = s;
    }
#pragma omp parallel for schedule(dynamic, 1024)
    for (int64_t v = 0; v < n; ++v) {
        int64_t w = 0;
        for (int64_t i = off[v]; i < off[v + 1]; ++i) w += od[tgt[i]];
        W[v] = w;
    }
    int64_t rows = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : rows)
    for (int64_t a = 0; a < n; ++a) {
        int64_t tot = 0;
        if (OK(a_ok, a)) {
            const int64_t ba = OK(b_ok, a) ? 1 : 0;
            int64_t s1 = 0, sw = 0, sb = 0, sc = 0;
            for (int64_t i = off[a]; i < off[a + 1]; ++i) {
                const int64_t v = tgt[i];
                s1 += od[v];
                if (hi >= 3) {
                    sw += W[v];
                    if (OK(b_ok, v)) {
                        sb += sl[v];
                        sc += count_in(tgt, off[v], off[v + 1], a);
                    }
                }
            }
            const int64_t len1 = od[a];
            const int64_t len2 = s1 - sl[a] * ba;
            const int64_t len3 = sw - (sl[a] * od[a] + sb + sc - 2 * sl[a] * ba);
            if (lo <= 1 && hi >= 1) tot += len1;
            if (lo <= 2 && hi >= 2) tot += len2;
            if (lo <= 3 && hi >= 3) tot += len3;
        }
        if (group_rows) group_rows[a] = tot;
        rows += tot;
    }
    *out_rows = rows;
    free(off); free(tgt); free(od); free(sl); free(W);
    return 0;
}

/* ---- C4 ------------------------------------------------------------------------------------- */
/* LSD radix sort of 64-bit keys on their low `bits` bits (8-bit digits); returns the buffer that
 * holds the result (a or tmp) */
/* The one four-hop term that is not a product of per-node vectors (cpu.py var_length4_closed_form, the block
 * {1,4} of the hop positions): T14(a) = sum_{r: a->y} b_ok(y) sum_{r': y->p} m(p, a), the closing
 * relationships of the 2-walks a -> y -> p counted with multiplicity = sum_y m(a,y) b_ok(y) |out(y) ∩ in(a)|
 * over multisets, by a merge of y's sorted out-list with a's sorted in-list (the wedges are never listed). */
int orc_vl4_t14(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* b_ok, int64_t* t14,
                int nthreads) {
    set_threads(nthreads);
    int64_t *ooff = NULL, *otg = NULL, *ioff = NULL, *isrc = NULL;
    if (sorted_csr(n, m, src, dst, &ooff, &otg)) return -1;
    if (sorted_csr(n, m, dst, src, &ioff, &isrc)) { free(ooff); free(otg); return -1; }
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t a = 0; a < n; ++a) {
        int64_t t = 0;
        const int64_t ib = ioff[a], ie = ioff[a + 1];
        for (int64_t i = ooff[a]; i < ooff[a + 1];) {
            const int64_t y = otg[i];
            int64_t k = 1;  /* m(a, y): the run of y in a's sorted out-list */
            while (i + k < ooff[a + 1] && otg[i + k] == y) ++k;
            i += k;
            if (!OK(b_ok, y) || ib == ie) continue;
            int64_t u = ooff[y], ue = ooff[y + 1], v = ib, c = 0;
            while (u < ue && v < ie) {
                if (otg[u] < isrc[v]) ++u;
                else if (otg[u] > isrc[v]) ++v;
                else {
                    const int64_t p = otg[u];
                    int64_t cu = 0, cv = 0;
                    while (u < ue && otg[u] == p) { ++u; ++cu; }
                    while (v < ie && isrc[v] == p) { ++v; ++cv; }
                    c += cu * cv;
                }
            }
            t += k * c;
        }
        t14[a] = t;
    }
    free(ooff); free(otg); free(ioff); free(isrc);
    return 0;
}

static uint64_t* radix_sort_u64(uint64_t* a, uint64_t* tmp, int64_t n, int bits) {
    for (int sh = 0; sh < bits; sh += 8) {
        int64_t cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (int64_t i = 0; i < n; ++i) cnt[((a[i] >> sh) & 255) + 1]++;
        for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
        for (int64_t i = 0; i < n; ++i) tmp[cnt[(a[i] >> sh) & 255]++] = a[i];
        uint64_t* t = a;
        a = tmp;
        tmp = t;
    }
    return a;
}

/* index of x in the sorted array a[lo, hi), or -1 */
static int64_t find_u64(const uint64_t* a, int64_t lo, int64_t hi, uint64_t x) {
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

typedef struct { int64_t nbr, fwd, bwd; } OEdge; /* oriented edge u->nbr with m(u,nbr), m(nbr,u) */

static int cmp_oedge(const void* a, const void* b) {
    const int64_t x = ((const OEdge*)a)->nbr, y = ((const OEdge*)b)->nbr;
    return (x > y) - (x < y);
}

/* C4 closed form: MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) WHERE n_ok(a,b,c) RETURN count(*),
 * r1, r2, r3 pairwise distinct.  Bindings split by which of a, b, c coincide (m(x,y) = multiplicity
 * of x->y, s(x) = self-loops at x):
 *   all distinct: a directed 3-cycle; each of the two cyclic orientations of a triangle {u,v,w} of the
 *     simple undirected graph is bound once per choice of a: 3 [m(u,v)m(v,w)m(w,u) + m(u,w)m(w,v)m(v,u)]
 *   exactly two equal (a=b, b=c or c=a): one hop is a self-loop at u, the other two go u->x->u (x != u):
 *     3 sum_{u, x != u} s(u) m(u,x) m(x,u)
 *   a = b = c: three distinct self-loops: s(u)(s(u)-1)(s(u)-2).
 * Triangles are listed once by orienting each simple edge from its lower (degree, id) end. */
int orc_triangle_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* n_ok,
                             int64_t* out_rows, int nthreads) {
    set_threads(nthreads);
    int bits = 1;
    while (bits < 62 && ((int64_t)1 << bits) < n) ++bits;
    if (2 * bits > 62) return -2;
    const uint64_t lowmask = ((uint64_t)1 << bits) - 1;
    uint64_t* k0 = (uint64_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(uint64_t));
    uint64_t* k1 = (uint64_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(uint64_t));
    int64_t* sl = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* deg = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    if (!k0 || !k1 || !sl || !deg) { free(k0); free(k1); free(sl); free(deg); return -1; }
    /* directed non-loop edges with both ends n_ok as keys (s << bits | t); self-loops per node */
    int64_t k = 0;
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        if (!OK(n_ok, s) || !OK(n_ok, t)) continue;
        if (s == t) { sl[s]++; continue; }
        k0[k++] = ((uint64_t)s << bits) | (uint64_t)t;
    }
    uint64_t* key = radix_sort_u64(k0, k1, k, 2 * bits);
    uint64_t* spare = key == k0 ? k1 : k0;
    /* distinct directed pairs and their multiplicities (spare reused as the multiplicity array) */
    int64_t nd = 0;
    int64_t* mult = (int64_t*)spare;
    for (int64_t i = 0; i < k;) {
        int64_t j = i;
        while (j < k && key[j] == key[i]) ++j;
        key[nd] = key[i];
        mult[nd] = j - i;
        ++nd;
        i = j;
    }
    /* simple undirected edges u < v with (m(u,v), m(v,u)); degrees */
    int64_t nu = 0;
    for (int64_t i = 0; i < nd; ++i) {
        const int64_t s = (int64_t)(key[i] >> bits), t = (int64_t)(key[i] & lowmask);
        const int64_t r = find_u64(key, 0, nd, ((uint64_t)t << bits) | (uint64_t)s);
        const int rev = r < nd && key[r] == (((uint64_t)t << bits) | (uint64_t)s);
        if (s < t || !rev) { deg[s]++; deg[t]++; nu++; }
    }
    int64_t* off = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    OEdge* oe = (OEdge*)malloc((size_t)(nu > 0 ? nu : 1) * sizeof(OEdge));
    int64_t* cur = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    if (!off || !oe || !cur) { free(k0); free(k1); free(sl); free(deg); free(off); free(oe); free(cur); return -1; }
#define LOWER(x, y) (deg[x] < deg[y] || (deg[x] == deg[y] && (x) < (y)))
    int64_t pair_sum = 0; /* sum over simple edges of m(u,v) m(v,u) (s(u) + s(v)) */
    for (int pass = 0; pass < 2; ++pass) {
        for (int64_t i = 0; i < nd; ++i) {
            const int64_t s = (int64_t)(key[i] >> bits), t = (int64_t)(key[i] & lowmask);
            const int64_t r = find_u64(key, 0, nd, ((uint64_t)t << bits) | (uint64_t)s);
            const int rev = r < nd && key[r] == (((uint64_t)t << bits) | (uint64_t)s);
            if (!(s < t || !rev)) continue;
            const int64_t mst = mult[i], mts = rev ? mult[r] : 0;
            const int64_t u = LOWER(s, t) ? s : t, v = u == s ? t : s;
            if (pass == 0) {
                off[u + 1]++;
                pair_sum += mst * mts * (sl[s] + sl[t]);
            } else {
                OEdge* o = &oe[cur[u]++];
                o->nbr = v;
                o->fwd = u == s ? mst : mts;
                o->bwd = u == s ? mts : mst;
            }
        }
        if (pass == 0) {
            for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
            memcpy(cur, off, (size_t)n * sizeof(int64_t));
        }
    }
#undef LOWER
    free(cur);
    free(k0); free(k1);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t u = 0; u < n; ++u)
        if (off[u + 1] - off[u] > 1) qsort(oe + off[u], (size_t)(off[u + 1] - off[u]), sizeof(OEdge), cmp_oedge);
    int64_t tri = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : tri)
    for (int64_t u = 0; u < n; ++u) {
        const int64_t ub = off[u], ue = off[u + 1];
        for (int64_t i = ub; i < ue; ++i) {
            const int64_t v = oe[i].nbr;
            for (int64_t j = off[v]; j < off[v + 1]; ++j) {
                const int64_t w = oe[j].nbr;
                int64_t l = ub, h = ue;
                while (l < h) { const int64_t mid = (l + h) / 2; if (oe[mid].nbr < w) l = mid + 1; else h = mid; }
                if (l == ue || oe[l].nbr != w) continue;
                /* m(u,v) m(v,w) m(w,u) + m(u,w) m(w,v) m(v,u) */
                tri += oe[i].fwd * oe[j].fwd * oe[l].bwd + oe[l].fwd * oe[j].bwd * oe[i].bwd;
            }
        }
    }
    int64_t loops3 = 0;
    for (int64_t u = 0; u < n; ++u) loops3 += sl[u] * (sl[u] - 1) * (sl[u] - 2);
    *out_rows = 3 * tri + 3 * pair_sum + loops3;
    free(sl); free(deg); free(off); free(oe);
    return 0;
}
