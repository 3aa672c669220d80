/*
 * oracle/rmat.c -- CPU restatement (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the checker for the capsmi HIP path.  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it.  The product
 * library (libcapsmi.so) never links or calls it.
 *
 * It restates, on the CPU, the relational semantics CAPS produces for the
 * benchmark patterns.  The reference computes them as Spark DataFrame joins
 * emitted by okapi-relational:
 *   - Expand  = src ⋈[id=source] rels ⋈[target=id] dst
 *               okapi-relational/.../planning/RelationalPlanner.scala:113-137
 *   - the front-end adds NOT(r_i = r_j) for every pair of relationship
 *               variables in one MATCH (okapi-ir/.../parse/CypherParser.scala:64-76),
 *               planned as Filter (RelationalOperator.scala:293-301)
 *   - count(*) / count(DISTINCT x) = Spark count(lit 0) / countDistinct
 *               spark-cypher/.../impl/table/SparkTable.scala:148-158
 * The enumeration functions below walk every binding exactly as the joins
 * would emit them (one row per (a, r1, b, r2, c) with r1 != r2); the
 * closed-form functions are an independent derivation used to pin the
 * enumeration and to check the GPU at sizes where enumeration is too slow.
 *
 * Synthetic input: R-MAT, Graph500-style quadrant recursion,
 * counter-based RNG so any partition of the edge index space regenerates the
 * identical edge.  The exact bit-level definition lives here and is mirrored by
 * the HIP generator; tests check the two agree edge for edge.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* R-MAT edge e of a graph with 2^scale vertices.
 * probabilities are given in percent: pa, pb, pc (pd = 100 - pa - pb - pc).
 * level l (0 = most significant bit) draws a 32-bit uniform u from
 *   r = splitmix64((seed << 40) | (e << 5) | (l >> 1)),  u = l even ? r >> 32 : r & 0xffffffff
 * quadrant: u < tA -> (0,0); u < tAB -> (0,1); u < tABC -> (1,0); else (1,1)
 * with tX = floor(cumulative_percent * 2^32 / 100).
 * Vertex ids are scrambled: id = (v * 0x9E3779B97F4A7C15) mod 2^scale. */
static inline void rmat_edge(int scale, int pa, int pb, int pc, uint64_t seed, uint64_t e,
                             int64_t* s_out, int64_t* d_out) {
    const uint64_t tA = ((uint64_t)pa << 32) / 100;
    const uint64_t tAB = ((uint64_t)(pa + pb) << 32) / 100;
    const uint64_t tABC = ((uint64_t)(pa + pb + pc) << 32) / 100;
    uint64_t s = 0, d = 0, r = 0;
    for (int l = 0; l < scale; ++l) {
        if ((l & 1) == 0) r = orc_splitmix64((seed << 40) | (e << 5) | (uint64_t)(l >> 1));
        uint64_t u = (l & 1) == 0 ? (r >> 32) : (r & 0xffffffffULL);
        uint64_t sb, db;
        if (u < tA) { sb = 0; db = 0; }
        else if (u < tAB) { sb = 0; db = 1; }
        else if (u < tABC) { sb = 1; db = 0; }
        else { sb = 1; db = 1; }
        s |= sb << (scale - 1 - l);
        d |= db << (scale - 1 - l);
    }
    const uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    *s_out = (int64_t)((s * 0x9E3779B97F4A7C15ULL) & mask);
    *d_out = (int64_t)((d * 0x9E3779B97F4A7C15ULL) & mask);
}

void orc_rmat_edges(int scale, int pa, int pb, int pc, uint64_t seed, int64_t e_begin, int64_t e_end,
                    int64_t* src, int64_t* dst) {
#pragma omp parallel for schedule(static)
    for (int64_t e = e_begin; e < e_end; ++e)
        rmat_edge(scale, pa, pb, pc, seed, (uint64_t)e, &src[e - e_begin], &dst[e - e_begin]);
}

/* C2 node tables: Person iff (splitmix64(id) & 3) != 0, age = splitmix64(seed ^ id) % 100. */
int orc_is_person(int64_t id) { return (orc_splitmix64((uint64_t)id) & 3ULL) != 0; }
int64_t orc_age(int64_t id, uint64_t seed) { return (int64_t)(orc_splitmix64(seed ^ (uint64_t)id) % 100ULL); }

/* Order-insensitive row-multiset fingerprint (SURVEY.md §8d parity check):
 * row hash h = fold over columns h = splitmix64(h ^ v) starting at 0x243F6A8885A308D3;
 * fingerprint = (count, sum of h mod 2^64, xor of h). */
uint64_t orc_row_hash(const int64_t* vals, int ncols) {
    uint64_t h = 0x243F6A8885A308D3ULL;
    for (int i = 0; i < ncols; ++i) h = orc_splitmix64(h ^ (uint64_t)vals[i]);
    return h;
}

/* ---- CSR helpers (counting sort by key), dense ids in [0, n) ---------------- */
static int64_t* csr_offsets(int64_t n, int64_t m, const int64_t* key) {
    int64_t* off = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    if (!off) return NULL;
    for (int64_t e = 0; e < m; ++e) off[key[e] + 1]++;
    for (int64_t v = 0; v < n; ++v) off[v + 1] += off[v];
    return off;
}

/* returns edge indices grouped by key (stable: ascending edge index inside a group) */
static int64_t* csr_edges(int64_t n, int64_t m, const int64_t* key, const int64_t* off) {
    int64_t* cur = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* adj = (int64_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    if (!cur || !adj) { free(cur); free(adj); return NULL; }
    memcpy(cur, off, (size_t)n * sizeof(int64_t));
    for (int64_t e = 0; e < m; ++e) adj[cur[key[e]]++] = e;
    free(cur);
    return adj;
}

#define OK(bm, v) ((bm) == NULL || (bm)[v])

/* C3 by literal enumeration of every binding (the reference's join semantics):
 *   MATCH (a)-[r1]->(b)-[r2]->(c) WHERE a_ok(a) AND b_ok(b) AND c_ok(c)  (label scans)
 *   uniqueness: r1 <> r2 (front-end rewrite)
 * out_rows = count(*), out_distinct = count(DISTINCT c).
 * Optional per-a output: if group_distinct != NULL, group_distinct[a] = count(DISTINCT c) for that a
 * and group_rows[a] = count(*) for that a.  Returns 0, or -1 on allocation failure. */
/* Undirected 2-hop by enumeration: MATCH (a)-[r1]-(b)-[r2]-(c) with r1 <> r2.  An undirected Expand is
 * the outgoing branch plus the incoming branch over relationships whose start differs from their end
 * (RelationalPlanner.scala:126-136): from a node, every relationship e = (s, t) is the arc s -> t and,
 * for s != t, the arc t -> s.  Every (arc1 into b, arc2 out of b) with different relationships is one
 * binding; count(*), count(DISTINCT c) and count(DISTINCT a).  Test oracle for the fused undirected
 * route (csrc/k_undirected.hip), pinned to oracle/enumerate.py in tests/test_oracle_pins.py. */
int orc_two_hop_undirected_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                                     const uint8_t* a_ok, const uint8_t* b_ok, const uint8_t* c_ok,
                                     int64_t* out_rows, int64_t* out_distinct_c, int64_t* out_distinct_a,
                                     int nthreads) {
    int64_t k = 0;
    for (int64_t e = 0; e < m; ++e) k += src[e] == dst[e] ? 1 : 2;
    int64_t* as = (int64_t*)malloc((size_t)(k ? k : 1) * sizeof(int64_t));
    int64_t* at = (int64_t*)malloc((size_t)(k ? k : 1) * sizeof(int64_t));
    int64_t* ae = (int64_t*)malloc((size_t)(k ? k : 1) * sizeof(int64_t));
    uint8_t* mc = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    uint8_t* ma = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
    if (!as || !at || !ae || !mc || !ma) { free(as); free(at); free(ae); free(mc); free(ma); return -1; }
    int64_t j = 0;
    for (int64_t e = 0; e < m; ++e) {
        as[j] = src[e]; at[j] = dst[e]; ae[j++] = e;
        if (src[e] != dst[e]) { as[j] = dst[e]; at[j] = src[e]; ae[j++] = e; }
    }
    int64_t* off = csr_offsets(n, k, as);
    int64_t* adj = off ? csr_edges(n, k, as, off) : NULL;
    if (!off || !adj) { free(as); free(at); free(ae); free(mc); free(ma); free(off); free(adj); return -1; }
    int64_t rows = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : rows)
    for (int64_t a = 0; a < n; ++a) {
        if (!OK(a_ok, a)) continue;
        int64_t arows = 0;
        for (int64_t i = off[a]; i < off[a + 1]; ++i) {
            const int64_t x1 = adj[i], b = at[x1];
            if (!OK(b_ok, b)) continue;
            for (int64_t q = off[b]; q < off[b + 1]; ++q) {
                const int64_t x2 = adj[q];
                if (ae[x2] == ae[x1]) continue; /* r1 = r2 */
                const int64_t c = at[x2];
                if (!OK(c_ok, c)) continue;
                ++arows;
                if (!mc[c]) mc[c] = 1; /* benign race: every writer stores 1 */
            }
        }
        if (arows) ma[a] = 1;
        rows += arows;
    }
    int64_t dc = 0, da = 0;
    for (int64_t i = 0; i < n; ++i) { dc += mc[i]; da += ma[i]; }
    *out_rows = rows;
    *out_distinct_c = dc;
    *out_distinct_a = da;
    free(as); free(at); free(ae); free(mc); free(ma); free(off); free(adj);
    return 0;
}

int orc_two_hop_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                          const uint8_t* a_ok, const uint8_t* b_ok, const uint8_t* c_ok,
                          int64_t* out_rows, int64_t* out_distinct,
                          int64_t* group_rows, int64_t* group_distinct, int nthreads) {
    int64_t* off = csr_offsets(n, m, src);
    if (!off) return -1;
    int64_t* adj = csr_edges(n, m, src, off);
    uint8_t* mark = (uint8_t*)calloc((size_t)n, 1);
    if (!adj || !mark) { free(off); free(adj); free(mark); return -1; }
    int64_t rows = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : rows)
    {
        int64_t* stamp = NULL;
        if (group_distinct) {
            stamp = (int64_t*)malloc((size_t)n * sizeof(int64_t));
            if (stamp) for (int64_t i = 0; i < n; ++i) stamp[i] = -1;
        }
#pragma omp for schedule(dynamic, 64)
        for (int64_t a = 0; a < n; ++a) {
            if (!OK(a_ok, a)) continue;
            int64_t arows = 0, adist = 0;
            for (int64_t i = off[a]; i < off[a + 1]; ++i) {
                const int64_t r1 = adj[i];
                const int64_t b = dst[r1];
                if (!OK(b_ok, b)) continue;
                for (int64_t j = off[b]; j < off[b + 1]; ++j) {
                    const int64_t r2 = adj[j];
                    if (r2 == r1) continue;
                    const int64_t c = dst[r2];
                    if (!OK(c_ok, c)) continue;
                    ++arows;
                    if (!mark[c]) mark[c] = 1; /* benign race: every writer stores 1 */
                    if (stamp && stamp[c] != a) { stamp[c] = a; ++adist; }
                }
            }
            rows += arows;
            if (group_rows) group_rows[a] = arows;
            if (group_distinct) group_distinct[a] = stamp ? adist : -1;
        }
        free(stamp);
    }
    int64_t d = 0;
    for (int64_t i = 0; i < n; ++i) d += mark[i];
    *out_rows = rows;
    *out_distinct = d;
    free(off); free(adj); free(mark);
    return 0;
}

/* C3 closed form (independent derivation, no enumeration):
 *   count(*) = sum_b [b_ok] * inA(b) * outC(b) - #{self-loops r at b : a_ok(b) b_ok(b) c_ok(b)}
 *     where inA(b) = #edges x->b with a_ok(x), outC(b) = #edges b->y with c_ok(y);
 *     a binding is lost to r1 <> r2 only when r1 = r2, i.e. a self-loop used twice.
 *   DISTINCT c: c is reached through r2 = (b -> c) iff b_ok(b), c_ok(c) and some r1 != r2 enters b
 *     from an a_ok node: for b != c any a_ok in-edge of b works; for a self-loop r2 (c = b) we need an
 *     a_ok in-edge other than r2 itself, i.e. inA(b) >= 2 (r2 is one of b's a_ok in-edges when a_ok(b)). */
int orc_two_hop_closed_form(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                            const uint8_t* a_ok, const uint8_t* b_ok, const uint8_t* c_ok,
                            int64_t* out_rows, int64_t* out_distinct) {
    int64_t* in_a = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    int64_t* out_c = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    uint8_t* mark = (uint8_t*)calloc((size_t)n, 1);
    if (!in_a || !out_c || !mark) { free(in_a); free(out_c); free(mark); return -1; }
    int64_t loops = 0;
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        if (OK(a_ok, s)) in_a[t]++;
        if (OK(c_ok, t)) out_c[s]++;
        if (s == t && OK(a_ok, s) && OK(b_ok, s) && OK(c_ok, s)) loops++;
    }
    int64_t rows = 0;
    for (int64_t b = 0; b < n; ++b)
        if (OK(b_ok, b)) rows += in_a[b] * out_c[b];
    rows -= loops;
    for (int64_t e = 0; e < m; ++e) {
        const int64_t b = src[e], c = dst[e];
        if (!OK(b_ok, b) || !OK(c_ok, c)) continue;
        const int64_t need = (b == c && OK(a_ok, b)) ? 2 : 1;
        if (in_a[b] >= need) mark[c] = 1;
    }
    int64_t d = 0;
    for (int64_t i = 0; i < n; ++i) d += mark[i];
    *out_rows = rows;
    *out_distinct = d;
    free(in_a); free(out_c); free(mark);
    return 0;
}

/* C2: MATCH (a)-[r]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), id(b)
 * fingerprint over the returned (id(a), id(b)) rows. */
void orc_expand_filter(int64_t m, const int64_t* src, const int64_t* dst,
                       const uint8_t* a_ok, const uint8_t* b_ok,
                       int64_t* out_rows, uint64_t* out_sum, uint64_t* out_xor) {
    int64_t rows = 0;
    uint64_t hs = 0, hx = 0;
#pragma omp parallel for reduction(+ : rows, hs) reduction(^ : hx) schedule(static)
    for (int64_t e = 0; e < m; ++e) {
        const int64_t s = src[e], t = dst[e];
        if (!OK(a_ok, s) || !OK(b_ok, t)) continue;
        int64_t row[2] = {s, t};
        uint64_t h = orc_row_hash(row, 2);
        rows++;
        hs += h;
        hx ^= h;
    }
    *out_rows = rows;
    *out_sum = hs;
    *out_xor = hx;
}

/* C4 by enumeration: MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) RETURN count(*)
 * with pairwise distinct r1, r2, r3 (front-end uniqueness).  Closing edge via a
 * per-(c, a) multiplicity scan over c's out-list (ExpandInto, RelationalPlanner.scala:139-148). */
int orc_triangle_enumerate(int64_t n, int64_t m, const int64_t* src, const int64_t* dst,
                           int64_t* out_rows, int nthreads) {
    int64_t* off = csr_offsets(n, m, src);
    if (!off) return -1;
    int64_t* adj = csr_edges(n, m, src, off);
    if (!adj) { free(off); return -1; }
    int64_t rows = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for reduction(+ : rows) schedule(dynamic, 16)
    for (int64_t a = 0; a < n; ++a) {
        for (int64_t i = off[a]; i < off[a + 1]; ++i) {
            const int64_t r1 = adj[i], b = dst[r1];
            for (int64_t j = off[b]; j < off[b + 1]; ++j) {
                const int64_t r2 = adj[j];
                if (r2 == r1) continue;
                const int64_t c = dst[r2];
                for (int64_t k = off[c]; k < off[c + 1]; ++k) {
                    const int64_t r3 = adj[k];
                    if (dst[r3] != a || r3 == r1 || r3 == r2) continue;
                    rows++;
                }
            }
        }
    }
    *out_rows = rows;
    free(off); free(adj);
    return 0;
}

/* C5 by enumeration: MATCH (a)-[:KNOWS*lo..hi]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a), count(*)
 * Paths never repeat an edge (VarLengthExpandPlanner.scala:97,133,179-180).
 * group_rows[a] += number of paths starting at a (all lengths lo..hi, lo >= 1). */
static void var_dfs(const int64_t* off, const int64_t* adj, const int64_t* dst, const uint8_t* b_ok, int64_t v,
                    int depth, int lo, int hi, int64_t* path, int64_t* cnt) {
    for (int64_t i = off[v]; i < off[v + 1]; ++i) {
        const int64_t r = adj[i];
        int dup = 0;
        for (int k = 0; k < depth; ++k) if (path[k] == r) { dup = 1; break; }
        if (dup) continue;
        path[depth] = r;
        if (depth + 1 >= lo && OK(b_ok, dst[r])) (*cnt)++;
        if (depth + 1 < hi) var_dfs(off, adj, dst, b_ok, dst[r], depth + 1, lo, hi, path, cnt);
    }
}

int orc_var_length_count(int64_t n, int64_t m, const int64_t* src, const int64_t* dst, const uint8_t* a_ok,
                         const uint8_t* b_ok, int lo, int hi, int64_t* group_rows, int64_t* out_rows, int nthreads) {
    if (lo < 1 || hi < lo || hi > 16) return -2;
    int64_t* off = csr_offsets(n, m, src);
    if (!off) return -1;
    int64_t* adj = csr_edges(n, m, src, off);
    if (!adj) { free(off); return -1; }
    int64_t rows = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for reduction(+ : rows) schedule(dynamic, 64)
    for (int64_t a = 0; a < n; ++a) {
        int64_t path[16];
        int64_t c = 0;
        if (OK(a_ok, a)) var_dfs(off, adj, dst, b_ok, a, 0, lo, hi, path, &c);
        if (group_rows) group_rows[a] = c;
        rows += c;
    }
    *out_rows = rows;
    free(off); free(adj);
    return 0;
}
