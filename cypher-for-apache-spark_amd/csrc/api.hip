// api.hip -- the C ABI (include/capsmi.h): CAPS Table[T] operators on device tables.
//
// Each capsmi_* operator mirrors one member of
//   okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala
// with the semantics DataFrameTable gives it
//   spark-cypher/src/main/scala/org/opencypher/spark/impl/table/SparkTable.scala
// Errors surface as status codes + a thread-local message, mapping the okapi exceptions.
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <unordered_set>

#include "capsmi_impl.h"
#include "part_common.h"

namespace capsmi {

namespace graph {
void expand_filter(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
                   const capsmi_bitmap* b, int nout, const int64_t* const* in_d, const uint8_t* const* in_v,
                   int64_t* const* out_d, uint8_t* const* out_v, int64_t* dev_count);
void hop1(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
          const capsmi_bitmap* b, uint32_t* M, uint32_t* S1, uint32_t* S2);
void mid_combine(capsmi_session* s, uint32_t* X1, uint32_t* X2, const uint32_t* S1, int64_t nw);
void hop2(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* c,
          const uint32_t* X1, const uint32_t* X2, int64_t mid_lo, int64_t mid_hi, uint32_t* C);
void degrees(capsmi_session* s, const int64_t* src, const int64_t* dst, int64_t m, const capsmi_bitmap* a,
             const capsmi_bitmap* b, const capsmi_bitmap* c, uint32_t* inA, uint32_t* outC, int64_t* loops);
void deg_product(capsmi_session* s, const uint32_t* inA, const uint32_t* outC, int64_t n, const capsmi_bitmap* b,
                 int64_t* out);
int64_t rmat(capsmi_session* s, int scale, int64_t e_begin, int64_t e_end, int pa, int pb, int pc, uint64_t seed,
             int part_col, int part, int nparts, Buf& id, Buf& so, Buf& dout);
void person_flags(capsmi_session* s, int64_t n, bool want_person, uint8_t* f);
void ages(capsmi_session* s, const int64_t* ids, int64_t n, uint64_t seed, int64_t* age);
void fingerprint(capsmi_session* s, int ncols, const int64_t* const* d, const uint8_t* const* v, int64_t n,
                 uint64_t* out_sum, uint64_t* out_xor);
}  // namespace graph

static thread_local std::string g_err;

void set_last_error(const std::string& m) { g_err = m; }
std::string last_error_string() { return g_err; }

[[noreturn]] void throw_hip(hipError_t e, const char* what, const char* file, int line) {
    const std::string msg = std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ") at " +
                            file + ":" + std::to_string(line) + ": " + what;
    throw Error(e == hipErrorOutOfMemory ? CAPSMI_ERR_OUT_OF_MEMORY : CAPSMI_ERR_DEVICE, msg);
}

// Device blocks are recycled per session: a freed block goes to its session's free list and the
// next request of the same size class in that session takes it back.  Every block of a session is
// used on the session's current stream, so stream order keeps reuse safe (everything that used the
// block was queued before whatever reuses it); a stream switch first drains the old stream
// (capsmi_session_set_stream / _use_stream), after which every cached block is idle.  This takes
// the hipMallocAsync / hipFreeAsync calls -- 0.1-0.2 ms of host time each for the multi-GiB
// layout buffers, during which the device idles -- out of every query after the first.  The lists
// are trimmed when an allocation fails (every session's), when the cached bytes of all sessions
// pass CAPSMI_CACHE_BYTES (default 1/4 of the device) and when the session is destroyed; a block
// freed after its session is gone goes straight back to the device.
struct AllocCtx {
    int device = 0;
    hipStream_t stream = nullptr;  // the owning session's current stream
    bool alive = true;
    std::multimap<size_t, void*> free;
};

namespace {

struct BlockCache {
    std::mutex mu;
    std::vector<std::weak_ptr<AllocCtx>> ctxs;  // every live session context (trim on OOM)
    size_t cached = 0, cap = 0;
};

BlockCache& block_cache() {
    static BlockCache* c = new BlockCache();  // never destroyed: DevBufs may die during exit
    return *c;
}

size_t size_class(size_t b) {  // <= 12.5% above the request
    if (b <= 4096) return 4096;
    size_t p = size_t(1) << (63 - __builtin_clzll(b));
    const size_t step = p / 8;
    return (b + step - 1) / step * step;
}

size_t cache_cap() {
    BlockCache& c = block_cache();
    static std::once_flag once;
    std::call_once(once, [&] {
        size_t fr = 0, tot = 0;
        if (const char* e = getenv("CAPSMI_CACHE_BYTES")) c.cap = std::max<size_t>(1, strtoull(e, nullptr, 10));
        else c.cap = hipMemGetInfo(&fr, &tot) == hipSuccess && tot ? tot / 4 : (size_t(16) << 30);
    });
    return c.cap;
}

// free every cached block of one context; caller holds mu
void trim_ctx_locked(BlockCache& c, AllocCtx& x) {
    for (auto& kv : x.free) {
        (void)hipFreeAsync(kv.second, x.stream);
        c.cached -= kv.first;
    }
    x.free.clear();
}

}  // namespace

DevBuf::~DevBuf() {
    if (!ptr) return;
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    if (!ctx || !ctx->alive) {  // the session is gone (its stream may be too): back to the device
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (ctx) (void)hipSetDevice(ctx->device);
        (void)hipFree(ptr);
        if (ctx) (void)hipSetDevice(dev);
        return;
    }
    ctx->free.emplace(bytes, ptr);
    c.cached += bytes;
    while (c.cached > cache_cap() && !ctx->free.empty()) {  // evict this session's largest blocks
        auto last = std::prev(ctx->free.end());
        (void)hipFreeAsync(last->second, ctx->stream);
        c.cached -= last->first;
        ctx->free.erase(last);
    }
}

Buf dev_alloc(size_t bytes, capsmi_session* s) {
    auto b = std::make_shared<DevBuf>();
    const size_t want = size_class(bytes ? bytes : 8);
    AllocCtx& x = *s->alloc;
    b->ctx = s->alloc;
    BlockCache& c = block_cache();
    (void)cache_cap();  // sized on the first allocation, not inside a destructor
    {
        std::lock_guard<std::mutex> g(c.mu);
        auto it = x.free.lower_bound(want);
        if (it != x.free.end() && it->first <= want + want / 4) {
            b->ptr = it->second;
            b->bytes = it->first;
            c.cached -= it->first;
            x.free.erase(it);
            return b;
        }
    }
    b->bytes = want;
    hipError_t e = hipMallocAsync(&b->ptr, want, s->stream);
    if (e == hipErrorOutOfMemory) {  // give every session's cached blocks back and try once more
        (void)hipGetLastError();
        (void)hipDeviceSynchronize();
        {
            std::lock_guard<std::mutex> g(c.mu);
            for (auto& w : c.ctxs)
                if (auto p = w.lock()) trim_ctx_locked(c, *p);
        }
        (void)hipDeviceSynchronize();
        hipMemPool_t pool;  // and the freed memory the stream-ordered pool still reserves
        if (hipDeviceGetDefaultMemPool(&pool, s->device) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
        e = hipMallocAsync(&b->ptr, want, s->stream);
    }
    if (e != hipSuccess) {
        b->ptr = nullptr;
        HIP_CHECK(e);
    }
    return b;
}

void alloc_ctx_open(capsmi_session* s) {
    s->alloc = std::make_shared<AllocCtx>();
    s->alloc->device = s->device;
    s->alloc->stream = s->stream;
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    c.ctxs.erase(std::remove_if(c.ctxs.begin(), c.ctxs.end(), [](const std::weak_ptr<AllocCtx>& w) { return w.expired(); }),
                 c.ctxs.end());
    c.ctxs.push_back(s->alloc);
}

// drain the old stream, then run the session (and its cache) on `st`
void alloc_ctx_switch(capsmi_session* s, hipStream_t st) {
    if (st == s->stream) return;
    HIP_CHECK(hipStreamSynchronize(s->stream));
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    s->stream = st;
    s->alloc->stream = st;
}

// session destroy: the stream is drained by the caller; every cached block goes back to the device
void alloc_ctx_close(capsmi_session* s) {
    BlockCache& c = block_cache();
    std::lock_guard<std::mutex> g(c.mu);
    trim_ctx_locked(c, *s->alloc);
    s->alloc->alive = false;
}

}  // namespace capsmi

using namespace capsmi;

namespace {

void set_err(const std::string& m) { g_err = m; }

#define API_BEGIN try {
#define API_END                                                         \
    }                                                                   \
    catch (const capsmi::Error& e) {                                    \
        set_err(e.what());                                              \
        return e.code;                                                  \
    }                                                                   \
    catch (const std::bad_alloc&) {                                     \
        set_err("host allocation failed");                              \
        return CAPSMI_ERR_OUT_OF_MEMORY;                                \
    }                                                                   \
    catch (const std::exception& e) {                                   \
        set_err(e.what());                                              \
        return CAPSMI_ERR_INTERNAL;                                     \
    }                                                                   \
    return CAPSMI_OK;

void need(const void* p, const char* what) {
    REQUIRE(p != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("null argument: ") + what);
}

void use_device(capsmi_session* s) { HIP_CHECK(hipSetDevice(s->device)); }

capsmi_table* new_table(capsmi_session* s, int64_t nrows) {
    auto* t = new capsmi_table();
    t->sess = s;
    t->nrows = nrows;
    return t;
}

int col_index(const capsmi_table* t, const char* name) {
    need(name, "column name");
    const int i = t->find(name);
    REQUIRE(i >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("no column named '") + name + "'");
    return i;
}

// gather every column of `t` at `idx` (n entries; -1 -> NULL)
void gather_into(capsmi_table* out, const capsmi_table* t, const Buf& idx, int64_t n, bool may_miss) {
    capsmi_session* s = t->sess;
    for (const Column& c : t->cols) {
        Column o;
        o.name = c.name;
        o.type = c.type;
        o.list = c.list;  // list rows are indices into the same store
        o.data = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
        if (c.valid || may_miss) o.valid = dev_alloc(n > 0 ? n : 1, s);
        gather_col(c.d(), c.v(), P<int64_t>(idx), n, P<int64_t>(o.data), P<uint8_t>(o.valid), s->stream);
        out->cols.push_back(std::move(o));
    }
}

KeyCols key_cols(const capsmi_table* t, const std::vector<int>& idx) {
    REQUIRE((int)idx.size() <= kMaxKeys, CAPSMI_ERR_NOT_IMPLEMENTED, "more than 8 key columns");
    for (int i : idx) no_list_key(t->cols[i].type, t->cols[i].name, "a key");
    KeyCols k;
    k.n = (int)idx.size();
    for (int i = 0; i < kMaxKeys; ++i) {
        k.data[i] = i < k.n ? t->cols[idx[i]].d() : nullptr;
        k.valid[i] = i < k.n ? t->cols[idx[i]].v() : nullptr;
    }
    return k;
}

// Grouping keys of any width (nulls compare equal, as groupBy / dropDuplicates treat them): keys
// beyond kMaxKeys are folded 8 at a time into a dense group-id column -- rows agree on the first
// columns iff their group ids agree -- which then joins the next columns.  `hold` keeps the
// folded columns alive while the returned KeyCols is in use.
KeyCols group_key_cols(capsmi_session* s, const capsmi_table* t, const std::vector<int>& idx, std::vector<Buf>& hold) {
    if ((int)idx.size() <= kMaxKeys) return key_cols(t, idx);
    for (int i : idx) no_list_key(t->cols[i].type, t->cols[i].name, "a key");
    KeyCols k;
    size_t next = 0;
    const int64_t* folded = nullptr;
    while (true) {
        k.n = 0;
        if (folded) {
            k.data[k.n] = folded;
            k.valid[k.n++] = nullptr;
        }
        while (k.n < kMaxKeys && next < idx.size()) {
            k.data[k.n] = t->cols[idx[next]].d();
            k.valid[k.n++] = t->cols[idx[next++]].v();
        }
        for (int i = k.n; i < kMaxKeys; ++i) k.data[i] = nullptr, k.valid[i] = nullptr;
        if (next == idx.size()) return k;
        HashTable ht;
        Buf sor, gid, rep;
        hash_build(s, k, t->nrows, /*skip_null_keys=*/false, ht, sor);
        (void)hash_group_ids(s, ht, sor, t->nrows, gid, rep);
        hold.push_back(gid);
        folded = P<int64_t>(gid);
    }
}

bool types_joinable(int a, int b) {
    const bool na = a == CAPSMI_I64 || a == CAPSMI_F64, nb = b == CAPSMI_I64 || b == CAPSMI_F64;
    return a == b || (na && nb);
}

// Join strategy (Spark picks broadcast-hash vs shuffled joins by size; this picks by key shape and
// build size): "direct" -- unique Long build keys in a dense range, a direct-address table; "hash"
// -- one global hash table, for builds whose table stays cache-resident; "radix" -- both sides
// radix-partitioned to LDS tables, for larger builds.  CAPSMI_JOIN=direct|hash|radix forces one for
// A/B runs (direct still falls back when the keys are not eligible).
enum JoinStrategy { JS_AUTO, JS_DIRECT, JS_HASH, JS_RADIX };  // Config::join
// from 2^22 build rows (a global table of ~128 MB, half the MALL) the radix join measured faster:
// 3.4 vs 3.9 ms at 2^22, 14.3 vs 16.2 at 2^24, 62.6 vs 70.1 at 2^26 (scripts/join_bench.py)
constexpr int64_t kRadixBuildRows = int64_t(1) << 22;

capsmi_table* join_impl(capsmi_table* l, capsmi_table* r, int jt, const std::vector<int>& lk,
                        const std::vector<int>& rk) {
    capsmi_session* s = l->sess;
    hipStream_t st = s->stream;
    for (const Column& a : l->cols)
        for (const Column& b : r->cols)
            REQUIRE(a.name != b.name, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    "join inputs share column '" + a.name + "' (RelationalPlanner renames to disjoint columns)");
    Buf li, ri;
    int64_t total = 0;
    bool lmiss = false, rmiss = false;
    if (jt == CAPSMI_JOIN_CROSS) {
        total = l->nrows * r->nrows;
        li = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
        ri = dev_alloc(sizeof(int64_t) * (total > 0 ? total : 1), s);
        cross_pairs(l->nrows, r->nrows, P<int64_t>(li), P<int64_t>(ri), st);
    } else {
        for (size_t i = 0; i < lk.size(); ++i)
            REQUIRE(types_joinable(l->cols[lk[i]].type, r->cols[rk[i]].type), CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    "join key types differ: " + l->cols[lk[i]].name + " vs " + r->cols[rk[i]].name);
        // inner: build on the smaller side; left outer / full outer: build right; right outer: build left
        bool build_left = false;
        if (jt == CAPSMI_JOIN_INNER) build_left = l->nrows < r->nrows;
        else if (jt == CAPSMI_JOIN_RIGHT_OUTER) build_left = true;
        capsmi_table* B = build_left ? l : r;
        capsmi_table* Pr = build_left ? r : l;
        KeyCols bk = key_cols(B, build_left ? lk : rk);
        KeyCols pk = key_cols(Pr, build_left ? rk : lk);
        // A Long key compared with a Double key: Spark's analyser casts the Long side to Double
        // (1 = 1.0 matches).  Equal-typed keys compare by their 64-bit words; Spark 2.2.1 does not
        // normalise -0.0 / NaN in join keys either (SPARK-26021 changed that only in 3.0).
        std::vector<Buf> widened;
        for (size_t i = 0; i < lk.size(); ++i) {
            const int bt = B->cols[(build_left ? lk : rk)[i]].type, pt = Pr->cols[(build_left ? rk : lk)[i]].type;
            if (bt == pt) continue;
            const bool widen_build = bt == CAPSMI_I64;
            KeyCols& kc = widen_build ? bk : pk;
            const int64_t rows = widen_build ? B->nrows : Pr->nrows;
            Buf w = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), s);
            i64_to_f64(kc.data[i], P<int64_t>(w), rows, st);
            kc.data[i] = P<int64_t>(w);
            widened.push_back(w);
        }
        const bool outer = jt != CAPSMI_JOIN_INNER;
        Buf pi, bi, matched;
        const JoinStrategy js = (JoinStrategy)s->cfg.join;
        bool done = false;
        if (jt != CAPSMI_JOIN_FULL_OUTER && (js == JS_AUTO || js == JS_DIRECT) && bk.n == 1 &&
            B->cols[(build_left ? lk : rk)[0]].type == CAPSMI_I64 && Pr->cols[(build_left ? rk : lk)[0]].type == CAPSMI_I64)
            done = direct_join(s, bk, B->nrows, pk, Pr->nrows, outer, pi, bi, &total);
        if (done) {
        } else if (jt != CAPSMI_JOIN_FULL_OUTER && (js == JS_RADIX || (js == JS_AUTO && B->nrows >= kRadixBuildRows))) {
            // radix-partitioned build / probe with LDS partition tables (k_rjoin.hip)
            total = radix_join(s, bk, B->nrows, pk, Pr->nrows, outer, pi, bi);
        } else {
            HashTable ht;
            Buf slot_of_row, slot_of_probe, offsets, rows;
            hash_build(s, bk, B->nrows, /*skip_null_keys=*/true, ht, slot_of_row);
            hash_group_rows(s, ht, slot_of_row, B->nrows, offsets, rows);
            hash_probe(s, pk, bk, Pr->nrows, ht, slot_of_probe);
            total = join_expand(s, slot_of_probe, Pr->nrows, ht, offsets, rows, outer, pi, bi,
                                jt == CAPSMI_JOIN_FULL_OUTER ? &matched : nullptr, B->nrows);
        }
        if (outer) (build_left ? lmiss : rmiss) = true;
        if (jt == CAPSMI_JOIN_FULL_OUTER) {
            // append build (right) rows that never matched, left side NULL
            Buf unm_flags = dev_alloc(B->nrows > 0 ? B->nrows : 1, s);
            invert_u8(P<uint8_t>(matched), P<uint8_t>(unm_flags), B->nrows, st);
            Buf unm_idx;
            const int64_t nu = flags_to_indices(s, P<uint8_t>(unm_flags), B->nrows, unm_idx);
            Buf pi2 = dev_alloc(sizeof(int64_t) * (total + nu > 0 ? total + nu : 1), s);
            Buf bi2 = dev_alloc(sizeof(int64_t) * (total + nu > 0 ? total + nu : 1), s);
            if (total) {
                HIP_CHECK(hipMemcpyAsync(P<void>(pi2), P<void>(pi), sizeof(int64_t) * total, hipMemcpyDeviceToDevice, st));
                HIP_CHECK(hipMemcpyAsync(P<void>(bi2), P<void>(bi), sizeof(int64_t) * total, hipMemcpyDeviceToDevice, st));
            }
            fill_i64(P<int64_t>(pi2) + total, -1, nu, st);
            if (nu) HIP_CHECK(hipMemcpyAsync(P<int64_t>(bi2) + total, P<void>(unm_idx), sizeof(int64_t) * nu,
                                             hipMemcpyDeviceToDevice, st));
            total += nu;
            pi = pi2;
            bi = bi2;
            lmiss = rmiss = true;
        }
        li = build_left ? bi : pi;
        ri = build_left ? pi : bi;
    }
    capsmi_table* out = new_table(s, total);
    gather_into(out, l, li, total, lmiss);
    capsmi_table tmp;
    tmp.sess = s;
    gather_into(&tmp, r, ri, total, rmiss);
    for (auto& c : tmp.cols) out->cols.push_back(std::move(c));
    return out;
}

// stable row permutation ordering `t` by keys (LSD: last key first; per key a 64-bit value pass,
// then an 8-bit pass on the null flag so that the flag dominates)
Buf order_perm(capsmi_table* t, const std::vector<int>& keys, const std::vector<int>& desc) {
    capsmi_session* s = t->sess;
    hipStream_t st = s->stream;
    const int64_t n = t->nrows;
    Buf perm = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    iota_i64(P<int64_t>(perm), 0, n, st);
    if (n <= 1) return perm;
    Buf kbuf = dev_alloc(sizeof(uint64_t) * n, s);
    for (int k = (int)keys.size() - 1; k >= 0; --k) {
        const Column& c = t->cols[keys[k]];
        no_list_key(c.type, c.name, "a sort key");
        order_keys(s, c.d(), c.v(), c.type, desc[k] != 0, false, P<int64_t>(perm), n, P<uint64_t>(kbuf));
        radix_sort_pairs(s, P<uint64_t>(kbuf), P<int64_t>(perm), n, 0, 64);
        if (c.valid) {
            order_keys(s, c.d(), c.v(), c.type, desc[k] != 0, true, P<int64_t>(perm), n, P<uint64_t>(kbuf));
            radix_sort_pairs(s, P<uint64_t>(kbuf), P<int64_t>(perm), n, 0, 8);
        }
    }
    return perm;
}

std::vector<int> names_to_idx(const capsmi_table* t, int32_t n, const char* const* names) {
    std::vector<int> v;
    for (int i = 0; i < n; ++i) v.push_back(col_index(t, names[i]));
    return v;
}

const Column& rel_col(const capsmi_table* t, const char* name) {
    const Column& c = t->cols[col_index(t, name)];
    REQUIRE(c.type == CAPSMI_I64, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("id column '") + name + "' must be Long");
    REQUIRE(c.valid == nullptr, CAPSMI_ERR_UNSUPPORTED,
            std::string("fused path needs a non-nullable id column ('") + name + "'; EntityTable.verify)");
    return c;
}

void check_bitmap(const capsmi_bitmap* b, const char* what) {
    need(b, what);
}

}  // namespace

// =============================== C ABI ========================================================
namespace capsmi {
namespace {
bool parse_int(const char* v, int64_t lo, int64_t hi, int64_t& out) {
    if (!v || !*v) return false;
    char* end = nullptr;
    const long long x = strtoll(v, &end, 10);
    if (*end != '\0' || x < lo || x > hi) return false;
    out = x;
    return true;
}
bool parse_choice(const char* v, std::initializer_list<const char*> names, int& out) {
    int k = 0;
    for (const char* n : names) {
        if (v && std::string(v) == n) {
            out = k;
            return true;
        }
        ++k;
    }
    return false;
}
// one knob from `v` (never NULL here); false = unknown name or bad value (c unchanged)
bool apply(Config& c, const std::string& name, const char* v) {
    int64_t x = 0;
    int k = 0;
    if (name == "CAPSMI_JOIN") {
        if (!parse_choice(v, {"auto", "direct", "hash", "radix"}, k)) return false;
        c.join = k;
    } else if (name == "CAPSMI_COUNT") {
        if (!parse_choice(v, {"rec", "atomic"}, k)) return false;
        c.count_atomic = k == 1;
    } else if (name == "CAPSMI_REC_FULL") {
        if (!parse_int(v, 0, 1, x)) return false;
        c.rec_full = x != 0;
    } else if (name == "CAPSMI_GROUPED") {
        if (!parse_choice(v, {"sets", "keys"}, k)) return false;
        c.grouped_keys = k == 1;
    } else if (name == "CAPSMI_PAIRS") {
        if (!parse_choice(v, {"auto", "packed", "uint2"}, k)) return false;
        c.pairs = k;
    } else if (name == "CAPSMI_TRI_BUILD") {
        if (!parse_choice(v, {"direct", "sorted"}, k)) return false;
        c.tri_sorted_build = k == 1;
    } else if (name == "CAPSMI_TRI_DEG_SAMPLE") {
        if (!parse_int(v, 0, 1 << 20, x)) return false;
        c.tri_deg_sample = (int)x;
    } else if (name == "CAPSMI_TRI_SPLIT") {
        if (!parse_int(v, 0, 1, x)) return false;
        c.tri_split = x != 0;
    } else if (name == "CAPSMI_TRI_VMODE_T") {
        if (!parse_int(v, 0, 1 << 30, x)) return false;
        c.tri_vmode_t = (int)x;
    } else if (name == "CAPSMI_UND") {
        if (!parse_choice(v, {"part", "stream"}, k)) return false;
        c.und_stream = k == 1;
    } else if (name == "CAPSMI_VL_BITS") {
        if (!parse_int(v, 2, 64, x)) return false;
        c.vl_bits = (int)x;
    } else if (name == "CAPSMI_VL_SUBLOG") {
        if (!parse_int(v, -1, 5, x)) return false;
        c.vl_sublog = (int)x;
    } else if (name == "CAPSMI_VL_F2") {
        if (!parse_int(v, 0, 1, x)) return false;
        c.vl_f2 = x != 0;
    } else if (name == "CAPSMI_COLL_CHUNK") {
        if (!parse_int(v, 1, int64_t(1) << 40, x)) return false;
        c.coll_chunk = x;
    } else if (name == "CAPSMI_INGEST_THREADS") {
        if (!parse_int(v, 0, 1024, x)) return false;
        c.ingest_threads = (int)x;
    } else {
        return false;
    }
    return true;
}
// every knob with its default's text (Config's initialisers)
const std::pair<const char*, const char*> kKnobs[] = {
    {"CAPSMI_JOIN", "auto"},         {"CAPSMI_COUNT", "rec"},        {"CAPSMI_REC_FULL", "1"},
    {"CAPSMI_GROUPED", "sets"},      {"CAPSMI_PAIRS", "auto"},       {"CAPSMI_TRI_BUILD", "direct"},
    {"CAPSMI_TRI_DEG_SAMPLE", "0"},  {"CAPSMI_TRI_SPLIT", "1"},      {"CAPSMI_TRI_VMODE_T", "256"},
    {"CAPSMI_UND", "part"},          {"CAPSMI_VL_BITS", "8"},        {"CAPSMI_VL_SUBLOG", "-1"},
    {"CAPSMI_VL_F2", "0"},           {"CAPSMI_COLL_CHUNK", "67108864"}, {"CAPSMI_INGEST_THREADS", "0"}};
}  // namespace

Config config_from_env() {
    Config c;
    for (const auto& k : kKnobs)
        if (const char* e = getenv(k.first))
            if (!apply(c, k.first, e)) fprintf(stderr, "capsmi: ignoring %s=%s (not a valid value)\n", k.first, e);
    return c;
}

bool config_set(Config& c, const char* name, const char* value) {
    if (!name) return false;
    const std::string n(name);
    if (value) return apply(c, n, value);
    for (const auto& k : kKnobs)  // back to the environment's value, or the default
        if (n == k.first) {
            const char* e = getenv(k.first);
            Config t = c;
            if (!(e && apply(t, n, e))) apply(t, n, k.second);
            c = t;
            return true;
        }
    return false;
}
}  // namespace capsmi

extern "C" {

size_t capsmi_last_error(char* buf, size_t n) {
    if (buf && n) {
        const size_t k = std::min(n - 1, g_err.size());
        std::memcpy(buf, g_err.data(), k);
        buf[k] = 0;
    }
    return g_err.size();
}

const char* capsmi_version(void) { return "capsmi 0.1.0 (gfx950)"; }

capsmi_status capsmi_session_create(int32_t device, capsmi_session** out) {
    API_BEGIN
    need(out, "out");
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    REQUIRE(device >= 0 && device < n, CAPSMI_ERR_ILLEGAL_ARGUMENT, "no such HIP device " + std::to_string(device));
    HIP_CHECK(hipSetDevice(device));
    auto* s = new capsmi_session();
    s->device = device;
    s->cfg = capsmi::config_from_env();  // the knobs, once
    HIP_CHECK(hipStreamCreateWithFlags(&s->own_stream, hipStreamNonBlocking));
    s->stream = s->own_stream;
    alloc_ctx_open(s);
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    s->num_cus = prop.multiProcessorCount;
    HIP_CHECK(hipHostMalloc((void**)&s->pinned, 64, hipHostMallocDefault));
    HIP_CHECK(hipEventCreateWithFlags(&s->ev_read, hipEventDisableTiming));
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
        // keep freed pool memory mapped (no unmap / remap per query); CAPSMI_POOL_KEEP_BYTES caps what the
        // pool keeps when several processes share one device (a rehearsal of N ranks on one GPU)
        uint64_t thr = UINT64_MAX;
        if (const char* e = getenv("CAPSMI_POOL_KEEP_BYTES")) thr = strtoull(e, nullptr, 10);
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
    *out = s;
    API_END
}

capsmi_status capsmi_session_destroy(capsmi_session* s) {
    API_BEGIN
    if (!s) return CAPSMI_OK;
    use_device(s);
    (void)hipStreamSynchronize(s->stream);
    (void)hipStreamSynchronize(s->own_stream);
    alloc_ctx_close(s);
    (void)hipStreamSynchronize(s->stream);
    (void)hipStreamSynchronize(s->own_stream);
    for (auto& p : s->pending) {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    for (hipEvent_t e : s->ev_pool) (void)hipEventDestroy(e);
    (void)hipHostFree(s->pinned);
    if (s->ev_read) (void)hipEventDestroy(s->ev_read);
    (void)hipStreamDestroy(s->own_stream);
    delete s;
    API_END
}

capsmi_status capsmi_session_set_stream(capsmi_session* s, void* hip_stream) {
    API_BEGIN
    need(s, "session");
    use_device(s);
    alloc_ctx_switch(s, hip_stream ? (hipStream_t)hip_stream : s->own_stream);
    API_END
}

capsmi_status capsmi_session_use_stream(capsmi_session* s, void* hip_stream) {
    API_BEGIN
    need(s, "session");
    use_device(s);
    alloc_ctx_switch(s, (hipStream_t)hip_stream);
    API_END
}

capsmi_status capsmi_session_set_profiling(capsmi_session* s, int32_t enabled) {
    API_BEGIN
    need(s, "session");
    s->prof = enabled != 0;
    if (s->prof) {  // the timers' events made here, not inside the timed queries
        use_device(s);
        while (s->ev_pool.size() < 1024) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            s->ev_pool.push_back(e);
        }
    }
    API_END
}

capsmi_status capsmi_session_set_profiling_names(capsmi_session* s, const char* names) {
    API_BEGIN
    need(s, "session");
    s->prof_names.clear();
    for (const char* p = names; p && *p;) {
        const char* e = strchr(p, ',');
        const std::string nm = e ? std::string(p, e) : std::string(p);
        if (!nm.empty()) s->prof_names.insert(nm);
        p = e ? e + 1 : nullptr;
    }
    API_END
}

capsmi_status capsmi_session_set_params(capsmi_session* s, int32_t nparams, const capsmi_param* params) {
    API_BEGIN
    need(s, "session");
    REQUIRE(nparams >= 0 && (nparams == 0 || params), CAPSMI_ERR_ILLEGAL_ARGUMENT, "parameters");
    std::vector<capsmi_session::Param> ps(nparams);
    for (int i = 0; i < nparams; ++i) {
        const capsmi_param& p = params[i];
        REQUIRE(p.type >= CAPSMI_I64 && p.type <= CAPSMI_STR, CAPSMI_ERR_ILLEGAL_ARGUMENT, "parameter type");
        REQUIRE(p.is_list ? p.count >= 0 : p.count == 1, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "a scalar parameter has one value, a list zero or more");
        REQUIRE(p.count == 0 || p.values, CAPSMI_ERR_ILLEGAL_ARGUMENT, "parameter values");
        ps[i].type = p.type;
        ps[i].list = p.is_list != 0;
        ps[i].values.assign(p.values, p.values + p.count);
    }
    s->params = std::move(ps);
    API_END
}

capsmi_status capsmi_session_kernel_bytes(capsmi_session* s, const char* name, double* bytes) {
    API_BEGIN
    need(s, "session");
    need(name, "name");
    need(bytes, "bytes");
    auto it = s->alg_bytes.find(name);
    *bytes = it == s->alg_bytes.end() ? 0.0 : it->second;
    if (it != s->alg_bytes.end()) s->alg_bytes.erase(it);
    API_END
}

capsmi_status capsmi_session_kernel_time(capsmi_session* s, const char* name, int64_t* launches, double* total_ms) {
    API_BEGIN
    need(s, "session");
    need(name, "name");
    use_device(s);
    for (auto& p : s->pending) {
        HIP_CHECK(hipEventSynchronize(p.b));
        float ms = 0.f;
        HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
        auto& t = s->totals[p.name];
        t.first += 1;
        t.second += ms;
        s->ev_pool.push_back(p.a);
        s->ev_pool.push_back(p.b);
    }
    s->pending.clear();
    auto it = s->totals.find(name);
    if (launches) *launches = it == s->totals.end() ? 0 : it->second.first;
    if (total_ms) *total_ms = it == s->totals.end() ? 0.0 : it->second.second;
    if (it != s->totals.end()) s->totals.erase(it);
    API_END
}

capsmi_status capsmi_session_set_config(capsmi_session* s, const char* name, const char* value) {
    API_BEGIN
    need(s, "session");
    REQUIRE(capsmi::config_set(s->cfg, name, value), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string("unknown configuration knob or value: ") + (name ? name : "(null)") + " = " +
                (value ? value : "(default)"));
    API_END
}

capsmi_status capsmi_config_check(const char* name, const char* value) {
    API_BEGIN
    capsmi::Config c;
    REQUIRE(capsmi::config_set(c, name, value), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string("unknown configuration knob or value: ") + (name ? name : "(null)") + " = " +
                (value ? value : "(default)"));
    API_END
}

capsmi_status capsmi_session_sync(capsmi_session* s) {
    API_BEGIN
    need(s, "session");
    use_device(s);
    HIP_CHECK(hipStreamSynchronize(s->stream));
    API_END
}

static capsmi_status table_from(capsmi_session* s, int32_t ncols, const capsmi_col_desc* cols, int64_t nrows,
                                capsmi_table** out, hipMemcpyKind kind) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(nrows >= 0 && ncols >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "negative table size");
    use_device(s);
    std::unordered_set<std::string> seen;
    auto* t = new_table(s, nrows);
    std::unique_ptr<capsmi_table> guard(t);
    for (int i = 0; i < ncols; ++i) {
        need(cols[i].name, "column name");
        REQUIRE(seen.insert(cols[i].name).second, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                std::string("duplicate column '") + cols[i].name + "'");
        const int32_t ty = cols[i].type;
        const bool narrow = ty >= CAPSMI_IN_I32 && ty <= CAPSMI_IN_BOOL8;
        REQUIRE((ty >= CAPSMI_I64 && ty <= CAPSMI_STR) || narrow, CAPSMI_ERR_ILLEGAL_ARGUMENT, "bad column type");
        REQUIRE(nrows == 0 || cols[i].data, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null column data");
        Column c;
        c.name = cols[i].name;
        c.type = ty;
        c.data = dev_alloc(sizeof(int64_t) * (nrows > 0 ? nrows : 1), s);
        if (narrow) {
            // Byte/Short/Integer -> Long, Float -> Double (DataFrameOps.withCypherCompatibleTypes)
            const size_t w = ty == CAPSMI_IN_I32 || ty == CAPSMI_IN_F32 ? 4 : (ty == CAPSMI_IN_I16 ? 2 : 1);
            c.type = ty == CAPSMI_IN_F32 ? CAPSMI_F64 : (ty == CAPSMI_IN_BOOL8 ? CAPSMI_BOOL : CAPSMI_I64);
            if (nrows) {
                Buf raw = dev_alloc(w * nrows, s);
                HIP_CHECK(hipMemcpyAsync(P<void>(raw), cols[i].data, w * nrows, kind, s->stream));
                widen_words(P<void>(raw), ty, P<int64_t>(c.data), nrows, s->stream);
                if (kind == hipMemcpyHostToDevice) HIP_CHECK(hipStreamSynchronize(s->stream));
            }
        } else if (nrows) {
            HIP_CHECK(hipMemcpyAsync(P<void>(c.data), cols[i].data, sizeof(int64_t) * nrows, kind, s->stream));
        }
        if (cols[i].valid) {
            c.valid = dev_alloc(nrows > 0 ? nrows : 1, s);
            if (nrows) HIP_CHECK(hipMemcpyAsync(P<void>(c.valid), cols[i].valid, nrows, kind, s->stream));
        }
        t->cols.push_back(std::move(c));
    }
    if (kind == hipMemcpyHostToDevice) HIP_CHECK(hipStreamSynchronize(s->stream));  // host buffers may go away
    *out = guard.release();
    API_END
}

capsmi_status capsmi_table_from_host(capsmi_session* s, int32_t ncols, const capsmi_col_desc* cols, int64_t nrows,
                                     capsmi_table** out) {
    return table_from(s, ncols, cols, nrows, out, hipMemcpyHostToDevice);
}

capsmi_status capsmi_table_from_device(capsmi_session* s, int32_t ncols, const capsmi_col_desc* cols, int64_t nrows,
                                       capsmi_table** out) {
    return table_from(s, ncols, cols, nrows, out, hipMemcpyDeviceToDevice);
}

capsmi_status capsmi_table_retain(capsmi_table* t) {
    API_BEGIN
    need(t, "table");
    t->refs.fetch_add(1);
    API_END
}

capsmi_status capsmi_table_release(capsmi_table* t) {
    API_BEGIN
    if (!t) return CAPSMI_OK;
    if (t->refs.fetch_sub(1) == 1) {
        use_device(t->sess);
        delete t;
    }
    API_END
}

capsmi_status capsmi_table_size(const capsmi_table* t, int64_t* out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    M(t);
    *out = t->nrows;
    API_END
}

capsmi_status capsmi_table_num_columns(const capsmi_table* t, int32_t* out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    *out = (int32_t)t->cols.size();
    API_END
}

capsmi_status capsmi_table_column_name(const capsmi_table* t, int32_t col, char* buf, size_t n) {
    API_BEGIN
    need(t, "table");
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    const std::string& nm = t->cols[col].name;
    REQUIRE(buf && n > nm.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "name buffer too small");
    std::memcpy(buf, nm.c_str(), nm.size() + 1);
    API_END
}

capsmi_status capsmi_table_column_type(const capsmi_table* t, int32_t col, int32_t* out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    *out = t->cols[col].type;
    API_END
}

capsmi_status capsmi_table_column_index(const capsmi_table* t, const char* name, int32_t* out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    need(name, "name");
    *out = t->find(name);
    API_END
}

capsmi_status capsmi_table_column_nullable(const capsmi_table* t, int32_t col, int32_t* out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    *out = t->cols[col].nullable() ? 1 : 0;
    API_END
}

capsmi_status capsmi_table_schema(const capsmi_table* t, int32_t* ncols, char* names, size_t names_len, int32_t* types,
                                  int32_t* nullable, int32_t max_cols) {
    API_BEGIN
    need(t, "table");
    need(ncols, "ncols");
    *ncols = (int32_t)t->cols.size();
    size_t pos = 0;
    for (size_t i = 0; i < t->cols.size() && (int32_t)i < max_cols; ++i) {
        const std::string& nm = t->cols[i].name;
        if (names) {
            REQUIRE(pos + nm.size() + 1 <= names_len, CAPSMI_ERR_ILLEGAL_ARGUMENT, "name buffer too small");
            std::memcpy(names + pos, nm.c_str(), nm.size() + 1);
        }
        pos += nm.size() + 1;
        if (types) types[i] = t->cols[i].type;
        if (nullable) nullable[i] = t->cols[i].nullable() ? 1 : 0;
    }
    API_END
}

capsmi_status capsmi_table_export(const capsmi_table* t, int32_t col, void* host_data, uint8_t* host_valid,
                                  int64_t offset, int64_t n) {
    API_BEGIN
    need(t, "table");
    M(t);
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    REQUIRE(offset >= 0 && n >= 0 && offset + n <= t->nrows, CAPSMI_ERR_ILLEGAL_ARGUMENT, "export range out of bounds");
    use_device(t->sess);
    const Column& c = t->cols[col];
    hipStream_t st = t->sess->stream;
    if (c.host && !c.valid && c.offset + offset + n <= (int64_t)c.host->size()) {  // host-built words
        if (n && host_data) std::memcpy(host_data, c.host->data() + c.offset + offset, sizeof(int64_t) * n);
        if (n && host_valid) std::memset(host_valid, 1, n);
        return CAPSMI_OK;
    }
    if (n && host_data)
        HIP_CHECK(hipMemcpyAsync(host_data, c.d() + offset, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
    if (n && host_valid) {
        if (c.valid) HIP_CHECK(hipMemcpyAsync(host_valid, c.v() + offset, n, hipMemcpyDeviceToHost, st));
        else std::memset(host_valid, 1, n);
    }
    HIP_CHECK(hipStreamSynchronize(st));
    API_END
}

capsmi_status capsmi_table_export_list(const capsmi_table* t, int32_t col, int64_t offset, int64_t n,
                                       int64_t* host_offsets, uint8_t* host_valid, void* host_values,
                                       int64_t values_cap, int64_t* nvalues) {
    API_BEGIN
    need(t, "table");
    need(nvalues, "nvalues");
    M(t);
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    REQUIRE(offset >= 0 && n >= 0 && offset + n <= t->nrows, CAPSMI_ERR_ILLEGAL_ARGUMENT, "export range out of bounds");
    const Column& c = t->cols[col];
    REQUIRE(is_list_type(c.type) && c.list, CAPSMI_ERR_ILLEGAL_ARGUMENT, "column '" + c.name + "' is not a list column");
    use_device(t->sess);
    hipStream_t st = t->sess->stream;
    const ListStore& L = *c.list;
    // the rows' list indices and validity first; then only the span of the store those rows reference
    // (the lists of a slice of a group result are one contiguous run of the store), so exporting a
    // slice moves the slice's lists, and the size probe (host_values == NULL) moves no values at all
    std::vector<int64_t> idx(n);
    std::vector<uint8_t> ok(n, 1);
    if (n) HIP_CHECK(hipMemcpyAsync(idx.data(), c.d() + offset, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
    if (n && c.valid) HIP_CHECK(hipMemcpyAsync(ok.data(), c.v() + offset, n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t lmin = INT64_MAX, lmax = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (!ok[i]) continue;
        REQUIRE(idx[i] >= 0 && idx[i] < L.nlists, CAPSMI_ERR_INTERNAL, "list row index out of range");
        lmin = std::min(lmin, idx[i]);
        lmax = std::max(lmax, idx[i]);
    }
    std::vector<int64_t> off;  // offsets of lists [lmin, lmax + 1]
    if (lmax >= 0) {
        off.resize(lmax - lmin + 2);
        HIP_CHECK(hipMemcpyAsync(off.data(), P<int64_t>(L.offsets) + lmin, sizeof(int64_t) * off.size(),
                                 hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i)
        if (ok[i]) total += off[idx[i] - lmin + 1] - off[idx[i] - lmin];
    *nvalues = total;
    if (!host_values) return CAPSMI_OK;
    need(host_offsets, "host_offsets");
    REQUIRE(values_cap >= total, CAPSMI_ERR_ILLEGAL_ARGUMENT, "list value buffer too small");
    std::vector<int64_t> vals;  // values of the span
    if (lmax >= 0 && off.back() > off.front()) {
        vals.resize(off.back() - off.front());
        HIP_CHECK(hipMemcpyAsync(vals.data(), P<int64_t>(L.values) + off.front(), sizeof(int64_t) * vals.size(),
                                 hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
    }
    int64_t* out = static_cast<int64_t*>(host_values);
    int64_t pos = 0;
    for (int64_t i = 0; i < n; ++i) {
        host_offsets[i] = pos;
        if (host_valid) host_valid[i] = ok[i];
        if (!ok[i]) continue;
        const int64_t b = off[idx[i] - lmin] - off.front(), e = off[idx[i] - lmin + 1] - off.front();
        for (int64_t k = b; k < e; ++k) out[pos++] = vals[k];
    }
    host_offsets[n] = pos;
    API_END
}

capsmi_status capsmi_table_column_device_ptr(const capsmi_table* t, int32_t col, const void** data,
                                             const uint8_t** valid) {
    API_BEGIN
    need(t, "table");
    M(t);
    REQUIRE(col >= 0 && col < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "column index out of range");
    if (data) *data = t->cols[col].d();
    if (valid) *valid = t->cols[col].v();
    API_END
}

}  // extern "C"

// Eager Table[T] operators over materialised inputs.  The public entry points (plan.hip) build lazy
// plan nodes; materialisation runs these (or a fused kernel the recogniser picked).
namespace capsmi {

// ---- Table[T] operators ---------------------------------------------------------------------
capsmi_status eager_select(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    auto idx = names_to_idx(t, ncols, cols);
    auto* o = new_table(t->sess, t->nrows);
    for (int i : idx) o->cols.push_back(t->cols[i]);
    *out = o;
    API_END
}

capsmi_status eager_drop(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    std::unordered_set<std::string> d;
    for (int i = 0; i < ncols; ++i) d.insert(cols[i]);  // Spark drop ignores unknown names
    auto* o = new_table(t->sess, t->nrows);
    for (const Column& c : t->cols)
        if (!d.count(c.name)) o->cols.push_back(c);
    *out = o;
    API_END
}

capsmi_status eager_with_column_renamed(capsmi_table* t, const char* old_name, const char* new_name,
                                         capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    need(new_name, "new name");
    const int i = col_index(t, old_name);
    const int j = t->find(new_name);
    REQUIRE(j < 0 || j == i, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("column '") + new_name + "' already exists");
    auto* o = new_table(t->sess, t->nrows);
    o->cols = t->cols;
    o->cols[i].name = new_name;
    *out = o;
    API_END
}

capsmi_status eager_filter(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(nnodes == 0 || prog, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null program");
    capsmi_session* s = t->sess;
    use_device(s);
    Buf flags = dev_alloc(t->nrows > 0 ? t->nrows : 1, s);
    eval_predicate(s, t, nnodes, prog, P<uint8_t>(flags));
    Buf idx;
    const int64_t n = flags_to_indices(s, P<uint8_t>(flags), t->nrows, idx);
    auto* o = new_table(s, n);
    gather_into(o, t, idx, n, false);
    *out = o;
    API_END
}

// Filter followed by a projection: only the `keep` columns of the surviving rows are gathered
capsmi_status eager_filter_keep(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog,
                                const std::vector<std::string>& keep, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    capsmi_session* s = t->sess;
    use_device(s);
    Buf flags = dev_alloc(t->nrows > 0 ? t->nrows : 1, s);
    eval_predicate(s, t, nnodes, prog, P<uint8_t>(flags));
    Buf idx;
    const int64_t n = flags_to_indices(s, P<uint8_t>(flags), t->nrows, idx);
    capsmi_table kept;
    kept.sess = s;
    kept.nrows = t->nrows;
    for (const std::string& k : keep) kept.cols.push_back(t->cols[col_index(t, k.c_str())]);
    auto* o = new_table(s, n);
    gather_into(o, &kept, idx, n, false);
    *out = o;
    API_END
}

capsmi_status eager_with_columns(capsmi_table* t, int32_t ncols, const capsmi_expr_column* cols, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    capsmi_session* s = t->sess;
    use_device(s);
    auto* o = new_table(s, t->nrows);
    o->cols = t->cols;
    for (int i = 0; i < ncols; ++i) {
        need(cols[i].name, "column name");
        Column c;
        if (cols[i].nnodes == 1 && cols[i].prog[0].op == CAPSMI_X_COL) {  // an alias: shares the buffers
            REQUIRE(cols[i].prog[0].arg >= 0 && cols[i].prog[0].arg < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    "column index out of range");
            c = t->cols[cols[i].prog[0].arg];
            c.name = cols[i].name;
            const int j = o->find(c.name);
            if (j >= 0) o->cols[j] = std::move(c);
            else o->cols.push_back(std::move(c));
            continue;
        }
        c.name = cols[i].name;
        c.data = dev_alloc(sizeof(int64_t) * (t->nrows > 0 ? t->nrows : 1), s);
        c.valid = dev_alloc(t->nrows > 0 ? t->nrows : 1, s);
        eval_expr(s, t, cols[i].nnodes, cols[i].prog, P<int64_t>(c.data), P<uint8_t>(c.valid), &c.type);
        const int j = o->find(c.name);
        if (j >= 0) o->cols[j] = std::move(c);  // replaced in place (SparkTable.scala:82-87)
        else o->cols.push_back(std::move(c));
    }
    *out = o;
    API_END
}

capsmi_status eager_join(capsmi_table* l, capsmi_table* r, int32_t join_type, int32_t npairs,
                          const char* const* lcols, const char* const* rcols, capsmi_table** out) {
    API_BEGIN
    need(l, "left");
    need(r, "right");
    need(out, "out");
    REQUIRE(l->sess == r->sess, CAPSMI_ERR_ILLEGAL_ARGUMENT, "tables belong to different sessions");
    REQUIRE(join_type >= CAPSMI_JOIN_INNER && join_type <= CAPSMI_JOIN_CROSS, CAPSMI_ERR_ILLEGAL_ARGUMENT, "join type");
    REQUIRE(join_type == CAPSMI_JOIN_CROSS || npairs > 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "equi-join needs key pairs");
    use_device(l->sess);
    std::vector<int> lk = names_to_idx(l, join_type == CAPSMI_JOIN_CROSS ? 0 : npairs, lcols);
    std::vector<int> rk = names_to_idx(r, join_type == CAPSMI_JOIN_CROSS ? 0 : npairs, rcols);
    *out = join_impl(l, r, join_type, lk, rk);
    API_END
}

capsmi_status eager_union_all(capsmi_table* a, capsmi_table* b, capsmi_table** out) {
    API_BEGIN
    need(a, "left");
    need(b, "right");
    need(out, "out");
    REQUIRE(a->cols.size() == b->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "union all: column counts differ");
    for (size_t i = 0; i < a->cols.size(); ++i)
        REQUIRE(a->cols[i].type == b->cols[i].type, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "Equal column data types for union all (differing nullability is OK): " + a->cols[i].name + " vs " +
                    b->cols[i].name);
    capsmi_session* s = a->sess;
    use_device(s);
    const int64_t n = a->nrows + b->nrows;
    auto* o = new_table(s, n);
    for (size_t i = 0; i < a->cols.size(); ++i) {
        const Column &x = a->cols[i], &y = b->cols[i];
        Column c;
        c.name = x.name;  // positional union, left names (Dataset.union)
        c.type = x.type;
        c.data = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
        if (a->nrows)
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(c.data), x.d(), sizeof(int64_t) * a->nrows, hipMemcpyDeviceToDevice, s->stream));
        if (b->nrows)
            HIP_CHECK(hipMemcpyAsync(P<int64_t>(c.data) + a->nrows, y.d(), sizeof(int64_t) * b->nrows,
                                     hipMemcpyDeviceToDevice, s->stream));
        if (is_list_type(x.type)) {
            REQUIRE(x.list && y.list, CAPSMI_ERR_INTERNAL, "list column without a store");
            // lists of both sides in one store: b's lists follow a's, b's row indices shift by a's list count
            c.list = x.list;
            if (x.list != y.list) {
                c.list = concat_lists(s, *x.list, *y.list);
                add_i64(P<int64_t>(c.data) + a->nrows, x.list->nlists, b->nrows, s->stream);
            }
        }
        if (x.valid || y.valid) {
            c.valid = dev_alloc(n > 0 ? n : 1, s);
            if (x.valid) { if (a->nrows) HIP_CHECK(hipMemcpyAsync(P<uint8_t>(c.valid), x.v(), a->nrows, hipMemcpyDeviceToDevice, s->stream)); }
            else fill_u8(P<uint8_t>(c.valid), 1, a->nrows, s->stream);
            if (y.valid) { if (b->nrows) HIP_CHECK(hipMemcpyAsync(P<uint8_t>(c.valid) + a->nrows, y.v(), b->nrows, hipMemcpyDeviceToDevice, s->stream)); }
            else fill_u8(P<uint8_t>(c.valid) + a->nrows, 1, b->nrows, s->stream);
        }
        o->cols.push_back(std::move(c));
    }
    *out = o;
    API_END
}

capsmi_status eager_order_by(capsmi_table* t, int32_t nkeys, const char* const* cols, const int32_t* descending,
                              capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    use_device(t->sess);
    auto keys = names_to_idx(t, nkeys, cols);
    std::vector<int> desc(nkeys);
    for (int i = 0; i < nkeys; ++i) desc[i] = descending ? descending[i] : 0;
    Buf perm = order_perm(t, keys, desc);
    auto* o = new_table(t->sess, t->nrows);
    gather_into(o, t, perm, t->nrows, false);
    *out = o;
    API_END
}

capsmi_status eager_skip(capsmi_table* t, int64_t n, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(n >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "negative skip");
    const int64_t k = std::min(n, t->nrows);
    auto* o = new_table(t->sess, t->nrows - k);
    o->cols = t->cols;
    for (auto& c : o->cols) c.offset += k;
    *out = o;
    API_END
}

capsmi_status eager_limit(capsmi_table* t, int64_t n, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(n >= 0 && n <= 2147483647LL, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "an integer: limit must fit an Int (SparkTable.scala:117)");
    auto* o = new_table(t->sess, std::min(n, t->nrows));
    o->cols = t->cols;
    *out = o;
    API_END
}

static capsmi_status distinct_impl(capsmi_table* t, const std::vector<int>& keys, capsmi_table** out) {
    API_BEGIN
    capsmi_session* s = t->sess;
    use_device(s);
    HashTable ht;
    Buf sor, gid, rep;
    std::vector<Buf> hold;
    hash_build(s, group_key_cols(s, t, keys, hold), t->nrows, /*skip_null_keys=*/false, ht, sor);
    const int64_t ng = hash_group_ids(s, ht, sor, t->nrows, gid, rep);
    auto* o = new_table(s, ng);
    gather_into(o, t, rep, ng, false);
    *out = o;
    API_END
}

capsmi_status eager_distinct(capsmi_table* t, capsmi_table** out) {
    if (!t || !out) { set_err("null argument"); return CAPSMI_ERR_ILLEGAL_ARGUMENT; }
    std::vector<int> keys;
    for (size_t i = 0; i < t->cols.size(); ++i) keys.push_back((int)i);
    return distinct_impl(t, keys, out);
}

capsmi_status eager_distinct_on(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    auto keys = names_to_idx(t, ncols, cols);
    const capsmi_status st = distinct_impl(t, keys, out);
    if (st != CAPSMI_OK) return st;
    API_END
}

capsmi_status eager_group(capsmi_table* t, int32_t nby, const char* const* by, int32_t naggs, const capsmi_agg* aggs,
                           capsmi_table** out) {
    API_BEGIN
    need(t, "table");
    need(out, "out");
    REQUIRE(naggs == 0 || aggs, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null aggregations");
    capsmi_session* s = t->sess;
    hipStream_t st = s->stream;
    use_device(s);
    const int64_t n = t->nrows;
    auto keys = names_to_idx(t, nby, by);
    Buf gid, rep;
    int64_t ng;
    HashTable ht;
    Buf sor;
    if (nby > 0) {
        std::vector<Buf> hold;
        hash_build(s, group_key_cols(s, t, keys, hold), n, /*skip_null_keys=*/false, ht, sor);
        ng = hash_group_ids(s, ht, sor, n, gid, rep);
    } else {
        ng = 1;  // global aggregate: exactly one row, also over empty input (Spark)
        gid = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
        fill_i64(P<int64_t>(gid), 0, n, st);
    }
    auto* o = new_table(s, ng);
    std::unique_ptr<capsmi_table> guard(o);
    if (nby > 0) {
        capsmi_table keyt;
        keyt.sess = s;
        keyt.nrows = n;
        for (int k : keys) keyt.cols.push_back(t->cols[k]);
        gather_into(o, &keyt, rep, ng, false);
    }
    for (int a = 0; a < naggs; ++a) {
        const capsmi_agg& ag = aggs[a];
        need(ag.output, "aggregate output name");
        Column c;
        c.name = ag.output;
        c.data = dev_alloc(sizeof(int64_t) * ng, s);
        const Column* in = nullptr;
        if (ag.kind != CAPSMI_AGG_COUNT_STAR) in = &t->cols[col_index(t, ag.input)];
        if (in && !(ag.kind == CAPSMI_AGG_COUNT && !ag.distinct)) no_list_key(in->type, in->name, "an aggregate input");
        switch (ag.kind) {
            case CAPSMI_AGG_COUNT_STAR:
                c.type = CAPSMI_I64;
                HIP_CHECK(hipMemsetAsync(P<void>(c.data), 0, sizeof(int64_t) * ng, st));
                agg_count(P<int64_t>(gid), nullptr, n, P<int64_t>(c.data), st);
                break;
            case CAPSMI_AGG_COUNT: {
                c.type = CAPSMI_I64;
                HIP_CHECK(hipMemsetAsync(P<void>(c.data), 0, sizeof(int64_t) * ng, st));
                if (!ag.distinct) {
                    agg_count(P<int64_t>(gid), in->v(), n, P<int64_t>(c.data), st);
                } else {
                    // countDistinct: distinct (group, value) pairs with a non-null value, counted per group
                    KeyCols k;
                    k.n = 2;
                    for (int i = 0; i < kMaxKeys; ++i) { k.data[i] = nullptr; k.valid[i] = nullptr; }
                    k.data[0] = P<int64_t>(gid);
                    k.data[1] = in->d();
                    k.valid[1] = in->v();
                    HashTable h2;
                    Buf sor2, gid2, rep2;
                    hash_build(s, k, n, /*skip_null_keys=*/true, h2, sor2);
                    const int64_t np = hash_group_ids(s, h2, sor2, n, gid2, rep2);
                    Buf pg = dev_alloc(sizeof(int64_t) * (np > 0 ? np : 1), s);
                    gather_col(P<int64_t>(gid), nullptr, P<int64_t>(rep2), np, P<int64_t>(pg), nullptr, st);
                    agg_count(P<int64_t>(pg), nullptr, np, P<int64_t>(c.data), st);
                }
                break;
            }
            case CAPSMI_AGG_SUM: {
                REQUIRE(in->type == CAPSMI_I64 || in->type == CAPSMI_F64, CAPSMI_ERR_ILLEGAL_ARGUMENT, "sum of non-number");
                c.type = in->type;
                c.valid = dev_alloc(ng, s);
                HIP_CHECK(hipMemsetAsync(P<void>(c.data), 0, sizeof(int64_t) * ng, st));
                HIP_CHECK(hipMemsetAsync(P<void>(c.valid), 0, ng, st));
                if (in->type == CAPSMI_I64) agg_sum_i64(P<int64_t>(gid), in->d(), in->v(), n, P<int64_t>(c.data), P<uint8_t>(c.valid), st);
                else agg_sum_f64(P<int64_t>(gid), in->d(), in->v(), n, P<double>(c.data), P<uint8_t>(c.valid), st);
                break;
            }
            case CAPSMI_AGG_MIN:
            case CAPSMI_AGG_MAX: {
                const bool mx = ag.kind == CAPSMI_AGG_MAX;
                c.type = in->type;
                c.valid = dev_alloc(ng, s);
                fill_i64(P<int64_t>(c.data), mx ? INT64_MIN : INT64_MAX, ng, st);
                HIP_CHECK(hipMemsetAsync(P<void>(c.valid), 0, ng, st));
                agg_minmax(P<int64_t>(gid), in->d(), in->v(), n, in->type, mx, P<int64_t>(c.data), P<uint8_t>(c.valid), st);
                minmax_finish(P<int64_t>(c.data), in->type, mx, ng, st);
                break;
            }
            case CAPSMI_AGG_AVG: {
                REQUIRE(in->type == CAPSMI_I64 || in->type == CAPSMI_F64, CAPSMI_ERR_ILLEGAL_ARGUMENT, "avg of non-number");
                c.type = in->type;  // avg(..).cast(cypherType): integer averages come back as Long
                c.valid = dev_alloc(ng, s);
                Buf sum = dev_alloc(sizeof(double) * ng, s), cnt = dev_alloc(sizeof(int64_t) * ng, s), seen = dev_alloc(ng, s);
                HIP_CHECK(hipMemsetAsync(P<void>(sum), 0, sizeof(double) * ng, st));
                HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(int64_t) * ng, st));
                if (in->type == CAPSMI_I64) {
                    // Spark casts Long input to Double before summing
                    Buf dv = dev_alloc(sizeof(double) * (n > 0 ? n : 1), s);
                    i64_to_f64(in->d(), P<int64_t>(dv), n, st);
                    agg_sum_f64(P<int64_t>(gid), P<int64_t>(dv), in->v(), n, P<double>(sum), P<uint8_t>(seen), st);
                } else {
                    agg_sum_f64(P<int64_t>(gid), in->d(), in->v(), n, P<double>(sum), P<uint8_t>(seen), st);
                }
                agg_count(P<int64_t>(gid), in->v(), n, P<int64_t>(cnt), st);
                avg_finish(P<double>(sum), P<int64_t>(cnt), ng, in->type == CAPSMI_I64, P<int64_t>(c.data),
                           P<uint8_t>(c.valid), st);
                break;
            }
            case CAPSMI_AGG_COLLECT: {
                // sort_array(collect_list / collect_set): row g of the result is list g of the store
                c.type = CAPSMI_LIST + in->type;
                c.list = collect_lists(s, P<int64_t>(gid), ng, in->d(), in->v(), in->type, n, ag.distinct != 0);
                iota_i64(P<int64_t>(c.data), 0, ng, st);
                break;
            }
            default:
                throw Error(CAPSMI_ERR_NOT_IMPLEMENTED, "Aggregation function " + std::to_string(ag.kind));
        }
        o->cols.push_back(std::move(c));
    }
    *out = guard.release();
    API_END
}

}  // namespace capsmi

extern "C" {

// ---- graph fast path ------------------------------------------------------------------------------
capsmi_status capsmi_bitmap_create(capsmi_session* s, int64_t id_lo, int64_t id_hi, capsmi_bitmap** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(id_hi >= id_lo, CAPSMI_ERR_ILLEGAL_ARGUMENT, "bitmap range");
    REQUIRE(id_hi - id_lo <= (int64_t(1) << 40), CAPSMI_ERR_UNSUPPORTED, "bitmap range above 2^40 ids");
    use_device(s);
    auto* b = new capsmi_bitmap();
    b->sess = s;
    b->lo = id_lo;
    b->hi = id_hi;
    b->nwords = (id_hi - id_lo + 31) / 32;
    b->words = dev_alloc(sizeof(uint32_t) * (b->nwords > 0 ? b->nwords : 1), s);
    HIP_CHECK(hipMemsetAsync(P<void>(b->words), 0, sizeof(uint32_t) * (b->nwords > 0 ? b->nwords : 1), s->stream));
    b->set_bits = 0;
    b->full = id_hi == id_lo;
    *out = b;
    API_END
}

capsmi_status capsmi_bitmap_add_scan(capsmi_bitmap* b, capsmi_table* nodes, const char* id_col, int32_t nnodes,
                                     const capsmi_expr* pred) {
    API_BEGIN
    need(b, "bitmap");
    need(nodes, "nodes");
    M(nodes);
    capsmi_session* s = b->sess;
    use_device(s);
    const int idx = col_index(nodes, id_col);
    const Column& idc = nodes->cols[idx];
    REQUIRE(idc.type == CAPSMI_I64, CAPSMI_ERR_ILLEGAL_ARGUMENT, "node id column must be Long");
    const EntityInfo* e = nodes->entity.get();
    if (nnodes == 0 && e && e->kind == 1 && e->ids_exact && e->id == idx && b->set_bits == 0 && b->rows_added == 0 &&
        e->lo >= b->lo && e->hi <= b->hi) {
        // a registered node table whose ids are exactly [lo, hi), each once (register_entity): the scan
        // sets that range, with no pass over the rows and no host round trip
        bitmap_set_range(b, e->lo - b->lo, e->hi - b->lo);
        b->rows_added = nodes->nrows;
        b->set_bits = nodes->nrows;
        b->full = b->set_bits == b->hi - b->lo;
        return CAPSMI_OK;
    }
    Buf flags;
    RangePred rp;
    std::vector<capsmi_expr> bound;
    if (nnodes > 0 && has_params(nnodes, pred)) {
        bound = bind_params(s, nnodes, pred);
        pred = bound.data();
        nnodes = (int32_t)bound.size();
    }
    if (nnodes > 0) {
        validate_program(nodes, nnodes, pred);
        if (!compile_range_pred(nodes, nnodes, pred, rp)) {  // general predicates: a flag column first
            flags = dev_alloc(nodes->nrows > 0 ? nodes->nrows : 1, s);
            eval_predicate(s, nodes, nnodes, pred, P<uint8_t>(flags));
        }
    }
    Buf cnt = dev_alloc(3 * sizeof(int64_t), s);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, 3 * sizeof(int64_t), s->stream));
    bitmap_add_rows(b, idc.d(), idc.v(), P<uint8_t>(flags), nodes->nrows, P<int64_t>(cnt), &rp);
    if (e && e->kind == 1 && e->ids_unique && e->id == idx && !idc.v() && b->set_bits == 0 && b->rows_added == 0 &&
        e->lo >= b->lo && e->hi <= b->hi) {
        // A registered node table without repeated or null ids, inside the window, into an empty bitmap:
        // no row can be out of range or a duplicate, so nothing needs reading back -- the scan costs no
        // host round trip.  With a predicate the set-bit count is left unknown (computed when asked).
        b->rows_added = nodes->nrows;
        b->set_bits = nnodes == 0 ? nodes->nrows : -1;
        b->full = b->set_bits == b->hi - b->lo;
        return CAPSMI_OK;
    }
    int64_t h[3];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(cnt), sizeof(h), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    REQUIRE(h[2] == 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::to_string(h[2]) + " node ids are null or outside the bitmap range [" + std::to_string(b->lo) + ", " +
                std::to_string(b->hi) + ")");
    b->rows_added += h[0];
    b->any_dup = b->any_dup || h[1] > 0;
    // every added row either set a fresh bit or was counted as a duplicate (exact, see k_bitmap_add)
    if (b->set_bits < 0) b->set_bits = words_popcount(s, P<uint32_t>(b->words), 0, b->nwords);
    b->set_bits += h[0] - h[1];
    b->full = b->set_bits == b->hi - b->lo;
    API_END
}

capsmi_status capsmi_bitmap_stats(capsmi_bitmap* b, int64_t* set_bits, int32_t* unique_rows) {
    API_BEGIN
    need(b, "bitmap");
    if (b->set_bits < 0) {  // left unknown by a scan with a predicate
        b->set_bits = words_popcount(b->sess, P<uint32_t>(b->words), 0, b->nwords);
        b->full = b->set_bits == b->hi - b->lo;
    }
    if (set_bits) *set_bits = b->set_bits;
    if (unique_rows) *unique_rows = b->any_dup ? 0 : 1;
    API_END
}

capsmi_status capsmi_bitmap_words(capsmi_bitmap* b, uint32_t** words, int64_t* nwords) {
    API_BEGIN
    need(b, "bitmap");
    if (words) *words = P<uint32_t>(b->words);
    if (nwords) *nwords = b->nwords;
    b->set_bits = -1;  // the caller may rewrite the words
    API_END
}

capsmi_status capsmi_bitmap_refresh(capsmi_bitmap* b, int32_t unique_rows) {
    API_BEGIN
    need(b, "bitmap");
    use_device(b->sess);
    b->set_bits = words_popcount(b->sess, P<uint32_t>(b->words), 0, b->nwords);
    b->full = b->set_bits == b->hi - b->lo;
    b->any_dup = unique_rows == 0;
    API_END
}

capsmi_status capsmi_bitmap_assume(capsmi_bitmap* b, int64_t set_bits, int32_t unique_rows) {
    API_BEGIN
    need(b, "bitmap");
    REQUIRE(set_bits >= 0 && set_bits <= b->hi - b->lo, CAPSMI_ERR_ILLEGAL_ARGUMENT, "set-bit count outside the domain");
    b->set_bits = set_bits;
    b->full = b->set_bits == b->hi - b->lo;
    b->any_dup = unique_rows == 0;
    API_END
}

capsmi_status capsmi_bitmap_copy_words(capsmi_bitmap* b, int64_t w_begin, int64_t w_end, uint32_t* ext,
                                       int32_t to_bitmap) {
    API_BEGIN
    need(b, "bitmap");
    need(ext, "ext");
    REQUIRE(w_begin >= 0 && w_begin <= w_end && w_end <= b->nwords, CAPSMI_ERR_ILLEGAL_ARGUMENT, "word range");
    use_device(b->sess);
    uint32_t* w = P<uint32_t>(b->words) + w_begin;
    const size_t bytes = sizeof(uint32_t) * (size_t)(w_end - w_begin);
    if (bytes)
        HIP_CHECK(hipMemcpyAsync(to_bitmap ? (void*)w : (void*)ext, to_bitmap ? (const void*)ext : (const void*)w, bytes,
                                 hipMemcpyDeviceToDevice, b->sess->stream));
    if (to_bitmap) b->set_bits = -1;
    API_END
}

capsmi_status capsmi_bitmap_release(capsmi_bitmap* b) {
    API_BEGIN
    if (b) {
        use_device(b->sess);
        delete b;
    }
    API_END
}

capsmi_status capsmi_expand_filter(capsmi_session* s, capsmi_table* rels, const char* src_col, const char* dst_col,
                                   const capsmi_bitmap* src_ok, const capsmi_bitmap* dst_ok, int32_t nout,
                                   const char* const* out_cols, const char* const* out_names, capsmi_table** out) {
    API_BEGIN
    need(s, "session");
    need(rels, "rels");
    M(rels);
    need(out, "out");
    check_bitmap(src_ok, "src_ok");
    check_bitmap(dst_ok, "dst_ok");
    REQUIRE(nout >= 1 && nout <= 4, CAPSMI_ERR_ILLEGAL_ARGUMENT, "expand_filter projects 1..4 columns");
    REQUIRE(!src_ok->any_dup && !dst_ok->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "fused expand needs each node id in one scanned row (ScanGraph.scala:72-76); use join");
    use_device(s);
    const Column& sc = rel_col(rels, src_col);
    const Column& dc = rel_col(rels, dst_col);
    const int64_t m = rels->nrows;
    auto* o = new_table(s, 0);
    std::unique_ptr<capsmi_table> guard(o);
    const int64_t* in_d[4];
    const uint8_t* in_v[4];
    int64_t* out_d[4];
    uint8_t* out_v[4];
    std::unordered_set<std::string> names;
    for (int i = 0; i < nout; ++i) {
        const Column& c = rels->cols[col_index(rels, out_cols[i])];
        Column oc;
        oc.name = out_names && out_names[i] ? out_names[i] : c.name;
        REQUIRE(names.insert(oc.name).second, CAPSMI_ERR_ILLEGAL_ARGUMENT, "duplicate output column " + oc.name);
        oc.type = c.type;
        oc.data = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s);
        if (c.valid) oc.valid = dev_alloc(m > 0 ? m : 1, s);
        in_d[i] = c.d();
        in_v[i] = c.v();
        out_d[i] = P<int64_t>(oc.data);
        out_v[i] = P<uint8_t>(oc.valid);
        o->cols.push_back(std::move(oc));
    }
    Buf cnt = dev_alloc(8, s);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, 8, s->stream));
    graph::expand_filter(s, sc.d(), dc.d(), m, src_ok, dst_ok, nout, in_d, in_v, out_d, out_v, P<int64_t>(cnt));
    o->nrows = read_scalar(s, P<int64_t>(cnt));
    *out = guard.release();
    API_END
}

static bool same_domain(const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c) {
    return a->lo == b->lo && a->hi == b->hi && b->lo == c->lo && b->hi == c->hi && b->hi > b->lo &&
           (uint64_t)(b->hi - b->lo) <= (uint64_t(1) << 32);
}

static void build_part(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                       const char* dst_col, int64_t lo, int64_t hi, RelPart& rp, const RelPartHop1* h1 = nullptr) {
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        srcs.push_back(rel_col(rels[i], src_col).d());
        dsts.push_back(rel_col(rels[i], dst_col).d());
        ms.push_back(rels[i]->nrows);
    }
    relpart_build(s, srcs.data(), dsts.data(), ms.data(), nrels, lo, hi, rp, h1);
}

// hop 1 on a partitioned layout into X1 (= M | S1) and X2 (= M | S2); S1 scratch
static void part_mid(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* X1,
                     uint32_t* X2, uint32_t* S1) {
    const int64_t nw = b->nwords;
    HIP_CHECK(hipMemsetAsync(X1, 0, sizeof(uint32_t) * nw, s->stream));
    HIP_CHECK(hipMemsetAsync(X2, 0, sizeof(uint32_t) * nw, s->stream));
    HIP_CHECK(hipMemsetAsync(S1, 0, sizeof(uint32_t) * nw, s->stream));
    relpart_hop1(s, rp, a, b, X1, S1, X2);
    graph::mid_combine(s, X1, X2, S1, nw);
}

// build + hop 1 in one go (hop 1 rides on the build's second pass when a is full)
static void build_part_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                           const char* dst_col, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* X1,
                           uint32_t* X2, uint32_t* S1, RelPart& rp, bool zeroed = false) {
    const int64_t nw = b->nwords;
    if (!zeroed) {  // zeroed: the caller cleared X1, X2, S1 with its own buffers in one fill
        HIP_CHECK(hipMemsetAsync(X1, 0, sizeof(uint32_t) * nw, s->stream));
        HIP_CHECK(hipMemsetAsync(X2, 0, sizeof(uint32_t) * nw, s->stream));
        HIP_CHECK(hipMemsetAsync(S1, 0, sizeof(uint32_t) * nw, s->stream));
    }
    const RelPartHop1 h1{a, b, X1, S1, X2};
    build_part(s, nrels, rels, src_col, dst_col, b->lo, b->hi, rp, &h1);
    graph::mid_combine(s, X1, X2, S1, nw);
}

static void two_hop_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                        const char* dst_col, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* X1, uint32_t* X2,
                        uint32_t* S1) {
    const int64_t nw = b->nwords;
    HIP_CHECK(hipMemsetAsync(X1, 0, sizeof(uint32_t) * nw, s->stream));
    HIP_CHECK(hipMemsetAsync(X2, 0, sizeof(uint32_t) * nw, s->stream));
    HIP_CHECK(hipMemsetAsync(S1, 0, sizeof(uint32_t) * nw, s->stream));
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        const Column& sc = rel_col(rels[i], src_col);
        const Column& dc = rel_col(rels[i], dst_col);
        graph::hop1(s, sc.d(), dc.d(), rels[i]->nrows, a, b, X1, S1, X2);
    }
    graph::mid_combine(s, X1, X2, S1, nw);
}

static void two_hop_dst(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                        const char* dst_col, const capsmi_bitmap* b, const capsmi_bitmap* c, const uint32_t* X1,
                        const uint32_t* X2, uint32_t* C) {
    HIP_CHECK(hipMemsetAsync(C, 0, sizeof(uint32_t) * c->nwords, s->stream));
    for (int i = 0; i < nrels; ++i) {
        M(rels[i]);
        const Column& sc = rel_col(rels[i], src_col);
        const Column& dc = rel_col(rels[i], dst_col);
        graph::hop2(s, sc.d(), dc.d(), rels[i]->nrows, c, X1, X2, b->lo, b->hi, C);
    }
}

capsmi_status capsmi_two_hop_count_distinct(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                            const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                            const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, int64_t* out_distinct) {
    API_BEGIN
    need(s, "session");
    need(out_distinct, "out");
    REQUIRE(nrels >= 0 && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT, "rels");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    use_device(s);
    const int64_t nw = b_ok->nwords > 0 ? b_ok->nwords : 1;
    if (same_domain(a_ok, b_ok, c_ok)) {
        // cold radix-partitioned path: partition + two LDS-resident hops; X1, X2, S1 and the
        // distinct targets' bitmap in one buffer, cleared by one fill
        Buf x = dev_alloc(sizeof(uint32_t) * nw * 4, s);
        uint32_t* X1 = P<uint32_t>(x);
        HIP_CHECK(hipMemsetAsync(X1, 0, sizeof(uint32_t) * nw * 4, s->stream));
        RelPart rp;
        build_part_mid(s, nrels, rels, src_col, dst_col, a_ok, b_ok, X1, X1 + nw, X1 + 2 * nw, rp, true);
        relpart_hop2(s, rp, c_ok, X1, X1 + nw, X1 + 3 * nw);
        *out_distinct = words_popcount(s, X1 + 3 * nw, 0, c_ok->nwords);
        return CAPSMI_OK;
    }
    Buf x = dev_alloc(sizeof(uint32_t) * nw * 3, s);
    Buf cw = dev_alloc(sizeof(uint32_t) * (c_ok->nwords > 0 ? c_ok->nwords : 1), s);
    uint32_t* X1 = P<uint32_t>(x);
    {
        two_hop_mid(s, nrels, rels, src_col, dst_col, a_ok, b_ok, X1, X1 + nw, X1 + 2 * nw);
        two_hop_dst(s, nrels, rels, src_col, dst_col, b_ok, c_ok, X1, X1 + nw, P<uint32_t>(cw));
    }
    *out_distinct = words_popcount(s, P<uint32_t>(cw), 0, c_ok->nwords);
    API_END
}

}  // extern "C"

struct capsmi_relpart {
    capsmi_session* sess = nullptr;
    capsmi::RelPart rp;
};

extern "C" {

capsmi_status capsmi_relpart_build(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                   const char* dst_col, int64_t id_lo, int64_t id_hi, capsmi_relpart** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(nrels >= 0 && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT, "rels");
    use_device(s);
    auto* p = new capsmi_relpart();
    std::unique_ptr<capsmi_relpart> guard(p);
    p->sess = s;
    build_part(s, nrels, rels, src_col, dst_col, id_lo, id_hi, p->rp);
    *out = guard.release();
    API_END
}

capsmi_status capsmi_relpart_build_mark_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                            const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                            const capsmi_bitmap* b_ok, uint32_t* mid_words, uint32_t* scratch_words,
                                            capsmi_relpart** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    need(mid_words, "mid_words");
    need(scratch_words, "scratch_words");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    REQUIRE(nrels >= 0 && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT, "rels");
    REQUIRE(a_ok->lo == b_ok->lo && a_ok->hi == b_ok->hi, CAPSMI_ERR_UNSUPPORTED, "a and b scans need one id domain");
    use_device(s);
    auto* p = new capsmi_relpart();
    std::unique_ptr<capsmi_relpart> guard(p);
    p->sess = s;
    build_part_mid(s, nrels, rels, src_col, dst_col, a_ok, b_ok, mid_words, mid_words + b_ok->nwords, scratch_words,
                   p->rp);
    *out = guard.release();
    API_END
}

capsmi_status capsmi_undirected_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                      const char* dst_col, int32_t hops, const capsmi_bitmap* a_ok,
                                      const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, int32_t kind, int64_t* out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    REQUIRE(hops == 1 || hops == 2, CAPSMI_ERR_ILLEGAL_ARGUMENT, "undirected patterns: 1 or 2 hops");
    REQUIRE(kind >= 0 && kind <= 2, CAPSMI_ERR_ILLEGAL_ARGUMENT, "undirected patterns: kind");
    if (hops == 2) check_bitmap(c_ok, "c_ok");
    use_device(s);
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        srcs.push_back(rel_col(rels[i], src_col).d());
        dsts.push_back(rel_col(rels[i], dst_col).d());
        ms.push_back(rels[i]->nrows);
    }
    *out = undirected_count(s, srcs.data(), dsts.data(), ms.data(), nrels, hops, a_ok, b_ok, hops == 2 ? c_ok : b_ok, kind);
    API_END
}

capsmi_status capsmi_var_length_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                      const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                      const capsmi_bitmap* b_ok, int32_t lower, int32_t upper, const char* id_name,
                                      const char* count_name, capsmi_table** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    need(id_name, "id_name");
    need(count_name, "count_name");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    REQUIRE(nrels >= 0 && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT, "rels");
    REQUIRE(lower >= 0 && lower <= upper && upper >= 1 && upper <= 4, CAPSMI_ERR_NOT_IMPLEMENTED,
            "fused var-length count supports 0 <= lower <= upper <= 4, upper >= 1 (use the join plan otherwise)");
    REQUIRE(a_ok->lo == b_ok->lo && a_ok->hi == b_ok->hi, CAPSMI_ERR_UNSUPPORTED, "a and b scans need one id domain");
    REQUIRE(!a_ok->any_dup && !b_ok->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "fused count(*) needs each node id in one scanned row");
    REQUIRE(upper <= 3 || a_ok->hi - a_ok->lo < (int64_t(1) << 24) - 1, CAPSMI_ERR_UNSUPPORTED,
            "fused var-length upper 4: at most 2^24 - 2 ids");
    REQUIRE(std::string(id_name) != count_name, CAPSMI_ERR_ILLEGAL_ARGUMENT, "output names must differ");
    use_device(s);
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        srcs.push_back(rel_col(rels[i], src_col).d());
        dsts.push_back(rel_col(rels[i], dst_col).d());
        ms.push_back(rels[i]->nrows);
    }
    Buf ids, cnt;
    const int64_t rows =
        var_length_count(s, srcs.data(), dsts.data(), ms.data(), nrels, a_ok, b_ok, lower, upper, ids, cnt);
    auto* o = new_table(s, rows);
    Column a, c;
    a.name = id_name;
    a.type = CAPSMI_I64;
    a.data = ids;
    c.name = count_name;
    c.type = CAPSMI_I64;
    c.data = cnt;
    o->cols.push_back(std::move(a));
    o->cols.push_back(std::move(c));
    *out = o;
    API_END
}

struct capsmi_varlen_shard {
    capsmi_session* sess = nullptr;
    capsmi::VarlenShard* v = nullptr;
    ~capsmi_varlen_shard() { capsmi::varlen_shard_free(v); }
};

capsmi_status capsmi_varlen_shard_begin(capsmi_session* s, int32_t nout, capsmi_table* const* out_rels, int32_t nin,
                                        capsmi_table* const* in_rels, const char* src_col, const char* dst_col,
                                        const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, int32_t lower,
                                        int32_t upper, int64_t own_lo, int64_t own_hi, int64_t* od,
                                        capsmi_varlen_shard** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    need(od, "od");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    REQUIRE(nout >= 0 && (nout == 0 || out_rels) && nin >= 0 && (nin == 0 || in_rels), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "rels");
    REQUIRE(lower >= 0 && lower <= upper && upper >= 1 && upper <= 3, CAPSMI_ERR_NOT_IMPLEMENTED,
            "fused var-length count supports 0 <= lower <= upper <= 3, upper >= 1 (use the join plan otherwise)");
    REQUIRE(a_ok->lo == b_ok->lo && a_ok->hi == b_ok->hi, CAPSMI_ERR_UNSUPPORTED, "a and b scans need one id domain");
    REQUIRE(!a_ok->any_dup && !b_ok->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "fused count(*) needs each node id in one scanned row");
    use_device(s);
    std::vector<const int64_t*> srcs, dsts, isrcs, idsts;
    std::vector<int64_t> ms, ims;
    for (int i = 0; i < nout; ++i) {
        need(out_rels[i], "out_rels[i]");
        M(out_rels[i]);
        srcs.push_back(rel_col(out_rels[i], src_col).d());
        dsts.push_back(rel_col(out_rels[i], dst_col).d());
        ms.push_back(out_rels[i]->nrows);
    }
    for (int i = 0; i < nin; ++i) {
        need(in_rels[i], "in_rels[i]");
        M(in_rels[i]);
        isrcs.push_back(rel_col(in_rels[i], src_col).d());
        idsts.push_back(rel_col(in_rels[i], dst_col).d());
        ims.push_back(in_rels[i]->nrows);
    }
    auto h = std::make_unique<capsmi_varlen_shard>();
    h->sess = s;
    h->v = varlen_shard_begin(s, srcs.data(), dsts.data(), ms.data(), nout, isrcs.data(), idsts.data(), ims.data(),
                              nin, a_ok, b_ok, lower, upper, own_lo, own_hi, od);
    *out = h.release();
    API_END
}

capsmi_status capsmi_varlen_shard_mid(capsmi_varlen_shard* v, int64_t* y) {
    API_BEGIN
    need(v, "shard");
    need(y, "y");
    use_device(v->sess);
    varlen_shard_mid(v->v, y);
    API_END
}

capsmi_status capsmi_varlen_shard_finish(capsmi_varlen_shard* v, const char* id_name, const char* count_name,
                                         capsmi_table** out) {
    API_BEGIN
    need(v, "shard");
    need(out, "out");
    need(id_name, "id_name");
    need(count_name, "count_name");
    REQUIRE(std::string(id_name) != count_name, CAPSMI_ERR_ILLEGAL_ARGUMENT, "output names must differ");
    use_device(v->sess);
    Buf ids, cnt;
    const int64_t rows = varlen_shard_finish(v->v, ids, cnt);
    auto* o = new_table(v->sess, rows);
    Column a, c;
    a.name = id_name;
    a.type = CAPSMI_I64;
    a.data = ids;
    c.name = count_name;
    c.type = CAPSMI_I64;
    c.data = cnt;
    o->cols.push_back(std::move(a));
    o->cols.push_back(std::move(c));
    *out = o;
    API_END
}

capsmi_status capsmi_varlen_shard_release(capsmi_varlen_shard* v) {
    API_BEGIN
    if (v) {
        use_device(v->sess);
        delete v;
    }
    API_END
}

}  // extern "C"

struct capsmi_trigraph {
    capsmi_session* sess = nullptr;
    capsmi::TriGraph g;
};

static void rel_cols(int32_t nrels, capsmi_table* const* rels, const char* src_col, const char* dst_col,
                     std::vector<const int64_t*>& srcs, std::vector<const int64_t*>& dsts, std::vector<int64_t>& ms) {
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        srcs.push_back(rel_col(rels[i], src_col).d());
        dsts.push_back(rel_col(rels[i], dst_col).d());
        ms.push_back(rels[i]->nrows);
    }
}

extern "C" {

capsmi_status capsmi_trigraph_build(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                    const char* dst_col, const capsmi_bitmap* n_ok, capsmi_trigraph** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    check_bitmap(n_ok, "n_ok");
    REQUIRE(!n_ok->any_dup, CAPSMI_ERR_UNSUPPORTED, "fused count(*) needs each node id in one scanned row");
    REQUIRE(nrels >= 0 && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT, "rels");
    use_device(s);
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    rel_cols(nrels, rels, src_col, dst_col, srcs, dsts, ms);
    auto* g = new capsmi_trigraph();
    std::unique_ptr<capsmi_trigraph> guard(g);
    g->sess = s;
    tri_build(s, srcs.data(), dsts.data(), ms.data(), nrels, n_ok, g->g);
    *out = guard.release();
    API_END
}

capsmi_status capsmi_trigraph_count(capsmi_session* s, const capsmi_trigraph* g, int32_t part, int32_t nparts,
                                    int64_t* out_rows) {
    API_BEGIN
    need(s, "session");
    need(g, "trigraph");
    need(out_rows, "out");
    REQUIRE(nparts >= 1 && part >= 0 && part < nparts, CAPSMI_ERR_ILLEGAL_ARGUMENT, "part");
    use_device(s);
    *out_rows = (int64_t)tri_count(s, g->g, part, nparts);
    API_END
}

capsmi_status capsmi_trigraph_stats(const capsmi_trigraph* g, int64_t* nodes, int64_t* oriented_edges) {
    API_BEGIN
    need(g, "trigraph");
    if (nodes) *nodes = g->g.n;
    if (oriented_edges) *oriented_edges = g->g.ne;
    API_END
}

capsmi_status capsmi_trigraph_release(capsmi_trigraph* g) {
    API_BEGIN
    if (g) {
        use_device(g->sess);
        delete g;
    }
    API_END
}

capsmi_status capsmi_triangle_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                    const char* dst_col, const capsmi_bitmap* n_ok, int64_t* out_rows) {
    capsmi_trigraph* g = nullptr;
    capsmi_status st = capsmi_trigraph_build(s, nrels, rels, src_col, dst_col, n_ok, &g);
    if (st != CAPSMI_OK) return st;
    st = capsmi_trigraph_count(s, g, 0, 1, out_rows);
    capsmi_trigraph_release(g);
    return st;
}

capsmi_status capsmi_relpart_size(const capsmi_relpart* p, int64_t* kept_rows) {
    API_BEGIN
    need(p, "relpart");
    need(kept_rows, "out");
    use_device(p->sess);
    *kept_rows = relpart_kept(p->sess, const_cast<capsmi_relpart*>(p)->rp);
    API_END
}

capsmi_status capsmi_relpart_digest(const capsmi_relpart* p, int64_t* ncells, int64_t* ns, int32_t* sbits,
                                    int32_t* tbits, int64_t* counts, uint64_t* sums, int64_t* misplaced) {
    API_BEGIN
    need(p, "relpart");
    need(ncells, "ncells");
    need(ns, "ns");
    need(sbits, "sbits");
    need(tbits, "tbits");
    const PartLayout& L = p->rp.L;
    *ncells = L.ncells;
    *ns = L.ns;
    *sbits = L.sbits;
    *tbits = L.tbits;
    if (counts || sums) {
        need(counts, "counts");
        need(sums, "sums");
        need(misplaced, "misplaced");
        use_device(p->sess);
        relpart_digest(p->sess, p->rp, counts, sums, misplaced);
    }
    API_END
}

capsmi_status capsmi_relpart_release(capsmi_relpart* p) {
    API_BEGIN
    if (p) {
        use_device(p->sess);
        delete p;
    }
    API_END
}

capsmi_status capsmi_two_hop_mark_mid_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* a_ok,
                                           const capsmi_bitmap* b_ok, uint32_t* mid_words, uint32_t* scratch_words) {
    API_BEGIN
    need(s, "session");
    need(p, "relpart");
    need(mid_words, "mid_words");
    need(scratch_words, "scratch_words");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    use_device(s);
    part_mid(s, p->rp, a_ok, b_ok, mid_words, mid_words + b_ok->nwords, scratch_words);
    API_END
}

capsmi_status capsmi_two_hop_mark_dst_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* b_ok,
                                           const capsmi_bitmap* c_ok, const uint32_t* mid_words, uint32_t* dst_words) {
    API_BEGIN
    need(s, "session");
    need(p, "relpart");
    need(mid_words, "mid_words");
    need(dst_words, "dst_words");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    REQUIRE(b_ok->lo == c_ok->lo && b_ok->hi == c_ok->hi, CAPSMI_ERR_UNSUPPORTED, "b and c scans need one id domain");
    use_device(s);
    HIP_CHECK(hipMemsetAsync(dst_words, 0, sizeof(uint32_t) * c_ok->nwords, s->stream));
    relpart_hop2(s, p->rp, c_ok, mid_words, mid_words + b_ok->nwords, dst_words);
    API_END
}

capsmi_status capsmi_two_hop_count_distinct_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* a_ok,
                                                 const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok,
                                                 int64_t* out_distinct) {
    API_BEGIN
    need(s, "session");
    need(p, "relpart");
    need(out_distinct, "out");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    REQUIRE(same_domain(a_ok, b_ok, c_ok), CAPSMI_ERR_UNSUPPORTED, "a, b, c scans need one id domain");
    use_device(s);
    const int64_t nw = b_ok->nwords > 0 ? b_ok->nwords : 1;
    Buf x = dev_alloc(sizeof(uint32_t) * nw * 4, s);
    uint32_t* X1 = P<uint32_t>(x);
    part_mid(s, p->rp, a_ok, b_ok, X1, X1 + nw, X1 + 2 * nw);
    HIP_CHECK(hipMemsetAsync(X1 + 3 * nw, 0, sizeof(uint32_t) * nw, s->stream));
    relpart_hop2(s, p->rp, c_ok, X1, X1 + nw, X1 + 3 * nw);
    *out_distinct = words_popcount(s, X1 + 3 * nw, 0, c_ok->nwords);
    API_END
}

capsmi_status capsmi_two_hop_mark_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                      const char* dst_col, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                      uint32_t* mid_words, uint32_t* scratch_words) {
    API_BEGIN
    need(s, "session");
    need(mid_words, "mid_words");
    need(scratch_words, "scratch_words");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    use_device(s);
    two_hop_mid(s, nrels, rels, src_col, dst_col, a_ok, b_ok, mid_words, mid_words + b_ok->nwords, scratch_words);
    API_END
}

capsmi_status capsmi_two_hop_mark_dst(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                      const char* dst_col, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok,
                                      const uint32_t* mid_words, uint32_t* dst_words) {
    API_BEGIN
    need(s, "session");
    need(mid_words, "mid_words");
    need(dst_words, "dst_words");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    use_device(s);
    two_hop_dst(s, nrels, rels, src_col, dst_col, b_ok, c_ok, mid_words, mid_words + b_ok->nwords, dst_words);
    API_END
}

capsmi_status capsmi_words_popcount(capsmi_session* s, const uint32_t* words, int64_t w_begin, int64_t w_end,
                                    int64_t* out) {
    API_BEGIN
    need(s, "session");
    need(words, "words");
    need(out, "out");
    use_device(s);
    *out = words_popcount(s, words, w_begin, w_end);
    API_END
}

capsmi_status capsmi_words_popcount_device(capsmi_session* s, const uint32_t* words, int64_t w_begin, int64_t w_end,
                                           int64_t* dev_out) {
    API_BEGIN
    need(s, "session");
    need(words, "words");
    need(dev_out, "dev_out");
    use_device(s);
    words_popcount_async(s, words, w_begin, w_end, dev_out);
    API_END
}

struct capsmi_count_shard {
    capsmi::CountRec cr;
    capsmi::Buf b_words;    // b_ok's words, read by finish: kept alive with the handle
    bool finished = false;  // finish adds into the handle's accumulator once
};

capsmi_status capsmi_count_shard_begin(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                       const char* dst_col, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                       const capsmi_bitmap* c_ok, int64_t own_lo, int64_t own_hi, uint32_t* owned_in,
                                       capsmi_count_shard** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    REQUIRE(!a_ok->any_dup && !b_ok->any_dup && !c_ok->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "closed-form count(*) needs each node id in one scanned row");
    const int64_t n = b_ok->hi - b_ok->lo;
    REQUIRE(a_ok->lo == b_ok->lo && a_ok->hi == b_ok->hi && c_ok->lo == b_ok->lo && c_ok->hi == b_ok->hi,
            CAPSMI_ERR_ILLEGAL_ARGUMENT, "count shard: the three bitmaps must share one id domain");
    REQUIRE(n > 0 && n <= (int64_t(1) << 26), CAPSMI_ERR_UNSUPPORTED, "count shard: id domain of 1 .. 2^26 ids");
    REQUIRE(0 <= own_lo && own_lo <= own_hi && own_hi <= n, CAPSMI_ERR_ILLEGAL_ARGUMENT, "count shard: owned range");
    REQUIRE(own_hi == own_lo || owned_in, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null argument: owned_in");
    use_device(s);
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        srcs.push_back(rel_col(rels[i], src_col).d());
        dsts.push_back(rel_col(rels[i], dst_col).d());
        ms.push_back(rels[i]->nrows);
    }
    auto h = std::make_unique<capsmi_count_shard>();
    h->b_words = b_ok->words;
    count_rec_begin(s, srcs.data(), dsts.data(), ms.data(), nrels, a_ok, b_ok, c_ok, h->cr);
    count_rec_fold(h->cr, own_lo, own_hi, owned_in);
    *out = h.release();
    API_END
}

capsmi_status capsmi_count_shard_finish(capsmi_count_shard* h, const uint32_t* in_all, int64_t* dev_out) {
    API_BEGIN
    need(h, "count shard");
    need(in_all, "in_all");
    need(dev_out, "dev_out");
    REQUIRE(!h->finished, CAPSMI_ERR_ILLEGAL_ARGUMENT, "count shard: finish called twice on one handle");
    use_device(h->cr.s);
    count_rec_finish(h->cr, in_all, dev_out);
    h->finished = true;
    API_END
}

capsmi_status capsmi_count_shard_release(capsmi_count_shard* h) {
    API_BEGIN
    if (!h) return CAPSMI_OK;
    use_device(h->cr.s);
    delete h;
    API_END
}

capsmi_status capsmi_two_hop_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                   const char* dst_col, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                   const capsmi_bitmap* c_ok, int64_t* out_rows) {
    API_BEGIN
    need(s, "session");
    need(out_rows, "out");
    check_bitmap(a_ok, "a_ok");
    check_bitmap(b_ok, "b_ok");
    check_bitmap(c_ok, "c_ok");
    REQUIRE(!a_ok->any_dup && !b_ok->any_dup && !c_ok->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "closed-form count(*) needs each node id in one scanned row");
    use_device(s);
    const int64_t n = b_ok->hi - b_ok->lo;
    const bool same_domain = a_ok->lo == b_ok->lo && a_ok->hi == b_ok->hi && c_ok->lo == b_ok->lo && c_ok->hi == b_ok->hi;
    // (config CAPSMI_COUNT=atomic forces the per-relationship atomic form below, the one above 2^26 ids)
    if (same_domain && n > 0 && n <= (int64_t(1) << 26) && !s->cfg.count_atomic) {
        std::vector<const int64_t*> srcs, dsts;
        std::vector<int64_t> ms;
        for (int i = 0; i < nrels; ++i) {
            need(rels[i], "rels[i]");
            M(rels[i]);
            srcs.push_back(rel_col(rels[i], src_col).d());
            dsts.push_back(rel_col(rels[i], dst_col).d());
            ms.push_back(rels[i]->nrows);
        }
        *out_rows = two_hop_count_rec(s, srcs.data(), dsts.data(), ms.data(), nrels, a_ok, b_ok, c_ok);
        return CAPSMI_OK;
    }
    Buf inA = dev_alloc(sizeof(uint32_t) * (n > 0 ? n : 1), s);
    Buf outC = dev_alloc(sizeof(uint32_t) * (n > 0 ? n : 1), s);
    Buf acc = dev_alloc(16, s);  // [0] = loops, [1] = sum of products
    HIP_CHECK(hipMemsetAsync(P<void>(inA), 0, sizeof(uint32_t) * (n > 0 ? n : 1), s->stream));
    HIP_CHECK(hipMemsetAsync(P<void>(outC), 0, sizeof(uint32_t) * (n > 0 ? n : 1), s->stream));
    HIP_CHECK(hipMemsetAsync(P<void>(acc), 0, 16, s->stream));
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        M(rels[i]);
        const Column& sc = rel_col(rels[i], src_col);
        const Column& dc = rel_col(rels[i], dst_col);
        graph::degrees(s, sc.d(), dc.d(), rels[i]->nrows, a_ok, b_ok, c_ok, P<uint32_t>(inA), P<uint32_t>(outC),
                       P<int64_t>(acc));
    }
    graph::deg_product(s, P<uint32_t>(inA), P<uint32_t>(outC), n, b_ok, P<int64_t>(acc) + 1);
    int64_t h[2];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(acc), 16, hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    *out_rows = h[1] - h[0];
    API_END
}

capsmi_status capsmi_cluster_by(capsmi_table* rels, const char* key_col, int64_t id_lo, int64_t id_hi,
                                capsmi_table** out) {
    API_BEGIN
    need(rels, "rels");
    M(rels);
    need(out, "out");
    capsmi_session* s = rels->sess;
    use_device(s);
    const Column& kc = rel_col(rels, key_col);
    const int64_t n = rels->nrows;
    // keys relative to id_lo; range checked on the host copy of min/max is avoided: ids outside
    // [lo, hi) would break the bit budget, so the sort covers all 64 bits when the range is unknown
    int bits = 1;
    while (bits < 64 && (int64_t(1) << bits) < (id_hi - id_lo)) ++bits;
    Buf keys = dev_alloc(sizeof(uint64_t) * (n > 0 ? n : 1), s);
    Buf perm = dev_alloc(sizeof(int64_t) * (n > 0 ? n : 1), s);
    HIP_CHECK(hipMemcpyAsync(P<void>(keys), kc.d(), sizeof(int64_t) * n, hipMemcpyDeviceToDevice, s->stream));
    iota_i64(P<int64_t>(perm), 0, n, s->stream);
    // validate range on device via a bitmap scan of the key column
    {
        capsmi_bitmap tmp;
        tmp.sess = s;
        tmp.lo = id_lo;
        tmp.hi = id_hi;
        tmp.nwords = (id_hi - id_lo + 31) / 32;
        tmp.words = dev_alloc(sizeof(uint32_t) * (tmp.nwords > 0 ? tmp.nwords : 1), s);
        HIP_CHECK(hipMemsetAsync(P<void>(tmp.words), 0, sizeof(uint32_t) * (tmp.nwords > 0 ? tmp.nwords : 1), s->stream));
        Buf cnt = dev_alloc(24, s);
        HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, 24, s->stream));
        bitmap_add_rows(&tmp, kc.d(), nullptr, nullptr, n, P<int64_t>(cnt));
        int64_t h[3];
        HIP_CHECK(hipMemcpyAsync(h, P<void>(cnt), 24, hipMemcpyDeviceToHost, s->stream));
        HIP_CHECK(hipStreamSynchronize(s->stream));
        REQUIRE(h[2] == 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "cluster_by: key outside [id_lo, id_hi)");
    }
    if (id_lo != 0) {
        // shift keys: reuse the expression-free path through a host round trip is too slow; fold lo into the
        // sort by sorting raw keys (order is the same for keys in [lo, hi)) over enough bits
        bits = 64;
    }
    radix_sort_pairs(s, P<uint64_t>(keys), P<int64_t>(perm), n, 0, (bits + 7) / 8 * 8);
    auto* o = new_table(s, n);
    gather_into(o, rels, perm, n, false);
    *out = o;
    API_END
}

capsmi_status capsmi_owner_words(int64_t nbits, int32_t part, int32_t nparts, int64_t* w_begin, int64_t* w_end) {
    API_BEGIN
    REQUIRE(nparts >= 1 && part >= 0 && part < nparts && nbits >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "owner_words");
    need(w_begin, "w_begin");
    need(w_end, "w_end");
    const int64_t nw = (nbits + 31) / 32;
    *w_begin = (int64_t)part * nw / nparts;
    *w_end = (int64_t)(part + 1) * nw / nparts;
    API_END
}

capsmi_status capsmi_rmat_rels(capsmi_session* s, int32_t scale, int64_t e_begin, int64_t e_end, int32_t pa, int32_t pb,
                               int32_t pc, uint64_t seed, int32_t part_col, int32_t part, int32_t nparts,
                               capsmi_table** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(scale >= 1 && scale <= 40, CAPSMI_ERR_ILLEGAL_ARGUMENT, "R-MAT scale must be in 1..40");
    REQUIRE(e_begin >= 0 && e_end >= e_begin && e_end < (int64_t(1) << 35), CAPSMI_ERR_ILLEGAL_ARGUMENT, "edge range");
    REQUIRE(seed < (1ULL << 24), CAPSMI_ERR_ILLEGAL_ARGUMENT, "seed must be < 2^24");
    REQUIRE(pa >= 0 && pb >= 0 && pc >= 0 && pa + pb + pc <= 100, CAPSMI_ERR_ILLEGAL_ARGUMENT, "R-MAT probabilities");
    REQUIRE(nparts >= 1 && part >= 0 && part < nparts, CAPSMI_ERR_ILLEGAL_ARGUMENT, "partition");
    use_device(s);
    Buf id, so, d;
    const int64_t m = graph::rmat(s, scale, e_begin, e_end, pa, pb, pc, seed, part_col, part, nparts, id, so, d);
    auto* o = new_table(s, m);
    const char* names[3] = {"id", "source", "target"};
    Buf bufs[3] = {id, so, d};
    for (int i = 0; i < 3; ++i) {
        Column c;
        c.name = names[i];
        c.type = CAPSMI_I64;
        c.data = bufs[i];
        o->cols.push_back(std::move(c));
    }
    attach_entity(o, 2, 0, int64_t(1) << scale);  // [id, source, target]: a registered relationship table
    *out = o;
    API_END
}

capsmi_status capsmi_rmat_nodes(capsmi_session* s, int32_t scale, int32_t kind, uint64_t seed, capsmi_table** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(scale >= 1 && scale <= 40, CAPSMI_ERR_ILLEGAL_ARGUMENT, "scale");
    REQUIRE(kind >= 0 && kind <= 2, CAPSMI_ERR_ILLEGAL_ARGUMENT, "kind");
    use_device(s);
    const int64_t n = int64_t(1) << scale;
    Buf ids;
    int64_t rows = n;
    if (kind == 0) {
        ids = dev_alloc(sizeof(int64_t) * n, s);
        iota_i64(P<int64_t>(ids), 0, n, s->stream);
    } else {
        Buf f = dev_alloc(n, s);
        graph::person_flags(s, n, kind == 1, P<uint8_t>(f));
        rows = flags_to_indices(s, P<uint8_t>(f), n, ids);  // id == row index of the full range
    }
    auto* o = new_table(s, rows);
    Column c;
    c.name = "id";
    c.type = CAPSMI_I64;
    c.data = ids;
    o->cols.push_back(c);
    if (kind == 1) {
        Column a;
        a.name = "age";
        a.type = CAPSMI_I64;
        a.data = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), s);
        graph::ages(s, P<int64_t>(ids), rows, seed, P<int64_t>(a.data));
        o->cols.push_back(std::move(a));
    }
    // [id] / [id, age]: a registered node table (all ids: exactly [0, n); each id generated once either way)
    attach_entity(o, 1, 0, n, kind == 0, true);
    *out = o;
    API_END
}

capsmi_status capsmi_read_csv(capsmi_session* s, int32_t nfiles, const char* const* paths, char delimiter, char comment,
                              int32_t ncols, const char* const* names, const int32_t* types, capsmi_intern_fn intern,
                              void* intern_ctx, const char* row_id_col, capsmi_table** out) {
    API_BEGIN
    need(s, "session");
    need(out, "out");
    REQUIRE(nfiles >= 0 && (nfiles == 0 || paths) && ncols >= 1 && names && types, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "read_csv arguments");
    use_device(s);
    std::vector<std::string> ps, ns;
    std::vector<int32_t> ts;
    std::unordered_set<std::string> seen;
    if (row_id_col) seen.insert(row_id_col);
    for (int i = 0; i < nfiles; ++i) {
        need(paths[i], "path");
        ps.push_back(paths[i]);
    }
    for (int k = 0; k < ncols; ++k) {
        need(names[k], "column name");
        REQUIRE(seen.insert(names[k]).second, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("duplicate column '") + names[k] + "'");
        REQUIRE(types[k] >= CAPSMI_I64 && types[k] <= CAPSMI_STR, CAPSMI_ERR_ILLEGAL_ARGUMENT, "bad column type");
        ns.push_back(names[k]);
        ts.push_back(types[k]);
    }
    *out = read_csv(s, ps, delimiter, comment, ns, ts, intern, intern_ctx, row_id_col);
    API_END
}

capsmi_status capsmi_table_fingerprint(capsmi_table* t, int32_t ncols, const char* const* cols, int64_t* count,
                                       uint64_t* sum, uint64_t* xr) {
    API_BEGIN
    need(t, "table");
    M(t);
    use_device(t->sess);
    auto idx = names_to_idx(t, ncols, cols);
    std::vector<const int64_t*> d;
    std::vector<const uint8_t*> v;
    for (int i : idx) {
        no_list_key(t->cols[i].type, t->cols[i].name, "a fingerprint column");
        d.push_back(t->cols[i].d());
        v.push_back(t->cols[i].v());
    }
    uint64_t hs = 0, hx = 0;
    graph::fingerprint(t->sess, ncols, d.data(), v.data(), t->nrows, &hs, &hx);
    if (count) *count = t->nrows;
    if (sum) *sum = hs;
    if (xr) *xr = hx;
    API_END
}

}  // extern "C"
