// capsmi_impl.h -- internal runtime of libcapsmi (not part of the ABI).
//
// Device tables are column-major: one 8-byte word per row and column, plus an
// optional byte-per-row validity map.  Columns share ref-counted device buffers,
// so select/drop/rename/skip/limit are metadata-only (the Spark analogue is a
// Catalyst projection, SparkTable.scala:61-92).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <map>
#include <set>
#include <memory>
#include <stdexcept>
#include <string>
#include <functional>
#include <vector>

#include "../../include/capsmi.h"

namespace capsmi {

// ---- errors ---------------------------------------------------------------------
struct Error : std::runtime_error {
    capsmi_status code;
    Error(capsmi_status c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void throw_hip(hipError_t e, const char* what, const char* file, int line);
#define HIP_CHECK(x)                                                     \
    do {                                                                 \
        hipError_t e__ = (x);                                            \
        if (e__ != hipSuccess) ::capsmi::throw_hip(e__, #x, __FILE__, __LINE__); \
    } while (0)
#define REQUIRE(cond, code, msg)                      \
    do {                                              \
        if (!(cond)) throw ::capsmi::Error((code), (msg)); \
    } while (0)

// ---- device memory --------------------------------------------------------------
// Stream-ordered allocations from the device's default pool (release threshold
// raised at session create, so freed blocks are recycled instead of unmapped).
// Per-session allocation context: the device, the stream the session currently runs on, and the
// session's cache of freed device blocks (api.hip).  Blocks hold it, so a block that outlives its
// session is returned to the device instead of to a dead cache.
struct AllocCtx;
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    std::shared_ptr<AllocCtx> ctx;
    ~DevBuf();
};
using Buf = std::shared_ptr<DevBuf>;
Buf dev_alloc(size_t bytes, capsmi_session* s);

template <class T>
inline T* P(const Buf& b) { return b ? static_cast<T*>(b->ptr) : nullptr; }

// Values of a list column (CAPSMI_LIST_*): list k holds values[offsets[k] .. offsets[k+1]).  A list
// column's row word is the index k of its list, so gathers (filter, join, order, union) move list
// rows like any other column and the store rides along by reference.
struct ListStore {
    int32_t elem = CAPSMI_I64;  // element type
    int64_t nlists = 0, nvalues = 0;
    Buf offsets;                // int64, nlists + 1
    Buf values;                 // int64 words, nvalues
};
inline bool is_list_type(int32_t t) { return t >= CAPSMI_LIST_I64 && t <= CAPSMI_LIST_STR; }

struct Column {
    std::string name;
    int32_t type = CAPSMI_I64;
    Buf data;              // int64 words
    Buf valid;             // uint8 per row, may be null (no nulls)
    std::shared_ptr<const ListStore> list;  // list columns only
    int64_t offset = 0;    // row offset into data/valid (zero-copy skip)
    bool lazy_nullable = false;  // schema of a lazy table's column (no data yet): may hold nulls
    // host copy of the words of a column built from host values (the fused routes' count rows):
    // exports read it without a device round trip
    std::shared_ptr<const std::vector<int64_t>> host;
    const int64_t* d() const { return P<int64_t>(data) + offset; }
    const uint8_t* v() const { return valid ? P<uint8_t>(valid) + offset : nullptr; }
    bool nullable() const { return valid != nullptr || lazy_nullable; }
};

// Entity-table contract of a registered node / relationship table (capsmi_node_table /
// capsmi_rel_table; EntityTable.verify, okapi-relational/.../api/io/EntityTable.scala:59-65,155-164).
struct EntityInfo {
    int kind = 0;                 // 1 node, 2 relationship
    int id = -1, src = -1, dst = -1;  // column indices of the key columns
    int64_t lo = 0, hi = 0;       // [min, max + 1) of the ids (node) or of both endpoints (relationship)
    int64_t rows = 0;
    bool ids_exact = false;       // node: the ids are exactly [lo, hi), each once (checked at registration)
    bool ids_unique = false;      // node: no id occurs twice and none is null (checked at registration)
};
struct PlanNode;  // lazy Table[T] operator (plan.hip)

// Dense id space of one graph (capsmi_graph_compact): every node id and relationship endpoint of
// the graph's entity tables numbered 0..n-1; orig[d] is the Long id of dense id d.  The fused
// routes run on dense ids when the Long ids do not fit one window of 2^30 ids.
struct DenseIds {
    int64_t n = 0;
    Buf orig;
    // a distributed graph's domain (capsmi_graph_distribute): dense = h(x) = ((x - lo) * mul) mod 2^kbits,
    // x = (dense * mul_inv mod 2^kbits) + lo; no orig table
    bool scrambled = false;
    int kbits = 0;
    uint64_t mul = 0, mul_inv = 0;
    int64_t lo = 0;
};

// A rank's shard of a distributed graph (capsmi_graph_distribute): owned dense ids are
// [rank * 32 * slice_words, (rank + 1) * 32 * slice_words) of the scrambled domain
struct Shard {
    int kind = 0;   // 1 node table, 2 relationship table
    int mode = 0;   // node: CAPSMI_NODES_*; relationship: CAPSMI_RELS_*
    int rank = 0, world = 1;
    int64_t slice_words = 0;
    // node table: its rows (over every rank's shard when OWNED) are each id of the whole scrambled
    // domain exactly once, so a predicate-free scan sets every bit without reading a row or exchanging
    bool covers = false;
};

}  // namespace capsmi

namespace capsmi {
// Session configuration: every CAPSMI_* knob of the library, read from the environment
// ONCE, when the session is created (capsmi_session_create), and changed afterwards only through
// capsmi_session_set_config -- no call site reads the environment.  The defaults are the measured
// choices; the non-defaults force the fallback forms (used above a size limit or when a layout does not
// fit) at sizes where tests can check them against the oracle.  Process-wide, outside this struct:
// CAPSMI_CACHE_BYTES (the block cache shared by all sessions, read at the first allocation) and
// CAPSMI_POOL_KEEP_BYTES (the device pool's release threshold, set at each session create).
struct Config {
    int join = 0;                 // CAPSMI_JOIN = auto | direct | hash | radix (0..3): force a join strategy
    bool count_atomic = false;    // CAPSMI_COUNT = atomic: 2-hop count(*) by per-relationship atomic degrees
                                  //   (the form above 2^26 ids) instead of the record partition
    bool rec_full = true;         // CAPSMI_REC_FULL = 0: the undirected record partition's general form also
                                  //   for full node filters
    bool grouped_keys = false;    // CAPSMI_GROUPED = keys: grouped count(DISTINCT c) by the per-binding key sort
    int pairs = 0;                // CAPSMI_PAIRS = packed | uint2 (1 | 2): force the cached layout's pair form
    bool tri_sorted_build = false;  // CAPSMI_TRI_BUILD = sorted: the sort-oriented trigraph build (above 2^24 ids)
    int tri_deg_sample = 0;       // CAPSMI_TRI_DEG_SAMPLE: 1 in k relationships for the degree order (0: auto)
    bool tri_split = true;        // CAPSMI_TRI_SPLIT = 0: the combined (not direction-split) triangle walks
    int tri_vmode_t = 256;        // CAPSMI_TRI_VMODE_T: od(v) threshold of the v-mode walks (0: all u-mode)
    bool und_stream = false;      // CAPSMI_UND = stream: undirected count(DISTINCT) by the streaming form
                                  //   (the form above 2^26 ids) instead of the cell layout
    int vl_bits = 8;              // CAPSMI_VL_BITS: bits per pair of the var-length reverse-pair filter
    int vl_sublog = -1;           // CAPSMI_VL_SUBLOG: filter regions per slice, log2 (-1: auto)
    bool vl_f2 = false;           // CAPSMI_VL_F2 = 1: the second-level filter in the T walk (the sharded form's)
    int64_t coll_chunk = int64_t(1) << 26;  // CAPSMI_COLL_CHUNK: elements per host collective call
    int ingest_threads = 0;       // CAPSMI_INGEST_THREADS (0: OMP_NUM_THREADS, else up to 16 hardware threads)
};
// the environment's values over the defaults
Config config_from_env();
// one knob by its environment name; value NULL = back to the environment's value (or the default).
// Returns false for an unknown name or an unparsable value.
bool config_set(Config& c, const char* name, const char* value);
}  // namespace capsmi

struct capsmi_session {
    capsmi::Config cfg;  // read once at create (capsmi::Config)
    std::shared_ptr<capsmi::AllocCtx> alloc;  // block cache of this session (api.hip)
    struct Param {
        int32_t type = 0;
        bool list = false;
        std::vector<capsmi_value> values;
    };
    std::vector<Param> params;  // query parameters (capsmi_session_set_params)
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;  // current (own or external)
    int num_cus = 256;
    // small pinned staging buffer for scalar read-backs ([0]: read_scalar, [1]: read_scalar_async)
    int64_t* pinned = nullptr;
    hipEvent_t ev_read = nullptr;  // read_scalar_async's copy done
    // per-kernel event timing (capsmi_session_set_profiling)
    bool prof = false;
    std::set<std::string> prof_names;  // the timers that record (empty: all; capsmi_session_set_profiling_names)
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> ev_pool;  // resolved timer events, reused (no event creation inside a timed query)
    hipEvent_t take_event() {
        hipEvent_t e = nullptr;
        if (!ev_pool.empty()) {
            e = ev_pool.back();
            ev_pool.pop_back();
        } else if (hipEventCreate(&e) != hipSuccess) {
            e = nullptr;
        }
        return e;
    }
    std::map<std::string, std::pair<int64_t, double>> totals;
    std::map<std::string, double> alg_bytes;  // algorithmic bytes of the timed launches, per name
    // fused-path routing of lazy plans (plan.hip): enabled flag and per-route counters
    bool fused = true;
    std::map<std::string, int64_t> routes;
    // multi-GPU rank view (capsmi_session_set_ranks): the host's collective on this session's stream
    int rank = 0, world = 1;
    capsmi_collective_fn coll = nullptr;
    void* coll_ctx = nullptr;
    // refuse unrouted joins whose estimated output exceeds this many bytes (0 = no limit;
    // capsmi_session_set_unrouted_limit)
    int64_t unrouted_limit = 0;
    // capsmi_read_csv row ids over Spark's file-scan partitions (capsmi_session_set_csv_partitioning;
    // parallelism 0: one partition)
    int64_t csv_parallelism = 0, csv_max_partition_bytes = int64_t(128) << 20, csv_open_cost = int64_t(4) << 20;
};

namespace capsmi {
// brackets one kernel launch with events on the session stream when profiling is on
struct KernelTimer {
    capsmi_session* s;
    const char* name;
    hipEvent_t a = nullptr, b = nullptr;
    // bytes: the launch's algorithmic bytes (inputs read once, outputs written once), if known
    KernelTimer(capsmi_session* s_, const char* n, double bytes = 0) : s(s_), name(n) {
        if (!s->prof || (!s->prof_names.empty() && !s->prof_names.count(name))) return;
        a = s->take_event();
        b = s->take_event();
        if (a && b) {
            (void)hipEventRecord(a, s->stream);
            if (bytes > 0) s->alg_bytes[name] += bytes;
        } else {
            for (hipEvent_t* e : {&a, &b})
                if (*e) s->ev_pool.push_back(*e);
            a = b = nullptr;
        }
    }
    ~KernelTimer() {
        if (a && b) {
            (void)hipEventRecord(b, s->stream);
            s->pending.push_back({name, a, b});
        }
    }
};
}  // namespace capsmi

struct capsmi_table {
    std::atomic<int> refs{1};
    capsmi_session* sess = nullptr;
    int64_t nrows = 0;               // valid once materialised (plan == null)
    std::vector<capsmi::Column> cols;  // lazy: the schema only (name, type, lazy_nullable)
    std::shared_ptr<capsmi::PlanNode> plan;            // non-null until materialised (plan.hip)
    std::shared_ptr<const capsmi::EntityInfo> entity;  // registered entity table
    // Table.cache on a relationship table (SparkTable.scala:240-246): fused routes keep the layouts
    // they build from it (partitioned 2-hop layout per orientation and id window), freed with the table
    bool keep_layouts = false;
    // dense ids of a compacted graph: node tables `did`, relationship tables `dsrc` / `ddst` (int64 per row)
    std::shared_ptr<capsmi::DenseIds> dense;
    capsmi::Column did, dsrc, ddst;
    std::shared_ptr<const capsmi::Shard> shard;  // this rank's shard of a distributed graph
    // the complement of a relationship shard (dense source / target, exchanged at capsmi_graph_distribute):
    // BY_SOURCE, the relationships of other ranks' sources into this rank's owned ids; BY_TARGET, those of
    // this rank's owned sources into other ranks' ids
    capsmi::Column in_src, in_dst;
    int64_t in_rows = 0;
    bool partitioned = false;  // rows are this rank's partition of a distributed result
    std::map<std::string, std::shared_ptr<capsmi_relpart>> layouts;
    bool lazy() const { return (bool)plan; }
    int find(const std::string& n) const {
        for (size_t i = 0; i < cols.size(); ++i)
            if (cols[i].name == n) return (int)i;
        return -1;
    }
};

struct capsmi_bitmap {
    capsmi_session* sess = nullptr;
    int64_t lo = 0, hi = 0;  // id range
    int64_t nwords = 0;      // ceil((hi - lo) / 32)
    capsmi::Buf words;       // uint32 per 32 ids
    int64_t rows_added = 0;  // rows that set a bit (duplicate detection)
    bool any_dup = false;
    int64_t set_bits = -1;   // cached popcount (-1 = stale)
    bool full = false;       // every id in [lo, hi) is set
};

namespace capsmi {

// ---- kernel launchers (k_*.hip) ------------------------------------------------
// scan / compaction / gather (k_basic.hip)
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, capsmi_session* s);  // out has n+1 entries
void fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t st);
void fill_u8(uint8_t* p, uint8_t v, int64_t n, hipStream_t st);
void iota_i64(int64_t* p, int64_t start, int64_t n, hipStream_t st);
// indices i (ascending) with flags[i] != 0; returns count (synchronises)
int64_t flags_to_indices(capsmi_session* s, const uint8_t* flags, int64_t n, Buf& out_idx);
// the rows i < n with flags[i] set, as (id_base + i, val[i]) columns in row order, sized n; returns the row
// count (read once, after the writes are queued)
int64_t flags_to_rows(capsmi_session* s, const uint8_t* flags, int64_t n, const int64_t* val, int64_t id_base,
                      Buf& out_ids, Buf& out_vals);
// dst[i] = idx[i] < 0 ? null : src[idx[i]]; dst_valid written iff non-null
void gather_col(const int64_t* src, const uint8_t* src_valid, const int64_t* idx, int64_t n,
                int64_t* dst, uint8_t* dst_valid, hipStream_t st);
int64_t read_scalar(capsmi_session* s, const int64_t* dev);
// the same in two halves: the copy is queued now and waited for by read_scalar_wait, so the kernels queued
// in between keep the device busy while the host waits (one outstanding read per session)
void read_scalar_async(capsmi_session* s, const int64_t* dev);
int64_t read_scalar_wait(capsmi_session* s);
void invert_u8(const uint8_t* a, uint8_t* b, int64_t n, hipStream_t st);
void add_i64(int64_t* p, int64_t v, int64_t n, hipStream_t st);
void i64_to_f64(const int64_t* a, int64_t* b, int64_t n, hipStream_t st);

// hashing & grouping (k_hash.hip)
constexpr int kMaxKeys = 8;
struct KeyCols {
    const int64_t* data[kMaxKeys];
    const uint8_t* valid[kMaxKeys];
    int32_t n;
};
struct HashTable {
    Buf slot_row;    // int64, -1 = empty; representative row
    Buf slot_count;  // int64 rows per slot
    int64_t cap = 0; // power of two
};
// Insert rows (skipping rows with a null key when skip_null_keys) into a fresh table.
// slot_of_row[i] = slot id or -1.  count=true maintains slot_count.
void hash_build(capsmi_session* s, const KeyCols& k, int64_t n, bool skip_null_keys, HashTable& ht,
                Buf& slot_of_row);
// For each probe row, the slot holding an equal key of the build side, or -1 (null keys never match).
void hash_probe(capsmi_session* s, const KeyCols& probe, const KeyCols& build, int64_t n,
                const HashTable& ht, Buf& slot_of_probe);
// group ids: dense numbering of occupied slots; gid_of_row[i] (-1 for skipped rows); returns #groups
int64_t hash_group_ids(capsmi_session* s, const HashTable& ht, const Buf& slot_of_row, int64_t n,
                       Buf& gid_of_row, Buf& rep_row_of_gid);
// join: rows of the build side grouped by slot: offsets[cap+1], rows[nbuild]
void hash_group_rows(capsmi_session* s, const HashTable& ht, const Buf& slot_of_row, int64_t n,
                     Buf& offsets, Buf& rows);
// load-balanced expansion: for each probe row p with cnt(p) matches emit (p, k) pairs.
//   cnt(p) = slot>=0 ? count[slot] : (outer ? 1 : 0); pairs written to out_l/out_r (r = -1 for outer pad).
int64_t join_expand(capsmi_session* s, const Buf& slot_of_probe, int64_t nprobe, const HashTable& ht,
                    const Buf& offsets, const Buf& rows, bool left_outer, Buf& out_l, Buf& out_r,
                    Buf* matched_build, int64_t nbuild);
// aggregates (per gid)
void agg_count(const int64_t* gid, const uint8_t* valid, int64_t n, int64_t* out, hipStream_t st);
void agg_sum_i64(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, int64_t* sum,
                 uint8_t* seen, hipStream_t st);
void agg_sum_f64(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, double* sum,
                 uint8_t* seen, hipStream_t st);
void agg_minmax(const int64_t* gid, const int64_t* v, const uint8_t* valid, int64_t n, int type, bool is_max,
                int64_t* out, uint8_t* seen, hipStream_t st);
void avg_finish(const double* sum, const int64_t* cnt, int64_t ng, bool to_i64, int64_t* out, uint8_t* valid,
                hipStream_t st);
void minmax_finish(int64_t* v, int type, bool is_max, int64_t ng, hipStream_t st);
// Collect (k_list.hip): sort_array(collect_list / collect_set) of column (v, valid) per group id
// (ng groups) into a list store
std::shared_ptr<ListStore> collect_lists(capsmi_session* s, const int64_t* gid, int64_t ng, const int64_t* v,
                                         const uint8_t* valid, int type, int64_t n, bool distinct);
// one store holding a's lists, then b's (b's list k becomes a.nlists + k)
std::shared_ptr<ListStore> concat_lists(capsmi_session* s, const ListStore& a, const ListStore& b);
// multi-GPU (k_dist.hip): the session's collective, stream-ordered (capsmi_collective_fn)
void collective(capsmi_session* s, int op, const void* send, void* recv, int64_t count, int dtype);
// calls of the host collective move at most coll_chunk() elements (CAPSMI_COLL_CHUNK); collective() and
// collective_a2av() split larger ones
int64_t coll_chunk(const capsmi_session* s);
// hipFuncAttributeMaxDynamicSharedMemorySize of `kernel`, set once per (device, kernel) and raised only when a
// launch needs more (the attribute call costs host time on every query otherwise; k_part.hip)
void lds_attr(const void* kernel, size_t bytes);
// ALL_TO_ALL_V with host count lists (world entries each); max_pair: the largest entry of the whole count
// matrix (equal on every rank), which fixes the number of rounds
void collective_a2av(capsmi_session* s, const void* send, const int64_t* send_counts, void* recv,
                     const int64_t* recv_counts, int dtype, int64_t max_pair);
int64_t matrix_max(const std::vector<int64_t>& m);
// hash Exchange of u64 words to rank dest[i] (low byte; 0xFF: not sent); dest / words are reordered
// scratch; returns the received words (rank-major), *nrecv of them; synchronises
Buf exchange_words(capsmi_session* s, uint64_t* dest, uint64_t* words, int64_t n, int64_t* nrecv);
// every rank's words concatenated in rank order; synchronises.  budget_bytes > 0: when the gathered words
// (padded staging + result) would exceed the smallest rank's budget, every rank returns an empty Buf with
// *ntotal = -1, together, right after the all-gather of the (count, budget) pairs
Buf gather_words(capsmi_session* s, const uint64_t* words, int64_t n, int64_t* ntotal, int64_t budget_bytes = 0);
// the generic operators' row exchanges over partitioned tables (k_dist.hip): rows to rank dest[r]; rows
// hash-partitioned by key columns; this rank's slice of a replicated table; every rank's rows
capsmi_table* exchange_rows(capsmi_session* s, const capsmi_table* t, uint64_t* dest);
capsmi_table* exchange_by_keys(capsmi_session* s, const capsmi_table* t, const std::vector<int>& keys,
                               const std::vector<int>& as_f64, bool null_local);
capsmi_table* slice_rows(capsmi_session* s, const capsmi_table* t);
capsmi_table* gather_rows(capsmi_session* s, const capsmi_table* t);
// the scrambled domain of [lo, hi) over `world` ranks: kbits, mul, mul_inv, slice words, domain size
struct Scramble {
    int kbits;
    uint64_t mul, mul_inv;
    int64_t lo, hi, slice_words, n;
};
Scramble make_scramble(int64_t lo, int64_t hi, int world);
// out[i] = h(in[i]); counts rows outside [lo, hi) into bad[0] and rows whose h is outside
// [own_lo, own_hi) into bad[1] (when own_lo < own_hi)
void scramble_ids(capsmi_session* s, const Scramble& sc, const int64_t* in, int64_t n, int64_t* out, int64_t own_lo,
                  int64_t own_hi, unsigned long long* bad);
// x = h^-1(d) for n dense ids, in place
void unscramble_ids(capsmi_session* s, const DenseIds& d, int64_t* v, int64_t n);
// flags[i] = h(in[i]) in [own_lo, own_hi) (ids outside [lo, hi): 0)
void owned_flags(capsmi_session* s, const Scramble& sc, const int64_t* in, int64_t n, int64_t own_lo, int64_t own_hi,
                 uint8_t* flags);
// REQUIRE(!is_list_type) for a column used as a key / expression operand
void no_list_key(int32_t type, const std::string& name, const char* what);
// radix-partitioned equi-join (k_rjoin.hip): (probe row, build row) pairs grouped by key-hash
// partition; build row -1 for an unmatched or null-key probe row when `outer`.  Returns #pairs.
int64_t radix_join(capsmi_session* s, const KeyCols& bk, int64_t nb, const KeyCols& pk, int64_t np, bool outer,
                   Buf& out_p, Buf& out_b);
// direct-address join (k_rjoin.hip): single Long key, unique build keys in a dense range; false if
// not eligible (then nothing was produced)
bool direct_join(capsmi_session* s, const KeyCols& bk, int64_t nb, const KeyCols& pk, int64_t np, bool outer,
                 Buf& out_p, Buf& out_b, int64_t* total);
// the same from two partitions of 2-byte records (k_count.hip rec::), the default
// undirected: the 2-hop of undirected Expands (both arcs of every relationship, r1 = r2 bindings subtracted)
int64_t two_hop_count_rec(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                          int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok,
                          bool undirected = false);
void cross_pairs(int64_t nl, int64_t nr, int64_t* out_l, int64_t* out_r, hipStream_t st);

// expressions (k_expr.hip)
struct ExprArgs;
void eval_expr(capsmi_session* s, const capsmi_table* t, int32_t nnodes, const capsmi_expr* prog,
               int64_t* out, uint8_t* out_valid, int32_t* out_type);
// filter flags: 1 where the predicate is TRUE
void eval_predicate(capsmi_session* s, const capsmi_table* t, int32_t nnodes, const capsmi_expr* prog,
                    uint8_t* flags);

// sort (k_sort.hip): stable ascending permutation of row indices by a 64-bit key
void radix_sort_pairs(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, int begin_bit,
                      int end_bit);
// the same over an explicit list of 8-bit digit positions (LSD order; digits no key uses skipped);
// vals may be null (keys only)
void radix_sort_digits(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts);
// the same, calling cb(keys as they stand) on the stream after the first `at` passes (an intermediate
// order, e.g. by the low digits alone; cb(keys) at once when nothing is sorted)
void radix_sort_digits(capsmi_session* s, uint64_t* keys, int64_t* vals, int64_t n, const std::vector<int>& shifts,
                       int at, const std::function<void(const uint64_t*)>& cb);
// keys only; an odd number of passes leaves the result in the sort's other buffer, which `keys` then holds
// (no copy back).  Key-only sorts run in tiles of kSortTile keys: a producer that counts its keys' first digit
// per tile (hist0[d * ntiles + tile], int64, ntiles = ceil(n / kSortTile)) hands that over and the first pass
// skips its histogram read
constexpr int kSortTile = 4096;
void radix_sort_keys(capsmi_session* s, Buf& keys, int64_t n, const std::vector<int>& shifts,
                     const int64_t* hist0 = nullptr);
void order_keys(capsmi_session* s, const int64_t* col, const uint8_t* valid, int type, bool desc, bool null_pass,
                const int64_t* perm, int64_t n, uint64_t* key);

// partitioned relationship layout (k_part.hip)
struct PartLayout {
    int64_t lo, hi;  // id domain of both endpoints
    int nt;          // target slices of 2^19 ids (<= 2048)
    int ns;          // source slices of 2^sbits ids
    int sbits;       // 19 while nt * ns <= 16384, coarser for larger domains
    int ncells;      // nt * ns, j-major (target slice major)
    int tbits;       // target slice = 2^tbits ids (19 for the 2-hop layout)
    int packed = 0;  // 2-hop layout: 5-byte cell-relative pairs (sbits + tbits <= 40), else uint2
};
struct RelPart {
    PartLayout L;
    // per kept relationship, grouped by cell: uint2 (source - lo, target - lo), or when L.packed the
    // cell-relative key k = (source low sbits) << tbits | (target low tbits) as two arrays, the low
    // word u32[cap] and the high byte u8[cap] behind it
    Buf pairs;
    int64_t cap = 0;  // entries per array (kept + slack)
    Buf boff;   // int64 cell offsets (ncells + 1); boff[ncells] = kept
    int64_t kept = 0;  // -1: on the device only (relpart_kept reads it)
    int64_t rows = 0;  // relationships offered to the build (>= kept)
};
int64_t relpart_kept(capsmi_session* s, RelPart& rp);
void relpart_digest(capsmi_session* s, const RelPart& rp, int64_t* counts, uint64_t* sums, int64_t* misplaced);
// hop 1 of a 2-hop run while the layout is built: M(t) |= a_ok(s) for s != t, a_ok self-loops ->
// S1 (first) / S2 (second), target filter b_ok; outputs zeroed by the caller
struct RelPartHop1 {
    const capsmi_bitmap* a;
    const capsmi_bitmap* b;
    uint32_t *M, *S1, *S2;
};
// unpacked: keep 8-byte pairs whatever the domain (a layout walked by kernels that read uint2 pairs only)
void relpart_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
                   int64_t lo, int64_t hi, RelPart& rp, const RelPartHop1* h1 = nullptr, bool unpacked = false);
void relpart_hop1(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* a, const capsmi_bitmap* b, uint32_t* M,
                  uint32_t* S1, uint32_t* S2);
void relpart_hop2(capsmi_session* s, const RelPart& rp, const capsmi_bitmap* c, const uint32_t* X1, const uint32_t* X2,
                  uint32_t* C);

// fused cyclic triangle count (k_tri.hip): the oriented simple graph with multiplicities
struct TriGraph {
    int64_t lo = 0, n = 0, ne = 0;
    Buf ok, ov, off;  // oriented keys (from<<32|to), payload (m(from,to)<<32|m(to,from)), CSR offsets (n + 1)
    // uint32 targets of the oriented edges (the `to` of ok, ib bits) with the edge's two multiplicities
    // in cb bits each above it (all-ones: read ov); ids are the degree order (0 = highest (degree, id))
    Buf tg;
    int ib = 0, cb = 0;
    Buf orig;         // int64 per vertex: relative id of the degree-order id (unused by the count)
    Buf ek, ev, sl;   // undirected keys / payload (pair terms), self-loop counts
    Buf pair;         // the direct build: the pair terms' sum (u64), added up while the runs are written
    Buf small_u, big_u;  // vertices with out-degree in [2, 64] / above 64
    int64_t nsmall = 0, nbig = 0;
    // Direction choice per oriented edge u -> v at position p of out(u) (out-lists are sorted, and
    // every wedge u -> v -> w that can close has w < v, so from v only the prefix out(u)[0, p) needs
    // walking; from u the whole out(v)): with vmt > 0 the edges with od(v) >= vmt and p < od(v) are
    // taken from v ("v-mode"), over the in-lists (ioff, itg, ipos: sources and positions p of the
    // oriented edges grouped by target; the edge is off[u] + p); vm_c = the v-mode centers.
    int vmt = 0;
    Buf ioff, itg, ipos, vm_c;
    // direction-split lists (k_tri.hip "direction-split lists"): tgs = every out_f(x) then every out_b(x),
    // fbo = their starts (2n + 2 uint32); with split set the in-lists are ikey (to << 40 | record index, sorted)
    // and irec (16-byte records: coded source word, pf | pb << 16, the source's f / b list starts) instead of
    // itg / ipos
    bool split = false;
    Buf tgs, fbo, ikey, irec;
    Buf vrec;  // per vertex {f start, b start, f len | b len << 16, od} (k_vrec): one load per list setup
    int64_t nvm = 0;
    // ek / ev entries (= ne on one device; on a rank of a distributed build the undirected edges whose
    // lower end it owns, while ok / tg hold every oriented edge)
    int64_t nek = 0;
    bool dist = false;
    // tri_count's part p of P takes every P-th center of big_u / vm_c / small_u from p (interleaved shares);
    // a distributed build's in-lists hold only the v-mode centers v with v mod world = rank, so vm_c is
    // exactly its share
    bool vm_own = false;
};
// a distributed build (multi-GPU C4): this rank's relationships are any 1/world of them; the owner of a
// dense id x is x / span
struct TriDist {
    int rank = 0, world = 1;
    int64_t span = 0;
};
void tri_build(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms, int nt,
               const capsmi_bitmap* n_ok, TriGraph& g, const TriDist* dd = nullptr);
uint64_t tri_count(capsmi_session* s, const TriGraph& g, int part, int nparts);

// undirected Expand patterns (k_undirected.hip): hops 1 or 2; kind 0 count(*), 1 count(DISTINCT end),
// 2 count(DISTINCT start); c unused for one hop.  marks (kinds 1, 2; b's nwords words): the distinct ids'
// bitmap is written there instead of counted (returns 0) -- a rank's partial marks of a distributed route
int64_t undirected_count(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                         int nt, int hops, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c,
                         int kind, uint32_t* marks = nullptr);
// the undirected 2-hop count(DISTINCT end) over the 2-D cell layout (k_und_part.hip), domains of at most
// 2^26 ids (undirected_distinct_part_ok); marks as above
bool undirected_distinct_part_ok(int64_t n);
int64_t undirected_distinct_part(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts,
                                 const int64_t* ms, int nt, const capsmi_bitmap* a, const capsmi_bitmap* b,
                                 const capsmi_bitmap* c, uint32_t* marks);

// the 2-hop chain grouped by its start (k_grouped.hip): rows (relative start id, count(*) or count(DISTINCT
// end)); false when the distinct keys would exceed key_budget bytes
// dd (a rank of a distributed graph, BY_SOURCE shards: sources owned, dense ids [rank * span, (rank + 1) *
// span) owned): the rows of the owned starts, outC / the hop-2 lists exchanged between the ranks
struct GroupedDist {
    int rank = 0, world = 1;
    int64_t span = 0;
};
bool grouped_two_hop(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                     int nt, const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c, bool distinct,
                     int64_t key_budget, Buf& out_ids, Buf& out_vals, int64_t* rows, const GroupedDist* dd = nullptr);

// fused var-length grouped count (k_varlen.hip)
int64_t var_length_count(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts, const int64_t* ms,
                         int nt, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, int lower, int upper,
                         Buf& out_ids, Buf& out_cnt);

// sharded var-length grouped count (multi-GPU C5; k_varlen.hip): begin -> caller sums od over ranks
// -> mid -> caller sums Y -> finish (rows of owned ids)
struct VarlenShard;
VarlenShard* varlen_shard_begin(capsmi_session* s, const int64_t* const* srcs, const int64_t* const* dsts,
                                const int64_t* ms, int nt, const int64_t* const* isrcs, const int64_t* const* idsts,
                                const int64_t* ims, int nin, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                int lower, int upper, int64_t own_lo, int64_t own_hi, int64_t* od);
void varlen_shard_mid(VarlenShard* v, int64_t* y);
int64_t varlen_shard_finish(VarlenShard* v, Buf& out_ids, Buf& out_cnt);
void varlen_shard_free(VarlenShard* v);

// [min, max] over `ncols` int64 columns of n rows into out[0], out[1] (synchronises); n > 0
void minmax_i64(capsmi_session* s, const int64_t* const* cols, int ncols, int64_t n, int64_t* out);
// widen n input values of width `code` (CAPSMI_IN_* of include/capsmi.h) to 8-byte words
void widen_words(const void* in, int code, int64_t* out, int64_t n, hipStream_t st);

// expressions: static result type and validation of a postfix program over a table's schema (k_expr.hip)
int32_t infer_type(const capsmi_table* t, int32_t nn, const capsmi_expr* prog);
// a program with every CAPSMI_X_PARAM replaced by its literal(s) from the session's parameters
std::vector<capsmi_expr> bind_params(const capsmi_session* s, int32_t nn, const capsmi_expr* prog);
bool has_params(int32_t nn, const capsmi_expr* prog);
void validate_program(const capsmi_table* t, int32_t nn, const capsmi_expr* prog);

// lazy plans (plan.hip): run the plan (a fused kernel when the recogniser matches) and keep the result
void materialize(capsmi_table* t);
// mark a materialised table in canonical entity layout (ids first) as a node (1) / relationship (2)
// table whose ids (endpoints) lie in [lo, hi)
void attach_entity(capsmi_table* t, int kind, int64_t lo, int64_t hi, bool ids_exact = false, bool ids_unique = false);
inline capsmi_table* M(const capsmi_table* t) {
    materialize(const_cast<capsmi_table*>(t));
    return const_cast<capsmi_table*>(t);
}

// eager Table[T] operators over materialised inputs (api.hip)
capsmi_status eager_select(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out);
capsmi_status eager_drop(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out);
capsmi_status eager_with_column_renamed(capsmi_table* t, const char* old_name, const char* new_name, capsmi_table** out);
capsmi_status eager_filter(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog, capsmi_table** out);
capsmi_status eager_filter_keep(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog,
                                const std::vector<std::string>& keep, capsmi_table** out);
capsmi_status eager_with_columns(capsmi_table* t, int32_t ncols, const capsmi_expr_column* cols, capsmi_table** out);
capsmi_status eager_join(capsmi_table* l, capsmi_table* r, int32_t join_type, int32_t npairs, const char* const* lcols,
                         const char* const* rcols, capsmi_table** out);
capsmi_status eager_union_all(capsmi_table* a, capsmi_table* b, capsmi_table** out);
capsmi_status eager_order_by(capsmi_table* t, int32_t nkeys, const char* const* cols, const int32_t* descending,
                             capsmi_table** out);
capsmi_status eager_skip(capsmi_table* t, int64_t n, capsmi_table** out);
capsmi_status eager_limit(capsmi_table* t, int64_t n, capsmi_table** out);
capsmi_status eager_distinct(capsmi_table* t, capsmi_table** out);
capsmi_status eager_distinct_on(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out);
capsmi_status eager_group(capsmi_table* t, int32_t nby, const char* const* by, int32_t naggs, const capsmi_agg* aggs,
                          capsmi_table** out);

// CSV ingest (ingest.hip)
capsmi_table* read_csv(capsmi_session* s, const std::vector<std::string>& paths, char delim, char comment,
                       const std::vector<std::string>& names, const std::vector<int32_t>& types, capsmi_intern_fn intern,
                       void* ctx, const char* row_id_col);

// graph (k_graph.hip)
// node predicate compiled for the bitmap scan: AND of range tests on Long columns (k_graph.hip)
constexpr int kMaxRangeTerms = 4;
struct RangePred {
    int n = 0;
    const int64_t* col[kMaxRangeTerms];
    const uint8_t* valid[kMaxRangeTerms];
    int64_t lo[kMaxRangeTerms], hi[kMaxRangeTerms];  // inclusive
};
// compile `prog` over table t (AND of comparisons Long column <op> Long literal); false if not of that form
bool compile_range_pred(const capsmi_table* t, int32_t nn, const capsmi_expr* prog, RangePred& rp);
void bitmap_add_rows(capsmi_bitmap* b, const int64_t* ids, const uint8_t* ids_valid, const uint8_t* flags, int64_t n,
                     int64_t* dev_counters, const RangePred* rp = nullptr);
void bitmap_set_range(capsmi_bitmap* b, int64_t b0, int64_t b1);  // bits [b0, b1) of the window
int64_t words_popcount(capsmi_session* s, const uint32_t* w, int64_t w_begin, int64_t w_end);
void words_popcount_async(capsmi_session* s, const uint32_t* w, int64_t w_begin, int64_t w_end, int64_t* dev_out);

}  // namespace capsmi
