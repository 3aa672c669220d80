/*
 * capsmi.h -- C ABI of the MI355X execution backend for CAPS pattern matching.
 *
 * This is the drop-in boundary.  In CAPS the backend plug-in
 * point is the Scala trait
 *     trait Table[T <: Table[T]] extends CypherTable
 *     okapi-relational/src/main/scala/org/opencypher/okapi/relational/api/table/Table.scala:43-176
 * implemented for Spark by DataFrameTable
 *     spark-cypher/src/main/scala/org/opencypher/spark/impl/table/SparkTable.scala:47-257
 * A JVM shim (`GpuTable extends Table[GpuTable]`) binds each
 * method below over JNI.  Every entry point cites the Scala member it replaces.
 *
 * Conventions
 *  - Every call returns capsmi_status (0 = OK).  On failure capsmi_last_error()
 *    returns a thread-local message.  The shim maps the codes to the okapi
 *    exception classes (okapi-api/.../impl/exception/InternalException.scala:34-59).
 *  - Handles are opaque and reference counted.  Tables are immutable: every op
 *    returns a NEW table and never modifies its inputs (Table.scala: each op
 *    returns T; inputs stay valid for DAG sharing / cached sub-trees).
 *  - Columns are addressed by name, as in Table.scala (`cols: String*`).
 *  - Values are 8 bytes per row: I64 (Spark LongType), BOOL (0/1), F64 (bits of
 *    an IEEE double), STR (order-preserving dictionary code assigned by the
 *    caller; equal strings <=> equal codes, string order <=> code order).
 *    Nullability is a byte per row (1 = valid), or absent when a column has no nulls.
 *  - A session is externally synchronised (one caller thread, like a CAPS
 *    driver) and owns one HIP stream on one gfx950 device.  Device work is
 *    stream-ordered; calls that return a size to the host synchronise.  Caller
 *    device buffers (ext words, owned_in, dev_out, ...) are read and written in
 *    the session stream's order only: the host orders its own writes to them
 *    before the call (one stream, or an event the session stream waits on).
 */
#ifndef CAPSMI_H
#define CAPSMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------- */
typedef int32_t capsmi_status;
enum {
    CAPSMI_OK = 0,
    CAPSMI_ERR_ILLEGAL_ARGUMENT = 1, /* okapi IllegalArgumentException */
    CAPSMI_ERR_NOT_IMPLEMENTED = 2,  /* okapi NotImplementedException */
    CAPSMI_ERR_UNSUPPORTED = 3,      /* okapi UnsupportedOperationException */
    CAPSMI_ERR_DEVICE = 4,           /* HIP runtime error (no GPU, fault, ...) */
    CAPSMI_ERR_OUT_OF_MEMORY = 5,
    CAPSMI_ERR_INTERNAL = 6          /* okapi InternalException */
};

/* ---- handles ----------------------------------------------------------------- */
typedef struct capsmi_session capsmi_session;
typedef struct capsmi_table capsmi_table;
typedef struct capsmi_bitmap capsmi_bitmap;

/* ---- value types (CypherType -> physical type, SparkConversions.scala:55-168) -- */
enum {
    CAPSMI_I64 = 0,  /* CTInteger, CTNode/CTRelationship ids (Long) */
    CAPSMI_BOOL = 1, /* CTBoolean, label / rel-type flag columns */
    CAPSMI_F64 = 2,  /* CTFloat */
    CAPSMI_STR = 3   /* CTString, dictionary code */
};

/* List columns (CTList(elem)): the result of a Collect aggregator (SparkTable.scala:169-177,
 * functions.sort_array(collect_list / collect_set)).  The column type is CAPSMI_LIST + element type
 * (CAPSMI_LIST_I64 ... CAPSMI_LIST_STR); rows are read with capsmi_table_export_list.  List columns
 * travel through select / drop / rename / filter / join payloads / union all / order-by payloads /
 * skip / limit; using one as a join, grouping, distinct or sort key, or inside an expression, is
 * CAPSMI_ERR_NOT_IMPLEMENTED. */
enum {
    CAPSMI_LIST = 8,
    CAPSMI_LIST_I64 = 8,
    CAPSMI_LIST_BOOL = 9,
    CAPSMI_LIST_F64 = 10,
    CAPSMI_LIST_STR = 11
};

/* Input-only value widths of capsmi_col_desc.type: widened at ingest the way
 * DataFrameOps.withCypherCompatibleTypes lifts Spark columns (spark-cypher/.../impl/DataFrameOps.scala:185-198,
 * SparkConversions.scala:162-168): Byte/Short/Integer -> Long, Float -> Double; a Boolean byte -> BOOL. */
enum {
    CAPSMI_IN_I32 = 16,  /* int32  -> CAPSMI_I64 */
    CAPSMI_IN_I16 = 17,  /* int16  -> CAPSMI_I64 */
    CAPSMI_IN_I8 = 18,   /* int8   -> CAPSMI_I64 */
    CAPSMI_IN_F32 = 19,  /* float  -> CAPSMI_F64 */
    CAPSMI_IN_BOOL8 = 20 /* uint8 0/1 -> CAPSMI_BOOL */
};

typedef struct {
    const char* name;
    int32_t type;         /* CAPSMI_I64 ... CAPSMI_STR, or a CAPSMI_IN_* width */
    const void* data;     /* nrows x 8 bytes (nrows x the CAPSMI_IN_* width) */
    const uint8_t* valid; /* nrows bytes (1 = non-null) or NULL (no nulls) */
} capsmi_col_desc;

/* ---- expressions: postfix programs over one row -------------------------------
 * Subset of SparkSQLExprMapper.asSparkSQLExpr (spark-cypher/.../impl/SparkSQLExprMapper.scala:81-312)
 * that the pattern-matching path needs: column refs (Var/Property/HasLabel/HasType/StartNode/EndNode
 * resolve to columns, :97-105), literals and params (:86-92, :111-117), Equals (:120), Not (:121),
 * IsNull/IsNotNull (:122-123), Ands/Ors (:132-136), In (:138-145), < <= > >= (:147-150), arithmetic.
 * Evaluation follows SQL three-valued logic; Filter keeps rows whose value is TRUE. */
enum {
    CAPSMI_X_COL = 0,      /* push column `arg` (index into the input table) */
    CAPSMI_X_LIT = 1,      /* push literal of type `type`, bits in `ival` */
    CAPSMI_X_NULL = 2,     /* push NULL; arg = 1 + declared type (0 = untyped) */
    CAPSMI_X_EQ = 3,       /* pop b, a; push a = b */
    CAPSMI_X_NEQ = 4,
    CAPSMI_X_LT = 5,
    CAPSMI_X_LE = 6,
    CAPSMI_X_GT = 7,
    CAPSMI_X_GE = 8,
    CAPSMI_X_NOT = 9,
    CAPSMI_X_AND = 10,     /* pop `arg` operands, push conjunction (3VL) */
    CAPSMI_X_OR = 11,      /* pop `arg` operands, push disjunction (3VL) */
    CAPSMI_X_ISNULL = 12,
    CAPSMI_X_ISNOTNULL = 13,
    CAPSMI_X_IN = 14,      /* stack [x, v1..v_arg]: x IN (v1..v_arg), 3VL */
    CAPSMI_X_ADD = 15,
    CAPSMI_X_SUB = 16,
    CAPSMI_X_MUL = 17,
    CAPSMI_X_NEG = 18,
    CAPSMI_X_COALESCE = 19, /* pop `arg` operands, push the first non-null */
    CAPSMI_X_BITAND = 20,   /* Long a & b (SparkSQLExprMapper.scala:264-265) */
    CAPSMI_X_BITOR = 21,    /* Long a | b (:267-268) */
    CAPSMI_X_SHL = 22,      /* Long a << (b & 63) (:270-271, functions.shiftLeft) */
    CAPSMI_X_SHRU = 23,     /* Long a >>> (b & 63) (:273-274, functions.shiftRightUnsigned) */
    CAPSMI_X_CASE = 24,     /* stack [p1, v1, .., p_arg, v_arg, default]: v_i of the first TRUE p_i, else
                               default (push a NULL for none); CaseExpr, :283-298 */
    CAPSMI_X_PARAM = 25     /* push query parameter `arg` of the session's table (capsmi_session_set_params);
                               bound to a literal when the program enters the library, as Param(name) ->
                               functions.lit (:86-92).  A list parameter may only be an element operand of
                               IN, where it expands to its values (:86-89, functions.array) */
};

typedef struct {
    int32_t op;
    int32_t arg;
    int32_t type; /* literal type for CAPSMI_X_LIT */
    int32_t reserved;
    int64_t ival; /* literal payload (int64 / 0|1 / dictionary code / double bits) */
} capsmi_expr;

typedef struct {
    const char* name;        /* output column (replaced if it exists, else appended) */
    int32_t nnodes;
    const capsmi_expr* prog;
} capsmi_expr_column;

/* ---- joins and aggregates (PhysicalConstants.scala:29-40, SparkTable.scala:121-188) ---- */
enum {
    CAPSMI_JOIN_INNER = 0,
    CAPSMI_JOIN_LEFT_OUTER = 1,
    CAPSMI_JOIN_RIGHT_OUTER = 2,
    CAPSMI_JOIN_FULL_OUTER = 3,
    CAPSMI_JOIN_CROSS = 4
};

enum {
    CAPSMI_AGG_COUNT_STAR = 0, /* count(lit 0)                  SparkTable.scala:148-149 */
    CAPSMI_AGG_COUNT = 1,      /* count / countDistinct         SparkTable.scala:152-158 */
    CAPSMI_AGG_MIN = 2,        /*                               SparkTable.scala:163-164 */
    CAPSMI_AGG_MAX = 3,        /*                               SparkTable.scala:160-161 */
    CAPSMI_AGG_SUM = 4,        /*                               SparkTable.scala:166-167 */
    CAPSMI_AGG_AVG = 5,        /* avg -> F64                    SparkTable.scala:141-146 */
    CAPSMI_AGG_COLLECT = 6     /* sort_array(collect_list) / sort_array(collect_set) when `distinct`:
                                  the group's non-null values in ascending order, a list column
                                  (an empty list for a group without values)  SparkTable.scala:169-177 */
};

typedef struct {
    int32_t kind;
    int32_t distinct;        /* COUNT only */
    const char* input;       /* input column (ignored for COUNT_STAR) */
    const char* output;      /* result column name */
} capsmi_agg;

/* ---- errors / session ----------------------------------------------------------- */
/* copies the calling thread's last error message into buf (NUL-terminated); returns its length */
size_t capsmi_last_error(char* buf, size_t n);
const char* capsmi_version(void);

/* CAPSSession.local()/create (spark-cypher/.../api/CAPSSession.scala:110-131): one device, one stream */
capsmi_status capsmi_session_create(int32_t device, capsmi_session** out);
capsmi_status capsmi_session_destroy(capsmi_session* s);
/* run subsequent work on an external hipStream_t (e.g. torch's current stream); NULL = session stream.
 * The previous stream is drained first (the session's cached device blocks then move with it); an
 * external stream must outlive the session or the next switch away from it. */
capsmi_status capsmi_session_set_stream(capsmi_session* s, void* hip_stream);
/* run subsequent work on exactly `hip_stream`; NULL = the HIP null (legacy default) stream -- what
 * torch's default stream is, so kernels and torch work stay ordered */
capsmi_status capsmi_session_use_stream(capsmi_session* s, void* hip_stream);
capsmi_status capsmi_session_sync(capsmi_session* s);
/* session configuration (ConfigOption / CoraConfiguration analogue): every CAPSMI_* knob is
 * read from the environment once, at capsmi_session_create; this changes one for this session only.
 * `name` is the knob's environment name (e.g. "CAPSMI_JOIN", "CAPSMI_COUNT"), `value` its text as the
 * environment would hold it, NULL = back to the environment's value at the time of the call (or the
 * default).  Unknown names and unparsable values are refused (CAPSMI_ERR_ILLEGAL_ARGUMENT).  The knobs and
 * their meaning: DESIGN.md §5a. */
capsmi_status capsmi_session_set_config(capsmi_session* s, const char* name, const char* value);
/* the same check without a session or device: CAPSMI_OK when capsmi_session_set_config would accept it */
capsmi_status capsmi_config_check(const char* name, const char* value);
/* per-kernel HIP-event timing of the fused graph kernels (off by default; SURVEY.md §5 tracing).
 * While enabled, each hot launch is bracketed by events on the session stream.  Enabling creates a pool of
 * events up front (resolved ones return to it), so timed queries make no event-creation calls. */
capsmi_status capsmi_session_set_profiling(capsmi_session* s, int32_t enabled);
/* which timers record while profiling is on: a comma-separated list of kernel names ("part_scatter1,hop2");
 * NULL or "" = every timer (the default).  Each timed launch adds two event records to the stream (a few
 * microseconds of device idle each), so a timed run can bracket only the launch it reports. */
capsmi_status capsmi_session_set_profiling_names(capsmi_session* s, const char* names);
/* resolve pending events (synchronises) and report totals for kernel `name` ("hop1", "hop2",
 * "expand_filter", "bitmap_add", ...): launches and summed milliseconds; then the counters reset. */
capsmi_status capsmi_session_kernel_time(capsmi_session* s, const char* name, int64_t* launches, double* total_ms);
/* summed algorithmic bytes (inputs read once, outputs written once) of the timed launches of `name`,
 * for kernels that declare them (the join kernels: "direct_join_probe", "radix_join_count",
 * "radix_join_write"); 0 otherwise; then the counter resets. */
capsmi_status capsmi_session_kernel_bytes(capsmi_session* s, const char* name, double* bytes);
/* fused-path routing of lazy plans: enable / disable (default on; off = operator by operator, for
 * A/B checks), and the number of plans routed to fused entry point `name` ("expand", "expand_count",
 * "two_hop", "triangle", "var_length") since the session started */
capsmi_status capsmi_session_set_fused(capsmi_session* s, int32_t enabled);
/* query parameters (the CypherMap handed to asSparkSQLExpr): CAPSMI_X_PARAM `arg` = index into
 * `params`.  A scalar has count 1 (is_list 0); a list has is_list 1 and `count` values.  Values are
 * copied; programs built after the call see them. */
typedef struct {
    int64_t ival;     /* literal payload, as capsmi_expr.ival */
    int32_t is_null;
    int32_t reserved;
} capsmi_value;
typedef struct {
    int32_t type;     /* CAPSMI_I64 / F64 / BOOL / STR (dictionary code) */
    int32_t is_list;
    int32_t count;
    int32_t reserved;
    const capsmi_value* values;
} capsmi_param;
capsmi_status capsmi_session_set_params(capsmi_session* s, int32_t nparams, const capsmi_param* params);
/* route "miss" counts materialisations in which a pattern over entity tables (joins of node and
 * relationship scans) matched no fused shape and ran operator by operator */
capsmi_status capsmi_session_route_count(capsmi_session* s, const char* name, int64_t* count);
/* refuse (CAPSMI_ERR_UNSUPPORTED, before any work) an unrouted join whose estimated output -- System-R
 * row estimates, entity key columns' distinct counts from their scans -- exceeds max_bytes of 8-byte
 * words; 0 (the default) = no limit.  A guard against a pattern that misses every fused shape and
 * would materialise its bindings (~10^13 rows at the C3 scale). */
capsmi_status capsmi_session_set_unrouted_limit(capsmi_session* s, int64_t max_bytes);

/* ---- tables (CypherTable: okapi-api/.../api/table/CypherTable.scala:41-68) -------- */
/* CAPSNodeTable/CAPSRelationshipTable ingest (spark-cypher/.../api/io/CAPSTable.scala:47-214): copies */
capsmi_status capsmi_table_from_host(capsmi_session* s, int32_t ncols, const capsmi_col_desc* cols,
                                     int64_t nrows, capsmi_table** out);
/* same, but `data`/`valid` are device pointers on this session's device (copied, stream-ordered) */
capsmi_status capsmi_table_from_device(capsmi_session* s, int32_t ncols, const capsmi_col_desc* cols,
                                       int64_t nrows, capsmi_table** out);
capsmi_status capsmi_table_retain(capsmi_table* t);
capsmi_status capsmi_table_release(capsmi_table* t);
/* CypherTable.size -> DataFrameTable.size = df.count() (SparkTable.scala:59) */
capsmi_status capsmi_table_size(const capsmi_table* t, int64_t* out);
/* CypherTable.physicalColumns / columnType (SparkTable.scala:51-53) */
capsmi_status capsmi_table_num_columns(const capsmi_table* t, int32_t* out);
capsmi_status capsmi_table_column_name(const capsmi_table* t, int32_t col, char* buf, size_t n);
capsmi_status capsmi_table_column_type(const capsmi_table* t, int32_t col, int32_t* out);
capsmi_status capsmi_table_column_index(const capsmi_table* t, const char* name, int32_t* out);
capsmi_status capsmi_table_column_nullable(const capsmi_table* t, int32_t col, int32_t* out);
/* the whole schema in one call (no materialisation): *ncols columns; names NUL-separated into
 * `names` (names_len bytes), types[i] and nullable[i] for i < min(*ncols, max_cols); ILLEGAL_ARGUMENT
 * if the names do not fit */
capsmi_status capsmi_table_schema(const capsmi_table* t, int32_t* ncols, char* names, size_t names_len, int32_t* types,
                                  int32_t* nullable, int32_t max_cols);
/* CypherTable.rows / CAPSRecords.collect (SparkTable.scala:55-57, CAPSRecords.scala:136-143):
 * copies rows [offset, offset+n) of one column to the host; host_valid may be NULL */
capsmi_status capsmi_table_export(const capsmi_table* t, int32_t col, void* host_data, uint8_t* host_valid,
                                  int64_t offset, int64_t n);
/* rows [offset, offset+n) of a list column (CAPSMI_LIST_*) to the host: row i's elements are
 * host_values[host_offsets[i] .. host_offsets[i+1]) (host_offsets has n + 1 entries; a null row is
 * empty with host_valid[i] = 0; host_valid may be NULL).  *nvalues = the number of elements of the
 * range; host_values == NULL only reports it (host_offsets may then be NULL too); otherwise
 * values_cap must be >= *nvalues, else ILLEGAL_ARGUMENT.  Elements are 8-byte words of the element
 * type.  (CAPSRecords.collect of a CTList column, rowToCypherMap.scala) */
capsmi_status capsmi_table_export_list(const capsmi_table* t, int32_t col, int64_t offset, int64_t n,
                                       int64_t* host_offsets, uint8_t* host_valid, void* host_values,
                                       int64_t values_cap, int64_t* nvalues);
/* zero-copy device view of a column (valid pointer NULL when the column has no nulls) */
capsmi_status capsmi_table_column_device_ptr(const capsmi_table* t, int32_t col, const void** data,
                                             const uint8_t** valid);

/* ---- entity tables (the input contract) ------------------------------------------------
 * CAPSNodeTable / CAPSRelationshipTable construction with EntityTable.verify
 * (okapi-relational/.../api/io/EntityTable.scala:59-65, 105-131, 155-164): the id keys must be
 * non-nullable Long columns ("id key", "start node", "end node"), optional-label and relationship-type
 * flag columns non-nullable Boolean, and the columns in canonical order
 *   node: [id, label flags..., properties sorted by name]
 *   rel:  [id, source, target, type flags..., properties sorted by name]     (EntityMapping.scala:50)
 * else CAPSMI_ERR_ILLEGAL_ARGUMENT.  The result shares the input's columns and is what the fused-path
 * recogniser (below) treats as a scanned entity table; registration records the id range. */
capsmi_status capsmi_node_table(capsmi_table* t, const char* id_col, int32_t nlabels, const char* const* label_cols,
                                capsmi_table** out);
capsmi_status capsmi_rel_table(capsmi_table* t, const char* id_col, const char* src_col, const char* dst_col,
                               int32_t ntypes, const char* const* type_cols, capsmi_table** out);
/* Graph-level id compaction (the analogue of caching a graph at creation, CAPSGraphFactory.create /
 * CachedDataSource): numbers every node id of `nodes` and every endpoint of `rels` densely and keeps
 * the dense columns with the tables, so graphs whose Long ids are sparse, large or carry tag bits
 * (Tags.scala:36-55) reach the fused kernels.  Results keep the original ids. */
capsmi_status capsmi_graph_compact(capsmi_session* s, int32_t nnodes, capsmi_table* const* nodes, int32_t nrels,
                                   capsmi_table* const* rels, int64_t* dense_ids);
/* kind 0 = plain table, 1 = node table, 2 = relationship table; [*id_lo, *id_hi) = range of the ids
 * (node) or of both endpoints (relationship) */
capsmi_status capsmi_table_entity(const capsmi_table* t, int32_t* kind, int64_t* id_lo, int64_t* id_hi);
/* CAPSRelationshipTable.fromMapping's relationship-type flattening (spark-cypher/.../api/io/CAPSTable.scala:189-204):
 * the String column `type_col` (dictionary codes) becomes one non-nullable Boolean column per type,
 * out_cols[i] = (type_col = type_codes[i]), and type_col is dropped. */
capsmi_status capsmi_flatten_rel_types(capsmi_table* t, const char* type_col, int32_t ntypes, const int64_t* type_codes,
                                       const char* const* out_cols, capsmi_table** out);

/* ---- Table[T] operators -------------------------------------------------------------
 * Operators are lazy, like DataFrameTable's Spark plans: each returns a table whose schema is known
 * at once (name / type / nullability queries, errors for unknown columns or bad programs) and whose
 * rows are computed when first needed -- capsmi_table_size, _export, _column_device_ptr,
 * _fingerprint, or a graph entry point consuming it (RelationalCypherRecords.size -> df.count(),
 * SparkTable.scala:59).  At that point the plan is matched against the fused graph kernels: joins of
 * registered node / relationship tables in the Expand / ExpandInto / BoundedVarLengthExpand shapes
 * RelationalPlanner emits (RelationalPlanner.scala:113-177, VarLengthExpandPlanner.scala:46-310),
 * their uniqueness and node filters, and the aggregate or projection on top run as one fused call;
 * anything else runs operator by operator.  A materialised table keeps its rows (shared sub-plans
 * run once: the Cache analogue). */
capsmi_status capsmi_cache(capsmi_table* t, capsmi_table** out);                         /* Table.scala:52  */
capsmi_status capsmi_select(capsmi_table* t, int32_t ncols, const char* const* cols,
                            capsmi_table** out);                                        /* Table.scala:60  */
capsmi_status capsmi_filter(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog,
                            capsmi_table** out);                                        /* Table.scala:70  */
capsmi_status capsmi_drop(capsmi_table* t, int32_t ncols, const char* const* cols,
                          capsmi_table** out);                                          /* Table.scala:78  */
capsmi_status capsmi_join(capsmi_table* l, capsmi_table* r, int32_t join_type, int32_t npairs,
                          const char* const* lcols, const char* const* rcols,
                          capsmi_table** out);                                          /* Table.scala:88  */
capsmi_status capsmi_union_all(capsmi_table* a, capsmi_table* b, capsmi_table** out);   /* Table.scala:96  */
capsmi_status capsmi_order_by(capsmi_table* t, int32_t nkeys, const char* const* cols,
                              const int32_t* descending, capsmi_table** out);           /* Table.scala:104 */
capsmi_status capsmi_skip(capsmi_table* t, int64_t n, capsmi_table** out);              /* Table.scala:112 */
capsmi_status capsmi_limit(capsmi_table* t, int64_t n, capsmi_table** out);             /* Table.scala:120 */
capsmi_status capsmi_distinct(capsmi_table* t, capsmi_table** out);                     /* Table.scala:127 */
capsmi_status capsmi_distinct_on(capsmi_table* t, int32_t ncols, const char* const* cols,
                                 capsmi_table** out);                                   /* SparkTable.scala:234-235 */
capsmi_status capsmi_group(capsmi_table* t, int32_t nby, const char* const* by, int32_t naggs,
                           const capsmi_agg* aggs, capsmi_table** out);                 /* Table.scala:147 */
capsmi_status capsmi_with_columns(capsmi_table* t, int32_t ncols, const capsmi_expr_column* cols,
                                  capsmi_table** out);                                  /* Table.scala:159 */
capsmi_status capsmi_with_column_renamed(capsmi_table* t, const char* old_name, const char* new_name,
                                         capsmi_table** out);                           /* Table.scala:168 */

/* ---- graph fast path ------------------------------------------------------------------
 * The relational planner lowers Expand into `join(relScan, source = start)` then
 * `join(nodeScan, end = target)` (RelationalPlanner.scala:113-137).  When the shim sees that
 * shape over base entity tables with dense Long ids it calls these fused entry points
 * instead; results are identical row multisets.
 *
 * A capsmi_bitmap is a node scan + label/property predicate (ScanGraph.scanOperator,
 * ScanGraph.scala:61-96, plus Filter) collapsed to one bit per id in [id_lo, id_hi). */
capsmi_status capsmi_bitmap_create(capsmi_session* s, int64_t id_lo, int64_t id_hi, capsmi_bitmap** out);
/* OR in the ids of node-table rows whose predicate is TRUE (nnodes = 0: every row).
 * Ids outside [id_lo, id_hi) or null ids are an ILLEGAL_ARGUMENT error. */
capsmi_status capsmi_bitmap_add_scan(capsmi_bitmap* b, capsmi_table* nodes, const char* id_col,
                                     int32_t nnodes, const capsmi_expr* pred);
/* number of set bits, and whether every scanned row contributed a distinct id (no id in two
 * scanned rows: the fused paths require it, since CAPS would emit one row per table occurrence,
 * ScanGraph.scala:72-76) */
capsmi_status capsmi_bitmap_stats(capsmi_bitmap* b, int64_t* set_bits, int32_t* unique_rows);
capsmi_status capsmi_bitmap_release(capsmi_bitmap* b);
/* the bitmap's device words (uint32, bit i of word w <-> id lo + 32w + i) for collectives: a rank
 * scans its owned node rows, the ranks all-gather their owned word slices into these words, then
 * capsmi_bitmap_refresh re-derives the set-bit count (synchronises); `unique_rows` states whether
 * every rank's scan was duplicate-free (the all-reduced AND of capsmi_bitmap_stats) */
capsmi_status capsmi_bitmap_words(capsmi_bitmap* b, uint32_t** words, int64_t* nwords);
capsmi_status capsmi_bitmap_refresh(capsmi_bitmap* b, int32_t unique_rows);
/* the same without the device popcount (no synchronisation): the caller states the set-bit count,
 * e.g. the all-reduced sum of every rank's capsmi_bitmap_stats over its owned rows, taken before
 * the all-gather */
capsmi_status capsmi_bitmap_assume(capsmi_bitmap* b, int64_t set_bits, int32_t unique_rows);
/* stream-ordered device copy of words [w_begin, w_end): to_bitmap = 0 copies bitmap -> ext,
 * 1 copies ext -> bitmap (ext: a caller device buffer of w_end - w_begin words).  Like every call
 * taking a caller device pointer, the copy is queued on the SESSION's stream: `ext` must already be
 * written (allocated, zero-filled, ...) in that stream's order -- run the host's own device work on
 * the same stream (capsmi_session_use_stream) or make the session stream wait on it -- and the host
 * may read it only after capsmi_session_sync or stream-ordered work behind it */
capsmi_status capsmi_bitmap_copy_words(capsmi_bitmap* b, int64_t w_begin, int64_t w_end, uint32_t* ext,
                                       int32_t to_bitmap);

/* 1-hop Expand + node filters, fused (C2):
 *   MATCH (a)-[r]->(b) WHERE src_ok(a) AND dst_ok(b)
 * = rels ⋈ a-scan ⋈ b-scan; returns the rel rows that survive, projected on `out_cols`
 * (renamed to `out_names`, or kept when out_names == NULL). */
capsmi_status capsmi_expand_filter(capsmi_session* s, capsmi_table* rels, const char* src_col,
                                   const char* dst_col, const capsmi_bitmap* src_ok,
                                   const capsmi_bitmap* dst_ok, int32_t nout, const char* const* out_cols,
                                   const char* const* out_names, capsmi_table** out);

/* 2-hop with relationship uniqueness (C3), fused, never materialising the bindings:
 *   MATCH (a)-[r1]->(b)-[r2]->(c) WHERE a_ok(a) AND b_ok(b) AND c_ok(c)   [r1 <> r2 implied]
 *   RETURN count(DISTINCT c)
 * `rels` is one or more relationship tables of the scanned type (their union is the rel scan). */
capsmi_status capsmi_two_hop_count_distinct(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                            const char* src_col, const char* dst_col,
                                            const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                            const capsmi_bitmap* c_ok, int64_t* out_distinct);
/* count(*) of the same MATCH, closed form: sum_b [b_ok] inA(b) * outC(b) - #eligible self-loops */
capsmi_status capsmi_two_hop_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                   const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                   const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, int64_t* out_rows);

/* Phased form of capsmi_two_hop_count_distinct for the multi-GPU path.  The caller
 * owns the exchange (RCCL all-gather of the owned bitmap slice between the two phases).
 * Bitmaps are uint32 words, bit i of word w <-> id lo+32w+i; mid_words span b_ok's id range and
 * dst_words c_ok's.
 * mid_words:  2 x nwords (X1 then X2), zeroed by the call.  X1(b): b can be the middle of a 2-hop
 *             whose second edge is not a self-loop; X2(b): ... whose second edge is a self-loop at b.
 * dst_words:  nwords, zeroed by the call; marks every reachable c.  `scratch_words`: nwords. */
capsmi_status capsmi_two_hop_mark_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                      const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                      const capsmi_bitmap* b_ok, uint32_t* mid_words, uint32_t* scratch_words);
capsmi_status capsmi_two_hop_mark_dst(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                      const char* src_col, const char* dst_col, const capsmi_bitmap* b_ok,
                                      const capsmi_bitmap* c_ok, const uint32_t* mid_words, uint32_t* dst_words);
/* Radix-partitioned relationship layout for the 2-hop kernels: rows of the union of `rels` with both
 * endpoints in [id_lo, id_hi) (hi - lo <= 2^30), packed to 32-bit ids and grouped by 2-D cell
 * (target slice of 2^19 ids) x (source slice).  Building it is part of the cold query; keeping it
 * across queries is the Cache analogue (DataFrameTable.cache, SparkTable.scala:240-246). */
typedef struct capsmi_relpart capsmi_relpart;
capsmi_status capsmi_relpart_build(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                   const char* dst_col, int64_t id_lo, int64_t id_hi, capsmi_relpart** out);
capsmi_status capsmi_relpart_size(const capsmi_relpart* p, int64_t* kept_rows);
capsmi_status capsmi_relpart_release(capsmi_relpart* p);
/* Layout check (test support, synchronous): per 2-D cell c (target slice major) the number of pairs and
   the wrapping sum of mix64((source - lo) << 32 | (target - lo)) over them; pairs stored outside their
   own cell are counted in *misplaced.  counts/sums hold *ncells entries each; pass NULL arrays to read
   the cell geometry only (*ncells, *ns = source slices per target slice, *sbits, *tbits). */
capsmi_status capsmi_relpart_digest(const capsmi_relpart* p, int64_t* ncells, int64_t* ns, int32_t* sbits,
                                    int32_t* tbits, int64_t* counts, uint64_t* sums, int64_t* misplaced);
/* capsmi_relpart_build followed by capsmi_two_hop_mark_mid_part, with hop 1 run by the build's second
 * pass when a_ok covers the whole id domain (the cold 2-hop: one pass fewer over the relationships) */
capsmi_status capsmi_relpart_build_mark_mid(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                            const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                            const capsmi_bitmap* b_ok, uint32_t* mid_words, uint32_t* scratch_words,
                                            capsmi_relpart** out);
/* the phased 2-hop over a partitioned layout (same contract as capsmi_two_hop_mark_mid/_dst) */
capsmi_status capsmi_two_hop_mark_mid_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* a_ok,
                                           const capsmi_bitmap* b_ok, uint32_t* mid_words, uint32_t* scratch_words);
capsmi_status capsmi_two_hop_mark_dst_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* b_ok,
                                           const capsmi_bitmap* c_ok, const uint32_t* mid_words, uint32_t* dst_words);
/* whole query over a cached layout */
capsmi_status capsmi_two_hop_count_distinct_part(capsmi_session* s, const capsmi_relpart* p, const capsmi_bitmap* a_ok,
                                                 const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok,
                                                 int64_t* out_distinct);
/* Undirected Expand patterns, fused.  An undirected Expand is the union of the outgoing branch and the
 * incoming branch over relationships whose start differs from their end (RelationalPlanner.scala:126-136):
 *   hops = 1: MATCH (a)-[r]-(b) WHERE a_ok(a) AND b_ok(b)
 *   hops = 2: MATCH (a)-[r1]-(b)-[r2]-(c) WHERE a_ok(a) AND b_ok(b) AND c_ok(c)   [r1 <> r2 implied]
 * RETURN count(*) (kind 0), count(DISTINCT the last node) (kind 1) or count(DISTINCT a) (kind 2); c_ok
 * is ignored for one hop.  The bitmaps share one id domain. */
capsmi_status capsmi_undirected_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                      const char* dst_col, int32_t hops, const capsmi_bitmap* a_ok,
                                      const capsmi_bitmap* b_ok, const capsmi_bitmap* c_ok, int32_t kind, int64_t* out);
/* BoundedVarLengthExpand + grouped count, fused (C5):
 *   MATCH (a)-[r*lower..upper]->(b) WHERE a_ok(a) AND b_ok(b) RETURN id(a) AS <id_name>, count(*) AS <count_name>
 * with edge-distinct paths (VarLengthExpandPlanner.scala:83-136, 179-180), 0 <= lower <= upper <= 4,
 * upper >= 1 (upper 4: ids below 2^24 - 1).  lower = 0 adds the zero-length path of every a_ok node (copyEntity, :146-153, 190-210:
 * b is a copy of a, without b's node scan).  One output row per a with at least one path.  a_ok and
 * b_ok must share one id domain. */
capsmi_status capsmi_var_length_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels,
                                      const char* src_col, const char* dst_col, const capsmi_bitmap* a_ok,
                                      const capsmi_bitmap* b_ok, int32_t lower, int32_t upper, const char* id_name,
                                      const char* count_name, capsmi_table** out);
/* Sharded form of capsmi_var_length_count for one rank of a multi-GPU run.  The
 * rank owns the source ids [own_lo, own_hi); `out_rels` hold the relationships whose source it
 * owns, `in_rels` those from other ranks' sources into its owned ids.  `od` and `y` are caller
 * device buffers of (b_ok->hi - b_ok->lo) int64 each:
 *   begin  writes the rank's partial out-degrees into od -> the caller sums od over ranks in place;
 *   mid    writes the rank's partial Y into y            -> the caller sums y over ranks in place;
 *   finish returns the (id, count) rows of the owned ids.  od / y must stay valid until finish. */
typedef struct capsmi_varlen_shard capsmi_varlen_shard;
capsmi_status capsmi_varlen_shard_begin(capsmi_session* s, int32_t nout, capsmi_table* const* out_rels, int32_t nin,
                                        capsmi_table* const* in_rels, const char* src_col, const char* dst_col,
                                        const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok, int32_t lower,
                                        int32_t upper, int64_t own_lo, int64_t own_hi, int64_t* od,
                                        capsmi_varlen_shard** out);
capsmi_status capsmi_varlen_shard_mid(capsmi_varlen_shard* v, int64_t* y);
capsmi_status capsmi_varlen_shard_finish(capsmi_varlen_shard* v, const char* id_name, const char* count_name,
                                         capsmi_table** out);
capsmi_status capsmi_varlen_shard_release(capsmi_varlen_shard* v);
/* Cyclic triangle count (C4), fused:
 *   MATCH (a)-[r1]->(b)-[r2]->(c)-[r3]->(a) WHERE n_ok(a) AND n_ok(b) AND n_ok(c) RETURN count(*)
 * (two Expands + ExpandInto on (c, a), RelationalPlanner.scala:113-154, plus pairwise uniqueness).
 * The oriented simple graph with multiplicities (a trigraph) is built once; counting can be split into
 * `nparts` interleaved shares of its centers (multi-GPU replicas: each rank counts its part, results sum). */
typedef struct capsmi_trigraph capsmi_trigraph;
capsmi_status capsmi_trigraph_build(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                    const char* dst_col, const capsmi_bitmap* n_ok, capsmi_trigraph** out);
capsmi_status capsmi_trigraph_count(capsmi_session* s, const capsmi_trigraph* g, int32_t part, int32_t nparts,
                                    int64_t* out_rows);
/* id-domain size and number of oriented (simple, both directions folded) edges of a trigraph */
capsmi_status capsmi_trigraph_stats(const capsmi_trigraph* g, int64_t* nodes, int64_t* oriented_edges);
capsmi_status capsmi_trigraph_release(capsmi_trigraph* g);
capsmi_status capsmi_triangle_count(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                    const char* dst_col, const capsmi_bitmap* n_ok, int64_t* out_rows);
/* count(*) of the 2-hop chain (capsmi_two_hop_count) on one rank of an owner(target) partition:
 * this rank's tables hold every relationship into its owned ids [own_lo, own_hi) (relative to the
 * bitmaps' lo).  begin partitions them and writes the owned ids' in-degrees inA (relationships from
 * a_ok sources, b_ok applied) to owned_in (device, own_hi - own_lo uint32), stream-ordered; the
 * caller all-gathers the owned slices into one array of every id's inA, and finish sums inA(b) over
 * this rank's relationships b -> y with c_ok(y), less its a/b/c-ok self-loops, into *dev_out (device
 * int64, stream-ordered): the all-reduced sum of the ranks' parts is the count.  Σ_b inA(b)·outC(b)
 * (RelationalPlanner.scala:113-177 join rows, closed form in DESIGN.md §4) */
typedef struct capsmi_count_shard capsmi_count_shard;
capsmi_status capsmi_count_shard_begin(capsmi_session* s, int32_t nrels, capsmi_table* const* rels, const char* src_col,
                                       const char* dst_col, const capsmi_bitmap* a_ok, const capsmi_bitmap* b_ok,
                                       const capsmi_bitmap* c_ok, int64_t own_lo, int64_t own_hi, uint32_t* owned_in,
                                       capsmi_count_shard** out);
/* finish runs once per handle (a second call is ILLEGAL_ARGUMENT); the handle keeps what it reads of
 * the bitmaps, so they may be released after begin */
capsmi_status capsmi_count_shard_finish(capsmi_count_shard* h, const uint32_t* in_all, int64_t* dev_out);
capsmi_status capsmi_count_shard_release(capsmi_count_shard* h);
/* popcount of words [w_begin, w_end) of a device bitmap, result in *out (host) */
capsmi_status capsmi_words_popcount(capsmi_session* s, const uint32_t* words, int64_t w_begin, int64_t w_end,
                                    int64_t* out);
/* the same into a device int64 (*dev_out, overwritten), stream-ordered, no host synchronisation (the
 * count feeds a collective directly) */
capsmi_status capsmi_words_popcount_device(capsmi_session* s, const uint32_t* words, int64_t w_begin, int64_t w_end,
                                           int64_t* dev_out);

/* Cache analogue (Table.cache -> DataFrameTable.cache, SparkTable.scala:240-246): a copy of a
 * relationship table with rows clustered by `key_col` (dense ids in [id_lo, id_hi)).  Row multiset
 * unchanged; the fused kernels then touch bitmaps in id order. */
capsmi_status capsmi_cluster_by(capsmi_table* rels, const char* key_col, int64_t id_lo, int64_t id_hi,
                                capsmi_table** out);

/* ---- multi-GPU: one process per GPU over a distributed graph -------------------
 * Spark runs each Table operator over partitions and inserts a hash Exchange before joins and
 * aggregations (SparkTable.scala:133, 226; partitions set in CAPSSession.scala:115-131).  Here every
 * rank runs the same query (the same Table[T] calls) over its shard of a distributed graph; the fused
 * routes call the host's collective at their exchange points, so one rank's materialisation is one
 * rank's share of the job and the collective completes the answer on every rank.
 *
 * Ownership (hash partitioning): ids of the graph's domain [id_lo, id_hi) are scrambled by the
 * bijection h(x) = ((x - id_lo) * 0x9E3779B97F4A7C15) mod 2^k (2^k >= id_hi - id_lo, k >= 5) and rank
 * r owns the h-range [r * 32 * S, (r + 1) * 32 * S), S = ceil(2^k / (32 * world)) words -- balanced
 * whatever the id order (hubs at small ids included); the fused kernels run on h(x).
 *
 * The collective: enqueue one collective on the session's stream, ordered after the work queued on it
 * and before the work queued after the call returns (e.g. torch.distributed / RCCL on that stream).
 * ALL_GATHER: `count` elements from every rank into recv, rank-major (world x count);
 * ALL_REDUCE_SUM / _MAX: `count` elements, send and recv may be equal;
 * ALL_TO_ALL_V (Spark's Exchange hashpartitioning, SparkTable.scala:133, 226): `send` and `recv` point to
 * host capsmi_coll_vec descriptors and `count` is the world size; this rank sends send->counts[q]
 * elements, the q-th rank-major segment of send->data, to rank q and receives recv->counts[q] elements
 * from rank q into the q-th segment of recv->data (the library has exchanged the counts beforehand with
 * an ALL_GATHER, so both lists agree across ranks).  dtype CAPSMI_I64 (int64) or CAPSMI_COLL_U32
 * (uint32 words).  No call moves more than CAPSMI_COLL_CHUNK elements in all (environment, default
 * 2^26): the library cuts larger all-gathers, all-reduces and exchanges into several calls itself, so a
 * transport maps each call to one collective.  Return 0 on success. */
enum { CAPSMI_COLL_ALL_GATHER = 0, CAPSMI_COLL_ALL_REDUCE_SUM = 1, CAPSMI_COLL_ALL_REDUCE_MAX = 2,
       CAPSMI_COLL_ALL_TO_ALL_V = 3 };
enum { CAPSMI_COLL_U32 = 100 };
typedef struct {
    void* data;             /* device buffer, rank-major segments */
    const int64_t* counts;  /* host, world entries (elements per rank) */
} capsmi_coll_vec;
typedef int32_t (*capsmi_collective_fn)(void* ctx, int32_t op, const void* send, void* recv, int64_t count,
                                        int32_t dtype);
/* this process is rank `rank` of `world`; fn may be NULL only for world == 1 */
capsmi_status capsmi_session_set_ranks(capsmi_session* s, int32_t rank, int32_t world, capsmi_collective_fn fn,
                                       void* ctx);
enum { CAPSMI_NODES_REPLICATED = 0, CAPSMI_NODES_OWNED = 1 };
enum { CAPSMI_RELS_BY_SOURCE = 0, CAPSMI_RELS_BY_TARGET = 1 };
/* Registers this rank's entity tables (capsmi_node_table / capsmi_rel_table) as its shard of a graph
 * over the id domain [id_lo, id_hi) (the same on every rank, covering every id; hi - lo <= 2^30):
 * node tables hold every node row (REPLICATED) or the rows of the ids this rank owns (OWNED);
 * relationship tables hold the relationships whose target (BY_TARGET) or source (BY_SOURCE) this rank
 * owns.  Checked: ids inside the domain and the shard's rows owned (else ILLEGAL_ARGUMENT).  The
 * tables keep their scrambled key columns.  With BY_SOURCE, registration also exchanges (ALL_TO_ALL_V)
 * every relationship whose target another rank owns to that rank, which keeps it as its shard's
 * in-relationships (the var-length and undirected routes need them).  Routed on a distributed graph:
 * Expand projections (rows of this rank's relationships) and count(*) (one SUM all-reduce); either mode:
 * the 2-hop count(*), count(DISTINCT end) and count(DISTINCT start) (all-gathers of owned frontier slices
 * when the walk's relationships arrive by their end's owner, an ALL_TO_ALL_V + OR of frontier and end
 * bitmap slices when by their start's owner; the count(*) through an all-gather of owned degrees) and the
 * cyclic triangle count (sampled degrees all-reduced, every relationship packed into its oriented key and
 * exchanged to the rank of its source's degree-order range, sorted and deduplicated there, the ranges
 * all-gathered into a replicated oriented graph, each rank counting an interleaved share of the centers, one
 * all-reduce); with BY_SOURCE also the var-length grouped count (od and Y all-reduced
 * between its phases; the rows of each rank's owned start nodes), the undirected 1- / 2-hop counts (the
 * middles restricted to owned ids over the relationships incident to them, marks OR-reduced) and the 2-hop
 * grouped by its start (outC and the deduplicated hop-2 lists all-gathered; rows of the owned starts).
 * Any other plan runs operator by operator with the Exchanges Spark would insert (hash-partitioned joins
 * and groupings, gathers for global aggregates and ordering); capsmi_table_partitioned tells which results
 * hold this rank's rows only.  A session given a collective at world size 1 runs the same
 * distributed routes over its single shard (every exchange then goes through the collective). */
capsmi_status capsmi_graph_distribute(capsmi_session* s, int64_t id_lo, int64_t id_hi, int32_t nnodes,
                                      capsmi_table* const* nodes, int32_t node_mode, int32_t nrels,
                                      capsmi_table* const* rels, int32_t rel_mode);
/* the rows of `t` whose Long column `col` holds an id this rank owns in [id_lo, id_hi) (ingest: a
 * rank keeps its shard of a table every rank read); a new materialised table */
capsmi_status capsmi_owned_rows(capsmi_session* s, capsmi_table* t, const char* col, int64_t id_lo, int64_t id_hi,
                                capsmi_table** out);
/* the rank owning Long id `id` of the domain [id_lo, id_hi) among `world` ranks, and its scrambled
 * dense id (host computation, no device) */
capsmi_status capsmi_id_owner(int64_t id_lo, int64_t id_hi, int32_t world, int64_t id, int32_t* owner,
                              int64_t* dense_id);
/* 1 when t's rows are this rank's partition of a distributed result, else 0 (materialises t) */
capsmi_status capsmi_table_partitioned(const capsmi_table* t, int32_t* out);

/* ---- synthetic input -----------------------------------------------------
 * R-MAT relationship table [id, source, target] generated on the device, identical edge for edge
 * to oracle/rmat.c.  Keeps edges e in [e_begin, e_end) whose `part_col` (0 = source, 1 = target,
 * -1 = no filter) id falls in the word-aligned owner range of part `part` of `nparts`. */
capsmi_status capsmi_rmat_rels(capsmi_session* s, int32_t scale, int64_t e_begin, int64_t e_end,
                               int32_t pa, int32_t pb, int32_t pc, uint64_t seed, int32_t part_col,
                               int32_t part, int32_t nparts, capsmi_table** out);
/* word range [w_begin, w_end) of part `part` of `nparts` for ids in [0, 2^scale) */
capsmi_status capsmi_owner_words(int64_t nbits, int32_t part, int32_t nparts, int64_t* w_begin,
                                 int64_t* w_end);
/* ---- ingest ----------------------------------------------------
 * DataFrameReader.csv with an explicit schema, as EdgeListDataSource (EdgeListDataSource.scala:76-97)
 * and the FS graph source read their tables: files in order, no header, `delimiter` one character
 * (as Spark's `sep`: "1  2" with ' ' is 1, null, 2; 0 = opt-in whitespace splitting, runs of blanks
 * separate fields), '"' quotes, an empty unquoted field is null, lines whose first character is
 * `comment` (0 = none) and lines of blanks skipped; Spark's PERMISSIVE token counts (missing trailing fields null, extra tokens dropped);
 * a token that does not parse as its column type is ILLEGAL_ARGUMENT.  Parsed by host threads
 * (CAPSMI_INGEST_THREADS, default OMP_NUM_THREADS), copied to the device.  types: CAPSMI_I64 /
 * F64 / BOOL / STR; STR fields go through `intern` (the caller's dictionary), in row order.
 * row_id_col != NULL prepends a Long column of monotonically_increasing_id values
 * (EdgeListDataSource.scala:86): by default those of one partition (the row numbers); see
 * capsmi_session_set_csv_partitioning for Spark's multi-partition ids. */
typedef int64_t (*capsmi_intern_fn)(void* ctx, const char* s, size_t len);
/* Row ids of capsmi_read_csv as monotonically_increasing_id over the partitions of Spark 2.2.1's file scan
 * (FileSourceScanExec.createNonBucketedReadRDD; third-party, restated in csrc/ingest.hip spark_row_ids):
 * maxSplitBytes = min(max_partition_bytes, max(open_cost_bytes, total / default_parallelism)), total =
 * sum of (file length + open_cost_bytes); files split every maxSplitBytes; splits sorted by length
 * (descending, stable) and packed next-fit into partitions; a line belongs to the split holding the byte
 * before its first byte (Hadoop's LineRecordReader); id = partition << 33 | row within the partition.
 * default_parallelism = the session's core count (CAPSSession.local(): local[*]); 0 restores one partition.
 * Spark's defaults: max_partition_bytes 128 MiB (spark.sql.files.maxPartitionBytes), open_cost_bytes 4 MiB
 * (spark.sql.files.openCostInBytes). */
capsmi_status capsmi_session_set_csv_partitioning(capsmi_session* s, int64_t default_parallelism,
                                                  int64_t max_partition_bytes, int64_t open_cost_bytes);
capsmi_status capsmi_read_csv(capsmi_session* s, int32_t nfiles, const char* const* paths, char delimiter, char comment,
                              int32_t ncols, const char* const* names, const int32_t* types, capsmi_intern_fn intern,
                              void* intern_ctx, const char* row_id_col, capsmi_table** out);

/* R-MAT node table(s): kind 0 -> one table [id] with every id 0..2^scale-1 (all Person);
 * kind 1 -> Person ids (splitmix64(id) & 3 != 0) with [id, age], age = splitmix64(seed ^ id) % 100;
 * kind 2 -> Company ids (the complement) with [id] */
capsmi_status capsmi_rmat_nodes(capsmi_session* s, int32_t scale, int32_t kind, uint64_t seed,
                                capsmi_table** out);
/* order-insensitive row fingerprint over `ncols` I64 columns (SURVEY.md §8d parity check):
 * count, sum and xor of h(row), h = fold splitmix64(h ^ v) from 0x243F6A8885A308D3 */
capsmi_status capsmi_table_fingerprint(capsmi_table* t, int32_t ncols, const char* const* cols,
                                       int64_t* count, uint64_t* sum, uint64_t* xr);

#ifdef __cplusplus
}
#endif
#endif /* CAPSMI_H */
