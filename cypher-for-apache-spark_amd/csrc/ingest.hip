// ingest.hip -- native CSV ingest to device tables (host code).
//
// Restates DataFrameReader.csv with an explicit schema as the reference's sources use it:
//   EdgeListDataSource.graph (spark-cypher/.../api/io/edgelist/EdgeListDataSource.scala:76-97): two
//     Long columns, reader options (delimiter, comment), `monotonically_increasing_id` row ids;
//   FSGraphSource CSV tables (spark-cypher/.../api/io/fs/FSGraphSource.scala, schema from
//     propertyGraphSchema.json): no header, ',' separated, '"' quoted, an empty field is null.
// Files are read whole, split at line boundaries (records never span lines: Spark's default
// multiLine = false) and parsed by one host thread per chunk; each thread's columns are copied to
// their place in the device table.  String fields are handed, in row order, to the caller's
// order-preserving dictionary (include/capsmi.h capsmi_intern_fn).
#include <algorithm>
#include <charconv>
#include <cstdio>
#include <atomic>
#include <cstring>
#include <strings.h>
#include <thread>

#include "capsmi_impl.h"

namespace capsmi {
namespace {

struct Chunk {
    const char* b = nullptr;
    const char* e = nullptr;
    int64_t rows = 0;
    std::vector<std::vector<int64_t>> data;
    std::vector<std::vector<uint8_t>> valid;
    std::vector<std::string> arena;                        // STR columns: the field texts back to back
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sref;  // per non-null STR field: (arena offset, length)
    std::vector<int64_t> lstart;  // byte offset in its file of each row's line (Spark partition ids only)
    std::string err;
};

int n_threads() {
    if (const char* e = getenv("CAPSMI_INGEST_THREADS")) return std::max(1, atoi(e));
    if (const char* e = getenv("OMP_NUM_THREADS")) return std::max(1, atoi(e));
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
}

inline bool blank(char c) { return c == ' ' || c == '\t'; }

// One field at p (line end le).  Quoted fields drop their quotes; "" and \" inside them are one
// quote (copied to `tmp`).  With collapse (delimiter 0, an opt-in), runs of blanks separate fields.
// On return p is past the field and its delimiter, `more` tells whether another field follows;
// false on a malformed (unterminated / trailing-garbage) quoted field.
bool next_field(const char*& p, const char* le, char delim, bool collapse, const char*& fb, const char*& fe,
                std::string& tmp, bool& quoted, bool& more) {
    quoted = false;
    if (p < le && *p == '"') {
        quoted = true;
        ++p;
        tmp.clear();
        bool esc = false;
        const char* s = p;
        while (p < le) {
            if ((*p == '\\' || *p == '"') && p + 1 < le && p[1] == '"') {
                tmp.append(s, p);
                tmp.push_back('"');
                p += 2;
                s = p;
                esc = true;
                continue;
            }
            if (*p == '"') break;
            ++p;
        }
        if (p >= le) return false;  // unterminated quote
        if (esc) {
            tmp.append(s, p);
            fb = tmp.data();
            fe = fb + tmp.size();
        } else {
            fb = s;
            fe = p;
        }
        ++p;
        if (collapse) {
            while (p < le && blank(*p)) ++p;
            more = p < le;
            return true;
        }
        more = p < le;
        if (more) {
            if (*p != delim) return false;
            ++p;
        }
        return true;
    }
    fb = p;
    if (collapse) {
        while (p < le && !blank(*p)) ++p;
        fe = p;
        while (p < le && blank(*p)) ++p;
        more = p < le;
    } else {
        while (p < le && *p != delim) ++p;
        fe = p;
        more = p < le;
        if (more) ++p;
    }
    return true;
}

// Records follow Spark's PERMISSIVE mode for token counts: missing trailing fields are null, extra
// tokens are dropped.  A token that does not parse as its column's type is an error (reported with
// its byte offset) rather than a silent null.
void parse_chunk(Chunk& c, const char* file_base, const std::string& fname, char delim, char comment,
                 const std::vector<int32_t>& types, bool want_pos) {
    const int nc = (int)types.size();
    const bool collapse = delim == 0;  // whitespace-separated (opt-in; Spark's sep is one character)
    c.data.assign(nc, {});
    c.valid.assign(nc, {});
    c.arena.assign(nc, {});
    c.sref.assign(nc, {});
    std::string tmp;
    const char* p = c.b;
    auto fail = [&](const char* at, const std::string& what) {
        c.err = fname + ": " + what + " (record at byte " + std::to_string(at - file_base) + ")";
    };
    while (p < c.e) {
        const char* le = (const char*)memchr(p, '\n', (size_t)(c.e - p));
        if (!le) le = c.e;
        const char* next = le + 1;
        const char* lend = le;
        if (lend > p && lend[-1] == '\r') --lend;
        const char* q = p;
        while (q < lend && blank(*q)) ++q;
        // a comment line starts with the comment character itself (univocity's comment test, which
        // Spark's CSV reader uses); a line of blanks holds no record
        if (q == lend || (comment && *p == comment)) {
            p = next;
            continue;
        }
        const char* fp = collapse ? q : p;
        bool more = true;
        for (int k = 0; k < nc; ++k) {
            const char *fb = nullptr, *fe = nullptr;
            bool quoted = false;
            if (!more) {
                fb = fe = lend;  // missing field -> null
            } else if (!next_field(fp, lend, delim, collapse, fb, fe, tmp, quoted, more)) {
                fail(p, "malformed quoted field");
                return;
            }
            const bool null = fe == fb && !quoted;
            int64_t w = 0;
            if (!null) {
                switch (types[k]) {
                    case CAPSMI_I64: {
                        const char* s = fb < fe && *fb == '+' ? fb + 1 : fb;
                        auto r = std::from_chars(s, fe, w);
                        if (r.ec != std::errc() || r.ptr != fe) {
                            fail(p, "not a Long: '" + std::string(fb, fe) + "'");
                            return;
                        }
                        break;
                    }
                    case CAPSMI_F64: {
                        double d = 0;
                        auto r = std::from_chars(fb, fe, d);
                        if (r.ec != std::errc() || r.ptr != fe) {
                            fail(p, "not a Double: '" + std::string(fb, fe) + "'");
                            return;
                        }
                        std::memcpy(&w, &d, 8);
                        break;
                    }
                    case CAPSMI_BOOL: {  // Spark's CSV BooleanType: "true" / "false", any case, nothing else
                        const size_t len = (size_t)(fe - fb);
                        if (len == 4 && strncasecmp(fb, "true", 4) == 0) w = 1;
                        else if (len == 5 && strncasecmp(fb, "false", 5) == 0) w = 0;
                        else {
                            fail(p, "not a Boolean: '" + std::string(fb, fe) + "'");
                            return;
                        }
                        break;
                    }
                    default:
                        c.sref[k].push_back({(uint64_t)c.arena[k].size(), (uint32_t)(fe - fb)});
                        c.arena[k].append(fb, fe);
                        break;
                }
            }
            c.data[k].push_back(w);
            c.valid[k].push_back(null ? 0 : 1);
        }
        if (want_pos) c.lstart.push_back((int64_t)(p - file_base));
        ++c.rows;
        p = next;
    }
}

// monotonically_increasing_id over the partitions of Spark 2.2.1's file scan (EdgeListDataSource.scala:86;
// FileSourceScanExec.createNonBucketedReadRDD, third-party, restated): maxSplitBytes = min(maxPartitionBytes,
// max(openCostInBytes, totalBytes / defaultParallelism)), totalBytes = sum of (length + openCostInBytes); each
// file is split every maxSplitBytes; the splits are sorted by length, descending and stable, and packed
// "next fit" into partitions (a split that would take the partition past maxSplitBytes closes it first; each
// split adds its length + openCostInBytes).  A split [o, o + len) reads the lines whose first byte lies in
// (o, o + len], and the file's first line (Hadoop's LineRecordReader skips a split's first, partial line and
// reads one line past its end).  Partition p's rows are numbered through its splits in order:
// id = p << 33 | row.  Rows (parsed records) come in file / line order; each gets its id.
void spark_row_ids(const std::vector<int64_t>& lens, const std::vector<Chunk>& chunks,
                   const std::vector<size_t>& chunk_file, int64_t par, int64_t max_part, int64_t open_cost,
                   std::vector<int64_t>& ids) {
    int64_t total = 0;
    for (int64_t L : lens) total += L + open_cost;
    const int64_t per_core = total / par;
    const int64_t split = std::max<int64_t>(1, std::min(max_part, std::max(open_cost, per_core)));
    struct Split {
        size_t f;
        int64_t k, len, part = 0, base = 0, rows = 0;
    };
    std::vector<Split> sp;
    std::vector<size_t> first(lens.size());  // index of file f's first split
    for (size_t f = 0; f < lens.size(); ++f) {
        first[f] = sp.size();
        for (int64_t o = 0, k = 0; o < lens[f]; o += split, ++k) sp.push_back({f, k, std::min(split, lens[f] - o)});
    }
    auto split_of = [&](size_t f, int64_t b) -> size_t {  // the split reading the line that starts at byte b
        const int64_t k = b == 0 ? 0 : (b - 1) / split;
        return first[f] + (size_t)k;
    };
    for (size_t ci = 0; ci < chunks.size(); ++ci)
        for (int64_t b : chunks[ci].lstart) sp[split_of(chunk_file[ci], b)].rows += 1;
    std::vector<size_t> order(sp.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return sp[a].len > sp[b].len; });
    int64_t part = 0, cur = 0, base = 0;
    bool open = false;
    for (size_t i : order) {
        if (open && cur + sp[i].len > split) {  // closePartition()
            ++part;
            cur = 0;
            base = 0;
        }
        sp[i].part = part;
        sp[i].base = base;
        base += sp[i].rows;
        cur += sp[i].len + open_cost;
        open = true;
    }
    std::vector<int64_t> seen(sp.size(), 0);
    for (size_t ci = 0; ci < chunks.size(); ++ci)
        for (int64_t b : chunks[ci].lstart) {
            Split& x = sp[split_of(chunk_file[ci], b)];
            ids.push_back((x.part << 33) | (x.base + seen[&x - sp.data()]++));
        }
}

std::string read_file(const char* path) {
    FILE* f = fopen(path, "rb");
    REQUIRE(f, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("cannot open ") + path);
    std::string s;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    s.resize(n > 0 ? (size_t)n : 0);
    const size_t got = n > 0 ? fread(&s[0], 1, (size_t)n, f) : 0;
    fclose(f);
    REQUIRE(got == s.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("short read of ") + path);
    return s;
}

}  // namespace

capsmi_table* read_csv(capsmi_session* s, const std::vector<std::string>& paths, char delim, char comment,
                       const std::vector<std::string>& names, const std::vector<int32_t>& types, capsmi_intern_fn intern,
                       void* ctx, const char* row_id_col) {
    const int nc = (int)types.size();
    const int nt = n_threads();
    std::vector<std::string> texts;
    std::vector<Chunk> chunks;
    std::vector<size_t> chunk_file;
    texts.reserve(paths.size());
    for (size_t f = 0; f < paths.size(); ++f) {
        texts.push_back(read_file(paths[f].c_str()));
        const std::string& t = texts.back();
        const char* b = t.data();
        const char* e = b + t.size();
        const size_t per = std::max<size_t>(1 << 16, t.size() / (size_t)nt + 1);
        while (b < e) {  // chunks end after a newline
            const char* ce = std::min(e, b + per);
            if (ce < e) {
                const char* nl = (const char*)memchr(ce, '\n', (size_t)(e - ce));
                ce = nl ? nl + 1 : e;
            }
            Chunk c;
            c.b = b;
            c.e = ce;
            chunks.push_back(std::move(c));
            chunk_file.push_back(f);
            b = ce;
        }
    }
    {
        std::vector<std::thread> th;
        std::atomic<size_t> next{0};
        for (int i = 0; i < std::min<int>(nt, (int)chunks.size()); ++i)
            th.emplace_back([&] {
                for (size_t k; (k = next.fetch_add(1)) < chunks.size();)
                    parse_chunk(chunks[k], texts[chunk_file[k]].data(), paths[chunk_file[k]], delim, comment, types,
                                row_id_col != nullptr && s->csv_parallelism > 0);
            });
        for (auto& x : th) x.join();
    }
    int64_t rows = 0;
    for (auto& c : chunks) {
        REQUIRE(c.err.empty(), CAPSMI_ERR_ILLEGAL_ARGUMENT, c.err);
        rows += c.rows;
    }
    // strings through the caller's dictionary, in row order
    for (int k = 0; k < nc; ++k) {
        if (types[k] != CAPSMI_STR) continue;
        REQUIRE(intern != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, "String column without a dictionary (intern)");
        for (auto& c : chunks) {
            size_t si = 0;
            for (int64_t r = 0; r < c.rows; ++r)
                if (c.valid[k][r]) {
                    const auto& ref = c.sref[k][si++];
                    c.data[k][r] = intern(ctx, c.arena[k].data() + ref.first, ref.second);
                }
        }
    }
    auto* t = new capsmi_table();
    std::unique_ptr<capsmi_table> g(t);
    t->sess = s;
    t->nrows = rows;
    hipStream_t st = s->stream;
    if (row_id_col) {  // monotonically_increasing_id: one partition (the row number) or Spark's file splits
        Column c;
        c.name = row_id_col;
        c.type = CAPSMI_I64;
        c.data = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), s);
        if (s->csv_parallelism > 0) {
            std::vector<int64_t> lens;
            for (auto& x : texts) lens.push_back((int64_t)x.size());
            std::vector<int64_t> ids;
            ids.reserve(rows);
            spark_row_ids(lens, chunks, chunk_file, s->csv_parallelism, s->csv_max_partition_bytes, s->csv_open_cost,
                          ids);
            if (rows)
                HIP_CHECK(hipMemcpyAsync(P<int64_t>(c.data), ids.data(), sizeof(int64_t) * rows, hipMemcpyHostToDevice,
                                         st));
            HIP_CHECK(hipStreamSynchronize(st));
        } else {
            iota_i64(P<int64_t>(c.data), 0, rows, st);
        }
        t->cols.push_back(std::move(c));
    }
    for (int k = 0; k < nc; ++k) {
        Column c;
        c.name = names[k];
        c.type = types[k];
        c.data = dev_alloc(sizeof(int64_t) * (rows > 0 ? rows : 1), s);
        bool any_null = false;
        for (auto& ch : chunks)
            for (uint8_t v : ch.valid[k]) if (!v) { any_null = true; break; }
        if (any_null) c.valid = dev_alloc(rows > 0 ? rows : 1, s);
        int64_t off = 0;
        for (auto& ch : chunks) {
            if (ch.rows) {
                HIP_CHECK(hipMemcpyAsync(P<int64_t>(c.data) + off, ch.data[k].data(), sizeof(int64_t) * ch.rows,
                                         hipMemcpyHostToDevice, st));
                if (any_null)
                    HIP_CHECK(hipMemcpyAsync(P<uint8_t>(c.valid) + off, ch.valid[k].data(), ch.rows, hipMemcpyHostToDevice,
                                             st));
            }
            off += ch.rows;
        }
        t->cols.push_back(std::move(c));
    }
    HIP_CHECK(hipStreamSynchronize(st));  // host chunks go away
    return g.release();
}

}  // namespace capsmi
