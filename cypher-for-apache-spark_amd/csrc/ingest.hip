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
#include "csv_parse.h"

namespace capsmi {
namespace {

int n_threads(const capsmi_session* s) {
    if (s->cfg.ingest_threads > 0) return s->cfg.ingest_threads;
    if (const char* e = getenv("OMP_NUM_THREADS")) return std::max(1, atoi(e));
    return (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
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
    const int nt = n_threads(s);
    std::vector<std::string> texts;
    std::vector<csv::Chunk> chunks;
    std::vector<size_t> chunk_file;
    texts.reserve(paths.size());
    for (size_t f = 0; f < paths.size(); ++f) texts.push_back(read_file(paths[f].c_str()));
    csv::split_chunks(texts, nt, chunks, chunk_file);
    csv::parse_chunks(chunks, chunk_file, texts, paths, delim, comment, types,
                      row_id_col != nullptr && s->csv_parallelism > 0, nt);
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
            csv::spark_row_ids(lens, chunks, chunk_file, s->csv_parallelism, s->csv_max_partition_bytes, s->csv_open_cost,
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
