// csv_parse.h -- the host-only half of the CSV reader (ingest.hip): chunking at line boundaries, the
// threaded field parser and Spark's file-scan row ids.  No HIP here, so the same code is built with
// AddressSanitizer / UndefinedBehaviorSanitizer / ThreadSanitizer by tests/sanitize.
#pragma once
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cstdint>
#include <cstring>
#include <string>
#include <strings.h>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/capsmi.h"

namespace capsmi {
namespace csv {

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

inline bool blank(char c) { return c == ' ' || c == '\t'; }

// One field at p (line end le).  Quoted fields drop their quotes; "" and \" inside them are one
// quote (copied to `tmp`).  With collapse (delimiter 0, an opt-in), runs of blanks separate fields.
// On return p is past the field and its delimiter, `more` tells whether another field follows;
// false on a malformed (unterminated / trailing-garbage) quoted field.
inline bool next_field(const char*& p, const char* le, char delim, bool collapse, const char*& fb, const char*& fe,
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
inline void parse_chunk(Chunk& c, const char* file_base, const std::string& fname, char delim, char comment,
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
inline void spark_row_ids(const std::vector<int64_t>& lens, const std::vector<Chunk>& chunks,
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

// files split into chunks that end after a newline (about one per thread, at least 64 KiB)
inline void split_chunks(const std::vector<std::string>& texts, int nt, std::vector<Chunk>& chunks,
                         std::vector<size_t>& chunk_file) {
    for (size_t f = 0; f < texts.size(); ++f) {
        const std::string& t = texts[f];
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
}

// every chunk parsed by `nt` threads taking chunks from a shared counter
inline void parse_chunks(std::vector<Chunk>& chunks, const std::vector<size_t>& chunk_file,
                         const std::vector<std::string>& texts, const std::vector<std::string>& names, char delim,
                         char comment, const std::vector<int32_t>& types, bool want_pos, int nt) {
    std::vector<std::thread> th;
    std::atomic<size_t> next{0};
    for (int i = 0; i < std::min<int>(nt, (int)chunks.size()); ++i)
        th.emplace_back([&] {
            for (size_t k; (k = next.fetch_add(1)) < chunks.size();)
                parse_chunk(chunks[k], texts[chunk_file[k]].data(), names[chunk_file[k]], delim, comment, types,
                            want_pos);
        });
    for (auto& x : th) x.join();
}

}  // namespace csv
}  // namespace capsmi
