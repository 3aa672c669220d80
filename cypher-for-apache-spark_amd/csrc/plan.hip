// plan.hip -- lazy Table[T] plans, materialisation and the fused-path recogniser.
//
// CAPS's backend sees a MATCH only as the Table[T] calls RelationalPlanner emits
// (okapi-relational/.../planning/RelationalPlanner.scala:113-177): an Expand is
//   join(nodeScan, relScan, (src.id, r.source)) then join(.., nodeScan, (r.target, dst.id)),
// an ExpandInto a 2-key join, a BoundedVarLengthExpand a union of unrolled join chains with
// isomorphism filters (VarLengthExpandPlanner.scala:46-310), followed by Filter (uniqueness
// NOT(r_i = r_j), node predicates) and Aggregate (RelationalOperator.scala:293-351).  DataFrameTable
// builds a lazy Spark plan from those calls and runs it at the first action (SparkTable.scala:59).
// libcapsmi does the same: every Table operator returns a lazy table (schema known, rows not yet
// computed); materialisation first matches the plan against the shapes the fused kernels compute
//   Expand + node filters, projected ........................ capsmi_expand_filter     ("expand")
//   Expand + node filters, count(*) ......................... expand count              ("expand_count")
//   2 x Expand + uniqueness, count(*) / count(DISTINCT end) . two-hop kernels           ("two_hop")
//   2 x Expand + ExpandInto closing a cycle, count(*) ....... triangle count            ("triangle")
//   var-length 0 <= l <= u <= 4, grouped count(*) by start .. var-length count          ("var_length")
// over registered entity tables (capsmi_node_table / capsmi_rel_table), and otherwise runs the
// operators one by one (api.hip eager_*).  Node predicates become node-scan bitmaps; ids must be
// unique per scan and inside one window of at most 2^30 ids, else the plan runs unfused.
#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <set>

#include "capsmi_impl.h"

namespace capsmi {

void set_last_error(const std::string& m);
std::string last_error_string();

struct AggSpec {
    int32_t kind = 0, distinct = 0;
    std::string input, output;
};

struct PlanNode {
    enum Kind { SELECT, DROP, RENAME, FILTER, WITH_COLUMNS, JOIN, UNION, DISTINCT, DISTINCT_ON, GROUP, ORDER, SKIP, LIMIT };
    Kind kind = SELECT;
    std::vector<capsmi_table*> in;            // retained inputs
    std::vector<std::string> a, b;            // column names (see builders)
    std::vector<std::vector<capsmi_expr>> progs;
    std::vector<int32_t> flags;               // ORDER: descending
    std::vector<AggSpec> aggs;
    int32_t jt = 0;
    int64_t n = 0;
    ~PlanNode() {
        for (capsmi_table* t : in) capsmi_table_release(t);
    }
};

namespace {

#define P_BEGIN try {
#define P_END                                                   \
    }                                                           \
    catch (const capsmi::Error& e) {                            \
        set_last_error(e.what());                               \
        return e.code;                                          \
    }                                                           \
    catch (const std::bad_alloc&) {                             \
        set_last_error("host allocation failed");               \
        return CAPSMI_ERR_OUT_OF_MEMORY;                        \
    }                                                           \
    catch (const std::exception& e) {                           \
        set_last_error(e.what());                               \
        return CAPSMI_ERR_INTERNAL;                             \
    }                                                           \
    return CAPSMI_OK;

void need(const void* p, const char* what) {
    REQUIRE(p != nullptr, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("null argument: ") + what);
}

void check(capsmi_status st) {
    if (st != CAPSMI_OK) throw Error(st, last_error_string());
}

int find_col(const capsmi_table* t, const std::string& name) {
    for (size_t i = 0; i < t->cols.size(); ++i)
        if (t->cols[i].name == name) return (int)i;
    return -1;
}

int col_of(const capsmi_table* t, const char* name) {
    need(name, "column name");
    const int i = find_col(t, name);
    REQUIRE(i >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("no column named '") + name + "'");
    return i;
}

Column schema_col(const std::string& name, int32_t type, bool nullable) {
    Column c;
    c.name = name;
    c.type = type;
    c.lazy_nullable = nullable;
    return c;
}

Column schema_of(const Column& c) { return schema_col(c.name, c.type, c.nullable()); }

// an input of a plan node: retained here, released by ~PlanNode (also when the builder throws)
void hold(PlanNode& p, capsmi_table* t) {
    t->refs.fetch_add(1);
    p.in.push_back(t);
}

// a lazy table over node `p` (inputs already held)
capsmi_table* lazy_table(capsmi_session* s, std::shared_ptr<PlanNode> p, std::vector<Column> schema) {
    auto* t = new capsmi_table();
    t->sess = s;
    t->nrows = -1;
    t->cols = std::move(schema);
    t->plan = std::move(p);
    return t;
}

std::vector<const char*> cstrs(const std::vector<std::string>& v) {
    std::vector<const char*> o;
    for (auto& x : v) o.push_back(x.c_str());
    return o;
}

int arity(const capsmi_expr& x) {
    switch (x.op) {
        case CAPSMI_X_COL: case CAPSMI_X_LIT: case CAPSMI_X_NULL: return 0;
        case CAPSMI_X_NOT: case CAPSMI_X_ISNULL: case CAPSMI_X_ISNOTNULL: case CAPSMI_X_NEG: return 1;
        case CAPSMI_X_AND: case CAPSMI_X_OR: case CAPSMI_X_COALESCE: return x.arg;
        case CAPSMI_X_IN: return x.arg + 1;
        case CAPSMI_X_CASE: return 2 * x.arg + 1;
        default: return 2;
    }
}

// ============================ operator-by-operator execution ===============================
capsmi_table* exec_node(const PlanNode& p) {
    capsmi_table* r = nullptr;
    capsmi_table* x = p.in.empty() ? nullptr : p.in[0];
    switch (p.kind) {
        case PlanNode::SELECT: { auto c = cstrs(p.a); check(eager_select(x, (int)c.size(), c.data(), &r)); break; }
        case PlanNode::DROP: { auto c = cstrs(p.a); check(eager_drop(x, (int)c.size(), c.data(), &r)); break; }
        case PlanNode::RENAME: check(eager_with_column_renamed(x, p.a[0].c_str(), p.b[0].c_str(), &r)); break;
        case PlanNode::FILTER: check(eager_filter(x, (int)p.progs[0].size(), p.progs[0].data(), &r)); break;
        case PlanNode::WITH_COLUMNS: {
            std::vector<capsmi_expr_column> cols(p.a.size());
            for (size_t i = 0; i < p.a.size(); ++i) {
                cols[i].name = p.a[i].c_str();
                cols[i].nnodes = (int32_t)p.progs[i].size();
                cols[i].prog = p.progs[i].data();
            }
            check(eager_with_columns(x, (int)cols.size(), cols.data(), &r));
            break;
        }
        case PlanNode::JOIN: {
            auto l = cstrs(p.a), rr = cstrs(p.b);
            check(eager_join(x, p.in[1], p.jt, (int)l.size(), l.data(), rr.data(), &r));
            break;
        }
        case PlanNode::UNION: check(eager_union_all(x, p.in[1], &r)); break;
        case PlanNode::DISTINCT: check(eager_distinct(x, &r)); break;
        case PlanNode::DISTINCT_ON: { auto c = cstrs(p.a); check(eager_distinct_on(x, (int)c.size(), c.data(), &r)); break; }
        case PlanNode::GROUP: {
            auto by = cstrs(p.a);
            std::vector<capsmi_agg> ag(p.aggs.size());
            for (size_t i = 0; i < p.aggs.size(); ++i) {
                ag[i].kind = p.aggs[i].kind;
                ag[i].distinct = p.aggs[i].distinct;
                ag[i].input = p.aggs[i].input.empty() ? nullptr : p.aggs[i].input.c_str();
                ag[i].output = p.aggs[i].output.c_str();
            }
            check(eager_group(x, (int)by.size(), by.data(), (int)ag.size(), ag.data(), &r));
            break;
        }
        case PlanNode::ORDER: { auto c = cstrs(p.a); check(eager_order_by(x, (int)c.size(), c.data(), p.flags.data(), &r)); break; }
        case PlanNode::SKIP: check(eager_skip(x, p.n, &r)); break;
        case PlanNode::LIMIT: check(eager_limit(x, p.n, &r)); break;
    }
    return r;
}

// move a materialised result into the lazy table `t` (names from t's schema)
void adopt(capsmi_table* t, capsmi_table* r) {
    std::unique_ptr<capsmi_table> g(r);
    REQUIRE(r->cols.size() == t->cols.size(), CAPSMI_ERR_INTERNAL, "materialised schema differs from the plan's");
    for (size_t i = 0; i < r->cols.size(); ++i) r->cols[i].name = t->cols[i].name;
    t->cols = std::move(r->cols);
    t->nrows = r->nrows;
}

// ================================ the recogniser ===========================================
enum { ROLE_NONE = 0, ROLE_ID = 1, ROLE_SRC = 2, ROLE_DST = 3 };

// A scan: union of registered entity tables, each column a base column or a per-table constant
// (ScanGraph.scanOperator's aligned entity tables, ScanGraph.scala:61-96).
struct Member {
    capsmi_table* base = nullptr;
    std::vector<int> src;            // per scan column: base column, or -1 (constant)
    std::vector<capsmi_expr> cst;    // the constant as a one-node program (LIT / NULL)
};
struct Scan {
    int kind = 0;  // 1 node, 2 relationship
    std::vector<Member> m;
    std::vector<int> role;  // per scan column: ROLE_* in every member, else ROLE_NONE
    // relationship scan filtered to start <> end: the incoming branch of an undirected Expand
    // (RelationalPlanner.scala:130-131)
    bool no_loops = false;
};

void scan_roles(Scan& sc, size_t ncols) {
    sc.role.assign(ncols, ROLE_NONE);
    for (size_t k = 0; k < ncols; ++k) {
        for (int r : {ROLE_ID, ROLE_SRC, ROLE_DST}) {
            bool all = !sc.m.empty();
            for (const Member& m : sc.m) {
                const EntityInfo& e = *m.base->entity;
                const int want = r == ROLE_ID ? e.id : (r == ROLE_SRC ? e.src : e.dst);
                if (want < 0 || m.src[k] != want) { all = false; break; }
            }
            if (all) { sc.role[k] = r; break; }
        }
    }
}

bool as_scan(const capsmi_table* t, Scan& sc) {
    if (!t->lazy()) {
        if (!t->entity) return false;
        sc = Scan();
        sc.kind = t->entity->kind;
        Member m;
        m.base = const_cast<capsmi_table*>(t);
        for (size_t k = 0; k < t->cols.size(); ++k) m.src.push_back((int)k);
        m.cst.resize(t->cols.size());
        sc.m.push_back(std::move(m));
        scan_roles(sc, t->cols.size());
        return true;
    }
    const PlanNode& p = *t->plan;
    const capsmi_table* in = p.in.empty() ? nullptr : p.in[0];
    switch (p.kind) {
        case PlanNode::WITH_COLUMNS: {
            if (!as_scan(in, sc)) return false;
            std::vector<std::string> names;
            for (auto& c : in->cols) names.push_back(c.name);
            const std::vector<Member> before = sc.m;  // expressions read the input columns
            for (size_t i = 0; i < p.a.size(); ++i) {
                if (p.progs[i].size() != 1) return false;
                const capsmi_expr& x = p.progs[i][0];
                if (x.op != CAPSMI_X_COL && x.op != CAPSMI_X_LIT && x.op != CAPSMI_X_NULL) return false;
                int j = -1;
                for (size_t q = 0; q < names.size(); ++q) if (names[q] == p.a[i]) j = (int)q;
                if (j < 0) {
                    j = (int)names.size();
                    names.push_back(p.a[i]);
                    for (Member& m : sc.m) { m.src.push_back(-1); m.cst.push_back(capsmi_expr{}); }
                }
                for (size_t q = 0; q < sc.m.size(); ++q) {
                    Member& m = sc.m[q];
                    if (x.op == CAPSMI_X_COL) {
                        m.src[j] = before[q].src[x.arg];
                        m.cst[j] = before[q].cst[x.arg];
                    } else {
                        m.src[j] = -1;
                        m.cst[j] = x;
                    }
                }
            }
            break;
        }
        case PlanNode::SELECT:
        case PlanNode::DROP:
        case PlanNode::RENAME: {
            if (!as_scan(in, sc)) return false;
            std::vector<int> pick;
            if (p.kind == PlanNode::SELECT) {
                for (auto& nm : p.a) pick.push_back(find_col(in, nm));
            } else if (p.kind == PlanNode::DROP) {
                std::set<std::string> d(p.a.begin(), p.a.end());
                for (size_t k = 0; k < in->cols.size(); ++k) if (!d.count(in->cols[k].name)) pick.push_back((int)k);
            } else {
                for (size_t k = 0; k < in->cols.size(); ++k) pick.push_back((int)k);
            }
            for (Member& m : sc.m) {
                Member o;
                o.base = m.base;
                for (int k : pick) { o.src.push_back(m.src[k]); o.cst.push_back(m.cst[k]); }
                m = std::move(o);
            }
            break;
        }
        case PlanNode::UNION: {
            Scan r;
            if (!as_scan(in, sc) || !as_scan(p.in[1], r) || sc.kind != r.kind || sc.no_loops || r.no_loops) return false;
            for (Member& m : r.m) sc.m.push_back(std::move(m));
            break;
        }
        case PlanNode::FILTER: {  // only NOT(start = end) / start <> end over a relationship scan
            if (!as_scan(in, sc) || sc.kind != 2 || sc.no_loops) return false;
            const auto& pr = p.progs[0];
            const bool neq = pr.size() == 3 && pr[2].op == CAPSMI_X_NEQ;
            const bool negated_eq = pr.size() == 4 && pr[2].op == CAPSMI_X_EQ && pr[3].op == CAPSMI_X_NOT;
            if (!(neq || negated_eq) || pr[0].op != CAPSMI_X_COL || pr[1].op != CAPSMI_X_COL) return false;
            const int r0 = sc.role[pr[0].arg], r1 = sc.role[pr[1].arg];
            if (!((r0 == ROLE_SRC && r1 == ROLE_DST) || (r0 == ROLE_DST && r1 == ROLE_SRC))) return false;
            sc.no_loops = true;
            return true;  // same columns, same roles
        }
        default: return false;
    }
    scan_roles(sc, t->cols.size());
    return true;
}

enum RK : int8_t { RK_EXPR, RK_CONST, RK_NODE, RK_REL };
struct Role {
    RK k = RK_EXPR;
    int inst = -1, scol = -1;
    capsmi_expr cst{};
};

struct ENode {
    capsmi_expr x{};
    Role role;  // CAPSMI_X_COL leaves
    std::vector<ENode> kids;
};

struct Hop {
    int rel = -1;          // instance of the relationship scan
    int from = -1, to = -1;  // positions
    int from_role = ROLE_SRC, to_role = ROLE_DST;
};

// A join chain over scans: positions (pattern nodes) joined by hops (relationships)
struct Path {
    std::vector<Scan> inst;
    std::vector<int> pos_node;  // per position: node-scan instance, or -1
    std::vector<Hop> hops;
    std::vector<Role> cols;     // per output column
    std::vector<ENode> conj;    // filter conjuncts
};

bool parse_prog(const std::vector<capsmi_expr>& prog, const std::vector<Role>& cols, ENode& out) {
    std::vector<ENode> st;
    for (const capsmi_expr& x : prog) {
        const int k = arity(x);
        if (k < 0 || (int)st.size() < k) return false;
        ENode n;
        n.x = x;
        n.kids.assign(st.end() - k, st.end());
        st.resize(st.size() - k);
        if (x.op == CAPSMI_X_COL) {
            if (x.arg < 0 || x.arg >= (int)cols.size()) return false;
            n.role = cols[x.arg];
        }
        st.push_back(std::move(n));
    }
    if (st.size() != 1) return false;
    out = std::move(st[0]);
    return true;
}

void flatten_and(const ENode& n, std::vector<ENode>& out) {
    if (n.x.op == CAPSMI_X_AND) {
        for (const ENode& k : n.kids) flatten_and(k, out);
    } else {
        out.push_back(n);
    }
}

// position a join column denotes: a node scan's id, or one end of a relationship hop
int position_of(const Path& P, const Role& r) {
    if (r.k == RK_NODE) {
        if (P.inst[r.inst].role[r.scol] != ROLE_ID) return -1;
        for (size_t p = 0; p < P.pos_node.size(); ++p)
            if (P.pos_node[p] == r.inst) return (int)p;
        return -1;
    }
    if (r.k == RK_REL) {
        const int role = P.inst[r.inst].role[r.scol];
        for (const Hop& h : P.hops) {
            if (h.rel != r.inst) continue;
            if (role == h.from_role) return h.from;
            if (role == h.to_role) return h.to;
        }
    }
    return -1;
}

bool as_paths(const capsmi_table* t, std::vector<Path>& out);

// one left path joined with scan R (JOIN node p over left input `in`): a node scan completes a position,
// a relationship scan adds a hop (Expand) or closes one (ExpandInto)
bool join_path(Path P, const capsmi_table* in, const PlanNode& p, const Scan& R, std::vector<Path>& out) {
    const int ri = (int)P.inst.size();
    std::vector<int> lk, rk;
    for (size_t i = 0; i < p.a.size(); ++i) {
        lk.push_back(find_col(in, p.a[i]));
        rk.push_back(find_col(p.in[1], p.b[i]));
        if (lk.back() < 0 || rk.back() < 0) return false;
    }
    P.inst.push_back(R);
    if (R.kind == 1) {
        if (lk.size() != 1 || R.role[rk[0]] != ROLE_ID) return false;
        const int pos = position_of(P, P.cols[lk[0]]);
        if (pos < 0 || P.pos_node[pos] >= 0) return false;
        P.pos_node[pos] = ri;
    } else {
        if (lk.size() == 1) {  // Expand: a new position
            const int pos = position_of(P, P.cols[lk[0]]);
            const int rr = R.role[rk[0]];
            if (pos < 0 || (rr != ROLE_SRC && rr != ROLE_DST)) return false;
            Hop h;
            h.rel = ri;
            h.from = pos;
            h.to = (int)P.pos_node.size();
            h.from_role = rr;
            h.to_role = rr == ROLE_SRC ? ROLE_DST : ROLE_SRC;
            P.pos_node.push_back(-1);
            P.hops.push_back(h);
        } else if (lk.size() == 2) {  // ExpandInto: both ends bound
            const int p1 = position_of(P, P.cols[lk[0]]), p2 = position_of(P, P.cols[lk[1]]);
            const int r1 = R.role[rk[0]], r2 = R.role[rk[1]];
            if (p1 < 0 || p2 < 0 || !((r1 == ROLE_SRC && r2 == ROLE_DST) || (r1 == ROLE_DST && r2 == ROLE_SRC)))
                return false;
            Hop h;
            h.rel = ri;
            h.from = r1 == ROLE_SRC ? p1 : p2;
            h.to = r1 == ROLE_SRC ? p2 : p1;
            P.hops.push_back(h);
        } else {
            return false;
        }
    }
    const capsmi_table* rt = p.in[1];
    for (size_t k = 0; k < rt->cols.size(); ++k) {
        Role r;
        r.k = R.kind == 1 ? RK_NODE : RK_REL;
        r.inst = ri;
        r.scol = (int)k;
        P.cols.push_back(r);
    }
    out.push_back(std::move(P));
    return true;
}

bool as_paths_node(const capsmi_table* t, std::vector<Path>& out) {
    const PlanNode& p = *t->plan;
    const capsmi_table* in = p.in[0];
    switch (p.kind) {
        case PlanNode::JOIN: {
            if (p.jt != CAPSMI_JOIN_INNER) return false;
            std::vector<Path> L;
            Scan R;
            if (!as_paths(in, L) || L.empty() || !as_scan(p.in[1], R)) return false;
            // a join over a union of branches is the union of the joins (the second hop of an
            // undirected Expand joins both branches of the first)
            for (Path& lp : L)
                if (!join_path(std::move(lp), in, p, R, out)) return false;
            return true;
        }
        case PlanNode::FILTER: {
            if (!as_paths(in, out)) return false;
            for (Path& P : out) {
                ENode e;
                if (!parse_prog(p.progs[0], P.cols, e)) return false;
                flatten_and(e, P.conj);
            }
            return true;
        }
        case PlanNode::WITH_COLUMNS: {
            if (!as_paths(in, out)) return false;
            for (Path& P : out) {
                std::vector<Role> cols = P.cols;
                std::vector<std::string> names;
                for (auto& c : in->cols) names.push_back(c.name);
                for (size_t i = 0; i < p.a.size(); ++i) {
                    Role r;
                    const auto& prog = p.progs[i];
                    if (prog.size() == 1 && prog[0].op == CAPSMI_X_COL) r = P.cols[prog[0].arg];
                    else if (prog.size() == 1 && (prog[0].op == CAPSMI_X_LIT || prog[0].op == CAPSMI_X_NULL)) {
                        r.k = RK_CONST;
                        r.cst = prog[0];
                    }
                    int j = -1;
                    for (size_t q = 0; q < names.size(); ++q) if (names[q] == p.a[i]) j = (int)q;
                    if (j < 0) { names.push_back(p.a[i]); cols.push_back(r); }
                    else cols[j] = r;
                }
                P.cols = std::move(cols);
            }
            return true;
        }
        case PlanNode::SELECT:
        case PlanNode::DROP:
        case PlanNode::RENAME: {
            if (!as_paths(in, out)) return false;
            std::vector<int> pick;
            if (p.kind == PlanNode::SELECT) {
                for (auto& nm : p.a) pick.push_back(find_col(in, nm));
            } else if (p.kind == PlanNode::DROP) {
                std::set<std::string> d(p.a.begin(), p.a.end());
                for (size_t k = 0; k < in->cols.size(); ++k) if (!d.count(in->cols[k].name)) pick.push_back((int)k);
            } else {
                for (size_t k = 0; k < in->cols.size(); ++k) pick.push_back((int)k);
            }
            for (Path& P : out) {
                std::vector<Role> c;
                for (int k : pick) c.push_back(P.cols[k]);
                P.cols = std::move(c);
            }
            return true;
        }
        case PlanNode::UNION: {
            std::vector<Path> r;
            if (!as_paths(in, out) || !as_paths(p.in[1], r)) return false;
            for (Path& x : r) out.push_back(std::move(x));
            return true;
        }
        default: return false;
    }
}

bool as_paths(const capsmi_table* t, std::vector<Path>& out) {
    Scan sc;
    if (as_scan(t, sc)) {  // a node scan starts a pattern
        if (sc.kind != 1) return false;
        Path P;
        P.inst.push_back(sc);
        P.pos_node.push_back(0);
        for (size_t k = 0; k < t->cols.size(); ++k) {
            Role r;
            r.k = RK_NODE;
            r.inst = 0;
            r.scol = (int)k;
            P.cols.push_back(r);
        }
        out.push_back(std::move(P));
        return true;
    }
    if (!t->lazy()) return false;
    return as_paths_node(t, out);
}

// ---- conjunct classification ----------------------------------------------------------------
int hop_of_rel_id(const Path& P, const ENode& n) {
    if (n.x.op != CAPSMI_X_COL || n.role.k != RK_REL) return -1;
    if (P.inst[n.role.inst].role[n.role.scol] != ROLE_ID) return -1;
    for (size_t h = 0; h < P.hops.size(); ++h)
        if (P.hops[h].rel == n.role.inst) return (int)h;
    return -1;
}

// NOT(r_i = r_j) / r_i <> r_j over two hops' relationship ids
bool uniqueness(const Path& P, const ENode& c, int* i, int* j) {
    const ENode* eq = nullptr;
    if (c.x.op == CAPSMI_X_NOT && c.kids[0].x.op == CAPSMI_X_EQ) eq = &c.kids[0];
    else if (c.x.op == CAPSMI_X_NEQ) eq = &c;
    if (!eq) return false;
    *i = hop_of_rel_id(P, eq->kids[0]);
    *j = hop_of_rel_id(P, eq->kids[1]);
    return *i >= 0 && *j >= 0 && *i != *j;
}

// leaves of a node predicate: one node instance's columns and constants; returns the instance or -1
bool node_leaves(const ENode& n, int* inst) {
    if (n.x.op == CAPSMI_X_COL) {
        if (n.role.k == RK_CONST) return true;
        if (n.role.k != RK_NODE) return false;
        if (*inst >= 0 && *inst != n.role.inst) return false;
        *inst = n.role.inst;
        return true;
    }
    for (const ENode& k : n.kids)
        if (!node_leaves(k, inst)) return false;
    return true;
}

// postfix program of a node predicate over one member's base table
void emit_pred(const ENode& n, const Member& m, std::vector<capsmi_expr>& out) {
    for (const ENode& k : n.kids) emit_pred(k, m, out);
    if (n.x.op == CAPSMI_X_COL) {
        if (n.role.k == RK_CONST) {
            out.push_back(n.role.cst);
        } else if (m.src[n.role.scol] >= 0) {
            capsmi_expr x{};
            x.op = CAPSMI_X_COL;
            x.arg = m.src[n.role.scol];
            out.push_back(x);
        } else {
            out.push_back(m.cst[n.role.scol]);
        }
    } else {
        out.push_back(n.x);
    }
}

struct Classified {
    std::set<std::pair<int, int>> uniq;         // hop pairs (i < j) with NOT(r_i = r_j)
    std::vector<std::vector<const ENode*>> pred; // per instance: node predicate conjuncts
};

bool classify(const Path& P, Classified& c) {
    c.pred.assign(P.inst.size(), {});
    for (const ENode& e : P.conj) {
        int i, j;
        if (uniqueness(P, e, &i, &j)) {
            c.uniq.insert({std::min(i, j), std::max(i, j)});
            continue;
        }
        int inst = -1;
        if (!node_leaves(e, &inst)) return false;
        if (inst < 0) {  // constant conjunct: only TRUE is harmless
            if (e.x.op == CAPSMI_X_LIT && e.x.type == CAPSMI_BOOL && e.x.ival != 0) continue;
            return false;
        }
        c.pred[inst].push_back(&e);
    }
    return true;
}

// The id domain the fused kernels run on: the Long ids' window when it holds at most 2^30 ids,
// else the dense ids of a compacted graph (capsmi_graph_compact) shared by every scanned table.
thread_local const DenseIds* g_dense = nullptr;  // domain of the route being planned (one at a time)

// The rank view of a route over a distributed graph (capsmi_graph_distribute, k_dist.hip): the scanned
// tables are this rank's shards; the route exchanges through the session's collective.
struct DistView {
    bool on = false;  // world > 1
    int rank = 0, world = 1;
    int64_t slice_words = 0;
    int rel_mode = -1;  // CAPSMI_RELS_* of the relationship shards
};
thread_local DistView g_dist;

// every scanned table a shard of one distributed graph (then g_dense / g_dist are set), none, or a mix (false)
bool dist_window(const std::vector<Path>& B, bool* any, int64_t* lo, int64_t* hi) {
    const DenseIds* d = nullptr;
    const Shard* sh = nullptr;
    const capsmi_session* sess = nullptr;
    bool all = true;
    int rel_mode = -1;
    *any = false;
    for (const Path& P : B)
        for (const Scan& sc : P.inst) {
            int node_mode = -1;
            for (const Member& m : sc.m) {
                const capsmi_table* t = m.base;
                if (!t->shard) { all = false; continue; }
                *any = true;
                sess = t->sess;
                const DenseIds* e = t->dense.get();  // one domain: equal scramble (tables distributed apart)
                if (d && (e->n != d->n || e->kbits != d->kbits || e->lo != d->lo || e->mul != d->mul)) return false;
                d = e;
                sh = t->shard.get();
                if (sh->kind == 2) {
                    if (rel_mode >= 0 && rel_mode != sh->mode) return false;
                    rel_mode = sh->mode;
                } else {  // one node scan: all members replicated or all owned
                    if (node_mode >= 0 && node_mode != sh->mode) return false;
                    node_mode = sh->mode;
                }
            }
        }
    if (!*any) return true;
    if (!all || !d || d->n > (int64_t(1) << 30)) return false;
    g_dense = d;
    *lo = 0;
    *hi = d->n;
    // world 1 with a collective: the distributed routes over the one shard (their exchanges run through
    // the collective, e.g. RCCL at world size 1)
    if (sh->world > 1 || (sess && sess->coll != nullptr)) {
        g_dist.on = true;
        g_dist.rank = sh->rank;
        g_dist.world = sh->world;
        g_dist.slice_words = sh->slice_words;
        g_dist.rel_mode = rel_mode;
    }
    return true;
}

bool id_window(const std::vector<Path>& B, int64_t* lo, int64_t* hi) {
    g_dist = DistView();
    g_dense = nullptr;
    bool any_shard = false;
    if (!dist_window(B, &any_shard, lo, hi)) return false;
    if (any_shard) return true;
    int64_t l = INT64_MAX, h = INT64_MIN;
    const DenseIds* d = nullptr;
    bool all_dense = true;
    for (const Path& P : B)
        for (const Scan& sc : P.inst)
            for (const Member& m : sc.m) {
                if (!m.base->dense || (d && m.base->dense.get() != d)) all_dense = false;
                else d = m.base->dense.get();
                if (m.base->entity->rows == 0) continue;
                l = std::min(l, m.base->entity->lo);
                h = std::max(h, m.base->entity->hi);
            }
    if (l < h && (uint64_t)(h - l) <= (uint64_t(1) << 30)) {
        *lo = l;
        *hi = h;
        return true;
    }
    if (all_dense && d && !d->scrambled && d->n > 0 && (uint64_t)d->n <= (uint64_t(1) << 30)) {
        g_dense = d;
        *lo = 0;
        *hi = d->n;
        return true;
    }
    return false;
}

// a zero-copy view of a base table with its dense key columns appended (dense domain only)
capsmi_table* dense_view(const capsmi_table* base) {
    auto* x = new capsmi_table();
    x->sess = base->sess;
    x->nrows = base->nrows;
    x->cols = base->cols;
    Column a = base->did, b = base->dsrc, c = base->ddst;
    a.name = "__dense_id";
    b.name = "__dense_src";
    c.name = "__dense_dst";
    if (base->entity->kind == 1) x->cols.push_back(a);
    else { x->cols.push_back(b); x->cols.push_back(c); }
    return x;
}

// ---- bitmaps of node scans (+ predicates) ------------------------------------------------------
struct BitmapSet {
    std::vector<std::pair<std::string, capsmi_bitmap*>> made;
    ~BitmapSet() {
        for (auto& x : made) capsmi_bitmap_release(x.second);
    }
};

std::string member_prog_key(const capsmi_table* base, const std::vector<capsmi_expr>& prog) {
    std::string k(reinterpret_cast<const char*>(&base), sizeof(base));
    k.append(reinterpret_cast<const char*>(prog.data()), prog.size() * sizeof(capsmi_expr));
    return k + "|";
}

// A node scan over OWNED shards (multi-GPU): every rank set the bits of the ids it owns, which lie in
// its slice of the words; one all-gather of the slices completes the bitmap on every rank, and one SUM
// all-reduce gives its set-bit count and whether any rank saw a duplicate row (an id's rows are all on
// its owner, so duplicates are rank-local).
void gather_owned_bitmap(capsmi_session* s, capsmi_bitmap* b) {
    const int64_t S = g_dist.slice_words;
    REQUIRE(b->nwords == S * g_dist.world, CAPSMI_ERR_INTERNAL, "distributed bitmap geometry");
    // a scan that left its count unknown (capsmi_bitmap_add_scan): this rank's bits, before the gather
    if (b->set_bits < 0) b->set_bits = words_popcount(s, P<uint32_t>(b->words), 0, b->nwords);
    Buf full = dev_alloc(sizeof(uint32_t) * (size_t)b->nwords, s);
    collective(s, CAPSMI_COLL_ALL_GATHER, P<uint32_t>(b->words) + (int64_t)g_dist.rank * S, P<uint32_t>(full), S,
               CAPSMI_COLL_U32);
    b->words = full;
    Buf st = dev_alloc(2 * sizeof(int64_t), s);
    fill_i64(P<int64_t>(st), b->set_bits, 1, s->stream);
    fill_i64(P<int64_t>(st) + 1, b->any_dup ? 1 : 0, 1, s->stream);
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(st), P<int64_t>(st), 2, CAPSMI_I64);
    int64_t h[2];
    HIP_CHECK(hipMemcpyAsync(h, P<void>(st), sizeof(h), hipMemcpyDeviceToHost, s->stream));
    HIP_CHECK(hipStreamSynchronize(s->stream));
    b->set_bits = h[0];
    b->any_dup = h[1] > 0;
    b->full = b->set_bits == b->hi - b->lo;
}

// bitmap of node instance `inst` with its predicate conjuncts over [lo, hi); identical scans share one.
// Returns null when an id occurs in two scanned rows (CAPS would bind it twice, ScanGraph.scala:72-76).
capsmi_bitmap* node_bitmap(capsmi_session* s, const Path& P, const Classified& c, int inst, int64_t lo, int64_t hi,
                           BitmapSet& bs, std::string* key_out = nullptr) {
    const Scan& sc = P.inst[inst];
    std::vector<std::vector<capsmi_expr>> progs;
    std::string key;
    for (const Member& m : sc.m) {
        std::vector<capsmi_expr> prog;
        for (const ENode* e : c.pred[inst]) emit_pred(*e, m, prog);
        if (c.pred[inst].size() > 1) {
            capsmi_expr a{};
            a.op = CAPSMI_X_AND;
            a.arg = (int32_t)c.pred[inst].size();
            prog.push_back(a);
        }
        key += member_prog_key(m.base, prog);
        progs.push_back(std::move(prog));
    }
    if (key_out) *key_out = key;
    for (auto& x : bs.made)
        if (x.first == key) return x.second;
    capsmi_bitmap* b = nullptr;
    check(capsmi_bitmap_create(s, lo, hi, &b));
    bs.made.push_back({key, b});
    if (g_dist.on && g_dense && sc.m.size() == 1 && progs[0].empty() && sc.m[0].base->shard &&
        sc.m[0].base->shard->covers && lo == 0 && hi == g_dense->n) {
        // a node table covering the whole domain (over the ranks' shards, checked at registration): every
        // bit set, no row read, no exchange
        bitmap_set_range(b, 0, hi);
        b->rows_added = b->set_bits = hi;
        b->full = true;
        return b;
    }
    for (size_t i = 0; i < sc.m.size(); ++i) {
        const Member& m = sc.m[i];
        const capsmi_expr* pr = progs[i].empty() ? nullptr : progs[i].data();
        if (g_dense) {  // predicate columns keep their indices: the dense id is appended
            capsmi_table* v = dense_view(m.base);
            const capsmi_status st = capsmi_bitmap_add_scan(b, v, "__dense_id", (int32_t)progs[i].size(), pr);
            capsmi_table_release(v);
            check(st);
        } else {
            check(capsmi_bitmap_add_scan(b, m.base, m.base->cols[m.base->entity->id].name.c_str(),
                                         (int32_t)progs[i].size(), pr));
        }
    }
    bool owned = false;
    for (const Member& m : sc.m) owned = owned || (m.base->shard && m.base->shard->mode == CAPSMI_NODES_OWNED);
    if (g_dist.on && owned) gather_owned_bitmap(s, b);
    return b->any_dup ? nullptr : b;
}

// the relationship tables of a hop as (source-side, target-side) column views, zero-copy
struct RelViews {
    std::vector<capsmi_table*> t;
    std::string sig;  // identity of the tables and oriented columns (hops over equal sets share kernels)
    ~RelViews() {
        for (auto* x : t) capsmi_table_release(x);
    }
};

void rel_views(const Path& P, const Hop& h, RelViews& v) {
    std::vector<std::string> sig;
    for (const Member& m : P.inst[h.rel].m) {
        const EntityInfo& e = *m.base->entity;
        const int fc = h.from_role == ROLE_SRC ? e.src : e.dst, tc = h.to_role == ROLE_SRC ? e.src : e.dst;
        auto* x = new capsmi_table();
        x->sess = m.base->sess;
        x->nrows = m.base->nrows;
        Column a = m.base->cols[fc], b = m.base->cols[tc];
        if (g_dense) {
            a = h.from_role == ROLE_SRC ? m.base->dsrc : m.base->ddst;
            b = h.to_role == ROLE_SRC ? m.base->dsrc : m.base->ddst;
        }
        a.name = "s";
        b.name = "t";
        x->cols = {a, b};
        v.t.push_back(x);
        std::string k(reinterpret_cast<const char*>(&m.base), sizeof(m.base));
        k += char(fc);
        k += char(tc);
        k += g_dense ? 'D' : 'L';
        sig.push_back(k);
    }
    std::sort(sig.begin(), sig.end());
    for (auto& k : sig) v.sig += k;
}

// the same relationship views read backwards: (s, t) <- (t, s), zero-copy
void reversed_views(const RelViews& v, RelViews& r) {
    for (capsmi_table* x : v.t) {
        auto* y = new capsmi_table();
        y->sess = x->sess;
        y->nrows = x->nrows;
        Column a = x->cols[1], b = x->cols[0];
        a.name = "s";
        b.name = "t";
        y->cols = {a, b};
        r.t.push_back(y);
    }
    r.sig = v.sig + "~";
}

bool id_like(const Path& P, const Role& r) {  // a non-null id / endpoint column
    if (r.k == RK_NODE) return P.inst[r.inst].role[r.scol] == ROLE_ID;
    if (r.k == RK_REL) return P.inst[r.inst].role[r.scol] != ROLE_NONE;
    return false;
}

capsmi_table* result_table(capsmi_session* s, int64_t rows) {
    auto* r = new capsmi_table();
    r->sess = s;
    r->nrows = rows;
    return r;
}

Column i64_column(capsmi_session* s, const std::vector<int64_t>& v) {
    Column c;
    c.type = CAPSMI_I64;
    c.data = dev_alloc(sizeof(int64_t) * (v.empty() ? 1 : v.size()), s);
    c.host = std::make_shared<const std::vector<int64_t>>(v);
    if (v.size() == 1) {  // one word: a fill kernel, so neither a copy nor a host sync
        fill_i64(P<int64_t>(c.data), v[0], 1, s->stream);
    } else if (!v.empty()) {
        HIP_CHECK(hipMemcpyAsync(P<void>(c.data), v.data(), sizeof(int64_t) * v.size(), hipMemcpyHostToDevice, s->stream));
        HIP_CHECK(hipStreamSynchronize(s->stream));
    }
    return c;
}

// ---- the shapes ---------------------------------------------------------------------------------
enum Agg1 { A_COUNT, A_DISTINCT_END, A_DISTINCT_START };

// count-like aggregates of a group over one branch
bool agg_kinds(const capsmi_table* in, const PlanNode& g, const Path& P, int start, int end, std::vector<int>& kinds) {
    for (const AggSpec& a : g.aggs) {
        if (a.kind == CAPSMI_AGG_COUNT_STAR) { kinds.push_back(A_COUNT); continue; }
        if (a.kind != CAPSMI_AGG_COUNT) return false;
        const int c = find_col(in, a.input);
        if (c < 0) return false;
        const Role& r = P.cols[c];
        if (!a.distinct) {
            if (!id_like(P, r)) return false;
            kinds.push_back(A_COUNT);
            continue;
        }
        const int pos = position_of(P, r);
        if (pos >= 0 && pos == end && end != start) kinds.push_back(A_DISTINCT_END);
        else if (pos >= 0 && pos == start && end != start) kinds.push_back(A_DISTINCT_START);
        else return false;
    }
    return true;
}

// chain P0 -h0-> P1 -h1-> ... with hop i from position i to i + 1; true if the hops form that chain
bool is_chain(const Path& P) {
    for (size_t i = 0; i < P.hops.size(); ++i)
        if (P.hops[i].from != (int)i || P.hops[i].to != (int)i + 1) return false;
    return P.pos_node.size() == P.hops.size() + 1;
}

bool same_orientation(const Path& P) {
    for (const Hop& h : P.hops)
        if (h.from_role != P.hops[0].from_role) return false;
    return true;
}

bool all_pairs_unique(const Classified& c, int nh) {
    for (int i = 0; i < nh; ++i)
        for (int j = i + 1; j < nh; ++j)
            if (!c.uniq.count({i, j})) return false;
    return (int)c.uniq.size() == nh * (nh - 1) / 2;
}

void route(capsmi_session* s, const char* name) { s->routes[name] += 1; }

bool any_no_loops(const Path& P) {  // an undirected branch: only fused_undirected takes it
    for (const Scan& sc : P.inst) if (sc.no_loops) return true;
    return false;
}
thread_local bool g_missed = false;  // a pattern shape went unrouted during the current materialisation

int bits_for_ids(int64_t n) {  // bits of the largest relative id (k_tri.hip bits_for)
    int b = 1;
    while (b < 63 && (int64_t(1) << b) < n) ++b;
    return b;
}

int64_t sum_over_ranks(capsmi_session* s, int64_t v) {
    Buf t = dev_alloc(sizeof(int64_t), s);
    fill_i64(P<int64_t>(t), v, 1, s->stream);
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(t), P<int64_t>(t), 1, CAPSMI_I64);
    return read_scalar(s, P<int64_t>(t));
}

// the owned X1 / X2 slices side by side (one all-gather for both), and back into [X1 | X2] after it
__global__ void k_pack_x12(const uint32_t* __restrict__ mid, int64_t nw, int64_t S, int64_t r, uint32_t* __restrict__ send) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * S; i += (int64_t)gridDim.x * blockDim.x)
        send[i] = mid[(i < S ? 0 : nw) + r * S + (i < S ? i : i - S)];
}
__global__ void k_unpack_x12(const uint32_t* __restrict__ got, int64_t nw, int64_t S, uint32_t* __restrict__ full) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * nw; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = (i / S) >> 1, h = (i / S) & 1, k = i % S;  // got = [rank][X1 | X2][S]
        full[h * nw + q * S + k] = got[i];
    }
}

// 2-hop count(DISTINCT end) over relationship shards BY_TARGET: hop 1 is complete for the
// middle ids this rank owns (their in-relationships are all here), one all-gather of the owned slices of
// the frontier (X1, X2) gives every rank the whole frontier, hop 2 marks the end ids this rank owns, and
// the owned popcounts add up in one all-reduce.  `cached`: the relationship layout kept by cache().
int64_t dist_two_hop_distinct(capsmi_session* s, const capsmi_relpart* cached, int32_t nt, capsmi_table* const* views,
                              const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c) {
    const int64_t S = g_dist.slice_words, nw = b->nwords, r = g_dist.rank;
    REQUIRE(nw == S * g_dist.world, CAPSMI_ERR_INTERNAL, "distributed bitmap geometry");
    Buf mid = dev_alloc(sizeof(uint32_t) * 2 * nw, s), scratch = dev_alloc(sizeof(uint32_t) * nw, s);
    Buf full = dev_alloc(sizeof(uint32_t) * 2 * nw, s), dst = dev_alloc(sizeof(uint32_t) * nw, s);
    capsmi_relpart* rp = nullptr;
    if (cached) check(capsmi_two_hop_mark_mid_part(s, cached, a, b, P<uint32_t>(mid), P<uint32_t>(scratch)));
    else check(capsmi_relpart_build_mark_mid(s, nt, views, "s", "t", a, b, P<uint32_t>(mid), P<uint32_t>(scratch), &rp));
    std::unique_ptr<capsmi_relpart, capsmi_status (*)(capsmi_relpart*)> hold(rp, capsmi_relpart_release);
    {  // one all-gather of the owned (X1, X2) slice pairs instead of one per frontier
        Buf x12 = dev_alloc(sizeof(uint32_t) * (2 * S + 2 * nw), s);
        uint32_t *send = P<uint32_t>(x12), *got = send + 2 * S;
        const unsigned gs = (unsigned)std::max<int64_t>(1, std::min<int64_t>((2 * S + 255) / 256, (int64_t)s->num_cus * 8));
        const unsigned gn = (unsigned)std::max<int64_t>(1, std::min<int64_t>((2 * nw + 255) / 256, (int64_t)s->num_cus * 8));
        hipLaunchKernelGGL(k_pack_x12, dim3(gs), dim3(256), 0, s->stream, P<uint32_t>(mid), nw, S, r, send);
        HIP_CHECK(hipGetLastError());
        collective(s, CAPSMI_COLL_ALL_GATHER, send, got, 2 * S, CAPSMI_COLL_U32);
        hipLaunchKernelGGL(k_unpack_x12, dim3(gn), dim3(256), 0, s->stream, got, nw, S, P<uint32_t>(full));
        HIP_CHECK(hipGetLastError());
    }
    check(capsmi_two_hop_mark_dst_part(s, cached ? cached : rp, b, c, P<uint32_t>(full), P<uint32_t>(dst)));
    Buf cnt = dev_alloc(sizeof(int64_t), s);
    check(capsmi_words_popcount_device(s, P<uint32_t>(dst), r * S, (r + 1) * S, P<int64_t>(cnt)));
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(cnt), P<int64_t>(cnt), 1, CAPSMI_I64);
    return read_scalar(s, P<int64_t>(cnt));
}

// [X1 | X2] (2 x W x S words) -> rank-major send segments [q][X1 slice q | X2 slice q] (2 x S each)
__global__ void k_x12_by_owner(const uint32_t* __restrict__ mid, int64_t nw, int64_t S, int W, uint32_t* __restrict__ send) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * nw; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = i / (2 * S), h = (i / S) & 1, k = i % S;
        send[i] = mid[h * nw + q * S + k];
    }
}
// OR of the W received [X1 | X2] slice pairs (got = [source rank][2][S]) into this rank's slices of full
// [X1 | X2] (words outside them zero: hop 2 reads X only at the owned sources of this rank's relationships)
__global__ void k_x12_or(const uint32_t* __restrict__ got, int W, int64_t nw, int64_t S, int64_t r,
                         uint32_t* __restrict__ full) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * S; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0;
        for (int q = 0; q < W; ++q) v |= got[(int64_t)q * 2 * S + i];
        const int64_t h = i / S, k = i % S;
        full[h * nw + r * S + k] = v;
    }
}
// popcount of the OR of W received slices of S words (got = [source rank][S]) added into *cnt
__global__ void k_or_popcount(const uint32_t* __restrict__ got, int W, int64_t S, unsigned long long* __restrict__ cnt) {
    unsigned long long c = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < S; k += (int64_t)gridDim.x * blockDim.x) {
        uint32_t v = 0;
        for (int q = 0; q < W; ++q) v |= got[(int64_t)q * S + k];
        c += __popc(v);
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

unsigned small_grid(capsmi_session* s, int64_t n) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, (int64_t)s->num_cus * 8));
}

// The union of every rank's partial bitmap `words` (W x S words, rank-major slices) counted: one equal-count
// ALL_TO_ALL_V gives each rank every rank's copy of its owned slice, ORed and popcounted on the device, and
// one all-reduce adds the owned counts -- the reduce-scatter(OR) + popcount of SURVEY.md 8e (bitwise OR is
// not an RCCL reduction).  Returns the count (the step's one host read).
int64_t or_reduce_count(capsmi_session* s, const uint32_t* words) {
    const int64_t S = g_dist.slice_words;
    const int W = g_dist.world;
    Buf got = dev_alloc(sizeof(uint32_t) * (size_t)W * S, s), cnt = dev_alloc(sizeof(int64_t), s);
    std::vector<int64_t> c(W, S);
    collective_a2av(s, words, c.data(), P<void>(got), c.data(), CAPSMI_COLL_U32, S);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(int64_t), s->stream));
    hipLaunchKernelGGL(k_or_popcount, dim3(small_grid(s, S)), dim3(256), 0, s->stream, P<uint32_t>(got), W, S,
                       P<unsigned long long>(cnt));
    HIP_CHECK(hipGetLastError());
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(cnt), P<int64_t>(cnt), 1, CAPSMI_I64);
    return read_scalar(s, P<int64_t>(cnt));
}

// 2-hop count(DISTINCT end) over relationship shards BY_SOURCE (north_star's owner(source)):
// hop 1 over this rank's relationships (sources owned, middles anywhere) marks a partial frontier
// X1 = M | S1, X2 = M | S2 for every id -- S1 / S2 (self-loops) are complete on the owner, and M is an OR
// over the ranks; one ALL_TO_ALL_V of the slices + OR gives each rank the whole frontier of its owned
// middles, which are exactly the sources of its hop-2 relationships; hop 2 marks ends anywhere, and the
// OR-reduce + popcount of the end bitmap gives the answer (or_reduce_count).
int64_t dist_two_hop_distinct_src(capsmi_session* s, const capsmi_relpart* cached, int32_t nt, capsmi_table* const* views,
                                  const capsmi_bitmap* a, const capsmi_bitmap* b, const capsmi_bitmap* c) {
    const int64_t S = g_dist.slice_words, nw = b->nwords, r = g_dist.rank;
    const int W = g_dist.world;
    REQUIRE(nw == S * W, CAPSMI_ERR_INTERNAL, "distributed bitmap geometry");
    Buf mid = dev_alloc(sizeof(uint32_t) * 2 * nw, s), scratch = dev_alloc(sizeof(uint32_t) * nw, s);
    Buf full = dev_alloc(sizeof(uint32_t) * 2 * nw, s), dst = dev_alloc(sizeof(uint32_t) * nw, s);
    capsmi_relpart* rp = nullptr;
    if (cached) check(capsmi_two_hop_mark_mid_part(s, cached, a, b, P<uint32_t>(mid), P<uint32_t>(scratch)));
    else check(capsmi_relpart_build_mark_mid(s, nt, views, "s", "t", a, b, P<uint32_t>(mid), P<uint32_t>(scratch), &rp));
    std::unique_ptr<capsmi_relpart, capsmi_status (*)(capsmi_relpart*)> hold(rp, capsmi_relpart_release);
    {
        Buf x12 = dev_alloc(sizeof(uint32_t) * 4 * nw, s);
        uint32_t *send = P<uint32_t>(x12), *got = send + 2 * nw;
        hipLaunchKernelGGL(k_x12_by_owner, dim3(small_grid(s, 2 * nw)), dim3(256), 0, s->stream, P<uint32_t>(mid), nw, S,
                           W, send);
        HIP_CHECK(hipGetLastError());
        std::vector<int64_t> cnt(W, 2 * S);
        collective_a2av(s, send, cnt.data(), got, cnt.data(), CAPSMI_COLL_U32, 2 * S);
        HIP_CHECK(hipMemsetAsync(P<void>(full), 0, sizeof(uint32_t) * 2 * nw, s->stream));
        hipLaunchKernelGGL(k_x12_or, dim3(small_grid(s, 2 * S)), dim3(256), 0, s->stream, got, W, nw, S, r,
                           P<uint32_t>(full));
        HIP_CHECK(hipGetLastError());
    }
    check(capsmi_two_hop_mark_dst_part(s, cached ? cached : rp, b, c, P<uint32_t>(full), P<uint32_t>(dst)));
    return or_reduce_count(s, P<uint32_t>(dst));
}

// 2-hop count(*) over relationship shards BY_TARGET: each rank's relationships into its owned ids give
// their complete in-degrees inA; one all-gather of the owned slices gives every rank inA of every id; each
// rank sums inA(source) over its relationships (less its self-loops) and one all-reduce adds the parts
int64_t dist_two_hop_count(capsmi_session* s, int32_t nt, capsmi_table* const* views, const capsmi_bitmap* a,
                           const capsmi_bitmap* b, const capsmi_bitmap* c) {
    const int64_t S = g_dist.slice_words, n = b->hi - b->lo, r = g_dist.rank;
    const int64_t own_lo = r * 32 * S, own_hi = std::min(own_lo + 32 * S, n);
    Buf owned = dev_alloc(sizeof(uint32_t) * 32 * S, s), in_all = dev_alloc(sizeof(uint32_t) * 32 * S * g_dist.world, s);
    Buf cnt = dev_alloc(sizeof(int64_t), s);
    capsmi_count_shard* h = nullptr;
    check(capsmi_count_shard_begin(s, nt, views, "s", "t", a, b, c, own_lo, own_hi, P<uint32_t>(owned), &h));
    std::unique_ptr<capsmi_count_shard, capsmi_status (*)(capsmi_count_shard*)> hold(h, capsmi_count_shard_release);
    collective(s, CAPSMI_COLL_ALL_GATHER, P<uint32_t>(owned), P<uint32_t>(in_all), 32 * S, CAPSMI_COLL_U32);
    check(capsmi_count_shard_finish(h, P<uint32_t>(in_all), P<int64_t>(cnt)));
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(cnt), P<int64_t>(cnt), 1, CAPSMI_I64);
    return read_scalar(s, P<int64_t>(cnt));
}

std::unique_ptr<capsmi_bitmap> owned_mask(capsmi_session* s, const capsmi_bitmap* b);

// count(*) over distributed shards without moving any per-id array.  A rank's shard and
// its complement (BY_SOURCE: the relationships from other ranks' sources into owned ids; BY_TARGET: those from
// owned sources into other ranks' ids; exchanged once at capsmi_graph_distribute) hold every relationship
// incident to an owned id exactly once, so for an owned middle b both inA(b) and outC(b) are complete here:
// count(*) = sum over the ranks of sum_{owned b} b_ok(b) inA(b) outC(b) - loops(b), one record-partition
// count over the union with b restricted to owned ids and one 8-byte all-reduce -- per-rank bytes received
// fall with N (the earlier BY_TARGET form all-gathered 4 B x every id's in-degree, 256 MiB at 2^26 ids).
// The walk's orientation picks which complement column is the source.
int64_t dist_two_hop_count_owned(capsmi_session* s, const Path& P, const RelViews& v0, const capsmi_bitmap* a,
                               const capsmi_bitmap* b, const capsmi_bitmap* c) {
    REQUIRE(!a->any_dup && !b->any_dup && !c->any_dup, CAPSMI_ERR_UNSUPPORTED,
            "closed-form count(*) needs each node id in one scanned row");
    const Hop& h = P.hops[0];
    const bool fwd = h.from_role == ROLE_SRC;
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (capsmi_table* t : v0.t) {
        srcs.push_back(t->cols[0].d());
        dsts.push_back(t->cols[1].d());
        ms.push_back(t->nrows);
    }
    for (const Member& m : P.inst[h.rel].m) {
        if (m.base->in_rows <= 0) continue;
        srcs.push_back(fwd ? m.base->in_src.d() : m.base->in_dst.d());
        dsts.push_back(fwd ? m.base->in_dst.d() : m.base->in_src.d());
        ms.push_back(m.base->in_rows);
    }
    std::unique_ptr<capsmi_bitmap> bown = owned_mask(s, b);
    const int64_t x = two_hop_count_rec(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), a, bown.get(), c);
    return sum_over_ranks(s, x);
}

// the cyclic triangle count over a distributed graph (any relationship mode): the distributed trigraph
// build (k_tri.hip tri_build: pairs exchanged to their lower end's owner, oriented ranges exchanged and
// all-gathered), this rank's work share of the centers, one all-reduce of the parts
int64_t dist_triangle_count(capsmi_session* s, const std::vector<capsmi_table*>& views, const capsmi_bitmap* n_ok) {
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (capsmi_table* t : views) {
        srcs.push_back(t->cols[0].d());
        dsts.push_back(t->cols[1].d());
        ms.push_back(t->nrows);
    }
    TriDist dd;
    dd.rank = g_dist.rank;
    dd.world = g_dist.world;
    dd.span = 32 * g_dist.slice_words;
    TriGraph g;
    tri_build(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), n_ok, g, &dd);
    const uint64_t part = tri_count(s, g, g_dist.rank, g_dist.world);
    return sum_over_ranks(s, (int64_t)part);
}

// count(*) / count(DISTINCT end | start) of one branch: 1 hop, a 2-hop chain, or the closed triangle.
// Returns false when the shape or a precondition does not hold.
bool fused_counts(capsmi_session* s, const Path& P, const std::vector<int>& kinds, std::vector<int64_t>& vals) {
    Classified c;
    if (any_no_loops(P) || !classify(P, c)) return false;
    for (int x : P.pos_node) if (x < 0) return false;
    const size_t nh = P.hops.size();
    if (nh < 1 || nh > 3) return false;
    std::vector<Path> one{P};
    int64_t lo, hi;
    if (!id_window(one, &lo, &hi)) return false;
    BitmapSet bs;
    RelViews v0;
    rel_views(P, P.hops[0], v0);
    const int64_t nt = (int64_t)v0.t.size();
    if (nh == 1 && is_chain(P) && c.uniq.empty()) {
        for (int k : kinds) if (k != A_COUNT) return false;
        capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs);
        capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[1], lo, hi, bs);
        if (!a || !b) return false;
        int64_t total = 0;
        for (capsmi_table* t : v0.t) {
            const char* sc[1] = {"s"};
            capsmi_table* o = nullptr;
            check(capsmi_expand_filter(s, t, "s", "t", a, b, 1, sc, nullptr, &o));
            total += o->nrows;
            capsmi_table_release(o);
        }
        if (g_dist.on) total = sum_over_ranks(s, total);  // each rank counted its own relationships
        vals.assign(kinds.size(), total);
        route(s, "expand_count");
        return true;
    }
    if (nh == 2 && is_chain(P) && same_orientation(P)) {
        RelViews v1;
        rel_views(P, P.hops[1], v1);
        if (v1.sig != v0.sig || !all_pairs_unique(c, 2)) return false;
        if (g_dist.on)  // the distributed count(*) folds in-degrees of at most 2^26 ids (k_count.hip)
            for (int k : kinds)
                if (k == A_COUNT && hi - lo > (int64_t(1) << 26)) return false;
        capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs);
        capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[1], lo, hi, bs);
        capsmi_bitmap* cc = node_bitmap(s, P, c, P.pos_node[2], lo, hi, bs);
        if (!a || !b || !cc) return false;
        // Cache analogue: relationship tables marked cache() keep the partitioned layout of the walk
        const Scan& R = P.inst[P.hops[0].rel];
        bool keep = !R.m.empty();
        for (const Member& m : R.m) keep = keep && m.base->keep_layouts;
        // the reversed relationships (distinct start = distinct end of the reversed walk)
        RelViews rv;
        reversed_views(v0, rv);
        const bool by_tgt = g_dist.rel_mode == CAPSMI_RELS_BY_TARGET;
        for (int k : kinds) {
            int64_t x = 0;
            const bool rev = k == A_DISTINCT_START;
            capsmi_table* const* vw = rev ? rv.t.data() : v0.t.data();
            const capsmi_bitmap* A = rev ? cc : a;
            const capsmi_bitmap* C = rev ? a : cc;
            const capsmi_relpart* lay = nullptr;
            if (keep && k != A_COUNT) {
                const std::string key = v0.sig + (rev ? "<" : ">") + std::to_string(lo) + ":" + std::to_string(hi);
                auto& cache = R.m[0].base->layouts;
                auto it = cache.find(key);
                if (it == cache.end()) {
                    capsmi_relpart* rp = nullptr;
                    check(capsmi_relpart_build(s, (int32_t)nt, vw, "s", "t", lo, hi, &rp));
                    it = cache.emplace(key, std::shared_ptr<capsmi_relpart>(rp, [](capsmi_relpart* q) {
                                           capsmi_relpart_release(q);
                                       })).first;
                }
                lay = it->second.get();
            }
            if (g_dist.on && k == A_COUNT) {
                // the shard and its complement around the owned middles, no per-id exchange (dense ids: the
                // complement's); without dense ids the all-gather form (BY_TARGET forwards, BY_SOURCE reversed)
                x = g_dense ? dist_two_hop_count_owned(s, P, v0, a, b, cc)
                    : by_tgt ? dist_two_hop_count(s, (int32_t)nt, v0.t.data(), a, b, cc)
                             : dist_two_hop_count(s, (int32_t)nt, rv.t.data(), cc, b, a);
            } else if (g_dist.on) {
                // the walk's relationships arrive by their end's owner (BY_TARGET forwards, BY_SOURCE reversed):
                // the all-gather form; by their start's owner: the OR-reduce form
                const bool end_owned = by_tgt != rev;
                x = end_owned ? dist_two_hop_distinct(s, lay, lay ? 0 : (int32_t)nt, lay ? nullptr : vw, A, b, C)
                              : dist_two_hop_distinct_src(s, lay, lay ? 0 : (int32_t)nt, lay ? nullptr : vw, A, b, C);
            } else if (k == A_COUNT) {
                check(capsmi_two_hop_count(s, (int32_t)nt, v0.t.data(), "s", "t", a, b, cc, &x));
            } else if (lay) {
                check(capsmi_two_hop_count_distinct_part(s, lay, A, b, C, &x));
            } else {
                check(capsmi_two_hop_count_distinct(s, (int32_t)nt, vw, "s", "t", A, b, C, &x));
            }
            vals.push_back(x);
        }
        route(s, "two_hop");
        return true;
    }
    if (nh == 3 && P.pos_node.size() == 3 && same_orientation(P)) {
        // P0 -h0-> P1 -h1-> P2 -h2-> P0 (the closing hop is the ExpandInto)
        const Hop &h0 = P.hops[0], &h1 = P.hops[1], &h2 = P.hops[2];
        if (!(h0.from == 0 && h0.to == 1 && h1.from == 1 && h1.to == 2 && h2.from == 2 && h2.to == 0)) return false;
        RelViews v1, v2;
        rel_views(P, h1, v1);
        rel_views(P, h2, v2);
        if (v1.sig != v0.sig || v2.sig != v0.sig || !all_pairs_unique(c, 3)) return false;
        for (int k : kinds) if (k != A_COUNT) return false;
        std::string k0, k1, k2;
        capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs, &k0);
        capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[1], lo, hi, bs, &k1);
        capsmi_bitmap* cc = node_bitmap(s, P, c, P.pos_node[2], lo, hi, bs, &k2);
        if (!a || !b || !cc || k0 != k1 || k1 != k2) return false;  // one node filter for all three
        // the distributed build codes oriented targets in 24 bits: larger domains take the generic plan
        if (g_dist.on && (bits_for_ids(hi - lo) + 7) / 8 * 8 > 24) return false;
        int64_t x = 0;
        if (g_dist.on) x = dist_triangle_count(s, v0.t, a);
        else check(capsmi_triangle_count(s, (int32_t)nt, v0.t.data(), "s", "t", a, &x));
        vals.assign(kinds.size(), x);
        route(s, "triangle");
        return true;
    }
    return false;
}

// a copy of bitmap b restricted to this rank's owned ids (whole word slices [rank * S, (rank + 1) * S))
std::unique_ptr<capsmi_bitmap> owned_mask(capsmi_session* s, const capsmi_bitmap* b) {
    const int64_t S = g_dist.slice_words, r = g_dist.rank;
    REQUIRE(b->nwords == S * g_dist.world, CAPSMI_ERR_INTERNAL, "distributed bitmap geometry");
    auto m = std::make_unique<capsmi_bitmap>();
    m->sess = s;
    m->lo = b->lo;
    m->hi = b->hi;
    m->nwords = b->nwords;
    m->words = dev_alloc(sizeof(uint32_t) * (size_t)b->nwords, s);
    m->any_dup = b->any_dup;
    HIP_CHECK(hipMemsetAsync(P<void>(m->words), 0, sizeof(uint32_t) * (size_t)b->nwords, s->stream));
    HIP_CHECK(hipMemcpyAsync(P<uint32_t>(m->words) + r * S, P<uint32_t>(b->words) + r * S, sizeof(uint32_t) * S,
                             hipMemcpyDeviceToDevice, s->stream));
    return m;
}

// The undirected 1- / 2-hop routes over BY_SOURCE shards.  A rank's relationships (sources owned) hold each
// relationship once over the ranks; with its in-relationships (targets owned, exchanged at registration)
// they are every relationship incident to an owned id.
//   1 hop: the arcs of the rank's own relationships: count(*) summed, distinct ends ORed over the ranks;
//   2 hops: the middle b restricted to owned ids, over every relationship incident to them, so inU(b),
//   outU(b), K(b) and x(b) are complete: count(*) summed, the distinct ends ORed (or_reduce_count).
void dist_undirected(capsmi_session* s, const Scan& R, const std::vector<const int64_t*>& srcs,
                     const std::vector<const int64_t*>& dsts, const std::vector<int64_t>& ms, int h,
                     const std::vector<capsmi_bitmap*>& pos, const std::vector<int>& kinds, std::vector<int64_t>& vals) {
    std::vector<const int64_t*> as = srcs, ad = dsts;  // + the in-relationships
    std::vector<int64_t> am = ms;
    for (const Member& m : R.m) {
        if (m.base->in_rows <= 0) continue;
        as.push_back(m.base->in_src.d());
        ad.push_back(m.base->in_dst.d());
        am.push_back(m.base->in_rows);
    }
    std::unique_ptr<capsmi_bitmap> bown;
    if (h == 2) bown = owned_mask(s, pos[1]);
    Buf marks = dev_alloc(sizeof(uint32_t) * (size_t)pos[0]->nwords, s);
    for (int k : kinds) {
        const int kind = k == A_COUNT ? 0 : (k == A_DISTINCT_END ? 1 : 2);
        int64_t x;
        if (h == 1) {
            x = undirected_count(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), 1, pos[0], pos[1], pos[1], kind,
                                 kind ? P<uint32_t>(marks) : nullptr);
        } else {
            x = undirected_count(s, as.data(), ad.data(), am.data(), (int)as.size(), 2, pos[0], bown.get(), pos[2], kind,
                                 kind ? P<uint32_t>(marks) : nullptr);
        }
        vals.push_back(kind ? or_reduce_count(s, P<uint32_t>(marks)) : sum_over_ranks(s, x));
    }
}

// Undirected Expand chains of 1 or 2 hops (RelationalPlanner.scala:126-136): 2^hops branches, one per
// orientation of the hops, the incoming hops over relationships with start <> end, the same node scans at
// every position, pairwise uniqueness of the relationships; count(*) / count(DISTINCT end | start).
bool fused_undirected(capsmi_session* s, const capsmi_table* in, const PlanNode& g, const std::vector<Path>& B,
                      std::vector<int64_t>& vals) {
    const size_t h = B[0].hops.size();
    if (h < 1 || h > 2 || B.size() != (size_t(1) << h)) return false;
    std::set<int> orients;
    std::vector<Classified> cls(B.size());
    std::vector<int> kinds;
    for (size_t bi = 0; bi < B.size(); ++bi) {
        const Path& P = B[bi];
        if (P.hops.size() != h || !is_chain(P)) return false;
        for (int x : P.pos_node) if (x < 0) return false;
        int o = 0;
        for (size_t i = 0; i < h; ++i) {
            const bool incoming = P.hops[i].from_role == ROLE_DST;
            if (P.inst[P.hops[i].rel].no_loops != incoming) return false;
            o |= (incoming ? 1 : 0) << i;
        }
        orients.insert(o);
        if (!classify(P, cls[bi])) return false;
        if (h == 2 ? !all_pairs_unique(cls[bi], 2) : !cls[bi].uniq.empty()) return false;
        std::vector<int> k;
        if (!agg_kinds(in, g, P, 0, (int)h, k)) return false;
        if (bi == 0) kinds = k;
        else if (k != kinds) return false;
    }
    if (orients.size() != B.size()) return false;
    int64_t lo, hi;
    if (!id_window(B, &lo, &hi)) return false;
    // distributed: BY_SOURCE shards, whose in-relationships complete every owned id's incident set
    if (g_dist.on && g_dist.rel_mode != CAPSMI_RELS_BY_SOURCE) return false;
    // one relationship set for every hop of every branch, read as (start, end)
    auto plain_views = [&](const Path& P, const Hop& hp, RelViews& v) {
        Hop fwd = hp;
        fwd.from_role = ROLE_SRC;
        fwd.to_role = ROLE_DST;
        rel_views(P, fwd, v);
    };
    RelViews v0;
    plain_views(B[0], B[0].hops[0], v0);
    for (const Path& P : B)
        for (const Hop& hp : P.hops) {
            RelViews v;
            plain_views(P, hp, v);
            if (v.sig != v0.sig) return false;
        }
    // one node scan per position, identical in every branch
    BitmapSet bs;
    std::vector<capsmi_bitmap*> pos(h + 1, nullptr);
    for (size_t q = 0; q <= h; ++q) {
        std::string k0;
        pos[q] = node_bitmap(s, B[0], cls[0], B[0].pos_node[q], lo, hi, bs, &k0);
        if (!pos[q]) return false;
        for (size_t bi = 1; bi < B.size(); ++bi) {
            std::string kq;
            if (!node_bitmap(s, B[bi], cls[bi], B[bi].pos_node[q], lo, hi, bs, &kq) || kq != k0) return false;
        }
    }
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (capsmi_table* t : v0.t) {
        srcs.push_back(t->cols[0].d());
        dsts.push_back(t->cols[1].d());
        ms.push_back(t->nrows);
    }
    if (g_dist.on) {
        dist_undirected(s, B[0].inst[B[0].hops[0].rel], srcs, dsts, ms, (int)h, pos, kinds, vals);
        route(s, "undirected");
        return true;
    }
    for (int k : kinds) {
        const int kind = k == A_COUNT ? 0 : (k == A_DISTINCT_END ? 1 : 2);
        vals.push_back(undirected_count(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), (int)h, pos[0], pos[1],
                                        h == 2 ? pos[2] : pos[1], kind));
    }
    route(s, "undirected");
    return true;
}

// the start ids of a route's rows back to the graph's Long ids (relative ids in [0, n) of the route's window)
void ids_to_long(capsmi_session* s, int64_t lo, int64_t* v, int64_t n) {
    if (n <= 0) return;
    if (!g_dense) {
        add_i64(v, lo, n, s->stream);
    } else if (g_dense->scrambled) {
        unscramble_ids(s, *g_dense, v, n);
    } else {
        Buf ids = dev_alloc(sizeof(int64_t) * n, s);
        gather_col(P<int64_t>(g_dense->orig), nullptr, v, n, P<int64_t>(ids), nullptr, s->stream);
        HIP_CHECK(hipMemcpyAsync(v, P<void>(ids), sizeof(int64_t) * n, hipMemcpyDeviceToDevice, s->stream));
    }
}

// C3's grouped form: the 2-hop chain grouped by its start node, count(*) / count(DISTINCT end)
bool fused_grouped_two_hop(capsmi_session* s, const capsmi_table* in, const PlanNode& g, const std::vector<Path>& B,
                           capsmi_table** out) {
    if (B.size() != 1 || g.a.size() != 1 || g.aggs.empty()) return false;
    const Path& P = B[0];
    if (any_no_loops(P) || P.hops.size() != 2 || !is_chain(P) || !same_orientation(P)) return false;
    for (int x : P.pos_node) if (x < 0) return false;
    const int gc = find_col(in, g.a[0]);
    if (gc < 0 || position_of(P, P.cols[gc]) != 0 || !id_like(P, P.cols[gc])) return false;
    std::vector<int> kinds;
    if (!agg_kinds(in, g, P, 0, 2, kinds)) return false;
    for (int k : kinds) if (k == A_DISTINCT_START) return false;
    Classified c;
    if (!classify(P, c) || !all_pairs_unique(c, 2)) return false;
    RelViews v0, v1;
    rel_views(P, P.hops[0], v0);
    rel_views(P, P.hops[1], v1);
    if (v0.sig != v1.sig) return false;
    std::vector<Path> one{P};
    int64_t lo, hi;
    if (!id_window(one, &lo, &hi)) return false;
    if (g_dist.on && g_dist.rel_mode != CAPSMI_RELS_BY_SOURCE) return false;  // the rows of owned starts
    BitmapSet bs;
    capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs);
    capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[1], lo, hi, bs);
    capsmi_bitmap* cc = node_bitmap(s, P, c, P.pos_node[2], lo, hi, bs);
    if (!a || !b || !cc) return false;
    std::vector<const int64_t*> srcs, dsts;
    std::vector<int64_t> ms;
    for (capsmi_table* t : v0.t) {
        srcs.push_back(t->cols[0].d());
        dsts.push_back(t->cols[1].d());
        ms.push_back(t->nrows);
    }
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    auto* r = result_table(s, 0);
    std::unique_ptr<capsmi_table> guard(r);
    int64_t rows = -1;
    for (size_t i = 0; i < kinds.size(); ++i) {
        Buf ids, vals;
        int64_t nrow = 0;
        GroupedDist gd;
        gd.rank = g_dist.rank;
        gd.world = g_dist.world;
        gd.span = 32 * g_dist.slice_words;
        if (!grouped_two_hop(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), a, b, cc, kinds[i] != A_COUNT,
                             (int64_t)(free_b / 2), ids, vals, &nrow, g_dist.on ? &gd : nullptr))
            return false;  // the keys would not fit: the generic plan (and its size guard) decides
        REQUIRE(rows < 0 || rows == nrow, CAPSMI_ERR_INTERNAL, "grouped 2-hop: aggregates disagree on the groups");
        if (i == 0) {
            rows = nrow;
            ids_to_long(s, lo, ::capsmi::P<int64_t>(ids), nrow);
            Column k;
            k.type = CAPSMI_I64;
            k.data = ids;
            r->cols.push_back(std::move(k));
        }
        Column v;
        v.type = CAPSMI_I64;
        v.data = vals;
        r->cols.push_back(std::move(v));
    }
    r->nrows = rows;
    r->partitioned = g_dist.on && g_dist.world > 1;  // the rows of this rank's owned start nodes
    *out = guard.release();
    route(s, "two_hop_grouped");
    return true;
}

// The var-length grouped count over BY_SOURCE shards: this rank owns the
// start ids [rank * span, (rank + 1) * span) and holds their out-relationships (`views`) plus the
// relationships into its owned ids from other ranks (the bases' in-shards, exchanged at registration).
// begin (owned od, reverse multiplicities) -> all-reduce od -> mid (owned Y) -> all-reduce Y -> finish:
// the (relative dense id, count) rows of the owned start nodes.
void dist_var_length(capsmi_session* s, const std::vector<capsmi_table*>& views,
                     const std::vector<const capsmi_table*>& bases, const capsmi_bitmap* a, const capsmi_bitmap* b,
                     int lower, int upper, const std::string& id_name, const std::string& count_name,
                     capsmi_table** out) {
    std::vector<const int64_t*> srcs, dsts, isrcs, idsts;
    std::vector<int64_t> ms, ims;
    for (capsmi_table* t : views) {
        srcs.push_back(t->cols[0].d());
        dsts.push_back(t->cols[1].d());
        ms.push_back(t->nrows);
    }
    for (const capsmi_table* t : bases) {
        if (t->in_rows <= 0) continue;
        isrcs.push_back(t->in_src.d());
        idsts.push_back(t->in_dst.d());
        ims.push_back(t->in_rows);
    }
    const int64_t n = b->hi - b->lo, span = 32 * g_dist.slice_words;
    const int64_t own_lo = std::min<int64_t>(g_dist.rank * span, n), own_hi = std::min<int64_t>(own_lo + span, n);
    Buf od = dev_alloc(sizeof(int64_t) * n, s), y = dev_alloc(sizeof(int64_t) * n, s);
    VarlenShard* v = varlen_shard_begin(s, srcs.data(), dsts.data(), ms.data(), (int)srcs.size(), isrcs.data(),
                                        idsts.data(), ims.data(), (int)isrcs.size(), a, b, lower, upper, own_lo + b->lo,
                                        own_hi + b->lo, P<int64_t>(od));
    std::unique_ptr<VarlenShard, void (*)(VarlenShard*)> hold(v, varlen_shard_free);
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(od), P<int64_t>(od), n, CAPSMI_I64);
    varlen_shard_mid(v, P<int64_t>(y));
    collective(s, CAPSMI_COLL_ALL_REDUCE_SUM, P<int64_t>(y), P<int64_t>(y), n, CAPSMI_I64);
    Buf ids, cnt;
    const int64_t rows = varlen_shard_finish(v, ids, cnt);
    auto* r = result_table(s, rows);
    Column ic, cc;
    ic.name = id_name;
    ic.type = CAPSMI_I64;
    ic.data = ids;
    cc.name = count_name;
    cc.type = CAPSMI_I64;
    cc.data = cnt;
    r->cols.push_back(std::move(ic));
    r->cols.push_back(std::move(cc));
    *out = r;
}

// group by the start node, count(*), over the branches of a bounded var-length expand
bool fused_var_length(capsmi_session* s, const capsmi_table* in, const PlanNode& g, const std::vector<Path>& B,
                      capsmi_table** out) {
    if (g.a.size() != 1 || g.aggs.size() != 1) return false;
    const AggSpec& ag = g.aggs[0];
    const int gc = find_col(in, g.a[0]);
    if (gc < 0) return false;
    std::set<int> lens;
    std::string akey, bkey, rsig;
    int64_t lo, hi;
    if (!id_window(B, &lo, &hi)) return false;
    // the sharded count needs every owned source's out-relationships (BY_SOURCE shards); decided before any
    // node scan, whose gathers would otherwise run for nothing
    if (g_dist.on && g_dist.rel_mode != CAPSMI_RELS_BY_SOURCE) return false;
    BitmapSet bs;
    capsmi_bitmap *abm = nullptr, *bbm = nullptr;
    RelViews views;
    std::vector<const capsmi_table*> bases;  // the relationship tables behind `views` (their in-shards)
    std::string zero_key;  // the zero-length branch's start scan (lower = 0)
    bool first = true;
    for (size_t bi = 0; bi < B.size(); ++bi) {
        const Path& P = B[bi];
        if (any_no_loops(P)) return false;
        const int k = (int)P.hops.size();
        if (k == 0) {
            // lower = 0: copyEntity(source -> target) of the start scan (VarLengthExpandPlanner.scala:146-153,
            // 190-210) -- one row per scanned start node, whatever the target's labels; count(*) only
            if (lens.count(0) || ag.kind != CAPSMI_AGG_COUNT_STAR || P.pos_node.empty() || P.pos_node[0] < 0) return false;
            if (position_of(P, P.cols[gc]) != 0 || !id_like(P, P.cols[gc])) return false;
            Classified c;
            if (!classify(P, c) || !c.uniq.empty()) return false;
            for (size_t q = 0; q < P.inst.size(); ++q)
                if (!c.pred[q].empty() && (int)q != P.pos_node[0]) return false;
            if (!node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs, &zero_key)) return false;
            lens.insert(0);
            continue;
        }
        if (k < 1 || !is_chain(P) || !same_orientation(P) || lens.count(k)) return false;
        lens.insert(k);
        for (int q = 1; q < k; ++q) if (P.pos_node[q] >= 0) return false;  // hops are not node-scanned
        if (P.pos_node[0] < 0 || P.pos_node[k] < 0) return false;
        if (position_of(P, P.cols[gc]) != 0 || !id_like(P, P.cols[gc])) return false;
        if (ag.kind == CAPSMI_AGG_COUNT) {
            const int c = find_col(in, ag.input);
            if (ag.distinct || c < 0 || !id_like(P, P.cols[c])) return false;
        } else if (ag.kind != CAPSMI_AGG_COUNT_STAR) {
            return false;
        }
        Classified c;
        if (!classify(P, c) || !all_pairs_unique(c, k)) return false;
        for (size_t q = 0; q < P.inst.size(); ++q)
            if (!c.pred[q].empty() && (int)q != P.pos_node[0] && (int)q != P.pos_node[k]) return false;
        std::string ka, kb;
        capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs, &ka);
        capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[k], lo, hi, bs, &kb);
        if (!a || !b) return false;
        for (int h = 0; h < k; ++h) {
            if (g_dist.on && P.hops[h].from_role != ROLE_SRC) return false;  // outgoing over BY_SOURCE shards
            RelViews v;
            rel_views(P, P.hops[h], v);
            if (first && h == 0) {
                rsig = v.sig;
                views.t.swap(v.t);
                for (const Member& m : P.inst[P.hops[h].rel].m) bases.push_back(m.base);
            } else if (v.sig != rsig) {
                return false;
            }
        }
        if (first) { akey = ka; bkey = kb; abm = a; bbm = b; first = false; }
        else if (ka != akey || kb != bkey) return false;
    }
    if (first || (lens.count(0) && zero_key != akey)) return false;  // a path of >= 1 hop; one start scan
    const int l = *lens.begin(), u = *lens.rbegin();
    // upper 4 on one device (var_length4, ids below 2^24 - 1); the sharded form stops at 3
    if (l < 0 || u > (g_dist.on ? 3 : 4) || u - l + 1 != (int)lens.size()) return false;
    if (u == 4 && hi - lo >= (int64_t(1) << 24) - 1) return false;
    if (g_dist.on) dist_var_length(s, views.t, bases, abm, bbm, l, u, g.a[0], ag.output, out);
    else
        check(capsmi_var_length_count(s, (int32_t)views.t.size(), views.t.data(), "s", "t", abm, bbm, l, u,
                                      g.a[0].c_str(), ag.output.c_str(), out));
    if (g_dense) {  // start ids back to the graph's Long ids
        capsmi_table* r = *out;
        Column& c = r->cols[0];
        Buf ids = dev_alloc(sizeof(int64_t) * (r->nrows > 0 ? r->nrows : 1), s);
        if (g_dense->scrambled) {
            if (r->nrows)
                HIP_CHECK(hipMemcpyAsync(::capsmi::P<int64_t>(ids), c.d(), sizeof(int64_t) * r->nrows,
                                         hipMemcpyDeviceToDevice, s->stream));
            unscramble_ids(s, *g_dense, ::capsmi::P<int64_t>(ids), r->nrows);
        } else {
            gather_col(P<int64_t>(g_dense->orig), nullptr, c.d(), r->nrows, ::capsmi::P<int64_t>(ids), nullptr, s->stream);
        }
        c.data = ids;
        c.offset = 0;
        c.host.reset();
    }
    (*out)->partitioned = g_dist.on && g_dist.world > 1;  // the rows of this rank's owned start nodes
    route(s, "var_length");
    return true;
}

// Expand + node filters projected on relationship / endpoint columns (C2)
bool fused_projection(capsmi_session* s, const capsmi_table* t, const std::vector<Path>& B, capsmi_table** out) {
    if (B.size() != 1) return false;
    const Path& P = B[0];
    if (P.hops.size() != 1 || !is_chain(P) || P.pos_node[0] < 0 || P.pos_node[1] < 0 || any_no_loops(P)) return false;
    Classified c;
    if (!classify(P, c) || !c.uniq.empty()) return false;
    const Hop& h = P.hops[0];
    const Scan& R = P.inst[h.rel];
    // output column -> (relationship scan column | endpoint role | constant)
    std::vector<int> rcol(P.cols.size(), -1), endp(P.cols.size(), ROLE_NONE);
    int ndata = 0;
    for (size_t i = 0; i < P.cols.size(); ++i) {
        const Role& r = P.cols[i];
        if (r.k == RK_CONST) continue;
        if (r.k == RK_REL && r.inst == h.rel) { rcol[i] = r.scol; ++ndata; continue; }
        const int pos = position_of(P, r);
        if (r.k == RK_NODE && pos == 0) { endp[i] = h.from_role; ++ndata; continue; }
        if (r.k == RK_NODE && pos == 1) { endp[i] = h.to_role; ++ndata; continue; }
        return false;  // node properties / labels: joined in the generic plan
    }
    if (ndata > 4) return false;
    std::vector<Path> one{P};
    int64_t lo, hi;
    if (!id_window(one, &lo, &hi)) return false;
    BitmapSet bs;
    capsmi_bitmap* a = node_bitmap(s, P, c, P.pos_node[0], lo, hi, bs);
    capsmi_bitmap* b = node_bitmap(s, P, c, P.pos_node[1], lo, hi, bs);
    if (!a || !b) return false;
    std::vector<capsmi_table*> parts;
    struct Release { std::vector<capsmi_table*>& v; ~Release() { for (auto* x : v) capsmi_table_release(x); } } rel{parts};
    for (const Member& m : R.m) {
        const EntityInfo& e = *m.base->entity;
        const int fc = h.from_role == ROLE_SRC ? e.src : e.dst, tc = h.to_role == ROLE_SRC ? e.src : e.dst;
        std::vector<const char*> ocols, onames;
        std::vector<std::string> tmpn;
        for (size_t i = 0; i < P.cols.size(); ++i) tmpn.push_back("c" + std::to_string(i));
        bool const_member = false;
        for (size_t i = 0; i < P.cols.size(); ++i) {
            int bc = -1;
            if (rcol[i] >= 0) bc = m.src[rcol[i]];
            else if (endp[i] != ROLE_NONE) bc = endp[i] == ROLE_SRC ? e.src : e.dst;
            else continue;
            if (bc < 0) { const_member = true; break; }  // a per-table constant in a relationship column
            ocols.push_back(m.base->cols[bc].name.c_str());
            onames.push_back(tmpn[i].c_str());
        }
        if (const_member) return false;
        const char* any[1] = {m.base->cols[fc].name.c_str()};
        const char* anyn[1] = {"c_"};
        capsmi_table* o = nullptr;
        // node tests on the (dense) endpoint columns, projections of the original columns
        capsmi_table* tab = g_dense ? dense_view(m.base) : m.base;
        const char* tf = g_dense ? (h.from_role == ROLE_SRC ? "__dense_src" : "__dense_dst") : m.base->cols[fc].name.c_str();
        const char* tt = g_dense ? (h.to_role == ROLE_SRC ? "__dense_src" : "__dense_dst") : m.base->cols[tc].name.c_str();
        capsmi_status st;
        if (ocols.empty()) st = capsmi_expand_filter(s, tab, tf, tt, a, b, 1, any, anyn, &o);
        else st = capsmi_expand_filter(s, tab, tf, tt, a, b, (int32_t)ocols.size(), ocols.data(), onames.data(), &o);
        if (g_dense) capsmi_table_release(tab);
        check(st);
        parts.push_back(o);
    }
    // assemble the output schema: data columns from the kernel, constants filled
    capsmi_table* acc = nullptr;
    for (capsmi_table* part : parts) {
        auto* r = result_table(s, part->nrows);
        for (size_t i = 0; i < P.cols.size(); ++i) {
            Column col;
            const int j = find_col(part, "c" + std::to_string(i));
            if (j >= 0) {
                col = part->cols[j];
            } else {
                const capsmi_expr& x = P.cols[i].cst;
                col.type = t->cols[i].type;
                col.data = dev_alloc(sizeof(int64_t) * (part->nrows > 0 ? part->nrows : 1), s);
                fill_i64(::capsmi::P<int64_t>(col.data), x.op == CAPSMI_X_LIT ? x.ival : 0, part->nrows, s->stream);
                if (x.op == CAPSMI_X_NULL || t->cols[i].nullable()) {
                    col.valid = dev_alloc(part->nrows > 0 ? part->nrows : 1, s);
                    fill_u8(::capsmi::P<uint8_t>(col.valid), x.op == CAPSMI_X_NULL ? 0 : 1, part->nrows, s->stream);
                }
            }
            col.name = t->cols[i].name;
            r->cols.push_back(col);
        }
        if (!acc) {
            acc = r;
        } else {
            capsmi_table* u = nullptr;
            const capsmi_status st = eager_union_all(acc, r, &u);
            capsmi_table_release(acc);
            capsmi_table_release(r);
            check(st);
            acc = u;
        }
    }
    acc->partitioned = g_dist.on;  // this rank's relationships' rows
    *out = acc;
    route(s, "expand");
    return true;
}

// try the fused shapes for lazy table `t`; on success *out is its materialised content
bool try_fused_shapes(capsmi_table* t, capsmi_table** out);

bool has_hop(const std::vector<Path>& B) {
    for (const Path& P : B) if (!P.hops.empty()) return true;
    return false;
}

// a plan over entity tables in a pattern shape that no fused route took: counted once per
// materialisation as route "miss" (capsmi_session_route_count)
bool try_fused(capsmi_table* t, capsmi_table** out) {
    if (try_fused_shapes(t, out)) return true;
    const PlanNode& p = *t->plan;
    std::vector<Path> B;
    if (as_paths(p.kind == PlanNode::GROUP ? p.in[0] : t, B) && has_hop(B)) g_missed = true;
    return false;
}

bool try_fused_shapes(capsmi_table* t, capsmi_table** out) {
    capsmi_session* s = t->sess;
    if (!s->fused) return false;
    const PlanNode& p = *t->plan;
    if (p.kind == PlanNode::GROUP) {
        const capsmi_table* in = p.in[0];
        std::vector<Path> B;
        if (!as_paths(in, B) || B.empty()) return false;
        if (p.a.empty()) {
            if (B.size() != 1) {
                std::vector<int64_t> vals;
                if (!fused_undirected(s, in, p, B, vals)) return false;
                auto* r = result_table(s, 1);
                for (size_t i = 0; i < vals.size(); ++i) {
                    Column c = i64_column(s, {vals[i]});
                    c.name = p.aggs[i].output;
                    r->cols.push_back(std::move(c));
                }
                *out = r;
                return true;
            }
            std::vector<int> kinds;
            const int end = (int)B[0].pos_node.size() - 1;
            if (!agg_kinds(in, p, B[0], 0, B[0].hops.size() == 3 ? 0 : end, kinds)) return false;
            std::vector<int64_t> vals;
            if (!fused_counts(s, B[0], kinds, vals)) return false;
            auto* r = result_table(s, 1);
            for (size_t i = 0; i < vals.size(); ++i) {
                Column c = i64_column(s, {vals[i]});
                c.name = p.aggs[i].output;
                r->cols.push_back(std::move(c));
            }
            *out = r;
            return true;
        }
        if (fused_grouped_two_hop(s, in, p, B, out)) return true;
        return fused_var_length(s, in, p, B, out);
    }
    std::vector<Path> B;
    if (!as_paths(t, B)) return false;
    return fused_projection(s, t, B, out);
}

}  // namespace

void attach_entity(capsmi_table* t, int kind, int64_t lo, int64_t hi, bool ids_exact, bool ids_unique) {
    auto e = std::make_shared<EntityInfo>();
    e->kind = kind;
    e->id = 0;
    if (kind == 2) {
        e->src = 1;
        e->dst = 2;
    }
    e->rows = t->nrows;
    e->lo = lo;
    e->hi = hi;
    e->ids_exact = ids_exact;
    e->ids_unique = ids_exact || ids_unique;
    t->entity = e;
}

// ============================ operator-by-operator execution, pruned ========================
// What Catalyst does to the DataFrame plan DataFrameTable builds before Spark runs it (the optimiser
// rules ColumnPruning and PushDownPredicate / PushPredicateThroughJoin): a plan that is not routed
// to a fused kernel executes with
//   - every Filter split into its conjuncts, each pushed below Select / Drop / WithColumnRenamed /
//     WithColumns (when it does not read a column they add) and into the side of a Join whose columns
//     it reads (inner and cross: either side; one-sided outer: the preserved side only), and applied
//     where it stops -- with the rows of only the columns still needed gathered;
//   - only the columns some operator above still reads computed and gathered (join outputs, filters,
//     WithColumns expressions nobody reads are skipped).
// Results are the same rows (conjunct order does not change a TRUE / not-TRUE filter under 3VL);
// columns are matched by name, and put back in schema order where position matters (union inputs,
// the materialised table).
// A sub-plan with two parents in the plan DAG is materialised once in place and shared.
namespace {

using Names = std::vector<std::string>;  // ordered, unique column names

bool has(const Names& v, const std::string& x) { return std::find(v.begin(), v.end(), x) != v.end(); }
void add(Names& v, const std::string& x) {
    if (!has(v, x)) v.push_back(x);
}

struct Pred {                     // one conjunct; COL args index `names`
    std::vector<capsmi_expr> prog;
    Names names;
};

// first node of the complete sub-expression that ends at prog[end] (postfix)
int subtree_start(const std::vector<capsmi_expr>& prog, int end) {
    int want = 1;
    for (int i = end; i >= 0; --i) {
        want += arity(prog[i]) - 1;
        if (want == 0) return i;
    }
    throw Error(CAPSMI_ERR_INTERNAL, "malformed expression program");
}

void conjuncts(const std::vector<capsmi_expr>& prog, int lo, int hi, std::vector<std::vector<capsmi_expr>>& out) {
    if (prog[hi].op == CAPSMI_X_AND) {
        std::vector<std::pair<int, int>> kids;
        int end = hi - 1;
        for (int k = 0; k < prog[hi].arg; ++k) {
            const int st = subtree_start(prog, end);
            kids.push_back({st, end});
            end = st - 1;
        }
        for (auto it = kids.rbegin(); it != kids.rend(); ++it) conjuncts(prog, it->first, it->second, out);
    } else {
        out.emplace_back(prog.begin() + lo, prog.begin() + hi + 1);
    }
}

Pred to_pred(const std::vector<capsmi_expr>& prog, const capsmi_table* schema) {
    Pred p;
    p.prog = prog;
    for (capsmi_expr& x : p.prog)
        if (x.op == CAPSMI_X_COL) {
            const std::string& n = schema->cols.at(x.arg).name;
            add(p.names, n);
            x.arg = (int32_t)(std::find(p.names.begin(), p.names.end(), n) - p.names.begin());
        }
    return p;
}

// a program over `from`'s columns re-indexed against `to` (by name)
std::vector<capsmi_expr> remap(std::vector<capsmi_expr> prog, const capsmi_table* from, const capsmi_table* to) {
    for (capsmi_expr& x : prog)
        if (x.op == CAPSMI_X_COL) x.arg = col_of(to, from->cols.at(x.arg).name.c_str());
    return prog;
}

struct Res {  // an operator's result: a table this executor owns, or a borrowed materialised input
    capsmi_table* t = nullptr;
    bool owned = false;
    Res() = default;
    Res(capsmi_table* x, bool o) : t(x), owned(o) {}
    Res(Res&& o) noexcept : t(o.t), owned(o.owned) { o.t = nullptr; }
    Res& operator=(Res&& o) noexcept {
        if (this != &o) {
            reset();
            t = o.t;
            owned = o.owned;
            o.t = nullptr;
        }
        return *this;
    }
    ~Res() { reset(); }
    void reset() {
        if (t && owned) capsmi_table_release(t);
        t = nullptr;
    }
};

Res owned(capsmi_table* t) { return Res(t, true); }

// apply the pending conjuncts, keep exactly `need` (in the table's order)
Res finish(Res r, const Names& need, const std::vector<Pred>& preds) {
    Names keep;
    for (const Column& c : r.t->cols)
        if (has(need, c.name)) keep.push_back(c.name);
    REQUIRE(keep.size() == need.size(), CAPSMI_ERR_INTERNAL, "pruned plan lost a column");
    capsmi_table* o = nullptr;
    if (!preds.empty()) {
        std::vector<capsmi_expr> prog;
        for (const Pred& p : preds)
            for (capsmi_expr x : p.prog) {
                if (x.op == CAPSMI_X_COL) x.arg = col_of(r.t, p.names.at(x.arg).c_str());
                prog.push_back(x);
            }
        if (preds.size() > 1) {
            capsmi_expr a{};
            a.op = CAPSMI_X_AND;
            a.arg = (int32_t)preds.size();
            prog.push_back(a);
        }
        check(eager_filter_keep(r.t, (int32_t)prog.size(), prog.data(), keep, &o));
        o->partitioned = r.t->partitioned;
        return owned(o);
    }
    if (keep.size() == r.t->cols.size()) return r;
    auto c = cstrs(keep);
    check(eager_select(r.t, (int32_t)c.size(), c.data(), &o));
    o->partitioned = r.t->partitioned;
    return owned(o);
}

// ---- Exchanges of the generic operators over a distributed result ------------------------------------
// A row-local operator keeps its input's partitioning.  An operator that needs rows of other ranks gets
// the Exchange Spark's planner would insert (SparkTable.scala:133 groupBy, :226 join; CAPSSession.scala:
// 118-119 partitions), built on the session's collective (k_dist.hip exchange_rows):
//   join: a broadcast join when one side is whole on every rank and the partitioned side is the one whose
//     rows the join type preserves (inner, cross, left outer with the left partitioned, right outer with the
//     right partitioned); else both sides hash-partitioned on the join keys (a whole side first takes its
//     slice; rows with a null key stay where they are: they match nothing).  The result is partitioned.
//   grouping with keys, distinct: hash-partitioned on the grouping / distinct columns (nulls form one
//     group), then the local operator: the result is partitioned (each group on one rank).
//   a global aggregate, order by, skip, limit: every rank's rows gathered (all-gather), then the local
//     operator: the result is whole on every rank.
//   union all of a partitioned and a whole input: the whole one takes its slice.
// String keys hash their dictionary codes: the ranks of a distributed graph share one dictionary (the same
// ingest on every rank, as the JVM shim's session-wide dictionary).
Res owned(capsmi_table* t);

std::vector<int> key_indices(const capsmi_table* t, const Names& cols) {
    std::vector<int> k;
    for (const std::string& c : cols) k.push_back(col_of(t, c.c_str()));
    return k;
}

// join inputs made co-partitioned (see above); false when neither side is partitioned
bool dist_join_inputs(capsmi_session* s, int jt, const Names& lk, const Names& rk, Res& a, Res& b) {
    const bool pa = a.t->partitioned, pb = b.t->partitioned;
    if (!pa && !pb) return false;
    if (jt == CAPSMI_JOIN_CROSS) {
        if (pa && pb) b = owned(gather_rows(s, b.t));  // broadcast the right side
        return true;
    }
    if ((jt == CAPSMI_JOIN_INNER && (!pa || !pb)) || (jt == CAPSMI_JOIN_LEFT_OUTER && pa && !pb) ||
        (jt == CAPSMI_JOIN_RIGHT_OUTER && !pa && pb))
        return true;  // broadcast join: the whole side is on every rank
    if (!pa) a = owned(slice_rows(s, a.t));
    if (!pb) b = owned(slice_rows(s, b.t));
    const std::vector<int> li = key_indices(a.t, lk), ri = key_indices(b.t, rk);
    std::vector<int> lf(li.size(), 0), rf(ri.size(), 0);
    for (size_t i = 0; i < li.size(); ++i) {  // a Long key joined with a Double key hashes as the double
        const int32_t x = a.t->cols[li[i]].type, y = b.t->cols[ri[i]].type;
        if (x == CAPSMI_F64 || y == CAPSMI_F64) {
            lf[i] = x == CAPSMI_F64 ? 2 : 1;
            rf[i] = y == CAPSMI_F64 ? 2 : 1;
        }
    }
    a = owned(exchange_by_keys(s, a.t, li, lf, true));
    b = owned(exchange_by_keys(s, b.t, ri, rf, true));
    return true;
}

// ---- unrouted-plan size guard (capsmi_session_set_unrouted_limit) ------------------------------------
// System-R estimates of a lazy plan's rows: a join emits |L| |R| / max(ndv(l), ndv(r)) rows, where the
// ndv of an entity key column is its scan's rows (node ids) or min(rows, id window) (endpoints).
double key_ndv(const capsmi_table* t, const std::string& col) {  // -1: not known (not an entity key)
    Scan sc;
    const int c = find_col(t, col);
    if (c < 0 || !as_scan(t, sc)) return -1;
    double n = 0, span = 0;
    for (const Member& m : sc.m) {
        n += (double)m.base->nrows;
        span = std::max(span, (double)(m.base->entity->hi - m.base->entity->lo));
    }
    if (sc.role[c] == ROLE_ID) return std::max(1.0, n);
    if (sc.role[c] == ROLE_SRC || sc.role[c] == ROLE_DST) return std::max(1.0, std::min(n, span));
    return -1;
}

double est_rows(const capsmi_table* t) {
    if (!t->lazy()) return (double)t->nrows;
    const PlanNode& p = *t->plan;
    switch (p.kind) {
        case PlanNode::UNION: return est_rows(p.in[0]) + est_rows(p.in[1]);
        case PlanNode::SKIP: return std::max(0.0, est_rows(p.in[0]) - (double)p.n);
        case PlanNode::LIMIT: return std::min((double)p.n, est_rows(p.in[0]));
        case PlanNode::JOIN: {
            const double l = est_rows(p.in[0]), r = est_rows(p.in[1]);
            if (p.jt == CAPSMI_JOIN_CROSS) return l * r;
            double ndv = -1;  // the larger known key cardinality (an intermediate result's keys: unknown)
            for (size_t i = 0; i < p.a.size(); ++i)
                ndv = std::max(ndv, std::max(key_ndv(p.in[0], p.a[i]), key_ndv(p.in[1], p.b[i])));
            if (ndv < 1) ndv = std::max(1.0, std::max(l, r));
            double e = l * r / ndv;
            if (p.jt == CAPSMI_JOIN_LEFT_OUTER || p.jt == CAPSMI_JOIN_FULL_OUTER) e = std::max(e, l);
            if (p.jt == CAPSMI_JOIN_RIGHT_OUTER || p.jt == CAPSMI_JOIN_FULL_OUTER) e = std::max(e, r);
            return e;
        }
        default: return est_rows(p.in[0]);
    }
}

void guard_join(const capsmi_table* t) {
    const int64_t limit = t->sess->unrouted_limit;
    if (limit <= 0) return;
    const double bytes = est_rows(t) * (double)t->cols.size() * 9.0;  // 8-B words + validity bytes
    REQUIRE(bytes <= (double)limit, CAPSMI_ERR_UNSUPPORTED,
            "unrouted join estimated at " + std::to_string((long long)(bytes / 1e9)) + " GB (" +
                std::to_string((long long)est_rows(t)) + " rows) exceeds the session limit of " +
                std::to_string((long long)(limit / 1000000000LL)) + " GB; no fused route matched this pattern");
}

using Parents = std::map<const capsmi_table*, int>;

void count_parents(const capsmi_table* t, Parents& par) {
    if (!t->lazy()) return;
    for (const capsmi_table* x : t->plan->in)
        if (++par[x] == 1) count_parents(x, par);
}

Names all_names(const capsmi_table* t) {
    Names v;
    for (const Column& c : t->cols) v.push_back(c.name);
    return v;
}

Res exec(capsmi_table* t, const Names& need, std::vector<Pred> preds, const Parents& par) {
    if (t->lazy()) {
        auto it = par.find(t);
        if (it != par.end() && it->second > 1) materialize(t);  // shared sub-plan: once, in place
    }
    if (!t->lazy()) return finish(Res(t, false), need, preds);
    capsmi_table* fr = nullptr;
    if (try_fused(t, &fr)) {
        REQUIRE(fr->cols.size() == t->cols.size(), CAPSMI_ERR_INTERNAL, "fused result schema differs from the plan's");
        for (size_t i = 0; i < fr->cols.size(); ++i) fr->cols[i].name = t->cols[i].name;
        return finish(owned(fr), need, preds);
    }
    std::shared_ptr<PlanNode> keep_alive = t->plan;
    const PlanNode& p = *keep_alive;
    capsmi_table* x = p.in.empty() ? nullptr : p.in[0];
    switch (p.kind) {
        case PlanNode::FILTER: {
            std::vector<std::vector<capsmi_expr>> cs;
            if (!p.progs[0].empty()) conjuncts(p.progs[0], 0, (int)p.progs[0].size() - 1, cs);
            for (auto& c : cs) preds.push_back(to_pred(c, x));
            return exec(x, need, std::move(preds), par);
        }
        case PlanNode::SELECT:
        case PlanNode::DROP:
            return exec(x, need, std::move(preds), par);
        case PlanNode::RENAME: {
            const std::string &a = p.a[0], &b = p.b[0];
            if (a == b) return exec(x, need, std::move(preds), par);
            Names nin;
            for (const std::string& n : need) nin.push_back(n == b ? a : n);
            for (Pred& pr : preds)
                for (std::string& n : pr.names)
                    if (n == b) n = a;
            Res r = exec(x, nin, std::move(preds), par);
            if (r.t->find(a) < 0) return r;
            capsmi_table* o = nullptr;
            check(eager_with_column_renamed(r.t, a.c_str(), b.c_str(), &o));
            o->partitioned = r.t->partitioned;
            return owned(o);
        }
        case PlanNode::WITH_COLUMNS: {
            std::vector<Pred> down, stay;
            for (Pred& pr : preds) {
                bool reads_new = false;
                for (const std::string& n : pr.names) reads_new |= has(p.a, n);
                (reads_new ? stay : down).push_back(std::move(pr));
            }
            Names out = need;
            for (const Pred& pr : stay)
                for (const std::string& n : pr.names) add(out, n);
            Names nin;
            std::vector<size_t> comp;
            for (const std::string& n : out)
                if (!has(p.a, n)) add(nin, n);
            for (size_t i = 0; i < p.a.size(); ++i) {
                if (!has(out, p.a[i])) continue;  // nobody reads it
                comp.push_back(i);
                for (const capsmi_expr& e : p.progs[i])
                    if (e.op == CAPSMI_X_COL) add(nin, x->cols.at(e.arg).name);
            }
            Res r = exec(x, nin, std::move(down), par);
            if (!comp.empty()) {
                std::vector<std::vector<capsmi_expr>> progs;
                for (size_t i : comp) progs.push_back(remap(p.progs[i], x, r.t));
                std::vector<capsmi_expr_column> cols(comp.size());
                for (size_t k = 0; k < comp.size(); ++k) {
                    cols[k].name = p.a[comp[k]].c_str();
                    cols[k].nnodes = (int32_t)progs[k].size();
                    cols[k].prog = progs[k].data();
                }
                capsmi_table* o = nullptr;
                check(eager_with_columns(r.t, (int32_t)cols.size(), cols.data(), &o));
                o->partitioned = r.t->partitioned;
                r = owned(o);
            }
            return finish(std::move(r), need, stay);
        }
        case PlanNode::JOIN: {
            capsmi_table* y = p.in[1];
            const Names L = all_names(x), R = all_names(y);
            const bool cross = p.jt == CAPSMI_JOIN_CROSS;
            const bool to_l = p.jt == CAPSMI_JOIN_INNER || cross || p.jt == CAPSMI_JOIN_LEFT_OUTER;
            const bool to_r = p.jt == CAPSMI_JOIN_INNER || cross || p.jt == CAPSMI_JOIN_RIGHT_OUTER;
            std::vector<Pred> pl, pr, stay;
            for (Pred& q : preds) {
                bool in_l = true, in_r = true;
                for (const std::string& n : q.names) {
                    in_l &= has(L, n);
                    in_r &= has(R, n);
                }
                if (to_l && in_l) pl.push_back(std::move(q));
                else if (to_r && in_r) pr.push_back(std::move(q));
                else stay.push_back(std::move(q));
            }
            Names out = need;
            for (const Pred& q : stay)
                for (const std::string& n : q.names) add(out, n);
            Names nl, nr;
            for (const std::string& n : out) add(has(L, n) ? nl : nr, n);
            for (const std::string& n : p.a) add(nl, n);
            for (const std::string& n : p.b) add(nr, n);
            guard_join(t);
            Res a = exec(x, nl, std::move(pl), par);
            Res b = exec(y, nr, std::move(pr), par);
            const bool part = dist_join_inputs(t->sess, p.jt, p.a, p.b, a, b);
            auto lk = cstrs(p.a), rk = cstrs(p.b);
            capsmi_table* o = nullptr;
            check(eager_join(a.t, b.t, p.jt, (int32_t)lk.size(), lk.data(), rk.data(), &o));
            o->partitioned = part;
            a.reset();
            b.reset();
            return finish(owned(o), need, stay);
        }
        default: {  // union, distinct, grouping, ordering, skip / limit: conjuncts stay above
            std::vector<Names> nin(p.in.size());
            for (size_t i = 0; i < p.in.size(); ++i) nin[i] = all_names(p.in[i]);
            if (p.kind == PlanNode::GROUP) {
                Names v = p.a;
                for (const AggSpec& ag : p.aggs)
                    if (!ag.input.empty()) add(v, ag.input);
                nin[0] = v;
            } else if (p.kind == PlanNode::ORDER || p.kind == PlanNode::SKIP || p.kind == PlanNode::LIMIT) {
                Names v = need;
                for (const std::string& n : p.a) add(v, n);
                for (const Pred& q : preds)
                    for (const std::string& n : q.names) add(v, n);
                nin[0] = v;
            }
            PlanNode run;  // the same operator over the pruned inputs
            run.kind = p.kind;
            run.a = p.a;
            run.b = p.b;
            run.progs = p.progs;
            run.flags = p.flags;
            run.aggs = p.aggs;
            run.jt = p.jt;
            run.n = p.n;
            bool part = false;
            std::vector<Res> ins;
            for (size_t i = 0; i < p.in.size(); ++i) {
                Res r = exec(p.in[i], nin[i], {}, par);
                if (r.t->partitioned && p.kind != PlanNode::UNION) {  // the Exchange this operator needs
                    capsmi_session* ss = t->sess;
                    if ((p.kind == PlanNode::GROUP && !p.a.empty()) || p.kind == PlanNode::DISTINCT_ON) {
                        r = owned(exchange_by_keys(ss, r.t, key_indices(r.t, p.a), {}, false));
                    } else if (p.kind == PlanNode::DISTINCT) {
                        std::vector<int> all(r.t->cols.size());
                        for (size_t k = 0; k < all.size(); ++k) all[k] = (int)k;
                        r = owned(exchange_by_keys(ss, r.t, all, {}, false));
                    } else {  // global aggregate, order by, skip, limit: every rank's rows
                        r = owned(gather_rows(ss, r.t));
                    }
                }
                part = part || r.t->partitioned;
                if (p.kind == PlanNode::UNION) {  // positional: the input's schema order
                    capsmi_table* o = nullptr;
                    auto c = cstrs(nin[i]);
                    check(eager_select(r.t, (int32_t)c.size(), c.data(), &o));
                    o->partitioned = r.t->partitioned;
                    r = owned(o);
                }
                ins.push_back(std::move(r));
            }
            if (p.kind == PlanNode::UNION && part)  // a whole input joins a partitioned one by its slice
                for (Res& r : ins)
                    if (!r.t->partitioned) r = owned(slice_rows(t->sess, r.t));
            for (Res& r : ins) hold(run, r.t);
            ins.clear();
            capsmi_table* o = exec_node(run);
            o->partitioned = part;
            return finish(owned(o), need, preds);
        }
    }
    return Res();
}

}  // namespace

// ================================ materialisation ===========================================
void materialize(capsmi_table* t) {
    if (!t || !t->plan) return;
    std::shared_ptr<PlanNode> p = t->plan;  // inputs stay alive while this runs
    Parents par;
    count_parents(t, par);
    const Names all = all_names(t);
    Names uniq;
    for (const std::string& n : all) add(uniq, n);
    capsmi_table* r = nullptr;
    const bool outer_missed = g_missed;  // a shared sub-plan materialises inside another materialisation
    g_missed = false;
    int64_t routed_before = 0;
    for (auto& kv : t->sess->routes) routed_before += kv.first == "miss" ? 0 : kv.second;
    {
        Res e = exec(t, uniq, {}, par);
        auto c = cstrs(all);
        check(eager_select(e.t, (int32_t)c.size(), c.data(), &r));  // schema order, an owned table
        r->partitioned = e.t->partitioned;
    }
    int64_t routed_after = 0;
    for (auto& kv : t->sess->routes) routed_after += kv.first == "miss" ? 0 : kv.second;
    if (g_missed && routed_after == routed_before) t->sess->routes["miss"] += 1;  // a pattern ran unrouted
    g_missed = outer_missed;
    const bool part = r->partitioned;
    adopt(t, r);
    t->partitioned = part;
    t->plan.reset();  // the inputs are released unless shared elsewhere
}

}  // namespace capsmi

using namespace capsmi;

// ===================================== C ABI ====================================================
extern "C" {

static capsmi_status build(capsmi_table* t, capsmi_table** out, const std::function<capsmi_table*()>& f) {
    P_BEGIN
    need(t, "table");
    need(out, "out");
    *out = f();
    P_END
}

capsmi_status capsmi_cache(capsmi_table* t, capsmi_table** out) {
    // a table keeps its rows once computed (DataFrameTable.cache, SparkTable.scala:240-246): same handle;
    // a cached relationship table also keeps the fused layouts built from it
    return build(t, out, [&] {
        t->keep_layouts = true;
        t->refs.fetch_add(1);
        return t;
    });
}

capsmi_status capsmi_select(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    return build(t, out, [&] {
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::SELECT;
        hold(*p, t);
        std::vector<Column> sch;
        for (int i = 0; i < ncols; ++i) {
            sch.push_back(schema_of(t->cols[col_of(t, cols[i])]));
            p->a.push_back(cols[i]);
        }
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_drop(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    return build(t, out, [&] {
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::DROP;
        hold(*p, t);
        std::set<std::string> d;
        for (int i = 0; i < ncols; ++i) {
            need(cols[i], "column name");
            d.insert(cols[i]);  // Spark drop ignores unknown names
            p->a.push_back(cols[i]);
        }
        std::vector<Column> sch;
        for (auto& c : t->cols) if (!d.count(c.name)) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_with_column_renamed(capsmi_table* t, const char* old_name, const char* new_name, capsmi_table** out) {
    return build(t, out, [&] {
        need(new_name, "new name");
        const int i = col_of(t, old_name);
        const int j = find_col(t, new_name);
        REQUIRE(j < 0 || j == i, CAPSMI_ERR_ILLEGAL_ARGUMENT, std::string("column '") + new_name + "' already exists");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::RENAME;
        hold(*p, t);
        p->a = {old_name};
        p->b = {new_name};
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        sch[i].name = new_name;
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_filter(capsmi_table* t, int32_t nnodes, const capsmi_expr* prog, capsmi_table** out) {
    return build(t, out, [&] {
        REQUIRE(nnodes == 0 || prog, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null program");
        std::vector<capsmi_expr> bound;
        if (has_params(nnodes, prog)) {  // parameters become literals now, as in the Spark plan
            bound = bind_params(t->sess, nnodes, prog);
            prog = bound.data();
            nnodes = (int32_t)bound.size();
        }
        validate_program(t, nnodes, prog);
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::FILTER;
        hold(*p, t);
        p->progs.emplace_back(prog, prog + nnodes);
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_with_columns(capsmi_table* t, int32_t ncols, const capsmi_expr_column* cols, capsmi_table** out) {
    return build(t, out, [&] {
        REQUIRE(ncols == 0 || cols, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null columns");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::WITH_COLUMNS;
        hold(*p, t);
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        for (int i = 0; i < ncols; ++i) {
            need(cols[i].name, "column name");
            REQUIRE(cols[i].nnodes == 0 || cols[i].prog, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null program");
            std::vector<capsmi_expr> prog(cols[i].prog, cols[i].prog + cols[i].nnodes);
            if (has_params(cols[i].nnodes, cols[i].prog)) prog = bind_params(t->sess, cols[i].nnodes, cols[i].prog);
            validate_program(t, (int32_t)prog.size(), prog.data());
            p->a.push_back(cols[i].name);
            Column c = schema_col(cols[i].name, infer_type(t, (int32_t)prog.size(), prog.data()), true);
            p->progs.push_back(std::move(prog));
            int j = -1;
            for (size_t q = 0; q < sch.size(); ++q) if (sch[q].name == c.name) j = (int)q;
            if (j >= 0) sch[j] = c;  // replaced in place (SparkTable.scala:82-87)
            else sch.push_back(c);
        }
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_join(capsmi_table* l, capsmi_table* r, int32_t join_type, int32_t npairs, const char* const* lcols,
                          const char* const* rcols, capsmi_table** out) {
    return build(l, out, [&] {
        need(r, "right");
        REQUIRE(l->sess == r->sess, CAPSMI_ERR_ILLEGAL_ARGUMENT, "tables belong to different sessions");
        REQUIRE(join_type >= CAPSMI_JOIN_INNER && join_type <= CAPSMI_JOIN_CROSS, CAPSMI_ERR_ILLEGAL_ARGUMENT, "join type");
        REQUIRE(join_type == CAPSMI_JOIN_CROSS || npairs > 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "equi-join needs key pairs");
        for (const Column& a : l->cols)
            for (const Column& b : r->cols)
                REQUIRE(a.name != b.name, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                        "join inputs share column '" + a.name + "' (RelationalPlanner renames to disjoint columns)");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::JOIN;
        hold(*p, l);
        hold(*p, r);
        p->jt = join_type;
        if (join_type != CAPSMI_JOIN_CROSS) {
            REQUIRE(npairs <= 8, CAPSMI_ERR_NOT_IMPLEMENTED, "more than 8 key columns");
            for (int i = 0; i < npairs; ++i) {
                const int a = col_of(l, lcols[i]), b = col_of(r, rcols[i]);
                const int ta = l->cols[a].type, tb = r->cols[b].type;
                no_list_key(ta, l->cols[a].name, "a join key");
                no_list_key(tb, r->cols[b].name, "a join key");
                const bool na = ta == CAPSMI_I64 || ta == CAPSMI_F64, nb = tb == CAPSMI_I64 || tb == CAPSMI_F64;
                REQUIRE(ta == tb || (na && nb), CAPSMI_ERR_ILLEGAL_ARGUMENT,
                        "join key types differ: " + l->cols[a].name + " vs " + r->cols[b].name);
                p->a.push_back(lcols[i]);
                p->b.push_back(rcols[i]);
            }
        }
        const bool lmiss = join_type == CAPSMI_JOIN_RIGHT_OUTER || join_type == CAPSMI_JOIN_FULL_OUTER;
        const bool rmiss = join_type == CAPSMI_JOIN_LEFT_OUTER || join_type == CAPSMI_JOIN_FULL_OUTER;
        std::vector<Column> sch;
        for (auto& c : l->cols) sch.push_back(schema_col(c.name, c.type, c.nullable() || lmiss));
        for (auto& c : r->cols) sch.push_back(schema_col(c.name, c.type, c.nullable() || rmiss));
        return lazy_table(l->sess, p, sch);
    });
}

capsmi_status capsmi_union_all(capsmi_table* a, capsmi_table* b, capsmi_table** out) {
    return build(a, out, [&] {
        need(b, "right");
        REQUIRE(a->cols.size() == b->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "union all: column counts differ");
        std::vector<Column> sch;
        for (size_t i = 0; i < a->cols.size(); ++i) {
            REQUIRE(a->cols[i].type == b->cols[i].type, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    "Equal column data types for union all (differing nullability is OK): " + a->cols[i].name + " vs " +
                        b->cols[i].name);
            sch.push_back(schema_col(a->cols[i].name, a->cols[i].type, a->cols[i].nullable() || b->cols[i].nullable()));
        }
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::UNION;
        hold(*p, a);
        hold(*p, b);
        return lazy_table(a->sess, p, sch);
    });
}

capsmi_status capsmi_order_by(capsmi_table* t, int32_t nkeys, const char* const* cols, const int32_t* descending,
                              capsmi_table** out) {
    return build(t, out, [&] {
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::ORDER;
        hold(*p, t);
        for (int i = 0; i < nkeys; ++i) {
            const int c = col_of(t, cols[i]);
            no_list_key(t->cols[c].type, t->cols[c].name, "a sort key");
            p->a.push_back(cols[i]);
            p->flags.push_back(descending ? descending[i] : 0);
        }
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_skip(capsmi_table* t, int64_t n, capsmi_table** out) {
    return build(t, out, [&] {
        REQUIRE(n >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "negative skip");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::SKIP;
        hold(*p, t);
        p->n = n;
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_limit(capsmi_table* t, int64_t n, capsmi_table** out) {
    return build(t, out, [&] {
        REQUIRE(n >= 0 && n <= 2147483647LL, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "an integer: limit must fit an Int (SparkTable.scala:117)");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::LIMIT;
        hold(*p, t);
        p->n = n;
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_distinct(capsmi_table* t, capsmi_table** out) {
    return build(t, out, [&] {
        for (auto& c : t->cols) no_list_key(c.type, c.name, "a distinct key");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::DISTINCT;
        hold(*p, t);
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_distinct_on(capsmi_table* t, int32_t ncols, const char* const* cols, capsmi_table** out) {
    return build(t, out, [&] {
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::DISTINCT_ON;
        hold(*p, t);
        for (int i = 0; i < ncols; ++i) {
            const int c = col_of(t, cols[i]);
            no_list_key(t->cols[c].type, t->cols[c].name, "a distinct key");
            p->a.push_back(cols[i]);
        }
        std::vector<Column> sch;
        for (auto& c : t->cols) sch.push_back(schema_of(c));
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_group(capsmi_table* t, int32_t nby, const char* const* by, int32_t naggs, const capsmi_agg* aggs,
                           capsmi_table** out) {
    return build(t, out, [&] {
        REQUIRE(naggs == 0 || aggs, CAPSMI_ERR_ILLEGAL_ARGUMENT, "null aggregations");
        auto p = std::make_shared<PlanNode>();
        p->kind = PlanNode::GROUP;
        hold(*p, t);
        std::vector<Column> sch;
        for (int i = 0; i < nby; ++i) {
            const int c = col_of(t, by[i]);
            no_list_key(t->cols[c].type, t->cols[c].name, "a grouping key");
            p->a.push_back(by[i]);
            sch.push_back(schema_of(t->cols[c]));
        }
        for (int i = 0; i < naggs; ++i) {
            const capsmi_agg& ag = aggs[i];
            need(ag.output, "aggregate output name");
            AggSpec sp;
            sp.kind = ag.kind;
            sp.distinct = ag.distinct;
            sp.output = ag.output;
            int32_t ty = CAPSMI_I64;
            bool nullable = false;
            switch (ag.kind) {
                case CAPSMI_AGG_COUNT_STAR: break;
                case CAPSMI_AGG_COUNT: sp.input = t->cols[col_of(t, ag.input)].name; break;
                case CAPSMI_AGG_SUM: case CAPSMI_AGG_AVG: {
                    const Column& c = t->cols[col_of(t, ag.input)];
                    REQUIRE(c.type == CAPSMI_I64 || c.type == CAPSMI_F64, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                            ag.kind == CAPSMI_AGG_SUM ? "sum of non-number" : "avg of non-number");
                    sp.input = c.name;
                    ty = c.type;
                    nullable = true;
                    break;
                }
                case CAPSMI_AGG_MIN: case CAPSMI_AGG_MAX: {
                    const Column& c = t->cols[col_of(t, ag.input)];
                    no_list_key(c.type, c.name, "an aggregate input");
                    sp.input = c.name;
                    ty = c.type;
                    nullable = true;
                    break;
                }
                case CAPSMI_AGG_COLLECT: {  // sort_array(collect_list / collect_set), SparkTable.scala:169-177
                    const Column& c = t->cols[col_of(t, ag.input)];
                    no_list_key(c.type, c.name, "an aggregate input");
                    sp.input = c.name;
                    ty = CAPSMI_LIST + c.type;
                    break;
                }
                default: throw Error(CAPSMI_ERR_NOT_IMPLEMENTED, "Aggregation function " + std::to_string(ag.kind));
            }
            p->aggs.push_back(sp);
            sch.push_back(schema_col(ag.output, ty, nullable));
        }
        return lazy_table(t->sess, p, sch);
    });
}

capsmi_status capsmi_session_set_fused(capsmi_session* s, int32_t enabled) {
    P_BEGIN
    need(s, "session");
    s->fused = enabled != 0;
    P_END
}

capsmi_status capsmi_session_set_csv_partitioning(capsmi_session* s, int64_t default_parallelism,
                                                  int64_t max_partition_bytes, int64_t open_cost_bytes) {
    P_BEGIN
    need(s, "session");
    REQUIRE(default_parallelism >= 0 && max_partition_bytes > 0 && open_cost_bytes >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "csv partitioning: parallelism >= 0, max partition bytes > 0, open cost >= 0");
    s->csv_parallelism = default_parallelism;
    s->csv_max_partition_bytes = max_partition_bytes;
    s->csv_open_cost = open_cost_bytes;
    P_END
}

capsmi_status capsmi_session_set_unrouted_limit(capsmi_session* s, int64_t max_bytes) {
    P_BEGIN
    need(s, "session");
    REQUIRE(max_bytes >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "negative limit");
    s->unrouted_limit = max_bytes;
    P_END
}

capsmi_status capsmi_session_route_count(capsmi_session* s, const char* name, int64_t* count) {
    P_BEGIN
    need(s, "session");
    need(name, "name");
    need(count, "count");
    auto it = s->routes.find(name);
    *count = it == s->routes.end() ? 0 : it->second;
    P_END
}

// ---- entity tables ------------------------------------------------------------------------------
static void verify_key(const capsmi_table* t, const char* name, const char* what, int32_t type) {
    need(name, what);
    const int i = find_col(t, name);
    REQUIRE(i >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string("table with column key ") + name + " (EntityTable.verify: no such column)");
    const Column& c = t->cols[i];
    const char* tn = type == CAPSMI_I64 ? "CTInteger" : "CTBoolean";
    REQUIRE(c.type == type, CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string(what) + " column `" + name + "` of type " + tn + " (incompatible column type)");
    REQUIRE(!c.nullable(), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            std::string("non-nullable type for ") + what + " column `" + name + "` (nullable type)");
}

static capsmi_table* register_entity(capsmi_table* t, int kind, const std::vector<const char*>& keys,
                                     const std::vector<const char*>& flags) {
    // canonical order: keys ++ flags ++ properties sorted (EntityMapping.allSourceKeys, EntityMapping.scala:50)
    std::vector<std::string> want(keys.begin(), keys.end());
    want.insert(want.end(), flags.begin(), flags.end());
    std::set<std::string> fixed(want.begin(), want.end());
    REQUIRE(fixed.size() == want.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT, "One-to-one mapping from entity elements to source keys");
    std::vector<std::string> props;
    for (auto& c : t->cols) if (!fixed.count(c.name)) props.push_back(c.name);
    std::sort(props.begin(), props.end());
    want.insert(want.end(), props.begin(), props.end());
    bool ok = want.size() == t->cols.size();
    for (size_t i = 0; ok && i < want.size(); ++i) ok = t->cols[i].name == want[i];
    if (!ok) {
        std::string exp, got;
        for (auto& w : want) exp += (exp.empty() ? "" : ", ") + w;
        for (auto& c : t->cols) got += (got.empty() ? "" : ", ") + c.name;
        throw Error(CAPSMI_ERR_ILLEGAL_ARGUMENT, "Columns: " + exp + " expected, got Columns: " + got +
                                                     " (use CAPS[Node|Relationship]Table#fromMapping to create a valid "
                                                     "EntityTable)");
    }
    materialize(t);
    auto e = std::make_shared<EntityInfo>();
    e->kind = kind;
    e->id = 0;
    if (kind == 2) {
        e->src = 1;
        e->dst = 2;
    }
    e->rows = t->nrows;
    if (t->nrows > 0) {
        capsmi_session* s = t->sess;
        HIP_CHECK(hipSetDevice(s->device));
        int64_t mm[2];
        if (kind == 1) {
            const int64_t* c[1] = {t->cols[0].d()};
            minmax_i64(s, c, 1, t->nrows, mm);
        } else {
            const int64_t* c[2] = {t->cols[1].d(), t->cols[2].d()};
            minmax_i64(s, c, 2, t->nrows, mm);
        }
        e->lo = mm[0];
        e->hi = mm[1] == INT64_MAX ? INT64_MAX : mm[1] + 1;
        if (kind == 1 && mm[1] != INT64_MAX && e->hi - e->lo <= (int64_t(1) << 31) && !t->cols[0].valid) {
            // one bitmap pass over [min, max]: whether an id repeats (a node scan of a table without
            // repeats then needs no count read back, capsmi_bitmap_add_scan), and whether the ids are
            // exactly that window (as many rows as ids in it, none repeated)
            capsmi_bitmap* b = nullptr;
            check(capsmi_bitmap_create(s, e->lo, e->hi, &b));
            const capsmi_status st = capsmi_bitmap_add_scan(b, t, t->cols[0].name.c_str(), 0, nullptr);
            e->ids_unique = st == CAPSMI_OK && !b->any_dup;
            e->ids_exact = e->ids_unique && b->set_bits == t->nrows && e->hi - e->lo == t->nrows;
            capsmi_bitmap_release(b);
            check(st);
        }
    }
    auto* o = new capsmi_table();
    o->sess = t->sess;
    o->nrows = t->nrows;
    o->cols = t->cols;
    o->entity = e;
    return o;
}

capsmi_status capsmi_node_table(capsmi_table* t, const char* id_col, int32_t nlabels, const char* const* label_cols,
                                capsmi_table** out) {
    return build(t, out, [&] {
        verify_key(t, id_col, "id key", CAPSMI_I64);
        std::vector<const char*> flags;
        for (int i = 0; i < nlabels; ++i) {
            verify_key(t, label_cols[i], "optional label", CAPSMI_BOOL);
            flags.push_back(label_cols[i]);
        }
        return register_entity(t, 1, {id_col}, flags);
    });
}

capsmi_status capsmi_rel_table(capsmi_table* t, const char* id_col, const char* src_col, const char* dst_col,
                               int32_t ntypes, const char* const* type_cols, capsmi_table** out) {
    return build(t, out, [&] {
        verify_key(t, id_col, "id key", CAPSMI_I64);
        verify_key(t, src_col, "start node", CAPSMI_I64);
        verify_key(t, dst_col, "end node", CAPSMI_I64);
        std::vector<const char*> flags;
        for (int i = 0; i < ntypes; ++i) {
            verify_key(t, type_cols[i], "relationship type", CAPSMI_BOOL);
            flags.push_back(type_cols[i]);
        }
        return register_entity(t, 2, {id_col, src_col, dst_col}, flags);
    });
}

}  // extern "C"

namespace capsmi {
namespace {

__global__ void k_dense_of(const int64_t* __restrict__ slot_of_probe, const int64_t* __restrict__ slot_row,
                           const int64_t* __restrict__ gid_of_row, int64_t n, int64_t* __restrict__ out,
                           uint8_t* __restrict__ miss) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t sl = slot_of_probe[i];
        out[i] = sl >= 0 ? gid_of_row[slot_row[sl]] : -1;
        miss[i] = sl < 0;
    }
}

__global__ void k_place_dense(const int64_t* __restrict__ idx, const int64_t* __restrict__ gid, int64_t n, int64_t base,
                              int64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[idx[i]] = base + gid[i];
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 65536)); }

KeyCols one_key(const int64_t* d) {
    KeyCols k;
    k.n = 1;
    for (int i = 0; i < kMaxKeys; ++i) { k.data[i] = nullptr; k.valid[i] = nullptr; }
    k.data[0] = d;
    return k;
}

}  // namespace

void graph_compact(capsmi_session* s, const std::vector<capsmi_table*>& nodes, const std::vector<capsmi_table*>& rels,
                   int64_t* n_out) {
    hipStream_t st = s->stream;
    int64_t nn = 0;
    for (auto* t : nodes) nn += t->nrows;
    // node ids of every node table, one key column
    Buf keys = dev_alloc(sizeof(int64_t) * (nn > 0 ? nn : 1), s);
    int64_t off = 0;
    for (auto* t : nodes) {
        if (t->nrows) HIP_CHECK(hipMemcpyAsync(::capsmi::P<int64_t>(keys) + off, t->cols[t->entity->id].d(),
                                               sizeof(int64_t) * t->nrows, hipMemcpyDeviceToDevice, st));
        off += t->nrows;
    }
    const KeyCols kc = one_key(::capsmi::P<int64_t>(keys));
    HashTable ht;
    Buf sor, gid, rep;
    hash_build(s, kc, nn, false, ht, sor);
    const int64_t ng = nn > 0 ? hash_group_ids(s, ht, sor, nn, gid, rep) : 0;
    // endpoints: probe the node ids; endpoints of no node table (dangling) are numbered after them
    struct Miss { Buf idx; int64_t n; Buf dense; };
    std::vector<Miss> miss;
    std::vector<std::pair<Buf, Buf>> rel_dense;
    for (auto* t : rels) {
        const int64_t m = t->nrows;
        Buf d[2];
        for (int k = 0; k < 2; ++k) {
            const Column& c = t->cols[k == 0 ? t->entity->src : t->entity->dst];
            d[k] = dev_alloc(sizeof(int64_t) * (m > 0 ? m : 1), s);
            if (m == 0) continue;
            Buf sop, fl = dev_alloc(m, s);
            hash_probe(s, one_key(c.d()), kc, m, ht, sop);
            hipLaunchKernelGGL(k_dense_of, dim3(grid_of(m)), dim3(256), 0, st, ::capsmi::P<int64_t>(sop),
                               ::capsmi::P<int64_t>(ht.slot_row), ::capsmi::P<int64_t>(gid), m,
                               ::capsmi::P<int64_t>(d[k]), ::capsmi::P<uint8_t>(fl));
            HIP_CHECK(hipGetLastError());
            Miss x;
            x.n = flags_to_indices(s, ::capsmi::P<uint8_t>(fl), m, x.idx);
            x.dense = d[k];
            if (x.n > 0) {
                // remember the missing keys next to their row indices
                Buf mk = dev_alloc(sizeof(int64_t) * x.n, s);
                gather_col(c.d(), nullptr, ::capsmi::P<int64_t>(x.idx), x.n, ::capsmi::P<int64_t>(mk), nullptr, st);
                miss.push_back(x);
                miss.push_back(Miss{mk, -1, Buf()});  // keys of the entry before
            }
        }
        rel_dense.push_back({d[0], d[1]});
    }
    int64_t nm = 0;
    for (size_t i = 0; i < miss.size(); i += 2) nm += miss[i].n;
    Buf mkeys = dev_alloc(sizeof(int64_t) * (nm > 0 ? nm : 1), s);
    off = 0;
    for (size_t i = 0; i < miss.size(); i += 2) {
        HIP_CHECK(hipMemcpyAsync(::capsmi::P<int64_t>(mkeys) + off, ::capsmi::P<int64_t>(miss[i + 1].idx),
                                 sizeof(int64_t) * miss[i].n, hipMemcpyDeviceToDevice, st));
        off += miss[i].n;
    }
    int64_t ng2 = 0;
    Buf gid2, rep2;
    if (nm > 0) {
        HashTable h2;
        Buf sor2;
        hash_build(s, one_key(::capsmi::P<int64_t>(mkeys)), nm, false, h2, sor2);
        ng2 = hash_group_ids(s, h2, sor2, nm, gid2, rep2);
        off = 0;
        for (size_t i = 0; i < miss.size(); i += 2) {
            hipLaunchKernelGGL(k_place_dense, dim3(grid_of(miss[i].n)), dim3(256), 0, st, ::capsmi::P<int64_t>(miss[i].idx),
                               ::capsmi::P<int64_t>(gid2) + off, miss[i].n, ng, ::capsmi::P<int64_t>(miss[i].dense));
            off += miss[i].n;
        }
        HIP_CHECK(hipGetLastError());
    }
    auto D = std::make_shared<DenseIds>();
    D->n = ng + ng2;
    D->orig = dev_alloc(sizeof(int64_t) * (D->n > 0 ? D->n : 1), s);
    if (ng) gather_col(::capsmi::P<int64_t>(keys), nullptr, ::capsmi::P<int64_t>(rep), ng, ::capsmi::P<int64_t>(D->orig),
                       nullptr, st);
    if (ng2) gather_col(::capsmi::P<int64_t>(mkeys), nullptr, ::capsmi::P<int64_t>(rep2), ng2,
                        ::capsmi::P<int64_t>(D->orig) + ng, nullptr, st);
    off = 0;
    for (auto* t : nodes) {
        t->dense = D;
        t->did = Column();
        t->did.type = CAPSMI_I64;
        t->did.data = gid;
        t->did.offset = off;
        off += t->nrows;
    }
    for (size_t i = 0; i < rels.size(); ++i) {
        auto* t = rels[i];
        t->dense = D;
        t->dsrc = Column();
        t->dsrc.type = CAPSMI_I64;
        t->dsrc.data = rel_dense[i].first;
        t->ddst = Column();
        t->ddst.type = CAPSMI_I64;
        t->ddst.data = rel_dense[i].second;
    }
    HIP_CHECK(hipStreamSynchronize(st));
    *n_out = D->n;
}

}  // namespace capsmi

extern "C" {

capsmi_status capsmi_graph_compact(capsmi_session* s, int32_t nnodes, capsmi_table* const* nodes, int32_t nrels,
                                   capsmi_table* const* rels, int64_t* dense_ids) {
    P_BEGIN
    need(s, "session");
    REQUIRE(nnodes >= 0 && nrels >= 0 && (nnodes == 0 || nodes) && (nrels == 0 || rels), CAPSMI_ERR_ILLEGAL_ARGUMENT,
            "tables");
    HIP_CHECK(hipSetDevice(s->device));
    std::vector<capsmi_table*> nv, rv;
    for (int i = 0; i < nnodes; ++i) {
        need(nodes[i], "nodes[i]");
        REQUIRE(nodes[i]->entity && nodes[i]->entity->kind == 1 && nodes[i]->sess == s, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "graph_compact: nodes[i] is not a node table of this session (capsmi_node_table)");
        nv.push_back(nodes[i]);
    }
    for (int i = 0; i < nrels; ++i) {
        need(rels[i], "rels[i]");
        REQUIRE(rels[i]->entity && rels[i]->entity->kind == 2 && rels[i]->sess == s, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "graph_compact: rels[i] is not a relationship table of this session (capsmi_rel_table)");
        rv.push_back(rels[i]);
    }
    int64_t n = 0;
    graph_compact(s, nv, rv, &n);
    if (dense_ids) *dense_ids = n;
    P_END
}

capsmi_status capsmi_table_entity(const capsmi_table* t, int32_t* kind, int64_t* id_lo, int64_t* id_hi) {
    P_BEGIN
    need(t, "table");
    if (kind) *kind = t->entity ? t->entity->kind : 0;
    if (id_lo) *id_lo = t->entity ? t->entity->lo : 0;
    if (id_hi) *id_hi = t->entity ? t->entity->hi : 0;
    P_END
}

capsmi_status capsmi_flatten_rel_types(capsmi_table* t, const char* type_col, int32_t ntypes, const int64_t* type_codes,
                                       const char* const* out_cols, capsmi_table** out) {
    return build(t, out, [&] {
        const int tc = col_of(t, type_col);
        REQUIRE(t->cols[tc].type == CAPSMI_STR, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                std::string("relationship type column `") + type_col + "` of type CTString");
        REQUIRE(ntypes >= 0 && (ntypes == 0 || (type_codes && out_cols)), CAPSMI_ERR_ILLEGAL_ARGUMENT, "types");
        materialize(t);
        capsmi_session* s = t->sess;
        HIP_CHECK(hipSetDevice(s->device));
        auto* o = new capsmi_table();
        std::unique_ptr<capsmi_table> g(o);
        o->sess = s;
        o->nrows = t->nrows;
        for (size_t i = 0; i < t->cols.size(); ++i)
            if ((int)i != tc) o->cols.push_back(t->cols[i]);
        for (int k = 0; k < ntypes; ++k) {
            need(out_cols[k], "type column name");
            REQUIRE(find_col(o, out_cols[k]) < 0, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    std::string("column '") + out_cols[k] + "' already exists");
            // coalesce(type = code, false): a non-nullable flag (setNonNullable, CAPSTable.scala:198-200)
            capsmi_expr prog[5] = {};
            prog[0].op = CAPSMI_X_COL;
            prog[0].arg = tc;
            prog[1].op = CAPSMI_X_LIT;
            prog[1].type = CAPSMI_STR;
            prog[1].ival = type_codes[k];
            prog[2].op = CAPSMI_X_EQ;
            prog[3].op = CAPSMI_X_LIT;
            prog[3].type = CAPSMI_BOOL;
            prog[3].ival = 0;
            prog[4].op = CAPSMI_X_COALESCE;
            prog[4].arg = 2;
            Column c;
            c.name = out_cols[k];
            c.data = dev_alloc(sizeof(int64_t) * (t->nrows > 0 ? t->nrows : 1), s);
            eval_expr(s, t, 5, prog, P<int64_t>(c.data), nullptr, &c.type);
            c.type = CAPSMI_BOOL;
            o->cols.push_back(std::move(c));
        }
        return g.release();
    });
}

}  // extern "C"
