// k_expr.hip -- row-wise evaluation of postfix expression programs.
//
// Restates the predicate subset of SparkSQLExprMapper.asSparkSQLExpr
// (spark-cypher/src/main/scala/org/opencypher/spark/impl/SparkSQLExprMapper.scala:81-312)
// with Spark SQL three-valued logic:
//   - comparisons with a NULL operand are NULL; comparisons between incomparable
//     types (Long vs String, ...) are NULL (Spark casts the string and gets null);
//   - NOT NULL = NULL; AND: any FALSE -> FALSE, else any NULL -> NULL; OR dually;
//   - x IN (..): TRUE on a match, else NULL if x or any element is NULL, else FALSE;
//   - Filter keeps a row iff the value is TRUE (SparkTable.scala:65-67; pinned by
//     PredicateBehaviour.scala:131-149);
//   - bitwise and shift operators on Long (the id-tag expressions of Tags.scala:101-123), NULL in ->
//     NULL out; CASE takes the first alternative whose predicate is TRUE (a NULL predicate is not).
#include "capsmi_impl.h"

namespace capsmi {

namespace {

constexpr int kMaxStack = 32;
constexpr int kMaxCols = 64;
constexpr int8_t kNull = -1;

struct ColPtrs {
    const int64_t* data[kMaxCols];
    const uint8_t* valid[kMaxCols];
    int8_t type[kMaxCols];
};

struct Val {
    int64_t b;
    int8_t t;  // CAPSMI_* or kNull
};

__device__ __forceinline__ bool numeric(int8_t t) { return t == CAPSMI_I64 || t == CAPSMI_F64; }
__device__ __forceinline__ double as_f64(const Val& v) {
    return v.t == CAPSMI_F64 ? __longlong_as_double(v.b) : (double)v.b;
}

// -2: incomparable / null, else -1, 0, 1
__device__ __forceinline__ int cmp3(const Val& a, const Val& b) {
    if (a.t == kNull || b.t == kNull) return -2;
    if (numeric(a.t) && numeric(b.t)) {
        if (a.t == CAPSMI_I64 && b.t == CAPSMI_I64) return a.b < b.b ? -1 : (a.b > b.b ? 1 : 0);
        const double x = as_f64(a), y = as_f64(b);
        if (x != x || y != y) return -2;
        return x < y ? -1 : (x > y ? 1 : 0);
    }
    if (a.t != b.t) return -2;
    return a.b < b.b ? -1 : (a.b > b.b ? 1 : 0);
}

__device__ __forceinline__ Val mk_bool(bool x) { return Val{x ? 1 : 0, (int8_t)CAPSMI_BOOL}; }
__device__ __forceinline__ Val mk_null() { return Val{0, kNull}; }

__device__ Val eval_row(const capsmi_expr* __restrict__ prog, int nn, const ColPtrs& cp, int64_t r) {
    Val st[kMaxStack];
    int sp = 0;
    for (int i = 0; i < nn; ++i) {
        const capsmi_expr x = prog[i];
        switch (x.op) {
            case CAPSMI_X_COL: {
                const int c = x.arg;
                const bool ok = cp.valid[c] == nullptr || cp.valid[c][r];
                st[sp++] = ok ? Val{cp.data[c][r], cp.type[c]} : mk_null();
                break;
            }
            case CAPSMI_X_LIT: st[sp++] = Val{x.ival, (int8_t)x.type}; break;
            case CAPSMI_X_NULL: st[sp++] = mk_null(); break;
            case CAPSMI_X_EQ: case CAPSMI_X_NEQ: case CAPSMI_X_LT: case CAPSMI_X_LE: case CAPSMI_X_GT: case CAPSMI_X_GE: {
                const Val b = st[--sp], a = st[--sp];
                const int c = cmp3(a, b);
                if (c == -2) { st[sp++] = mk_null(); break; }
                bool res = false;
                switch (x.op) {
                    case CAPSMI_X_EQ: res = c == 0; break;
                    case CAPSMI_X_NEQ: res = c != 0; break;
                    case CAPSMI_X_LT: res = c < 0; break;
                    case CAPSMI_X_LE: res = c <= 0; break;
                    case CAPSMI_X_GT: res = c > 0; break;
                    default: res = c >= 0; break;
                }
                st[sp++] = mk_bool(res);
                break;
            }
            case CAPSMI_X_NOT: {
                const Val a = st[--sp];
                st[sp++] = a.t == kNull ? mk_null() : mk_bool(a.b == 0);
                break;
            }
            case CAPSMI_X_AND: case CAPSMI_X_OR: {
                const bool is_and = x.op == CAPSMI_X_AND;
                bool any_null = false, decided = false;
                for (int k = 0; k < x.arg; ++k) {
                    const Val a = st[--sp];
                    if (a.t == kNull) any_null = true;
                    else if (is_and ? a.b == 0 : a.b != 0) decided = true;
                }
                if (decided) st[sp++] = mk_bool(!is_and);
                else if (any_null) st[sp++] = mk_null();
                else st[sp++] = mk_bool(is_and);
                break;
            }
            case CAPSMI_X_ISNULL: { const Val a = st[--sp]; st[sp++] = mk_bool(a.t == kNull); break; }
            case CAPSMI_X_ISNOTNULL: { const Val a = st[--sp]; st[sp++] = mk_bool(a.t != kNull); break; }
            case CAPSMI_X_IN: {
                bool hit = false, any_null = false;
                const Val v = st[sp - x.arg - 1];
                for (int k = 0; k < x.arg; ++k) {
                    const int c = cmp3(v, st[sp - x.arg + k]);
                    if (c == 0) hit = true;
                    else if (c == -2) any_null = true;
                }
                sp -= x.arg + 1;
                st[sp++] = hit ? mk_bool(true) : (any_null || v.t == kNull ? mk_null() : mk_bool(false));
                break;
            }
            case CAPSMI_X_ADD: case CAPSMI_X_SUB: case CAPSMI_X_MUL: {
                const Val b = st[--sp], a = st[--sp];
                if (a.t == kNull || b.t == kNull || !numeric(a.t) || !numeric(b.t)) { st[sp++] = mk_null(); break; }
                if (a.t == CAPSMI_I64 && b.t == CAPSMI_I64) {
                    const uint64_t ua = (uint64_t)a.b, ub = (uint64_t)b.b;  // Spark Long arithmetic wraps
                    const uint64_t r2 = x.op == CAPSMI_X_ADD ? ua + ub : (x.op == CAPSMI_X_SUB ? ua - ub : ua * ub);
                    st[sp++] = Val{(int64_t)r2, (int8_t)CAPSMI_I64};
                } else {
                    const double p = as_f64(a), q = as_f64(b);
                    const double r2 = x.op == CAPSMI_X_ADD ? p + q : (x.op == CAPSMI_X_SUB ? p - q : p * q);
                    st[sp++] = Val{__double_as_longlong(r2), (int8_t)CAPSMI_F64};
                }
                break;
            }
            case CAPSMI_X_NEG: {
                const Val a = st[--sp];
                if (a.t == CAPSMI_I64) st[sp++] = Val{(int64_t)(0ULL - (uint64_t)a.b), (int8_t)CAPSMI_I64};
                else if (a.t == CAPSMI_F64) st[sp++] = Val{__double_as_longlong(-__longlong_as_double(a.b)), (int8_t)CAPSMI_F64};
                else st[sp++] = mk_null();
                break;
            }
            case CAPSMI_X_COALESCE: {
                Val res = mk_null();
                for (int k = 0; k < x.arg; ++k) {
                    const Val a = st[sp - x.arg + k];
                    if (res.t == kNull && a.t != kNull) res = a;
                }
                sp -= x.arg;
                st[sp++] = res;
                break;
            }
            case CAPSMI_X_BITAND: case CAPSMI_X_BITOR: case CAPSMI_X_SHL: case CAPSMI_X_SHRU: {
                const Val b = st[--sp], a = st[--sp];
                if (a.t != CAPSMI_I64 || b.t != CAPSMI_I64) { st[sp++] = mk_null(); break; }
                const uint64_t ua = (uint64_t)a.b, ub = (uint64_t)b.b;
                uint64_t r2;
                switch (x.op) {
                    case CAPSMI_X_BITAND: r2 = ua & ub; break;
                    case CAPSMI_X_BITOR: r2 = ua | ub; break;
                    case CAPSMI_X_SHL: r2 = ua << (ub & 63); break;  // Java long shift semantics
                    default: r2 = ua >> (ub & 63); break;
                }
                st[sp++] = Val{(int64_t)r2, (int8_t)CAPSMI_I64};
                break;
            }
            case CAPSMI_X_CASE: {
                const int base = sp - (2 * x.arg + 1);
                Val res = st[sp - 1];  // default
                for (int k = x.arg - 1; k >= 0; --k) {  // the first TRUE predicate wins
                    const Val p = st[base + 2 * k];
                    if (p.t == CAPSMI_BOOL && p.b != 0) res = st[base + 2 * k + 1];
                }
                sp = base;
                st[sp++] = res;
                break;
            }
            default: st[sp++] = mk_null(); break;
        }
    }
    return sp > 0 ? st[sp - 1] : mk_null();
}

__global__ void k_eval(const capsmi_expr* __restrict__ prog, int nn, ColPtrs cp, int64_t n, int64_t* __restrict__ out,
                       uint8_t* __restrict__ out_valid, uint8_t* __restrict__ flags) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const Val v = eval_row(prog, nn, cp, r);
        if (flags) flags[r] = (v.t == CAPSMI_BOOL && v.b != 0) ? 1 : 0;
        if (out) out[r] = v.t == kNull ? 0 : v.b;
        if (out_valid) out_valid[r] = v.t == kNull ? 0 : 1;
    }
}

}  // namespace

// static type of a program (host): literal / column types propagate, comparisons -> BOOL
int32_t infer_type(const capsmi_table* t, int32_t nn, const capsmi_expr* prog) {
    std::vector<int> st;
    for (int i = 0; i < nn; ++i) {
        const capsmi_expr& x = prog[i];
        auto pop = [&]() { int v = st.empty() ? -1 : st.back(); if (!st.empty()) st.pop_back(); return v; };
        switch (x.op) {
            case CAPSMI_X_COL: st.push_back(t->cols[x.arg].type); break;
            case CAPSMI_X_LIT: st.push_back(x.type); break;
            case CAPSMI_X_NULL: st.push_back(x.arg > 0 ? x.arg - 1 : -1); break;  // arg = 1 + declared type
            case CAPSMI_X_AND: case CAPSMI_X_OR: for (int k = 0; k < x.arg; ++k) pop(); st.push_back(CAPSMI_BOOL); break;
            case CAPSMI_X_IN: for (int k = 0; k < x.arg + 1; ++k) pop(); st.push_back(CAPSMI_BOOL); break;
            case CAPSMI_X_NOT: case CAPSMI_X_ISNULL: case CAPSMI_X_ISNOTNULL: pop(); st.push_back(CAPSMI_BOOL); break;
            case CAPSMI_X_NEG: break;
            case CAPSMI_X_COALESCE: {
                int ty = -1;
                for (int k = 0; k < x.arg; ++k) { int v = pop(); if (v >= 0) ty = v; }
                st.push_back(ty);
                break;
            }
            case CAPSMI_X_ADD: case CAPSMI_X_SUB: case CAPSMI_X_MUL: {
                int b = pop(), a = pop();
                st.push_back((a == CAPSMI_F64 || b == CAPSMI_F64) ? CAPSMI_F64 : CAPSMI_I64);
                break;
            }
            case CAPSMI_X_BITAND: case CAPSMI_X_BITOR: case CAPSMI_X_SHL: case CAPSMI_X_SHRU:
                pop(); pop(); st.push_back(CAPSMI_I64); break;
            case CAPSMI_X_CASE: {
                int ty = pop();  // default, then the values (predicates are BOOL)
                for (int k = 0; k < x.arg; ++k) {
                    const int v = pop();
                    pop();
                    if (v >= 0) ty = v;
                }
                st.push_back(ty);
                break;
            }
            default: pop(); pop(); st.push_back(CAPSMI_BOOL); break;
        }
    }
    const int ty = st.empty() ? -1 : st.back();
    return ty < 0 ? CAPSMI_I64 : ty;
}

bool has_params(int32_t nn, const capsmi_expr* prog) {
    for (int i = 0; i < nn; ++i)
        if (prog[i].op == CAPSMI_X_PARAM) return true;
    return false;
}

// Param(name) -> functions.lit(parameters(name)) (SparkSQLExprMapper.scala:86-92).  Each stack entry
// of the postfix program is tracked with the number of values it stands for: 1, or a list
// parameter's length, which only IN may consume (its element count grows by the list's values).
std::vector<capsmi_expr> bind_params(const capsmi_session* s, int32_t nn, const capsmi_expr* prog) {
    std::vector<capsmi_expr> out;
    std::vector<int> width;  // per stack entry: values it contributes (-1 - k: a list of k values)
    auto lit = [](int32_t type, const capsmi_value& v) {
        capsmi_expr x{};
        if (v.is_null) {
            x.op = CAPSMI_X_NULL;
            x.arg = type + 1;
        } else {
            x.op = CAPSMI_X_LIT;
            x.type = type;
            x.ival = v.ival;
        }
        return x;
    };
    for (int i = 0; i < nn; ++i) {
        const capsmi_expr& x = prog[i];
        if (x.op == CAPSMI_X_PARAM) {
            REQUIRE(x.arg >= 0 && x.arg < (int)s->params.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT,
                    "expression parameter " + std::to_string(x.arg) + " is not set (capsmi_session_set_params)");
            const capsmi_session::Param& p = s->params[x.arg];
            if (!p.list) {
                out.push_back(lit(p.type, p.values[0]));
                width.push_back(1);
            } else {
                for (const capsmi_value& v : p.values) out.push_back(lit(p.type, v));
                width.push_back(-1 - (int)p.values.size());
            }
            continue;
        }
        int pops = 0;
        switch (x.op) {
            case CAPSMI_X_COL: case CAPSMI_X_LIT: case CAPSMI_X_NULL: pops = 0; break;
            case CAPSMI_X_NOT: case CAPSMI_X_ISNULL: case CAPSMI_X_ISNOTNULL: case CAPSMI_X_NEG: pops = 1; break;
            case CAPSMI_X_AND: case CAPSMI_X_OR: case CAPSMI_X_COALESCE: pops = x.arg; break;
            case CAPSMI_X_IN: pops = x.arg + 1; break;
            case CAPSMI_X_CASE: pops = 2 * x.arg + 1; break;
            default: pops = 2; break;
        }
        REQUIRE(pops >= 0 && (int)width.size() >= pops, CAPSMI_ERR_ILLEGAL_ARGUMENT,
                "malformed expression program (stack underflow)");
        capsmi_expr y = x;
        if (x.op == CAPSMI_X_IN) {
            const size_t first = width.size() - pops;  // the tested value, then the elements
            REQUIRE(width[first] == 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "a list parameter is not a single value");
            int n = 0;
            for (size_t k = first + 1; k < width.size(); ++k) n += width[k] >= 0 ? width[k] : -1 - width[k];
            y.arg = n;
        } else {
            for (size_t k = width.size() - pops; k < width.size(); ++k)
                REQUIRE(width[k] == 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "a list parameter may only be an element of IN");
        }
        width.resize(width.size() - pops);
        width.push_back(1);
        out.push_back(y);
    }
    return out;
}

void validate_program(const capsmi_table* t, int32_t nn, const capsmi_expr* prog) {
    int depth = 0, maxd = 0;
    for (int i = 0; i < nn; ++i) {
        const capsmi_expr& x = prog[i];
        int pops = 0;
        switch (x.op) {
            case CAPSMI_X_COL:
                REQUIRE(x.arg >= 0 && x.arg < (int)t->cols.size(), CAPSMI_ERR_ILLEGAL_ARGUMENT,
                        "expression column index out of range");
                REQUIRE(x.arg < kMaxCols, CAPSMI_ERR_NOT_IMPLEMENTED, "expression references column >= 64");
                if (nn > 1) no_list_key(t->cols[x.arg].type, t->cols[x.arg].name, "an expression operand");
                pops = 0; break;
            case CAPSMI_X_LIT: case CAPSMI_X_NULL: pops = 0; break;
            case CAPSMI_X_NOT: case CAPSMI_X_ISNULL: case CAPSMI_X_ISNOTNULL: case CAPSMI_X_NEG: pops = 1; break;
            case CAPSMI_X_AND: case CAPSMI_X_OR: case CAPSMI_X_COALESCE:
                REQUIRE(x.arg >= 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "n-ary operator needs >= 1 operand");
                pops = x.arg; break;
            case CAPSMI_X_IN: REQUIRE(x.arg >= 0, CAPSMI_ERR_ILLEGAL_ARGUMENT, "IN arity"); pops = x.arg + 1; break;
            case CAPSMI_X_EQ: case CAPSMI_X_NEQ: case CAPSMI_X_LT: case CAPSMI_X_LE: case CAPSMI_X_GT: case CAPSMI_X_GE:
            case CAPSMI_X_ADD: case CAPSMI_X_SUB: case CAPSMI_X_MUL:
            case CAPSMI_X_BITAND: case CAPSMI_X_BITOR: case CAPSMI_X_SHL: case CAPSMI_X_SHRU: pops = 2; break;
            case CAPSMI_X_CASE:
                REQUIRE(x.arg >= 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "CASE needs >= 1 alternative");
                pops = 2 * x.arg + 1; break;
            default: throw Error(CAPSMI_ERR_NOT_IMPLEMENTED, "unknown expression op " + std::to_string(x.op));
        }
        REQUIRE(depth >= pops, CAPSMI_ERR_ILLEGAL_ARGUMENT, "malformed expression program (stack underflow)");
        depth = depth - pops + 1;
        if (depth > maxd) maxd = depth;
    }
    REQUIRE(nn == 0 || depth == 1, CAPSMI_ERR_ILLEGAL_ARGUMENT, "expression program must leave one value");
    REQUIRE(maxd <= kMaxStack, CAPSMI_ERR_NOT_IMPLEMENTED, "expression too deep");
}

namespace {

void launch_eval(capsmi_session* s, const capsmi_table* t, int32_t nn, const capsmi_expr* prog, int64_t* out,
                 uint8_t* out_valid, uint8_t* flags) {
    validate_program(t, nn, prog);
    const int64_t n = t->nrows;
    if (n == 0) return;
    ColPtrs cp;
    for (int c = 0; c < kMaxCols; ++c) { cp.data[c] = nullptr; cp.valid[c] = nullptr; cp.type[c] = 0; }
    for (size_t c = 0; c < t->cols.size() && c < (size_t)kMaxCols; ++c) {
        cp.data[c] = t->cols[c].d();
        cp.valid[c] = t->cols[c].v();
        cp.type[c] = (int8_t)t->cols[c].type;
    }
    Buf dprog = dev_alloc(sizeof(capsmi_expr) * (nn > 0 ? nn : 1), s);
    if (nn > 0)
        HIP_CHECK(hipMemcpyAsync(P<void>(dprog), prog, sizeof(capsmi_expr) * nn, hipMemcpyHostToDevice, s->stream));
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_eval, dim3((unsigned)g), dim3(256), 0, s->stream, P<capsmi_expr>(dprog), nn, cp, n, out,
                       out_valid, flags);
    HIP_CHECK(hipGetLastError());
}

}  // namespace

void eval_expr(capsmi_session* s, const capsmi_table* t, int32_t nnodes, const capsmi_expr* prog, int64_t* out,
               uint8_t* out_valid, int32_t* out_type) {
    if (out_type) *out_type = infer_type(t, nnodes, prog);
    launch_eval(s, t, nnodes, prog, out, out_valid, nullptr);
}

void eval_predicate(capsmi_session* s, const capsmi_table* t, int32_t nnodes, const capsmi_expr* prog, uint8_t* flags) {
    if (nnodes == 0) {
        fill_u8(flags, 1, t->nrows, s->stream);
        return;
    }
    launch_eval(s, t, nnodes, prog, nullptr, nullptr, flags);
}

}  // namespace capsmi
