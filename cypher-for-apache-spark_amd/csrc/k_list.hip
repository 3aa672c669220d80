// k_list.hip -- the Collect aggregator (spark-cypher/.../impl/table/SparkTable.scala:169-177):
//   collect_list(x) / collect_set(x) per group, each list sorted ascending (functions.sort_array),
//   nulls skipped (Spark's collect functions ignore them), a group without values -> empty list.
// Device form: one stable LSD sort of the rows by (group, value) -- the value's order key first,
// then the group id -- drops the rows that do not contribute, removes (group, value) repeats for
// collect_set, and the per-group counts become the list offsets.  Equal values are equal 64-bit
// words (Spark 2.2.1's collect_set hashes the raw values; -0.0 and 0.0 stay apart).
#include "capsmi_impl.h"

namespace capsmi {

namespace {

inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// second sort pass key: the row's group, or ng when the row contributes nothing (null value)
__global__ void k_collect_gkey(const int64_t* __restrict__ perm, const int64_t* __restrict__ gid,
                               const uint8_t* __restrict__ valid, int64_t n, int64_t ng, uint64_t* __restrict__ key) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = perm[i];
        const int64_t g = gid[r];
        key[i] = ((valid == nullptr || valid[r]) && g >= 0) ? (uint64_t)g : (uint64_t)ng;
    }
}

// row i of the (group, value) order is kept when it contributes and, for collect_set, differs from
// the previous row of its group
__global__ void k_collect_keep(const uint64_t* __restrict__ key, const int64_t* __restrict__ perm,
                               const int64_t* __restrict__ v, int64_t n, int64_t ng, int distinct,
                               uint8_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool keep = key[i] < (uint64_t)ng;
        if (keep && distinct && i > 0 && key[i - 1] == key[i] && v[perm[i - 1]] == v[perm[i]]) keep = false;
        flags[i] = keep ? 1 : 0;
    }
}

}  // namespace

void no_list_key(int32_t type, const std::string& name, const char* what) {
    REQUIRE(!is_list_type(type), CAPSMI_ERR_NOT_IMPLEMENTED,
            std::string("list column '") + name + "' as " + what + " on the device path");
}

std::shared_ptr<ListStore> collect_lists(capsmi_session* s, const int64_t* gid, int64_t ng, const int64_t* v,
                                         const uint8_t* valid, int type, int64_t n, bool distinct) {
    REQUIRE(type >= CAPSMI_I64 && type <= CAPSMI_STR, CAPSMI_ERR_NOT_IMPLEMENTED, "collect of a list column");
    hipStream_t st = s->stream;
    auto L = std::make_shared<ListStore>();
    L->elem = type;
    L->nlists = ng;
    L->offsets = dev_alloc(sizeof(int64_t) * (ng + 1), s);
    if (n == 0 || ng == 0) {
        HIP_CHECK(hipMemsetAsync(P<void>(L->offsets), 0, sizeof(int64_t) * (ng + 1), st));
        L->values = dev_alloc(sizeof(int64_t), s);
        return L;
    }
    Buf perm = dev_alloc(sizeof(int64_t) * n, s), key = dev_alloc(sizeof(uint64_t) * n, s);
    iota_i64(P<int64_t>(perm), 0, n, st);
    // value order (ascending, the element type's order: ORDER BY's keys), then the group, stably
    order_keys(s, v, valid, type, /*desc=*/false, /*null_pass=*/false, P<int64_t>(perm), n, P<uint64_t>(key));
    radix_sort_pairs(s, P<uint64_t>(key), P<int64_t>(perm), n, 0, 64);
    hipLaunchKernelGGL(k_collect_gkey, dim3(grid_for(n)), dim3(256), 0, st, P<int64_t>(perm), gid, valid, n, ng,
                       P<uint64_t>(key));
    HIP_CHECK(hipGetLastError());
    int bits = 1;
    while (bits < 63 && (uint64_t(1) << bits) <= (uint64_t)ng) ++bits;  // keys 0..ng
    radix_sort_pairs(s, P<uint64_t>(key), P<int64_t>(perm), n, 0, bits);
    Buf flags = dev_alloc(n, s);
    hipLaunchKernelGGL(k_collect_keep, dim3(grid_for(n)), dim3(256), 0, st, P<uint64_t>(key), P<int64_t>(perm), v, n,
                       ng, distinct ? 1 : 0, P<uint8_t>(flags));
    HIP_CHECK(hipGetLastError());
    Buf idx;
    const int64_t k = flags_to_indices(s, P<uint8_t>(flags), n, idx);
    L->nvalues = k;
    Buf rows = dev_alloc(sizeof(int64_t) * (k > 0 ? k : 1), s);
    L->values = dev_alloc(sizeof(int64_t) * (k > 0 ? k : 1), s);
    Buf gk = dev_alloc(sizeof(int64_t) * (k > 0 ? k : 1), s);
    gather_col(P<int64_t>(perm), nullptr, P<int64_t>(idx), k, P<int64_t>(rows), nullptr, st);
    gather_col(v, nullptr, P<int64_t>(rows), k, P<int64_t>(L->values), nullptr, st);
    gather_col(reinterpret_cast<const int64_t*>(P<uint64_t>(key)), nullptr, P<int64_t>(idx), k, P<int64_t>(gk), nullptr,
               st);
    Buf cnt = dev_alloc(sizeof(int64_t) * ng, s);
    HIP_CHECK(hipMemsetAsync(P<void>(cnt), 0, sizeof(int64_t) * ng, st));
    agg_count(P<int64_t>(gk), nullptr, k, P<int64_t>(cnt), st);
    exclusive_scan_i64(P<int64_t>(cnt), P<int64_t>(L->offsets), ng, s);
    return L;
}

std::shared_ptr<ListStore> concat_lists(capsmi_session* s, const ListStore& a, const ListStore& b) {
    REQUIRE(a.elem == b.elem, CAPSMI_ERR_ILLEGAL_ARGUMENT, "union all of lists of different element types");
    hipStream_t st = s->stream;
    auto L = std::make_shared<ListStore>();
    L->elem = a.elem;
    L->nlists = a.nlists + b.nlists;
    L->nvalues = a.nvalues + b.nvalues;
    L->offsets = dev_alloc(sizeof(int64_t) * (L->nlists + 1), s);
    L->values = dev_alloc(sizeof(int64_t) * (L->nvalues > 0 ? L->nvalues : 1), s);
    if (a.nlists)
        HIP_CHECK(hipMemcpyAsync(P<int64_t>(L->offsets), P<int64_t>(a.offsets), sizeof(int64_t) * a.nlists,
                                 hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipMemcpyAsync(P<int64_t>(L->offsets) + a.nlists, P<int64_t>(b.offsets), sizeof(int64_t) * (b.nlists + 1),
                             hipMemcpyDeviceToDevice, st));
    add_i64(P<int64_t>(L->offsets) + a.nlists, a.nvalues, b.nlists + 1, st);
    if (a.nvalues)
        HIP_CHECK(hipMemcpyAsync(P<int64_t>(L->values), P<int64_t>(a.values), sizeof(int64_t) * a.nvalues,
                                 hipMemcpyDeviceToDevice, st));
    if (b.nvalues)
        HIP_CHECK(hipMemcpyAsync(P<int64_t>(L->values) + a.nvalues, P<int64_t>(b.values), sizeof(int64_t) * b.nvalues,
                                 hipMemcpyDeviceToDevice, st));
    return L;
}

}  // namespace capsmi
