// a2: normalized bipartite adjacency  A^ = D^-1/2 [[0,R],[R^T,0]] D^-1/2  built on the GPU.
//
// Reference: Loader.getSparseGraph build branch (lightGCN/LightGCN-PyTorch-master/code/
// dataloader.py:339-376) and Data.get_adj_mat pre_adj branch (LightGCN-tf/utility/load_data.py:
// 91-104).  The reference builds it on the host through scipy dok/lil matrices (seconds at
// Gowalla scale, impractical at 10^9 nonzeros); here it is one radix sort of packed 64-bit
// (row, col) keys plus five streaming passes.
//
// Semantics kept bit-exact with the shipped s_pre_adj_mat.npz:
//   deg_r  = number of (duplicate-summed | de-duplicated) entries of row r
//   d_r    = (float)(1.0 / sqrt((double)deg_r)), 0 for deg_r == 0   (np.power(rowsum,-0.5), inf->0)
//   val_rc = (d_r * a_rc) * d_c in float32                          (d_mat.dot(adj).dot(d_mat))
#include <hipcub/hipcub.hpp>

#include "lgx_common.h"

namespace lgx {
namespace {

constexpr int kBlock = 256;

__global__ void make_keys(const int32_t* __restrict__ users, const int32_t* __restrict__ items,
                          int64_t n_edges, int64_t n_users, uint64_t* __restrict__ keys) {
    int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= n_edges) return;
    const uint64_t u = (uint32_t)users[e];
    const uint64_t i = (uint64_t)(n_users + items[e]);
    keys[2 * e] = (u << 32) | i;      // user row -> item column  (R block)
    keys[2 * e + 1] = (i << 32) | u;  // item row -> user column  (R^T block)
}

__global__ void unique_flags(const uint64_t* __restrict__ keys, int64_t m, int32_t* __restrict__ flags) {
    int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= m) return;
    flags[j] = (j == 0 || keys[j] != keys[j - 1]) ? 1 : 0;
}

// starts[p] = first raw position of unique entry p; starts[nnz] = m; indices[p] = column
__global__ void scatter_unique(const uint64_t* __restrict__ keys, const int32_t* __restrict__ flags,
                               const int64_t* __restrict__ pos, int64_t m, int64_t* __restrict__ starts,
                               int32_t* __restrict__ indices) {
    int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= m) return;
    if (flags[j]) {
        const int64_t p = pos[j];
        starts[p] = j;
        indices[p] = (int32_t)(keys[j] & 0xffffffffull);
    }
    if (j == m - 1) starts[pos[j] + flags[j]] = m;
}

// indptr[r] = first unique entry whose row >= r   (rows with no entries get empty ranges)
__global__ void fill_indptr(const uint64_t* __restrict__ keys, const int32_t* __restrict__ flags,
                            const int64_t* __restrict__ pos, const int64_t* __restrict__ starts,
                            int64_t m, int64_t n_rows, int64_t* __restrict__ indptr) {
    int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j > m) return;
    int64_t p, r_cur;
    if (j == m) {
        p = pos[m - 1] + flags[m - 1];  // nnz
        r_cur = n_rows;
    } else {
        if (!flags[j]) return;
        p = pos[j];
        r_cur = (int64_t)(keys[j] >> 32);
    }
    const int64_t r_prev = (p == 0) ? -1 : (int64_t)(keys[starts[p - 1]] >> 32);
    for (int64_t r = r_prev + 1; r <= r_cur; ++r) indptr[r] = p;
}

__global__ void degree_rsqrt(const int64_t* __restrict__ indptr, const int64_t* __restrict__ starts,
                             int64_t n_rows, int dedup, float* __restrict__ dinv) {
    int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const int64_t b = indptr[r], e = indptr[r + 1];
    const int64_t deg = dedup ? (e - b) : (starts[e] - starts[b]);
    dinv[r] = deg > 0 ? (float)(1.0 / sqrt((double)deg)) : 0.0f;
}

__global__ void norm_values(const uint64_t* __restrict__ keys, const int64_t* __restrict__ starts,
                            const float* __restrict__ dinv, const int64_t* __restrict__ nnz_ptr,
                            int dedup, float* __restrict__ vals) {
    int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (p >= *nnz_ptr) return;
    const int64_t j = starts[p];
    const uint64_t key = keys[j];
    const int64_t row = (int64_t)(key >> 32), col = (int64_t)(key & 0xffffffffull);
    const float a = dedup ? 1.0f : (float)(starts[p + 1] - j);
    const float t = __fmul_rn(dinv[row], a);  // d_mat.dot(adj)   (dataloader.py:362)
    vals[p] = __fmul_rn(t, dinv[col]);        // .dot(d_mat)      (dataloader.py:363)
}

__global__ void rows_to_indptr(const int64_t* __restrict__ rows, int64_t nnz, int64_t n_rows,
                               int64_t* __restrict__ indptr) {
    int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (p > nnz) return;
    const int64_t r_cur = (p == nnz) ? n_rows : rows[p];
    const int64_t r_prev = (p == 0) ? -1 : rows[p - 1];
    for (int64_t r = r_prev + 1; r <= r_cur; ++r) indptr[r] = p;
}

struct I32ToI64 {
    __host__ __device__ int64_t operator()(const int32_t& x) const { return (int64_t)x; }
};

struct AdjLayout {
    size_t keys_a, keys_b, flags, pos, dinv, temp, temp_bytes, total;
};

int adj_layout(int64_t n_edges, int64_t n_rows, AdjLayout* L) {
    const int64_t m = 2 * n_edges;
    size_t sort_bytes = 0, scan_bytes = 0;
    hipcub::DoubleBuffer<uint64_t> db(nullptr, nullptr);
    LGX_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, db, (int)m, 0, 64));
    hipcub::TransformInputIterator<int64_t, I32ToI64, const int32_t*> it(nullptr, I32ToI64());
    LGX_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, it, (int64_t*)nullptr, (int)m));
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += align_up(bytes); return o; };
    L->keys_a = take(sizeof(uint64_t) * (m + 1));
    L->keys_b = take(sizeof(uint64_t) * (m + 1));
    L->flags = take(sizeof(int32_t) * (m + 1));
    L->pos = take(sizeof(int64_t) * (m + 1));
    L->dinv = take(sizeof(float) * (n_rows + 1));
    L->temp_bytes = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
    L->temp = take(L->temp_bytes);
    L->total = off;
    return LGX_OK;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_build_norm_adj_workspace(int64_t n_edges, int64_t n_users, int64_t n_items,
                                            size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && n_edges >= 0 && n_users >= 0 && n_items >= 0, LGX_ERR_INVALID_ARG,
                "lgx_build_norm_adj_workspace: bad arguments");
    LGX_REQUIRE(2 * n_edges < (int64_t)INT32_MAX && n_users + n_items < (int64_t)INT32_MAX,
                LGX_ERR_UNSUPPORTED, "lgx_build_norm_adj: 2*n_edges and N must be < 2^31");
    AdjLayout L;
    int rc = adj_layout(n_edges, n_users + n_items, &L);
    if (rc) return rc;
    *ws_bytes = L.total;
    return LGX_OK;
}

extern "C" int lgx_build_norm_adj(const int32_t* user_idx, const int32_t* item_idx, int64_t n_edges,
                                  int64_t n_users, int64_t n_items, int dedup, int64_t* indptr,
                                  int32_t* indices, float* vals, void* ws, size_t ws_bytes,
                                  lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    const int64_t N = n_users + n_items;
    const int64_t m = 2 * n_edges;
    LGX_REQUIRE(indptr && n_edges >= 0 && n_users >= 0 && n_items >= 0, LGX_ERR_INVALID_ARG,
                "lgx_build_norm_adj: bad arguments");
    LGX_REQUIRE(m < (int64_t)INT32_MAX && N < (int64_t)INT32_MAX, LGX_ERR_UNSUPPORTED,
                "lgx_build_norm_adj: 2*n_edges and N must be < 2^31");
    if (m == 0) {
        LGX_HIP_CHECK(hipMemsetAsync(indptr, 0, sizeof(int64_t) * (N + 1), stream));
        return LGX_OK;
    }
    LGX_REQUIRE(user_idx && item_idx && indices && vals && ws, LGX_ERR_INVALID_ARG,
                "lgx_build_norm_adj: null pointer");
    AdjLayout L;
    int rc = adj_layout(n_edges, N, &L);
    if (rc) return rc;
    LGX_REQUIRE(ws_bytes >= L.total, LGX_ERR_WORKSPACE, "lgx_build_norm_adj: workspace %zu < %zu",
                ws_bytes, L.total);
    char* base = static_cast<char*>(ws);
    uint64_t* keys_a = reinterpret_cast<uint64_t*>(base + L.keys_a);
    uint64_t* keys_b = reinterpret_cast<uint64_t*>(base + L.keys_b);
    int32_t* flags = reinterpret_cast<int32_t*>(base + L.flags);
    int64_t* pos = reinterpret_cast<int64_t*>(base + L.pos);
    float* dinv = reinterpret_cast<float*>(base + L.dinv);
    void* temp = base + L.temp;

    const int64_t gE = ceil_div(n_edges, kBlock), gM = ceil_div(m, kBlock), gM1 = ceil_div(m + 1, kBlock);
    make_keys<<<gE, kBlock, 0, stream>>>(user_idx, item_idx, n_edges, n_users, keys_a);
    LGX_LAUNCH_CHECK();
    int end_bit = 32;
    while ((1ll << (end_bit - 32)) < N) ++end_bit;  // row id bits above the 32 column bits
    hipcub::DoubleBuffer<uint64_t> db(keys_a, keys_b);
    size_t tb = L.temp_bytes;
    LGX_HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(temp, tb, db, (int)m, 0, end_bit, stream));
    const uint64_t* keys = db.Current();
    int64_t* starts = reinterpret_cast<int64_t*>(db.Alternate());  // free after the sort

    unique_flags<<<gM, kBlock, 0, stream>>>(keys, m, flags);
    LGX_LAUNCH_CHECK();
    hipcub::TransformInputIterator<int64_t, I32ToI64, const int32_t*> it(flags, I32ToI64());
    tb = L.temp_bytes;
    LGX_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(temp, tb, it, pos, (int)m, stream));
    scatter_unique<<<gM, kBlock, 0, stream>>>(keys, flags, pos, m, starts, indices);
    LGX_LAUNCH_CHECK();
    fill_indptr<<<gM1, kBlock, 0, stream>>>(keys, flags, pos, starts, m, N, indptr);
    LGX_LAUNCH_CHECK();
    degree_rsqrt<<<ceil_div(N, kBlock), kBlock, 0, stream>>>(indptr, starts, N, dedup, dinv);
    LGX_LAUNCH_CHECK();
    norm_values<<<gM, kBlock, 0, stream>>>(keys, starts, dinv, indptr + N, dedup, vals);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_csr_from_coo_rows(const int64_t* coo_rows, int64_t nnz, int64_t n_rows,
                                     int64_t* indptr, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(indptr && nnz >= 0 && n_rows >= 0 && (nnz == 0 || coo_rows), LGX_ERR_INVALID_ARG,
                "lgx_csr_from_coo_rows: bad arguments");
    if (nnz == 0) {
        LGX_HIP_CHECK(hipMemsetAsync(indptr, 0, sizeof(int64_t) * (n_rows + 1), stream));
        return LGX_OK;
    }
    rows_to_indptr<<<ceil_div(nnz + 1, kBlock), kBlock, 0, stream>>>(coo_rows, nnz, n_rows, indptr);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}
