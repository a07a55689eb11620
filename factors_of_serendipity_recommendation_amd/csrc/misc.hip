// Library plumbing (version / errors / device info), candidate-list similarity (recommend.py) and
// the deterministic synthetic-data generators used by the bench.
#include <cstring>
#include <mutex>

#include "lgx_common.h"

namespace lgx {

static thread_local char g_err[1024];

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

namespace {

// recommend.py:167-171 / :214-217: per user, dot(E_u[1,d], E_i[cand]^T).  One G-lane group per
// (user, candidate) pair, G = d/4 (f32 rows read as 16-B chunks), reduced with xor-shuffles.
template <int G>
__global__ __launch_bounds__(256) void gather_scores_kernel(const float* __restrict__ eu, const float* __restrict__ ei,
                                                            int64_t n_users, int64_t n_items, int64_t d,
                                                            const int64_t* __restrict__ cand_indptr,
                                                            const int32_t* __restrict__ cand_items,
                                                            int64_t n_pairs, float* __restrict__ out) {
    const int gl = threadIdx.x & (G - 1);
    const int64_t p = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    if (p >= n_pairs) return;
    // owner user of pair p: binary search in cand_indptr (upper_bound - 1)
    int64_t lo = 0, hi = n_users;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cand_indptr[mid + 1] <= p) lo = mid + 1; else hi = mid;
    }
    const int64_t item = cand_items[p];
    if (item < 0 || item >= n_items) {  // never read outside the item table (the host raises first)
        if (gl == 0) out[p] = __builtin_nanf("");
        return;
    }
    const float* a = eu + lo * d;
    const float* b = ei + item * d;
    float s = 0.0f;
    for (int64_t off = (int64_t)gl * 4; off < d; off += 4 * G) {
        const float4 x = *reinterpret_cast<const float4*>(a + off);
        const float4 y = *reinterpret_cast<const float4*>(b + off);
        s = fmaf(x.x, y.x, s); s = fmaf(x.y, y.y, s); s = fmaf(x.z, y.z, s); s = fmaf(x.w, y.w, s);
    }
#pragma unroll
    for (int m = G >> 1; m > 0; m >>= 1) s += __shfl_xor(s, m, G);
    if (gl == 0) out[p] = s;
}

// The same dots walked user by user: one wave per user, 64/G groups of G lanes each take every
// (64/G)-th candidate, the user's row stays in registers and U item rows are in flight per group.
// No per-pair search for the owning user; per lane the same fmaf order and the same xor-shuffle
// reduction as gather_scores_kernel, so the scores are bit-identical.
template <int G, int CH, int U>
__global__ __launch_bounds__(256) void gather_scores_by_user(const float* __restrict__ eu, const float* __restrict__ ei,
                                                             int64_t n_users, int64_t n_items, int64_t d,
                                                             const int64_t* __restrict__ cand_indptr,
                                                             const int32_t* __restrict__ cand_items,
                                                             float* __restrict__ out) {
    constexpr int GPW = 64 / G;
    const int lane = threadIdx.x & 63, gl = lane & (G - 1), grp = lane / G;
    const int64_t u = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (u >= n_users) return;
    const int64_t p0 = cand_indptr[u], p1 = cand_indptr[u + 1];
    float4 x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int64_t off = (int64_t)(gl + c * G) * 4;
        x[c] = off < d ? *reinterpret_cast<const float4*>(eu + u * d + off) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int64_t pb = p0 + grp; pb < p1; pb += (int64_t)GPW * U) {
        float4 y[U][CH];
        bool ok[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t q = pb + (int64_t)j * GPW;
            const int64_t item = q < p1 ? (int64_t)cand_items[q] : 0;
            ok[j] = item >= 0 && item < n_items;  // never read outside the item table
            const float* b = ei + (ok[j] ? item : 0) * d;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int64_t off = (int64_t)(gl + c * G) * 4;
                y[j][c] = (q < p1 && ok[j] && off < d) ? *reinterpret_cast<const float4*>(b + off)
                                                       : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t q = pb + (int64_t)j * GPW;
            float s = 0.0f;
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if ((int64_t)(gl + c * G) * 4 >= d) break;
                s = fmaf(x[c].x, y[j][c].x, s); s = fmaf(x[c].y, y[j][c].y, s);
                s = fmaf(x[c].z, y[j][c].z, s); s = fmaf(x[c].w, y[j][c].w, s);
            }
#pragma unroll
            for (int m = G >> 1; m > 0; m >>= 1) s += __shfl_xor(s, m, G);
            if (gl == 0 && q < p1) out[q] = ok[j] ? s : __builtin_nanf("");
        }
    }
}

__global__ void synth_edges_kernel(uint64_t seed, const int64_t* __restrict__ offsets, int64_t n_users,
                                   const float* __restrict__ cdf, const int32_t* __restrict__ perm,
                                   int64_t n_items, int64_t n_edges, int32_t* __restrict__ users_out,
                                   int32_t* __restrict__ items_out) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= n_edges) return;
    int64_t lo = 0, hi = n_users - 1;  // owner: last u with offsets[u] <= e
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (offsets[mid] <= e) lo = mid; else hi = mid - 1;
    }
    users_out[e] = (int32_t)lo;
    const float r = u01(splitmix64(seed ^ splitmix64((uint64_t)e)));
    lo = 0;
    hi = n_items - 1;  // first i with cdf[i] >= r
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cdf[mid] < r) lo = mid + 1; else hi = mid;
    }
    items_out[e] = perm ? perm[lo] : (int32_t)lo;
}

// element j of the output is element first + j of the seeded sequence (counter-based: any range of
// the sequence is generated alone, so a rank fills only its own rows of a table)
__global__ void fill_normal_kernel(void* out, int64_t first, int64_t n, float std_, uint64_t seed, int dtype) {
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t i = first + j;
    const uint64_t h = splitmix64(seed ^ splitmix64((uint64_t)(i >> 1)));
    const float u1 = u01(h), u2 = u01(h << 24);
    const float r = sqrtf(-2.0f * logf(u1));
    const float z = (i & 1) ? r * sinf(6.283185307179586f * u2) : r * cosf(6.283185307179586f * u2);
    const float v = z * std_;
    if (dtype == LGX_DTYPE_F32) static_cast<float*>(out)[j] = v;
    else static_cast<uint16_t*>(out)[j] = f32_to_bf16(v);
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" const char* lgx_version(void) { return "lgx 0.1.0 (gfx950)"; }

extern "C" const char* lgx_last_error(void) { return g_err; }

extern "C" int lgx_device_info(int device, int* cu_count, int* xcd_count, char* arch_out, size_t arch_len) {
    hipDeviceProp_t prop;
    LGX_HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (cu_count) *cu_count = prop.multiProcessorCount;
    if (xcd_count) *xcd_count = 8;  // MI355X: 8 XCDs x 32 CUs
    if (arch_out && arch_len) {
        strncpy(arch_out, prop.gcnArchName, arch_len - 1);
        arch_out[arch_len - 1] = 0;
    }
    return LGX_OK;
}

extern "C" int lgx_gather_scores(const float* emb_user, const float* emb_item, int64_t n_users, int64_t n_items,
                                   int64_t d, const int64_t* cand_indptr, const int32_t* cand_items, int64_t n_pairs,
                                   float* scores, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(emb_user && emb_item && cand_indptr && scores && n_users >= 0 && n_items > 0 && n_pairs >= 0,
                LGX_ERR_INVALID_ARG, "lgx_gather_scores: bad arguments");
    LGX_REQUIRE(d > 0 && d % 4 == 0, LGX_ERR_UNSUPPORTED, "lgx_gather_scores: d must be a multiple of 4");
    if (n_pairs == 0) return LGX_OK;
    const int64_t chunks = d / 4;
    if (chunks <= 64 * 4) {  // by user: one wave per user
        const unsigned grid = (unsigned)ceil_div(n_users * 64, 256);
#define LGX_GU(GV, CHV, UV) \
    gather_scores_by_user<GV, CHV, UV><<<grid, 256, 0, stream>>>(emb_user, emb_item, n_users, n_items, d, cand_indptr, \
                                                                cand_items, scores)
        if (chunks <= 4) LGX_GU(4, 1, 4);
        else if (chunks <= 8) LGX_GU(8, 1, 4);
        else if (chunks <= 16) LGX_GU(16, 1, 4);
        else if (chunks <= 32) LGX_GU(32, 1, 4);
        else if (chunks <= 64) LGX_GU(64, 1, 4);
        else if (chunks <= 128) LGX_GU(64, 2, 2);
        else LGX_GU(64, 4, 1);
#undef LGX_GU
        LGX_LAUNCH_CHECK();
        return LGX_OK;
    }
#define LGX_GS(GV)                                                                                      \
    gather_scores_kernel<GV><<<ceil_div(n_pairs * GV, 256), 256, 0, stream>>>(emb_user, emb_item, n_users, \
                                                                              n_items, d, cand_indptr, cand_items, \
                                                                              n_pairs, scores)
    if (chunks <= 4) LGX_GS(4);
    else if (chunks <= 8) LGX_GS(8);
    else if (chunks <= 16) LGX_GS(16);
    else if (chunks <= 32) LGX_GS(32);
    else LGX_GS(64);
#undef LGX_GS
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_synth_edges(uint64_t seed, const int64_t* user_offsets, int64_t n_users,
                               const float* item_cdf, const int32_t* item_perm, int64_t n_items,
                               int64_t n_edges, int32_t* users_out, int32_t* items_out, lgx_stream_t stream) {
    LGX_REQUIRE(user_offsets && item_cdf && users_out && items_out && n_users >= 0 && n_items > 0,
                LGX_ERR_INVALID_ARG, "lgx_synth_edges: bad arguments");
    if (n_users == 0 || n_edges == 0) return LGX_OK;
    synth_edges_kernel<<<ceil_div(n_edges, 256), 256, 0, as_hip(stream)>>>(seed, user_offsets, n_users, item_cdf,
                                                                          item_perm, n_items, n_edges, users_out,
                                                                          items_out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_fill_normal_at(void* out, int64_t first, int64_t n, float std_, uint64_t seed, int dtype,
                                  lgx_stream_t stream) {
    LGX_REQUIRE(out && n >= 0 && first >= 0, LGX_ERR_INVALID_ARG, "lgx_fill_normal: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_fill_normal: dtype");
    if (n == 0) return LGX_OK;
    fill_normal_kernel<<<ceil_div(n, 256), 256, 0, as_hip(stream)>>>(out, first, n, std_, seed, dtype);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_fill_normal(void* out, int64_t n, float std_, uint64_t seed, int dtype, lgx_stream_t stream) {
    return lgx_fill_normal_at(out, 0, n, std_, seed, dtype, stream);
}
