// BPR triple sampling on the GPU.
//
// Reference: sources/sampling.cpp:27-86 (sample_negative / sample_negative_ByUser) behind
// utils.UniformSample_original (code/utils.py:55-64): for every user, train_num / user_num rows of
// [user, one of its positives, neg_num items that are not positives] (rejection sampling); the
// ByUser variant does one row per listed user.  The reference draws with libc rand() seeded from
// the clock, so the GPU sampler matches its distribution, not its bits: a counter-based generator
// (splitmix64 of the seed and the row), rejection by binary search in the user's SORTED positive
// list, and a bounded number of draws so every thread terminates -- a row whose user has no
// positive, or whose draws all hit positives, gets -1 in the affected columns.
#include "lgx_common.h"

namespace lgx {
namespace {

constexpr int kMaxDraws = 4096;

__device__ __forceinline__ uint64_t next_u64(uint64_t& x) {
    x += 0x9E3779B97F4A7C15ull;
    return splitmix64(x);
}

// uniform integer in [0, n) (multiply-shift; n < 2^32)
__device__ __forceinline__ int64_t draw(uint64_t& x, int64_t n) {
    return (int64_t)(((next_u64(x) >> 32) * (uint64_t)n) >> 32);
}

// is v in the ascending array a[begin, end)?
__device__ __forceinline__ bool in_sorted(const int32_t* __restrict__ a, int64_t begin, int64_t end, int32_t v) {
    int64_t lo = begin, hi = end;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo < end && a[lo] == v;
}

// one thread per output row [user, pos, neg_1 .. neg_m]
__global__ __launch_bounds__(256) void sample_bpr_kernel(const int64_t* __restrict__ pos_indptr,
                                                        const int32_t* __restrict__ pos_items,
                                                        const int32_t* __restrict__ users, int64_t n_users,
                                                        int64_t n_rows, int64_t per_user, int64_t n_items,
                                                        int neg_num, uint64_t seed, int32_t* __restrict__ out) {
    const int64_t row = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (row >= n_rows) return;
    const int64_t user = users ? (int64_t)users[row] : row / per_user;
    const int width = neg_num + 2;
    int32_t* o = out + row * width;
    o[0] = (int32_t)user;
    const bool known = user >= 0 && user < n_users;
    const int64_t p0 = known ? pos_indptr[user] : 0, p1 = known ? pos_indptr[user + 1] : 0;
    uint64_t x = splitmix64(seed ^ splitmix64((uint64_t)row + 1));
    if (p1 <= p0) {  // unknown user or no positive to pair with
        for (int j = 1; j < width; ++j) o[j] = -1;
        return;
    }
    o[1] = pos_items[p0 + draw(x, p1 - p0)];
    for (int j = 2; j < width; ++j) {
        int32_t neg = -1;
        for (int t = 0; t < kMaxDraws; ++t) {
            const int32_t c = (int32_t)draw(x, n_items);
            if (!in_sorted(pos_items, p0, p1, c)) {
                neg = c;
                break;
            }
        }
        o[j] = neg;
    }
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_sample_bpr(const int64_t* pos_indptr, const int32_t* pos_items, int64_t n_users, int64_t n_items,
                              const int32_t* users, int64_t n_rows, int64_t per_user, int neg_num, uint64_t seed,
                              int32_t* out, lgx_stream_t stream) {
    LGX_REQUIRE(n_users >= 0 && n_items > 0 && n_items < INT32_MAX && n_rows >= 0 && neg_num >= 0,
                LGX_ERR_INVALID_ARG, "lgx_sample_bpr: bad sizes");
    LGX_REQUIRE(users || per_user > 0, LGX_ERR_INVALID_ARG, "lgx_sample_bpr: per_user must be > 0 without a user list");
    LGX_REQUIRE(users || n_rows <= n_users * per_user, LGX_ERR_INVALID_ARG,
                "lgx_sample_bpr: n_rows exceeds n_users * per_user");
    if (n_rows == 0) return LGX_OK;
    LGX_REQUIRE(pos_indptr && out, LGX_ERR_INVALID_ARG, "lgx_sample_bpr: null pointer");
    sample_bpr_kernel<<<(unsigned)ceil_div(n_rows, (int64_t)256), 256, 0, as_hip(stream)>>>(
        pos_indptr, pos_items, users, n_users, n_rows, per_user, n_items, neg_num, seed, out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}
