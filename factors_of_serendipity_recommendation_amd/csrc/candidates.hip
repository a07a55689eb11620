// candidate-level similarity on the matrix cores.
//
// lgx_list_dot_reduce: for every user u and every entry a of u's list A,
//     out[a] = max over b in u's list B of <T[a], T[b]>        (LGX_REDUCE_MAX)
//     out[a] = sum over b in u's list B of <T[a], T[b]>        (LGX_REDUCE_SUM)
// This is the per-user [|A|, d] x [d, |B|] product followed by a row reduction that the reference
// runs per user in numpy:
//   recommend.difference   max over the train history   (recommend.py:287-312; recommend_combination.py:282-305)
//   utils.ser1_sub         max over test / train         (utils.py:23-38)
//   utils.ser2_sub         max over train                (utils.py:117-121)
//   utils.diversity_sub    mean over the list itself     (utils.py:265-267) -- sum / (|A| |B|)
//
// MI355X design: one 256-thread workgroup per user, its 4 waves striding over 32-entry blocks of A.
// A block's 32 rows are the MFMA B operand, held in VGPRs; B's rows are the A operand in 32-row
// tiles, staged once per user into a padded LDS image when they fit in 48 KB (every block of A
// reads them; 2.25 -> 1.73 ms on the f1 row) and gathered per block from HBM/L2 otherwise, so each
// lane ends a tile holding 16 products of ONE entry of A and reduces them in registers.  fp32: v_mfma_f32_32x32x2_f32 (the exact fp32 fmaf
// chain); bf16: v_mfma_f32_32x32x16_bf16 with fp32 accumulation.
#include "lgx_common.h"

namespace lgx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// chunk c of lane half h: f32 features [8c + 4h, +4) (k-steps 4c..4c+3); bf16 features [16c + 8h, +8)
template <int DT>
struct RowFrag;

template <>
struct RowFrag<LGX_DTYPE_F32> {
    typedef float4 chunk;
    static constexpr int FEATS = 8;  // features per chunk index (both halves)
    __device__ static __forceinline__ chunk load(const void* base, int64_t row, int64_t d, int c, int h, bool ok) {
        const int64_t off = (int64_t)c * 8 + 4 * h;
        if (!ok || off >= d) return make_float4(0.f, 0.f, 0.f, 0.f);
        return *reinterpret_cast<const float4*>(static_cast<const float*>(base) + row * d + off);
    }
    __device__ static __forceinline__ f32x16 mma(const chunk& a, const chunk& b, f32x16 acc) {
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc, 0, 0, 0);
        return acc;
    }
};

template <>
struct RowFrag<LGX_DTYPE_BF16> {
    typedef uint4 chunk;
    static constexpr int FEATS = 16;
    __device__ static __forceinline__ chunk load(const void* base, int64_t row, int64_t d, int c, int h, bool ok) {
        const int64_t off = (int64_t)c * 16 + 8 * h;
        if (!ok || off >= d) return make_uint4(0u, 0u, 0u, 0u);
        return *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(base) + row * d + off);
    }
    __device__ static __forceinline__ f32x16 mma(const chunk& a, const chunk& b, f32x16 acc) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       acc, 0, 0, 0);
    }
};

// accumulator register r of lane half h holds row (r & 3) + 8 (r >> 2) + 4 h of the 32-row tile
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

constexpr int kListWaves = 4;
constexpr int kListLdsBytes = 32 * 1024;  // B-list image: 5 workgroups (20 waves) per CU

template <int DT, int KCH, bool MAX>
__global__ __launch_bounds__(256) void list_dot_reduce_kernel(const void* __restrict__ table, int64_t d,
                                                             const int64_t* __restrict__ a_indptr,
                                                             const int32_t* __restrict__ a_items,
                                                             const int64_t* __restrict__ b_indptr,
                                                             const int32_t* __restrict__ b_items,
                                                             float* __restrict__ out) {
    typedef RowFrag<DT> F;
    // B image in LDS: row r, chunk c, half h at 16-B slot r * RS + 2c + h; the odd row stride RS
    // puts the 32 rows of a fragment read on distinct bank quads (conflict-free ds_read_b128)
    constexpr int RS = 2 * KCH + 1;
    constexpr int kMaxTiles = kListLdsBytes / (32 * RS * 16);
    __shared__ uint4 bimg[kMaxTiles > 0 ? kMaxTiles * 32 * RS : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t u = blockIdx.x;
    const int64_t a0 = a_indptr[u], a1 = a_indptr[u + 1];
    const int64_t b0 = b_indptr[u], b1 = b_indptr[u + 1];
    const int64_t nbt = (b1 - b0 + 31) / 32;
    if (a1 > a0 && nbt > 0 && nbt <= kMaxTiles) {
        // the user's B rows are read by every block of A: stage them once (zero rows past |B|)
        for (int64_t i = threadIdx.x; i < nbt * 32 * 2 * KCH; i += 256) {
            const int64_t r = i / (2 * KCH);
            const int ch = (int)(i % (2 * KCH));
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (b0 + r < b1) {
                const typename F::chunk c = F::load(table, b_items[b0 + r], d, ch >> 1, ch & 1, true);
                v = __builtin_bit_cast(uint4, c);
            }
            bimg[r * RS + ch] = v;
        }
        __syncthreads();
        for (int64_t blk = a0 + (int64_t)wave * 32; blk < a1; blk += kListWaves * 32) {
            const int64_t p = blk + col;
            const bool ok = p < a1;
            const int64_t arow = ok ? a_items[p] : 0;
            typename F::chunk af[KCH];
#pragma unroll
            for (int c = 0; c < KCH; ++c) af[c] = F::load(table, arow, d, c, h, ok);
            float red = MAX ? -INFINITY : 0.0f;
            for (int64_t t = 0; t < nbt; ++t) {
                const uint4* brow = bimg + (t * 32 + col) * RS + h;
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
                for (int c = 0; c < KCH; ++c)
                    acc = F::mma(__builtin_bit_cast(typename F::chunk, brow[2 * c]), af[c], acc);
                const int64_t t0 = b0 + t * 32;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (t0 + acc_row(r, h) < b1) red = MAX ? fmaxf(red, acc[r]) : red + acc[r];
                }
            }
            const float other = __shfl_xor(red, 32, 64);
            red = MAX ? fmaxf(red, other) : red + other;
            if (h == 0 && ok) out[p] = red;
        }
        return;
    }
    // |B| beyond the LDS image (or empty): B tiles gathered from global memory per block of A
    for (int64_t blk = a0 + (int64_t)wave * 32; blk < a1; blk += kListWaves * 32) {
        const int64_t p = blk + col;  // this lane's entry of A (column of the product tile)
        const bool ok = p < a1;
        const int64_t arow = ok ? a_items[p] : 0;
        typename F::chunk af[KCH];
#pragma unroll
        for (int c = 0; c < KCH; ++c) af[c] = F::load(table, arow, d, c, h, ok);
        float red = MAX ? -INFINITY : 0.0f;
        for (int64_t t0 = b0; t0 < b1; t0 += 32) {
            const int64_t q = t0 + col;  // tile row loaded by this lane
            const bool okb = q < b1;
            const int64_t brow = okb ? b_items[q] : 0;
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
            for (int c = 0; c < KCH; ++c) acc = F::mma(F::load(table, brow, d, c, h, okb), af[c], acc);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (t0 + acc_row(r, h) < b1) red = MAX ? fmaxf(red, acc[r]) : red + acc[r];
            }
        }
        const float other = __shfl_xor(red, 32, 64);  // the other half holds the other 16 rows of each tile
        red = MAX ? fmaxf(red, other) : red + other;
        if (h == 0 && ok) out[p] = red;
    }
}

template <int DT, bool MAX>
int launch_list(const void* table, int64_t d, int64_t n_users, const int64_t* a_indptr, const int32_t* a_items,
                const int64_t* b_indptr, const int32_t* b_items, float* out, hipStream_t stream) {
    const int64_t kch = ceil_div(d, (int64_t)RowFrag<DT>::FEATS);
    const dim3 grid((unsigned)n_users);
#define LGX_LD(K)                                                                                      \
    list_dot_reduce_kernel<DT, K, MAX><<<grid, 256, 0, stream>>>(table, d, a_indptr, a_items, b_indptr, \
                                                                 b_items, out)
    if (kch <= 1) LGX_LD(1);
    else if (kch <= 2) LGX_LD(2);
    else if (kch <= 4) LGX_LD(4);
    else if (kch <= 8) LGX_LD(8);
    else if (kch <= 16) LGX_LD(16);
    else LGX_LD(32);
#undef LGX_LD
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_list_dot_reduce(const void* table, int64_t d, int dtype, int64_t n_users,
                                   const int64_t* a_indptr, const int32_t* a_items, const int64_t* b_indptr,
                                   const int32_t* b_items, int reduce, float* out, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(n_users >= 0 && d > 0, LGX_ERR_INVALID_ARG, "lgx_list_dot_reduce: bad sizes");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG,
                "lgx_list_dot_reduce: dtype");
    LGX_REQUIRE(reduce == LGX_REDUCE_MAX || reduce == LGX_REDUCE_SUM, LGX_ERR_INVALID_ARG,
                "lgx_list_dot_reduce: reduce");
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    LGX_REQUIRE(d % vec == 0 && d <= 256, LGX_ERR_UNSUPPORTED,
                "lgx_list_dot_reduce: d=%lld must be a multiple of %lld and <= 256", (long long)d, (long long)vec);
    LGX_REQUIRE(n_users < (int64_t)INT32_MAX, LGX_ERR_UNSUPPORTED, "lgx_list_dot_reduce: too many users");
    if (n_users == 0) return LGX_OK;
    LGX_REQUIRE(table && a_indptr && b_indptr && out, LGX_ERR_INVALID_ARG, "lgx_list_dot_reduce: null pointer");
    const bool mx = reduce == LGX_REDUCE_MAX;
    if (dtype == LGX_DTYPE_F32)
        return mx ? launch_list<LGX_DTYPE_F32, true>(table, d, n_users, a_indptr, a_items, b_indptr, b_items, out, stream)
                  : launch_list<LGX_DTYPE_F32, false>(table, d, n_users, a_indptr, a_items, b_indptr, b_items, out,
                                                      stream);
    return mx ? launch_list<LGX_DTYPE_BF16, true>(table, d, n_users, a_indptr, a_items, b_indptr, b_items, out, stream)
              : launch_list<LGX_DTYPE_BF16, false>(table, d, n_users, a_indptr, a_items, b_indptr, b_items, out,
                                                   stream);
}
