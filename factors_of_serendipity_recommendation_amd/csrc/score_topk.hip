// a6-a9, a11: full-catalog user x item scoring on the matrix cores, with the positive-item mask,
// the running top-k and the global min/max fused into the MFMA epilogue.
//
// Reference: LightGCN.getUsersRating (lightGCN/LightGCN-PyTorch-master/code/model.py:179-184)
// + Procedure.Test mask / torch.topk (code/Procedure.py:127-135); TF batch_ratings
// (LightGCN-tf/LightGCN.py:148) + batch_test.test mask (utility/batch_test.py:63-65) + the C++
// top-k (evaluator/cpp/include/tools.h:13-22); recommend.py full U x I dot + global min/max
// (recommend.py:163-164, :375-377).  The reference materialises the [B, I] rating matrix; here it
// never leaves the accumulators.
//
// MI355X design:
//   * one 256-thread workgroup = 4 waves x 32 query users; a wave keeps its 32 users' embedding
//     fragments in VGPRs for the whole sweep and walks 32-item tiles of its item split;
//   * items are the MFMA A operand and users the B operand, so each lane ends a tile holding 16
//     item scores of ONE user: the top-k filter is one compare per score against a per-lane
//     threshold (the user's current k-th best), and only survivors (~k ln(I/k) per user over the
//     whole catalog) take the slow path (mask lookup + sorted insertion into the user's list in
//     LDS);
//   * bf16: v_mfma_f32_32x32x16_bf16 (fragments are plain 16-B loads); fp32 parity path:
//     v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chain) with the reduction index permuted so each
//     lane still loads 16-B chunks;
//   * small query batches split the catalog over workgroups (grid.y); every split writes its
//     sorted partial list and a one-wave-per-user merge (register bitonic network) finishes, adds
//     the masked tail when fewer than k unmasked items exist, applies the optional sigmoid.
#include <algorithm>

#include "wave_topk.h"

namespace lgx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kWavesPerBlock = 4;
constexpr int kUsersPerWave = 32;
constexpr int kUsersPerBlock = kWavesPerBlock * kUsersPerWave;

// ---------------------------------------------------------------------------- fragments
// f32: chunk c of lane half h = features [8c + 4h, 8c + 4h + 4) -> k-steps 4c..4c+3
// bf16: chunk c of lane half h = features [16c + 8h, 16c + 8h + 8) -> k-step c
template <int DT>
struct Frag;

template <>
struct Frag<LGX_DTYPE_F32> {
    typedef float4 chunk;
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
struct Frag<LGX_DTYPE_BF16> {
    typedef uint4 chunk;
    __device__ static __forceinline__ chunk load(const void* base, int64_t row, int64_t d, int c, int h, bool ok) {
        const int64_t off = (int64_t)c * 16 + 8 * h;
        if (!ok || off >= d) return make_uint4(0u, 0u, 0u, 0u);
        return *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(base) + row * d + off);
    }
    __device__ static __forceinline__ f32x16 mma(const chunk& a, const chunk& b, f32x16 acc) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
    }
};

struct ScoreArgs {
    const void* Q;
    const int64_t* user_rows;
    const void* items;
    int64_t B;
    int64_t n_items;
    int64_t d;
    const int64_t* mask_indptr;
    const int32_t* mask_indices;
    int k;
    int n_splits;
    int64_t split_items;  // items per split (multiple of 32)
    float* part_score;    // [B, n_splits, k]
    int32_t* part_idx;    // [B, n_splits, k]
    uint32_t* minmax;     // ordered {min, max} or nullptr
};

__device__ __forceinline__ bool better(float s1, int32_t i1, float s2, int32_t i2) {
    return s1 > s2 || (s1 == s2 && i1 < i2);
}

__device__ __forceinline__ bool is_masked(const ScoreArgs& a, int64_t b, int32_t item) {
    if (!a.mask_indptr) return false;
    int64_t lo = a.mask_indptr[b], hi = a.mask_indptr[b + 1];
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.mask_indices[mid] < item) lo = mid + 1; else hi = mid;
    }
    return lo < a.mask_indptr[b + 1] && a.mask_indices[lo] == item;
}

// output row (item offset inside the 32-item tile) of accumulator register r for lane half h
__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int DT, int KCH>
__global__ __launch_bounds__(256) void score_topk_kernel(ScoreArgs a) {
    typedef Frag<DT> F;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int k = a.k;
    // per-wave lists: score [32][k], index [32][k], length [32]
    float* ls = reinterpret_cast<float*>(smem) + (size_t)wave * kUsersPerWave * k;
    int32_t* li = reinterpret_cast<int32_t*>(smem + (size_t)kWavesPerBlock * kUsersPerWave * k * 4) +
                  (size_t)wave * kUsersPerWave * k;
    int32_t* ln = reinterpret_cast<int32_t*>(smem + (size_t)kWavesPerBlock * kUsersPerWave * k * 8) +
                  wave * kUsersPerWave;

    const int64_t b = (int64_t)blockIdx.x * kUsersPerBlock + wave * kUsersPerWave + col;  // this lane's user
    const bool user_ok = b < a.B;
    const int64_t qrow = user_ok ? (a.user_rows ? a.user_rows[b] : b) : 0;

    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(a.Q, qrow, a.d, c, h, user_ok);

    if (h == 0) ln[col] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float* my_ls = ls + col * k;
    int32_t* my_li = li + col * k;
    float tau = -INFINITY;
    int32_t tau_i = 0x7fffffff;
    bool full = false;
    float mn = INFINITY, mx = -INFINITY;

    const int split = blockIdx.y;
    const int64_t i_begin = (int64_t)split * a.split_items;
    const int64_t i_end = min(a.n_items, i_begin + a.split_items);

    for (int64_t i0 = i_begin; i0 < i_end; i0 += 32) {
        const int64_t item_row = i0 + col;
        const bool item_ok = item_row < i_end;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            const typename F::chunk ia = F::load(a.items, item_row, a.d, c, h, item_ok);
            acc = F::mma(ia, uf[c], acc);
        }
        uint32_t cmask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int32_t it = (int32_t)(i0 + tile_row(r, h));
            const float s = acc[r];
            if (user_ok && it < i_end) {
                mn = fminf(mn, s);
                mx = fmaxf(mx, s);
                if (!full || better(s, it, tau, tau_i)) cmask |= 1u << r;
            }
        }
        if (__ballot(cmask != 0) == 0ull) continue;  // wave-uniform fast path
        // slow path: the two lane halves hold different items of the same 32 users -> serialise
        for (int ph = 0; ph < 2; ++ph) {
            if (ph == h && cmask) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (!((cmask >> r) & 1u)) continue;
                    const int32_t it = (int32_t)(i0 + tile_row(r, h));
                    const float s = acc[r];
                    int len = ln[col];
                    if (len == k && !better(s, it, my_ls[k - 1], my_li[k - 1])) continue;
                    if (is_masked(a, b, it)) continue;
                    int pos = len < k ? len : k - 1;
                    while (pos > 0 && better(s, it, my_ls[pos - 1], my_li[pos - 1])) {
                        my_ls[pos] = my_ls[pos - 1];
                        my_li[pos] = my_li[pos - 1];
                        --pos;
                    }
                    my_ls[pos] = s;
                    my_li[pos] = it;
                    if (len < k) ln[col] = len + 1;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        const int len = ln[col];
        full = len == k;
        if (full) {
            tau = my_ls[k - 1];
            tau_i = my_li[k - 1];
        }
    }

    // partial list of this split
    if (user_ok && h == 0) {
        const int len = ln[col];
        float* ps = a.part_score + ((size_t)b * a.n_splits + split) * k;
        int32_t* pi = a.part_idx + ((size_t)b * a.n_splits + split) * k;
        for (int j = 0; j < k; ++j) {
            ps[j] = j < len ? my_ls[j] : -INFINITY;
            pi[j] = j < len ? my_li[j] : -1;
        }
    }
    if (a.minmax) {
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            mn = fminf(mn, __shfl_xor(mn, m, 64));
            mx = fmaxf(mx, __shfl_xor(mx, m, 64));
        }
        if (lane == 0 && mn <= mx) {
            atomicMin(a.minmax, ord_f32(mn));
            atomicMax(a.minmax + 1, ord_f32(mx));
        }
    }
}

// one wave per query: merge the split lists, masked tail, optional sigmoid
__global__ __launch_bounds__(64) void score_topk_finalize(ScoreArgs a, float mask_value, int apply_sigmoid,
                                                          int32_t* __restrict__ out_idx, float* __restrict__ out_val,
                                                          float* __restrict__ minmax_out) {
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int k = a.k;
    const int64_t total = (int64_t)a.n_splits * k;
    const float* ps = a.part_score + (size_t)b * total;
    const int32_t* pi = a.part_idx + (size_t)b * total;
    uint64_t top = 0;
    for (int64_t base = 0; base < total; base += 64) {
        const int64_t j = base + lane;
        const uint64_t cand = (j < total && pi[j] >= 0) ? make_key(ps[j], pi[j]) : 0ull;
        wave_topk_push(top, cand, k, lane);
    }
    const int n_real = __popcll(__ballot(top != 0ull));
    if (lane < k) {
        int32_t idx = -1;
        float val = mask_value;
        if (top) {
            idx = key_index(top);
            const float s = key_score(top);
            val = apply_sigmoid ? 1.0f / (1.0f + expf(-s)) : s;
        } else if (a.mask_indptr) {
            const int64_t m0 = a.mask_indptr[b], m1 = a.mask_indptr[b + 1];
            const int64_t j = m0 + (lane - n_real);
            if (j < m1) idx = a.mask_indices[j];
        }
        out_idx[b * k + lane] = idx;
        if (out_val) out_val[b * k + lane] = val;
    }
    if (minmax_out && b == 0 && lane == 0) {
        minmax_out[0] = unord_f32(a.minmax[0]);
        minmax_out[1] = unord_f32(a.minmax[1]);
    }
}

__global__ void minmax_init(uint32_t* mm) {
    mm[0] = 0xffffffffu;  // ord(+NaN) upper bound: any real min is smaller
    mm[1] = 0u;
}

// ---------------------------------------------------------------------------- dense scores
// getUsersRating: users are the A operand (rows), items the B operand (lane columns) so that
// each store instruction writes 32 consecutive floats of one user row.
template <int DT, int KCH>
__global__ __launch_bounds__(256) void score_dense_kernel(const void* Q, const int64_t* user_rows, const void* items,
                                                          int64_t B, int64_t n_items, int64_t d, int apply_sigmoid,
                                                          float* __restrict__ out) {
    typedef Frag<DT> F;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t u0 = (int64_t)blockIdx.x * 32;
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    const int64_t qrow = user_ok ? (user_rows ? user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(Q, qrow, d, c, h, user_ok);
    const int64_t tiles = (n_items + 31) / 32;
    for (int64_t t = (int64_t)blockIdx.y * kWavesPerBlock + wave; t < tiles; t += (int64_t)gridDim.y * kWavesPerBlock) {
        const int64_t i0 = t * 32;
        const int64_t item_row = i0 + col;
        const bool item_ok = item_row < n_items;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) acc = F::mma(uf[c], F::load(items, item_row, d, c, h, item_ok), acc);
        if (!item_ok) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t u = u0 + tile_row(r, h);
            if (u < B) {
                const float s = acc[r];
                out[u * n_items + item_row] = apply_sigmoid ? 1.0f / (1.0f + expf(-s)) : s;
            }
        }
    }
}

int kch_for(int dtype, int64_t d) {
    const int64_t per = dtype == LGX_DTYPE_F32 ? 8 : 16;
    const int64_t c = (d + per - 1) / per;
    if (c <= 2) return 2;
    if (c <= 4) return 4;
    if (c <= 8) return 8;
    if (c <= 16) return 16;
    if (c <= 32) return 32;
    return -1;
}

struct SplitPlan {
    int n_splits;
    int64_t split_items;
};

SplitPlan plan_splits(int64_t B, int64_t n_items) {
    const int64_t user_blocks = ceil_div(B, kUsersPerBlock);
    const int64_t tiles = ceil_div(n_items, 32);
    int64_t s = ceil_div(2048, user_blocks);          // aim for >= ~8 workgroups per CU
    s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / 8));  // >= 8 tiles per split
    s = std::max<int64_t>(1, std::min<int64_t>(s, 64));
    const int64_t per = ceil_div(tiles, s) * 32;
    return {(int)ceil_div(n_items, per), per};
}

template <int DT>
int launch_score_topk(const ScoreArgs& a0, int kch, float mask_value, int apply_sigmoid, int32_t* out_idx,
                      float* out_val, float* minmax_out, hipStream_t stream) {
    ScoreArgs a = a0;
    const size_t shmem = (size_t)kWavesPerBlock * kUsersPerWave * (a.k * 8 + 4);
    dim3 grid((unsigned)ceil_div(a.B, kUsersPerBlock), (unsigned)a.n_splits);
    if (a.minmax) {
        minmax_init<<<1, 1, 0, stream>>>(a.minmax);
        LGX_LAUNCH_CHECK();
    }
#define LGX_SK(KC)                                                                                      \
    do {                                                                                                \
        if (shmem > 65536)                                                                              \
            LGX_HIP_CHECK(hipFuncSetAttribute((const void*)score_topk_kernel<DT, KC>,                  \
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem)); \
        score_topk_kernel<DT, KC><<<grid, 256, shmem, stream>>>(a);                                     \
    } while (0)
    switch (kch) {
        case 2: LGX_SK(2); break;
        case 4: LGX_SK(4); break;
        case 8: LGX_SK(8); break;
        case 16: LGX_SK(16); break;
        default: LGX_SK(32); break;
    }
#undef LGX_SK
    LGX_LAUNCH_CHECK();
    score_topk_finalize<<<(unsigned)a.B, 64, 0, stream>>>(a, mask_value, apply_sigmoid, out_idx, out_val, minmax_out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

size_t topk_ws_bytes(int64_t B, int64_t n_items, int k) {
    const SplitPlan p = plan_splits(B, n_items);
    return align_up((size_t)B * p.n_splits * k * 4) * 2 + 256;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_score_topk_workspace(int64_t B, int64_t n_items, int k, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && B >= 0 && n_items >= 0 && k >= 1, LGX_ERR_INVALID_ARG,
                "lgx_score_topk_workspace: bad arguments");
    *ws_bytes = topk_ws_bytes(B, n_items, k);
    return LGX_OK;
}

extern "C" int lgx_score_topk(const void* Q, const int64_t* user_rows, const void* items, int64_t B,
                              int64_t n_items, int64_t d, int dtype, const int64_t* mask_indptr,
                              const int32_t* mask_indices, int k, float mask_value, int apply_sigmoid,
                              int32_t* out_idx, float* out_val, float* minmax_out, void* ws,
                              size_t ws_bytes, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(B >= 0 && n_items >= 0 && out_idx, LGX_ERR_INVALID_ARG, "lgx_score_topk: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_score_topk: dtype");
    LGX_REQUIRE(k >= 1 && k <= 64, LGX_ERR_UNSUPPORTED, "lgx_score_topk: k=%d outside [1, 64]", k);
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    const int kch = kch_for(dtype, d);
    LGX_REQUIRE(d > 0 && d % vec == 0 && kch > 0, LGX_ERR_UNSUPPORTED,
                "lgx_score_topk: d=%lld must be a multiple of %lld and <= 256", (long long)d, (long long)vec);
    if (B == 0) return LGX_OK;
    LGX_REQUIRE(n_items > 0 && n_items < INT32_MAX && Q && items, LGX_ERR_INVALID_ARG,
                "lgx_score_topk: empty or oversized catalog");
    const size_t need = topk_ws_bytes(B, n_items, k);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_score_topk: workspace %zu < %zu", ws_bytes, need);
    const SplitPlan p = plan_splits(B, n_items);
    char* base = static_cast<char*>(ws);
    const size_t list_bytes = align_up((size_t)B * p.n_splits * k * 4);
    ScoreArgs a{Q, user_rows, items, B, n_items, d, mask_indptr, mask_indices, k, p.n_splits, p.split_items,
                reinterpret_cast<float*>(base), reinterpret_cast<int32_t*>(base + list_bytes),
                minmax_out ? reinterpret_cast<uint32_t*>(base + 2 * list_bytes) : nullptr};
    if (dtype == LGX_DTYPE_F32)
        return launch_score_topk<LGX_DTYPE_F32>(a, kch, mask_value, apply_sigmoid, out_idx, out_val, minmax_out, stream);
    return launch_score_topk<LGX_DTYPE_BF16>(a, kch, mask_value, apply_sigmoid, out_idx, out_val, minmax_out, stream);
}

extern "C" int lgx_score_dense(const void* Q, const int64_t* user_rows, const void* items, int64_t B,
                               int64_t n_items, int64_t d, int dtype, int apply_sigmoid, float* scores,
                               lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(B >= 0 && n_items >= 0 && (B == 0 || (Q && items && scores)), LGX_ERR_INVALID_ARG,
                "lgx_score_dense: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_score_dense: dtype");
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    const int kch = kch_for(dtype, d);
    LGX_REQUIRE(d > 0 && d % vec == 0 && kch > 0, LGX_ERR_UNSUPPORTED,
                "lgx_score_dense: d=%lld must be a multiple of %lld and <= 256", (long long)d, (long long)vec);
    if (B == 0 || n_items == 0) return LGX_OK;
    const int64_t ub = ceil_div(B, 32);
    const int64_t tiles = ceil_div(n_items, 32);
    int64_t gy = std::max<int64_t>(1, std::min<int64_t>(ceil_div(2048, ub), ceil_div(tiles, kWavesPerBlock)));
    dim3 grid((unsigned)ub, (unsigned)std::min<int64_t>(gy, 65535));
#define LGX_SD(DTV, KC) score_dense_kernel<DTV, KC><<<grid, 256, 0, stream>>>(Q, user_rows, items, B, n_items, d, \
                                                                              apply_sigmoid, scores)
#define LGX_SD_ALL(DTV)                  \
    switch (kch) {                       \
        case 2: LGX_SD(DTV, 2); break;   \
        case 4: LGX_SD(DTV, 4); break;   \
        case 8: LGX_SD(DTV, 8); break;   \
        case 16: LGX_SD(DTV, 16); break; \
        default: LGX_SD(DTV, 32); break; \
    }
    if (dtype == LGX_DTYPE_F32) { LGX_SD_ALL(LGX_DTYPE_F32) } else { LGX_SD_ALL(LGX_DTYPE_BF16) }
#undef LGX_SD_ALL
#undef LGX_SD
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}
