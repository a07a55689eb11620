// a4/a5: LightGCN K-layer propagation -- CSR SpMM with the layer-sum / layer-mean fused into the
// epilogue.
//
// Reference: LightGCN.computer() (lightGCN/LightGCN-PyTorch-master/code/model.py:145-177):
//   all_emb = cat(user_w, item_w); K x all_emb = torch.sparse.mm(G, all_emb) (:171);
//   embs = stack([E0..EK]) ; light_out = mean(embs, dim=1) (:173-175)
// and the TF row-folded equivalent (LightGCN-tf/LightGCN.py:232-253).
//
// MI355X design (bandwidth-bound; no MFMA):
//   * one G-lane group per row segment, G = row bytes / 16 rounded up to a power of two, so each
//     lane moves exactly one 16-B chunk of every gathered embedding row (d=64 f32 or d=128 bf16:
//     16 lanes, 4 rows per wave64);
//   * the group loads G (col, val) pairs with one coalesced load each and broadcasts them with
//     width-G shuffles, then issues UNROLL independent 16-B row gathers before the FMAs so every
//     lane keeps several HBM/LLC requests in flight;
//   * rows are cut into segments of <= seg_len nonzeros and scheduled longest-first (plan built
//     host-side), so power-law hub rows neither serialise one group nor leave a tail; split rows
//     reduce their fp32 partials in slot order in a fix-up pass (deterministic, no atomics);
//   * the epilogue writes the next layer table AND folds the layer into the fp32 running sum, and
//     the last layer writes the mean directly: the [K+1, N, d] stack of the reference is never
//     materialised;
//   * bf16 storage (LGX_DTYPE_BF16) halves the gathered bytes; arithmetic is fp32 throughout;
//   * optional column blocking of the item rows (lgx_csr cb_*): they gather the large user table,
//     so they run as a few launches, each over one column range of every item row, so that one
//     launch's gathers fall in a 1/nb slice of the table (640 MiB at C4 f32: NOT Infinity-Cache
//     resident -- the MALL is 256 MiB -- but a narrower working set for the L2s and the MALL, which
//     measured 57.2 -> 53.6 ms per layer); the row sums are carried in an f32 scratch between them.
#include "lgx_common.h"

namespace lgx {
namespace {

constexpr int kThreads = 256;

// the CSR arrays are plain loads: non-temporal CSR streams and non-temporal cold-column gathers
// measured neutral (profiles/r02_spmm_nt_probe.txt)
template <typename V>
__device__ __forceinline__ V stream_load(const V* p) { return *p; }

template <typename T>
struct Vec;
template <>
struct Vec<float> {
    static constexpr int N = 4;
    typedef float4 raw;
    __device__ static __forceinline__ raw load_raw(const float* p) { return *reinterpret_cast<const float4*>(p); }
    __device__ static __forceinline__ void unpack(const raw& x, float (&v)[4]) {
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
    __device__ static __forceinline__ void load(const float* p, float (&v)[4]) {
        const float4 x = *reinterpret_cast<const float4*>(p);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    }
    __device__ static __forceinline__ void store(float* p, const float (&v)[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    }
};
template <>
struct Vec<uint16_t> {
    static constexpr int N = 8;
    typedef uint4 raw;
    __device__ static __forceinline__ raw load_raw(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }
    __device__ static __forceinline__ void unpack(const raw& x, float (&v)[8]) {
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[2 * j] = __uint_as_float(w[j] << 16);
            v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
        }
    }
    __device__ static __forceinline__ void load(const uint16_t* p, float (&v)[8]) {
        const uint4 x = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[2 * j] = __uint_as_float(w[j] << 16);
            v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
        }
    }
    __device__ static __forceinline__ void store(uint16_t* p, const float (&v)[8]) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            w[j] = (uint32_t)f32_to_bf16(v[2 * j]) | ((uint32_t)f32_to_bf16(v[2 * j + 1]) << 16);
        *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    }
};

struct LayerArgs {
    const int64_t* indptr;
    const int32_t* indices;
    const float* vals;
    const int32_t* seg_row;
    const int32_t* seg_part;
    const int32_t* seg_slot;
    int64_t n_segs;
    int64_t seg_len;
    const int32_t* split_row;
    const int32_t* split_ptr;
    int64_t n_split;
    float* partials;
    const void* X;
    void* Y;
    const void* E0;
    float* acc;
    float* out;
    int64_t d;
    int mode;
    float n_mean;
    const void* prev[7];  // LGX_LAYER_STACK: the kept layer tables
    int n_prev;
    // nonzero range of row r: [row_begin[r], row_end[r]) -- indptr / indptr + 1, or the column
    // block's slice of a blocked row (lgx_csr cb_*)
    const int64_t* row_begin;
    const int64_t* row_end;
    // column-blocked rows: the row sum is carried across the block launches in carry [R, d] f32
    // (row r at carry + (r - carry_row0) * d): kCarryNone, or store / add (then nothing else) /
    // take (v = carry + v, then the mode's epilogue)
    float* carry;
    int64_t carry_row0;
    int carry_mode;
};
constexpr int kMaxPrev = 7;
constexpr int kCarryNone = 0, kCarryStore = 1, kCarryAdd = 2, kCarryTake = 3;

// finish one 16-B chunk (VEC values, columns [off, off+VEC)) of output row `row`
template <typename T>
__device__ __forceinline__ void finish_chunk(const LayerArgs& a, int64_t row, int64_t off,
                                             float (&v)[Vec<T>::N]) {
    constexpr int VEC = Vec<T>::N;
    if (a.carry_mode != kCarryNone) {
        float* cp = a.carry + (row - a.carry_row0) * a.d + off;
#pragma unroll
        for (int j = 0; j < VEC; j += 4) {
            float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.carry_mode != kCarryStore) c = *reinterpret_cast<const float4*>(cp + j);
            if (a.carry_mode == kCarryTake) {
                v[j] = c.x + v[j]; v[j + 1] = c.y + v[j + 1]; v[j + 2] = c.z + v[j + 2]; v[j + 3] = c.w + v[j + 3];
            } else {
                *reinterpret_cast<float4*>(cp + j) =
                    make_float4(c.x + v[j], c.y + v[j + 1], c.z + v[j + 2], c.w + v[j + 3]);
            }
        }
        if (a.carry_mode != kCarryTake) return;
    }
    const int64_t o = row * a.d + off;
    switch (a.mode) {
        case LGX_LAYER_PLAIN:
            Vec<T>::store(static_cast<T*>(a.Y) + o, v);
            break;
        case LGX_LAYER_FIRST: {
            Vec<T>::store(static_cast<T*>(a.Y) + o, v);
            float e[VEC];
            Vec<T>::load(static_cast<const T*>(a.E0) + o, e);
#pragma unroll
            for (int j = 0; j < VEC; ++j) e[j] += v[j];
#pragma unroll
            for (int j = 0; j < VEC; j += 4)
                *reinterpret_cast<float4*>(a.acc + o + j) = make_float4(e[j], e[j + 1], e[j + 2], e[j + 3]);
            break;
        }
        case LGX_LAYER_MID: {
            Vec<T>::store(static_cast<T*>(a.Y) + o, v);
#pragma unroll
            for (int j = 0; j < VEC; j += 4) {
                float4 s = *reinterpret_cast<const float4*>(a.acc + o + j);
                s.x += v[j]; s.y += v[j + 1]; s.z += v[j + 2]; s.w += v[j + 3];
                *reinterpret_cast<float4*>(a.acc + o + j) = s;
            }
            break;
        }
        case LGX_LAYER_LAST: {
#pragma unroll
            for (int j = 0; j < VEC; j += 4) {
                float4 s = *reinterpret_cast<const float4*>(a.acc + o + j);
                s.x = (s.x + v[j]) / a.n_mean;
                s.y = (s.y + v[j + 1]) / a.n_mean;
                s.z = (s.z + v[j + 2]) / a.n_mean;
                s.w = (s.w + v[j + 3]) / a.n_mean;
                *reinterpret_cast<float4*>(a.out + o + j) = s;
            }
            break;
        }
        case LGX_LAYER_STACK: {
            float e[VEC];
            Vec<T>::load(static_cast<const T*>(a.E0) + o, e);
#pragma unroll
            for (int p = 0; p < kMaxPrev; ++p) {  // static indices: the table pointers stay in SGPRs
                if (p >= a.n_prev) break;
                float y[VEC];
                Vec<T>::load(static_cast<const T*>(a.prev[p]) + o, y);
#pragma unroll
                for (int j = 0; j < VEC; ++j) e[j] += y[j];
            }
#pragma unroll
            for (int j = 0; j < VEC; j += 4)
                *reinterpret_cast<float4*>(a.out + o + j) =
                    make_float4((e[j] + v[j]) / a.n_mean, (e[j + 1] + v[j + 1]) / a.n_mean,
                                (e[j + 2] + v[j + 2]) / a.n_mean, (e[j + 3] + v[j + 3]) / a.n_mean);
            break;
        }
        case LGX_LAYER_PARTIAL: {
#pragma unroll
            for (int j = 0; j < VEC; j += 4)
                *reinterpret_cast<float4*>(a.out + o + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
            break;
        }
        default: {  // LGX_LAYER_ONLY
            float e[VEC];
            Vec<T>::load(static_cast<const T*>(a.E0) + o, e);
#pragma unroll
            for (int j = 0; j < VEC; j += 4)
                *reinterpret_cast<float4*>(a.out + o + j) =
                    make_float4((e[j] + v[j]) / a.n_mean, (e[j + 1] + v[j + 1]) / a.n_mean,
                                (e[j + 2] + v[j + 2]) / a.n_mean, (e[j + 3] + v[j + 3]) / a.n_mean);
            break;
        }
    }
}

template <typename T, int G, int CPL, int UNROLL>
__global__ __launch_bounds__(kThreads) void spmm_segments(LayerArgs a) {
    constexpr int VEC = Vec<T>::N;
    const int gl = threadIdx.x & (G - 1);
    const int64_t seg = (blockIdx.x * (int64_t)kThreads + threadIdx.x) / G;
    if (seg >= a.n_segs) return;  // whole groups exit together (n_segs boundary is group-aligned)
    const int64_t row = a.seg_row[seg];
    const int part = a.seg_part[seg];
    const int slot = a.seg_slot[seg];
    const int64_t rb = a.row_begin[row], re = a.row_end[row];
    const int64_t b = rb + (int64_t)part * a.seg_len;
    const int64_t e = slot < 0 ? re : min(re, b + a.seg_len);
    const T* __restrict__ X = static_cast<const T*>(a.X);
    const int64_t d = a.d;

    float acc[CPL][VEC];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[c][j] = 0.0f;

    for (int64_t base = b; base < e; base += G) {
        const int n = (int)min((int64_t)G, e - base);
        const int my_col = gl < n ? stream_load(a.indices + base + gl) : 0;
        const float my_val = gl < n ? stream_load(a.vals + base + gl) : 0.0f;
        for (int t = 0; t < n; t += UNROLL) {
            // the gathered chunks stay packed (bf16: 4 VGPRs per 16 B, not 8) until their FMAs,
            // so more of them fit in flight per wave
            typename Vec<T>::raw x[UNROLL][CPL];
            float w[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const int src = t + u;  // group-uniform
                const int col = __shfl(my_col, src < n ? src : 0, G);
                w[u] = src < n ? __shfl(my_val, src, G) : 0.0f;
                const T* xr = X + (int64_t)col * d;
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const int64_t off = (int64_t)(c * G + gl) * VEC;
                    if (src < n && off < d) x[u][c] = Vec<T>::load_raw(xr + off);
                    else x[u][c] = typename Vec<T>::raw{};
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    float v[VEC];
                    Vec<T>::unpack(x[u][c], v);
#pragma unroll
                    for (int j = 0; j < VEC; ++j) acc[c][j] = fmaf(w[u], v[j], acc[c][j]);
                }
        }
    }

#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int64_t off = (int64_t)(c * G + gl) * VEC;
        if (off >= d) continue;
        if (slot >= 0) {
            float* p = a.partials + (int64_t)slot * d + off;
#pragma unroll
            for (int j = 0; j < VEC; j += 4)
                *reinterpret_cast<float4*>(p + j) = make_float4(acc[c][j], acc[c][j + 1], acc[c][j + 2], acc[c][j + 3]);
        } else {
            finish_chunk<T>(a, row, off, acc[c]);
        }
    }
}

// split rows: one workgroup per split row.  Its kThreads/G groups each sum every NG-th segment
// partial (a hub row's hundreds of partials become NG short independent chains instead of one
// long one: the Gowalla-shape fix-up went from 56.6 us to a fraction of the layer), then group 0 adds the NG sums in
// group order and runs the same epilogue.  The order is fixed, so the result is deterministic.
template <typename T, int G, int CPL>
__global__ __launch_bounds__(kThreads) void spmm_fixup(LayerArgs a) {
    constexpr int VEC = Vec<T>::N;
    constexpr int NG = kThreads / G;
    constexpr int W = G * CPL * VEC;  // floats per group row in LDS (>= d)
    __shared__ float4 red[NG * W / 4];
    const int gl = threadIdx.x & (G - 1), gi = threadIdx.x / G;
    const int64_t s = blockIdx.x;
    const int64_t row = a.split_row[s];
    const int p0 = a.split_ptr[s], p1 = a.split_ptr[s + 1];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int64_t off = (int64_t)(c * G + gl) * VEC;
        float v[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = 0.0f;
        if (off < a.d) {
#pragma unroll 4
            for (int p = p0 + gi; p < p1; p += NG) {
                const float* q = a.partials + (int64_t)p * a.d + off;
#pragma unroll
                for (int j = 0; j < VEC; j += 4) {
                    const float4 t = *reinterpret_cast<const float4*>(q + j);
                    v[j] += t.x; v[j + 1] += t.y; v[j + 2] += t.z; v[j + 3] += t.w;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < VEC; j += 4)
            red[(gi * W + (c * G + gl) * VEC + j) / 4] = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
    }
    __syncthreads();
    if (gi != 0) return;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int64_t off = (int64_t)(c * G + gl) * VEC;
        if (off >= a.d) continue;
        float v[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = 0.0f;
        for (int g = 0; g < NG; ++g) {
#pragma unroll
            for (int j = 0; j < VEC; j += 4) {
                const float4 t = red[(g * W + (c * G + gl) * VEC + j) / 4];
                v[j] += t.x; v[j + 1] += t.y; v[j + 2] += t.z; v[j + 3] += t.w;
            }
        }
        finish_chunk<T>(a, row, off, v);
    }
}

// gathers in flight per lane: a 16-lane group (d=128 bf16 / d=64 f32) issues all 16 rows of a
// CSR chunk at once -- 29.9 vs 31.2 ms per C4 layer against 8 (tools/spmm_probe.py, same box)
template <typename T, int G, int CPL, int UNROLL = (CPL == 1 ? (G == 16 ? 16 : 8) : (CPL == 2 ? 4 : 2))>
int launch_layer(const LayerArgs& a, hipStream_t stream) {
    constexpr int groups_per_block = kThreads / G;
    if (a.n_segs > 0) {
        const int64_t blocks = ceil_div(a.n_segs, groups_per_block);
        spmm_segments<T, G, CPL, UNROLL><<<blocks, kThreads, 0, stream>>>(a);
        LGX_LAUNCH_CHECK();
    }
    if (a.n_split > 0) {
        spmm_fixup<T, G, CPL><<<(unsigned)a.n_split, kThreads, 0, stream>>>(a);
        LGX_LAUNCH_CHECK();
    }
    return LGX_OK;
}

template <typename T>
int dispatch_layer(const LayerArgs& a, hipStream_t stream) {
    constexpr int VEC = Vec<T>::N;
    const int64_t chunks = a.d / VEC;
    if (chunks <= 4) return launch_layer<T, 4, 1>(a, stream);
    if (chunks <= 8) return launch_layer<T, 8, 1>(a, stream);
    if (chunks <= 16) {
        // short segments (the plan of an L2/MALL-resident graph, graph.choose_seg_len): 8 gathers
        // in flight per lane and more waves per SIMD beat 16 (tools/segprobe.py: ML-1M 37.8 ->
        // 35.8 us, Amazon-book shape 144.3 -> 126.6 us per layer); C4-sized plans keep 16
        if (a.seg_len <= 128) return launch_layer<T, 16, 1, 8>(a, stream);
        return launch_layer<T, 16, 1>(a, stream);
    }
    if (chunks <= 32) return launch_layer<T, 32, 1>(a, stream);
    if (chunks <= 64) return launch_layer<T, 64, 1>(a, stream);
    if (chunks <= 128) return launch_layer<T, 64, 2>(a, stream);
    return launch_layer<T, 64, 4>(a, stream);
}

// the instantiation dispatch_layer launches, as text (lgx_spmm_kernel_name): kept next to it so
// that the two cannot drift apart
template <typename T>
int dispatch_name(int64_t d, int64_t seg_len, char* buf, size_t len) {
    constexpr int VEC = Vec<T>::N;
    const int64_t chunks = d / VEC;
    int G, CPL, U;
    if (chunks <= 4) G = 4, CPL = 1;
    else if (chunks <= 8) G = 8, CPL = 1;
    else if (chunks <= 16) G = 16, CPL = 1;
    else if (chunks <= 32) G = 32, CPL = 1;
    else if (chunks <= 64) G = 64, CPL = 1;
    else if (chunks <= 128) G = 64, CPL = 2;
    else G = 64, CPL = 4;
    U = CPL == 1 ? (G == 16 ? 16 : 8) : (CPL == 2 ? 4 : 2);
    if (G == 16 && CPL == 1 && seg_len <= 128) U = 8;
    snprintf(buf, len, "spmm_segments<%s,%d,%d,%d>", sizeof(T) == 4 ? "f32" : "bf16", G, CPL, U);
    return LGX_OK;
}

template <typename T>
__global__ void to_f32_scaled(const T* __restrict__ src, float* __restrict__ dst, int64_t n) {
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if constexpr (sizeof(T) == 4) dst[i] = src[i];
    else dst[i] = bf16_to_f32(src[i]);
}

int check_csr(const lgx_csr* A, int64_t d, int dtype) {
    LGX_REQUIRE(A && A->indptr, LGX_ERR_INVALID_ARG, "lgx: null CSR operator");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG,
                "lgx: unknown dtype %d", dtype);
    const int vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    LGX_REQUIRE(d > 0 && d % vec == 0 && d <= 1024, LGX_ERR_UNSUPPORTED,
                "lgx: embedding dim %lld must be a multiple of %d and <= 1024", (long long)d, vec);
    const int64_t planned_rows = A->cb_n > 0 ? A->cb_row0 : A->n_rows;
    LGX_REQUIRE(A->n_segs >= planned_rows, LGX_ERR_INVALID_ARG,
                "lgx: plan has %lld segments for %lld rows", (long long)A->n_segs, (long long)planned_rows);
    LGX_REQUIRE(A->seg_row && A->seg_part && A->seg_slot, LGX_ERR_INVALID_ARG, "lgx: CSR plan missing");
    LGX_REQUIRE(A->n_split == 0 || (A->split_row && A->split_ptr && A->partials), LGX_ERR_INVALID_ARG,
                "lgx: split rows need split_row / split_ptr / partials");
    LGX_REQUIRE(A->seg_len > 0, LGX_ERR_INVALID_ARG, "lgx: seg_len must be > 0");
    if (A->cb_n > 0) {
        const int64_t R = A->n_rows - A->cb_row0;
        LGX_REQUIRE(A->cb_row0 >= 0 && R >= 0 && A->cb_ptr && A->cb_plans && (R == 0 || A->cb_carry),
                    LGX_ERR_INVALID_ARG, "lgx: column blocks need cb_ptr / cb_plans / cb_carry");
        LGX_REQUIRE(A->n_segs >= A->cb_row0, LGX_ERR_INVALID_ARG, "lgx: plan misses unblocked rows");
        for (int64_t b = 0; b < A->cb_n; ++b) {
            const lgx_plan& P = A->cb_plans[b];
            LGX_REQUIRE(P.n_segs >= R && P.seg_row && P.seg_part && P.seg_slot && P.seg_len > 0 &&
                            (P.n_split == 0 || (P.split_row && P.split_ptr && P.partials)),
                        LGX_ERR_INVALID_ARG, "lgx: column block %lld has a bad plan", (long long)b);
        }
    } else {
        LGX_REQUIRE(A->cb_n == 0, LGX_ERR_INVALID_ARG, "lgx: cb_n < 0");
    }
    return LGX_OK;
}

// the plan fields of a LayerArgs from a segment plan
inline void set_plan(LayerArgs& a, const int32_t* seg_row, const int32_t* seg_part, const int32_t* seg_slot,
                     int64_t n_segs, int64_t seg_len, const int32_t* split_row, const int32_t* split_ptr,
                     int64_t n_split, float* partials) {
    a.seg_row = seg_row;
    a.seg_part = seg_part;
    a.seg_slot = seg_slot;
    a.n_segs = n_segs;
    a.seg_len = seg_len;
    a.split_row = split_row;
    a.split_ptr = split_ptr;
    a.n_split = n_split;
    a.partials = partials;
}

// one layer over every row of A: the unblocked rows in one launch (+ fix-up), then the column
// blocks in order, the row sums carried between them
template <typename T>
int run_layer(const lgx_csr* A, LayerArgs a, hipStream_t stream) {
    a.indptr = A->indptr;
    a.indices = A->indices;
    a.vals = A->vals;
    a.row_begin = A->indptr;
    a.row_end = A->indptr + 1;
    a.carry = nullptr;
    a.carry_row0 = 0;
    a.carry_mode = kCarryNone;
    set_plan(a, A->seg_row, A->seg_part, A->seg_slot, A->n_segs, A->seg_len, A->split_row, A->split_ptr,
             A->n_split, A->partials);
    int rc = dispatch_layer<T>(a, stream);
    if (rc || A->cb_n <= 0) return rc;
    const int64_t R = A->n_rows - A->cb_row0;
    if (R == 0) return LGX_OK;
    a.carry = A->cb_carry;
    a.carry_row0 = A->cb_row0;
    for (int64_t b = 0; b < A->cb_n; ++b) {
        const lgx_plan& P = A->cb_plans[b];
        set_plan(a, P.seg_row, P.seg_part, P.seg_slot, P.n_segs, P.seg_len, P.split_row, P.split_ptr, P.n_split,
                 P.partials);
        // row r of block b: cb_ptr[b R + (r - cb_row0)], indexed by the global row
        a.row_begin = A->cb_ptr + b * R - A->cb_row0;
        a.row_end = A->cb_ptr + (b + 1) * R - A->cb_row0;
        a.carry_mode = A->cb_n == 1 ? kCarryNone
                       : (b == 0 ? kCarryStore : (b + 1 == A->cb_n ? kCarryTake : kCarryAdd));
        rc = dispatch_layer<T>(a, stream);
        if (rc) return rc;
    }
    return LGX_OK;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_propagate_layer(const lgx_csr* A, const void* X, void* Y, const void* E0,
                                   float* acc, float* out, int64_t d, int dtype, int mode,
                                   float n_mean, lgx_stream_t stream) {
    int rc = check_csr(A, d, dtype);
    if (rc) return rc;
    LGX_REQUIRE(mode >= LGX_LAYER_PLAIN && mode <= LGX_LAYER_PARTIAL, LGX_ERR_INVALID_ARG,
                "lgx_propagate_layer: bad mode %d", mode);
    LGX_REQUIRE(X || A->nnz == 0, LGX_ERR_INVALID_ARG, "lgx_propagate_layer: X is null");
    const bool needY = mode <= LGX_LAYER_MID, needE0 = mode == LGX_LAYER_FIRST || mode == LGX_LAYER_ONLY;
    const bool needAcc = mode >= LGX_LAYER_FIRST && mode <= LGX_LAYER_LAST;
    const bool needOut = mode >= LGX_LAYER_LAST;  // LAST, ONLY, PARTIAL
    LGX_REQUIRE((!needY || Y) && (!needE0 || E0) && (!needAcc || acc) && (!needOut || out),
                LGX_ERR_INVALID_ARG, "lgx_propagate_layer: missing buffer for mode %d", mode);
    LGX_REQUIRE(!needOut || n_mean > 0.0f, LGX_ERR_INVALID_ARG, "lgx_propagate_layer: n_mean <= 0");
    if (A->n_rows == 0) return LGX_OK;
    LayerArgs a{};
    a.X = X;
    a.Y = Y;
    a.E0 = E0;
    a.acc = acc;
    a.out = out;
    a.d = d;
    a.mode = mode;
    a.n_mean = n_mean;
    if (dtype == LGX_DTYPE_F32) return run_layer<float>(A, a, as_hip(stream));
    return run_layer<uint16_t>(A, a, as_hip(stream));
}

extern "C" int lgx_propagate_layer_stack(const lgx_csr* A, const void* X, const void* E0, const void* const* prev,
                                         int n_prev, float* out, int64_t d, int dtype, float n_mean,
                                         lgx_stream_t stream) {
    int rc = check_csr(A, d, dtype);
    if (rc) return rc;
    LGX_REQUIRE(n_prev >= 0 && n_prev <= kMaxPrev && (n_prev == 0 || prev), LGX_ERR_INVALID_ARG,
                "lgx_propagate_layer_stack: n_prev %d outside [0, %d]", n_prev, kMaxPrev);
    LGX_REQUIRE((X || A->nnz == 0) && E0 && out && n_mean > 0.0f, LGX_ERR_INVALID_ARG,
                "lgx_propagate_layer_stack: bad arguments");
    for (int p = 0; p < n_prev; ++p)
        LGX_REQUIRE(prev[p], LGX_ERR_INVALID_ARG, "lgx_propagate_layer_stack: prev[%d] is null", p);
    if (A->n_rows == 0) return LGX_OK;
    LayerArgs a{};
    a.X = X;
    a.E0 = E0;
    a.out = out;
    a.d = d;
    a.mode = LGX_LAYER_STACK;
    a.n_mean = n_mean;
    a.n_prev = n_prev;
    for (int p = 0; p < n_prev; ++p) a.prev[p] = prev[p];
    if (dtype == LGX_DTYPE_F32) return run_layer<float>(A, a, as_hip(stream));
    return run_layer<uint16_t>(A, a, as_hip(stream));
}

namespace lgx {
namespace {
// one thread per 16-B output chunk: the fused path's finish_chunk on precomputed row sums
template <typename T>
__global__ __launch_bounds__(kThreads) void layer_epilogue_kernel(LayerArgs a, const float* __restrict__ y,
                                                                  int64_t rows) {
    constexpr int VEC = Vec<T>::N;
    const int64_t cpr = a.d / VEC;
    const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (c >= rows * cpr) return;
    const int64_t row = c / cpr, off = (c % cpr) * VEC;
    float v[VEC];
#pragma unroll
    for (int j = 0; j < VEC; j += 4) {
        const float4 q = *reinterpret_cast<const float4*>(y + row * a.d + off + j);
        v[j] = q.x; v[j + 1] = q.y; v[j + 2] = q.z; v[j + 3] = q.w;
    }
    finish_chunk<T>(a, row, off, v);
}
// Cross-rank sum of the push partials of the sharded layer (distributed.py): dst = src[0] + src[1]
// + ... + src[n-1], added left to right in fp32, slab j at src + j * slab_elems.  One fixed order,
// so the sum does not depend on how the exchange was chunked or which collective moved the slabs
// (a reduce-scatter's order follows its ring / channel assignment).  HBM-bound: n + 1 slab passes.
__global__ __launch_bounds__(kThreads) void sum_slabs_kernel(const float* __restrict__ src, int64_t n_slabs,
                                                             int64_t slab_elems, int64_t n4, float* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;  // float4 index
    if (i >= n4) return;
    float4 acc = reinterpret_cast<const float4*>(src)[i];
    for (int64_t j = 1; j < n_slabs; ++j) {
        const float4 v = reinterpret_cast<const float4*>(src + j * slab_elems)[i];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = acc;
}

}  // namespace
}  // namespace lgx

extern "C" int lgx_layer_epilogue(const float* y, int64_t rows, void* Y, const void* E0, float* acc, float* out,
                                  int64_t d, int dtype, int mode, float n_mean, lgx_stream_t stream) {
    LGX_REQUIRE(rows >= 0 && d > 0 && (rows == 0 || y), LGX_ERR_INVALID_ARG, "lgx_layer_epilogue: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_layer_epilogue: dtype");
    LGX_REQUIRE(mode >= LGX_LAYER_PLAIN && mode <= LGX_LAYER_ONLY, LGX_ERR_INVALID_ARG,
                "lgx_layer_epilogue: bad mode %d", mode);
    const int vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    LGX_REQUIRE(d % vec == 0, LGX_ERR_UNSUPPORTED, "lgx_layer_epilogue: d=%lld must be a multiple of %d",
                (long long)d, vec);
    const bool needY = mode <= LGX_LAYER_MID, needE0 = mode == LGX_LAYER_FIRST || mode == LGX_LAYER_ONLY;
    const bool needAcc = mode >= LGX_LAYER_FIRST && mode <= LGX_LAYER_LAST, needOut = mode >= LGX_LAYER_LAST;
    LGX_REQUIRE((!needY || Y) && (!needE0 || E0) && (!needAcc || acc) && (!needOut || out),
                LGX_ERR_INVALID_ARG, "lgx_layer_epilogue: missing buffer for mode %d", mode);
    LGX_REQUIRE(!needOut || n_mean > 0.0f, LGX_ERR_INVALID_ARG, "lgx_layer_epilogue: n_mean <= 0");
    if (rows == 0) return LGX_OK;
    LayerArgs a{};
    a.Y = Y;
    a.E0 = E0;
    a.acc = acc;
    a.out = out;
    a.d = d;
    a.mode = mode;
    a.n_mean = n_mean;
    const int64_t chunks = rows * (d / vec);
    const unsigned grid = (unsigned)ceil_div(chunks, (int64_t)kThreads);
    if (dtype == LGX_DTYPE_F32) layer_epilogue_kernel<float><<<grid, kThreads, 0, as_hip(stream)>>>(a, y, rows);
    else layer_epilogue_kernel<uint16_t><<<grid, kThreads, 0, as_hip(stream)>>>(a, y, rows);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_sum_slabs(const float* src, int64_t n_slabs, int64_t slab_elems, float* dst,
                             lgx_stream_t stream) {
    LGX_REQUIRE(n_slabs >= 1 && slab_elems >= 0 && (slab_elems == 0 || (src && dst)), LGX_ERR_INVALID_ARG,
                "lgx_sum_slabs: bad arguments");
    LGX_REQUIRE(slab_elems % 4 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0,
                LGX_ERR_UNSUPPORTED, "lgx_sum_slabs: slabs must be whole, 16-B aligned float4 runs");
    if (slab_elems == 0) return LGX_OK;
    const int64_t n4 = slab_elems / 4;
    sum_slabs_kernel<<<(unsigned)ceil_div(n4, (int64_t)kThreads), kThreads, 0, as_hip(stream)>>>(src, n_slabs,
                                                                                              slab_elems, n4, dst);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_spmm_kernel_name(int64_t d, int dtype, int64_t seg_len, char* buf, size_t len) {
    LGX_REQUIRE(buf && len > 0 && d > 0 && seg_len > 0, LGX_ERR_INVALID_ARG, "lgx_spmm_kernel_name: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_spmm_kernel_name: dtype");
    return dtype == LGX_DTYPE_F32 ? dispatch_name<float>(d, seg_len, buf, len)
                                  : dispatch_name<uint16_t>(d, seg_len, buf, len);
}

extern "C" int lgx_spmm_csr(const lgx_csr* A, const void* X, void* Y, int64_t d, int dtype,
                            lgx_stream_t stream) {
    return lgx_propagate_layer(A, X, Y, nullptr, nullptr, nullptr, d, dtype, LGX_LAYER_PLAIN, 1.0f, stream);
}

extern "C" int lgx_propagate_workspace(int64_t n_rows, int64_t d, int dtype, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && n_rows >= 0 && d > 0, LGX_ERR_INVALID_ARG, "lgx_propagate_workspace: bad args");
    const size_t es = dtype == LGX_DTYPE_F32 ? 4 : 2;
    *ws_bytes = 2 * align_up(n_rows * d * es) + align_up(n_rows * d * 4);
    return LGX_OK;
}

extern "C" int lgx_propagate(const lgx_csr* A, const void* E0, float* out, int64_t d, int K,
                             int dtype, void* ws, size_t ws_bytes, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    int rc = check_csr(A, d, dtype);
    if (rc) return rc;
    LGX_REQUIRE(E0 && out && K >= 0, LGX_ERR_INVALID_ARG, "lgx_propagate: bad arguments");
    LGX_REQUIRE(A->n_rows == A->n_cols, LGX_ERR_INVALID_ARG, "lgx_propagate: operator must be square");
    const int64_t N = A->n_rows;
    if (N == 0) return LGX_OK;
    if (K == 0) {  // mean of the single layer E0
        const int64_t n = N * d;
        if (dtype == LGX_DTYPE_F32)
            to_f32_scaled<float><<<ceil_div(n, 256), 256, 0, stream>>>(static_cast<const float*>(E0), out, n);
        else
            to_f32_scaled<uint16_t><<<ceil_div(n, 256), 256, 0, stream>>>(static_cast<const uint16_t*>(E0), out, n);
        LGX_LAUNCH_CHECK();
        return LGX_OK;
    }
    size_t need = 0;
    lgx_propagate_workspace(N, d, dtype, &need);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_propagate: workspace %zu < %zu", ws_bytes, need);
    const size_t es = dtype == LGX_DTYPE_F32 ? 4 : 2;
    char* base = static_cast<char*>(ws);
    const float n_mean = (float)(K + 1);
    // keep the K-1 intermediate tables when they fit the workspace: the last layer forms the mean
    // from them (no f32 running sum read and written by every layer)
    const size_t tbl = align_up(N * d * es);
    if (K >= 2 && K - 1 <= kMaxPrev && (size_t)(K - 1) * tbl <= ws_bytes) {
        const void* prev[kMaxPrev];
        const void* X = E0;
        for (int k = 1; k < K; ++k) {
            void* Y = base + (size_t)(k - 1) * tbl;
            rc = lgx_propagate_layer(A, X, Y, nullptr, nullptr, nullptr, d, dtype, LGX_LAYER_PLAIN, 1.0f, stream_);
            if (rc) return rc;
            prev[k - 1] = Y;
            X = Y;
        }
        return lgx_propagate_layer_stack(A, X, E0, prev, K - 1, out, d, dtype, n_mean, stream_);
    }
    void* buf[2] = {base, base + tbl};
    float* acc = reinterpret_cast<float*>(base + 2 * tbl);
    const void* X = E0;
    for (int k = 1; k <= K; ++k) {
        int mode;
        if (K == 1) mode = LGX_LAYER_ONLY;
        else if (k == 1) mode = LGX_LAYER_FIRST;
        else if (k == K) mode = LGX_LAYER_LAST;
        else mode = LGX_LAYER_MID;
        void* Y = buf[k & 1];
        rc = lgx_propagate_layer(A, X, Y, E0, acc, out, d, dtype, mode, n_mean, stream_);
        if (rc) return rc;
        X = Y;
    }
    return LGX_OK;
}
