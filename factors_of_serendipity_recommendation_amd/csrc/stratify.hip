// stratified candidate sets on the GPU.
//
// Reference: recommend.create_candidates_stratification (recommend.py:359-452) with
// create_candidates_stratification_sub / sample_list (:314-356):
//   mat_dis   = (E_user . E_item^T).astype(float16)                                   (:375)
//   label     = floor((mat_dis - min_dis) / inter).astype(int8),
//               inter = (max(mat_dis) + epsilon - min(mat_dis)) / num_fold           (:377-381)
//   per user: the items outside its train set, grouped by label; from every group
//             rint(K * |group| / |items|) items at random, shuffled; then sample_list pads (by
//             re-drawing from the list) or trims the list to K                         (:327-356)
//
// lgx_strat_labels   one workgroup per user row of precomputed fp32 scores: the float16 arithmetic
//                    of numpy (each operation in float, rounded to half), the train mask (label -1)
//                    and the per-user label histogram (LDS atomics, one global add per bin).
// lgx_strat_select   one workgroup per user: every eligible item gets a distinct 64-bit hash key, and
//                    a radix select over 8 x 8-bit digits -- all labels at once, histograms in LDS --
//                    finds each label's threshold so that exactly its n smallest keys are taken: a
//                    uniform random subset.  The picks are ordered by key (a random order, fixed by the
//                    seed) and padded / trimmed to K as sample_list does.  The reference draws with
//                    pandas' global numpy generator, so the sets match in distribution, not in bits.
#include "lgx_common.h"

#include <hip/hip_fp16.h>

#include <algorithm>
#include <cfloat>
#include <cstring>

namespace lgx {
namespace {

constexpr int kStratThreads = 256;
constexpr int kMaxFolds = 32;
constexpr int kMaxStratK = 1024;  // candidates per user that the selection kernel keeps in LDS
constexpr int kMaxCand = 2048;    // fast-path candidates (12 B each) in the radix histogram's 32 KB

__host__ __device__ __forceinline__ float half_round(float x) { return __half2float(__float2half_rn(x)); }

__host__ __device__ __forceinline__ int label_of(float sc, float min16, float inter16, int num_fold) {
    // numpy float16: every operation in float, rounded back to half
    const float d = half_round(half_round(sc) - min16);
    const float q = half_round(d / inter16);
    if (!(q < (float)num_fold)) return num_fold;  // the top bin is label num_fold (also q = +inf)
    if (q < 0.0f) return 0;                       // scores below min_dis (d >= 0 for real rows)
    return (int)floorf(q);
}

// Labels of every item first (4 per thread and float4 / 32-bit accesses when rows are 16-B
// aligned), then the user's train items are relabelled -1 and taken out of the histogram: one
// pass over the row instead of a binary search of the mask per item.
template <bool VEC4>
__global__ __launch_bounds__(kStratThreads) void strat_labels_kernel(const float* __restrict__ scores, int64_t n_items,
                                                                    float min16, float inter16, int num_fold,
                                                                    const int64_t* __restrict__ mask_indptr,
                                                                    const int32_t* __restrict__ mask_indices,
                                                                    int8_t* __restrict__ labels,
                                                                    int32_t* __restrict__ hist) {
    // per-thread counters (column = thread: conflict-free, no atomics) -- one LDS atomic per item on
    // ~10 hot bins serialised the whole row; summed into h after the sweep
    __shared__ uint32_t hp[kMaxFolds * kStratThreads];
    __shared__ int32_t h[kMaxFolds];
    const int64_t u = blockIdx.x;
    const int tid = threadIdx.x;
#pragma unroll
    for (int b = 0; b < kMaxFolds; ++b) hp[b * kStratThreads + tid] = 0;
    __syncthreads();
    const float* s = scores + u * n_items;
    int8_t* lab = labels + u * n_items;
    if (VEC4) {
        // 4 float4 loads in flight per thread per iteration
        constexpr int kU = 4;
        const int64_t n4 = n_items >> 2;
        for (int64_t q0 = threadIdx.x; q0 < n4; q0 += kU * kStratThreads) {
            float4 v[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int64_t q = q0 + j * kStratThreads;
                v[j] = q < n4 ? reinterpret_cast<const float4*>(s)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const int64_t q = q0 + j * kStratThreads;
                if (q >= n4) break;
                const int l0 = label_of(v[j].x, min16, inter16, num_fold), l1 = label_of(v[j].y, min16, inter16, num_fold);
                const int l2 = label_of(v[j].z, min16, inter16, num_fold), l3 = label_of(v[j].w, min16, inter16, num_fold);
                hp[l0 * kStratThreads + tid] += 1;
                hp[l1 * kStratThreads + tid] += 1;
                hp[l2 * kStratThreads + tid] += 1;
                hp[l3 * kStratThreads + tid] += 1;
                reinterpret_cast<uint32_t*>(lab)[q] = (uint32_t)(l0 & 255) | ((uint32_t)(l1 & 255) << 8) |
                                                      ((uint32_t)(l2 & 255) << 16) | ((uint32_t)(l3 & 255) << 24);
            }
        }
    } else {
        for (int64_t i = threadIdx.x; i < n_items; i += kStratThreads) {
            const int lv = label_of(s[i], min16, inter16, num_fold);
            hp[lv * kStratThreads + tid] += 1;
            lab[i] = (int8_t)lv;
        }
    }
    __syncthreads();
    if (tid < kMaxFolds) {
        uint32_t c = 0;
        for (int t = 0; t < kStratThreads; ++t) c += hp[tid * kStratThreads + ((t + tid) & (kStratThreads - 1))];
        h[tid] = (int32_t)c;
    }
    __syncthreads();  // the row's labels (global) and counts are complete before the mask fix-up
    if (mask_indptr) {
        const int64_t m0 = mask_indptr[u], m1 = mask_indptr[u + 1];
        for (int64_t j = m0 + threadIdx.x; j < m1; j += kStratThreads) {
            const int32_t it = mask_indices[j];
            if (it < 0 || it >= n_items || (j > m0 && mask_indices[j - 1] == it)) continue;  // sorted: skip repeats
            atomicSub(&h[label_of(s[it], min16, inter16, num_fold)], 1);
            lab[it] = -1;
        }
    }
    __syncthreads();
    if (threadIdx.x <= num_fold) hist[u * (num_fold + 1) + threadIdx.x] = h[threadIdx.x];
}

// Counts of an int8 label row (per-thread LDS counters, summed per bin), then the masked items
// relabelled -1 and taken out: the tail of strat_labels_kernel for rows the fused scoring kernel
// (lgx_strat_labels_fused) labelled.  16 labels per 16-B load when the rows allow it.
template <bool VEC16>
__global__ __launch_bounds__(kStratThreads) void strat_hist_kernel(int8_t* __restrict__ labels, int64_t n_items,
                                                                  int num_fold, const int64_t* __restrict__ mask_indptr,
                                                                  const int32_t* __restrict__ mask_indices,
                                                                  int32_t* __restrict__ hist) {
    __shared__ uint32_t hp[kMaxFolds * kStratThreads];
    __shared__ int32_t h[kMaxFolds];
    const int64_t u = blockIdx.x;
    const int tid = threadIdx.x;
#pragma unroll
    for (int b = 0; b < kMaxFolds; ++b) hp[b * kStratThreads + tid] = 0;
    __syncthreads();
    int8_t* lab = labels + u * n_items;
    if (VEC16) {
        const int64_t n16 = n_items >> 4;
        for (int64_t q = tid; q < n16; q += kStratThreads) {
            const uint4 w = reinterpret_cast<const uint4*>(lab)[q];
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int j = 0; j < 16; ++j) hp[((ws[j >> 2] >> (8 * (j & 3))) & 255) * kStratThreads + tid] += 1;
        }
    } else {
        for (int64_t i = tid; i < n_items; i += kStratThreads) hp[(uint8_t)lab[i] * kStratThreads + tid] += 1;
    }
    __syncthreads();
    if (tid < kMaxFolds) {
        uint32_t c = 0;
        for (int t = 0; t < kStratThreads; ++t) c += hp[tid * kStratThreads + ((t + tid) & (kStratThreads - 1))];
        h[tid] = (int32_t)c;
    }
    __syncthreads();
    if (mask_indptr) {
        const int64_t m0 = mask_indptr[u], m1 = mask_indptr[u + 1];
        for (int64_t j = m0 + threadIdx.x; j < m1; j += kStratThreads) {
            const int32_t it = mask_indices[j];
            if (it < 0 || it >= n_items || (j > m0 && mask_indices[j - 1] == it)) continue;  // sorted: skip repeats
            atomicSub(&h[lab[it]], 1);
            lab[it] = -1;
        }
    }
    __syncthreads();
    if (threadIdx.x <= num_fold) hist[u * (num_fold + 1) + threadIdx.x] = h[threadIdx.x];
}

// The masked items of labelled rows relabelled -1 and taken out of the counts: one thread per mask
// entry (sorted rows: repeats skipped)
__global__ __launch_bounds__(kStratThreads) void strat_mask_kernel(int8_t* __restrict__ labels, int64_t n_items,
                                                                  int num_fold,
                                                                  const int64_t* __restrict__ mask_indptr,
                                                                  const int32_t* __restrict__ mask_indices,
                                                                  int32_t* __restrict__ hist) {
    const int64_t u = blockIdx.y;
    const int64_t m0 = mask_indptr[u], m1 = mask_indptr[u + 1];
    for (int64_t j = m0 + (int64_t)blockIdx.x * kStratThreads + threadIdx.x; j < m1;
         j += (int64_t)gridDim.x * kStratThreads) {
        const int32_t it = mask_indices[j];
        if (it < 0 || it >= n_items || (j > m0 && mask_indices[j - 1] == it)) continue;
        int8_t* p = labels + u * n_items + it;
        const int l = *p;
        if (l < 0 || l > num_fold) continue;
        atomicSub(hist + u * (num_fold + 1) + l, 1);
        *p = -1;
    }
}

// per-user random order of the items: high word = a 32-bit bijection of the item index (odd
// multiply, xor with the user's seed word, murmur3 fmix32), low word = the index -- distinct keys,
// ~7 32-bit ops per item instead of two 64-bit splitmix rounds (the select's dominant cost)
__device__ __forceinline__ uint32_t user_seed_word(uint64_t seed, int64_t u) {
    return (uint32_t)(splitmix64(seed ^ splitmix64((uint64_t)u ^ 0xA5A5A5A5ull)) >> 32);
}
__device__ __forceinline__ uint32_t item_hash(uint32_t us, int64_t i) {
    uint32_t x = ((uint32_t)i * 0x9E3779B1u) ^ us;
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint64_t item_key(uint32_t us, int64_t i) {
    return ((uint64_t)item_hash(us, i) << 32) | (uint32_t)i;
}

// Ascending bitonic sort of n (a power of two) (key, value) pairs in LDS by the whole workgroup;
// the caller pads with ~0 keys.  O(n log^2 n / threads) with one barrier per stage, instead of the
// O(n^2 / threads) rank loop whose LDS reads each waited on the one before.
__device__ __forceinline__ void lds_bitonic(uint64_t* k, int32_t* v, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (int t = threadIdx.x; t < n / 2; t += kStratThreads) {
                const int i = 2 * t - (t & (stride - 1)), j = i + stride;
                const uint64_t a = k[i], b = k[j];
                if ((a > b) == ((i & size) == 0)) {
                    k[i] = b;
                    k[j] = a;
                    const int32_t x = v[i];
                    v[i] = v[j];
                    v[j] = x;
                }
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int pow2_at_least(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// np.rint: round half to even
__device__ __forceinline__ int64_t rint_even(double x) { return (int64_t)rint(x); }

template <bool VEC16>
__global__ __launch_bounds__(kStratThreads) void strat_select_kernel(const int8_t* __restrict__ labels, int64_t n_items,
                                                                    const int32_t* __restrict__ hist, int n_bins,
                                                                    const int32_t* __restrict__ targets, uint64_t seed,
                                                                    int32_t* __restrict__ out, int out_stride,
                                                                    int32_t* __restrict__ out_count, int force_exact) {
    // per (label, 8-bit digit) counts of the exact radix path; the fast path keeps its candidates
    // (keys, items, labels) in the same bytes
    __shared__ __attribute__((aligned(16))) uint32_t dh[kMaxFolds * 256];
    __shared__ int32_t n_cand, cand_l[kMaxFolds];
    __shared__ uint64_t cut[kMaxFolds];
    __shared__ int fast_ok;
    __shared__ int64_t need[kMaxFolds];       // keys still to take below the threshold being refined
    __shared__ uint64_t prefix[kMaxFolds];    // threshold bits fixed so far
    __shared__ uint64_t keys_sh[kMaxStratK];
    __shared__ int32_t items_sh[kMaxStratK];
    __shared__ int32_t n_sel;
    // high word of cut[l] by the label's byte (0 for labels with nothing to take and for -1 = 255):
    // the per-item test is one hash and one compare against it; the full key test runs only for
    // the few items at or under it
    __shared__ uint32_t cut_hi[256];
    const int64_t u = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t us = user_seed_word(seed, u);
    const int8_t* lab = labels + u * n_items;
    // per-label quotas: K = min(target, eligible items), n_l = rint(K * hist_l / eligible)
    const int target = min(targets[u], out_stride);
    if (tid == 0) {
        int64_t total = 0;
        for (int l = 0; l < n_bins; ++l) total += hist[u * n_bins + l];
        const int64_t K = min<int64_t>(target, total);
        for (int l = 0; l < n_bins; ++l) {
            need[l] = total > 0 ? rint_even((double)K * hist[u * n_bins + l] / (double)total) : 0;
            prefix[l] = 0;
        }
        n_sel = 0;
    }
    __syncthreads();
    // Fast path: the keys are uniform 64-bit hashes, so the need[l] smallest of label l lie below
    // cut[l] = 2^64 (need[l] + 6 sqrt(need[l]) + 16) / hist[l] but for a ~5.7-sigma shortfall (a
    // 4-sigma margin failed for ~1 user per 4096-user batch, and that user's 8-pass radix select
    // stretched the launch 2.3 -> 11 ms).  One pass gathers every key under its label's cut into LDS
    // (expected K + 6 sum sqrt(need) + 16 n_bins, ~1840 at K = 1024 over 11 labels, under the 2048
    // slots), and the exact need[l] smallest per label are ranked there: the same picks as the radix
    // select below, which runs only when a label came up short or the buffer overflowed.
    uint64_t* ck = reinterpret_cast<uint64_t*>(dh);
    int32_t* ci = reinterpret_cast<int32_t*>(ck + kMaxCand);
    if (tid < n_bins) {
        const int64_t hl = hist[u * n_bins + tid], nl = need[tid];
        const double frac = hl > 0 ? ((double)nl + 6.0 * sqrt((double)nl) + 16.0) / (double)hl : 2.0;
        cut[tid] = nl <= 0 ? 0ull : (frac >= 1.0 ? ~0ull : (uint64_t)(frac * 18446744073709551616.0));
        cand_l[tid] = 0;
    }
    if (tid == 0) n_cand = 0;
    __syncthreads();
    cut_hi[tid] = (tid < n_bins && need[tid] > 0) ? (uint32_t)(cut[tid] >> 32) : 0u;
    __syncthreads();
    // a candidate's sort key: label above the hash (the hash is a bijection of the item index, so
    // ordering by it orders by the full (hash, item) key)
    auto consider = [&](int64_t i, int l) {
        const uint32_t x = item_hash(us, i);
        if (x > cut_hi[l & 255]) return;  // most items stop here
        if (l < 0 || l >= n_bins || need[l] <= 0) return;
        if (item_key(us, i) > cut[l]) return;
        atomicAdd(&cand_l[l], 1);
        const int slot = atomicAdd(&n_cand, 1);
        if (slot < kMaxCand) {
            ck[slot] = ((uint64_t)l << 32) | x;
            ci[slot] = (int32_t)i;
        }
    };
    if (VEC16) {  // 16 labels per 16-B load; the 16 table lookups issue together, then the rare hits
        const int64_t n16 = n_items >> 4;
        for (int64_t q = tid; q < n16; q += kStratThreads) {
            const uint4 w = reinterpret_cast<const uint4*>(lab)[q];
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
            uint32_t hit = 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t lb = (ws[j >> 2] >> (8 * (j & 3))) & 255u;
                hit |= (item_hash(us, 16 * q + j) <= cut_hi[lb] ? 1u : 0u) << j;
            }
            while (hit) {
                const int j = __builtin_ctz(hit);
                hit &= hit - 1;
                consider(16 * q + j, (int)(int8_t)(ws[j >> 2] >> (8 * (j & 3))));
            }
        }
    } else {
        for (int64_t i = tid; i < n_items; i += kStratThreads) consider(i, lab[i]);
    }
    __syncthreads();
    if (tid == 0) {
        int ok = n_cand <= kMaxCand && !force_exact;
        for (int l = 0; l < n_bins; ++l) ok &= need[l] <= 0 || cand_l[l] >= need[l];
        fast_ok = ok;
    }
    __syncthreads();
    if (fast_ok) {
        // sort the candidates by (label, hash): label l's run starts at the count of the labels
        // below it, and its first need[l] entries are its picks (placed at fixed slots, no atomics)
        const int m = n_cand, P = pow2_at_least(m);
        for (int a = m + tid; a < P; a += kStratThreads) ck[a] = ~0ull;
        lds_bitonic(ck, ci, P);
        __shared__ int32_t run0[kMaxFolds], pick0[kMaxFolds];
        if (tid == 0) {
            int r = 0, q = 0;
            for (int l = 0; l < n_bins; ++l) {
                run0[l] = r;
                pick0[l] = q;
                r += cand_l[l];
                q += need[l] > 0 ? (int)need[l] : 0;
            }
            n_sel = q;
        }
        __syncthreads();
        for (int a = tid; a < m; a += kStratThreads) {
            const int l = (int)(ck[a] >> 32), r = a - run0[l];
            const int slot = pick0[l] + r;
            if (r < need[l] && slot < kMaxStratK) {
                keys_sh[slot] = ((ck[a] & 0xffffffffull) << 32) | (uint32_t)ci[a];
                items_sh[slot] = ci[a];
            }
        }
        __syncthreads();
    }
    // radix select, 8 passes of 8 bits from the top: after pass p, prefix[l] holds the top 8(p+1)
    // bits of the need[l]-th smallest key of label l (need[l] counts down the keys already below it)
    for (int pass = 0; pass < 8 && !fast_ok; ++pass) {
        const int shift = 56 - 8 * pass;
        for (int j = tid; j < n_bins * 256; j += kStratThreads) dh[j] = 0;
        __syncthreads();
        for (int64_t i = tid; i < n_items; i += kStratThreads) {
            const int l = lab[i];
            if (l < 0 || l >= n_bins || need[l] <= 0) continue;
            const uint64_t k = item_key(us, i);
            const uint64_t hi_mask = pass == 0 ? 0ull : (~0ull << (shift + 8));
            if ((k & hi_mask) != prefix[l]) continue;
            atomicAdd(&dh[l * 256 + ((k >> shift) & 255)], 1u);
        }
        __syncthreads();
        if (tid < n_bins && need[tid] > 0) {
            int64_t acc = 0;
            int dsel = 255;
            for (int dgt = 0; dgt < 256; ++dgt) {
                const int64_t c = dh[tid * 256 + dgt];
                if (acc + c >= need[tid]) {
                    dsel = dgt;
                    break;
                }
                acc += c;
            }
            need[tid] -= acc;  // keys strictly below the chosen digit are taken
            prefix[tid] |= (uint64_t)dsel << shift;
        }
        __syncthreads();
    }
    // take every key below the label's threshold, plus need[l] keys equal to it (keys are distinct,
    // so at most the one threshold key itself)
    for (int64_t i = tid; i < n_items && !fast_ok; i += kStratThreads) {
        const int l = lab[i];
        if (l < 0 || l >= n_bins) continue;
        const uint64_t k = item_key(us, i);
        bool take = false;
        if (k < prefix[l]) take = true;
        else if (k == prefix[l] && need[l] > 0)  // signed: the count may go below zero under contention
            take = (int64_t)atomicAdd((unsigned long long*)&need[l], (unsigned long long)-1) > 0;
        if (take) {
            const int slot = atomicAdd(&n_sel, 1);
            if (slot < kMaxStratK) {
                keys_sh[slot] = k;
                items_sh[slot] = (int32_t)i;
            }
        }
    }
    __syncthreads();
    const int n = min(n_sel, kMaxStratK);
    // order the picks by key (keys are distinct): a random order fixed by the seed
    {
        const int P = pow2_at_least(n);
        for (int a = n + tid; a < P; a += kStratThreads) keys_sh[a] = ~0ull;
        lds_bitonic(keys_sh, items_sh, P);
    }
    const int32_t* ranked = items_sh;
    // sample_list (recommend.py:314-325): trim to K, or pad with distinct draws from the list
    const int K = target;
    int32_t* o = out + u * (int64_t)out_stride;
    const int written = n >= K ? K : min(K, 2 * n);
    for (int j = tid; j < written; j += kStratThreads) o[j] = ranked[j < n ? j : j - n];
    if (tid == 0) out_count[u] = written;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_strat_labels(const float* scores, int64_t n_users, int64_t n_items, float min16, float inter16,
                                int num_fold, const int64_t* mask_indptr, const int32_t* mask_indices, int8_t* labels,
                                int32_t* hist, lgx_stream_t stream) {
    LGX_REQUIRE(n_users >= 0 && n_items >= 0 && num_fold >= 1 && num_fold < kMaxFolds && n_items < INT32_MAX,
                LGX_ERR_INVALID_ARG, "lgx_strat_labels: bad sizes (num_fold in [1, %d))", kMaxFolds);
    LGX_REQUIRE(inter16 > 0.0f, LGX_ERR_INVALID_ARG, "lgx_strat_labels: inter must be > 0");
    if (n_users == 0) return LGX_OK;
    LGX_REQUIRE(scores && labels && hist && (!mask_indptr || mask_indices), LGX_ERR_INVALID_ARG,
                "lgx_strat_labels: null pointer");
    const bool vec4 = n_items % 4 == 0 && ((uintptr_t)scores & 15) == 0 && ((uintptr_t)labels & 3) == 0;
    if (vec4)
        strat_labels_kernel<true><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            scores, n_items, min16, inter16, num_fold, mask_indptr, mask_indices, labels, hist);
    else
        strat_labels_kernel<false><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            scores, n_items, min16, inter16, num_fold, mask_indptr, mask_indices, labels, hist);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_strat_hist(int8_t* labels, int64_t n_users, int64_t n_items, int num_fold,
                              const int64_t* mask_indptr, const int32_t* mask_indices, int32_t* hist,
                              lgx_stream_t stream) {
    LGX_REQUIRE(n_users >= 0 && n_items >= 0 && num_fold >= 1 && num_fold < kMaxFolds && n_items < INT32_MAX,
                LGX_ERR_INVALID_ARG, "lgx_strat_hist: bad sizes (num_fold in [1, %d))", kMaxFolds);
    if (n_users == 0) return LGX_OK;
    LGX_REQUIRE(labels && hist && (!mask_indptr || mask_indices), LGX_ERR_INVALID_ARG, "lgx_strat_hist: null pointer");
    const bool vec16 = n_items % 16 == 0 && ((uintptr_t)labels & 15) == 0;
    if (vec16)
        strat_hist_kernel<true><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            labels, n_items, num_fold, mask_indptr, mask_indices, hist);
    else
        strat_hist_kernel<false><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            labels, n_items, num_fold, mask_indptr, mask_indices, hist);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_strat_mask(int8_t* labels, int64_t n_users, int64_t n_items, int num_fold,
                              const int64_t* mask_indptr, const int32_t* mask_indices, int32_t* hist,
                              lgx_stream_t stream) {
    LGX_REQUIRE(n_users >= 0 && n_items >= 0 && num_fold >= 1 && num_fold < kMaxFolds, LGX_ERR_INVALID_ARG,
                "lgx_strat_mask: bad sizes");
    if (n_users == 0 || !mask_indptr) return LGX_OK;
    LGX_REQUIRE(labels && hist && mask_indices, LGX_ERR_INVALID_ARG, "lgx_strat_mask: null pointer");
    // grid.y is capped at 65535: users beyond it go in further launches
    for (int64_t u0 = 0; u0 < n_users; u0 += 65535) {
        const int64_t nu = std::min<int64_t>(65535, n_users - u0);
        strat_mask_kernel<<<dim3(1, (unsigned)nu), kStratThreads, 0, as_hip(stream)>>>(
            labels + u0 * n_items, n_items, num_fold, mask_indptr + u0, mask_indices, hist + u0 * (num_fold + 1));
        LGX_LAUNCH_CHECK();
    }
    return LGX_OK;
}

// The label of a score is a monotone step function of it (each float16 rounding, the subtraction,
// the division by inter16 > 0 and the floor are monotone), so thr[j-1] = the smallest f32 x with
// label_of(x) >= j, found by bisection over the ordered f32 bit patterns, gives
// label_of(s) = #{j : s >= thr[j-1]} for every finite s.
extern "C" int lgx_strat_thresholds(float min16, float inter16, int num_fold, float* thr) {
    LGX_REQUIRE(thr && num_fold >= 1 && num_fold < kMaxFolds && inter16 > 0.0f, LGX_ERR_INVALID_ARG,
                "lgx_strat_thresholds: bad arguments");
    auto key = [](float f) {  // order-preserving f32 -> int64
        int32_t b;
        memcpy(&b, &f, 4);
        return b >= 0 ? (int64_t)b : -(int64_t)(b & 0x7fffffff);
    };
    auto unkey = [](int64_t k) {
        const int32_t b = k >= 0 ? (int32_t)k : (int32_t)((uint32_t)(-k) | 0x80000000u);
        float f;
        memcpy(&f, &b, 4);
        return f;
    };
    const int64_t kmin = key(-FLT_MAX), kmax = key(FLT_MAX);
    for (int j = 1; j <= num_fold; ++j) {
        int64_t lo = kmin, hi = kmax;  // invariant: label(unkey(hi)) >= j, or hi == kmax
        if (label_of(unkey(hi), min16, inter16, num_fold) < j) {
            thr[j - 1] = INFINITY;  // no finite score reaches label j
            continue;
        }
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (label_of(unkey(mid), min16, inter16, num_fold) >= j) hi = mid;
            else lo = mid + 1;
        }
        thr[j - 1] = unkey(lo);
    }
    return LGX_OK;
}

extern "C" int lgx_strat_select_ex(const int8_t* labels, int64_t n_users, int64_t n_items, const int32_t* hist,
                                   int n_bins, const int32_t* targets, uint64_t seed, int32_t* out, int out_stride,
                                   int32_t* out_count, int flags, lgx_stream_t stream) {
    LGX_REQUIRE((flags & ~LGX_STRAT_EXACT) == 0, LGX_ERR_INVALID_ARG, "lgx_strat_select: unknown flags 0x%x", flags);
    LGX_REQUIRE(n_users >= 0 && n_items >= 0 && n_bins >= 1 && n_bins <= kMaxFolds && n_items < INT32_MAX,
                LGX_ERR_INVALID_ARG, "lgx_strat_select: bad sizes (n_bins in [1, %d])", kMaxFolds);
    LGX_REQUIRE(out_stride >= 1 && out_stride <= kMaxStratK, LGX_ERR_UNSUPPORTED,
                "lgx_strat_select: at most %d candidates per user", kMaxStratK);
    if (n_users == 0) return LGX_OK;
    LGX_REQUIRE(labels && hist && targets && out && out_count, LGX_ERR_INVALID_ARG, "lgx_strat_select: null pointer");
    const bool vec16 = n_items % 16 == 0 && ((uintptr_t)labels & 15) == 0;
    // LGX_STRAT_EXACT skips the cut-and-rank fast path (the radix select must pick the same sets)
    const int force_exact = (flags & LGX_STRAT_EXACT) ? 1 : 0;
    if (vec16)
        strat_select_kernel<true><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            labels, n_items, hist, n_bins, targets, seed, out, out_stride, out_count, force_exact);
    else
        strat_select_kernel<false><<<(unsigned)n_users, kStratThreads, 0, as_hip(stream)>>>(
            labels, n_items, hist, n_bins, targets, seed, out, out_stride, out_count, force_exact);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_strat_select(const int8_t* labels, int64_t n_users, int64_t n_items, const int32_t* hist,
                                int n_bins, const int32_t* targets, uint64_t seed, int32_t* out, int out_stride,
                                int32_t* out_count, lgx_stream_t stream) {
    return lgx_strat_select_ex(labels, n_users, n_items, hist, n_bins, targets, seed, out, out_stride, out_count, 0,
                               stream);
}
