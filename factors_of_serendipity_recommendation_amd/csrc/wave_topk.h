// Wave64 top-k helpers shared by the scoring / top-k kernels.
//
// An entry (score, index) is packed into one 64-bit key that orders exactly like the ranking
// used everywhere in this library -- higher score first, ties broken by the LOWER index:
//     key = ord(score) << 32 | (0xffffffff - index)
// ord() maps IEEE floats to unsigned ints monotonically; key 0 is "empty" and loses to every
// real entry (including -inf scores).  A wave keeps a running top-k list with lane j holding the
// j-th best key; a batch of 64 new keys (one per lane) is merged by a filter against the k-th
// key, a bitonic sort of the survivors and one bitonic merge -- all in registers via shuffles.
#pragma once

#include "lgx_common.h"

namespace lgx {

__device__ __forceinline__ uint32_t ord_f32(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u ^ 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t o) {
    return __uint_as_float((o & 0x80000000u) ? (o ^ 0x80000000u) : ~o);
}
__device__ __forceinline__ uint64_t make_key(float s, int32_t idx) {
    return ((uint64_t)ord_f32(s) << 32) | (uint64_t)(0xffffffffu - (uint32_t)idx);
}
__device__ __forceinline__ float key_score(uint64_t k) { return unord_f32((uint32_t)(k >> 32)); }
__device__ __forceinline__ int32_t key_index(uint64_t k) {
    return (int32_t)(0xffffffffu - (uint32_t)(k & 0xffffffffu));
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const int lo = __shfl((int)(uint32_t)v, src, 64);
    const int hi = __shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const int hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// full bitonic sort of 64 keys (one per lane), descending: lane 0 holds the largest
__device__ __forceinline__ uint64_t wave_sort_desc(uint64_t key, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = shfl_xor_u64(key, j);
            const bool desc = (lane & k) == 0;
            const bool low = (lane & j) == 0;
            const bool big = desc == low;
            key = big ? (key > o ? key : o) : (key < o ? key : o);
        }
    }
    return key;
}

// sort a bitonic sequence descending
__device__ __forceinline__ uint64_t wave_merge_desc(uint64_t key, int lane) {
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        const uint64_t o = shfl_xor_u64(key, j);
        const bool low = (lane & j) == 0;
        key = low ? (key > o ? key : o) : (key < o ? key : o);
    }
    return key;
}

// Merge one batch of 64 candidate keys into the running list `top` (lane j = j-th best, lanes
// >= k hold 0).  Must be called by all 64 lanes of the wave (wave-uniform control flow).
__device__ __forceinline__ void wave_topk_push(uint64_t& top, uint64_t cand, int k, int lane) {
    const uint64_t thr = shfl_u64(top, k - 1);
    const bool c = cand > thr;
    if (__ballot(c) == 0ull) return;
    cand = c ? cand : 0ull;
    cand = wave_sort_desc(cand, lane);
    const uint64_t rev = shfl_u64(cand, 63 - lane);
    top = top > rev ? top : rev;
    top = wave_merge_desc(top, lane);
    if (lane >= k) top = 0ull;
}

}  // namespace lgx
