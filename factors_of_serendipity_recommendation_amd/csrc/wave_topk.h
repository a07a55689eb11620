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

// The same running list for k up to 64 R: element e = 64 r + lane lives in register r of lane
// `lane`, sorted descending over e.  Exchanges at distances >= 64 stay inside a lane (register r
// with r ^ (j / 64)); shorter ones are the xor-shuffles of the R = 1 network.  The reference's
// top-k has no size limit (tools.h:13-33 partial_sort_copy, torch.topk); R = 4 covers k <= 256.
template <int R>
struct WaveList {
    uint64_t t[R];  // t[r] in lane l: element 64 r + l

    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int r = 0; r < R; ++r) t[r] = 0ull;
    }
    __device__ __forceinline__ uint64_t at(int e) const {  // wave-uniform e
        uint64_t v = t[0];
#pragma unroll
        for (int r = 1; r < R; ++r) v = (e >> 6) == r ? t[r] : v;
        return shfl_u64(v, e & 63);
    }
    // bitonic merge (descending) of a bitonic sequence of 64 R elements
    __device__ __forceinline__ void merge_desc(int lane) {
#pragma unroll
        for (int j = 32 * R; j >= 64; j >>= 1) {
            const int jr = j >> 6;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r & jr) continue;
                const uint64_t a = t[r], b = t[r | jr];
                t[r] = a > b ? a : b;
                t[r | jr] = a > b ? b : a;
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) t[r] = wave_merge_desc(t[r], lane);
    }
    // merge one batch of 64 candidates (one per lane); all 64 lanes, wave-uniform control flow
    __device__ __forceinline__ void push(uint64_t cand, int k, int lane) {
        if (R == 1) {
            wave_topk_push(t[0], cand, k, lane);
            return;
        }
        const uint64_t thr = at(k - 1);
        const bool c = cand > thr;
        if (__ballot(c) == 0ull) return;
        cand = wave_sort_desc(c ? cand : 0ull, lane);
        // half-cleaner of [list (desc) | candidates reversed and zero-padded (asc)]: only the last
        // register block meets a non-zero partner; the result is bitonic over the 64 R elements
        const uint64_t rev = shfl_u64(cand, 63 - lane);
        t[R - 1] = t[R - 1] > rev ? t[R - 1] : rev;
        merge_desc(lane);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (64 * r + lane >= k) t[r] = 0ull;
    }
};

}  // namespace lgx
