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
#include <cstdlib>

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

// LDS bytes of the per-wave lists: keys [32][kstride] u64 + meta [32][2] i32 (16-B aligned rows,
// plus one spare row so the vectorised rescan of the last user stays inside the allocation)
__host__ __device__ constexpr int kstride(int k) { return (k + 1) & ~1; }
constexpr int kListSpare = 8;  // the 8-key rescan of user 31 may read past its row
__host__ __device__ constexpr size_t list_bytes_per_wave(int k) {
    return ((size_t)kUsersPerWave * kstride(k) + kListSpare) * 8 + kUsersPerWave * 8;
}

// Running top-k of the 32 users of one wave (lanes col and col+32 share user col).  User col's
// list is an UNSORTED array of k packed keys in LDS (wave_topk.h key order) plus {len, argmin};
// the lane mirrors the worst kept entry (tau, tau_i) in registers for the per-score filter.  An
// accepted candidate overwrites the worst entry and the new worst is found by one scan of k
// independent LDS reads -- no dependent shift chain.  Lists are sorted only when merged.
template <int KMAX>
struct WaveTopK {
    uint64_t* keys;  // this lane's user: [k]
    int32_t* meta;   // this lane's user: {len, argmin}
    int k, col, h;
    int64_t b;       // query index of this lane's user
    bool user_ok;
    float tau;
    int32_t tau_i;
    bool full;
    float mn, mx;
    // 256-bit Bloom filter of the user's masked items (2 hashes), as 8 scalars so that the
    // word select stays in registers
    uint32_t bl0, bl1, bl2, bl3, bl4, bl5, bl6, bl7;

    __device__ __forceinline__ static uint32_t bloom_h1(int32_t x) { return ((uint32_t)x * 0x9E3779B1u) >> 24; }
    __device__ __forceinline__ static uint32_t bloom_h2(int32_t x) { return ((uint32_t)x * 0x85EBCA77u) >> 24; }
    __device__ __forceinline__ bool bloom_test(uint32_t hv) const {
        // AND with per-word masks: no select over loaded members (which the compiler would turn
        // into a load through a selected pointer and force the state into scratch)
        const uint32_t q = hv >> 5, m = 1u << (hv & 31);
        const uint32_t hit = (bl0 & (q == 0 ? m : 0u)) | (bl1 & (q == 1 ? m : 0u)) |
                             (bl2 & (q == 2 ? m : 0u)) | (bl3 & (q == 3 ? m : 0u)) |
                             (bl4 & (q == 4 ? m : 0u)) | (bl5 & (q == 5 ? m : 0u)) |
                             (bl6 & (q == 6 ? m : 0u)) | (bl7 & (q == 7 ? m : 0u));
        return hit != 0u;
    }
    __device__ __forceinline__ void bloom_set(uint32_t hv) {
        const uint32_t q = hv >> 5, m = 1u << (hv & 31);
        bl0 |= q == 0 ? m : 0u; bl1 |= q == 1 ? m : 0u; bl2 |= q == 2 ? m : 0u; bl3 |= q == 3 ? m : 0u;
        bl4 |= q == 4 ? m : 0u; bl5 |= q == 5 ? m : 0u; bl6 |= q == 6 ? m : 0u; bl7 |= q == 7 ? m : 0u;
    }
    // exact test only when the filter cannot rule the item out
    __device__ __forceinline__ bool masked(const ScoreArgs& a, int32_t it) const {
        if (!a.mask_indptr) return false;
        if (!bloom_test(bloom_h1(it)) || !bloom_test(bloom_h2(it))) return false;
        return is_masked(a, b, it);
    }
    __device__ __forceinline__ void build_bloom(const ScoreArgs& a) {
        bl0 = bl1 = bl2 = bl3 = bl4 = bl5 = bl6 = bl7 = 0u;
        if (!a.mask_indptr || !user_ok) return;
        const int64_t m0 = a.mask_indptr[b], m1 = a.mask_indptr[b + 1];
        for (int64_t j = m0; j < m1; ++j) {
            const int32_t x = a.mask_indices[j];
            bloom_set(bloom_h1(x));
            bloom_set(bloom_h2(x));
        }
    }

    __device__ __forceinline__ void init(uint64_t* keys_w, int32_t* meta_w, int k_, int lane, int64_t b_, bool ok) {
        k = k_;
        col = lane & 31;
        h = lane >> 5;
        b = b_;
        user_ok = ok;
        keys = keys_w + col * kstride(k);
        meta = meta_w + col * 2;
        if (h == 0) {
            meta[0] = 0;
            meta[1] = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        tau = ok ? -INFINITY : INFINITY;  // padding users never produce candidates
        tau_i = 0x7fffffff;
        full = false;
        mn = INFINITY;
        mx = -INFINITY;
    }

    // new worst entry: 8 keys (four 16-byte reads issued together) per LDS round trip
    __device__ __forceinline__ void rescan() {
        uint64_t m = ~0ull;
        int mp = 0;
        for (int j0 = 0; j0 < k; j0 += 8) {
            uint64_t v[8];
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(keys + j0 + j);
                v[j] = p.x;
                v[j + 1] = p.y;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t x = (j0 + j < k) ? v[j] : ~0ull;
                if (x < m) {
                    m = x;
                    mp = j0 + j;
                }
            }
        }
        meta[1] = mp;
    }

    // consume one 32-item accumulator tile whose item rows start at i0 (items >= i_end ignored).
    // Fast path: ONE compare per score against tau (-inf until the list is full, +inf for padding
    // users), OR-ed into a wave-wide flag; only a tile with a survivor re-tests exactly (bounds,
    // index tie-break) and inserts.  FULL: the whole 32-item tile is inside [i0, i_end).
    template <bool MINMAX, bool FULL, bool FASTONLY = false>
    __device__ __forceinline__ void tile(const ScoreArgs& a, const f32x16& acc, int64_t i0, int64_t i_end) {
        bool any = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float s = acc[r];
            const bool in = FULL || (i0 + tile_row(r, h)) < i_end;
            if (MINMAX && in && user_ok) {
                mn = fminf(mn, s);
                mx = fmaxf(mx, s);
            }
            any |= in && s >= tau;
        }
        if (FASTONLY) {  // development ablation: filter only
            mn = fminf(mn, __ballot(any) ? 1.0f : 0.0f);
            return;
        }
        if (__ballot(any) == 0ull) return;  // wave-uniform fast path
        uint32_t cmask = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int32_t it = (int32_t)(i0 + tile_row(r, h));
            if (user_ok && it < i_end && (!full || better(acc[r], it, tau, tau_i))) cmask |= 1u << r;
        }
        // the two lane halves hold different items of the same 32 users -> serialise them
        for (int ph = 0; ph < 2; ++ph) {
            if (__ballot(ph == h && cmask != 0) == 0ull) continue;
            if (ph == h && cmask) {
                int len = meta[0];
                uint32_t todo = cmask;
                while (todo) {  // one copy of the insertion code, one iteration per survivor
                    const int r = __builtin_ctz(todo);
                    todo &= todo - 1;
                    float sc = acc[0];
#pragma unroll
                    for (int q = 1; q < 16; ++q) sc = (r == q) ? acc[q] : sc;
                    const int32_t it = (int32_t)(i0 + tile_row(r, h));
                    const uint64_t key = make_key(sc, it);
                    if (len == k) {
                        const int mp = meta[1];
                        if (key <= keys[mp] || masked(a, it)) continue;
                        keys[mp] = key;
                        rescan();
                    } else {
                        if (masked(a, it)) continue;
                        keys[len++] = key;
                        if (len == k) rescan();
                    }
                }
                meta[0] = len;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        full = meta[0] == k;
        if (full && user_ok) {
            const uint64_t m = keys[meta[1]];
            tau = key_score(m);
            tau_i = key_index(m);
        }
    }

    __device__ __forceinline__ void flush(const ScoreArgs& a, int split, int lane) {
        if (user_ok && h == 0) {
            const int len = meta[0];
            float* ps = a.part_score + ((size_t)b * a.n_splits + split) * k;
            int32_t* pi = a.part_idx + ((size_t)b * a.n_splits + split) * k;
            for (int j = 0; j < k; ++j) {
                ps[j] = j < len ? key_score(keys[j]) : -INFINITY;
                pi[j] = j < len ? key_index(keys[j]) : -1;
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
};


template <int DT, int KCH, bool MINMAX>
__global__ __launch_bounds__(256) void score_topk_kernel(ScoreArgs a) {
    typedef Frag<DT> F;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int k = a.k;
    uint64_t* lk = reinterpret_cast<uint64_t*>(smem + (size_t)wave * list_bytes_per_wave(k));
    int32_t* lm = reinterpret_cast<int32_t*>(lk + (size_t)kUsersPerWave * kstride(k) + kListSpare);

    const int64_t b = (int64_t)blockIdx.x * kUsersPerBlock + wave * kUsersPerWave + col;  // this lane's user
    const bool user_ok = b < a.B;
    const int64_t qrow = user_ok ? (a.user_rows ? a.user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(a.Q, qrow, a.d, c, h, user_ok);
    WaveTopK<64> st;
    st.init(lk, lm, k, lane, b, user_ok);
    st.build_bloom(a);

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
        if (i0 + 32 <= i_end) st.template tile<MINMAX, true>(a, acc, i0, i_end);
        else st.template tile<MINMAX, false>(a, acc, i0, i_end);
    }
    st.flush(a, split, lane);
}

// ---------------------------------------------------------------------------- bf16 LDS kernel
// 512 threads = 8 waves x 32 users; the workgroup streams 64-item tiles of its catalog split
// through a double-buffered LDS ring filled by LDS-DMA (global_load_lds_dwordx4), so every item
// byte crosses L2 -> CU once per workgroup and feeds 8 waves.  Rows are stored with their 16-B
// chunks XOR-swizzled by (item & 15) so the fragment reads (32 items, same chunk) are
// conflict-free ds_read_b128s; the swizzle is applied to the DMA SOURCE address because the LDS
// destination of an LDS-DMA is lane-linear.  Splits are assigned so that the workgroups one XCD
// runs concurrently (blockIdx = xcd mod 8) sweep the same catalog slice and share its L2.
constexpr int kLdsWaves = 8;
constexpr int kLdsUsers = kLdsWaves * kUsersPerWave;  // 256 users per workgroup
constexpr int kTileItems = 64;

template <int KSTEPS>
struct LdsGeom {
    static constexpr int RB = KSTEPS * 32;              // bytes per bf16 item row (d = 16*KSTEPS)
    static constexpr int CPR = RB / 16;                 // 16-B chunks per row
    static constexpr int TILE = kTileItems * RB;        // bytes per tile
    static constexpr int PIECES = TILE / 1024;          // 1-KiB LDS-DMA wave instructions per tile
    static constexpr int PPW = (PIECES + kLdsWaves - 1) / kLdsWaves;
    static constexpr int SWZ = (CPR < 16 ? CPR : 16) - 1;
};

template <int KSTEPS, bool MINMAX, int ABLATE = 0>
__global__ __launch_bounds__(512) void score_topk_bf16_lds(ScoreArgs a, int xcd_affine, int64_t n_utiles) {
    typedef LdsGeom<KSTEPS> G;
    typedef Frag<LGX_DTYPE_BF16> F;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* tiles = smem;  // [2][TILE]
    const int k = a.k;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    uint64_t* lk = reinterpret_cast<uint64_t*>(smem + 2 * G::TILE + (size_t)wave * list_bytes_per_wave(k));
    int32_t* lm = reinterpret_cast<int32_t*>(lk + (size_t)kUsersPerWave * kstride(k) + kListSpare);

    // workgroup -> (catalog split, user tile)
    const int64_t bid = blockIdx.x;
    int split;
    int64_t utile;
    if (xcd_affine) {
        const int64_t per = a.n_splits / 8;
        const int64_t r = bid / 8;
        split = (int)(bid % 8 + 8 * (r % per));
        utile = r / per;
    } else {
        split = (int)(bid % a.n_splits);
        utile = bid / a.n_splits;
    }
    if (utile >= n_utiles) return;

    const int64_t b = utile * kLdsUsers + wave * kUsersPerWave + col;
    const bool user_ok = b < a.B;
    const int64_t qrow = user_ok ? (a.user_rows ? a.user_rows[b] : b) : 0;
    typename F::chunk uf[KSTEPS];
#pragma unroll
    for (int c = 0; c < KSTEPS; ++c) uf[c] = F::load(a.Q, qrow, a.d, c, h, user_ok);
    WaveTopK<32> st;
    st.init(lk, lm, k, lane, b, user_ok);
    st.build_bloom(a);

    const int64_t i_begin = (int64_t)split * a.split_items;
    const int64_t i_end = min(a.n_items, i_begin + a.split_items);
    const int64_t ntiles = i_end > i_begin ? (i_end - i_begin + kTileItems - 1) / kTileItems : 0;
    // single split: every workgroup sweeps the whole catalog, starting at a rotation shared by the
    // workgroups of its XCD (blockIdx mod 8) so that co-resident workgroups read the same tiles
    const int64_t rot = a.n_splits == 1 ? (bid % 8) * (ntiles / 8) : 0;
    const unsigned char* items = static_cast<const unsigned char*>(a.items);

    auto stage = [&](int buf, int64_t t0) {
#pragma unroll
        for (int p = 0; p < G::PPW; ++p) {
            const int piece = wave * G::PPW + p;
            if (piece < G::PIECES) {
                const int q = piece * 64 + lane;  // 16-B LDS slot written by this lane
                const int item = q / G::CPR, pch = q % G::CPR;
                const int src = pch ^ (item & G::SWZ);
                const int64_t gi = min(t0 + item, i_end - 1);  // tail rows: any valid row, masked later
                const unsigned char* gp = items + gi * G::RB + src * 16;
                __builtin_amdgcn_global_load_lds(
                    gp, (__attribute__((address_space(3))) void*)(tiles + buf * G::TILE + piece * 1024), 16, 0, 0);
            }
        }
    };

    auto tile_start = [&](int64_t t) {
        int64_t u = t + rot;
        if (u >= ntiles) u -= ntiles;
        return i_begin + u * kTileItems;
    };
    if (ntiles > 0) stage(0, tile_start(0));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int64_t t = 0; t < ntiles; ++t) {
        const int buf = (int)(t & 1);
        const int64_t t0 = tile_start(t);
        if (t + 1 < ntiles) stage(buf ^ 1, tile_start(t + 1));
        const unsigned char* T = tiles + buf * G::TILE;
        f32x16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc0[r] = 0.0f;
            acc1[r] = 0.0f;
        }
        const int it0 = col, it1 = 32 + col;
#pragma unroll
        for (int c = 0; c < KSTEPS; ++c) {
            const int pch = 2 * c + h;
            const uint4 a0 = *reinterpret_cast<const uint4*>(T + it0 * G::RB + ((pch ^ (it0 & G::SWZ)) * 16));
            const uint4 a1 = *reinterpret_cast<const uint4*>(T + it1 * G::RB + ((pch ^ (it1 & G::SWZ)) * 16));
            acc0 = F::mma(a0, uf[c], acc0);
            acc1 = F::mma(a1, uf[c], acc1);
        }
        if (ABLATE == 1) {  // development: MFMA + LDS pipeline only (keeps the accumulators live)
            float z = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) z += acc0[r] + acc1[r];
            st.mx = fmaxf(st.mx, z);
        } else if (ABLATE == 3) {  // development: filter fast path only
            st.template tile<MINMAX, true, true>(a, acc0, t0, i_end);
            st.template tile<MINMAX, true, true>(a, acc1, t0 + 32, i_end);
        } else {
            if (t0 + kTileItems <= i_end) {
                st.template tile<MINMAX, true>(a, acc0, t0, i_end);
                st.template tile<MINMAX, true>(a, acc1, t0 + 32, i_end);
            } else {
                st.template tile<MINMAX, false>(a, acc0, t0, i_end);
                st.template tile<MINMAX, false>(a, acc1, t0 + 32, i_end);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    st.flush(a, split, lane);
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

// ---------------------------------------------------------------------------- bf16 LDS ring kernel
// Same data path as score_topk_bf16_lds but without a workgroup barrier per tile: the 8 waves
// run decoupled over a ring of kRingSlots 32-item slots, so a wave that takes the top-k slow path
// delays only itself (the ring absorbs up to kRingSlots-1 tiles of drift).
// Every refill is split into 8 shares (wave w moves pieces [w*PPW, (w+1)*PPW) by LDS-DMA).  Two
// monotonic LDS counters per slot carry the protocol:
//   done[s]   += 1 when a wave has finished reading the slot's current tile;
//   filled[s] += 1 when a wave's share of the slot's next tile has landed (published after that
//               wave's s_waitcnt vmcnt(0), lazily at its next service point).
// Tile t lives in slot t % R during occupancy j = t / R: it is readable once filled >= 8(j+1), and
// a wave may issue its share of tile t once done >= 8 j (everybody finished tile t - R).  Each wave
// services its obligations (publish landed shares, issue allowed ones) at every tile boundary and
// inside every wait, so the wave waiting on the oldest tile always makes progress (no deadlock).
// All spins are bounded (timeout -> error word, sweep abandoned: wrong results, never a hang).
constexpr int kRingSlots = 6;  // even: a pair of tiles never wraps inside one slot
constexpr int kRingItems = 32;
constexpr uint32_t kSpinLimit = 1u << 22;

template <int KSTEPS>
struct RingGeom {
    static constexpr int RB = KSTEPS * 32;
    static constexpr int CPR = RB / 16;
    static constexpr int SLOT = kRingItems * RB;  // bytes per slot (16 KiB at d = 256)
    static constexpr int PIECES = SLOT / 1024;    // 1-KiB LDS-DMA instructions per slot
    static constexpr int PPW = (PIECES + kLdsWaves - 1) / kLdsWaves;
    static constexpr int SWZ = (CPR < 16 ? CPR : 16) - 1;
};

// issue the LDS-DMA pieces [p0, p1) of the tile starting at item t0 into one ring slot
template <typename G>
__device__ __forceinline__ void ring_stage(unsigned char* slot, const unsigned char* items, int64_t t0, int64_t i_end,
                                           int p0, int p1, int lane) {
#pragma unroll 1  // keep the per-piece address math inside the loop (no hoisted live ranges)
    for (int piece = p0; piece < p1; ++piece) {
        const int q = piece * 64 + lane;
        const int item = q / G::CPR, pch = q % G::CPR;
        const int src = pch ^ (item & G::SWZ);
        int64_t gi = t0 + item;
        if (gi > i_end - 1) gi = i_end - 1;  // tail rows: any valid row, masked later
        const unsigned char* gp = items + gi * G::RB + src * 16;
        __builtin_amdgcn_global_load_lds(gp, (__attribute__((address_space(3))) void*)(slot + piece * 1024), 16, 0, 0);
    }
}

template <int KSTEPS, bool MINMAX, int ABLATE = 0>
__global__ __launch_bounds__(512) void score_topk_bf16_ring(ScoreArgs a, int xcd_affine, int64_t n_utiles,
                                                            int* err) {
    typedef RingGeom<KSTEPS> G;
    typedef Frag<LGX_DTYPE_BF16> F;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* ring = smem;  // [kRingSlots][SLOT]
    int* filled = reinterpret_cast<int*>(smem + kRingSlots * G::SLOT);
    int* done = filled + kRingSlots;
    unsigned char* lists = smem + kRingSlots * G::SLOT + 2 * kRingSlots * sizeof(int) + 16;
    const int k = a.k;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    uint64_t* lk = reinterpret_cast<uint64_t*>(lists + (size_t)wave * list_bytes_per_wave(k));
    int32_t* lm = reinterpret_cast<int32_t*>(lk + (size_t)kUsersPerWave * kstride(k) + kListSpare);

    const int64_t bid = blockIdx.x;
    int split;
    int64_t utile;
    if (xcd_affine) {
        const int64_t per = a.n_splits / 8;
        const int64_t r = bid / 8;
        split = (int)(bid % 8 + 8 * (r % per));
        utile = r / per;
    } else {
        split = (int)(bid % a.n_splits);
        utile = bid / a.n_splits;
    }
    if (utile >= n_utiles) return;

    const int64_t b = utile * kLdsUsers + wave * kUsersPerWave + col;
    const bool user_ok = b < a.B;
    const int64_t qrow = user_ok ? (a.user_rows ? a.user_rows[b] : b) : 0;
    typename F::chunk uf[KSTEPS];
#pragma unroll
    for (int c = 0; c < KSTEPS; ++c) uf[c] = F::load(a.Q, qrow, a.d, c, h, user_ok);
    WaveTopK<32> st;
    st.init(lk, lm, k, lane, b, user_ok);
    st.build_bloom(a);

    const int64_t i_begin = (int64_t)split * a.split_items;
    const int64_t i_end = min(a.n_items, i_begin + a.split_items);
    const int64_t ntiles = i_end > i_begin ? (i_end - i_begin + kRingItems - 1) / kRingItems : 0;
    // single split: every workgroup sweeps the whole catalog, starting at a rotation shared by the
    // workgroups of its XCD (blockIdx mod 8) so that co-resident workgroups read the same tiles
    const int64_t rot = a.n_splits == 1 ? (bid % 8) * (ntiles / 8) : 0;
    const unsigned char* items = static_cast<const unsigned char*>(a.items);
    auto tile_start = [&](int64_t t) {
        int64_t u = t + rot;
        if (u >= ntiles) u -= ntiles;
        return i_begin + u * kRingItems;
    };
    const int p0 = wave * G::PPW;
    const int p1 = (p0 + G::PPW < G::PIECES) ? p0 + G::PPW : (int)G::PIECES;

    // prologue: every wave loads its share of the first kRingSlots tiles
    const int64_t pro = ntiles < kRingSlots ? ntiles : kRingSlots;
    for (int64_t t = 0; t < pro; ++t)
        if (p0 < p1) ring_stage<G>(ring + (int)t * G::SLOT, items, tile_start(t), i_end, p0, p1, lane);
    if (threadIdx.x < kRingSlots) {
        filled[threadIdx.x] = threadIdx.x < pro ? kLdsWaves : 0;
        done[threadIdx.x] = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    int64_t next_share = pro;  // next tile this wave owes a share to
    int64_t pend_lo = pro, pend_hi = pro;  // issued in an EARLIER service call, not yet published
    // One service call: (1) issue up to two newly allowed shares, (2) retire the shares issued by
    // the previous call with a COUNTED wait that leaves the new ones in flight, (3) publish them.
    // A share's DMA therefore gets one whole iteration to land before anyone waits on it.
    auto service = [&]() {
        int n_new = 0;
        const int64_t new_lo = next_share;
        while (n_new < 2 && next_share < ntiles) {
            const int s = (int)(next_share % kRingSlots);
            const int need = kLdsWaves * (int)(next_share / kRingSlots);
            if (__hip_atomic_load(&done[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) break;
            if (p0 < p1) ring_stage<G>(ring + s * G::SLOT, items, tile_start(next_share), i_end, p0, p1, lane);
            ++next_share;
            ++n_new;
        }
        if (pend_lo < pend_hi) {
            const int inflight = (p1 > p0 ? p1 - p0 : 0) * n_new;  // DMA instructions just issued
            if (inflight == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if (inflight == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            else if (inflight == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else if (inflight == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            if (lane == 0)
                for (int64_t q = pend_lo; q < pend_hi; ++q)
                    __hip_atomic_fetch_add(&filled[q % kRingSlots], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        pend_lo = new_lo;
        pend_hi = next_share;
    };

    bool ok = true;
    // tiles are consumed in pairs (two independent MFMA chains, one wait / release / epilogue
    // branch per 64 items); an odd tail tile is paired with itself and masked out
    auto wait_tile = [&](int64_t t) {
        const int s = (int)(t % kRingSlots);
        const int need = kLdsWaves * (int)(t / kRingSlots + 1);
        uint32_t spins = 0;
        while (__hip_atomic_load(&filled[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need) {
            if (++spins > kSpinLimit) return false;
            service();
            __builtin_amdgcn_s_sleep(1);
        }
        return true;
    };
    for (int64_t t = 0; t < ntiles && ok; t += 2) {
        const bool two = t + 1 < ntiles;
        if (ABLATE != 2) {  // ABLATE == 2 (development): resident slots only, no refills / waits
            service();
            ok = wait_tile(t) && (!two || wait_tile(t + 1));
            if (!ok) break;
        }
        const int s0 = (int)(t % kRingSlots), s1 = (int)((two ? t + 1 : t) % kRingSlots);
        const unsigned char* T0 = ring + s0 * G::SLOT + col * G::RB;
        const unsigned char* T1 = ring + s1 * G::SLOT + col * G::RB;
        f32x16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc0[r] = 0.0f;
            acc1[r] = 0.0f;
        }
        // 2-deep fragment window per chain
        uint4 fa0[2], fa1[2];
#pragma unroll
        for (int c = 0; c < 2 && c < KSTEPS; ++c) {
            const int off = ((2 * c + h) ^ (col & G::SWZ)) * 16;
            fa0[c] = *reinterpret_cast<const uint4*>(T0 + off);
            fa1[c] = *reinterpret_cast<const uint4*>(T1 + off);
        }
#pragma unroll
        for (int c = 0; c < KSTEPS; ++c) {
            const uint4 c0 = fa0[c & 1], c1 = fa1[c & 1];
            if (c + 2 < KSTEPS) {
                const int off = ((2 * (c + 2) + h) ^ (col & G::SWZ)) * 16;
                fa0[c & 1] = *reinterpret_cast<const uint4*>(T0 + off);
                fa1[c & 1] = *reinterpret_cast<const uint4*>(T1 + off);
            }
            acc0 = F::mma(c0, uf[c], acc0);
            acc1 = F::mma(c1, uf[c], acc1);
            __builtin_amdgcn_sched_barrier(0);
        }
        // every fragment read of the pair has returned (the MFMAs consumed them): release
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0 && ABLATE != 2) {
            __hip_atomic_fetch_add(&done[s0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (two) __hip_atomic_fetch_add(&done[s1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const int64_t ta = tile_start(t);
        const int64_t tb = two ? tile_start(t + 1) : i_end;  // tb = i_end: tile fully masked
        if (ABLATE) {  // development: pipeline only
            float z = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) z += acc0[r] + acc1[r];
            st.mx = fmaxf(st.mx, z);
        } else {
            if (ta + kRingItems <= i_end) st.template tile<MINMAX, true>(a, acc0, ta, i_end);
            else st.template tile<MINMAX, false>(a, acc0, ta, i_end);
            if (tb + kRingItems <= i_end) st.template tile<MINMAX, true>(a, acc1, tb, i_end);
            else st.template tile<MINMAX, false>(a, acc1, tb, i_end);
        }
    }
    // remaining obligations: shares of tiles other waves still need
    uint32_t spins = 0;
    while (ABLATE != 2 && ok && (next_share < ntiles || pend_lo < pend_hi)) {
        service();
        if (next_share < ntiles) {
            if (++spins > kSpinLimit) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (!ok && lane == 0) atomicExch(err, 1);
    st.flush(a, split, lane);
}

struct SplitPlan {
    int n_splits;
    int64_t split_items;
    bool lds;        // bf16 LDS-DMA kernel
    bool xcd_affine;
    int64_t n_utiles;
};

// LDS kernel applies to bf16, d a multiple of 16 up to 256, k <= 32 (LDS budget)
bool lds_eligible(int dtype, int64_t d, int k) {
    return dtype == LGX_DTYPE_BF16 && d % 16 == 0 && d >= 32 && d <= 256 && k <= 32;
}

SplitPlan plan_splits(int64_t B, int64_t n_items, int dtype, int64_t d, int k) {
    const int64_t tiles32 = ceil_div(n_items, 32);
    if (lds_eligible(dtype, d, k)) {
        const int64_t ut = ceil_div(B, kLdsUsers);
        const int64_t tiles = ceil_div(n_items, kTileItems);
        if (ut >= 512)  // >= 2 rounds of one workgroup per CU: no catalog split, XCD-rotated sweeps
            return {1, tiles * kTileItems, true, false, ut};
        // >= 2 workgroups (512 threads) per CU, >= 4 tiles per split, a multiple of 8 when possible
        int64_t s = ceil_div(512, ut);
        s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / 4));
        s = std::max<int64_t>(1, std::min<int64_t>(s, 256));
        if (s >= 8) s = s / 8 * 8;
        const int64_t per = ceil_div(tiles, s) * kTileItems;
        const int n = (int)ceil_div(n_items, per);
        return {n, per, true, n % 8 == 0, ut};
    }
    const int64_t user_blocks = ceil_div(B, kUsersPerBlock);
    int64_t s = ceil_div(2048, user_blocks);                       // aim for >= ~8 workgroups per CU
    s = std::min<int64_t>(s, std::max<int64_t>(1, tiles32 / 8));  // >= 8 tiles per split
    s = std::max<int64_t>(1, std::min<int64_t>(s, 64));
    const int64_t per = ceil_div(tiles32, s) * 32;
    return {(int)ceil_div(n_items, per), per, false, false, user_blocks};
}

template <typename KernelT>
int set_lds_limit(KernelT kernel, size_t shmem) {
    if (shmem > 65536)
        LGX_HIP_CHECK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
    return LGX_OK;
}

template <int DT, bool MM>
int launch_v1(const ScoreArgs& a, int kch, hipStream_t stream) {
    const size_t shmem = (size_t)kWavesPerBlock * list_bytes_per_wave(a.k);
    dim3 grid((unsigned)ceil_div(a.B, kUsersPerBlock), (unsigned)a.n_splits);
#define LGX_SK(KC)                                                                     \
    do {                                                                               \
        int rc_ = set_lds_limit(score_topk_kernel<DT, KC, MM>, shmem);                \
        if (rc_) return rc_;                                                           \
        score_topk_kernel<DT, KC, MM><<<grid, 256, shmem, stream>>>(a);                \
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
    return LGX_OK;
}

template <bool MM, int ABL = 0>
int launch_lds(const ScoreArgs& a, const SplitPlan& p, hipStream_t stream) {
    const int ksteps = (int)(a.d / 16);
    const unsigned grid = (unsigned)(p.n_utiles * p.n_splits);
#define LGX_SL(KS)                                                                                          \
    do {                                                                                                    \
        const size_t shmem = 2 * (size_t)LdsGeom<KS>::TILE + (size_t)kLdsWaves * list_bytes_per_wave(a.k);     \
        int rc_ = set_lds_limit(score_topk_bf16_lds<KS, MM, ABL>, shmem);                                 \
        if (rc_) return rc_;                                                                                \
        score_topk_bf16_lds<KS, MM, ABL><<<grid, 512, shmem, stream>>>(a, p.xcd_affine ? 1 : 0, p.n_utiles); \
    } while (0)
    switch (ksteps) {
        case 2: LGX_SL(2); break;
        case 4: LGX_SL(4); break;
        case 6: LGX_SL(6); break;
        case 8: LGX_SL(8); break;
        case 10: LGX_SL(10); break;
        case 12: LGX_SL(12); break;
        case 14: LGX_SL(14); break;
        case 16: LGX_SL(16); break;
        default:
            set_error("lgx_score_topk: no LDS kernel for d=%lld", (long long)a.d);
            return LGX_ERR_UNSUPPORTED;
    }
#undef LGX_SL
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

template <bool MM, int ABL = 0>
int launch_ring(const ScoreArgs& a, const SplitPlan& p, int* err, hipStream_t stream) {
    const int ksteps = (int)(a.d / 16);
    const unsigned grid = (unsigned)(p.n_utiles * p.n_splits);
#define LGX_SR(KS)                                                                                           \
    do {                                                                                                     \
        const size_t shmem = (size_t)kRingSlots * RingGeom<KS>::SLOT + 2 * kRingSlots * sizeof(int) + 16 +  \
                             (size_t)kLdsWaves * list_bytes_per_wave(a.k);                                  \
        int rc_ = set_lds_limit(score_topk_bf16_ring<KS, MM, ABL>, shmem);                                 \
        if (rc_) return rc_;                                                                                 \
        score_topk_bf16_ring<KS, MM, ABL><<<grid, 512, shmem, stream>>>(a, p.xcd_affine ? 1 : 0, p.n_utiles, err); \
    } while (0)
    switch (ksteps) {
        case 2: LGX_SR(2); break;
        case 4: LGX_SR(4); break;
        case 6: LGX_SR(6); break;
        case 8: LGX_SR(8); break;
        case 10: LGX_SR(10); break;
        case 12: LGX_SR(12); break;
        case 14: LGX_SR(14); break;
        case 16: LGX_SR(16); break;
        default:
            set_error("lgx_score_topk: no ring kernel for d=%lld", (long long)a.d);
            return LGX_ERR_UNSUPPORTED;
    }
#undef LGX_SR
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

size_t topk_ws_bytes(int64_t B, int64_t n_items, int k, int dtype, int64_t d) {
    const SplitPlan p = plan_splits(B, n_items, dtype, d, k);
    return align_up((size_t)B * p.n_splits * k * 4) * 2 + 512;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_score_topk_workspace(int64_t B, int64_t n_items, int k, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && B >= 0 && n_items >= 0 && k >= 1, LGX_ERR_INVALID_ARG,
                "lgx_score_topk_workspace: bad arguments");
    // the split plan depends on dtype / d; report the maximum over every kernel variant
    size_t m = topk_ws_bytes(B, n_items, k, LGX_DTYPE_F32, 64);
    for (int64_t d = 32; d <= 256; d += 16) m = std::max(m, topk_ws_bytes(B, n_items, k, LGX_DTYPE_BF16, d));
    *ws_bytes = m;
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
    const size_t need = topk_ws_bytes(B, n_items, k, dtype, d);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_score_topk: workspace %zu < %zu", ws_bytes, need);
    const SplitPlan p = plan_splits(B, n_items, dtype, d, k);
    char* base = static_cast<char*>(ws);
    const size_t list_bytes = align_up((size_t)B * p.n_splits * k * 4);
    ScoreArgs a{Q, user_rows, items, B, n_items, d, mask_indptr, mask_indices, k, p.n_splits, p.split_items,
                reinterpret_cast<float*>(base), reinterpret_cast<int32_t*>(base + list_bytes),
                minmax_out ? reinterpret_cast<uint32_t*>(base + 2 * list_bytes) : nullptr};
    if (a.minmax) {
        minmax_init<<<1, 1, 0, stream>>>(a.minmax);
        LGX_LAUNCH_CHECK();
    }
    const bool mm = minmax_out != nullptr;
    int rc;
    // development switches (A/B and ablation only): LGX_SCORE_KERNEL=ring selects the decoupled
    // ring kernel; LGX_SCORE_ABLATE=1 drops the top-k work, =3 the mask path (timing studies)
    static const char* abl_env = getenv("LGX_SCORE_ABLATE");
    static const bool ablate = abl_env && abl_env[0] == '1';
    static const bool ablate2 = abl_env && abl_env[0] == '2';
    static const bool ablate3 = abl_env && abl_env[0] == '3';
    static const bool ring = getenv("LGX_SCORE_KERNEL") && getenv("LGX_SCORE_KERNEL")[0] == 'r';
    int* err = reinterpret_cast<int*>(base + 2 * list_bytes + 256);
    if (p.lds && ablate && ring) rc = launch_ring<false, 1>(a, p, err, stream);
    else if (p.lds && ablate2 && ring) rc = launch_ring<false, 2>(a, p, err, stream);
    else if (p.lds && ablate) rc = launch_lds<false, 1>(a, p, stream);
    else if (p.lds && ablate3) rc = launch_lds<false, 3>(a, p, stream);
    else if (p.lds && ring) rc = mm ? launch_ring<true>(a, p, err, stream) : launch_ring<false>(a, p, err, stream);
    else if (p.lds) rc = mm ? launch_lds<true>(a, p, stream) : launch_lds<false>(a, p, stream);
    else if (dtype == LGX_DTYPE_F32) rc = mm ? launch_v1<LGX_DTYPE_F32, true>(a, kch, stream)
                                             : launch_v1<LGX_DTYPE_F32, false>(a, kch, stream);
    else rc = mm ? launch_v1<LGX_DTYPE_BF16, true>(a, kch, stream) : launch_v1<LGX_DTYPE_BF16, false>(a, kch, stream);
    if (rc) return rc;
    score_topk_finalize<<<(unsigned)a.B, 64, 0, stream>>>(a, mask_value, apply_sigmoid, out_idx, out_val, minmax_out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
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
