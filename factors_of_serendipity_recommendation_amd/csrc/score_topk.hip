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
// MI355X design (one file, three kernel families):
//   * score_topk_bf16_lds / score_topk_f32_lds -- the LDS-ring walk: a workgroup keeps its users'
//     rows in VGPRs (the MFMA B operand) and streams 64-item tiles of the catalog (the A operand)
//     through an LDS ring filled by LDS-DMA; v_mfma_f32_16x16x32_bf16 / 16x16x4_f32.  Its modes:
//     the running top-k with the mask (kTopK), the global min / max (kMinMaxOnly) and the per-user
//     score floors (kFloorOnly) that start an unseeded sweep's lists;
//   * score_topk_kernel -- a register-fragment walk (v_mfma_f32_32x32x16_bf16 / 32x32x2_f32) for
//     the shapes the LDS walk does not cover; score_dense_lds / score_dense_kernel (getUsersRating's
//     dense scores) and strat_label_lds (recommend.py's stratification labels) on the same
//     register-staged 32x32 walk, so fused labels are the labels of the dense scores bit for bit
//     (the 16x16x4 LDS ring measured slower for these write-heavy modes at every d:
//     profiles/r04_walk_lab.txt);
//   * score_topk_finalize -- one wave per user merges split lists (register bitonic network), adds
//     the masked tail when fewer than k unmasked items exist and applies the optional sigmoid.
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cfloat>
#include <cstdlib>
#include <cstring>

#include "wave_topk.h"

namespace lgx {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kUsersPerWave = 32;
// waves per workgroup of the register-fragment kernel: its per-user lists live in LDS (k keys per
// user), so the largest k run one wave per workgroup
__host__ __device__ constexpr int v1_waves(int k) { return k <= 128 ? 4 : 1; }

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
    uint64_t* susp;       // [B, n_splits, 2, kSuspSlots] parked keys (LDS kernel), or nullptr
    // seeded sweep (LDS kernel, full sweep): each user's exact top-k over items [0, seed_items),
    // [B, k] (index -1 = empty); the sweep then covers [seed_items, n_items) only
    const float* seed_score;
    const int32_t* seed_idx;
    int64_t seed_items;
    // score floor [B, n_splits] (LDS kernel): written by the kFloorOnly walk over the first
    // floor_items items of each split, read by an unseeded sweep as every list's starting threshold
    float* floor;
    int64_t floor_items;
};

// Candidates whose mask test the Bloom filter cannot settle ("suspects", ~10 % of the survivors) are
// parked in the workspace and settled by exact searches once, at the flush: an exact search in the
// sweep is a chain of dependent global loads that also waits for the in-flight tile DMA (vmcnt
// completes in order), and the per-tile barrier makes every wave of the workgroup wait for it.  A
// lane with all its slots taken searches at once, as before.
constexpr int kSuspSlots = 32;  // per (user, split, lane half); resolve_suspects' keep mask is 32 bits
constexpr int kBloomWords = 8;  // 256-bit filter: 8 VGPRs
constexpr int kBloomShift = 32 - 5 - 3;

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

// LDS bytes of the per-wave lists: keys [32][kstride] u64 (16-B aligned rows, plus spare keys so
// that the vectorised rescan of user 31 stays inside the allocation), then the deferred-candidate
// slots [64 lanes][kPendSlots + 1] u64 (the last slot of a lane takes the branch-free event path's
// writes once its real slots are full)
__host__ __device__ constexpr int kstride(int k) { return (k + 1) & ~1; }
constexpr int kListSpare = 8;  // the 8-key rescan of user 31 may read past its row
// deferred slots per lane: 4 in the register-fragment and fp32 LDS kernels; 12 in the bf16 LDS kernel,
// whose events are 16x more frequent per MFMA cycle: a lane overflows its slots (and sends the
// wave down the exact path) 3x less often.  tools/score_lab (131072 users x 1M items, d=256,
// profiles/r03_score_lab_pend.txt): 4 slots + 3 ring buffers 59.50 ms over the 7 seeded stages,
// 1073 TF/s masked one-sweep; 4 slots + 2 buffers 60.18 ms; 8 slots 58.29 ms, 1103; 12 slots
// 57.75 ms, 1103 (1168 unmasked, +4 %).  12 slots take the LDS of the third ring buffer (the
// ring's depth measured neutral) and fit d = 256 up to k = 20.
constexpr int kPendSlots = 4;
constexpr int kPendBf16Lds = 12;
// deferred slots of the LDS walk: 12 for bf16, and for fp32 up to d = 128, whose tiles leave the LDS
// for them; fp32 at d = 256 keeps 4 (two 64 KB tiles and four waves' lists fill the 160 KB).  fp32
// with 12 (profiles/r04_eval_probe_ab.txt, masked top-20): Gowalla shape 3.67 -> 3.30 ms, Amazon-book
// shape 17.6 -> 16.6 ms
// ... and 16 in the 4-wave fp32 walk up to d = 128 (one wave per SIMD, LDS to spare: 4 x 14 KB of
// lists beside a 4-tile ring at d = 64), where an exact path is the wave's own time and fewer of
// them pay (Gowalla shape, profiles/r05_pend16_ab.txt: route 3.12 -> 3.05 ms)
__host__ __device__ constexpr int lds_pend(bool f32, int ksteps, int waves = 8) {
    return f32 && ksteps > 8 ? kPendSlots : f32 && waves == 4 ? 16 : kPendBf16Lds;
}
__host__ __device__ constexpr size_t list_keys_per_wave(int k) { return (size_t)kUsersPerWave * kstride(k) + kListSpare; }
// ... then one int per lane: the count of its parked keys (kSuspSlots)
__host__ __device__ constexpr size_t list_bytes_per_wave(int k, int pend = kPendSlots) {
    return (list_keys_per_wave(k) + 64 * (pend + 1)) * 8 + 64 * 4;
}

// value held by lane (lane ^ 32): one v_permlane32_swap, no LDS traffic
__device__ __forceinline__ uint32_t other_half(uint32_t x) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (threadIdx.x & 32) ? r[0] : r[1];
}

// Running top-k of the 32 users of one wave (lanes col and col+32 share user col).  User col's
// list is an UNSORTED array of k packed keys in LDS (wave_topk.h key order); its length, the slot
// of its worst entry and that entry's key live in registers, identical in both lanes of the user.
// The lane mirrors the worst kept entry (tau, tau_i) for the per-score filter.  An accepted
// candidate overwrites the worst entry and the new worst is found by one scan of k independent
// LDS reads -- no dependent shift chain.  Lists are sorted only when merged.
// REDEFER: after a drain, the block that overran a lane's slots is deferred again against the drained
// lists before any direct insert (the fp32 walks with 12-16 slots per lane: Amazon-book shape 14.13 ->
// 13.78 ms; with 4 slots, fp32 at d = 256, it costs 4.5 %, and bf16 C5 0.6 %: profiles/r06_pc_variants_ab.txt)
template <int PEND, bool REDEFER = false>
struct WaveTopKT {
    uint64_t* keys;  // this lane's user: [k]
    int k, h;
    int64_t b;       // query index of this lane's user
    bool user_ok;
    int len, mp;     // list length, slot of the worst entry (valid when len == k)
    uint64_t kmin;   // worst kept key (valid when len == k)
    // deferred candidates of THIS lane (its half's items), inserted into the list in batches so
    // that a late-sweep survivor costs a few register moves instead of LDS round trips
    static constexpr int kPend = PEND;
    static_assert(kPend >= 1 && kPend <= 16, "deferred slots: 1..16 per lane");
    // this lane's kPend (+1 scratch) slots in LDS; a slot holds the raw pair (score bits, item << 32)
    uint64_t* pend;
    int pcnt;
    float tau;       // filter threshold: -inf until the list is full, +inf for padding users
    int32_t tau_i;
    float mn, mx;
    bool park;       // parked keys enabled (LDS kernel with a mask); count in LDS (scnt())
    int sp;          // catalog split of this workgroup (its parked keys' region)
    // 256-bit Bloom filter of the user's masked items (2 hashes; false-positive rate ~10% at 50
    // masked items), as 16 scalars so that the word select stays in registers
    uint32_t bl[kBloomWords];

    __device__ __forceinline__ static uint32_t bloom_h1(int32_t x) { return ((uint32_t)x * 0x9E3779B1u) >> kBloomShift; }
    __device__ __forceinline__ static uint32_t bloom_h2(int32_t x) { return ((uint32_t)x * 0x85EBCA77u) >> kBloomShift; }
    __device__ __forceinline__ bool bloom_test(uint32_t hv) const {
        // AND with per-word masks: no select over loaded members (which the compiler would turn
        // into a load through a selected pointer and force the state into scratch)
        const uint32_t q = hv >> 5, m = 1u << (hv & 31);
        uint32_t hit = 0;
#pragma unroll
        for (int w = 0; w < kBloomWords; ++w) hit |= bl[w] & (q == (uint32_t)w ? m : 0u);
        return hit != 0u;
    }
    __device__ __forceinline__ void bloom_set(uint32_t hv) {
        const uint32_t q = hv >> 5, m = 1u << (hv & 31);
#pragma unroll
        for (int w = 0; w < kBloomWords; ++w) bl[w] |= q == (uint32_t)w ? m : 0u;
    }
    // true when the key must not enter the list now: masked, or parked for the flush's exact test
    // (the exact test runs at once only when the filter cannot rule the item out and no slot is free)
    __device__ __forceinline__ bool masked(const ScoreArgs& a, uint64_t key) {
        const int32_t it = key_index(key);
        if (!a.mask_indptr) return false;
        if (!bloom_test(bloom_h1(it)) || !bloom_test(bloom_h2(it))) return false;
        if (park) {
            const int c = *scnt();
            if (c < kSuspSlots) {
                susp_slots(a)[c] = key;
                *scnt() = c + 1;
                return true;
            }
        }
        return is_masked(a, b, it);
    }
    __device__ __forceinline__ void build_bloom(const ScoreArgs& a) {
#pragma unroll
        for (int w = 0; w < kBloomWords; ++w) bl[w] = 0u;
        if (!a.mask_indptr || !user_ok) return;
        const int64_t m0 = a.mask_indptr[b], m1 = a.mask_indptr[b + 1];
        for (int64_t j = m0; j < m1; ++j) {
            const int32_t x = a.mask_indices[j];
            bloom_set(bloom_h1(x));
            bloom_set(bloom_h2(x));
        }
    }

    __device__ __forceinline__ void init(uint64_t* keys_w, uint64_t* pend_w, int k_, int lane, int64_t b_, bool ok) {
        k = k_;
        h = lane >> 5;
        b = b_;
        user_ok = ok;
        keys = keys_w + (lane & 31) * kstride(k);
        len = 0;
        mp = 0;
        kmin = 0;
        pend = pend_w + lane * (kPend + 1);
        pcnt = 0;
        tau = ok ? -INFINITY : INFINITY;  // padding users never produce candidates
        tau_i = 0x7fffffff;
        mn = INFINITY;
        mx = -INFINITY;
        park = false;
    }
    // the list starts as the user's top-k over the seed items (already mask-filtered, so the keys go
    // in without tests); both lane halves read the same entries and hold the same {len, mp, kmin}
    __device__ __forceinline__ void seed(const ScoreArgs& a) {
        if (!user_ok) return;
        const float* ss = a.seed_score + (size_t)b * k;
        const int32_t* si = a.seed_idx + (size_t)b * k;
        int n = 0;
        for (int j = 0; j < k; ++j) {
            const int32_t it = si[j];
            if (it < 0) continue;
            if (h == 0) keys[n] = make_key(ss[j], it);
            ++n;
        }
        __builtin_amdgcn_wave_barrier();  // half 0's list writes precede half 1's reads
        len = n;
        if (len == k) rescan();
        refresh_tau();
    }
    // every LDS launch with a mask: each (user, split) has its own region, so the splits of a
    // split launch park too.  With propagated LightGCN tables a user's masked (train) items are
    // among its best scores, so each of them reaches the filter once per sweep: searched at once in
    // the sweep that is a chain of dependent global loads per masked item (Procedure.Test's shapes)
    __device__ __forceinline__ void enable_suspects(const ScoreArgs& a, int split) {
        park = a.susp && a.mask_indptr;  // wave-uniform
        sp = split;
        if (park) *scnt() = 0;
    }
    // this lane's parked-key count: the int after the wave's pending slots (list_bytes_per_wave)
    __device__ __forceinline__ int* scnt() const {
        const int l = (int)(threadIdx.x & 63);
        return reinterpret_cast<int*>(pend + (64 - l) * (kPend + 1)) + l;
    }
    // recomputed on use (rare) instead of held in registers
    __device__ __forceinline__ uint64_t* susp_slots(const ScoreArgs& a) const {
        return a.susp + (((size_t)b * a.n_splits + sp) * 2 + h) * kSuspSlots;
    }

    // new worst entry: 8 keys (four 16-byte reads issued together) per LDS round trip.  The whole
    // 8-key groups need no bounds test; the tail group (k % 8 keys) reads only the pairs it needs
    // when it holds at most 4 (k = 20: two whole groups and two reads)
    template <int N, bool MASK>
    __device__ __forceinline__ void rescan_group(int j0, uint64_t& m, int& p) const {
        uint64_t v[N];
#pragma unroll
        for (int j = 0; j < N; j += 2) {
            const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(keys + j0 + j);
            v[j] = q.x;
            v[j + 1] = q.y;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const uint64_t x = (!MASK || j0 + j < k) ? v[j] : ~0ull;
            if (x < m) {
                m = x;
                p = j0 + j;
            }
        }
    }
    __device__ __forceinline__ void rescan() {
        uint64_t m = ~0ull;
        int p = 0;
        const int kw = k & ~7;  // keys in whole groups
        for (int j0 = 0; j0 < kw; j0 += 8) rescan_group<8, false>(j0, m, p);
        if (k - kw > 4) rescan_group<8, true>(kw, m, p);
        else if (k > kw) rescan_group<4, true>(kw, m, p);
        mp = p;
        kmin = m;
    }

    // consume NACC (1 or 2) 32-item accumulator tiles; tile j's item rows start at i0 + 32 j
    // (items >= i_end ignored).  Fast path: a max tree and ONE compare per lane against tau,
    // OR-ed into a wave-wide flag.  Rows past i_end (tail block only) are set to -inf first.
    // L16: the scores come from the 16x16x32 main loop after its lane exchange (exchange16): lane
    // half h holds items 16 q + 8 h + (r & 7) of 16-item block q = 2 j + (r >> 3); otherwise the
    // 32x32x16 accumulator layout, items 32 j + (r & 3) + 8 (r >> 2) + 4 h
    // TAIL: the block may run past i_end (callers that know it does not pass false, so that the
    // common path never rewrites the accumulators and the compiler keeps them where they are)
    template <bool MINMAX, int NACC, bool L16 = false, bool TAIL = true>
    __device__ __forceinline__ void block(const ScoreArgs& a, f32x16 acc0, f32x16 acc1, int64_t i0, int64_t i_end) {
        const int64_t ib = i0 + (L16 ? 8 : 4) * h;  // item of accumulator row 0 of this lane half
        const bool tail = TAIL && i0 + 32 * NACC > i_end;
        const int64_t rem64 = i_end - ib;
        const int32_t rem = rem64 > (1 << 30) ? (1 << 30) : (int32_t)rem64;  // offsets < rem are items
        if (tail) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (row_off<L16>(0, r) >= rem) acc0[r] = -INFINITY;
                if (NACC == 2 && row_off<L16>(1, r) >= rem) acc1[r] = -INFINITY;
            }
        }
        // maxima of the 8-score groups {acc0 rows 0-7, 8-15, acc1 rows 0-7, 8-15}: the fast-path
        // test, and the event path visits only groups whose maximum reaches tau
        float g[2 * NACC];
#pragma unroll
        for (int q = 0; q < 2 * NACC; ++q) {
            const f32x16& acc = q < 2 ? acc0 : acc1;
            const int r0 = (q & 1) * 8;
            g[q] = fmaxf(fmaxf(fmaxf(acc[r0], acc[r0 + 1]), fmaxf(acc[r0 + 2], acc[r0 + 3])),
                         fmaxf(fmaxf(acc[r0 + 4], acc[r0 + 5]), fmaxf(acc[r0 + 6], acc[r0 + 7])));
        }
        float m = fmaxf(g[0], g[1]);
        if (NACC == 2) m = fmaxf(m, fmaxf(g[2], g[3]));
        if (MINMAX && user_ok) {
            float lo = INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                lo = fminf(lo, acc0[r] == -INFINITY ? INFINITY : acc0[r]);
                if (NACC == 2) lo = fminf(lo, acc1[r] == -INFINITY ? INFINITY : acc1[r]);
            }
            mn = fminf(mn, lo);
            mx = fmaxf(mx, m);
        }
        if (__ballot(m >= tau) == 0ull) return;  // wave-uniform fast path
        // the wave with an event is the one the workgroup barrier waits for: its VALU work goes
        // ahead of the partner's issue (+1.3 % at the C5 probe; static priority per wave half
        // measured no change)
        __builtin_amdgcn_s_setprio(2);
        slow<NACC, L16>(a, acc0, acc1, g, ib, rem);
        __builtin_amdgcn_s_setprio(0);
    }

    template <bool L16 = false>
    __device__ __forceinline__ static int32_t row_off(int j, int r) {
        return L16 ? 32 * j + 16 * (r >> 3) + (r & 7) : 32 * j + (r & 3) + 8 * (r >> 2);
    }

    __device__ __forceinline__ static int32_t pend_item(uint64_t v) { return (int32_t)(v >> 32); }
    __device__ __forceinline__ static uint64_t pend_key(uint64_t v) {
        return make_key(__uint_as_float((uint32_t)v), pend_item(v));
    }

    // true while some lane's filter admits every score: a list still filling with no floor under it
    // (the sweep's first block); such a wave takes the exact path, deferring would overflow at once
    __device__ __forceinline__ bool unbounded() const { return len < k && tau == -INFINITY; }

    template <int NACC, bool L16>
    __device__ __forceinline__ void slow(const ScoreArgs& a, const f32x16& acc0, const f32x16& acc1, const float* g,
                                         int64_t ib, int32_t rem) {
        // Every filter bounded (full lists, or filling lists above their floor): each score >= tau of
        // a group some lane flagged is appended to this lane's deferred slots without branching -- an
        // unconditional 8-B LDS write to slot min(n, kPend) and n += (score >= tau) -- so an event
        // costs a few instructions per score whatever the lanes do.  Ties at tau and masked items are
        // sorted out when the slots are drained (exact key compare, mask test).  A lane that runs past
        // its slots (n > kPend) drains every lane's slots; with REDEFER the block is then deferred again
        // against the drained lists (their thresholds rose, the slots are empty), and only a lane that
        // overruns them still sends the block down the exact path: insert every survivor directly.  An
        // unbounded filter takes that path too.
        auto defer = [&]() -> bool {
            int n = pcnt;
#pragma unroll
            for (int q = 0; q < 2 * NACC; ++q) {
                if (__ballot(g[q] >= tau) == 0ull) continue;  // no lane has a survivor in this group
#pragma unroll
                for (int rr = 0; rr < 8; ++rr) {
                    const int j = q >> 1, r = (q & 1) * 8 + rr;
                    const float sc = j ? acc1[r] : acc0[r];
                    const uint32_t item = (uint32_t)((int32_t)ib + row_off<L16>(j, r));
                    pend[min(n, kPend)] = ((uint64_t)item << 32) | __float_as_uint(sc);
                    n += sc >= tau ? 1 : 0;
                }
            }
            if (__ballot(n > kPend) != 0ull) return false;
            pcnt = n;
            return true;
        };
        if (__ballot(unbounded()) == 0ull && defer()) return;
        drain(a);
        if (REDEFER && __ballot(unbounded()) == 0ull && defer()) return;
        insert_now<NACC, L16>(a, acc0, acc1, ib, survivors<NACC, L16>(acc0, acc1, ib, rem));
    }

    template <bool L16>
    __device__ __forceinline__ int32_t item_of(int64_t ib, int r) const {
        return (int32_t)ib + row_off<L16>(r >> 4, r & 15);
    }
    template <int NACC>
    __device__ __forceinline__ static float pick(const f32x16& acc0, const f32x16& acc1, int r) {
        float sc = acc0[0];
#pragma unroll
        for (int q = 1; q < 16; ++q) sc = ((r & 15) == q) ? acc0[q] : sc;
        if (NACC == 2 && r >= 16) {
            sc = acc1[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) sc = ((r & 15) == q) ? acc1[q] : sc;
        }
        return sc;
    }
    // exact survivors of a block against the current list (bounds, index tie-break), branch-free;
    // item tests are relative to the lane's first item so the per-score offsets are constants
    template <int NACC, bool L16>
    __device__ __forceinline__ uint32_t survivors(const f32x16& acc0, const f32x16& acc1, int64_t ib,
                                                  int32_t rem) const {
        // a filling list takes every score at or above its floor (tau: -inf without one)
        const bool notfull = len < k;
        const int64_t l64 = (int64_t)tau_i - ib;
        const int32_t lim = l64 > (1 << 30) ? (1 << 30) : l64 < -1 ? -1 : (int32_t)l64;
        uint32_t cmask = 0;
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float sc = j ? acc1[r] : acc0[r];
                const int32_t off = row_off<L16>(j, r);
                const bool beats = (notfull & (sc >= tau)) | (sc > tau) | ((sc == tau) & (off < lim));
                cmask |= (user_ok & (off < rem) & beats) ? (1u << (16 * j + r)) : 0u;
            }
        }
        return cmask;
    }

    // one candidate into this lane's user list (the caller serialises the two lane halves);
    // CHECK: test the mask here (drained keys were already filtered by drop_masked)
    template <bool CHECK>
    __device__ __forceinline__ void insert_key(const ScoreArgs& a, uint64_t key) {
        if (len == k) {
            if (key <= kmin || (CHECK && masked(a, key))) return;
            keys[mp] = key;
            rescan();
        } else {
            if (CHECK && masked(a, key)) return;
            keys[len++] = key;
            if (len == k) rescan();
        }
    }

    // bit j of the result: pending key j is NOT masked.  The filter rules most keys out; the rest
    // are looked up by up to kPend binary searches advanced in lockstep, so each level issues its
    // loads together and waits once (a global load also waits for the in-flight tile DMA).
    __device__ __forceinline__ uint32_t drop_masked(const ScoreArgs& a) {
        uint32_t keep = (1u << pcnt) - 1u;
        if (!a.mask_indptr) return keep;
        int32_t it[kPend];
        uint32_t need = 0;
#pragma unroll
        for (int j = 0; j < kPend; ++j) {
            it[j] = j < pcnt ? pend_item(pend[j]) : 0;
            if (j < pcnt && bloom_test(bloom_h1(it[j])) && bloom_test(bloom_h2(it[j]))) need |= 1u << j;
        }
        if (__ballot(need != 0u) == 0ull) return keep;
        if (park) {  // park them while slots last
            int c = *scnt();
            for (int j = 0; j < kPend; ++j) {
                if (((need >> j) & 1u) && c < kSuspSlots) {
                    susp_slots(a)[c] = pend_key(pend[j]);
                    ++c;
                    keep &= ~(1u << j);
                    need &= ~(1u << j);
                }
            }
            *scnt() = c;
            if (__ballot(need != 0u) == 0ull) return keep;
        }
        const int64_t m0 = need ? a.mask_indptr[b] : 0, m1 = need ? a.mask_indptr[b + 1] : 0;
        const int32_t* mi = a.mask_indices + m0;
        // the searches run kSearch keys at a time: all kPend at once would hold 5 x kPend registers
        // live here, which at 12 slots pushes the walk's long-lived state into scratch
        constexpr int kSearch = kPend < 4 ? kPend : 4;
        for (int j0 = 0; j0 < kPend; j0 += kSearch) {
            if (__ballot(((need >> j0) & ((1u << kSearch) - 1u)) != 0u) == 0ull) continue;
            int32_t lo[kSearch], hi[kSearch], its[kSearch];
#pragma unroll
            for (int j = 0; j < kSearch; ++j) {
                lo[j] = 0;
                hi[j] = j0 + j < kPend && ((need >> (j0 + j)) & 1u) ? (int32_t)(m1 - m0) : 0;
                its[j] = 0;
#pragma unroll
                for (int q = 0; q < kPend; ++q) its[j] = q == j0 + j ? it[q] : its[j];
            }
            // first index with mi[idx] >= it, for every needed key of the batch at once
            auto searching = [&]() {
                bool any = false;
#pragma unroll
                for (int j = 0; j < kSearch; ++j) any |= lo[j] < hi[j];
                return any;
            };
            while (__ballot(searching()) != 0ull) {
                int32_t v[kSearch];
#pragma unroll
                for (int j = 0; j < kSearch; ++j) v[j] = lo[j] < hi[j] ? mi[(lo[j] + hi[j]) >> 1] : 0;
#pragma unroll
                for (int j = 0; j < kSearch; ++j) {
                    if (lo[j] < hi[j]) {
                        const int32_t mid = (lo[j] + hi[j]) >> 1;
                        if (v[j] < its[j]) lo[j] = mid + 1;
                        else hi[j] = mid;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kSearch; ++j) {
                const bool needed = j0 + j < kPend && ((need >> (j0 + j)) & 1u);
                const int32_t w = needed && lo[j] < (int32_t)(m1 - m0) ? mi[lo[j]] : -1;
                if (needed && w == its[j]) keep &= ~(1u << (j0 + j));
            }
        }
        return keep;
    }

    // after half ph changed the list: the other half adopts {len, mp, kmin} (cross-half swap)
    __device__ __forceinline__ void sync_from(int ph) {
        __builtin_amdgcn_wave_barrier();  // list writes of half ph precede the other half's reads
        const uint32_t lm = other_half((uint32_t)len | ((uint32_t)mp << 16));
        const uint32_t klo = other_half((uint32_t)kmin), khi = other_half((uint32_t)(kmin >> 32));
        if (ph != h) {
            len = (int)(lm & 0xffffu);
            mp = (int)(lm >> 16);
            kmin = ((uint64_t)khi << 32) | klo;
        }
    }
    __device__ __forceinline__ void refresh_tau() {
        if (len == k && user_ok) {
            tau = key_score(kmin);
            tau_i = key_index(kmin);
        }
    }
    // insert every deferred candidate of the wave: mask filter for both halves at once, then the
    // list updates half by half
    __device__ __forceinline__ void drain(const ScoreArgs& a) {
        if (__ballot(pcnt > 0) == 0ull) return;
        const uint32_t keep = drop_masked(a);
        for (int ph = 0; ph < 2; ++ph) {
            if (__ballot(ph == h && pcnt > 0) == 0ull) continue;
            if (ph == h) {
                for (int j = 0; j < pcnt; ++j)
                    if ((keep >> j) & 1u) insert_key<false>(a, pend_key(pend[j]));
            }
            sync_from(ph);
        }
        pcnt = 0;
        refresh_tau();
    }
    // insert a block's survivors directly (pending list already drained)
    template <int NACC, bool L16>
    __device__ __forceinline__ void insert_now(const ScoreArgs& a, const f32x16& acc0, const f32x16& acc1, int64_t ib,
                                               uint32_t cmask) {
        for (int ph = 0; ph < 2; ++ph) {
            if (__ballot(ph == h && cmask != 0) == 0ull) continue;
            if (ph == h) {
                uint32_t todo = cmask;
                while (todo) {  // one copy of the insertion code, one iteration per survivor
                    const int r = __builtin_ctz(todo);
                    todo &= todo - 1;
                    insert_key<true>(a, make_key(pick<NACC>(acc0, acc1, r), item_of<L16>(ib, r)));
                }
            }
            sync_from(ph);
        }
        refresh_tau();
    }

    template <bool MINMAX>
    __device__ __forceinline__ void tile(const ScoreArgs& a, const f32x16& acc, int64_t i0, int64_t i_end) {
        block<MINMAX, 1>(a, acc, acc, i0, i_end);
    }

    // exact mask test of the parked keys, then the survivors go in half by half
    __device__ __forceinline__ void resolve_suspects(const ScoreArgs& a) {
        if (!park) return;
        const int n = user_ok ? *scnt() : 0;
        if (__ballot(n > 0) == 0ull) return;
        const uint64_t* susp = susp_slots(a);
        uint32_t ok = 0;
        for (int j = 0; j < n; ++j)
            if (!is_masked(a, b, key_index(susp[j]))) ok |= 1u << j;
        for (int ph = 0; ph < 2; ++ph) {
            if (__ballot(ph == h && ok != 0u) == 0ull) continue;
            if (ph == h) {
                for (int j = 0; j < n; ++j)
                    if ((ok >> j) & 1u) insert_key<false>(a, susp[j]);
            }
            sync_from(ph);
        }
        *scnt() = 0;
        refresh_tau();
    }

    __device__ __forceinline__ void flush(const ScoreArgs& a, int split, int lane) {
        drain(a);
        resolve_suspects(a);
        if (user_ok && h == 0) {
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
typedef WaveTopKT<kPendSlots> WaveTopK;


template <int DT, int KCH, bool MINMAX, int WPB>
__global__ __launch_bounds__(WPB * 64) void score_topk_kernel(ScoreArgs a) {
    typedef Frag<DT> F;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int k = a.k;
    uint64_t* lk = reinterpret_cast<uint64_t*>(smem + (size_t)wave * list_bytes_per_wave(k));

    const int64_t b = (int64_t)blockIdx.x * (WPB * kUsersPerWave) + wave * kUsersPerWave + col;  // this lane's user
    const bool user_ok = b < a.B;
    const int64_t qrow = user_ok ? (a.user_rows ? a.user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(a.Q, qrow, a.d, c, h, user_ok);
    WaveTopK st;
    st.init(lk, lk + list_keys_per_wave(k), k, lane, b, user_ok);
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
        st.template tile<MINMAX>(a, acc, i0, i_end);
    }
    st.flush(a, split, lane);
}

// ---------------------------------------------------------------------------- bf16 LDS kernel
// 512 threads = 8 waves x 32 users; the workgroup streams 64-item tiles of its catalog split
// through a 2-4 buffer LDS ring filled by LDS-DMA (global_load_lds_dwordx4), so every item
// byte crosses L2 -> CU once per workgroup and feeds 8 waves.  Rows are stored with their 16-B
// chunks XOR-swizzled by (item & 15) so the fragment reads (32 items, same chunk) are
// conflict-free ds_read_b128s; the swizzle is applied to the DMA SOURCE address because the LDS
// destination of an LDS-DMA is lane-linear.  Splits are assigned so that the workgroups one XCD
// runs concurrently (blockIdx = xcd mod 8) sweep the same catalog slice and share its L2.
// Workgroup shape: WAVES x 32 users, tiles of 32*NACC items.  <8, 2> (one 512-thread workgroup per
// CU, 64-item tiles) is the one launched; see lds_waves() for the measured alternative.

// Modes of the LDS walk.  kTopK: the running top-k (lgx_score_topk).  kMinMaxOnly: only the
// global min / max of the scores (no top-k state touched): lgx_score_minmax, the reference's np.max /
// np.min over the full U x I matrix (recommend.py:163-164, :377).
constexpr int kTopK = 0;
constexpr int kMinMaxOnly = 1;
// kFloorOnly: the walk that writes each user's score floor (ScoreArgs::floor) over the first
// floor_items items of its split instead of a top-k: the items are cut into 64 groups by their
// position in the 64-item tile, a group holding a masked item of the user is dropped, and the floor
// is the k-th largest of the remaining group maxima.  Those are k distinct unmasked items scoring
// at least the floor, so the user's k-th best (over the split, hence over the catalog) is never below
// it, and a sweep that starts its lists with this threshold drops no item of the exact top-k (ties
// at the floor included: a filling list takes scores >= floor).  A product mode.
constexpr int kFloorOnly = 2;

template <int KSTEPS, int WAVES = 8, int NACC = 2, int ESZ = 2>
struct LdsGeom {
    static constexpr int TILE_ITEMS = 32 * NACC;
    static constexpr int USERS = WAVES * kUsersPerWave;
    static constexpr int RB = KSTEPS * 16 * ESZ;        // bytes per item row (d = 16*KSTEPS, ESZ-byte elements)
    static constexpr int CPR = RB / 16;                 // 16-B chunks per row
    static constexpr int TILE = TILE_ITEMS * RB;        // bytes per tile
    static constexpr int PIECES = TILE / 1024;          // 1-KiB LDS-DMA wave instructions per tile
    static constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
    // XOR swizzle inside aligned groups of P chunks, P = the largest power of two (<= 16)
    // dividing CPR, so that chunk ^ (row & SWZ) is a permutation of the row's chunks
    static constexpr int SWZ = ((CPR & -CPR) < 16 ? (CPR & -CPR) : 16) - 1;
};

// LDS-DMA of one 1-KiB piece: lane l copies 16 B from sbase + voff (its own offset) to LDS byte
// lds_addr + 16 l.  Issued from inline asm ON PURPOSE: the compiler's wait-count pass cannot tell
// the tiles of the LDS ring apart and would put an s_waitcnt vmcnt(0) in front of every later LDS
// read, which serialises the prefetch.  The kernel orders the DMA itself: counted vmcnt (this
// wave's pieces) + workgroup barrier (everyone's), as the hardware requires.
// M0 is a reserved register: clang accepts but ignores the clobber (-Winline-asm).  That is safe
// here because nothing else in this file uses M0 (the generated code's only M0 writes are these).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void lds_dma16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}
#pragma clang diagnostic pop

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (conservative above 15)
__device__ __forceinline__ void wait_vmcnt_le(int n) {
#define LGX_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    switch (n) {
        LGX_VMW(1) LGX_VMW(2) LGX_VMW(3) LGX_VMW(4) LGX_VMW(5) LGX_VMW(6) LGX_VMW(7) LGX_VMW(8)
        LGX_VMW(9) LGX_VMW(10) LGX_VMW(11) LGX_VMW(12) LGX_VMW(13) LGX_VMW(14) LGX_VMW(15)
        default:
            if (n >= 16) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#undef LGX_VMW
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Pipeline: nbuf tile buffers, nbuf-1 tiles in flight.  Iteration t issues tile t+nbuf-1 into the
// buffer tile t-1 used (every wave left it at the barrier closing t-1), computes tile t, then
// waits for its own pieces of tile t+1 (vmcnt leaves the younger tiles' pieces in flight) and
// joins the barrier that publishes tile t+1 to all waves.
//
// Stagger (STAGGER): waves w and w + WAVES/2 share a SIMD and would otherwise reach their MFMAs,
// their top-k epilogues and the barrier in lockstep, leaving the matrix unit idle during the
// epilogue.  The upper half of the waves runs each tile's epilogue one iteration late -- right after
// the barrier, before the MFMAs of the next tile -- so on every SIMD one wave's epilogue (VALU, LDS,
// mask loads) overlaps its partner's MFMAs.  The late epilogue only reads the accumulators, which
// stay in registers across the barrier; results are bit for bit those of the unstaggered order.
//
// MFMA shape: v_mfma_f32_16x16x32_bf16 holds a higher clock than 32x32x16 on random operands
// (tools/mfma_peak: 1962 vs 1615 TF/s bare, same FLOPs per cycle).  A wave's 32 users are two
// 16-user B blocks and its 64-item tile four 16-item A blocks: 8 accumulators of 4 scores.  One
// v_permlane16_swap per accumulator register then regroups them so that lane l holds 32 scores of
// user l & 31 (items 16 q + 8 h + 0..7 of block q), the layout the top-k state expects: lanes l and
// l + 32 still share a user.
//
// fp32 (DT = LGX_DTYPE_F32, score_topk_f32_lds): the same walk on v_mfma_f32_16x16x4_f32 (exact f32
// products and sums, the reference's precision).  A 16-B chunk of a row now holds 4 features, and
// the MFMA's k index q4 = lane >> 4 takes feature 16 s + 4 q4 + e at step (s, e): the same chunk
// (4 s + q4) of the item row and of the user row as the bf16 walk reads, so the LDS ring, the
// swizzle and the accumulator layout (hence the whole top-k epilogue) are shared.  At 1/16 of the
// bf16 MFMA rate a 64-item tile is 16 K MFMA cycles per wave, so the workgroup is 4 waves x 32 users,
// ONE wave per SIMD with the full 512-register file (the 32 users' f32 rows take 128 VGPRs), no
// stagger (no partner wave to overlap), a 2-buffer ring of 64 KB tiles at d = 256.
constexpr int kBf16LdsWaves = 8;
constexpr int kF32LdsWaves = 4;
// Producer / consumer walk (PC, fp32 at d = 64): WAVES = 8 waves, waves 0-3 consumers and 4-7
// producers; consumer w and producer w + 4 share a SIMD and 32 users.  The producer streams the tiles
// (LDS-DMA ring) and issues the MFMAs; it hands each tile's 32 x 64 scores, still in the MFMA layout,
// to its consumer through an LDS score buffer (two slots per pair), and the consumer runs the top-k
// epilogue, the mask and the exact path -- so a tile's events run on the SIMD beside the next tile's
// MFMAs instead of after them.  One workgroup barrier per tile: producer p writes tile t - 1's scores
// while it has tile t's MFMAs in flight, consumer p ranks tile t - 2.  kPcScoreSlot bytes per slot.
constexpr int kPcScoreSlot = 8 * 1024;
template <int DT, int KSTEPS, bool MINMAX, int MODE, int WAVES, int NACC, bool STAGGER, bool PC = false>
__device__ __forceinline__ void score_topk_lds_body(unsigned char* smem, ScoreArgs a, int xcd_affine,
                                                    int64_t n_utiles, int nbuf) {
    constexpr bool F32 = DT == LGX_DTYPE_F32;
    static_assert(NACC == 2 && (F32 || KSTEPS % 2 == 0), "16x16 walk: 64-item tiles, bf16 d a multiple of 32");
    static_assert(!PC || (F32 && WAVES == 8 && !STAGGER && !MINMAX && MODE != kMinMaxOnly), "PC: fp32 top-k / floor walk");
    constexpr int UW = PC ? WAVES / 2 : WAVES;  // waves that own users (and their lists)
    // SKIP: the fast-path test runs on the MFMA output layout itself (lane l holds 16 scores of user
    // l & 15 and 16 of user 16 + (l & 15)); the regroup into the top-k layout (16 v_permlane16_swap)
    // is paid only by tiles that have a survivor.  Min / max needs every score: not with MINMAX.
    constexpr bool SKIP = !MINMAX && MODE == kTopK;
    typedef LdsGeom<KSTEPS, UW, NACC, F32 ? 4 : 2> G;  // USERS = UW x 32; PPW: pieces per staging wave
    typedef Frag<DT> F;
    constexpr int NS = G::CPR / 4;                  // 16x16 walk: chunk groups (k-steps of 4 chunks) per row
    constexpr int UFN = 2 * NS;                     // user fragment registers (16 B each)
    unsigned char* tiles = smem;  // [nbuf][TILE]
    const int k = a.k;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, col = lane & 31;
    const bool producer = PC && wave >= UW;  // wave-uniform
    const int uwave = PC ? wave % UW : wave;  // the user block of this wave (its pair's, PC)
    typedef WaveTopKT<lds_pend(F32, KSTEPS, PC ? UW : WAVES), F32 && KSTEPS <= 8> TopK;
    unsigned char* sbuf_pc = smem + (size_t)nbuf * G::TILE;  // PC: [UW pairs][2 slots][kPcScoreSlot]
    uint64_t* lk = reinterpret_cast<uint64_t*>(sbuf_pc + (PC ? (size_t)UW * 2 * kPcScoreSlot : 0) +
                                               (size_t)uwave * list_bytes_per_wave(k, TopK::kPend));

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

    const int64_t b = utile * G::USERS + uwave * kUsersPerWave + col;
    const bool user_ok = b < a.B;
    uint4 uf[UFN];
    const int r16 = lane & 15, q4 = lane >> 4;
    // B fragment (ub, s) at uf[ub * NS + s]: user 16 ub + r16, 16-B chunk 4 s + q4 of its row
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
        const int64_t bu = utile * G::USERS + uwave * kUsersPerWave + 16 * ub + r16;
        const bool ok = bu < a.B && !(PC && !producer);  // PC: only producers hold the users' rows
        const int64_t qr = ok ? (a.user_rows ? a.user_rows[bu] : bu) : 0;
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2)
            uf[ub * NS + s2] = __builtin_bit_cast(uint4, F::load(a.Q, qr, a.d, 2 * s2 + (q4 >> 1), q4 & 1, ok));
    }
    TopK st;
    st.init(lk, lk + list_keys_per_wave(k), k, lane, b, user_ok && !producer);
    if (!producer) {
        st.enable_suspects(a, split);
        st.build_bloom(a);
        if (a.seed_score) st.seed(a);
        else if (MODE != kFloorOnly && a.floor && user_ok) st.tau = a.floor[b * a.n_splits + split];
    }
    // consume the prologue loads here: otherwise the compiler treats them as possibly pending at
    // the loop header and waits vmcnt(0) -- i.e. for the tile prefetch -- in every iteration
#pragma unroll
    for (int c = 0; c < UFN; ++c) {
        u32x4 t = __builtin_bit_cast(u32x4, uf[c]);
        asm volatile("" : "+v"(t));
        uf[c] = __builtin_bit_cast(uint4, t);
    }
#pragma unroll
    for (int w = 0; w < kBloomWords; ++w) asm volatile("" : "+v"(st.bl[w]));

    const int64_t i_begin = a.seed_items + (int64_t)split * a.split_items;
    const int64_t i_end = min(a.n_items, i_begin + (MODE == kFloorOnly ? min(a.split_items, a.floor_items) : a.split_items));
    const int64_t ntiles = i_end > i_begin ? (i_end - i_begin + G::TILE_ITEMS - 1) / G::TILE_ITEMS : 0;
    // single split: every workgroup sweeps the whole catalog, starting at a rotation shared by the
    // workgroups of its XCD (blockIdx mod 8) so that co-resident workgroups read the same tiles
    const int64_t rot = a.n_splits == 1 ? (bid % 8) * (ntiles / 8) : 0;
    const unsigned char* items = static_cast<const unsigned char*>(a.items);

    // this wave's pieces of a tile: LDS slot q = piece*64 + lane holds 16-B chunk (q % CPR) of tile
    // row q / CPR, fetched from source chunk (q % CPR) ^ (row & SWZ) (the swizzle lives on the source
    // side because the DMA's LDS destination is lane-linear)
    constexpr int PPW = G::PPW;
    const int swave = PC ? (producer ? uwave : UW) : wave;  // staging index (PC consumers stage nothing)
    const int my_pieces = max(0, min(PPW, G::PIECES - swave * PPW));
    const uint32_t lds_tiles = lds_u32(tiles);

    auto tile_start = [&](int64_t t) {
        int64_t u = t + rot;
        if (u >= ntiles) u -= ntiles;
        return i_begin + u * G::TILE_ITEMS;
    };
    auto stage_piece = [&](int buf, int64_t t0, int p) {
        if (p < my_pieces) {
            // wave-uniform by construction; readfirstlane keeps the base in SGPRs for the asm operand
            const uint64_t bu = reinterpret_cast<uint64_t>(items + t0 * G::RB);
            const unsigned char* base = reinterpret_cast<const unsigned char*>(
                ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bu));
            const bool tail = t0 + G::TILE_ITEMS > i_end;
            const int last = (int)(i_end - 1 - t0);  // tail rows re-read the split's last row (masked later)
            // offsets recomputed per tile: cheaper than holding them in registers
            const int q = (swave * PPW + p) * 64 + lane;
            const int row = q / G::CPR;
            const int src = (q % G::CPR) ^ (row & G::SWZ);
            const int srow = tail && row > last ? last : row;
            lds_dma16(base, (uint32_t)(srow * G::RB + src * 16),
                      __builtin_amdgcn_readfirstlane(lds_tiles + buf * G::TILE + (swave * PPW + p) * 1024));
        }
    };
    auto stage = [&](int buf, int64_t t0) {
#pragma unroll
        for (int p = 0; p < PPW; ++p) stage_piece(buf, t0, p);
    };

    const int ahead = nbuf - 1;
    for (int j = 0; j < ahead && j < ntiles; ++j) stage(j, tile_start(j));
    wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(ahead, ntiles) - 1));
    __syncthreads();
    int buf = 0, sbuf = ahead;  // buffer of tile t / of tile t + ahead
    const bool late = STAGGER && MODE != kMinMaxOnly && wave >= WAVES / 2;  // wave-uniform
    f32x16 acc0, acc1;  // late waves: tile t-1's scores, held across the barrier
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 c[2][4];      // 16x16x32 accumulators: c[ub][ib] = items 16 ib + 4 (lane >> 4) + reg, user 16 ub + (lane & 15)
    int64_t prev_t0 = 0;
    // SKIP: the thresholds of this lane's two MFMA-layout users (refreshed after every event)
    float tauA = st.tau, tauB = st.tau;
    auto refresh_taus = [&]() {
        tauA = __shfl(st.tau, lane & 15);
        tauB = __shfl(st.tau, 16 + (lane & 15));
    };
    if (SKIP) refresh_taus();
    // regroup: swap(X = user block 0, Y = user block 1) between rows 2m and 2m+1 (lanes l, l^16)
    // leaves X' = items 16 ib + 8 h + reg, Y' = items 16 ib + 8 h + 4 + reg of user l & 31
    auto regroup = [&]() {
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(c[0][ib][reg]),
                                                                 __float_as_uint(c[1][ib][reg]), false, false);
                const int r = 8 * (ib & 1) + reg;
                if (ib < 2) {
                    acc0[r] = __uint_as_float(sw[0]);
                    acc0[r + 4] = __uint_as_float(sw[1]);
                } else {
                    acc1[r] = __uint_as_float(sw[0]);
                    acc1[r + 4] = __uint_as_float(sw[1]);
                }
            }
        }
    };
    // scores of the tile in ring buffer `buf` into cc (c, or a PC producer's own pair of sets); with
    // MINMAX top-k also into acc0 / acc1 (the same code for both wave kinds)
    auto compute_into = [&](f32x4 (&cc)[2][4]) {
        const unsigned char* T = tiles + buf * G::TILE;
        constexpr int KS2 = NS;
#pragma unroll
        for (int ub = 0; ub < 2; ++ub)
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) cc[ub][ib] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        // A fragment (s, ib): item 16 ib + r16, source chunk 4 s + q4 (LDS chunk ^ row swizzle)
        const unsigned char* rowp = T + r16 * G::RB;
        auto frag = [&](int s2, int ib) {
            return *reinterpret_cast<const uint4*>(rowp + ib * 16 * G::RB + (((4 * s2 + q4) ^ (r16 & G::SWZ)) * 16));
        };
        // one fragment register per item block: its next k-step is read right after the two
        // MFMAs that consume it, so every read has the following 6 MFMAs to land
        uint4 fa[4];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) fa[ib] = frag(0, ib);
#pragma unroll
        for (int s2 = 0; s2 < KS2; ++s2) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
#pragma unroll
                for (int ub = 0; ub < 2; ++ub) {
                    if constexpr (F32) {
                        const float4 av = __builtin_bit_cast(float4, fa[ib]);
                        const float4 bv = __builtin_bit_cast(float4, uf[ub * KS2 + s2]);
                        cc[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, cc[ub][ib], 0, 0, 0);
                        cc[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, cc[ub][ib], 0, 0, 0);
                        cc[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, cc[ub][ib], 0, 0, 0);
                        cc[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, cc[ub][ib], 0, 0, 0);
                    } else {
                        cc[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, fa[ib]), __builtin_bit_cast(bf16x8, uf[ub * KS2 + s2]),
                            cc[ub][ib], 0, 0, 0);
                    }
                }
                if (s2 + 1 < KS2) fa[ib] = frag(s2 + 1, ib);
            }
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int s2 = 0; s2 < KS2; ++s2) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
                __builtin_amdgcn_sched_group_barrier(0x008, F32 ? 8 : 2, 0);
                if (s2 + 1 < KS2) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
        if (!SKIP && MODE == kTopK) regroup();
    };
    auto compute = [&]() { compute_into(c); };
    // the split's last tile is the only one that can run past i_end: a block variant of its own
    // min / max mode: every score of the tile straight from the MFMA layout.  Rows past the split's
    // end re-read its last item (stage_piece), so they hold real scores; padding users do not.
    const bool uok0 = utile * G::USERS + uwave * kUsersPerWave + r16 < a.B;
    const bool uok1 = utile * G::USERS + uwave * kUsersPerWave + 16 + r16 < a.B;
    auto minmax_tile = [&]() {
        float lo0 = c[0][0][0], hi0 = c[0][0][0], lo1 = c[1][0][0], hi1 = c[1][0][0];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                lo0 = fminf(lo0, c[0][ib][r]);
                hi0 = fmaxf(hi0, c[0][ib][r]);
                lo1 = fminf(lo1, c[1][ib][r]);
                hi1 = fmaxf(hi1, c[1][ib][r]);
            }
        st.mn = fminf(st.mn, fminf(uok0 ? lo0 : INFINITY, uok1 ? lo1 : INFINITY));
        st.mx = fmaxf(st.mx, fmaxf(uok0 ? hi0 : -INFINITY, uok1 ? hi1 : -INFINITY));
    };
    // floor mode: running maxima per (user, position in the tile), in the MFMA layout: gm[ub][ib][r]
    // = group 16 ib + 4 q4 + r of user 16 ub + r16.  Positions past the split's end (the tail tile's
    // re-read rows) stay out.
    f32x4 gm[2][4];
#pragma unroll
    for (int ub = 0; ub < 2; ++ub)
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) gm[ub][ib] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    auto floor_tile = [&](int64_t e0) {
        const int64_t rem = i_end - e0;
        if (rem >= G::TILE_ITEMS) {
#pragma unroll
            for (int ub = 0; ub < 2; ++ub)
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                    for (int r = 0; r < 4; ++r) gm[ub][ib][r] = fmaxf(gm[ub][ib][r], c[ub][ib][r]);
            return;
        }
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool in = 16 * ib + 4 * q4 + r < rem;
                gm[0][ib][r] = in ? fmaxf(gm[0][ib][r], c[0][ib][r]) : gm[0][ib][r];
                gm[1][ib][r] = in ? fmaxf(gm[1][ib][r], c[1][ib][r]) : gm[1][ib][r];
            }
    };
    auto epilogue = [&](int64_t e0) {
        if constexpr (MODE == kMinMaxOnly) {
            minmax_tile();
            return;
        }
        if constexpr (MODE == kFloorOnly) {
            floor_tile(e0);
            return;
        }
        const bool tail = e0 + G::TILE_ITEMS > i_end;
        if constexpr (SKIP) {
            if (!tail) {
                float m0 = c[0][0][0], m1 = c[1][0][0];
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        m0 = fmaxf(m0, c[0][ib][r]);
                        m1 = fmaxf(m1, c[1][ib][r]);
                    }
                if (__ballot((m0 >= tauA) | (m1 >= tauB)) == 0ull) return;  // wave-uniform fast path
                // maxima of one item block's 4-score groups (both user blocks), re-derived on events
                auto flagged = [&](int ib) {
                    const float a0 = fmaxf(fmaxf(c[0][ib][0], c[0][ib][1]), fmaxf(c[0][ib][2], c[0][ib][3]));
                    const float a1 = fmaxf(fmaxf(c[1][ib][0], c[1][ib][1]), fmaxf(c[1][ib][2], c[1][ib][3]));
                    return __ballot((a0 >= tauA) | (a1 >= tauB)) != 0ull;
                };
                // Every filter bounded (the sweep past its first tiles, or lists filling above their
                // floor): defer the flagged item blocks'
                // scores straight from the MFMA layout -- 4 v_permlane16_swap per block bring a
                // user's 8 scores of that block to its own lanes -- instead of regrouping all 32
                // scores and re-deriving the group maxima.  A lane whose slots would run over goes
                // down the full path below, which re-appends from pcnt (the writes here only went
                // to slots at or past it).
                if (__ballot(st.unbounded()) == 0ull) {
                    int n = st.pcnt;
                    const uint32_t ibase = (uint32_t)(e0 + 8 * h);
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib) {
                        if (!flagged(ib)) continue;
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg) {
                            const auto sw = __builtin_amdgcn_permlane16_swap(
                                __float_as_uint(c[0][ib][reg]), __float_as_uint(c[1][ib][reg]), false, false);
                            const uint32_t it = ibase + 16 * ib + reg;
                            st.pend[min(n, TopK::kPend)] = ((uint64_t)it << 32) | sw[0];
                            n += __uint_as_float(sw[0]) >= st.tau ? 1 : 0;
                            st.pend[min(n, TopK::kPend)] = ((uint64_t)(it + 4) << 32) | sw[1];
                            n += __uint_as_float(sw[1]) >= st.tau ? 1 : 0;
                        }
                    }
                    if (__ballot(n > TopK::kPend) == 0ull) {
                        st.pcnt = n;
                        return;
                    }
                }
            }
            regroup();
        }
        const float tau_before = st.tau;
        if (tail) st.template block<MINMAX, NACC, true, true>(a, acc0, acc1, e0, i_end);
        else st.template block<MINMAX, NACC, true, false>(a, acc0, acc1, e0, i_end);
        // the thresholds move only when a drain or a direct insert ran: most events only defer
        // candidates, and skip the two cross-lane reads
        if (SKIP && __ballot(st.tau != tau_before) != 0ull) refresh_taus();
    };
    // the refill is issued where the wave's issue port is least busy: the late waves before their
    // (VALU) epilogue, the early waves of a staggered walk between their MFMAs and their epilogue
    // (an LDS-DMA piece costs ~100-185 issue cycles inside the MFMA + fragment-read phase, ~25-60 in
    // a VALU phase: MI355X_MICROARCH.md).  Either way it lands in the buffer every wave released at
    // the previous barrier, and before this iteration's vmcnt wait.
    const bool stage_after = STAGGER && !late;  // wave-uniform
    if constexpr (PC) {
        // slot s of pair uwave: 8 lane-linear 16-B chunks per lane, c[ub][ib] at chunk 4 ub + ib
        auto slot = [&](int64_t t) { return sbuf_pc + ((size_t)uwave * 2 + (size_t)(t & 1)) * kPcScoreSlot + lane * 16; };
        // producer: tile t into one register set while the other (tile t - 1, its MFMAs issued an
        // iteration ago) goes to the score buffer -- no wait on this tile's MFMAs before the barrier.
        // The two roles run separate loops with the same barrier count, so their registers overlap.
        if (producer) {
            f32x4 cA[2][4], cB[2][4];
            auto iter = [&](int64_t t, f32x4 (&cur)[2][4], f32x4 (&prev)[2][4]) {
                if (t > 0 && t <= ntiles) {
                    unsigned char* sp = slot(t - 1);
#pragma unroll
                    for (int ub = 0; ub < 2; ++ub)
#pragma unroll
                        for (int ib = 0; ib < 4; ++ib)
                            *reinterpret_cast<f32x4*>(sp + (4 * ub + ib) * 1024) = prev[ub][ib];
                }
                if (t < ntiles) {
                    if (t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));
                    compute_into(cur);
                }
                wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));
                __syncthreads();
                buf = buf + 1 == nbuf ? 0 : buf + 1;
                sbuf = sbuf + 1 == nbuf ? 0 : sbuf + 1;
            };
            for (int64_t t = 0; t < ntiles + 2; t += 2) {
                iter(t, cA, cB);
                if (t + 1 < ntiles + 2) iter(t + 1, cB, cA);
            }
            return;
        }
        for (int64_t t = 0; t < ntiles + 2; ++t) {
            if (t >= 2) {  // tile t - 2, published by the previous barrier
                const unsigned char* sp = slot(t - 2);
#pragma unroll
                for (int ub = 0; ub < 2; ++ub)
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib) c[ub][ib] = *reinterpret_cast<const f32x4*>(sp + (4 * ub + ib) * 1024);
                epilogue(tile_start(t - 2));
            }
            __syncthreads();
        }
    } else
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t t0 = tile_start(t);
        if (!stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));
        if (late && t > 0) epilogue(prev_t0);
        compute();
        if (stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));
        if (!late) epilogue(t0);
        prev_t0 = t0;
        // tiles t+2 .. t+ahead may stay in flight; tile t+1 must have landed
        wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));
        __syncthreads();
        buf = buf + 1 == nbuf ? 0 : buf + 1;
        sbuf = sbuf + 1 == nbuf ? 0 : sbuf + 1;
    }
    if (late && ntiles > 0) epilogue(prev_t0);
    if constexpr (MODE == kMinMaxOnly) {
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
            st.mn = fminf(st.mn, __shfl_xor(st.mn, m, 64));
            st.mx = fmaxf(st.mx, __shfl_xor(st.mx, m, 64));
        }
        if (lane == 0 && st.mn <= st.mx) {
            atomicMin(a.minmax, ord_f32(st.mn));
            atomicMax(a.minmax + 1, ord_f32(st.mx));
        }
        return;
    }
    if constexpr (MODE == kFloorOnly) {
#pragma unroll
        for (int ub = 0; ub < 2; ++ub) {
            const int64_t bu = utile * G::USERS + uwave * kUsersPerWave + 16 * ub + r16;
            const bool ok = bu < a.B;
            // drop the groups that hold a masked item of the user (the mask rows are sorted)
            if (a.mask_indptr && ok) {
                const int64_t m1 = a.mask_indptr[bu + 1];
                for (int64_t j = a.mask_indptr[bu]; j < m1; ++j) {
                    const int64_t it = a.mask_indices[j];
                    if (it >= i_end) break;
                    if (it < i_begin) continue;
                    const int pos = (int)((it - i_begin) & 63);
                    if (((pos >> 2) & 3) != q4) continue;
#pragma unroll
                    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (pos == 16 * ib + 4 * q4 + r) gm[ub][ib][r] = -INFINITY;
                }
            }
            // k-th largest of the user's 64 group maxima (4 lanes q4 x 16 registers): k rounds of
            // take the maximum, then remove one copy of it (from the lowest q4 holding it)
            float kth = -INFINITY;
            for (int round = 0; round < k; ++round) {
                float lm = gm[ub][0][0];
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                    for (int r = 0; r < 4; ++r) lm = fmaxf(lm, gm[ub][ib][r]);
                float wm = fmaxf(lm, __shfl_xor(lm, 16, 64));
                wm = fmaxf(wm, __shfl_xor(wm, 32, 64));
                int owner = lm == wm ? q4 : 4;
                owner = min(owner, __shfl_xor(owner, 16, 64));
                owner = min(owner, __shfl_xor(owner, 32, 64));
                bool done = owner != q4;
#pragma unroll
                for (int ib = 0; ib < 4; ++ib)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const bool hit = !done && gm[ub][ib][r] == wm;
                        gm[ub][ib][r] = hit ? -INFINITY : gm[ub][ib][r];
                        done = done || hit;
                    }
                kth = wm;
            }
            if (ok && q4 == 0) a.floor[bu * a.n_splits + split] = kth;
        }
        return;
    }
    st.flush(a, split, lane);
}

template <int KSTEPS, bool MINMAX, int MODE = kTopK>
__global__ __launch_bounds__(kBf16LdsWaves * 64) __attribute__((amdgpu_waves_per_eu(2, 2)))
void score_topk_bf16_lds(ScoreArgs a, int xcd_affine, int64_t n_utiles, int nbuf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    score_topk_lds_body<LGX_DTYPE_BF16, KSTEPS, MINMAX, MODE, kBf16LdsWaves, 2, true>(
        smem, a, xcd_affine, n_utiles, nbuf);
}

// WAVES = 4: one wave per SIMD (d = 192, 256: the users' rows take 96-128 VGPRs).  WAVES = 8 (d <= 128,
// whose rows take <= 64 VGPRs): two waves per SIMD in the bf16 walk's staggered order, so one wave's
// top-k epilogue runs under its partner's MFMAs instead of between its own tiles.
template <int KSTEPS, bool MINMAX, int MODE = 0, int WAVES = kF32LdsWaves>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(WAVES / 4, WAVES / 4)))
void score_topk_f32_lds(ScoreArgs a, int xcd_affine, int64_t n_utiles, int nbuf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    score_topk_lds_body<LGX_DTYPE_F32, KSTEPS, MINMAX, MODE, WAVES, 2, (WAVES > 4)>(
        smem, a, xcd_affine, n_utiles, nbuf);
}

// the producer / consumer walk (PC) for fp32 d = 64: 4 consumer + 4 producer waves, 128 users
template <int KSTEPS, int MODE = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void score_topk_f32_pc(ScoreArgs a, int xcd_affine, int64_t n_utiles, int nbuf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    score_topk_lds_body<LGX_DTYPE_F32, KSTEPS, false, MODE, 8, 2, false, true>(smem, a, xcd_affine, n_utiles, nbuf);
}

__global__ void minmax_finish(const uint32_t* mm, float* out) {
    out[0] = unord_f32(mm[0]);
    out[1] = unord_f32(mm[1]);
}

// one wave per query: merge the split lists, masked tail, optional sigmoid (k <= 64 R)
template <int R>
__global__ __launch_bounds__(64) void score_topk_finalize(ScoreArgs a, float mask_value, int apply_sigmoid,
                                                          int32_t* __restrict__ out_idx, float* __restrict__ out_val,
                                                          float* __restrict__ minmax_out) {
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int k = a.k;
    const int64_t total = (int64_t)a.n_splits * k;
    const float* ps = a.part_score + (size_t)b * total;
    const int32_t* pi = a.part_idx + (size_t)b * total;
    WaveList<R> top;
    top.clear();
    for (int64_t base = 0; base < total; base += 64) {
        const int64_t j = base + lane;
        const uint64_t cand = (j < total && pi[j] >= 0) ? make_key(ps[j], pi[j]) : 0ull;
        top.push(cand, k, lane);
    }
    int n_real = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) n_real += __popcll(__ballot(top.t[r] != 0ull));
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = 64 * r + lane;
        if (e >= k) continue;
        const uint64_t key = top.t[r];
        int32_t idx = -1;
        float val = mask_value;
        if (key) {
            idx = key_index(key);
            const float s = key_score(key);
            val = apply_sigmoid ? 1.0f / (1.0f + expf(-s)) : s;
        } else if (a.mask_indptr) {
            const int64_t m0 = a.mask_indptr[b], m1 = a.mask_indptr[b + 1];
            const int64_t j = m0 + (e - n_real);
            if (j < m1) idx = a.mask_indices[j];
        }
        out_idx[b * k + e] = idx;
        if (out_val) out_val[b * k + e] = val;
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
// A workgroup is 8 waves x 32 users = 256 users that walk the SAME 32-item tiles of one catalog
// split in the same order, so a tile comes from HBM once per 256 users (the other waves find it in
// L1/L2) instead of once per 32: at [4096, 1M] d=256 that is 8 GB of item reads next to the 16 GB of
// scores written, not 64 GB.  Workgroup -> (user group, split) is XCD-aware: the workgroups of one
// XCD (blockIdx mod 8) take splits s = xcd (mod 8), all user groups of a split back to back, so the
// groups sharing a split also share that XCD's L2.
// the reference's sigmoid (model.py:183) over dense score matrices: exp2 and reciprocal on the
// transcendental unit, ~1e-6 relative to 1 / (1 + e^-x) (tests: 1e-5); the exact expf / IEEE division
// form is ~20 VALU per score and made the bf16 [4096, 1M] getUsersRating VALU-bound (3.67 -> 5.37 ms).
// Limits hold: x -> -inf gives rcp(inf) = 0, x -> +inf rcp(1) = 1.
__device__ __forceinline__ float fast_sigmoid(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
}

constexpr int kDenseWaves = 8;
constexpr int kDenseUsers = kDenseWaves * kUsersPerWave;

// SIG: the reference's sigmoid (model.py:183) as a template parameter: a runtime flag let the
// compiler evaluate expf for every score and select (profiles/r03_a6_runtime_sigmoid_flag.json,
// r03_a6_sigmoid_template.json: 3.83 -> 3.61 ms at [4096, 1M] d=256 bf16 on one box)
template <int DT, int KCH, bool SIG>
__global__ __launch_bounds__(kDenseWaves * 64) void score_dense_kernel(const void* Q, const int64_t* user_rows,
                                                                        const void* items, int64_t B, int64_t n_items,
                                                                        int64_t d, float* __restrict__ out,
                                                                        int64_t n_ug, int64_t split_items) {
    typedef Frag<DT> F;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug;
    const int64_t split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kDenseUsers + (int64_t)wave * kUsersPerWave;
    if (u0 >= B) return;  // whole wave idle (no workgroup barrier in this kernel)
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    const int64_t qrow = user_ok ? (user_rows ? user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(Q, qrow, d, c, h, user_ok);
    const int64_t i_begin = split * split_items;
    const int64_t i_end = std::min(n_items, i_begin + split_items);
    // the next tile's item fragments are in flight while this tile's MFMAs and stores run
    typename F::chunk fr[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) fr[c] = F::load(items, i_begin + col, d, c, h, i_begin + col < i_end);
    for (int64_t i0 = i_begin; i0 < i_end; i0 += 32) {
        const int64_t item_row = i0 + col;
        const bool item_ok = item_row < i_end;
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            acc = F::mma(uf[c], fr[c], acc);
            fr[c] = F::load(items, item_row + 32, d, c, h, item_row + 32 < i_end);
        }
        if (!item_ok) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int64_t u = u0 + tile_row(r, h);
            if (u < B) {
                const float sc = acc[r];
                out[u * n_items + item_row] = SIG ? fast_sigmoid(sc) : sc;
            }
        }
    }
}

// The same walk with the item tile staged in LDS once per workgroup (KCH >= 8): one 16-B global
// load per slot for the whole workgroup instead of one per wave, fragments read back with
// ds_read_b128 from an XOR-swizzled image (slot ^ (row & 15): the 16 rows a lane group reads sit in
// 16 different 4-bank groups).  Double-buffered: the next tile's loads are in flight during this
// tile's MFMAs and stores; one barrier per tile, so idle waves (past B) still take part.
//
// Occupancy and stores (round 3, tools/dense_lab.hip, profiles/r03_dense_lab*.txt): with <= 16 chunks
// (bf16; <= 8 for fp32) the kernel is held to 128 VGPRs, i.e. 4 waves per SIMD = two workgroups per CU, so one
// workgroup's MFMAs and stores run while the other waits for its tile (at 166 VGPRs a CU held one
// workgroup, whose waves all stall on the same tile load at each barrier).  The 16 score stores of
// a tile go out as a wave-uniform row base (SGPRs) plus one 32-bit lane byte offset instead of 16
// live 64-bit addresses, which is what makes 128 VGPRs fit without scratch.  [4096, 1M] d=256
// bf16: 4.40-4.96 -> 3.41-3.57 ms (same bits), against 2.45-3.01 ms for the bare store pattern.
// (fp32 rows hold half the features per chunk, and the f32 KCH = 16 walk needs a few more registers
// for its 4 MFMAs per chunk: 12 B of scratch at 128 VGPRs, so it keeps two waves per SIMD)
__host__ __device__ constexpr int dense_waves_per_simd(int dt, int kch) {
    return kch <= (dt == LGX_DTYPE_BF16 ? 16 : 8) ? 4 : 2;
}

template <int DT, int KCH, bool SIG>
__global__ __launch_bounds__(kDenseWaves * 64)
__attribute__((amdgpu_waves_per_eu(dense_waves_per_simd(DT, KCH), dense_waves_per_simd(DT, KCH))))
void score_dense_lds(const void* Q, const int64_t* user_rows, const void* items, int64_t B, int64_t n_items,
                     int64_t d, float* __restrict__ out, int64_t n_ug, int64_t split_items) {
    static_assert(KCH >= 8, "swizzle needs >= 16 slots per row");
    typedef Frag<DT> F;
    constexpr int SPR = 2 * KCH;           // 16-B slots per item row (a chunk = 32 B = two halves)
    constexpr int RB = SPR * 16;           // row bytes of the image
    constexpr int TILE = 32 * RB;
    constexpr int NL = 32 * SPR / (kDenseWaves * 64);  // slots per thread per tile
    static_assert(NL >= 1 && 32 * SPR % (kDenseWaves * 64) == 0, "tile slots must divide over the workgroup");
    __shared__ __attribute__((aligned(16))) unsigned char img[2][TILE];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug;
    const int64_t split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kDenseUsers + (int64_t)wave * kUsersPerWave;  // wave-uniform
    const bool wave_on = u0 < B;
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    const int64_t qrow = user_ok ? (user_rows ? user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(Q, qrow, d, c, h, user_ok);
    const int64_t i_begin = split * split_items;
    const int64_t i_end = std::min(n_items, i_begin + split_items);
    const int64_t row_bytes = d * (DT == LGX_DTYPE_F32 ? 4 : 2);
    const unsigned char* ib = static_cast<const unsigned char*>(items);
    uint4 nx[NL];
    auto load_tile = [&](int64_t i0) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kDenseWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            const int64_t it = i0 + r;
            nx[j] = (it < i_end && q * 16 < row_bytes)
                        ? *reinterpret_cast<const uint4*>(ib + it * row_bytes + q * 16)
                        : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kDenseWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            *reinterpret_cast<uint4*>(&img[buf][r * RB + ((q ^ (r & 15)) * 16)]) = nx[j];
        }
    };
    if (i_begin >= i_end) return;  // workgroup-uniform
    load_tile(i_begin);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    for (int64_t i0 = i_begin; i0 < i_end; i0 += 32) {
        const bool more = i0 + 32 < i_end;  // workgroup-uniform
        if (more) load_tile(i0 + 32);
        if (wave_on) {
            const unsigned char* rowp = &img[buf][col * RB];
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
            for (int c = 0; c < KCH; ++c) {
                const uint4 fr = *reinterpret_cast<const uint4*>(rowp + (((2 * c + h) ^ (col & 15)) * 16));
                acc = F::mma(uf[c], __builtin_bit_cast(typename F::chunk, fr), acc);
            }
            if (i0 + col < i_end) {
                // row base of register r: out + (u0 + tile_row(r, 0)) * n_items + i0 (uniform), lane
                // offset (4 h rows + col) in bytes (< 2^32: asserted by the host, 4 * n_items * 4 + 128)
                const uint32_t boff = ((uint32_t)(4 * h) * (uint32_t)n_items + (uint32_t)col) * 4u;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (u0 + tile_row(r, h) < B) {
                        const float sc = acc[r];
                        char* base = reinterpret_cast<char*>(out + (u0 + tile_row(r, 0)) * n_items + i0);
                        *reinterpret_cast<float*>(base + boff) = SIG ? fast_sigmoid(sc) : sc;
                    }
                }
            }
        }
        if (more) store_tile(buf ^ 1);  // last read in the previous iteration, before its barrier
        __syncthreads();
        buf ^= 1;
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

// ---------------------------------------------------------------------------- stratification labels
// f4 (recommend.py:375-381) fused: score_dense_lds's walk with the operands swapped (items are the
// A operand, users the B operand -- the same k order, so the same f32 sums bit for bit), so that lane
// (col, h) ends a tile holding 16 scores of ONE user (user u0 + col, items tile_row(r, h)): the
// labels of items 8q + 4h + 0..3 pack into one dword store.  A label is the count of thresholds the
// score reaches (lgx_strat_thresholds); nothing but the int8 labels leaves the chip.
struct StratThr {
    float t[32];
    int n;
    // estimate: floor(fma(s, inv, off)) is the label within +-1 (thresholds ~ evenly spaced; off =
    // -base * inv, one FMA per score instead of a subtract and a multiply)
    float base, inv, off;
};

// the label estimate of the kernel, on the host (the same single-rounding FMA as v_fma_f32)
inline int strat_estimate(float sc, const StratThr& thr) {
    const float x = std::fmaf(sc, thr.inv, thr.off);
    return (x >= (float)thr.n || x != x) ? thr.n : (x < 0.0f ? 0 : (int)x);
}
inline int strat_label_host(float sc, const StratThr& thr) {
    int l = 0;
    for (int j = 0; j < thr.n; ++j) l += sc >= thr.t[j] ? 1 : 0;
    return l;
}
// true when the estimate is within one of the label for every f32 score: both are monotone step
// functions, so it suffices to look at both ends of every interval on which the estimate is
// constant (found by bisection over the ordered f32 bit patterns)
inline bool strat_estimate_within_one(const StratThr& thr) {
    auto key = [](float f) {
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
    int64_t start = kmin;  // first f32 of the current estimate's interval
    while (true) {
        const int m = strat_estimate(unkey(start), thr);
        // last f32 whose estimate is m
        int64_t lo = start, hi = kmax;
        while (lo < hi) {
            const int64_t mid = lo + (hi - lo + 1) / 2;
            if (strat_estimate(unkey(mid), thr) <= m) lo = mid;
            else hi = mid - 1;
        }
        const int la = strat_label_host(unkey(start), thr), lb = strat_label_host(unkey(lo), thr);
        if (la < m - 1 || lb > m + 1) return false;
        if (lo >= kmax) return true;
        start = lo + 1;
    }
}

// label counts of the workgroup's 256 users kept in LDS (stride 17: the 32 users of a wave sit in
// 32 different banks), added to the global histogram once per workgroup
constexpr int kHistStride = 17;

template <int DT, int KCH, bool VEC4, bool EST1>
__global__ __launch_bounds__(kDenseWaves * 64) void strat_label_lds(const void* Q, const int64_t* user_rows,
                                                                     const void* items, int64_t B, int64_t n_items,
                                                                     int64_t d, StratThr thr,
                                                                     int8_t* __restrict__ labels,
                                                                     int32_t* __restrict__ hist, int64_t n_ug,
                                                                     int64_t split_items) {
    static_assert(KCH >= 8, "swizzle needs >= 16 slots per row");
    typedef Frag<DT> F;
    constexpr int SPR = 2 * KCH;
    constexpr int RB = SPR * 16;
    constexpr int TILE = 32 * RB;
    constexpr int NL = 32 * SPR / (kDenseWaves * 64);
    static_assert(NL >= 1 && 32 * SPR % (kDenseWaves * 64) == 0, "tile slots must divide over the workgroup");
    __shared__ __attribute__((aligned(16))) unsigned char img[2][TILE];
    // T[j] = the score where label j starts (T[0] = -inf, T[n + 1] = +inf): the label of s is the
    // estimate e corrected by one compare on each side, s < T[e] and s >= T[e + 1]
    __shared__ float T[34];
    __shared__ float2 TP[33];  // {T[j], T[j + 1]}: the estimate path's two thresholds in one 8-B read
    __shared__ uint32_t hc[kDenseUsers * kHistStride];  // hist != nullptr: per-user label counts
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    auto thr_at = [&](int j) { return j == 0 ? -INFINITY : (j <= thr.n ? thr.t[j - 1] : INFINITY); };
    if (threadIdx.x < 34) T[threadIdx.x] = thr_at(threadIdx.x);
    // TP[n].y = NaN: the estimate path's upper compare is false at the last label without a guard
    if (threadIdx.x < 33)
        TP[threadIdx.x] = make_float2(thr_at(threadIdx.x), (int)threadIdx.x < thr.n ? thr_at(threadIdx.x + 1) : NAN);
    if (hist)
        for (int e = threadIdx.x; e < kDenseUsers * kHistStride; e += kDenseWaves * 64) hc[e] = 0u;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug;
    const int64_t split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kDenseUsers + (int64_t)wave * kUsersPerWave;
    const bool wave_on = u0 < B;
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    const int64_t qrow = user_ok ? (user_rows ? user_rows[b] : b) : 0;
    typename F::chunk uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c) uf[c] = F::load(Q, qrow, d, c, h, user_ok);
    const int64_t i_begin = split * split_items;
    const int64_t i_end = std::min(n_items, i_begin + split_items);
    const int64_t row_bytes = d * (DT == LGX_DTYPE_F32 ? 4 : 2);
    const unsigned char* ib = static_cast<const unsigned char*>(items);
    int8_t* lab = labels + b * n_items;
    uint4 nx[NL];
    auto load_tile = [&](int64_t i0) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kDenseWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            const int64_t it = i0 + r;
            nx[j] = (it < i_end && q * 16 < row_bytes)
                        ? *reinterpret_cast<const uint4*>(ib + it * row_bytes + q * 16)
                        : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kDenseWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            *reinterpret_cast<uint4*>(&img[buf][r * RB + ((q ^ (r & 15)) * 16)]) = nx[j];
        }
    };
    auto label = [&](float sc) {
        const float x = __builtin_fmaf(sc, thr.inv, thr.off);
        int l = (int)__builtin_amdgcn_fmed3f(x, 0.0f, (float)thr.n);  // clamp to [0, n], then truncate
        if (x != x) l = thr.n;                                       // NaN -> n, as label_of
        if (EST1) {
            // the host proved |estimate - label| <= 1: one branch-free step each way.  TP[l] = {T[l],
            // T[l + 1]} with TP[0].x = -inf and TP[n].y = NaN, so neither compare needs a range guard
            const float2 tp = TP[l];
            return (uint32_t)(l - (sc < tp.x ? 1 : 0) + (sc >= tp.y ? 1 : 0));
        }
        while (l > 0 && sc < T[l]) --l;  // exact whatever the estimate
        while (l < thr.n && sc >= T[l + 1]) ++l;
        return (uint32_t)l;
    };
    if (i_begin >= i_end) return;  // workgroup-uniform
    auto mfmas = [&](int bf) {
        const unsigned char* rowp = &img[bf][col * RB];
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            const uint4 fr = *reinterpret_cast<const uint4*>(rowp + (((2 * c + h) ^ (col & 15)) * 16));
            acc = F::mma(__builtin_bit_cast(typename F::chunk, fr), uf[c], acc);
        }
        return acc;
    };
    // labels, counts and the packed stores of the tile at e0
    auto epilogue = [&](const f32x16& acc, int64_t e0) {
        // whole tiles (all but a split's last) skip the per-item bounds tests
        auto emit = [&](auto whole_tag) {
            constexpr bool WHOLE = decltype(whole_tag)::value;
            uint32_t* hu = hc + (wave * kUsersPerWave + col) * kHistStride;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t it = e0 + 8 * q + 4 * h;  // items it .. it + 3: acc rows 4q .. 4q + 3
                const uint32_t l0 = label(acc[4 * q]), l1 = label(acc[4 * q + 1]);
                const uint32_t l2 = label(acc[4 * q + 2]), l3 = label(acc[4 * q + 3]);
                const uint32_t w = l0 | (l1 << 8) | (l2 << 16) | (l3 << 24);
                if (hist) {  // items past the split's end are not counted
                    if (WHOLE || it < i_end) atomicAdd(hu + l0, 1u);
                    if (WHOLE || it + 1 < i_end) atomicAdd(hu + l1, 1u);
                    if (WHOLE || it + 2 < i_end) atomicAdd(hu + l2, 1u);
                    if (WHOLE || it + 3 < i_end) atomicAdd(hu + l3, 1u);
                }
                if (VEC4 && (WHOLE || it + 4 <= i_end)) {
                    *reinterpret_cast<uint32_t*>(lab + it) = w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (it + e < i_end) lab[it + e] = (int8_t)((w >> (8 * e)) & 255);
                }
            }
        };
        if (user_ok) {
            if (e0 + 32 <= i_end) emit(std::true_type{});
            else emit(std::false_type{});
        }
    };
    // Staggered halves, as in score_dense_lds: the late waves (4-7) label tile t-1 right after the
    // barrier and run tile t's MFMAs last, so each SIMD issues one wave's MFMAs while the other
    // labels.  One loop per half (the halves take the same barriers), so only the late loop carries
    // accumulators across its barrier.
    const bool late = wave >= kDenseWaves / 2;  // wave-uniform
    load_tile(i_begin);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    if (late) {
        f32x16 acc;
        int64_t prev_i0 = -1;
        for (int64_t t0 = i_begin; t0 < i_end; t0 += 32) {
            const bool more = t0 + 32 < i_end;  // workgroup-uniform
            if (more) load_tile(t0 + 32);
            if (wave_on) {
                if (prev_i0 >= 0) epilogue(acc, prev_i0);
                acc = mfmas(buf);
            }
            if (more) store_tile(buf ^ 1);
            prev_i0 = t0;
            __syncthreads();
            buf ^= 1;
        }
        if (wave_on) epilogue(acc, prev_i0);
        __syncthreads();  // the counts of the last tile, before the flush below
    } else {
        for (int64_t t0 = i_begin; t0 < i_end; t0 += 32) {
            const bool more = t0 + 32 < i_end;  // workgroup-uniform
            if (more) load_tile(t0 + 32);
            if (wave_on) epilogue(mfmas(buf), t0);
            if (more) store_tile(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
        __syncthreads();
    }
    if (hist) {  // the last barrier has published every count
        const int64_t ub = ug * kDenseUsers;
        for (int e = threadIdx.x; e < kDenseUsers * kHistStride; e += kDenseWaves * 64) {
            const int uu = e / kHistStride, l = e % kHistStride;
            const uint32_t c = hc[e];
            if (c && l <= thr.n && ub + uu < B) atomicAdd(hist + (ub + uu) * (thr.n + 1) + l, (int32_t)c);
        }
    }
}

struct SplitPlan {
    int n_splits;
    int64_t split_items;
    bool lds;        // LDS-DMA kernel (score_topk_bf16_lds / score_topk_f32_lds)
    bool xcd_affine;
    int64_t n_utiles;
    int waves;       // LDS kernel workgroup: 8 waves (bf16, two per SIMD) or 4 (f32, one per SIMD)
};

// LDS kernel shape.  bf16: <8 waves, 64-item tiles>, one workgroup per CU; the two-workgroups-per-CU
// shape <4, 1> was measured slower (902 vs 1079 TF/s unmasked, 131072 users, d=256): halving the tile
// doubles the barriers per MFMA, which costs more than the overlap of two independent workgroups
// recovers.  f32: <4 waves, 64-item tiles>, one workgroup (one wave per SIMD) per CU.  Either way one
// workgroup per CU, 256 resident.
inline int64_t lds_resident() { return 256; }

constexpr size_t kLdsBytes = 160 * 1024;
constexpr int kTileItems = 64;
// fp32 LDS walk: 8 staggered waves (two per SIMD) where the users' rows leave the registers for it
// (d <= 128) and two tiles fit beside 8 waves' lists, else 4 waves
inline bool f32_lds8_fits(int64_t d, int k) {
    return d <= 128 && 2 * (size_t)kTileItems * d * 4 + 8 * list_bytes_per_wave(k, lds_pend(true, (int)(d / 16))) <= kLdsBytes;
}
inline int lds_waves(int dtype, int64_t d, int k) {
    return dtype == LGX_DTYPE_F32 ? (f32_lds8_fits(d, k) ? 8 : kF32LdsWaves) : kBf16LdsWaves;
}
// LDS kernel applies to bf16 with d a multiple of 32 up to 256 (even k-step counts are
// instantiated) and to f32 with d a multiple of 64 up to 256, whenever two 64-item tiles fit beside
// the top-k lists (8 waves with 12 deferred slots per lane / 4 waves with 4): d = 256 up to k = 20
// (both dtypes), bf16 d <= 128 up to k = 32; other shapes run the register-fragment kernel
bool lds_eligible(int dtype, int64_t d, int k) {
    if (dtype == LGX_DTYPE_BF16)
        return d % 32 == 0 && d >= 32 && d <= 256 && k <= 32 &&
               2 * (size_t)kTileItems * d * 2 + 8 * list_bytes_per_wave(k, kPendBf16Lds) <= kLdsBytes;
    if (dtype != LGX_DTYPE_F32 || d % 64 != 0 || d < 64 || d > 256 || k > 32) return false;
    return 2 * (size_t)kTileItems * d * 4 + (size_t)kF32LdsWaves * list_bytes_per_wave(k, lds_pend(true, (int)(d / 16), kF32LdsWaves)) <=
           kLdsBytes;
}

SplitPlan plan_lds_splits(int64_t B, int64_t n_items, int dtype, int waves);

SplitPlan plan_splits(int64_t B, int64_t n_items, int dtype, int64_t d, int k) {
    const int64_t tiles32 = ceil_div(n_items, 32);
    if (lds_eligible(dtype, d, k)) {
        const int waves = lds_waves(dtype, d, k);
        if (dtype == LGX_DTYPE_F32 && waves == 8) {
            // 256-user workgroups halve the user tiles: where that alone turns one catalog sweep into
            // a split launch, the 4-wave walk without splits is faster (Gowalla shape, 27 522 users:
            // 4 waves x 1 split 3.07 ms, 8 waves x 2 splits 3.20-3.23 ms unmasked top-20,
            // profiles/r05_eval_shapes_ab_*.txt)
            const SplitPlan p8 = plan_lds_splits(B, n_items, dtype, 8);
            const SplitPlan p4 = plan_lds_splits(B, n_items, dtype, kF32LdsWaves);
            return p8.n_splits > 1 && p4.n_splits == 1 ? p4 : p8;
        }
        return plan_lds_splits(B, n_items, dtype, waves);
    }
    const int64_t user_blocks = ceil_div(B, (int64_t)v1_waves(k) * kUsersPerWave);
    int64_t s = ceil_div(2048, user_blocks);                       // aim for >= ~8 workgroups per CU
    s = std::min<int64_t>(s, std::max<int64_t>(1, tiles32 / 8));  // >= 8 tiles per split
    s = std::max<int64_t>(1, std::min<int64_t>(s, 64));
    const int64_t per = ceil_div(tiles32, s) * 32;
    return {(int)ceil_div(n_items, per), per, false, false, user_blocks, 0};
}

SplitPlan plan_lds_splits(int64_t B, int64_t n_items, int dtype, int waves) {
    {
        const int64_t users = waves * kUsersPerWave, tile_items = kTileItems;
        const int64_t resident = lds_resident();
        const int64_t ut = ceil_div(B, users);
        const int64_t tiles = ceil_div(n_items, tile_items);
        // a full round or more: no catalog split -- every split repeats the list-filling phase, which
        // costs more than a partly filled last round (which plan_ranges moves to a split launch)
        if (ut >= resident) return {1, tiles * tile_items, true, false, ut, waves};
        // under one round: split the catalog.  Time ~ rounds / s * f(s): each split repeats the
        // list-filling phase, measured +18 / +25 / +31 % per doubling of s from 2 to 16 (bf16, C5
        // catalog), i.e. log2 f = 0.12 L + 0.04 L^2 with L = log2 s.  fp32 at the evaluation shapes
        // (catalogs of 40-90 K items, every tile of a split's start an event) pays more per split:
        // log2 f = 0.25 L + 0.04 L^2 there.  Take the best s among 1-7 and multiples of 8
        // (XCD-affine), >= 4 tiles per split
        const double a1 = dtype == LGX_DTYPE_F32 ? 0.25 : 0.12;
        int64_t s = 1;
        double best = 1e300;
        const int64_t s_max = std::max<int64_t>(1, std::min<int64_t>(256, tiles / 4));
        for (int64_t c = 1; c <= s_max; c = c < 8 ? c + 1 : c + 8) {
            const double L = std::log2((double)c);
            const double t = (double)ceil_div(ut * c, resident) / (double)c * std::exp2(a1 * L + 0.04 * L * L);
            if (t < best - 1e-12) {
                best = t;
                s = c;
            }
        }
        const int64_t per = ceil_div(tiles, s) * tile_items;
        const int n = (int)ceil_div(n_items, per);
        return {n, per, true, n % 8 == 0, ut, waves};
    }
}

template <typename KernelT>
int set_lds_limit(KernelT kernel, size_t shmem) {
    if (shmem > 65536)
        LGX_HIP_CHECK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
    return LGX_OK;
}

template <int DT, bool MM, int WPB>
int launch_v1_waves(const ScoreArgs& a, int kch, hipStream_t stream) {
    const size_t shmem = (size_t)WPB * list_bytes_per_wave(a.k);
    dim3 grid((unsigned)ceil_div(a.B, (int64_t)WPB * kUsersPerWave), (unsigned)a.n_splits);
#define LGX_SK(KC)                                                                      \
    do {                                                                                \
        int rc_ = set_lds_limit(score_topk_kernel<DT, KC, MM, WPB>, shmem);            \
        if (rc_) return rc_;                                                            \
        score_topk_kernel<DT, KC, MM, WPB><<<grid, WPB * 64, shmem, stream>>>(a);      \
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

template <int DT, bool MM>
int launch_v1(const ScoreArgs& a, int kch, hipStream_t stream) {
    return v1_waves(a.k) == 4 ? launch_v1_waves<DT, MM, 4>(a, kch, stream) : launch_v1_waves<DT, MM, 1>(a, kch, stream);
}

// tile buffers of the LDS kernel: as many as fit beside the top-k lists in the workgroup's share of
// the CU's LDS, 2..4
inline int lds_ring_buffers(size_t tile, size_t lists, int wg_per_cu) {
    const size_t budget = kLdsBytes / wg_per_cu;
    const size_t fit = lists < budget ? (budget - lists) / tile : 0;
    return (int)std::max<size_t>(2, std::min<size_t>(4, fit));
}

template <int KS, bool MM, int MODE>
int launch_bf16_lds_kernel(const ScoreArgs& a, const SplitPlan& p, hipStream_t stream) {
    typedef LdsGeom<KS, kBf16LdsWaves, 2> G;
    const size_t lists = (size_t)kBf16LdsWaves * list_bytes_per_wave(a.k, kPendBf16Lds);
    const int nbuf = lds_ring_buffers(G::TILE, lists, 1);
    const size_t shmem = (size_t)nbuf * G::TILE + lists;
    int rc = set_lds_limit(score_topk_bf16_lds<KS, MM, MODE>, shmem);
    if (rc) return rc;
    const unsigned grid = (unsigned)(p.n_utiles * p.n_splits);
    score_topk_bf16_lds<KS, MM, MODE><<<grid, kBf16LdsWaves * 64, shmem, stream>>>(a, p.xcd_affine ? 1 : 0,
                                                                                    p.n_utiles, nbuf);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

template <int KS, bool MM, int MODE, int WAVES = kF32LdsWaves>
int launch_f32_lds_kernel(const ScoreArgs& a, const SplitPlan& p, hipStream_t stream) {
    typedef LdsGeom<KS, WAVES, 2, 4> G;
    const size_t lists = (size_t)WAVES * list_bytes_per_wave(a.k, lds_pend(true, KS, WAVES));
    const int nbuf = lds_ring_buffers(G::TILE, lists, 1);
    const size_t shmem = (size_t)nbuf * G::TILE + lists;
    if (shmem > kLdsBytes) {
        set_error("lgx_score_topk: f32 LDS kernel needs %zu B of LDS", shmem);
        return LGX_ERR_UNSUPPORTED;
    }
    int rc = set_lds_limit(score_topk_f32_lds<KS, MM, MODE, WAVES>, shmem);
    if (rc) return rc;
    const unsigned grid = (unsigned)(p.n_utiles * p.n_splits);
    score_topk_f32_lds<KS, MM, MODE, WAVES><<<grid, WAVES * 64, shmem, stream>>>(a, p.xcd_affine ? 1 : 0,
                                                                                  p.n_utiles, nbuf);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

// the producer / consumer walk replaces the 4-wave fp32 walk at d = 64: the top-k sweep and, since
// the roles run separate loops (no spill), its floor pass (Gowalla route 2.77 -> 2.66 ms, r06w)
// where two ring tiles, the score buffers and the 4 consumers' lists fit the LDS (k <= 24 at 16 slots)
inline bool f32_pc(const SplitPlan& p, int64_t d, int k, bool mm) {
    return p.waves == kF32LdsWaves && d == 64 && !mm &&
           2 * (size_t)kTileItems * 64 * 4 + (size_t)kF32LdsWaves * 2 * kPcScoreSlot +
                   (size_t)kF32LdsWaves * list_bytes_per_wave(k, lds_pend(true, 4, kF32LdsWaves)) <= kLdsBytes;
}

template <int KS, int MODE>
int launch_f32_pc_kernel(const ScoreArgs& a, const SplitPlan& p, hipStream_t stream) {
    typedef LdsGeom<KS, kF32LdsWaves, 2, 4> G;
    const size_t lists = (size_t)kF32LdsWaves * list_bytes_per_wave(a.k, lds_pend(true, KS, kF32LdsWaves));
    const size_t sb = (size_t)kF32LdsWaves * 2 * kPcScoreSlot;
    const int nbuf = lds_ring_buffers(G::TILE, lists + sb, 1);
    const size_t shmem = (size_t)nbuf * G::TILE + sb + lists;
    if (shmem > kLdsBytes) {
        set_error("lgx_score_topk: f32 producer/consumer kernel needs %zu B of LDS", shmem);
        return LGX_ERR_UNSUPPORTED;
    }
    int rc = set_lds_limit(score_topk_f32_pc<KS, MODE>, shmem);
    if (rc) return rc;
    const unsigned grid = (unsigned)(p.n_utiles * p.n_splits);
    score_topk_f32_pc<KS, MODE><<<grid, 512, shmem, stream>>>(a, p.xcd_affine ? 1 : 0, p.n_utiles, nbuf);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

template <bool MM, int MODE = kTopK>
int launch_lds(const ScoreArgs& a, const SplitPlan& p, hipStream_t stream, int dtype = LGX_DTYPE_BF16) {
    const int ksteps = (int)(a.d / 16);
    {
        if (dtype == LGX_DTYPE_F32) {
            if (p.waves == 8) {
                switch (ksteps) {
                    case 4: return launch_f32_lds_kernel<4, MM, MODE, 8>(a, p, stream);
                    case 8: return launch_f32_lds_kernel<8, MM, MODE, 8>(a, p, stream);
                    default:
                        set_error("lgx_score_topk: no 8-wave f32 LDS kernel for d=%lld", (long long)a.d);
                        return LGX_ERR_UNSUPPORTED;
                }
            }
            if constexpr (!MM && MODE != kMinMaxOnly)  // the top-k sweep and its floor pass
                if (f32_pc(p, a.d, a.k, MM)) return launch_f32_pc_kernel<4, MODE>(a, p, stream);
            switch (ksteps) {
                case 4: return launch_f32_lds_kernel<4, MM, MODE>(a, p, stream);
                case 8: return launch_f32_lds_kernel<8, MM, MODE>(a, p, stream);
                case 12: return launch_f32_lds_kernel<12, MM, MODE>(a, p, stream);
                case 16: return launch_f32_lds_kernel<16, MM, MODE>(a, p, stream);
                default:
                    set_error("lgx_score_topk: no f32 LDS kernel for d=%lld", (long long)a.d);
                    return LGX_ERR_UNSUPPORTED;
            }
        }
    }
#define LGX_SL(KS) return launch_bf16_lds_kernel<KS, MM, MODE>(a, p, stream)
    switch (ksteps) {
        case 2: LGX_SL(2);
        case 4: LGX_SL(4);
        case 6: LGX_SL(6);
        case 8: LGX_SL(8);
        case 10: LGX_SL(10);
        case 12: LGX_SL(12);
        case 14: LGX_SL(14);
        case 16: LGX_SL(16);
        default:
            set_error("lgx_score_topk: no LDS kernel for d=%lld", (long long)a.d);
            return LGX_ERR_UNSUPPORTED;
    }
#undef LGX_SL
}

// A batch runs as up to two launches over user ranges.  In the LDS kernel's full-sweep mode every
// round runs the resident workgroups; when the last round would leave most of them idle, the users
// of that partial round become a second launch whose catalog splits fill the chip.
struct UserRange {
    int64_t u0, u1;
    SplitPlan p;
    size_t ws_off;  // partial lists of this range inside the workspace
};

// workspace of one range: the split lists (scores, then indices), then the LDS kernel's parked keys
size_t range_list_bytes(const UserRange& r, int k) { return align_up((size_t)(r.u1 - r.u0) * r.p.n_splits * k * 4); }
size_t range_susp_bytes(const UserRange& r) {
    return r.p.lds ? align_up((size_t)(r.u1 - r.u0) * r.p.n_splits * 2 * kSuspSlots * 8) : 0;
}
// the LDS kernel's score floors [users, n_splits]
size_t range_floor_bytes(const UserRange& r) { return r.p.lds ? align_up((size_t)(r.u1 - r.u0) * r.p.n_splits * 4) : 0; }
size_t range_ws_bytes(const UserRange& r, int k) {
    return 2 * range_list_bytes(r, k) + range_susp_bytes(r) + range_floor_bytes(r);
}

int plan_ranges(int64_t B, int64_t n_items, int dtype, int64_t d, int k, UserRange* r) {
    const SplitPlan p = plan_splits(B, n_items, dtype, d, k);
    int n = 0;
    int64_t full = B;
    const int64_t resident = lds_resident();
    if (p.lds && p.n_splits == 1 && p.n_utiles >= resident) {  // full-sweep mode
        const int64_t rem_tiles = p.n_utiles % resident;
        // measured: a 67-tile tail (of 256) runs faster as a split launch, a 135-tile one slower (bf16,
        // C5); fp32 tiles are 16x longer per event, and a 156-tile tail of the Amazon-book shape runs
        // 9 % faster split (profiles/r04_eval_probe_ab.txt)
        const int64_t cut = dtype == LGX_DTYPE_F32 ? 75 : 35;
        if (rem_tiles != 0 && rem_tiles * 100 < resident * cut) full = (p.n_utiles - rem_tiles) * p.waves * kUsersPerWave;
    }
    size_t off = 0;
    r[n++] = {0, full, plan_splits(full, n_items, dtype, d, k), 0};
    if (full < B) r[n++] = {full, B, plan_splits(B - full, n_items, dtype, d, k), 0};
    for (int i = 0; i < n; ++i) {
        r[i].ws_off = off;
        off += range_ws_bytes(r[i], k);
    }
    return n;
}

// Seeded full sweeps: the catalog is swept in stages [0, 16384), [16384, 32768), ... (doubling while
// a stage ends before 2/3 of the catalog), then the rest; each stage is a launch of its own whose
// lists (the split-list workspace) seed the next, which reads and overwrites them in place.  Exact
// (same kernel, same scores, the lists are sets).  The event-dense start of the sweep runs apart from
// its quiet remainder, and every stage restarts the co-resident workgroups of an XCD on the same
// tile, so their drift (and L2 misses) stays bounded.  Lab, 983 040 users x 1M items, masked: one
// sweep 463.7 ms, these 7 stages 431.9 ms (-6.9 %); 2 stages -2 %, 3 stages -4 %
// (profiles/r02_score_lab_seeded.txt, profiles/r02_score_lab_stages.txt).
constexpr int64_t kSeedItems = 16384;
inline bool seeded_sweep(const SplitPlan& p, bool minmax, int64_t n_items) {
    return p.lds && p.n_splits == 1 && !minmax && n_items >= 16 * kSeedItems;
}
// Score floors (kFloorOnly): an unseeded LDS sweep -- the first stage of a seeded sweep, or every
// split of a split launch -- starts its lists at a floor taken from its first kFloorItems items
// instead of at -inf, which turns the list-filling start (every tile an event for every wave, the
// exact path throughout) into a filter that passes about k scores per user.  Lab, 131072 users x
// 1M items, d=256 bf16, masked (profiles/r03_score_lab_stageprof.txt, r03_score_lab_floor.txt): the
// first stage [0, 16384) 5.10 ms, of which 4.24 ms events; with floors over its first 2048 / 4096 /
// 8192 / 16384 items (the pass included) 4.26 / 3.78 / 3.30 / 2.87 ms, all 7 stages 57.84 ->
// 54.40 ms at 16384, lists identical.  Splits shorter than 4 x kFloorItems go without.
// fp32: at the C5 catalog (seeded stages) its events are cheap beside its 16x slower tiles and the
// pass cost more than it saved (bench fp32 leg 1044 -> 1052 ms with floors).  At the evaluation
// shapes (catalogs under 262 144 items, no seeded stages) the one-wave-per-SIMD walk (4 waves) has
// no partner wave to hide its events under, and a streaming top-k meets most of its ~k ln(n / k)
// insertions early: there the floor over each split's first eighth pays (Gowalla shape, propagated
// tables, the route's fused part 3.25 -> 2.89 ms; profiles/r05_eval_variants.txt).  The 8-wave walk
// hides its events under the partner's MFMAs and gained nothing (Amazon-book shape 14.95 -> 15.08 ms),
// nor did top-1 (few events: 1.89 -> 1.96 ms).
constexpr int64_t kFloorItems = 16384;
constexpr int64_t kF32FloorMinSplit = 4096;
inline int64_t floor_items_for(const SplitPlan& p, int dtype, int64_t n_items, int k) {
    if (dtype == LGX_DTYPE_BF16) return p.split_items >= 4 * kFloorItems ? kFloorItems : 0;
    if (p.waves != kF32LdsWaves || k < 8 || n_items >= 16 * kSeedItems || p.split_items < kF32FloorMinSplit) return 0;
    return ceil_div(ceil_div(p.split_items, 8), (int64_t)kTileItems) * kTileItems;
}
inline bool floored(const SplitPlan& p, bool minmax, int dtype, int64_t n_items, int k) {
    return p.lds && !minmax && floor_items_for(p, dtype, n_items, k) > 0;
}

size_t topk_ws_bytes(int64_t B, int64_t n_items, int k, int dtype, int64_t d) {
    UserRange r[2];
    const int n = plan_ranges(B, n_items, dtype, d, k, r);
    size_t bytes = 0;
    for (int i = 0; i < n; ++i) bytes += range_ws_bytes(r[i], k);
    return bytes + 512;  // + the global min / max words
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_score_topk_workspace(int64_t B, int64_t n_items, int k, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && B >= 0 && n_items >= 0 && k >= 1, LGX_ERR_INVALID_ARG,
                "lgx_score_topk_workspace: bad arguments");
    // the split plan depends on dtype / d; report the maximum over every kernel variant
    size_t m = 0;
    for (int64_t d = 16; d <= 256; d += 16)
        m = std::max({m, topk_ws_bytes(B, n_items, k, LGX_DTYPE_BF16, d), topk_ws_bytes(B, n_items, k, LGX_DTYPE_F32, d)});
    *ws_bytes = m;
    return LGX_OK;
}

extern "C" int lgx_score_topk_plan(int64_t B, int64_t n_items, int64_t d, int dtype, int k, char* buf, size_t len) {
    LGX_REQUIRE(buf && len > 0 && B > 0 && n_items > 0 && k >= 1 && k <= kMaxTopK, LGX_ERR_INVALID_ARG,
                "lgx_score_topk_plan: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_score_topk_plan: dtype");
    UserRange r[2];
    const int n = plan_ranges(B, n_items, dtype, d, k, r);
    size_t off = 0;
    for (int i = 0; i < n && off < len; ++i) {
        const SplitPlan& p = r[i].p;
        const char* kern = p.lds ? (dtype == LGX_DTYPE_F32 ? (p.waves == 8 ? "score_topk_f32_lds<8 waves, 64-item tiles, 16x16x4>"
                                                              : f32_pc(p, d, k, false) ? "score_topk_f32_lds<4 waves + 4 producers, 64-item tiles, 16x16x4>"
                                                                                    : "score_topk_f32_lds<4 waves, 64-item tiles, 16x16x4>")
                                                           : "score_topk_bf16_lds<8 waves, 64-item tiles, 16x16x32>")
                                 : (v1_waves(k) == 4 ? "score_topk_kernel<4 waves>" : "score_topk_kernel<1 wave>");
        const char* mode = p.lds ? (p.n_splits == 1 ? "full-sweep" : (p.xcd_affine ? "split-xcd" : "split"))
                                 : "split";
        off += snprintf(buf + off, len - off, "%s%s users[%lld,%lld) %s%s%s n_splits=%d utiles=%lld",
                        i ? "; " : "", kern, (long long)r[i].u0, (long long)r[i].u1, mode,
                        seeded_sweep(p, false, n_items) ? " (seeded in stages)" : "",
                        floored(p, false, dtype, n_items, k) ? " (score floors)" : "", p.n_splits,
                        (long long)p.n_utiles);
    }
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
    LGX_REQUIRE(k >= 1 && k <= kMaxTopK, LGX_ERR_UNSUPPORTED, "lgx_score_topk: k=%d outside [1, %d]", k, kMaxTopK);
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    const int kch = kch_for(dtype, d);
    LGX_REQUIRE(d > 0 && d % vec == 0 && kch > 0, LGX_ERR_UNSUPPORTED,
                "lgx_score_topk: d=%lld must be a multiple of %lld and <= 256", (long long)d, (long long)vec);
    if (B == 0) return LGX_OK;
    LGX_REQUIRE(n_items > 0 && n_items < INT32_MAX && Q && items, LGX_ERR_INVALID_ARG,
                "lgx_score_topk: empty or oversized catalog");
    const size_t need = topk_ws_bytes(B, n_items, k, dtype, d);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_score_topk: workspace %zu < %zu", ws_bytes, need);
    UserRange ranges[2];
    const int n_ranges = plan_ranges(B, n_items, dtype, d, k, ranges);
    char* base = static_cast<char*>(ws);
    uint32_t* minmax = minmax_out ? reinterpret_cast<uint32_t*>(base + need - 512) : nullptr;
    if (minmax) {
        minmax_init<<<1, 1, 0, stream>>>(minmax);
        LGX_LAUNCH_CHECK();
    }
    const bool mm = minmax_out != nullptr;
    const size_t esz = dtype == LGX_DTYPE_F32 ? 4 : 2;
    for (int i = 0; i < n_ranges; ++i) {
        const UserRange& R = ranges[i];
        const SplitPlan& p = R.p;
        const int64_t Bi = R.u1 - R.u0;
        const size_t list_bytes = range_list_bytes(R, k);
        char* wsr = base + R.ws_off;
        const void* Qi = user_rows ? Q : static_cast<const void*>(static_cast<const char*>(Q) + R.u0 * d * esz);
        ScoreArgs a{Qi, user_rows ? user_rows + R.u0 : nullptr, items, Bi, n_items, d,
                    mask_indptr ? mask_indptr + R.u0 : nullptr, mask_indices, k, p.n_splits, p.split_items,
                    reinterpret_cast<float*>(wsr), reinterpret_cast<int32_t*>(wsr + list_bytes), minmax,
                    range_susp_bytes(R) ? reinterpret_cast<uint64_t*>(wsr + 2 * list_bytes) : nullptr};
        int rc;
        if (floored(p, mm, dtype, n_items, k)) {  // every split's floor over its first items; the sweep reads them
            a.floor = reinterpret_cast<float*>(wsr + 2 * list_bytes + range_susp_bytes(R));
            a.floor_items = floor_items_for(p, dtype, n_items, k);
            rc = launch_lds<false, kFloorOnly>(a, p, stream, dtype);
            if (rc) return rc;
        }
        if (seeded_sweep(p, mm, n_items)) {
            rc = LGX_OK;
            for (int64_t lo = 0, hi = kSeedItems; lo < n_items && rc == LGX_OK; lo = hi, hi *= 2) {
                ScoreArgs st = a;
                st.n_items = 3 * hi < 2 * n_items ? hi : n_items;
                st.seed_items = lo;
                st.split_items = st.n_items - lo;
                if (lo > 0) {  // seeded: the floor is for the unseeded first stage only
                    st.seed_score = a.part_score;
                    st.seed_idx = a.part_idx;
                    st.floor = nullptr;
                }
                rc = launch_lds<false>(st, p, stream, dtype);
                if (st.n_items == n_items) break;
            }
        } else if (p.lds) rc = mm ? launch_lds<true>(a, p, stream, dtype) : launch_lds<false>(a, p, stream, dtype);
        else if (dtype == LGX_DTYPE_F32) rc = mm ? launch_v1<LGX_DTYPE_F32, true>(a, kch, stream)
                                                 : launch_v1<LGX_DTYPE_F32, false>(a, kch, stream);
        else rc = mm ? launch_v1<LGX_DTYPE_BF16, true>(a, kch, stream)
                     : launch_v1<LGX_DTYPE_BF16, false>(a, kch, stream);
        if (rc) return rc;
        // min / max is final after the last range's kernel (stream order): only its finalize reports it
        int32_t* oi = out_idx + R.u0 * k;
        float* ov = out_val ? out_val + R.u0 * k : nullptr;
        float* om = i + 1 == n_ranges ? minmax_out : nullptr;
        if (k <= 64) score_topk_finalize<1><<<(unsigned)Bi, 64, 0, stream>>>(a, mask_value, apply_sigmoid, oi, ov, om);
        else if (k <= 128) score_topk_finalize<2><<<(unsigned)Bi, 64, 0, stream>>>(a, mask_value, apply_sigmoid, oi, ov, om);
        else score_topk_finalize<4><<<(unsigned)Bi, 64, 0, stream>>>(a, mask_value, apply_sigmoid, oi, ov, om);
        LGX_LAUNCH_CHECK();
    }
    return LGX_OK;
}

extern "C" int lgx_score_minmax_workspace(int64_t B, int64_t n_items, size_t* ws_bytes) {
    LGX_REQUIRE(ws_bytes && B >= 0 && n_items >= 0, LGX_ERR_INVALID_ARG, "lgx_score_minmax_workspace: bad arguments");
    size_t topk = 0;
    const int rc = lgx_score_topk_workspace(B, n_items, 1, &topk);
    if (rc) return rc;
    // the LDS walk needs the 2 ordered words only; shapes it does not cover go through the top-1
    // path, which needs its workspace plus [B] index / value outputs
    *ws_bytes = 512 + align_up(topk) + 2 * align_up((size_t)B * 4);
    return LGX_OK;
}

extern "C" int lgx_score_minmax(const void* Q, const int64_t* user_rows, const void* items, int64_t B, int64_t n_items,
                                int64_t d, int dtype, float* minmax_out, void* ws, size_t ws_bytes,
                                lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(B > 0 && n_items > 0 && n_items < INT32_MAX && Q && items && minmax_out, LGX_ERR_INVALID_ARG,
                "lgx_score_minmax: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG, "lgx_score_minmax: dtype");
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    LGX_REQUIRE(d > 0 && d % vec == 0 && kch_for(dtype, d) > 0, LGX_ERR_UNSUPPORTED,
                "lgx_score_minmax: d=%lld must be a multiple of %lld and <= 256", (long long)d, (long long)vec);
    size_t need = 0;
    lgx_score_minmax_workspace(B, n_items, &need);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_score_minmax: workspace %zu < %zu", ws_bytes, need);
    char* base = static_cast<char*>(ws);
    uint32_t* mm = reinterpret_cast<uint32_t*>(base);
    const bool lds_ok = lds_eligible(dtype, d, 1) &&
                        (dtype == LGX_DTYPE_BF16 ? (d / 16) % 2 == 0 : (d / 16) % 4 == 0);
    if (!lds_ok) {  // the top-1 launch with its min / max output
        size_t topk = 0;
        lgx_score_topk_workspace(B, n_items, 1, &topk);
        int32_t* oi = reinterpret_cast<int32_t*>(base + 512 + align_up(topk));
        float* ov = reinterpret_cast<float*>(base + 512 + align_up(topk) + align_up((size_t)B * 4));
        return lgx_score_topk(Q, user_rows, items, B, n_items, d, dtype, nullptr, nullptr, 1, -INFINITY, 0, oi, ov,
                              minmax_out, base + 512, align_up(topk), stream_);
    }
    minmax_init<<<1, 1, 0, stream>>>(mm);
    LGX_LAUNCH_CHECK();
    const SplitPlan p = plan_splits(B, n_items, dtype, d, 1);
    ScoreArgs a{Q, user_rows, items, B, n_items, d, nullptr, nullptr, 1, p.n_splits, p.split_items,
                nullptr, nullptr, mm, nullptr};
    const int rc = launch_lds<false, kMinMaxOnly>(a, p, stream, dtype);
    if (rc) return rc;
    minmax_finish<<<1, 1, 0, stream>>>(mm, minmax_out);
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
    // splits: a multiple of 8 (one residue class per XCD), enough workgroups to fill the chip
    const int64_t n_ug = ceil_div(B, (int64_t)kDenseUsers);
    const int64_t tiles = ceil_div(n_items, 32);
    const int64_t n_splits = std::max<int64_t>(8, std::min(8 * ceil_div(ceil_div(2048, n_ug), 8), 8 * ceil_div(tiles, 8)));
    const int64_t split_items = 32 * ceil_div(tiles, n_splits);
    const int64_t grid = n_ug * n_splits;
    LGX_REQUIRE(grid < (1LL << 31), LGX_ERR_UNSUPPORTED, "lgx_score_dense: %lld users is too many", (long long)B);
    LGX_REQUIRE(n_items < (1LL << 27), LGX_ERR_UNSUPPORTED, "lgx_score_dense: %lld items is too many (< 2^27)",
                (long long)n_items);
#define LGX_SD3(DTV, KC, SG)                                                                                   \
    if constexpr (KC >= 8)                                                                                     \
        score_dense_lds<DTV, KC, SG><<<(unsigned)grid, kDenseWaves * 64, 0, stream>>>(Q, user_rows, items, B,   \
                                                                                      n_items, d, scores, n_ug,  \
                                                                                      split_items);              \
    else                                                                                                       \
        score_dense_kernel<DTV, KC, SG><<<(unsigned)grid, kDenseWaves * 64, 0, stream>>>(Q, user_rows, items, B, \
                                                                                         n_items, d, scores, n_ug, \
                                                                                         split_items)
#define LGX_SD(DTV, KC)                  \
    do {                                 \
        if (apply_sigmoid) {             \
            LGX_SD3(DTV, KC, true);      \
        } else {                         \
            LGX_SD3(DTV, KC, false);     \
        }                                \
    } while (0)
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
#undef LGX_SD3
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_strat_labels_fused(const void* Q, const int64_t* user_rows, const void* items, int64_t B,
                                      int64_t n_items, int64_t d, int dtype, float min16, float inter16,
                                      int num_fold, const int64_t* mask_indptr, const int32_t* mask_indices,
                                      int8_t* labels, int32_t* hist, lgx_stream_t stream_) {
    hipStream_t stream = as_hip(stream_);
    LGX_REQUIRE(B >= 0 && n_items >= 0 && n_items < INT32_MAX && (B == 0 || (Q && items && labels && hist)),
                LGX_ERR_INVALID_ARG, "lgx_strat_labels_fused: bad arguments");
    LGX_REQUIRE(dtype == LGX_DTYPE_F32 || dtype == LGX_DTYPE_BF16, LGX_ERR_INVALID_ARG,
                "lgx_strat_labels_fused: dtype");
    const int64_t vec = dtype == LGX_DTYPE_F32 ? 4 : 8;
    const int kch = kch_for(dtype, d);
    LGX_REQUIRE(d > 0 && d % vec == 0 && kch >= 8, LGX_ERR_UNSUPPORTED,
                "lgx_strat_labels_fused: d=%lld: a multiple of %lld with 5..32 MFMA chunks (use lgx_score_dense + "
                "lgx_strat_labels)", (long long)d, (long long)vec);
    StratThr thr{};
    LGX_REQUIRE(num_fold >= 1 && num_fold < 32, LGX_ERR_INVALID_ARG, "lgx_strat_labels_fused: num_fold in [1, 32)");
    int rc = lgx_strat_thresholds(min16, inter16, num_fold, thr.t);
    if (rc) return rc;
    thr.n = num_fold;
    // the estimate's grid: label j starts near thr[j-1]; evenly spaced by the mean gap
    thr.base = thr.t[0] - (num_fold > 1 && std::isfinite(thr.t[num_fold - 1])
                               ? (thr.t[num_fold - 1] - thr.t[0]) / (num_fold - 1) : inter16);
    thr.inv = num_fold > 1 && std::isfinite(thr.t[num_fold - 1]) && thr.t[num_fold - 1] > thr.t[0]
                  ? (float)(num_fold - 1) / (thr.t[num_fold - 1] - thr.t[0]) : 1.0f / inter16;
    thr.off = -(thr.base * thr.inv);  // any value serves: the host proof below runs the same FMA
    if (B == 0 || n_items == 0) return LGX_OK;
    const int64_t n_ug = ceil_div(B, (int64_t)kDenseUsers);
    const int64_t tiles = ceil_div(n_items, 32);
    const int64_t n_splits = std::max<int64_t>(8, std::min(8 * ceil_div(ceil_div(2048, n_ug), 8), 8 * ceil_div(tiles, 8)));
    const int64_t split_items = 32 * ceil_div(tiles, n_splits);
    const int64_t grid = n_ug * n_splits;
    LGX_REQUIRE(grid < (1LL << 31), LGX_ERR_UNSUPPORTED, "lgx_strat_labels_fused: %lld users is too many", (long long)B);
    const bool vec4 = n_items % 4 == 0 && ((uintptr_t)labels & 3) == 0;
    const bool est1 = strat_estimate_within_one(thr);
    // counts in the scoring kernel (num_fold + 1 <= 17 bins), else a counting pass over the labels
    const bool fuse_hist = num_fold + 1 <= kHistStride;
    if (fuse_hist) LGX_HIP_CHECK(hipMemsetAsync(hist, 0, (size_t)B * (num_fold + 1) * sizeof(int32_t), stream));
#define LGX_SL3(DTV, KC, V4)                                                                                      \
    if (est1)                                                                                                     \
        strat_label_lds<DTV, KC, V4, true><<<(unsigned)grid, kDenseWaves * 64, 0, stream>>>(                      \
            Q, user_rows, items, B, n_items, d, thr, labels, fuse_hist ? hist : nullptr, n_ug, split_items);      \
    else                                                                                                          \
        strat_label_lds<DTV, KC, V4, false><<<(unsigned)grid, kDenseWaves * 64, 0, stream>>>(                     \
            Q, user_rows, items, B, n_items, d, thr, labels, fuse_hist ? hist : nullptr, n_ug, split_items)
#define LGX_SL2(DTV, KC, V4) do { LGX_SL3(DTV, KC, V4); } while (0)
#define LGX_SL_ALL(DTV)                                                              \
    switch (kch) {                                                                   \
        case 8: if (vec4) LGX_SL2(DTV, 8, true); else LGX_SL2(DTV, 8, false); break;    \
        case 16: if (vec4) LGX_SL2(DTV, 16, true); else LGX_SL2(DTV, 16, false); break; \
        default: if (vec4) LGX_SL2(DTV, 32, true); else LGX_SL2(DTV, 32, false); break; \
    }
    if (dtype == LGX_DTYPE_F32) { LGX_SL_ALL(LGX_DTYPE_F32) } else { LGX_SL_ALL(LGX_DTYPE_BF16) }
#undef LGX_SL_ALL
#undef LGX_SL2
#undef LGX_SL3
    LGX_LAUNCH_CHECK();
    if (fuse_hist) return lgx_strat_mask(labels, B, n_items, num_fold, mask_indptr, mask_indices, hist, stream_);
    return lgx_strat_hist(labels, B, n_items, num_fold, mask_indptr, mask_indices, hist, stream_);
}
