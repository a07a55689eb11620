// a9: row-wise top-k of a dense score matrix + a10: fold-out metric curves.
//
// Reference: c_top_k_index / c_top_k_array_index (LightGCN-tf/evaluator/cpp/include/tools.h:
// 13-33: std::partial_sort_copy per row on a host thread pool) and evaluate_foldout
// (evaluator/cpp/include/evaluate_foldout.h:16-195).
//
// Long rows: one 256-thread workgroup per row, each of its 4 waves streams an interleaved quarter
// of the row with coalesced 1-KB (float4) loads, filters against its running k-th key and merges
// survivors with the register bitonic network of wave_topk.h; the row's first wave then merges the
// other three lists.  Short rows (< 16 K columns): one wave per row, 4 rows per workgroup.
#include "wave_topk.h"

namespace lgx {
namespace {

constexpr int kUnroll = 3;  // 4 float4 per lane took 77 VGPRs (spills at the 64 of 8 waves per SIMD)

// WPR waves per row (4 for long rows, 1 for short ones: 4 rows per workgroup).  VEC: rows are
// 16-B aligned, so each lane loads float4s (1 KB per wave instruction).  Per batch of loads one
// integer compare of ord(score) against the running k-th key's score bits rules out the batch
// (exact: ties and NaNs go to the merge, which orders by the full key).
// R: list registers per lane (k <= 64 R, WaveList of wave_topk.h)
// Occupancy (tools/topk_lab.hip): a long row is 4 MB of reads for one workgroup, so the launch runs in
// rounds of resident workgroups.  At 77 VGPRs a CU held 6 of them: [4096, 1M] took 2.67 rounds
// (the last one a third full).  With 3 loads in flight per lane (56 VGPRs, 8 waves per SIMD) a CU
// holds 8: two full rounds.  A batch's survivors go through one merge (packed in LDS), not one merge
// per (load, element).  [4096, 1M] k=20: 1.195x -> 1.12x the time of the same reads with no top-k
// (profiles/r03_topk_lab*.txt).
__host__ __device__ constexpr int topk_rows_waves_per_simd(int r) { return r == 1 ? 8 : 4; }

template <int WPR, bool VEC, int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(topk_rows_waves_per_simd(R), topk_rows_waves_per_simd(R))))
void topk_rows_kernel(const float* __restrict__ S, int64_t rows, int64_t cols,
                                                        int64_t ld, int k, int32_t* __restrict__ out_idx,
                                                        float* __restrict__ out_val) {
    __shared__ uint64_t lists[4][R][kWave];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int sub = wave % WPR;                       // this wave's part of its row
    const int64_t row = (int64_t)blockIdx.x * (4 / WPR) + wave / WPR;
    if (row >= rows) return;                          // no barrier is reached by a missing row's waves
    const float* s = S + row * ld;
    WaveList<R> top;
    top.clear();
    constexpr int V = VEC ? 4 : 1;
    const int64_t stride = (int64_t)kWave * V * WPR;  // columns per wave round
    for (int64_t base = (int64_t)sub * kWave * V; base < cols; base += stride * kUnroll) {
        float v[kUnroll][V];
        const float* sb = s + base;  // wave-uniform: the loads are a scalar base + a 32-bit lane offset
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int off = u * (int)stride + lane * V;
            const int64_t c0 = base + off;
            if (VEC) {
                if (c0 + 3 < cols) {
                    const float4 q = *reinterpret_cast<const float4*>(sb + off);
                    v[u][0] = q.x; v[u][V > 1 ? 1 : 0] = q.y; v[u][V > 2 ? 2 : 0] = q.z; v[u][V > 3 ? 3 : 0] = q.w;
                } else {
#pragma unroll
                    for (int j = 0; j < V; ++j) v[u][j] = c0 + j < cols ? s[c0 + j] : 0.0f;
                }
            } else {
                v[u][0] = c0 < cols ? s[c0] : 0.0f;
            }
        }
        const uint32_t thr_hi = (uint32_t)(top.at(k - 1) >> 32);
        bool any = false;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
#pragma unroll
            for (int j = 0; j < V; ++j) any |= base + u * stride + (int64_t)lane * V + j < cols && ord_f32(v[u][j]) >= thr_hi;
        if (__ballot(any) == 0ull) continue;
        // survivors of the batch (score bits >= the k-th key's) packed into one 64-lane candidate
        // vector through this wave's LDS row, so a batch costs one merge instead of one per (u, j);
        // a batch with more than 64 survivors (a list still filling) merges per (u, j) as before
        uint64_t* pk = &lists[wave][0][0];
        int n = 0;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const int64_t c = base + u * stride + (int64_t)lane * V + j;
                const bool pass = c < cols && ord_f32(v[u][j]) >= thr_hi;
                const uint64_t m = __ballot(pass);
                const int pos = n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                if (pass && pos < kWave) pk[pos] = make_key(v[u][j], (int32_t)c);
                n += __popcll(m);
            }
        if (n <= kWave) {
            __builtin_amdgcn_wave_barrier();
            const uint64_t cand = lane < n ? pk[lane] : 0ull;
            __builtin_amdgcn_wave_barrier();
            top.push(cand, k, lane);
            continue;
        }
        // one merge instance in a rolled loop (the value picked by a select chain, so v stays in
        // registers): twelve inlined merges cost the registers of the 8-waves-per-SIMD budget
#pragma unroll 1
        for (int t = 0; t < kUnroll * V; ++t) {
            float x = v[0][0];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
#pragma unroll
                for (int j = 0; j < V; ++j) x = t == u * V + j ? v[u][j] : x;
            const int64_t c = base + (t / V) * stride + (int64_t)lane * V + t % V;
            top.push(c < cols ? make_key(x, (int32_t)c) : 0ull, k, lane);
        }
    }
    if (WPR > 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) lists[wave][r][lane] = top.t[r];
        __syncthreads();
        if (sub != 0) return;
#pragma unroll
        for (int w = 1; w < WPR; ++w)
#pragma unroll
            for (int r = 0; r < R; ++r) top.push(lists[wave + w][r][lane], k, lane);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = 64 * r + lane;
        if (e < k) {
            const uint64_t key = top.t[r];
            out_idx[row * k + e] = key ? key_index(key) : -1;
            if (out_val) out_val[row * k + e] = key ? key_score(key) : -INFINITY;
        }
    }
}

__device__ __forceinline__ bool in_list(const int32_t* t, int64_t n, int32_t x) {
    for (int64_t j = 0; j < n; ++j)
        if (t[j] == x) return true;
    return false;
}

// a user's truth list in registers when it has at most kTruthRegs items: the hit test of a rank is
// then kTruthRegs compares instead of a chain of dependent global loads (which bounded the kernel:
// ~200 loads per user at k = 20 and 10 truths)
constexpr int kTruthRegs = 16;
struct TruthRegs {
    int32_t t[kTruthRegs];
    int64_t n;
    const int32_t* g;  // the list in global memory (used when n > kTruthRegs)
    __device__ __forceinline__ void load(const int32_t* truth, int64_t tl) {
        n = tl;
        g = truth;
#pragma unroll
        for (int j = 0; j < kTruthRegs; ++j) t[j] = j < tl ? truth[j] : 0;
    }
    __device__ __forceinline__ bool has(int32_t x) const {
        if (n > kTruthRegs) return in_list(g, n, x);
        bool h = false;
#pragma unroll
        for (int j = 0; j < kTruthRegs; ++j) h |= j < n && t[j] == x;
        return h;
    }
};

// a long truth list (more than kTruthRegs items) against up to 32 ranks, in any order: the list is
// streamed once (independent loads) and each item compared with the ranks held in registers, instead
// of a scan of the list per rank.  A power-law user with 1000 test items made that scan 20 000 loads in
// one lane, and its wave the kernel's tail (batch_test at the Gowalla shape: 2.5 ms for 27 522 users).
// A long list that is sorted (evaluator.batch_test sorts its truth lists) takes hit_bits_sorted.
constexpr int kStreamRanks = 32;
__device__ __forceinline__ uint32_t hit_bits_streamed(const int32_t* rank, int k, const int32_t* truth, int64_t tl) {
    int32_t rr[kStreamRanks];
#pragma unroll
    for (int i = 0; i < kStreamRanks; ++i) rr[i] = i < k ? rank[i] : -2;  // bits past k are cleared below
    uint32_t bits = 0;
    for (int64_t j = 0; j < tl; ++j) {
        const int32_t x = truth[j];
#pragma unroll
        for (int i = 0; i < kStreamRanks; ++i) bits |= rr[i] == x ? (1u << i) : 0u;
    }
    return bits & (k >= 32 ? ~0u : ((1u << k) - 1u));
}

// the same hit bits for a long truth list that is sorted ascending: a lower-bound search per rank,
// the k searches advanced in lockstep (each level's loads issued together), ~log2(tl) round trips
// instead of tl * 32 compares (a 1 669-item list: ~11 levels against 53 000 compares in one lane)
__device__ __forceinline__ uint32_t hit_bits_sorted(const int32_t* rank, int k, const int32_t* truth, int64_t tl) {
    int32_t rr[kStreamRanks], lo[kStreamRanks], hi[kStreamRanks];
#pragma unroll
    for (int i = 0; i < kStreamRanks; ++i) {
        rr[i] = i < k ? rank[i] : 0;
        lo[i] = 0;
        hi[i] = i < k ? (int32_t)tl : 0;
    }
    bool any = true;
    while (any) {
        any = false;
        int32_t v[kStreamRanks];
#pragma unroll
        for (int i = 0; i < kStreamRanks; ++i) v[i] = lo[i] < hi[i] ? truth[(lo[i] + hi[i]) >> 1] : 0;
#pragma unroll
        for (int i = 0; i < kStreamRanks; ++i) {
            if (lo[i] < hi[i]) {
                const int32_t mid = (lo[i] + hi[i]) >> 1;
                if (v[i] < rr[i]) lo[i] = mid + 1;
                else hi[i] = mid;
                any |= lo[i] < hi[i];
            }
        }
    }
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < kStreamRanks; ++i)
        bits |= (i < k && lo[i] < (int32_t)tl && truth[lo[i]] == rr[i]) ? (1u << i) : 0u;
    return bits;
}

__device__ __forceinline__ bool is_ascending(const int32_t* t, int64_t n) {
    bool ok = true;
    for (int64_t j = 1; j < n; ++j) ok &= t[j - 1] <= t[j];
    return ok;
}

// evaluate_foldout.h:16-112 per user; float accumulators with double increments as in the C++.
// out[c * ostride + i] for curve c (precision, recall, map, ndcg, mrr) at rank i.
__device__ __forceinline__ void foldout_user(const int32_t* rank, const int32_t* truth, int64_t tl, int k,
                                             const double* __restrict__ inv_log2, float* out) {
    int hits = 0;
    float sum_pre = 0.0f, dcg = 0.0f, idcg = 0.0f;
    bool found = false;
    TruthRegs tr;
    const bool streamed = tl > kTruthRegs && k <= kStreamRanks;
    uint32_t hb = 0;
    if (streamed) hb = is_ascending(truth, tl) ? hit_bits_sorted(rank, k, truth, tl) : hit_bits_streamed(rank, k, truth, tl);
    else tr.load(truth, tl);
    for (int i = 0; i < k; ++i) {
        const bool hit = streamed ? ((hb >> i) & 1u) != 0u : tr.has(rank[i]);
        if (hit) {
            hits += 1;
            const float pre = (float)(1.0 * hits / (i + 1));
            sum_pre += pre;
            dcg = (float)((double)dcg + inv_log2[i]);
        }
        if (i < tl) idcg = (float)((double)idcg + inv_log2[i]);
        out[i] = (float)(1.0 * hits / (i + 1));
        out[k + i] = (float)(1.0 * hits / (double)tl);
        out[2 * k + i] = sum_pre / (float)tl;
        out[3 * k + i] = dcg / idcg;
        if (!found && hit) {
            found = true;
            const float rr = (float)(1.0 / (i + 1));
            for (int j = i; j < k; ++j) out[4 * k + j] = rr;
        } else if (!found) {
            out[4 * k + i] = 0.0f;
        }
    }
}

__global__ void foldout_kernel(const int32_t* __restrict__ rankings, int64_t users, int k,
                               const int64_t* __restrict__ truth_indptr,
                               const int32_t* __restrict__ truth_indices,
                               const double* __restrict__ inv_log2, float* __restrict__ results) {
    const int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (u >= users) return;
    const int64_t t0 = truth_indptr[u];
    foldout_user(rankings + u * k, truth_indices + t0, truth_indptr[u + 1] - t0, k, inv_log2,
                 results + u * 5 * (int64_t)k);
}

// k <= kFoldStagedK: the block's 64 ranking rows come in and its 64 x 5k result rows go out as
// contiguous coalesced runs through LDS (odd row strides: conflict-free per-thread rows); a thread
// per user writing its own 5k-float row directly was a strided store per element (1.77 ms for
// 1 M users at k=20).
constexpr int kFoldUsers = 64;
constexpr int kFoldStagedK = 64;

__global__ __launch_bounds__(kFoldUsers) void foldout_staged_kernel(const int32_t* __restrict__ rankings,
                                                                   int64_t users, int k,
                                                                   const int64_t* __restrict__ truth_indptr,
                                                                   const int32_t* __restrict__ truth_indices,
                                                                   const double* __restrict__ inv_log2,
                                                                   float* __restrict__ results) {
    extern __shared__ float fold_sm[];
    const int S = 5 * k + 1, RK = k | 1;
    float* oimg = fold_sm;
    int32_t* rimg = reinterpret_cast<int32_t*>(fold_sm + kFoldUsers * S);
    const int64_t u0 = blockIdx.x * (int64_t)kFoldUsers;
    const int nu = (int)min((int64_t)kFoldUsers, users - u0);
    const int t = threadIdx.x;
    for (int i = t; i < nu * k; i += kFoldUsers) rimg[(i / k) * RK + i % k] = rankings[u0 * k + i];
    __syncthreads();
    if (t < nu) {
        const int64_t a = truth_indptr[u0 + t];
        foldout_user(rimg + t * RK, truth_indices + a, truth_indptr[u0 + t + 1] - a, k, inv_log2, oimg + t * S);
    }
    __syncthreads();
    const int W = 5 * k;
    for (int i = t; i < nu * W; i += kFoldUsers) results[u0 * W + i] = oimg[(i / W) * S + i % W];
}

// np.mean(a, axis=0) of a C-contiguous float32 [rows, cols] array, as numpy computes it: per column a
// float32 sum over the rows in row order (numpy's axis-0 add.reduce adds whole rows, no pairwise
// blocking), then one float32 division by the row count.  The order makes each column one chain of
// dependent adds; what must not sit on that chain is the load latency.  A workgroup owns
// kMeanCols = 16 columns, so that a [rows, 100] array (batch_test's 5 x 20 curves) spreads its loads
// over 7 CUs: with 64 columns per workgroup two CUs each pulled ~25 GB/s and the kernel took 10 ns
// per row (0.55 ms at 52 643 rows).  Its 512 threads stage blocks of kMeanRows rows into LDS (one
// block ahead in registers while the current one is summed), and lanes 0-15 of wave 0 add them,
// lane = column, row by row, 64 rows per LDS round trip with the next 64 in flight (the image is
// column-major, each column's rows 16-B aligned and 4 banks from the next column's).
constexpr int kMeanRows = 256;
constexpr int kMeanWaves = 8;
constexpr int kMeanCols = 16;
constexpr int kMeanPad = kMeanRows + 4;
__global__ __launch_bounds__(kMeanWaves * 64) void column_mean_kernel(const float* __restrict__ src, int64_t rows,
                                                                     int64_t cols, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float blk[2][kMeanCols][kMeanPad];
    constexpr int kRowsPerPass = kMeanWaves * 64 / kMeanCols;  // 32 rows per load instruction of the workgroup
    constexpr int J = kMeanRows / kRowsPerPass;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int cl = t % kMeanCols, rr = t / kMeanCols;  // staging: column cl of rows rr + 32 j
    const int64_t c0 = (int64_t)blockIdx.x * kMeanCols;
    const int64_t lcol = c0 + cl;
    float nxa[J], nxb[J];
    auto load = [&](float (&nx)[J], int64_t r0) {
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int64_t r = r0 + kRowsPerPass * j + rr;
            nx[j] = (r < rows && lcol < cols) ? src[r * cols + lcol] : 0.0f;
        }
    };
    auto store = [&](const float (&nx)[J], int b) {
#pragma unroll
        for (int j = 0; j < J; ++j) blk[b][cl][kRowsPerPass * j + rr] = nx[j];
    };
    float acc = -0.0f;  // -0 + x == x for every x: the same sums as numpy's, which starts from row 0
    auto sum = [&](int b, int64_t r0) {
        if (w != 0) return;
        const int n = (int)min((int64_t)kMeanRows, rows - r0);
        const float* cp = &blk[b][lane % kMeanCols][0];
        if (n == kMeanRows) {
            float4 v[2][16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[0][q] = *reinterpret_cast<const float4*>(cp + 4 * q);
#pragma unroll
            for (int r = 0; r < kMeanRows; r += 64) {
                const int cur = (r / 64) & 1;
                if (r + 64 < kMeanRows) {
#pragma unroll
                    for (int q = 0; q < 16; ++q) v[cur ^ 1][q] = *reinterpret_cast<const float4*>(cp + r + 64 + 4 * q);
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) {  // row order
                    acc = acc + v[cur][q].x;
                    acc = acc + v[cur][q].y;
                    acc = acc + v[cur][q].z;
                    acc = acc + v[cur][q].w;
                }
            }
        } else {
            for (int r = 0; r < n; ++r) acc = acc + cp[r];
        }
    };
    // block r0 is in LDS buffer b, block r0 + R in registers `next`; block r0 + 2R goes into `into`
    auto step = [&](int64_t r0, int b, const float (&next)[J], float (&into)[J]) {
        if (r0 + 2 * kMeanRows < rows) load(into, r0 + 2 * kMeanRows);
        sum(b, r0);
        if (r0 + kMeanRows < rows) store(next, b ^ 1);  // buffer b ^ 1 was last read before the previous barrier
        __syncthreads();
    };
    load(nxa, 0);
    store(nxa, 0);
    if (kMeanRows < rows) load(nxb, kMeanRows);
    __syncthreads();
    for (int64_t r0 = 0; r0 < rows; r0 += 2 * kMeanRows) {
        step(r0, 0, nxb, nxa);
        if (r0 + kMeanRows < rows) step(r0 + kMeanRows, 1, nxa, nxb);
    }
    const int64_t col = c0 + lane;
    if (w == 0 && lane < kMeanCols && col < cols) out[col] = rows > 0 ? acc / (float)rows : NAN;
}

// Procedure.Test's metrics (Procedure.py:60-72 -> utils.getLabel, RecallPrecision_ATk, NDCGatK_r,
// code/utils.py:218-285) for every test user at once: one thread per user marks which of its top-k
// items are test items (binary search in its sorted, deduplicated test list; the list's own length,
// duplicates included, is test_len), forms the per-user terms of each
// topk in float64 -- right / |test|, right, dcg / idcg with idcg over min(k, |test|) ranks and the
// reference's idcg == 0 -> 1, NaN -> 0 -- and the workgroup adds them in a fixed order; a second
// launch adds the workgroups' partial sums in workgroup order.  Deterministic; the reference adds
// the same terms batch by batch, so the sums agree to float64 rounding.
constexpr int kTmUsers = 256;
constexpr int kTmMaxTopks = 8;
__global__ __launch_bounds__(kTmUsers) void test_metrics_kernel(const int32_t* __restrict__ rankings, int64_t users,
                                                                int k, const int64_t* __restrict__ truth_indptr,
                                                                const int32_t* __restrict__ truth_indices,
                                                                const int64_t* __restrict__ test_len,
                                                                const int32_t* __restrict__ topks, int n_topks,
                                                                const double* __restrict__ inv_log2,
                                                                double* __restrict__ partial) {
    __shared__ double red[kTmUsers];
    const int t = threadIdx.x;
    const int64_t u = blockIdx.x * (int64_t)kTmUsers + t;
    double term[3 * kTmMaxTopks];
#pragma unroll
    for (int i = 0; i < 3 * kTmMaxTopks; ++i) term[i] = 0.0;
    if (u < users) {
        const int64_t a = truth_indptr[u], L = truth_indptr[u + 1] - a;
        const int64_t n_test = test_len ? test_len[u] : L;  // len(test list), duplicates included
        const int32_t* tl = truth_indices + a;
        const int32_t* rk = rankings + u * k;
        int right = 0, tp = 0;
        double dcg = 0.0, idcg = 0.0;
        for (int j = 0; j < k; ++j) {
            const int32_t x = rk[j];
            int64_t lo = 0, hi = L;  // first position with tl[pos] >= x
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (tl[mid] < x) lo = mid + 1;
                else hi = mid;
            }
            const bool hit = x >= 0 && lo < L && tl[lo] == x;
            right += hit ? 1 : 0;
            dcg += hit ? inv_log2[j] : 0.0;  // r * (1 / log2(j + 2)), summed over j in rank order
            if (j < n_test) idcg += inv_log2[j];
            while (tp < n_topks && topks[tp] == j + 1) {
                const double id = idcg == 0.0 ? 1.0 : idcg;
                const double nd = dcg / id;
                term[3 * tp + 0] = (double)right / (double)n_test;  // recall: right / len(test) (NaN as numpy at 0)
                term[3 * tp + 1] = (double)right;               // precision: summed, then / k on the host
                term[3 * tp + 2] = nd != nd ? 0.0 : nd;
                ++tp;
            }
        }
    }
    for (int i = 0; i < 3 * n_topks; ++i) {
        red[t] = term[i];
        __syncthreads();
        for (int s = kTmUsers / 2; s > 0; s >>= 1) {
            if (t < s) red[t] += red[t + s];
            __syncthreads();
        }
        if (t == 0) partial[blockIdx.x * (int64_t)(3 * n_topks) + i] = red[0];
        __syncthreads();
    }
}

__global__ void test_metrics_sum_kernel(const double* __restrict__ partial, int64_t blocks, int n, double* __restrict__ out) {
    const int i = threadIdx.x;
    if (i >= n) return;
    double acc = 0.0;
    for (int64_t b = 0; b < blocks; ++b) acc += partial[b * n + i];
    out[i] = acc;
}

template <int R>
int launch_topk_rows(const float* S, int64_t rows, int64_t cols, int64_t ld, int k, int32_t* out_idx,
                     float* out_val, bool vec, hipStream_t st) {
    if (cols >= 16384) {
        if (vec) topk_rows_kernel<4, true, R><<<(unsigned)rows, 256, 0, st>>>(S, rows, cols, ld, k, out_idx, out_val);
        else topk_rows_kernel<4, false, R><<<(unsigned)rows, 256, 0, st>>>(S, rows, cols, ld, k, out_idx, out_val);
    } else {
        const unsigned grid = (unsigned)ceil_div(rows, 4);
        if (vec) topk_rows_kernel<1, true, R><<<grid, 256, 0, st>>>(S, rows, cols, ld, k, out_idx, out_val);
        else topk_rows_kernel<1, false, R><<<grid, 256, 0, st>>>(S, rows, cols, ld, k, out_idx, out_val);
    }
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

}  // namespace
}  // namespace lgx

using namespace lgx;

extern "C" int lgx_topk_rows(const float* S, int64_t rows, int64_t cols, int64_t ld, int k,
                             int32_t* out_idx, float* out_val, lgx_stream_t stream) {
    LGX_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols && out_idx && (rows == 0 || S), LGX_ERR_INVALID_ARG,
                "lgx_topk_rows: bad arguments");
    LGX_REQUIRE(k >= 1 && k <= kMaxTopK, LGX_ERR_UNSUPPORTED, "lgx_topk_rows: k=%d outside [1, %d]", k, kMaxTopK);
    if (rows == 0) return LGX_OK;
    const bool vec = ld % 4 == 0 && ((uintptr_t)S & 15) == 0;
    hipStream_t st = as_hip(stream);
    if (k <= 64) return launch_topk_rows<1>(S, rows, cols, ld, k, out_idx, out_val, vec, st);
    if (k <= 128) return launch_topk_rows<2>(S, rows, cols, ld, k, out_idx, out_val, vec, st);
    return launch_topk_rows<4>(S, rows, cols, ld, k, out_idx, out_val, vec, st);
}

extern "C" int lgx_foldout_metrics(const int32_t* rankings, int64_t users, int k,
                                   const int64_t* truth_indptr, const int32_t* truth_indices,
                                   const double* inv_log2, float* results, lgx_stream_t stream) {
    LGX_REQUIRE(users >= 0 && k >= 1, LGX_ERR_INVALID_ARG, "lgx_foldout_metrics: bad sizes");
    if (users == 0) return LGX_OK;
    LGX_REQUIRE(rankings && truth_indptr && inv_log2 && results, LGX_ERR_INVALID_ARG,
                "lgx_foldout_metrics: null pointer");
    if (k <= kFoldStagedK) {
        const size_t lds = (size_t)kFoldUsers * ((5 * k + 1) * sizeof(float) + (k | 1) * sizeof(int32_t));
        foldout_staged_kernel<<<(unsigned)ceil_div(users, (int64_t)kFoldUsers), kFoldUsers, lds, as_hip(stream)>>>(
            rankings, users, k, truth_indptr, truth_indices, inv_log2, results);
    } else {
        foldout_kernel<<<ceil_div(users, 128), 128, 0, as_hip(stream)>>>(rankings, users, k, truth_indptr,
                                                                          truth_indices, inv_log2, results);
    }
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_column_mean_f32(const float* src, int64_t rows, int64_t cols, float* out, lgx_stream_t stream) {
    LGX_REQUIRE(rows >= 0 && cols >= 0 && (cols == 0 || out) && (rows == 0 || cols == 0 || src), LGX_ERR_INVALID_ARG,
                "lgx_column_mean_f32: bad arguments");
    LGX_REQUIRE(rows < (1LL << 24), LGX_ERR_UNSUPPORTED,
                "lgx_column_mean_f32: %lld rows (the float32 row count is exact below 2^24)", (long long)rows);
    if (cols == 0) return LGX_OK;
    column_mean_kernel<<<(unsigned)ceil_div(cols, (int64_t)kMeanCols), kMeanWaves * 64, 0, as_hip(stream)>>>(src, rows, cols, out);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}

extern "C" int lgx_test_metrics_workspace(int64_t users, int n_topks, size_t* bytes) {
    LGX_REQUIRE(users >= 0 && n_topks >= 1 && n_topks <= kTmMaxTopks && bytes, LGX_ERR_INVALID_ARG,
                "lgx_test_metrics_workspace: bad arguments");
    *bytes = (size_t)std::max<int64_t>(1, ceil_div(users, (int64_t)kTmUsers)) * 3 * n_topks * sizeof(double);
    return LGX_OK;
}

extern "C" int lgx_test_metrics(const int32_t* rankings, int64_t users, int k, const int64_t* truth_indptr,
                                const int32_t* truth_indices, const int64_t* test_len, const int32_t* topks, int n_topks,
                                const double* inv_log2, double* sums, void* ws, size_t ws_bytes,
                                lgx_stream_t stream) {
    LGX_REQUIRE(users >= 0 && k >= 1 && n_topks >= 1 && n_topks <= kTmMaxTopks, LGX_ERR_INVALID_ARG,
                "lgx_test_metrics: bad sizes (1 <= n_topks <= %d)", kTmMaxTopks);
    LGX_REQUIRE(sums && topks && inv_log2 && (users == 0 || (rankings && truth_indptr)), LGX_ERR_INVALID_ARG,
                "lgx_test_metrics: null pointer");
    size_t need = 0;
    lgx_test_metrics_workspace(users, n_topks, &need);
    LGX_REQUIRE(ws && ws_bytes >= need, LGX_ERR_WORKSPACE, "lgx_test_metrics: workspace %zu < %zu bytes", ws_bytes, need);
    const int64_t blocks = std::max<int64_t>(1, ceil_div(users, (int64_t)kTmUsers));
    double* partial = static_cast<double*>(ws);
    test_metrics_kernel<<<(unsigned)blocks, kTmUsers, 0, as_hip(stream)>>>(rankings, users, k, truth_indptr, truth_indices,
                                                                         test_len, topks, n_topks, inv_log2, partial);
    LGX_LAUNCH_CHECK();
    test_metrics_sum_kernel<<<1, 64, 0, as_hip(stream)>>>(partial, blocks, 3 * n_topks, sums);
    LGX_LAUNCH_CHECK();
    return LGX_OK;
}
