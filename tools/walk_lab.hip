// Development: the fp32 dense walk (score_walk_f32_lds) beside the register-staged kernels it
// replaced (score_dense_lds / strat_label_lds), on f4's batch shape (4096 users x 1M items) and the
// a6 fp32 shape; labels with and without the fused counts.  hipEvents, median of 5.
//   make -C tools walk_lab && tools/walk_lab [d] [B]
#include "../factors_of_serendipity_recommendation_amd/csrc/score_topk.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define LK(...) do { int r_ = (__VA_ARGS__); if (r_) { std::printf("%s -> %d %s\n", #__VA_ARGS__, r_, lgx_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const int64_t d = argc > 1 ? std::atoll(argv[1]) : 64;
    const int64_t B = argc > 2 ? std::atoll(argv[2]) : 4096;
    const int64_t I = 1000000;
    void *Q, *items;
    HK(hipMalloc(&Q, B * d * 4));
    HK(hipMalloc(&items, I * d * 4));
    LK(lgx_fill_normal(Q, B * d, 1.0f / 8, 777, LGX_DTYPE_F32, nullptr));
    LK(lgx_fill_normal(items, I * d, 1.0f / 8, 4242, LGX_DTYPE_F32, nullptr));
    float* scores;
    int8_t* labels;
    int32_t* hist;
    HK(hipMalloc(&scores, B * I * 4));
    HK(hipMalloc(&labels, B * I));
    HK(hipMalloc(&hist, B * 32 * 4));
    StratThr thr{};
    const int nf = 10;
    LK(lgx_strat_thresholds(-2.0f, 0.4f, nf, thr.t));
    thr.n = nf;
    thr.base = thr.t[0] - (thr.t[nf - 1] - thr.t[0]) / (nf - 1);
    thr.inv = (float)(nf - 1) / (thr.t[nf - 1] - thr.t[0]);
    const bool est1 = strat_estimate_within_one(thr);
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    const double flops = 2.0 * B * I * d;
    auto timeit = [&](const char* name, const std::function<int()>& f) -> int {
        if (f()) return 1;
        std::vector<float> t;
        for (int r = 0; r < 5; ++r) {
            HK(hipEventRecord(e0, nullptr));
            if (f()) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            float ms;
            HK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        std::printf("%-44s %8.3f ms  %6.1f TF/s  frac %.3f\n", name, t[2], flops / t[2] / 1e9, flops / t[2] * 1e3 / 157.3e12);
        return 0;
    };
    std::printf("B=%lld I=%lld d=%lld f32 (est1=%d)\n", (long long)B, (long long)I, (long long)d, (int)est1);
    auto walk = [&](int mode, bool h) -> int {
        WalkOut o{};
        o.scores = scores;
        o.labels = labels;
        o.hist = h ? hist : nullptr;
        o.thr = thr;
        o.vec4 = 1;
        o.est1 = est1 ? 1 : 0;
        int rc = mode == kStratLabels ? launch_f32_walk<kStratLabels>(Q, nullptr, items, B, I, d, o, nullptr)
               : mode == kDenseSigmoid ? launch_f32_walk<kDenseSigmoid>(Q, nullptr, items, B, I, d, o, nullptr)
                                       : launch_f32_walk<kDenseScores>(Q, nullptr, items, B, I, d, o, nullptr);
        if (rc) std::printf("walk -> %d %s\n", rc, lgx_last_error());
        return rc;
    };
    if (timeit("walk labels + counts", [&] { return walk(kStratLabels, true); })) return 1;
    if (timeit("walk labels", [&] { return walk(kStratLabels, false); })) return 1;
    if (timeit("walk dense", [&] { return walk(kDenseScores, false); })) return 1;
    if (timeit("walk dense sigmoid", [&] { return walk(kDenseSigmoid, false); })) return 1;
    // the register-staged kernels (32x32x2), launched as the product launched them in round 3
    const int64_t n_ug = ceil_div(B, (int64_t)kDenseUsers);
    const int64_t tiles = ceil_div(I, 32);
    const int64_t n_splits = std::max<int64_t>(8, std::min(8 * ceil_div(ceil_div(2048, n_ug), 8), 8 * ceil_div(tiles, 8)));
    const int64_t split_items = 32 * ceil_div(tiles, n_splits);
    const unsigned grid = (unsigned)(n_ug * n_splits);
    const int kch = kch_for(LGX_DTYPE_F32, d);
    auto old_labels = [&]() -> int {
#define WL(KC) if (est1) strat_label_lds<LGX_DTYPE_F32, KC, true, true><<<grid, kDenseWaves * 64>>>(Q, nullptr, items, B, I, d, thr, labels, hist, n_ug, split_items); \
               else strat_label_lds<LGX_DTYPE_F32, KC, true, false><<<grid, kDenseWaves * 64>>>(Q, nullptr, items, B, I, d, thr, labels, hist, n_ug, split_items)
        if (kch == 8) { WL(8); } else if (kch == 16) { WL(16); } else { WL(32); }
#undef WL
        return (int)hipGetLastError();
    };
    auto old_dense = [&]() -> int {
        if (kch == 8) score_dense_lds<LGX_DTYPE_F32, 8, false><<<grid, kDenseWaves * 64>>>(Q, nullptr, items, B, I, d, scores, n_ug, split_items);
        else if (kch == 16) score_dense_lds<LGX_DTYPE_F32, 16, false><<<grid, kDenseWaves * 64>>>(Q, nullptr, items, B, I, d, scores, n_ug, split_items);
        else score_dense_lds<LGX_DTYPE_F32, 32, false><<<grid, kDenseWaves * 64>>>(Q, nullptr, items, B, I, d, scores, n_ug, split_items);
        return (int)hipGetLastError();
    };
    if (timeit("strat_label_lds labels + counts", old_labels)) return 1;
    if (timeit("score_dense_lds", old_dense)) return 1;
    return 0;
}
