// Development: the candidate sweep of lgx_score_topk (score floors -> candidates -> per-user select)
// phase by phase, beside the product call, on the bench's scoring shape (B users x 1M items, d=256,
// top-20, 50 masked items per user); bf16 (the product path) and f32 (the same three phases through
// the f32 walk, which the product still sweeps in seeded stages).  hipEvents, median of 3.  The
// lists of the phase-by-phase run are compared with the product call's, as sets.
//   make -C tools cand_lab && tools/cand_lab [B] [bf16|f32]
#include "../factors_of_serendipity_recommendation_amd/csrc/score_topk.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
#define LK(...) do { int r_ = (__VA_ARGS__); if (r_) { std::printf("%s -> %d %s\n", #__VA_ARGS__, r_, lgx_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 262144;
    const int dt = argc > 2 && std::string(argv[2]) == "f32" ? LGX_DTYPE_F32 : LGX_DTYPE_BF16;
    const int64_t I = 1000000, d = 256, M = 50;
    const int k = 20;
    const size_t es = dt == LGX_DTYPE_F32 ? 4 : 2;
    void *Q, *items;
    HK(hipMalloc(&Q, B * d * es));
    HK(hipMalloc(&items, I * d * es));
    LK(lgx_fill_normal(Q, B * d, 1.0f / 16, 777, dt, nullptr));
    LK(lgx_fill_normal(items, I * d, 1.0f / 16, 4242, dt, nullptr));
    std::vector<int64_t> hp(B + 1);
    std::vector<int32_t> hi(B * M);
    std::mt19937_64 rng(5);
    for (int64_t b = 0; b < B; ++b) {
        hp[b] = b * M;
        for (int j = 0; j < M; ++j) hi[b * M + j] = (int32_t)(rng() % I);
        std::sort(hi.begin() + b * M, hi.begin() + (b + 1) * M);
    }
    hp[B] = B * M;
    int64_t* mp;
    int32_t* mi;
    HK(hipMalloc(&mp, (B + 1) * 8));
    HK(hipMalloc(&mi, B * M * 4));
    HK(hipMemcpy(mp, hp.data(), (B + 1) * 8, hipMemcpyHostToDevice));
    HK(hipMemcpy(mi, hi.data(), B * M * 4, hipMemcpyHostToDevice));
    size_t wsb = 0;
    LK(lgx_score_topk_workspace(B, I, k, &wsb));
    void* ws;
    HK(hipMalloc(&ws, wsb));
    int32_t *oi, *oi2;
    float *ov, *ov2;
    HK(hipMalloc(&oi, B * k * 4));
    HK(hipMalloc(&oi2, B * k * 4));
    HK(hipMalloc(&ov, B * k * 4));
    HK(hipMalloc(&ov2, B * k * 4));
    hipEvent_t e[6];
    for (auto& x : e) HK(hipEventCreate(&x));
    char plan[512];
    LK(lgx_score_topk_plan(B, I, d, dt, k, plan, sizeof(plan)));
    std::printf("B=%lld %s: %s\n", (long long)B, dt == LGX_DTYPE_F32 ? "f32" : "bf16", plan);
    const double flops = 2.0 * B * I * d, peak = dt == LGX_DTYPE_F32 ? 157.3e12 : 2.5e15;
    auto median3 = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    // the product call
    LK(lgx_score_topk(Q, nullptr, items, B, I, d, dt, mp, mi, k, -INFINITY, 0, oi, ov, nullptr, ws, wsb, nullptr));
    std::vector<float> tp;
    for (int r = 0; r < 3; ++r) {
        HK(hipEventRecord(e[0], nullptr));
        LK(lgx_score_topk(Q, nullptr, items, B, I, d, dt, mp, mi, k, -INFINITY, 0, oi, ov, nullptr, ws, wsb, nullptr));
        HK(hipEventRecord(e[1], nullptr));
        HK(hipEventSynchronize(e[1]));
        float ms;
        HK(hipEventElapsedTime(&ms, e[0], e[1]));
        tp.push_back(ms);
    }
    const float mp_ = median3(tp);
    std::printf("product call        %9.2f ms  %7.1f TF/s  frac %.3f\n", mp_, flops / mp_ / 1e9, flops / mp_ * 1e3 / peak);
    // the three phases by hand (one user range: B must be a whole number of 256-tile rounds)
    const SplitPlan p = plan_splits(B, I, dt, d, k);
    if (p.n_splits != 1) { std::printf("not a full-sweep plan\n"); return 1; }
    const int64_t users = (int64_t)p.waves * kUsersPerWave;
    if (B % (users * lds_resident())) std::printf("(B is not whole rounds: the product splits a tail)\n");
    float* floor;
    uint64_t* cand;
    int32_t* cnt;
    HK(hipMalloc(&floor, B * 4));
    HK(hipMalloc(&cand, (size_t)B * 4 * kCandCap * 8));
    HK(hipMalloc(&cnt, B * 4 * 4));
    ScoreArgs a{Q, nullptr, items, B, I, d, mp, mi, k, 1, p.split_items, nullptr, nullptr, nullptr, nullptr};
    a.floor = floor;
    a.floor_items = kFloorItems;
    a.cand = cand;
    a.cand_cnt = cnt;
    a.cand_cap = kCandCap;
    std::vector<float> t1, t2, t3;
    for (int r = 0; r < 3; ++r) {
        HK(hipEventRecord(e[0], nullptr));
        LK(launch_lds<false, kFloorOnly>(a, p, nullptr, dt));
        HK(hipEventRecord(e[1], nullptr));
        LK(launch_lds<false, kCandidates>(a, p, nullptr, dt));
        HK(hipEventRecord(e[2], nullptr));
        score_topk_cand_select<1><<<(unsigned)B, 64>>>(a, -INFINITY, 0, oi2, ov2);
        HK(hipGetLastError());
        HK(hipEventRecord(e[3], nullptr));
        HK(hipEventSynchronize(e[3]));
        float x, y, z;
        HK(hipEventElapsedTime(&x, e[0], e[1]));
        HK(hipEventElapsedTime(&y, e[1], e[2]));
        HK(hipEventElapsedTime(&z, e[2], e[3]));
        t1.push_back(x);
        t2.push_back(y);
        t3.push_back(z);
    }
    const float f = median3(t1), c = median3(t2), s = median3(t3);
    std::printf("floors %8.2f ms | candidates %8.2f ms (%7.1f TF/s over the catalog) | select %7.2f ms | "
                "total %8.2f ms  %7.1f TF/s  frac %.3f\n", f, c, flops / c / 1e9, s, f + c + s,
                flops / (f + c + s) / 1e9, flops / (f + c + s) * 1e3 / peak);
    std::vector<int32_t> hc(B * 4);
    HK(hipMemcpy(hc.data(), cnt, B * 4 * 4, hipMemcpyDeviceToHost));
    double tot = 0;
    int mx = 0;
    for (int32_t x : hc) { tot += x; mx = std::max(mx, x); }
    std::printf("candidates kept per user %.1f (regions: max %d of %d)\n", tot / B, mx, kCandCap);
    // the product's lists (its tail range included) vs the phase-by-phase lists, as sets
    std::vector<int32_t> h1(B * k), h2(B * k);
    HK(hipMemcpy(h1.data(), oi, B * k * 4, hipMemcpyDeviceToHost));
    HK(hipMemcpy(h2.data(), oi2, B * k * 4, hipMemcpyDeviceToHost));
    int64_t diff = 0;
    for (int64_t b = 0; b < B; ++b) {
        std::sort(h1.begin() + b * k, h1.begin() + (b + 1) * k);
        std::sort(h2.begin() + b * k, h2.begin() + (b + 1) * k);
        diff += !std::equal(h1.begin() + b * k, h1.begin() + (b + 1) * k, h2.begin() + b * k);
    }
    std::printf("users whose lists differ from the product call: %lld of %lld\n", (long long)diff, (long long)B);
    return 0;
}
