// Development: per-wave statistics of the bf16 LDS scoring kernel on the C5 shape (B users x 1M
// items, d=256, top-20, 50 masked items per user).  Builds the kernel source with
// LGX_SCORE_STATS (counters + s_memtime stamps, never in liblgx.so) and prints per-wave means.
//   make -C tools score_stats && tools/score_stats [B] [masked 0|1]
#define LGX_SCORE_STATS 1
#include "../factors_of_serendipity_recommendation_amd/csrc/score_topk.hip"

#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { int rc_ = (x); if (rc_) { std::printf("%s -> %d: %s\n", #x, rc_, lgx_last_error()); return 1; } } while (0)
#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 131072;
    const bool masked = argc > 2 ? std::atoi(argv[2]) != 0 : true;
    const int64_t I = 1000000, d = 256, M = 50;
    const int k = 20;
    void *Q, *items, *ws;
    int32_t *oi, *mi;
    int64_t* mp;
    float* ov;
    HK(hipMalloc(&Q, B * d * 2));
    HK(hipMalloc(&items, I * d * 2));
    HK(hipMalloc(&oi, B * k * 4));
    HK(hipMalloc(&ov, B * k * 4));
    CK(lgx_fill_normal(Q, B * d, 1.0f / 16, 2, LGX_DTYPE_BF16, nullptr));
    CK(lgx_fill_normal(items, I * d, 1.0f / 16, 1, LGX_DTYPE_BF16, nullptr));
    std::vector<int64_t> hp(B + 1);
    std::vector<int32_t> hi(B * M);
    std::mt19937_64 rng(5);
    for (int64_t b = 0; b < B; ++b) {
        hp[b] = b * M;
        for (int j = 0; j < M; ++j) hi[b * M + j] = (int32_t)(rng() % I);
        std::sort(hi.begin() + b * M, hi.begin() + (b + 1) * M);
    }
    hp[B] = B * M;
    HK(hipMalloc(&mp, (B + 1) * 8));
    HK(hipMalloc(&mi, B * M * 4));
    HK(hipMemcpy(mp, hp.data(), (B + 1) * 8, hipMemcpyHostToDevice));
    HK(hipMemcpy(mi, hi.data(), B * M * 4, hipMemcpyHostToDevice));
    size_t wsb = 0;
    CK(lgx_score_topk_workspace(B, I, k, &wsb));
    HK(hipMalloc(&ws, wsb));
    auto run = [&]() {
        return lgx_score_topk(Q, nullptr, items, B, I, d, LGX_DTYPE_BF16, masked ? mp : nullptr, masked ? mi : nullptr,
                              k, -1e30f, 0, oi, ov, nullptr, ws, wsb, nullptr);
    };
    CK(run());
    HK(hipDeviceSynchronize());
    unsigned long long zero[24] = {0};
    HK(hipMemcpyToSymbol(HIP_SYMBOL(lgx::g_score_stats), zero, sizeof(zero)));
    const auto t0 = std::chrono::steady_clock::now();
    CK(run());
    HK(hipDeviceSynchronize());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    unsigned long long st[24];
    HK(hipMemcpyFromSymbol(st, HIP_SYMBOL(lgx::g_score_stats), sizeof(st)));
    const double waves = (double)((B + 255) / 256) * 8;
    std::printf("B=%lld masked=%d: %.1f ms (%.0f TF/s, stats build)\n", (long long)B, (int)masked, ms,
                2.0 * B * I * d / (ms * 1e-3) / 1e12);
    const char* names[25] = {"tiles", "events", "drains", "cyc epi t<1024", "cyc topk", "cyc stage+mfma", "cyc wait+bar t>=1024", "cyc events", "mask tests", "exact searches", "cyc searches", "cyc epi t>=1024", "cyc wait+bar t<1024", "tiles t<1024", "tiles t>=1024", "cyc exact path", "exact path entries", "exact (lists filling)", "insert_now iters (lane 0)", "rescans (lane 0)", "cyc rescans", "cyc drains", "-", "-"};
    for (int i = 0; i < 22; ++i) std::printf("  per wave %-18s %14.1f\n", names[i], st[i] / waves);
    std::printf("  per tile: topk %.0f  stage+mfma %.0f  wait+barrier %.0f cycles (s_memtime units)\n",
                (double)st[4] / st[0], (double)st[5] / st[0], (double)st[6] / st[0]);
    return 0;
}
