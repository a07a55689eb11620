// Development: A/B timing of score_topk_bf16_lds variants on the C5 shape (B users x 1M items,
// d=256, top-20, 50 masked items per user), launched directly (no finalize), hipEvents, best of 3.
//   make -C tools score_lab && tools/score_lab [B]
#include "../factors_of_serendipity_recommendation_amd/csrc/score_topk.hip"
#include "score_lab_ws.h"
#include "score_lab_w1.h"

#include <cstdio>
#include <random>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int ABL, int DMAPOS, bool SKIP = true, bool STAG = true>
int launch(const ScoreArgs& a, const SplitPlan& p, hipStream_t s) {
    return launch_lds_kernel<16, false, ABL, 8, 2, STAG, true, DMAPOS, SKIP>(a, p, s);
}

// the wave-specialised walk (score_topk_bf16_ws), d = 256, full sweep
template <int WSV>
int launch_ws_v(const ScoreArgs& a, const SplitPlan& p, hipStream_t s) {
    typedef LdsGeom<16, kWsMfma, 2, 2> G;
    const int nbuf = 2;
    const WsLayout L = ws_layout(a.k, (size_t)nbuf * G::TILE);
    if (L.total > kLdsBytes) { std::printf("ws: %zu B of LDS\n", L.total); return 1; }
    if (hipFuncSetAttribute((const void*)score_topk_bf16_ws<16, WSV>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.total))
        return 1;
    score_topk_bf16_ws<16, WSV><<<(unsigned)p.n_utiles, kWsWaves * 64, L.total, s>>>(a, p.n_utiles, nbuf);
    return hipGetLastError() != hipSuccess;
}
int launch_ws(const ScoreArgs& a, const SplitPlan& p, hipStream_t s) {
    const char* v = getenv("LAB_WS");
    if (v && v[0] == '1') return launch_ws_v<1>(a, p, s);
    if (v && v[0] == '2') return launch_ws_v<2>(a, p, s);
    if (v && v[0] == '3') return launch_ws_v<3>(a, p, s);
    return launch_ws_v<0>(a, p, s);
}

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 131072;
    const int64_t I = getenv("LAB_I") ? std::atoll(getenv("LAB_I")) : 1000000, d = 256, M = 50;
    const int k = 20;
    void *Q, *items, *ws;
    int32_t* mi;
    int64_t* mp;
    HK(hipMalloc(&Q, B * d * 2));
    HK(hipMalloc(&items, I * d * 2));
    if (lgx_fill_normal(Q, B * d, 1.0f / 16, 2, LGX_DTYPE_BF16, nullptr)) return 1;
    if (lgx_fill_normal(items, I * d, 1.0f / 16, 1, LGX_DTYPE_BF16, nullptr)) return 1;
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
    const SplitPlan p = plan_splits(B, I, LGX_DTYPE_BF16, d, k);
    HK(hipMalloc(&ws, (size_t)B * p.n_splits * k * 8 + (size_t)B * p.n_splits * 2 * kSuspSlots * 8 + 4096));
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    std::printf("B=%lld splits=%d utiles=%lld\n", (long long)B, p.n_splits, (long long)p.n_utiles);
    const bool dyn = false;
    auto timeit = [&](const char* name, auto fn, bool masked) -> int {
        ScoreArgs a{Q, nullptr, items, B, I, d, masked ? mp : nullptr, masked ? mi : nullptr, k, p.n_splits,
                    p.split_items, reinterpret_cast<float*>(ws),
                    reinterpret_cast<int32_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 4), nullptr,
                    getenv("LAB_NOSUSP") ? nullptr : reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 8)};
        if (fn(a, p, nullptr)) { std::printf("%s: launch failed: %s\n", name, lgx_last_error()); return 1; }
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            HK(hipEventRecord(e0, nullptr));
            fn(a, p, nullptr);
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            float ms;
            HK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        std::printf("%s%-30s masked=%d %9.2f ms %7.0f TF/s\n", dyn ? "dyn " : "    ", name, (int)masked, best, 2.0 * B * I * d / (best * 1e-3) / 1e12);
        std::fflush(stdout);
        return 0;
    };
#ifdef LGX_MASK_ABL
    std::printf("LGX_MASK_ABL=%d\n", LGX_MASK_ABL);
    if (timeit("full", launch<0, 0>, true)) return 1;
#else
    if (getenv("LAB_TAILCONC")) {  // the bench plan: staged full sweep of B users + a split tail of T users,
        // one stream after the other vs the tail on a second stream beside the stages
        const int64_t T = std::atoll(getenv("LAB_TAILCONC"));
        void *Qt, *wst;
        HK(hipMalloc(&Qt, T * d * 2));
        if (lgx_fill_normal(Qt, T * d, 1.0f / 16, 3, LGX_DTYPE_BF16, nullptr)) return 1;
        const SplitPlan pt = plan_splits(T, I, LGX_DTYPE_BF16, d, k);
        HK(hipMalloc(&wst, (size_t)T * pt.n_splits * k * 8 + 4096));
        std::vector<int64_t> cut;
        for (int64_t hi = 16384; 3 * hi < 2 * I; hi *= 2) cut.push_back(hi);
        cut.push_back(I);
        uint64_t* susp = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 8);
        float* ps = reinterpret_cast<float*>(ws);
        int32_t* pi = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + (size_t)B * k * 4);
        SplitPlan q = p;
        q.n_splits = 1;
        std::vector<ScoreArgs> st;
        for (size_t j = 0; j < cut.size(); ++j) {
            const int64_t lo = j ? cut[j - 1] : 0;
            ScoreArgs x{Q, nullptr, items, B, cut[j], d, mp, mi, k, 1, cut[j] - lo, ps, pi, nullptr, susp,
                        j ? ps : nullptr, j ? pi : nullptr, lo};
            st.push_back(x);
        }
        ScoreArgs tail{Qt, nullptr, items, T, I, d, nullptr, nullptr, k, pt.n_splits, pt.split_items,
                       reinterpret_cast<float*>(wst),
                       reinterpret_cast<int32_t*>(static_cast<char*>(wst) + (size_t)T * pt.n_splits * k * 4), nullptr,
                       nullptr};
        hipStream_t s2;
        HK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        hipEvent_t fork, join;
        HK(hipEventCreate(&fork));
        HK(hipEventCreate(&join));
        float seq = 1e30f, conc = 1e30f, tl = 1e30f;
        for (int r = 0; r < 3; ++r) {
            float ms;
            HK(hipEventRecord(e0, nullptr));
            for (auto& x : st) if (launch<0, 0>(x, q, nullptr)) return 1;
            if (launch<0, 0>(tail, pt, nullptr)) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            HK(hipEventElapsedTime(&ms, e0, e1));
            seq = std::min(seq, ms);
            HK(hipEventRecord(e0, nullptr));
            if (launch<0, 0>(tail, pt, nullptr)) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            HK(hipEventElapsedTime(&ms, e0, e1));
            tl = std::min(tl, ms);
            HK(hipEventRecord(e0, nullptr));
            HK(hipEventRecord(fork, nullptr));
            HK(hipStreamWaitEvent(s2, fork, 0));
            if (launch<0, 0>(tail, pt, s2)) return 1;
            HK(hipEventRecord(join, s2));
            for (auto& x : st) if (launch<0, 0>(x, q, nullptr)) return 1;
            HK(hipStreamWaitEvent(nullptr, join, 0));
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            HK(hipEventElapsedTime(&ms, e0, e1));
            conc = std::min(conc, ms);
        }
        std::printf("B=%lld + tail %lld (splits %d): stages then tail %.2f ms (tail alone %.2f) | tail beside the stages %.2f ms (%.1f %%)\n",
                    (long long)B, (long long)T, pt.n_splits, seq, tl, conc, 100.0 * (seq - conc) / seq);
    } else if (getenv("LAB_W1")) {  // one-wave-per-SIMD walk ceiling vs the product walk's fast path, one sweep
        SplitPlan q = p;
        q.n_splits = 1;
        ScoreArgs x{Q, nullptr, items, B, I, d, nullptr, nullptr, k, 1, I, reinterpret_cast<float*>(ws),
                    reinterpret_cast<int32_t*>(static_cast<char*>(ws) + (size_t)B * k * 4), nullptr, nullptr};
        unsigned* evd;
        HK(hipMalloc(&evd, 4));
        const int64_t ut1 = (B + kW1Waves * kW1Users - 1) / (kW1Waves * kW1Users);
        const double fl = 2.0 * B * I * d;
        for (int nb = 2; nb <= 4; ++nb) {
            const size_t shm = (size_t)nb * 64 * 512;
            HK(hipFuncSetAttribute((const void*)score_w1_ceiling<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
            float best = 1e30f;
            for (int r = 0; r < 4; ++r) {
                HK(hipMemset(evd, 0, 4));
                float ms;
                HK(hipEventRecord(e0, nullptr));
                score_w1_ceiling<16><<<(unsigned)ut1, kW1Waves * 64, shm>>>(x, ut1, nb, INFINITY, evd);
                HK(hipEventRecord(e1, nullptr));
                HK(hipEventSynchronize(e1));
                HK(hipEventElapsedTime(&ms, e0, e1));
                if (r) best = std::min(best, ms);
            }
            std::printf("w1 ceiling nbuf=%d: %.2f ms %.0f TF/s\n", nb, best, fl / (best * 1e-3) / 1e12);
            std::fflush(stdout);
        }
        float best = 1e30f;
        for (int r = 0; r < 4; ++r) {
            float ms;
            HK(hipEventRecord(e0, nullptr));
            if (launch<9, 0>(x, q, nullptr)) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            HK(hipEventElapsedTime(&ms, e0, e1));
            if (r) best = std::min(best, ms);
        }
        std::printf("product fast path only (one sweep): %.2f ms %.0f TF/s\n", best, fl / (best * 1e-3) / 1e12);
    } else if (getenv("LAB_STAGEPROF")) {  // the product's seeded stages, each timed after its predecessors ran
        // untimed (so its seed is what the chain hands it), vs the same stage with tau = +inf (fast path only)
        // LAB_CUTS: other stage boundaries (comma list; the catalog's end is appended)
        std::vector<int64_t> cut;
        if (getenv("LAB_CUTS")) {
            for (const char* c = getenv("LAB_CUTS"); *c;) {
                cut.push_back(std::atoll(c));
                while (*c && *c != ',') ++c;
                if (*c) ++c;
            }
        } else {
            for (int64_t hi = 16384; 3 * hi < 2 * I; hi *= 2) cut.push_back(hi);
        }
        cut.push_back(I);
        const bool um = getenv("LAB_UNMASKED") != nullptr;
        uint64_t* susp = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 8);
        float* ps = reinterpret_cast<float*>(ws);
        int32_t* pi = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + (size_t)B * k * 4);
        SplitPlan q = p;
        q.n_splits = 1;
        std::vector<ScoreArgs> st;
        for (size_t j = 0; j < cut.size(); ++j) {
            const int64_t lo = j ? cut[j - 1] : 0;
            ScoreArgs x{Q, nullptr, items, B, cut[j], d, um ? nullptr : mp, um ? nullptr : mi, k, 1, cut[j] - lo, ps, pi, nullptr, susp,
                        j ? ps : nullptr, j ? pi : nullptr, lo};
            st.push_back(x);
        }
        // LAB_FLOOR=S: the first stage starts from the score floors of items [0, S) (kFloorOnly walk,
        // timed with the stage and on its own)
        const int64_t S0 = getenv("LAB_FLOOR") ? std::atoll(getenv("LAB_FLOOR")) : 0;
        float* fl = nullptr;
        if (S0 > 0) {
            HK(hipMalloc(&fl, B * 4));
            st[0].floor = fl;
            st[0].floor_items = S0;
        }
        // LAB_WS: the stages run the wave-specialised walk
        const bool wsk = getenv("LAB_WS") != nullptr;
        auto main_launch = [&](const ScoreArgs& x) { return wsk ? launch_ws(x, q, nullptr) : launch<0, 0>(x, q, nullptr); };
        auto first = [&](const ScoreArgs& x) -> int {
            if (S0 > 0 && launch_lds_kernel<16, false, kFloorOnly, 8, 2, true, true, 0, true>(x, q, nullptr)) return 1;
            return main_launch(x);
        };
        if (S0 > 0) {
            float bestfl = 1e30f;
            for (int r = 0; r < 3; ++r) {
                float ms;
                HK(hipEventRecord(e0, nullptr));
                if (launch_lds_kernel<16, false, kFloorOnly, 8, 2, true, true, 0, true>(st[0], q, nullptr)) return 1;
                HK(hipEventRecord(e1, nullptr));
                HK(hipEventSynchronize(e1));
                HK(hipEventElapsedTime(&ms, e0, e1));
                bestfl = std::min(bestfl, ms);
            }
            std::printf("floor pass over [0, %lld): %.3f ms\n", (long long)S0, bestfl);
        }
        double tot = 0, totf = 0;
        for (size_t j = 0; j < st.size(); ++j) {
            float best = 1e30f, bestf = 1e30f;
            for (int r = 0; r < 3; ++r) {
                for (size_t i = 0; i < j; ++i)
                    if (i ? main_launch(st[i]) : first(st[i])) return 1;
                float ms;
                HK(hipEventRecord(e0, nullptr));
                if (j ? main_launch(st[j]) : first(st[j])) return 1;
                HK(hipEventRecord(e1, nullptr));
                HK(hipEventSynchronize(e1));
                HK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
                HK(hipEventRecord(e0, nullptr));
                if (launch<9, 0>(st[j], q, nullptr)) return 1;
                HK(hipEventRecord(e1, nullptr));
                HK(hipEventSynchronize(e1));
                HK(hipEventElapsedTime(&ms, e0, e1));
                bestf = std::min(bestf, ms);
            }
            const double fl = 2.0 * B * st[j].split_items * d;
            std::printf("stage [%7lld, %7lld) %8.3f ms %6.0f TF/s | fast path only %8.3f ms %6.0f TF/s | events +%.3f ms\n",
                        (long long)st[j].seed_items, (long long)cut[j], best, fl / (best * 1e-3) / 1e12, bestf,
                        fl / (bestf * 1e-3) / 1e12, best - bestf);
            std::fflush(stdout);
            tot += best;
            totf += bestf;
        }
        std::printf("stages%s: %.2f ms, fast path only %.2f ms (%.0f vs %.0f TF/s)\n", um ? " (unmasked)" : "", tot, totf,
                    2.0 * B * I * d / (tot * 1e-3) / 1e12, 2.0 * B * I * d / (totf * 1e-3) / 1e12);
        // the chain's lists against a plain one-sweep top-k (as sets per user)
        for (size_t i = 0; i < st.size(); ++i)
            if (i ? main_launch(st[i]) : first(st[i])) return 1;
        HK(hipDeviceSynchronize());
        const size_t lk = (size_t)B * k;
        std::vector<float> a1(lk), a2(lk);
        std::vector<int32_t> b1(lk), b2(lk);
        HK(hipMemcpy(a2.data(), ps, lk * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(b2.data(), pi, lk * 4, hipMemcpyDeviceToHost));
        ScoreArgs one{Q, nullptr, items, B, I, d, um ? nullptr : mp, um ? nullptr : mi, k, 1, I, ps, pi, nullptr, susp};
        if (launch<0, 0>(one, q, nullptr)) return 1;
        HK(hipDeviceSynchronize());
        HK(hipMemcpy(a1.data(), ps, lk * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(b1.data(), pi, lk * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t u = 0; u < B; ++u) {
            std::vector<std::pair<int32_t, float>> x, y;
            for (int j = 0; j < k; ++j) {
                x.push_back({b1[u * k + j], a1[u * k + j]});
                y.push_back({b2[u * k + j], a2[u * k + j]});
            }
            std::sort(x.begin(), x.end());
            std::sort(y.begin(), y.end());
            if (x != y) ++bad;
        }
        std::printf("staged%s%s vs one sweep: %lld of %lld users differ\n", S0 > 0 ? " (floored)" : "", wsk ? " (ws)" : "", (long long)bad, (long long)B);
    } else if (getenv("LAB_STAGES")) {  // seeded stages at the given item boundaries (comma list), vs one sweep
        std::vector<int64_t> cut;
        for (const char* c = getenv("LAB_STAGES"); *c;) {
            cut.push_back(std::atoll(c));
            while (*c && *c != ',') ++c;
            if (*c) ++c;
        }
        cut.push_back(I);
        const bool um = getenv("LAB_UNMASKED") != nullptr;
        uint64_t* susp = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 8);
        float* ps = reinterpret_cast<float*>(ws);
        int32_t* pi = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + (size_t)B * k * 4);
        SplitPlan q = p;
        q.n_splits = 1;
        std::vector<ScoreArgs> st;
        for (size_t j = 0; j < cut.size(); ++j) {
            const int64_t lo = j ? cut[j - 1] : 0;
            ScoreArgs x{Q, nullptr, items, B, cut[j], d, um ? nullptr : mp, um ? nullptr : mi, k, 1, cut[j] - lo, ps, pi, nullptr, susp,
                        j ? ps : nullptr, j ? pi : nullptr, lo};
            st.push_back(x);
        }
        ScoreArgs one{Q, nullptr, items, B, I, d, um ? nullptr : mp, um ? nullptr : mi, k, 1, I, ps, pi, nullptr, susp};
        float best1 = 1e30f, bestS = 1e30f;
        for (int r = 0; r < 3; ++r) {
            HK(hipEventRecord(e0, nullptr));
            if (launch<0, 0>(one, q, nullptr)) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            float ms;
            HK(hipEventElapsedTime(&ms, e0, e1));
            best1 = std::min(best1, ms);
            HK(hipEventRecord(e0, nullptr));
            for (auto& x : st)
                if (launch<0, 0>(x, q, nullptr)) return 1;
            HK(hipEventRecord(e1, nullptr));
            HK(hipEventSynchronize(e1));
            HK(hipEventElapsedTime(&ms, e0, e1));
            bestS = std::min(bestS, ms);
        }
        std::printf("stages %s%s: one sweep %.2f ms, %zu stages %.2f ms (%.1f %%)\n", um ? "(unmasked) " : "", getenv("LAB_STAGES"), best1,
                    st.size(), bestS, 100.0 * (best1 - bestS) / best1);
    } else if (getenv("LAB_SEED")) {  // seeded sweep: exact top-k over items [0, S) first, then [S, I)
        const int64_t S = std::atoll(getenv("LAB_SEED"));
        const int masked = getenv("LAB_UNMASKED") ? 0 : 1;
        const int64_t* mp_ = masked ? mp : nullptr;
        const int32_t* mi_ = masked ? mi : nullptr;
        const size_t lk = (size_t)B * k;
        float *sv, *fv;
        int32_t *si, *fi;
        HK(hipMalloc(&sv, lk * 4));
        HK(hipMalloc(&si, lk * 4));
        HK(hipMalloc(&fv, lk * 4));
        HK(hipMalloc(&fi, lk * 4));
        uint64_t* susp = reinterpret_cast<uint64_t*>(static_cast<char*>(ws) + (size_t)B * p.n_splits * k * 8);
        ScoreArgs full{Q, nullptr, items, B, I, d, mp_, mi_, k, 1, I, fv, fi, nullptr, susp};
        ScoreArgs pre{Q, nullptr, items, B, S, d, mp_, mi_, k, 1, S, sv, si, nullptr, susp};
        ScoreArgs main_{Q, nullptr, items, B, I, d, mp_, mi_, k, 1, I - S, reinterpret_cast<float*>(ws),
                        reinterpret_cast<int32_t*>(static_cast<char*>(ws) + lk * 4), nullptr, susp, sv, si, S};
        SplitPlan q = p;
        q.n_splits = 1;
        auto run = [&](const ScoreArgs& x) { return launch<0, 0>(x, q, nullptr); };
        float t[3] = {1e30f, 1e30f, 1e30f};
        for (int r = 0; r < 3; ++r) {
            const ScoreArgs* xs[3] = {&full, &pre, &main_};
            for (int v = 0; v < 3; ++v) {
                HK(hipEventRecord(e0, nullptr));
                if (run(*xs[v])) { std::printf("launch failed: %s\n", lgx_last_error()); return 1; }
                HK(hipEventRecord(e1, nullptr));
                HK(hipEventSynchronize(e1));
                float ms;
                HK(hipEventElapsedTime(&ms, e0, e1));
                t[v] = std::min(t[v], ms);
            }
        }
        const double fl = 2.0 * B * I * d;
        std::printf("masked=%d S=%lld: full %.2f ms (%.0f TF/s) | pre [0,S) %.2f ms | seeded [S,I) %.2f ms (%.0f TF/s over I) | pre+seeded %.2f ms\n",
                    masked, (long long)S, t[0], fl / (t[0] * 1e-3) / 1e12, t[1], t[2], fl / (t[2] * 1e-3) / 1e12, t[1] + t[2]);
        // the seeded lists must equal the one-sweep lists as (score, index) sets
        std::vector<float> a1(lk), a2(lk);
        std::vector<int32_t> b1(lk), b2(lk);
        HK(hipMemcpy(a1.data(), fv, lk * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(b1.data(), fi, lk * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(a2.data(), ws, lk * 4, hipMemcpyDeviceToHost));
        HK(hipMemcpy(b2.data(), static_cast<char*>(ws) + lk * 4, lk * 4, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t u = 0; u < B; ++u) {
            std::vector<std::pair<int32_t, float>> x, y;
            for (int j = 0; j < k; ++j) {
                x.push_back({b1[u * k + j], a1[u * k + j]});
                y.push_back({b2[u * k + j], a2[u * k + j]});
            }
            std::sort(x.begin(), x.end());
            std::sort(y.begin(), y.end());
            if (x != y) ++bad;
        }
        std::printf("seeded vs one sweep: %lld of %lld users differ\n", (long long)bad, (long long)B);
        if (getenv("LAB_SEED1")) {  // three stages: [0, S1), [S1, S), [S, I), each seeding the next
            const int64_t S1 = std::atoll(getenv("LAB_SEED1"));
            ScoreArgs s0{Q, nullptr, items, B, S1, d, mp_, mi_, k, 1, S1, main_.part_score, main_.part_idx, nullptr, susp};
            ScoreArgs s1{Q, nullptr, items, B, S, d, mp_, mi_, k, 1, S - S1, main_.part_score, main_.part_idx, nullptr, susp,
                         main_.part_score, main_.part_idx, S1};
            ScoreArgs s2 = main_;
            s2.seed_score = main_.part_score;
            s2.seed_idx = main_.part_idx;
            float u[3] = {1e30f, 1e30f, 1e30f};
            for (int r = 0; r < 3; ++r) {
                const ScoreArgs* xs[3] = {&s0, &s1, &s2};
                for (int v = 0; v < 3; ++v) {
                    HK(hipEventRecord(e0, nullptr));
                    if (run(*xs[v])) return 1;
                    HK(hipEventRecord(e1, nullptr));
                    HK(hipEventSynchronize(e1));
                    float ms;
                    HK(hipEventElapsedTime(&ms, e0, e1));
                    u[v] = std::min(u[v], ms);
                }
            }
            // the timed repetitions re-seed from lists already past [S1, I): rerun the chain once for the check
            for (int v = 0; v < 3; ++v) {
                const ScoreArgs* xs[3] = {&s0, &s1, &s2};
                if (run(*xs[v])) return 1;
            }
            HK(hipDeviceSynchronize());
            HK(hipMemcpy(a2.data(), ws, lk * 4, hipMemcpyDeviceToHost));
            HK(hipMemcpy(b2.data(), static_cast<char*>(ws) + lk * 4, lk * 4, hipMemcpyDeviceToHost));
            bad = 0;
            for (int64_t uu = 0; uu < B; ++uu) {
                std::vector<std::pair<int32_t, float>> x, y;
                for (int j = 0; j < k; ++j) {
                    x.push_back({b1[uu * k + j], a1[uu * k + j]});
                    y.push_back({b2[uu * k + j], a2[uu * k + j]});
                }
                std::sort(x.begin(), x.end());
                std::sort(y.begin(), y.end());
                if (x != y) ++bad;
            }
            std::printf("3 stages S1=%lld S=%lld: %.2f + %.2f + %.2f = %.2f ms; %lld users differ\n", (long long)S1,
                        (long long)S, u[0], u[1], u[2], u[0] + u[1] + u[2], (long long)bad);
        }
    } else if (getenv("LAB_EVT")) {  // where the top-k time goes: events dropped, slots never drained
        for (int masked = 0; masked <= 1; ++masked) {
            if (timeit("full", launch<0, 0>, masked)) return 1;
            if (timeit("fast path only (tau = +inf)", launch<9, 0>, masked)) return 1;
            if (timeit("events detected, dropped", launch<11, 0>, masked)) return 1;
            if (timeit("deferred slots, never drained", launch<12, 0>, masked)) return 1;
        }
    } else if (getenv("LAB_ABL")) {  // the MFMA / LDS-read / refill ladder (unmasked)
        if (timeit("full", launch<0, 0>, false)) return 1;
        if (timeit("no-topk", launch<1, 0>, false)) return 1;
        if (timeit("fast path only (no events)", launch<9, 0>, false)) return 1;
        if (timeit("no-topk no-refill", launch<5, 0>, false)) return 1;
        if (timeit("no-topk no-refill no-barrier", launch<7, 0>, false)) return 1;
        if (timeit("... one fragment read per tile", launch<8, 0>, false)) return 1;
    } else {
        for (int masked = 1; masked >= 0; --masked)
            if (timeit("full", launch<0, 0>, masked)) return 1;
    }
#endif
    std::printf("done\n");
    return 0;
}
