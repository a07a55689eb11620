"""Development: build a cycle-stamped copy of liblgx.so (tools/_ab/lab/liblgx.so) for
tools/score_stats.py.  The LDS scoring walk (score_topk_lds_body) gets s_memtime stamps around its
phases and counters on its epilogue paths, summed per wave into a device array read back by
lgx_lab_stats().  The product sources are copied and patched here, never edited: the product
library has no lab switches.  Stamping costs ~10 % of wave cycles (MI355X_MICROARCH.md); the
numbers are a breakdown, not a timing.

  python tools/make_stats_lab.py        # then: python tools/score_stats.py
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAB = os.path.join(ROOT, "tools", "_ab", "lab")

# [index, name] of the per-wave sums (tools/score_stats.py reads the same list)
FIELDS = ["waves", "tiles", "cyc_loop", "cyc_stage", "cyc_epi_late", "cyc_compute", "cyc_epi_early", "cyc_wait",
          "n_fast", "n_defer", "n_full", "cyc_full", "cyc_flush", "n_event_tiles", "cyc_detect", "cyc_defer",
          "cyc_dropmasked", "cyc_drain_ins", "cyc_insert_now", "n_unbounded", "n_rescan", "n_drain_steps",
          # producer / consumer walk (PC): the producers' score writes, refill + MFMA issue, vmcnt wait and
          # barrier wait, the consumers' barrier wait (the consumers' epilogue is cyc_epi_early)
          "pc_waves", "cyc_pc_write", "cyc_pc_compute", "cyc_pc_vm", "cyc_pc_pwait", "cyc_pc_cwait"]


def patch(src: str) -> str:
    def rep(old, new, count=1):
        nonlocal src
        assert src.count(old) >= 1, old[:80]
        src = src.replace(old, new, count)

    # device sums + host accessor
    rep("namespace lgx {\nnamespace {\n", "namespace lgx {\n__device__ unsigned long long g_lab[32];\nnamespace {\n")
    # full-path split: the mask filter of the drain, the drain's insertions, the block's direct
    # insertions; rescans summed over lanes; the drain's wave-serial insertion steps
    rep("    float tau;       // filter threshold",
        "    unsigned long long lab_dm = 0, lab_dr = 0, lab_in = 0, lab_unb = 0, lab_resc = 0, lab_steps = 0;\n"
        "    float tau;       // filter threshold")
    rep("            keys[mp] = key;\n            rescan();\n", "            keys[mp] = key;\n            ++lab_resc;\n            rescan();\n")
    rep("        const uint32_t keep = drop_masked(a);\n",
        "        const unsigned long long D0 = __builtin_amdgcn_s_memtime();\n"
        "        const uint32_t keep = drop_masked(a);\n"
        "        const unsigned long long D1 = __builtin_amdgcn_s_memtime();\n        lab_dm += D1 - D0;\n"
        "        { int mx = pcnt; for (int m = 16; m > 0; m >>= 1) mx = max(mx, __shfl_xor(mx, m, 64)); lab_steps += 2 * mx; }\n")
    rep("        pcnt = 0;\n        refresh_tau();\n    }\n",
        "        pcnt = 0;\n        refresh_tau();\n        lab_dr += __builtin_amdgcn_s_memtime() - D1;\n    }\n")
    rep("                                               uint32_t cmask) {\n",
        "                                               uint32_t cmask) {\n        const unsigned long long I0 = __builtin_amdgcn_s_memtime();\n")
    rep("            sync_from(ph);\n        }\n        refresh_tau();\n    }\n\n    template <bool MINMAX>",
        "            sync_from(ph);\n        }\n        refresh_tau();\n        lab_in += __builtin_amdgcn_s_memtime() - I0;\n    }\n\n    template <bool MINMAX>")
    rep("        if (__ballot(unbounded()) == 0ull && defer()) return;\n        drain(a);",
        "        if (__ballot(unbounded()) == 0ull && defer()) return;\n"
        "        if (__ballot(unbounded()) != 0ull) ++lab_unb;\n        drain(a);")
    # per-wave accumulators at the loop
    # the producer / consumer loops (separate loops, same barrier count)
    rep("            auto iter = [&](int64_t t, f32x4 (&cur)[2][4], f32x4 (&prev)[2][4]) {\n                if (t > 0 && t <= ntiles) {\n",
        "            auto iter = [&](int64_t t, f32x4 (&cur)[2][4], f32x4 (&prev)[2][4]) {\n"
        "                const unsigned long long P0 = __builtin_amdgcn_s_memtime();\n"
        "                if (t > 0 && t <= ntiles) {\n")
    rep("                if (t < ntiles) {\n                    if (t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "                    compute_into(cur);\n                }\n",
        "                const unsigned long long P1 = __builtin_amdgcn_s_memtime();\n"
        "                if (t < ntiles) {\n                    if (t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "                    compute_into(cur);\n                }\n"
        "                const unsigned long long P2 = __builtin_amdgcn_s_memtime();\n"
        "                L_pc_write += P1 - P0; L_pc_compute += P2 - P1;\n")
    rep("                wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));\n"
        "                __syncthreads();\n                buf = buf + 1 == nbuf ? 0 : buf + 1;\n",
        "                wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));\n"
        "                const unsigned long long PB = __builtin_amdgcn_s_memtime();\n"
        "                L_pc_vm += PB - P0;\n"
        "                __syncthreads();\n"
        "                L_pc_pwait += __builtin_amdgcn_s_memtime() - PB;\n"
        "                buf = buf + 1 == nbuf ? 0 : buf + 1;\n")
    rep("                if (t + 1 < ntiles + 2) iter(t + 1, cB, cA);\n            }\n            return;\n",
        "                if (t + 1 < ntiles + 2) iter(t + 1, cB, cA);\n            }\n"
        "            if (lane == 0) {\n"
        "                atomicAdd(&g_lab[22], 1ull); atomicAdd(&g_lab[23], L_pc_write); atomicAdd(&g_lab[24], L_pc_compute);\n"
        "                atomicAdd(&g_lab[25], L_pc_vm - L_pc_write - L_pc_compute); atomicAdd(&g_lab[26], L_pc_pwait);\n"
        "            }\n            return;\n")
    rep("            if (t >= 2) {  // tile t - 2, published by the previous barrier\n",
        "            const unsigned long long C0 = __builtin_amdgcn_s_memtime();\n"
        "            if (t >= 2) {  // tile t - 2, published by the previous barrier\n")
    rep("                epilogue(tile_start(t - 2));\n            }\n            __syncthreads();\n        }\n",
        "                epilogue(tile_start(t - 2));\n                ++L_tiles;\n"
        "                L_epi_early += __builtin_amdgcn_s_memtime() - C0;\n            }\n"
        "            const unsigned long long CB = __builtin_amdgcn_s_memtime();\n"
        "            __syncthreads();\n"
        "            L_pc_cwait += __builtin_amdgcn_s_memtime() - CB;\n        }\n")
    rep("    const bool stage_after = STAGGER && !late;  // wave-uniform\n",
        "    const bool stage_after = STAGGER && !late;  // wave-uniform\n"
        "    unsigned long long L_loop0 = __builtin_amdgcn_s_memtime();\n"
        "    unsigned long long L_pc_write = 0, L_pc_compute = 0, L_pc_vm = 0, L_pc_pwait = 0, L_pc_cwait = 0;\n")
    rep("    } else\n    for (int64_t t = 0; t < ntiles; ++t) {\n"
        "        const int64_t t0 = tile_start(t);\n"
        "        if (!stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "        if (late && t > 0) epilogue(prev_t0);\n"
        "        compute();\n"
        "        if (stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "        if (!late) epilogue(t0);\n",
        "    } else\n"
        "    for (int64_t t = 0; t < ntiles; ++t) {\n"
        "        const int64_t t0 = tile_start(t);\n"
        "        const unsigned long long T0 = __builtin_amdgcn_s_memtime();\n"
        "        if (!stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "        const unsigned long long T1 = __builtin_amdgcn_s_memtime();\n"
        "        if (late && t > 0) epilogue(prev_t0);\n"
        "        const unsigned long long T2 = __builtin_amdgcn_s_memtime();\n"
        "        compute();\n"
        "        const unsigned long long T3 = __builtin_amdgcn_s_memtime();\n"
        "        if (stage_after && t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));\n"
        "        const unsigned long long T4 = __builtin_amdgcn_s_memtime();\n"
        "        if (!late) epilogue(t0);\n"
        "        const unsigned long long T5 = __builtin_amdgcn_s_memtime();\n"
        "        L_stage += (T1 - T0) + (T4 - T3); L_epi_late += T2 - T1; L_compute += T3 - T2; L_epi_early += T5 - T4;\n")
    rep("        __syncthreads();\n        buf = buf + 1 == nbuf ? 0 : buf + 1;\n",
        "        __syncthreads();\n        L_wait += __builtin_amdgcn_s_memtime() - T5;\n        ++L_tiles;\n"
        "        buf = buf + 1 == nbuf ? 0 : buf + 1;\n")
    rep("    if (late && ntiles > 0) epilogue(prev_t0);\n",
        "    if (late && ntiles > 0) epilogue(prev_t0);\n"
        "    const unsigned long long L_loop = __builtin_amdgcn_s_memtime() - L_loop0;\n")
    # declarations before the epilogue lambda
    rep("    auto epilogue = [&](int64_t e0) {\n",
        "    unsigned long long L_stage = 0, L_epi_late = 0, L_compute = 0, L_epi_early = 0, L_wait = 0, L_tiles = 0;\n"
        "    unsigned long long L_fast = 0, L_defer = 0, L_full = 0, L_cyc_full = 0, L_ev = 0, L_detect = 0, L_defer_cyc = 0;\n"
        "    auto epilogue = [&](int64_t e0) {\n")
    rep("        const bool tail = e0 + G::TILE_ITEMS > i_end;\n        if constexpr (SKIP) {\n",
        "        const bool tail = e0 + G::TILE_ITEMS > i_end;\n        const unsigned long long E0 = __builtin_amdgcn_s_memtime();\n"
        "        if constexpr (SKIP) {\n")
    rep("                if (__ballot((m0 >= tauA) | (m1 >= tauB)) == 0ull) return;  // wave-uniform fast path\n",
        "                const bool any_ev = __ballot((m0 >= tauA) | (m1 >= tauB)) != 0ull;\n"
        "                const unsigned long long E1 = __builtin_amdgcn_s_memtime();\n"
        "                L_detect += E1 - E0;\n"
        "                if (!any_ev) { ++L_fast; return; }  // wave-uniform fast path\n"
        "                ++L_ev;\n")
    rep("                    if (__ballot(n > TopK::kPend) == 0ull) {\n                        st.pcnt = n;\n"
        "                        return;\n                    }\n",
        "                    if (__ballot(n > TopK::kPend) == 0ull) {\n                        st.pcnt = n;\n"
        "                        ++L_defer;\n                        L_defer_cyc += __builtin_amdgcn_s_memtime() - E1;\n"
        "                        return;\n                    }\n")
    rep("        const float tau_before = st.tau;\n",
        "        const unsigned long long F0 = __builtin_amdgcn_s_memtime();\n        ++L_full;\n"
        "        const float tau_before = st.tau;\n")
    rep("        if (SKIP && __ballot(st.tau != tau_before) != 0ull) refresh_taus();\n    };\n",
        "        if (SKIP && __ballot(st.tau != tau_before) != 0ull) refresh_taus();\n"
        "        L_cyc_full += __builtin_amdgcn_s_memtime() - F0;\n    };\n")
    # the sums, then the flush (top-k mode only)
    rep("    st.flush(a, split, lane);\n}\n\ntemplate <int KSTEPS, bool MINMAX, int MODE = kTopK>",
        "    const unsigned long long FL0 = __builtin_amdgcn_s_memtime();\n"
        "    st.flush(a, split, lane);\n"
        "    const unsigned long long L_flush = __builtin_amdgcn_s_memtime() - FL0;\n"
        "    unsigned long long resc = st.lab_resc;\n"
        "    for (int m = 32; m > 0; m >>= 1) resc += __shfl_xor(resc, m, 64);\n"
        "    if (lane == 0) {\n"
        "        const unsigned long long v[22] = {1ull, L_tiles, L_loop, L_stage, L_epi_late, L_compute, L_epi_early,\n"
        "                                          L_wait, L_fast, L_defer, L_full, L_cyc_full, L_flush, L_ev, L_detect,\n"
        "                                          L_defer_cyc, st.lab_dm, st.lab_dr, st.lab_in, st.lab_unb, resc, st.lab_steps};\n"
        "        for (int j = 0; j < 22; ++j) atomicAdd(&g_lab[j], v[j]);\n"
        "        atomicAdd(&g_lab[27], L_pc_cwait);\n"
        "    }\n"
        "}\n\ntemplate <int KSTEPS, bool MINMAX, int MODE = kTopK>")
    src += ("\nextern \"C\" int lgx_lab_stats(unsigned long long* out, int reset) {\n"
            "    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lgx::g_lab), sizeof(lgx::g_lab)) != hipSuccess) return 1;\n"
            "    if (reset) {\n        unsigned long long z[32] = {0};\n"
            "        if (hipMemcpyToSymbol(HIP_SYMBOL(lgx::g_lab), z, sizeof(z)) != hipSuccess) return 1;\n    }\n"
            "    return 0;\n}\n")
    return src


def main():
    if os.path.isdir(LAB):
        shutil.rmtree(LAB)
    pkg = os.path.join(LAB, "factors_of_serendipity_recommendation_amd")
    shutil.copytree(os.path.join(ROOT, "factors_of_serendipity_recommendation_amd", "csrc"), os.path.join(pkg, "csrc"),
                    ignore=shutil.ignore_patterns("_build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(LAB, "include"))
    p = os.path.join(pkg, "csrc", "score_topk.hip")
    with open(p) as f:
        src = f.read()
    with open(p, "w") as f:
        f.write(patch(src))
    subprocess.check_call(["make", "-s", f"-j{min(8, os.cpu_count() or 8)}", "-C", os.path.join(pkg, "csrc")])
    print(os.path.join(pkg, "liblgx.so"))


if __name__ == "__main__":
    sys.exit(main())
