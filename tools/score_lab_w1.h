// Development only (tools/score_lab LAB_W1=1): the ceiling of a one-wave-per-SIMD bf16 walk.  4 waves x
// 64 users (4 user blocks of 16 as the MFMA B operand, 128 VGPRs of user rows), the LDS-DMA ring of
// 64-item tiles as score_topk_bf16_lds, 128 v_mfma_f32_16x16x32_bf16 per tile and wave, and the
// fast-path test of tile t-1 (per-user maxima against tau) issued between tile t's MFMAs from a second
// accumulator set.  Events are counted, not processed (tau fixed), so the lists are not produced:
// timing only, against the product walk's fast path (ABLATE 9).  Included by score_lab.hip after
// csrc/score_topk.hip.
#pragma once

namespace lgx {
namespace {

constexpr int kW1Waves = 4, kW1Users = 64;

template <int KSTEPS>
__global__ __launch_bounds__(kW1Waves * 64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void score_w1_ceiling(ScoreArgs a, int64_t n_utiles, int nbuf, float tau_all, unsigned* events) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    typedef LdsGeom<KSTEPS, 8, 2, 2> G;  // 64-item tiles of d = 16 KSTEPS bf16 (USERS unused)
    typedef Frag<LGX_DTYPE_BF16> F;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int NS = G::CPR / 4;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r16 = lane & 15, q4 = lane >> 4;
    const int64_t utile = blockIdx.x;
    if (utile >= n_utiles) return;
    unsigned char* tiles = smem;
    const uint32_t lds_tiles = lds_u32(tiles);
    uint4 uf[4 * NS];
#pragma unroll
    for (int ub = 0; ub < 4; ++ub) {
        const int64_t bu = utile * (kW1Waves * kW1Users) + w * kW1Users + 16 * ub + r16;
        const bool ok = bu < a.B;
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2)
            uf[ub * NS + s2] = __builtin_bit_cast(uint4, F::load(a.Q, ok ? bu : 0, a.d, 2 * s2 + (q4 >> 1), q4 & 1, ok));
    }
#pragma unroll
    for (int c = 0; c < 4 * NS; ++c) {
        u32x4 t = __builtin_bit_cast(u32x4, uf[c]);
        asm volatile("" : "+v"(t));
        uf[c] = __builtin_bit_cast(uint4, t);
    }
    const int64_t i_begin = a.seed_items, i_end = min(a.n_items, i_begin + a.split_items);
    const int64_t ntiles = i_end > i_begin ? (i_end - i_begin + 63) / 64 : 0;
    const int64_t rot = ((int64_t)blockIdx.x % 8) * (ntiles / 8);
    const unsigned char* items = static_cast<const unsigned char*>(a.items);
    auto tile_start = [&](int64_t t) {
        int64_t u = t + rot;
        if (u >= ntiles) u -= ntiles;
        return i_begin + u * 64;
    };
    constexpr int PPW = G::PIECES / kW1Waves;
    auto stage = [&](int buf, int64_t t0) {
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
            const uint64_t bu = reinterpret_cast<uint64_t>(items + t0 * G::RB);
            const unsigned char* base = reinterpret_cast<const unsigned char*>(
                ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32)) << 32) |
                (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bu));
            const bool tl = t0 + 64 > i_end;
            const int last = (int)(i_end - 1 - t0);
            const int q = (w * PPW + p) * 64 + lane;
            const int row = q / G::CPR;
            const int src = (q % G::CPR) ^ (row & G::SWZ);
            const int srow = tl && row > last ? last : row;
            lds_dma16(base, (uint32_t)(srow * G::RB + src * 16),
                      __builtin_amdgcn_readfirstlane(lds_tiles + buf * G::TILE + (w * PPW + p) * 1024));
        }
    };
    const int ahead = nbuf - 1;
    for (int j = 0; j < ahead && j < ntiles; ++j) stage(j, tile_start(j));
    wait_vmcnt_le(PPW * (int)max<int64_t>(0, min<int64_t>(ahead, ntiles) - 1));
    __syncthreads();
    f32x4 c[2][4][4];  // [set][ub][ib]
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int ub = 0; ub < 4; ++ub)
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) c[s][ub][ib] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    unsigned ev = 0;
    int buf = 0, sbuf = ahead;
    // one tile: MFMAs into set S, the fast-path test of set S ^ 1 (the previous tile) between them
    auto step = [&](auto Sc) __attribute__((always_inline)) {
        constexpr int S = decltype(Sc)::value;
        const unsigned char* T = tiles + buf * G::TILE;
        const unsigned char* rowp = T + r16 * G::RB;
        auto frag = [&](int s2, int ib) __attribute__((always_inline)) {
            return *reinterpret_cast<const uint4*>(rowp + ib * 16 * G::RB + (((4 * s2 + q4) ^ (r16 & G::SWZ)) * 16));
        };
        float m[4];
#pragma unroll
        for (int ub = 0; ub < 4; ++ub) {
            m[ub] = c[S ^ 1][ub][0][0];
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) c[S][ub][ib] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        }
        uint4 fa[4];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) fa[ib] = frag(0, ib);
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
#pragma unroll
                for (int ub = 0; ub < 4; ++ub) {
                    c[S][ub][ib] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fa[ib]), __builtin_bit_cast(bf16x8, uf[ub * NS + s2]), c[S][ub][ib], 0, 0, 0);
                    // previous tile's maxima: one max per MFMA, spread over the first 16 MFMAs x 4 = 64 values
                    if (s2 < 4) {
                        const int g = s2 * 16 + ib * 4 + ub;  // 0..63 -> (ub', ib', r')
                        const int ub2 = g >> 4, ib2 = (g >> 2) & 3, r2 = g & 3;
                        m[ub2] = fmaxf(m[ub2], c[S ^ 1][ub2][ib2][r2]);
                    }
                }
                if (s2 + 1 < NS) fa[ib] = frag(s2 + 1, ib);
            }
        }
        const bool hit = (m[0] >= tau_all) | (m[1] >= tau_all) | (m[2] >= tau_all) | (m[3] >= tau_all);
        if (__ballot(hit) != 0ull) ++ev;
    };
    for (int64_t t = 0; t < ntiles; ++t) {
        if (t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));
        if (t & 1) step(std::integral_constant<int, 1>());
        else step(std::integral_constant<int, 0>());
        wait_vmcnt_le(PPW * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));
        __syncthreads();
        buf = buf + 1 == nbuf ? 0 : buf + 1;
        sbuf = sbuf + 1 == nbuf ? 0 : sbuf + 1;
    }
    if (lane == 0) atomicAdd(events, ev);
}

}  // namespace
}  // namespace lgx
