// Development only (tools/score_lab LAB_WS=0..3): the wave-specialised bf16 walk, measured and not
// taken (profiles/r03_score_lab_ws.txt).  Included by score_lab.hip after csrc/score_topk.hip.
#pragma once

namespace lgx {
namespace {

// ---------------------------------------------------------------- wave-specialised LDS walk
// the bf16 full-sweep walk with the top-k taken off the
// MFMA waves.  8 MFMA waves (32 users each, the LDS tile ring, the 16x16x32 main loop and the
// per-tile fast-path test, as score_topk_bf16_lds) post every flagged 16-item block -- both user
// halves' f32 scores, 32 B per lane -- to a ring of kWsRing entries per wave in LDS and go on; 4
// helper waves, one per SIMD, each own the 64 users of the two MFMA waves sharing its SIMD, ONE user
// per lane: the lists, the Bloom filter, parked mask suspects and the threshold each user's MFMA
// lanes test against (tau in LDS, refreshed by the MFMA waves every tile; a stale tau is lower, so
// it only admits more blocks).  The helpers serve their rings until both waves have posted the
// tile's epilogue, then join the tile barrier; an MFMA wave finding its ring full waits for the
// helper (which never waits at a barrier while one of its waves has an epilogue to post).
constexpr int kWsRing = 3;
constexpr int kWsMfma = 8, kWsHelpers = 4, kWsWaves = kWsMfma + kWsHelpers;
struct WsLayout {
    size_t lists, tau, ring, hdr, ctr, total;
};
__host__ __device__ inline WsLayout ws_layout(int k, size_t tiles_bytes) {
    WsLayout L;
    L.lists = tiles_bytes;
    L.tau = L.lists + ((size_t)kWsMfma * kUsersPerWave * kstride(k) + kListSpare) * 8;
    L.ring = L.tau + (size_t)kWsMfma * kUsersPerWave * 4;
    L.hdr = L.ring + (size_t)kWsMfma * kWsRing * 2048;
    L.ctr = L.hdr + (size_t)kWsMfma * kWsRing * 4;
    L.total = L.ctr + 3 * kWsMfma * 4 + 16;  // + the MFMA waves' arrival counter (WSV 3)
    return L;
}

__device__ __forceinline__ void lds_order() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// WSV (development): 0 as described, 1 helpers poll without sleeping, 2 the MFMA waves never post
// (their threshold forced to +inf: the walk's structural cost alone; lists wrong), 3 the MFMA waves
// sync the tile ring through an LDS arrival counter and the helpers join no tile barrier at all
// (they serve their rings until every MFMA wave has posted its last epilogue)
template <int KSTEPS, int WSV = 0>
__global__ __launch_bounds__(kWsWaves * 64) __attribute__((amdgpu_waves_per_eu(3, 3)))
void score_topk_bf16_ws(ScoreArgs a, int64_t n_utiles, int nbuf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    typedef LdsGeom<KSTEPS, kWsMfma, 2, 2> G;
    typedef Frag<LGX_DTYPE_BF16> F;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    constexpr int NS = G::CPR / 4;
    static_assert(KSTEPS % 2 == 0, "16x16x32 walk: d a multiple of 32");
    const int k = a.k;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WsLayout L = ws_layout(k, (size_t)nbuf * G::TILE);
    unsigned char* tiles = smem;
    uint64_t* lists = reinterpret_cast<uint64_t*>(smem + L.lists);
    float* tau_l = reinterpret_cast<float*>(smem + L.tau);
    unsigned char* ring = smem + L.ring;
    int* hdr = reinterpret_cast<int*>(smem + L.hdr);
    volatile int* head = reinterpret_cast<int*>(smem + L.ctr);
    volatile int* tail = head + kWsMfma;
    volatile int* done = head + 2 * kWsMfma;
    volatile int* arrive = head + 3 * kWsMfma;

    const int64_t utile = blockIdx.x;
    if (utile >= n_utiles) return;
    const int64_t i_begin = a.seed_items;
    const int64_t i_end = min(a.n_items, i_begin + a.split_items);
    const int64_t ntiles = i_end > i_begin ? (i_end - i_begin + G::TILE_ITEMS - 1) / G::TILE_ITEMS : 0;
    const int64_t rot = ((int64_t)blockIdx.x % 8) * (ntiles / 8);
    const unsigned char* items = static_cast<const unsigned char*>(a.items);
    const uint32_t lds_tiles = lds_u32(tiles);
    auto tile_start = [&](int64_t t) __attribute__((always_inline)) {
        int64_t u = t + rot;
        if (u >= ntiles) u -= ntiles;
        return i_begin + u * G::TILE_ITEMS;
    };
    if (threadIdx.x < 3 * kWsMfma + 1) head[threadIdx.x] = 0;  // head, tail, done, arrive

    if (wave >= kWsMfma) {
        // ------------------------------------------------------------ helper wave
        const int hh = wave - kWsMfma;
        const int mw = lane < 32 ? hh : hh + kWsHelpers;  // the MFMA wave whose user this lane owns
        const int ul = mw * kUsersPerWave + (lane & 31);  // user inside the workgroup
        const int64_t b = utile * G::USERS + ul;
        const bool ok = b < a.B;
        uint64_t* keys = lists + (size_t)ul * kstride(k);
        int len = 0, mp = 0;
        uint64_t kmin = 0;
        float fl = -INFINITY;
        auto rescan = [&]() __attribute__((always_inline)) {
            uint64_t m = ~0ull;
            int p = 0;
            for (int j0 = 0; j0 < k; j0 += 8) {
                uint64_t v[8];
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(keys + j0 + j);
                    v[j] = q.x;
                    v[j + 1] = q.y;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint64_t x = (j0 + j < k) ? v[j] : ~0ull;
                    if (x < m) {
                        m = x;
                        p = j0 + j;
                    }
                }
            }
            mp = p;
            kmin = m;
        };
        uint32_t bl[kBloomWords];
#pragma unroll
        for (int w = 0; w < kBloomWords; ++w) bl[w] = 0u;
        auto bloom_test = [&](uint32_t hv) __attribute__((always_inline)) {
            const uint32_t q = hv >> 5, m = 1u << (hv & 31);
            uint32_t hit = 0;
#pragma unroll
            for (int w = 0; w < kBloomWords; ++w) hit |= bl[w] & (q == (uint32_t)w ? m : 0u);
            return hit != 0u;
        };
        int scnt = 0;  // parked suspects of this user
        uint64_t* susp = a.susp ? a.susp + (size_t)b * 2 * kSuspSlots : nullptr;
        if (ok) {
            if (a.mask_indptr) {
                for (int64_t j = a.mask_indptr[b]; j < a.mask_indptr[b + 1]; ++j) {
                    const int32_t x = a.mask_indices[j];
#pragma unroll
                    for (int hsel = 0; hsel < 2; ++hsel) {
                        const uint32_t hv = hsel ? WaveTopK::bloom_h2(x) : WaveTopK::bloom_h1(x);
                        const uint32_t q = hv >> 5, m = 1u << (hv & 31);
#pragma unroll
                        for (int w = 0; w < kBloomWords; ++w) bl[w] |= q == (uint32_t)w ? m : 0u;
                    }
                }
            }
            if (a.seed_score) {
                const float* ss = a.seed_score + (size_t)b * k;
                const int32_t* si = a.seed_idx + (size_t)b * k;
                for (int j = 0; j < k; ++j)
                    if (si[j] >= 0) keys[len++] = make_key(ss[j], si[j]);
                if (len == k) rescan();
            } else if (a.floor) {
                fl = a.floor[b];
            }
        }
        auto publish_tau = [&]() __attribute__((always_inline)) { tau_l[ul] = !ok ? INFINITY : (len == k ? key_score(kmin) : fl); };
        publish_tau();
        // true: the key must not enter now (masked, or parked for the flush's exact test)
        auto masked = [&](uint64_t key) __attribute__((always_inline)) {
            if (!a.mask_indptr) return false;
            const int32_t it = key_index(key);
            if (!bloom_test(WaveTopK::bloom_h1(it)) || !bloom_test(WaveTopK::bloom_h2(it))) return false;
            if (susp && scnt < 2 * kSuspSlots) {
                susp[scnt++] = key;
                return true;
            }
            return is_masked(a, b, it);
        };
        auto insert = [&](uint64_t key, bool check) __attribute__((always_inline)) {
            if (len == k) {
                if (key <= kmin || (check && masked(key))) return;
                keys[mp] = key;
                rescan();
            } else {
                if (check && masked(key)) return;
                keys[len++] = key;
                if (len == k) rescan();
            }
        };
        int tl0 = 0, tl1 = 0;  // entries consumed from the rings of waves hh and hh + 4
        auto process = [&](int s, int slot) __attribute__((always_inline)) {
            const int w = s ? hh + kWsHelpers : hh;
            const unsigned char* e = ring + ((size_t)w * kWsRing + slot) * 2048;
            const int i0 = __builtin_amdgcn_readfirstlane(hdr[w * kWsRing + slot]);
            if (ok && (lane >> 5) == s) {
                const int u = lane & 31, ub = u >> 4, r = u & 15;
                float sc[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 v = *reinterpret_cast<const f32x4*>(e + (r + 16 * q) * 32 + ub * 16);
#pragma unroll
                    for (int g = 0; g < 4; ++g) sc[4 * q + g] = v[g];
                }
                // candidates against the list as it stands (insert re-tests each against the moving kmin)
                uint32_t cm = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const bool in = i0 + j < i_end;
                    const bool pass = len == k ? make_key(sc[j], i0 + j) > kmin : sc[j] >= fl;
                    cm |= in && pass ? 1u << j : 0u;
                }
                if (cm) {
                    while (cm) {
                        const int j = __builtin_ctz(cm);
                        cm &= cm - 1;
                        float v = sc[0];
#pragma unroll
                        for (int q = 1; q < 16; ++q) v = j == q ? sc[q] : v;
                        insert(make_key(v, i0 + j), true);
                    }
                    publish_tau();
                }
            }
        };
        // Serve both rings until wave hh has posted n0 epilogues and wave hh + 4 n1; entries still
        // queued then wait for the next tile (served while the MFMA waves compute it), so the barrier
        // never waits for an insertion.  all: until every entry is done (after the sweep).  No
        // deadlock: a wave waiting for ring space has not posted its epilogue, so its helper is here.
        auto serve = [&](int n0, int n1, bool all) __attribute__((always_inline)) {
            while (true) {
                const int d0 = __builtin_amdgcn_readfirstlane(done[hh]);
                const int d1 = __builtin_amdgcn_readfirstlane(done[hh + kWsHelpers]);
                const int h0 = __builtin_amdgcn_readfirstlane(head[hh]);
                const int h1 = __builtin_amdgcn_readfirstlane(head[hh + kWsHelpers]);
                asm volatile("" ::: "memory");  // the entries are read after the heads
                const bool posted = d0 >= n0 && d1 >= n1;
                const bool pending = tl0 < h0 || tl1 < h1;
                if (posted && (!all || !pending)) break;  // heads read after the done counts
                if (!pending) {
                    if (WSV != 1) __builtin_amdgcn_s_sleep(2);
                    continue;
                }
                // the ring further behind first
                const int s = tl0 < h0 && (tl1 >= h1 || h0 - tl0 >= h1 - tl1) ? 0 : 1;
                process(s, (s ? tl1 : tl0) % kWsRing);
                tl0 += s ? 0 : 1;
                tl1 += s;
                lds_order();
                if (lane == 0) tail[s ? hh + kWsHelpers : hh] = s ? tl1 : tl0;
            }
        };
        __syncthreads();  // the prologue barrier: lists, filters and tau ready
        if (WSV != 3) {
            for (int64_t t = 0; t < ntiles; ++t) {
                serve((int)t + 1, (int)t, false);  // early waves post epilogue t before barrier t, late waves t - 1
                __syncthreads();
            }
        }
        serve((int)ntiles, (int)ntiles, true);
        // parked suspects: exact test, then into the list
        if (ok && susp) {
            for (int j = 0; j < scnt; ++j)
                if (!is_masked(a, b, key_index(susp[j]))) insert(susp[j], false);
        }
        if (ok) {
            float* ps = a.part_score + (size_t)b * k;
            int32_t* pi = a.part_idx + (size_t)b * k;
            for (int j = 0; j < k; ++j) {
                ps[j] = j < len ? key_score(keys[j]) : -INFINITY;
                pi[j] = j < len ? key_index(keys[j]) : -1;
            }
        }
        return;
    }

    // ---------------------------------------------------------------- MFMA wave
    const int w = wave;
    const int r16 = lane & 15, q4 = lane >> 4;
    uint4 uf[2 * NS];
#pragma unroll
    for (int ub = 0; ub < 2; ++ub) {
        const int64_t bu = utile * G::USERS + w * kUsersPerWave + 16 * ub + r16;
        const bool ok = bu < a.B;
        const int64_t qr = ok ? (a.user_rows ? a.user_rows[bu] : bu) : 0;
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2)
            uf[ub * NS + s2] = __builtin_bit_cast(uint4, F::load(a.Q, qr, a.d, 2 * s2 + (q4 >> 1), q4 & 1, ok));
    }
#pragma unroll
    for (int c = 0; c < 2 * NS; ++c) {
        u32x4 t = __builtin_bit_cast(u32x4, uf[c]);
        asm volatile("" : "+v"(t));
        uf[c] = __builtin_bit_cast(uint4, t);
    }
    constexpr int PPW = (G::PIECES + kWsMfma - 1) / kWsMfma;
    const int my_pieces = max(0, min(PPW, G::PIECES - w * PPW));
    auto stage = [&](int buf, int64_t t0) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
            if (p < my_pieces) {
                const uint64_t bu = reinterpret_cast<uint64_t>(items + t0 * G::RB);
                const unsigned char* base = reinterpret_cast<const unsigned char*>(
                    ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bu));
                const bool tl_ = t0 + G::TILE_ITEMS > i_end;
                const int last = (int)(i_end - 1 - t0);
                const int q = (w * PPW + p) * 64 + lane;
                const int row = q / G::CPR;
                const int src = (q % G::CPR) ^ (row & G::SWZ);
                const int srow = tl_ && row > last ? last : row;
                lds_dma16(base, (uint32_t)(srow * G::RB + src * 16),
                          __builtin_amdgcn_readfirstlane(lds_tiles + buf * G::TILE + (w * PPW + p) * 1024));
            }
        }
    };
    const int ahead = nbuf - 1;
    for (int j = 0; j < ahead && j < ntiles; ++j) stage(j, tile_start(j));
    wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(ahead, ntiles) - 1));
    __syncthreads();
    int buf = 0, sbuf = ahead;
    const bool late = w >= kWsMfma / 2;
    f32x4 c[2][4];
    int64_t prev_t0 = 0;
    int head_r = 0, tail_r = 0, epi = 0;
    auto compute = [&]() __attribute__((always_inline)) {
        const unsigned char* T = tiles + buf * G::TILE;
#pragma unroll
        for (int ub = 0; ub < 2; ++ub)
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) c[ub][ib] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const unsigned char* rowp = T + r16 * G::RB;
        auto frag = [&](int s2, int ib) __attribute__((always_inline)) {
            return *reinterpret_cast<const uint4*>(rowp + ib * 16 * G::RB + (((4 * s2 + q4) ^ (r16 & G::SWZ)) * 16));
        };
        uint4 fa[4];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib) fa[ib] = frag(0, ib);
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
#pragma unroll
                for (int ub = 0; ub < 2; ++ub)
                    c[ub][ib] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        __builtin_bit_cast(bf16x8, fa[ib]), __builtin_bit_cast(bf16x8, uf[ub * NS + s2]), c[ub][ib], 0, 0, 0);
                if (s2 + 1 < NS) fa[ib] = frag(s2 + 1, ib);
            }
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                if (s2 + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
    };
    auto epilogue = [&](int64_t e0) __attribute__((always_inline)) {
        float tA = tau_l[w * kUsersPerWave + r16], tB = tau_l[w * kUsersPerWave + 16 + r16];
        if (WSV == 2) tA = tB = INFINITY;
        float m0 = c[0][0][0], m1 = c[1][0][0];
#pragma unroll
        for (int ib = 0; ib < 4; ++ib)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                m0 = fmaxf(m0, c[0][ib][r]);
                m1 = fmaxf(m1, c[1][ib][r]);
            }
        if (__ballot((m0 >= tA) | (m1 >= tB)) != 0ull) {
#pragma unroll
            for (int ib = 0; ib < 4; ++ib) {
                const float a0 = fmaxf(fmaxf(c[0][ib][0], c[0][ib][1]), fmaxf(c[0][ib][2], c[0][ib][3]));
                const float a1 = fmaxf(fmaxf(c[1][ib][0], c[1][ib][1]), fmaxf(c[1][ib][2], c[1][ib][3]));
                if (__ballot((a0 >= tA) | (a1 >= tB)) == 0ull) continue;
                while (head_r - tail_r >= kWsRing) {  // ring full: the helper is serving it
                    __builtin_amdgcn_s_sleep(1);
                    tail_r = __builtin_amdgcn_readfirstlane(tail[w]);
                }
                const int slot = head_r % kWsRing;
                unsigned char* e = ring + ((size_t)w * kWsRing + slot) * 2048 + lane * 32;
                *reinterpret_cast<f32x4*>(e) = c[0][ib];
                *reinterpret_cast<f32x4*>(e + 16) = c[1][ib];
                if (lane == 0) hdr[w * kWsRing + slot] = (int)(e0 + 16 * ib);
                ++head_r;
                lds_order();
                if (lane == 0) head[w] = head_r;
            }
        }
        ++epi;
        lds_order();
        if (lane == 0) done[w] = epi;
    };
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t t0 = tile_start(t);
        if (t + ahead < ntiles) stage(sbuf, tile_start(t + ahead));
        if (late && t > 0) epilogue(prev_t0);
        compute();
        if (!late) epilogue(t0);
        prev_t0 = t0;
        wait_vmcnt_le(my_pieces * (int)max<int64_t>(0, min<int64_t>(t + ahead, ntiles - 1) - (t + 1)));
        if (WSV == 3) {
            // this wave's pieces of tile t+1 have landed and it is done reading tile t: arrive, then
            // wait for the other MFMA waves (a wave's LDS operations complete in order)
            lds_order();
            if (lane == 0) __hip_atomic_fetch_add(const_cast<int*>(arrive), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int target = kWsMfma * (int)(t + 1);
            while (__builtin_amdgcn_readfirstlane(*arrive) < target) __builtin_amdgcn_s_sleep(0);
            asm volatile("" ::: "memory");
        } else {
            __syncthreads();
        }
        buf = buf + 1 == nbuf ? 0 : buf + 1;
        sbuf = sbuf + 1 == nbuf ? 0 : sbuf + 1;
    }
    if (late && ntiles > 0) epilogue(prev_t0);
}


}  // namespace
}  // namespace lgx
