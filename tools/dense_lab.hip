// Development: A/B timing of getUsersRating's dense [B, I] scoring (lgx_score_dense, bf16 d=256) on
// the a6 row's shape (4096 users x 1M items, f32 out = 16.4 GB), hipEvents, median of 5.
//   make -C tools dense_lab && tools/dense_lab [B]
// Standalone kernels (linked against liblgx.so for the product call and fill_normal, so a rebuild
// takes seconds).  W0 / W1 are write ceilings: a linear float4 stream of the same 16.4 GB, and the
// product's store pattern without loads or MFMAs.  Every variant's output is compared with the
// product's, bit for bit.
#include "lgx_common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int kWaves = 8, kUPW = 32, kUsers = kWaves * kUPW;

__device__ __forceinline__ int tile_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ f32x16 mma(uint4 a, uint4 b, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}

__global__ void w_linear(float4* out, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) out[i] = v;
}

__global__ __launch_bounds__(512) void w_pattern(float* out, int64_t B, int64_t n_items, int64_t n_ug, int64_t split_items) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug, split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kUsers + (int64_t)wave * kUPW;
    const int64_t i_begin = split * split_items, i_end = std::min(n_items, i_begin + split_items);
    for (int64_t i0 = i_begin; i0 < i_end; i0 += 32) {
        const int64_t item_row = i0 + col;
        if (item_row < i_end)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t u = u0 + tile_row(r, h);
                if (u < B) out[u * n_items + item_row] = (float)r;
            }
    }
}

// score_dense_lds (d = 256 bf16: 16 chunks) with TI-item tiles per barrier.
// ABL 1: no global loads (the first tile stays in LDS: MFMA + stores only; output differs)
// ABL 2: no MFMAs (the fragment bits are stored: loads + stores only; output differs)
// PIPE: the 16 stores of a 32-item block issue between the MFMAs of the next block (one
//       accumulator in flight to memory while the other fills)
template <int TI, int ABL, bool PIPE, bool SB>
__device__ __forceinline__ void dense_body(const void* Q, const void* items, int64_t B, int64_t n_items,
                                           float* __restrict__ out, int64_t n_ug, int64_t split_items) {
    constexpr int KCH = 16, SPR = 32, RB = 512, TILE = TI * RB, NL = TI * SPR / (kWaves * 64);
    __shared__ __attribute__((aligned(16))) unsigned char img[2][TILE];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug, split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kUsers + (int64_t)wave * kUPW;
    const bool wave_on = u0 < B;
    const int64_t b = u0 + col;
    (void)0;
    const bool user_ok = b < B;
    uint4 uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c)
        uf[c] = user_ok ? *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(Q) + b * 256 + c * 16 + 8 * h)
                        : make_uint4(0u, 0u, 0u, 0u);
    const int64_t i_begin = split * split_items, i_end = std::min(n_items, i_begin + split_items);
    const unsigned char* ib = static_cast<const unsigned char*>(items);
    uint4 nx[NL];
    auto load_tile = [&](int64_t i0) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            const int64_t it = i0 + r;
            nx[j] = it < i_end ? *reinterpret_cast<const uint4*>(ib + it * RB + q * 16) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * kWaves * 64;
            const int r = sl / SPR, q = sl % SPR;
            *reinterpret_cast<uint4*>(&img[buf][r * RB + ((q ^ (r & 15)) * 16)]) = nx[j];
        }
    };
    if (i_begin >= i_end) return;
    load_tile(i_begin);
    store_tile(0);
    __syncthreads();
    int buf = 0;
    f32x16 pend;
    int64_t pend_item = -1;
    // SB: stores as a wave-uniform row base (SGPRs) + a 32-bit lane byte offset (one VGPR), instead
    // of 16 live 64-bit addresses
    const int64_t u0s = (int64_t)__builtin_amdgcn_readfirstlane((int)(u0 & 0x7fffffff));
    auto store_acc = [&](const f32x16& v, int64_t item_row) {
        if (item_row >= 0 && item_row < i_end) {
            if (SB) {
                const int64_t i0s = item_row - col;  // the block's first item: wave-uniform
                const uint32_t boff = (uint32_t)(4 * h * n_items + col) * 4u;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const char* base = reinterpret_cast<const char*>(out + (u0s + tile_row(r, 0)) * n_items + i0s);
                    if (u0s + tile_row(r, h) < B) *reinterpret_cast<float*>(const_cast<char*>(base) + boff) = v[r];
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t u = u0 + tile_row(r, h);
                    if (u < B) out[u * n_items + item_row] = v[r];
                }
            }
        }
    };
    for (int64_t i0 = i_begin; i0 < i_end; i0 += TI) {
        const bool more = i0 + TI < i_end;
        if (more && ABL != 1) load_tile(i0 + TI);
        if (wave_on) {
#pragma unroll
            for (int hh = 0; hh < TI / 32; ++hh) {
                const unsigned char* rowp = &img[buf][(32 * hh + col) * RB];
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
                for (int c = 0; c < KCH; ++c) {
                    const uint4 fr = *reinterpret_cast<const uint4*>(rowp + (((2 * c + h) ^ (col & 15)) * 16));
                    if (ABL == 2) acc[c] = __uint_as_float(fr.x ^ fr.y ^ uf[c].x);
                    else acc = mma(uf[c], fr, acc);
                }
                const int64_t item_row = i0 + 32 * hh + col;
                if (PIPE) {
                    store_acc(pend, pend_item);
                    // the previous block's stores between this block's MFMAs
#pragma unroll
                    for (int c = 0; c < KCH; ++c) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
                        __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);   // 1 VMEM write
                    }
                    pend = acc;
                    pend_item = item_row;
                } else {
                    store_acc(acc, item_row);
                }
            }
        }
        if (more && ABL != 1) store_tile(buf ^ 1);
        __syncthreads();
        if (ABL != 1) buf ^= 1;
    }
    if (PIPE && wave_on) store_acc(pend, pend_item);
}

template <int TI, int ABL, bool PIPE, bool SB = false>
__global__ __launch_bounds__(kWaves * 64) void dense_v(const void* Q, const void* items, int64_t B, int64_t n_items,
                                                       float* __restrict__ out, int64_t n_ug, int64_t split_items) {
    dense_body<TI, ABL, PIPE, SB>(Q, items, B, n_items, out, n_ug, split_items);
}
// the same with the register budget of 4 waves per SIMD (two 8-wave workgroups per CU)
template <int TI, int ABL, bool PIPE, bool SB = false>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(4, 4)))
void dense_w4(const void* Q, const void* items, int64_t B, int64_t n_items, float* __restrict__ out, int64_t n_ug,
              int64_t split_items) {
    dense_body<TI, ABL, PIPE, SB>(Q, items, B, n_items, out, n_ug, split_items);
}
// second round: 32-item tiles, scalar-base stores, WV waves per workgroup (WV x 32 users), the next
// tile's loads PF (1 or 2) tiles ahead in registers (PF 2: the loop unrolled by two so the two
// register sets keep their names); ABL 3: every tile load reads the split's first 64 items
// (L2-resident: the loads' ceiling, output differs)
template <int WV, int PF, int ABL>
__device__ __forceinline__ void dense2_body(const void* Q, const void* items, int64_t B, int64_t n_items,
                                            float* __restrict__ out, int64_t n_ug, int64_t split_items) {
    constexpr int KCH = 16, SPR = 32, RB = 512, TI = 32, TILE = TI * RB, NT = WV * 64, NL = TI * SPR / NT;
    constexpr int USERS = WV * kUPW;
    __shared__ __attribute__((aligned(16))) unsigned char img[2][TILE];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug, split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * USERS + (int64_t)wave * kUPW;
    const bool wave_on = u0 < B;
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    uint4 uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c)
        uf[c] = user_ok ? *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(Q) + b * 256 + c * 16 + 8 * h)
                        : make_uint4(0u, 0u, 0u, 0u);
    const int64_t i_begin = split * split_items, i_end = std::min(n_items, i_begin + split_items);
    const unsigned char* ib = static_cast<const unsigned char*>(items);
    auto load_tile = [&](uint4* nx, int64_t i0) {
        if (ABL == 3) i0 = i_begin + (i0 & 32);
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * NT;
            const int r = sl / SPR, q = sl % SPR;
            const int64_t it = i0 + r;
            nx[j] = it < i_end ? *reinterpret_cast<const uint4*>(ib + it * RB + q * 16) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_tile = [&](const uint4* nx, int buf) {
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int sl = threadIdx.x + j * NT;
            const int r = sl / SPR, q = sl % SPR;
            *reinterpret_cast<uint4*>(&img[buf][r * RB + ((q ^ (r & 15)) * 16)]) = nx[j];
        }
    };
    const uint32_t boff = (uint32_t)(4 * h * n_items + col) * 4u;
    auto tile = [&](int buf, int64_t i0) {
        if (!wave_on) return;
        const unsigned char* rowp = &img[buf][col * RB];
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
        for (int c = 0; c < KCH; ++c) {
            const uint4 fr = *reinterpret_cast<const uint4*>(rowp + (((2 * c + h) ^ (col & 15)) * 16));
            acc = mma(uf[c], fr, acc);
        }
        if (i0 + col < i_end) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const char* base = reinterpret_cast<const char*>(out + (u0 + tile_row(r, 0)) * n_items + i0);
                if (u0 + tile_row(r, h) < B) *reinterpret_cast<float*>(const_cast<char*>(base) + boff) = acc[r];
            }
        }
    };
    if (i_begin >= i_end) return;
    uint4 na[NL], nb[NL];
    load_tile(na, i_begin);
    store_tile(na, 0);
    if (PF == 2 && i_begin + TI < i_end) load_tile(na, i_begin + TI);
    __syncthreads();
    if (PF == 1) {
        int buf = 0;
        for (int64_t i0 = i_begin; i0 < i_end; i0 += TI) {
            const bool more = i0 + TI < i_end;
            if (more) load_tile(na, i0 + TI);
            tile(buf, i0);
            if (more) store_tile(na, buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    } else {
        // na holds tile t + 1 on entry to an even step, nb on entry to an odd one
        for (int64_t i0 = i_begin; i0 < i_end; i0 += 2 * TI) {
            if (i0 + 2 * TI < i_end) load_tile(nb, i0 + 2 * TI);
            tile(0, i0);
            if (i0 + TI < i_end) store_tile(na, 1);
            __syncthreads();
            if (i0 + TI >= i_end) break;
            if (i0 + 3 * TI < i_end) load_tile(na, i0 + 3 * TI);
            tile(1, i0 + TI);
            if (i0 + 2 * TI < i_end) store_tile(nb, 0);
            __syncthreads();
        }
    }
}

template <int WV, int PF, int ABL, int WPE>
__global__ __launch_bounds__(WV * 64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void dense2(const void* Q, const void* items, int64_t B, int64_t n_items, float* __restrict__ out, int64_t n_ug,
            int64_t split_items) {
    dense2_body<WV, PF, ABL>(Q, items, B, n_items, out, n_ug, split_items);
}
// third round: the tile ring filled by LDS-DMA (global_load_lds_dwordx4, no VGPR staging), NBUF
// buffers with NBUF-1 tiles in flight.  vmcnt counts the score stores as well as the DMA (gfx9
// counts both, in order), so the wait for tile t+1 allows this iteration's own DMA pieces plus its
// 16 stores -- only when the wave issued exactly 16 (a full wave on a whole tile), else vmcnt(0).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}
#pragma clang diagnostic pop

template <int NBUF>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4)))
void dense_dma(const void* Q, const void* items, int64_t B, int64_t n_items, float* __restrict__ out, int64_t n_ug,
               int64_t split_items) {
    constexpr int KCH = 16, RB = 512, TILE = 32 * RB, PPW = TILE / 1024 / kWaves;  // 2 pieces per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char ring[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, col = lane & 31;
    const int64_t L = blockIdx.x, kk = L >> 3;
    const int64_t ug = kk % n_ug, split = (kk / n_ug) * 8 + (L & 7);
    const int64_t u0 = ug * kUsers + (int64_t)wave * kUPW;
    const bool wave_on = u0 < B, full_wave = u0 + kUPW <= B;
    const int64_t b = u0 + col;
    const bool user_ok = b < B;
    uint4 uf[KCH];
#pragma unroll
    for (int c = 0; c < KCH; ++c)
        uf[c] = user_ok ? *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(Q) + b * 256 + c * 16 + 8 * h)
                        : make_uint4(0u, 0u, 0u, 0u);
    const int64_t i_begin = split * split_items, i_end = std::min(n_items, i_begin + split_items);
    if (i_begin >= i_end) return;
    const int64_t ntiles = (i_end - i_begin + 31) / 32;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ring;
    const unsigned char* ib = static_cast<const unsigned char*>(items);
    auto stage = [&](int buf, int64_t t) {
        const int64_t t0 = i_begin + t * 32;
        const uint64_t bu = reinterpret_cast<uint64_t>(ib + t0 * RB);
        const unsigned char* base = reinterpret_cast<const unsigned char*>(
            ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(bu >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)bu));
        const int last = (int)(i_end - 1 - t0);
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
            const int q = (wave * PPW + p) * 64 + lane;   // LDS slot: row q / 32, chunk q % 32
            const int row = q / 32, src = (q % 32) ^ (row & 15);
            const int srow = row > last ? last : row;
            dma16(base, (uint32_t)(srow * RB + src * 16),
                  __builtin_amdgcn_readfirstlane(lds0 + buf * TILE + (wave * PPW + p) * 1024));
        }
    };
    const uint32_t boff = (uint32_t)(4 * h * n_items + col) * 4u;
    for (int j = 0; j < NBUF - 1 && j < ntiles; ++j) stage(j, j);
    if (ntiles > 1 && NBUF > 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int buf = 0, sbuf = NBUF - 1;
    for (int64_t t = 0; t < ntiles; ++t) {
        const int64_t i0 = i_begin + t * 32;
        const bool refill = t + NBUF - 1 < ntiles;
        if (refill) stage(sbuf, t + NBUF - 1);
        int nst = 0;
        if (wave_on) {
            const unsigned char* rowp = ring + buf * TILE + col * RB;
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll
            for (int c = 0; c < KCH; ++c) {
                const uint4 fr = *reinterpret_cast<const uint4*>(rowp + (((2 * c + h) ^ (col & 15)) * 16));
                acc = mma(uf[c], fr, acc);
            }
            if (i0 + col < i_end) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const char* base = reinterpret_cast<const char*>(out + (u0 + tile_row(r, 0)) * n_items + i0);
                    if (u0 + tile_row(r, h) < B) *reinterpret_cast<float*>(const_cast<char*>(base) + boff) = acc[r];
                }
            }
            nst = full_wave && i0 + 32 <= i_end ? 16 : -1;
        }
        // tile t+1 must have landed: allow the pieces issued this iteration (+ its 16 stores)
        if (t + 1 < ntiles) {
            if (refill && nst == 16) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
            else if (refill && !wave_on) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        buf = buf + 1 == NBUF ? 0 : buf + 1;
        sbuf = sbuf + 1 == NBUF ? 0 : sbuf + 1;
    }
}
}  // namespace

using lgx::ceil_div;

__global__ void diff_count(const float* a, const float* b, int64_t n, unsigned long long* cnt) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    unsigned long long c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        c += __float_as_uint(a[i]) != __float_as_uint(b[i]);
    if (c) atomicAdd(cnt, c);
}

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 4096;
    const int64_t I = 1000000, d = 256;
    void *Q, *items;
    float *out, *ref;
    unsigned long long* cnt;
    HK(hipMalloc(&Q, B * d * 2));
    HK(hipMalloc(&items, I * d * 2));
    HK(hipMalloc(&out, B * I * 4));
    HK(hipMalloc(&ref, B * I * 4));
    HK(hipMalloc(&cnt, 8));
    if (lgx_fill_normal(Q, B * d, 1.0f / 16, 1, LGX_DTYPE_BF16, nullptr)) return 1;
    if (lgx_fill_normal(items, I * d, 1.0f / 16, 2, LGX_DTYPE_BF16, nullptr)) return 1;
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    const double gb = B * I * 4 / 1e9;
    auto timeit = [&](const char* name, auto&& fn, bool check) -> int {
        std::vector<float> ts;
        for (int r = 0; r < 6; ++r) {
            HK(hipEventRecord(e0, 0));
            fn();
            HK(hipEventRecord(e1, 0));
            HK(hipEventSynchronize(e1));
            float ms;
            HK(hipEventElapsedTime(&ms, e0, e1));
            if (r) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const float ms = ts[ts.size() / 2];
        unsigned long long nd = 0;
        if (check) {
            HK(hipMemset(cnt, 0, 8));
            diff_count<<<4096, 256>>>(out, ref, B * I, cnt);
            HK(hipMemcpy(&nd, cnt, 8, hipMemcpyDeviceToHost));
        }
        std::printf("%-48s %7.3f ms  %6.2f TB/s of output  %s\n", name, ms, gb / ms, check ? (nd ? "DIFFERS" : "same bits") : "");
        std::fflush(stdout);
        return 0;
    };
    if (timeit("product lgx_score_dense", [&] { lgx_score_dense(Q, nullptr, items, B, I, d, LGX_DTYPE_BF16, 0, ref, nullptr); }, false)) return 1;
    HK(hipDeviceSynchronize());
    const int64_t n_ug = ceil_div(B, (int64_t)kUsers);
    const int64_t tiles = ceil_div(I, 32);
    const int64_t n_splits = std::max<int64_t>(8, std::min(8 * ceil_div(ceil_div(2048, n_ug), 8), 8 * ceil_div(tiles, 8)));
    const int64_t split32 = 32 * ceil_div(tiles, n_splits);
    const int64_t split64 = 64 * ceil_div(ceil_div(I, 64), n_splits);
    const unsigned grid = (unsigned)(n_ug * n_splits);
    timeit("W0 linear float4 write", [&] { w_linear<<<256 * 16, 256>>>((float4*)out, B * I / 4); }, false);
    timeit("W1 product store pattern", [&] { w_pattern<<<grid, 512>>>(out, B, I, n_ug, split32); }, false);
    timeit("V0 32 items", [&] { dense_v<32, 0, false><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("V2 64 items", [&] { dense_v<64, 0, false><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, true);
    timeit("V2a 64 items, no loads (MFMA + stores)", [&] { dense_v<64, 1, false><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, false);
    timeit("V2b 64 items, no MFMA (loads + stores)", [&] { dense_v<64, 2, false><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, false);
    timeit("V6 32 items, pipelined stores", [&] { dense_v<32, 0, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("V7 64 items, pipelined stores", [&] { dense_v<64, 0, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, true);
    timeit("V7a 64 items, pipelined, no loads", [&] { dense_v<64, 1, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, false);
    const int64_t split128 = 128 * ceil_div(ceil_div(I, 128), n_splits);
    timeit("V8 128 items, pipelined stores", [&] { dense_v<128, 0, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split128); }, true);
    timeit("S0 32 items, scalar-base stores", [&] { dense_v<32, 0, false, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("S2 64 items, scalar-base stores", [&] { dense_v<64, 0, false, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, true);
    timeit("S6 32 items, pipelined, scalar-base", [&] { dense_v<32, 0, true, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("S7 64 items, pipelined, scalar-base", [&] { dense_v<64, 0, true, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, true);
    timeit("X0 32 items, scalar-base, 4 waves/SIMD", [&] { dense_w4<32, 0, false, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("X2 64 items, scalar-base, 4 waves/SIMD", [&] { dense_w4<64, 0, false, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split64); }, true);
    timeit("X6 32 items, pipelined, 4 waves/SIMD", [&] { dense_w4<32, 0, true, true><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("Z0 = X0 (dense2 8 waves, PF1, 4/SIMD)", [&] { dense2<8, 1, 0, 4><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("Z0a Z0 with L2-resident loads", [&] { dense2<8, 1, 3, 4><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, false);
    timeit("Z1 8 waves, PF2, 4/SIMD", [&] { dense2<8, 2, 0, 4><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    // 4-wave workgroups: 128 users, twice the user groups; splits as the product would plan them
    const int64_t n_ug4 = ceil_div(B, 128);
    const int64_t ns4 = std::max<int64_t>(8, std::min(8 * ceil_div(ceil_div(2048, n_ug4), 8), 8 * ceil_div(tiles, 8)));
    const int64_t sp4 = 32 * ceil_div(tiles, ns4);
    const unsigned grid4 = (unsigned)(n_ug4 * ns4);
    timeit("Z2 4 waves, PF1, 4/SIMD", [&] { dense2<4, 1, 0, 4><<<grid4, 256>>>(Q, items, B, I, out, n_ug4, sp4); }, true);
    timeit("Z3 4 waves, PF2, 4/SIMD", [&] { dense2<4, 2, 0, 4><<<grid4, 256>>>(Q, items, B, I, out, n_ug4, sp4); }, true);
    timeit("Z2a 4 waves, PF1, L2-resident loads", [&] { dense2<4, 1, 3, 4><<<grid4, 256>>>(Q, items, B, I, out, n_ug4, sp4); }, false);
    timeit("Z4 8 waves, PF1, 3/SIMD", [&] { dense2<8, 1, 0, 3><<<grid, 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    HK(hipFuncSetAttribute((const void*)dense_dma<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 32 * 512));
    HK(hipFuncSetAttribute((const void*)dense_dma<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 32 * 512));
    timeit("D3 LDS-DMA ring, 3 buffers", [&] { dense_dma<3><<<grid, 512, 3 * 32 * 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    timeit("D4 LDS-DMA ring, 4 buffers", [&] { dense_dma<4><<<grid, 512, 4 * 32 * 512>>>(Q, items, B, I, out, n_ug, split32); }, true);
    HK(hipDeviceSynchronize());
    return 0;
}
