// Shared helpers for the liblgx HIP sources (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/lgx.h"

namespace lgx {

// thread-local last-error message behind lgx_last_error()
void set_error(const char* fmt, ...);

#define LGX_HIP_CHECK(expr)                                                              \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            ::lgx::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,               \
                             hipGetErrorString(_e));                                     \
            return LGX_ERR_HIP;                                                          \
        }                                                                                \
    } while (0)

#define LGX_REQUIRE(cond, code, ...)                                                     \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            ::lgx::set_error(__VA_ARGS__);                                               \
            return (code);                                                               \
        }                                                                                \
    } while (0)

// launch-status check (kernel launches report errors lazily)
#define LGX_LAUNCH_CHECK() LGX_HIP_CHECK(hipGetLastError())

inline hipStream_t as_hip(lgx_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;  // CDNA wavefront
constexpr int kMaxTopK = 256;  // largest k of the top-k entry points (WaveList<4>)

// ------------------------------------------------------------------ bf16 <-> f32
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
    return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
// round-to-nearest-even (finite inputs; NaN stays NaN via the quiet bit)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>(u >> 16);
}

// ------------------------------------------------------------------ counter-based RNG
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
// uniform in (0, 1] from the top 24 bits
__host__ __device__ __forceinline__ float u01(uint64_t h) {
    return (static_cast<float>(h >> 40) + 1.0f) * (1.0f / 16777216.0f);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

}  // namespace lgx
