// Development: the read ceiling under the a9 row top-K (lgx_topk_rows, tools.h:13-33) on its row's
// shape ([4096, 1M] f32 = 16.4 GB, k = 20), hipEvents, median of 5.
//   make -C tools topk_lab && tools/topk_lab
// R1 reads every row with the product's grid and load pattern (one 256-thread workgroup per row,
// 4 float4 loads in flight per lane) and keeps only a running max; R2 is a grid-stride float4 read
// of the whole matrix.
#include "lgx_common.h"

#include <algorithm>
#include <cstdio>
#include <vector>

#define HK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int UNROLL>
__global__ __launch_bounds__(256) void r_rows(const float* __restrict__ S, int64_t cols, float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float* s = S + (int64_t)blockIdx.x * cols;
    const int64_t stride = 64 * 4 * 4;
    float m = -INFINITY;
    for (int64_t base = (int64_t)wave * 256; base < cols; base += stride * UNROLL) {
        float4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t c0 = base + u * stride + lane * 4;
            v[u] = c0 + 3 < cols ? *reinterpret_cast<const float4*>(s + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) m = fmaxf(m, fmaxf(fmaxf(v[u].x, v[u].y), fmaxf(v[u].z, v[u].w)));
    }
    if (m == 12345.0f) out[0] = m;  // keeps the loads
}

__global__ void r_stream(const float4* __restrict__ S, int64_t n4, float* out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    float m = -INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = S[i];
        m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    if (m == 12345.0f) out[0] = m;
}

int main() {
    const int64_t R = 4096, C = 1000000;
    const int k = 20;
    float *S, *vals, *dummy;
    int32_t* idx;
    HK(hipMalloc(&S, R * C * 4));
    HK(hipMalloc(&vals, R * k * 4));
    HK(hipMalloc(&idx, R * k * 4));
    HK(hipMalloc(&dummy, 4));
    if (lgx_fill_normal(S, R * C, 1.0f, 3, LGX_DTYPE_F32, nullptr)) return 1;
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    const double gb = R * C * 4 / 1e9;
    auto timeit = [&](const char* name, auto&& fn) -> int {
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
        std::printf("%-44s %7.3f ms  %6.2f TB/s\n", name, ms, gb / ms);
        std::fflush(stdout);
        return 0;
    };
    timeit("product lgx_topk_rows k=20", [&] { lgx_topk_rows(S, R, C, C, k, idx, vals, nullptr); });
    timeit("R1 rows, product pattern, unroll 4", [&] { r_rows<4><<<R, 256>>>(S, C, dummy); });
    timeit("R1b rows, unroll 8", [&] { r_rows<8><<<R, 256>>>(S, C, dummy); });
    timeit("R2 grid-stride float4 read", [&] { r_stream<<<256 * 16, 256>>>((const float4*)S, R * C / 4, dummy); });
    timeit("R2b grid-stride, 4x the workgroups", [&] { r_stream<<<256 * 64, 256>>>((const float4*)S, R * C / 4, dummy); });
    HK(hipDeviceSynchronize());
    return 0;
}
