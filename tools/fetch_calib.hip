// FETCH_SIZE calibration for the SpMM's access pattern (development tool, not part of the library).
//
// MI355X_MICROARCH.md (HBM section): FETCH_SIZE reports 1/2 of the bytes of a wide coalesced
// STREAMING read on gfx950, other patterns are uncalibrated, and Infinity-Cache (MALL) hits
// appear to be counted.  The SpMM's traffic is random whole-row gathers (16 lanes x 16 B per bf16
// d=128 row, 32 x 16 B per fp32 row), so this program reads KNOWN byte counts in exactly that
// pattern, one kernel per case, and the rocprofv3 --pmc passes of tools/fetch_calib.sh divide the
// counter by the known bytes:
//   stream      : 2 GiB read once, 16 B per lane, coalesced (the guide's calibrated case)
//   once_256    : every row of a 2.56 GB table (10 M x 256 B) exactly once, in a random order
//   once_512    : every row of a 5.12 GB table (10 M x 512 B) exactly once, in a random order
//   hot_mall    : 40 M random 256-B rows of a 128 MiB table (fits the 256 MiB Infinity Cache)
//   hot_l2      : 40 M random 256-B rows of a 2 MiB table (fits one XCD's 4 MiB L2)
// Each kernel also prints its own rate (HIP events), which is the gather ceiling per cache level.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void calib_stream(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
    uint32_t s = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[blockIdx.x] = s;  // practically never: keeps the loads live
}

// one G-lane group per row (G = ROWB / 16), UNROLL rows in flight per group, like spmm_segments
template <int ROWB, int UNROLL>
__global__ __launch_bounds__(256) void calib_gather_once(const unsigned char* __restrict__ table,
                                                         const int32_t* __restrict__ perm, int64_t rows,
                                                         uint32_t* out) {
    constexpr int G = ROWB / 16 > 64 ? 64 : ROWB / 16;
    constexpr int CPL = ROWB / 16 / G;
    const int gl = threadIdx.x & (G - 1);
    const int64_t g0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngroups = (int64_t)gridDim.x * blockDim.x / G;
    uint32_t s = 0;
    for (int64_t r0 = g0 * UNROLL; r0 < rows; r0 += ngroups * UNROLL) {
        uint4 v[UNROLL][CPL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t r = r0 + u;
            const int64_t row = r < rows ? perm[r] : 0;
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                v[u][c] = r < rows ? *reinterpret_cast<const uint4*>(table + row * ROWB + (c * G + gl) * 16)
                                   : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int c = 0; c < CPL; ++c) s ^= v[u][c].x ^ v[u][c].y ^ v[u][c].z ^ v[u][c].w;
    }
    if (s == 0x12345678u) out[blockIdx.x] = s;
}

// n_gathers random rows (hash of the gather number) of a table of `rows` rows (a power of two:
// the row is hash & (rows - 1), no 64-bit division in the loop)
template <int ROWB, int UNROLL>
__global__ __launch_bounds__(256) void calib_gather_hot(const unsigned char* __restrict__ table, int64_t rows,
                                                        int64_t n_gathers, uint32_t* out) {
    constexpr int G = ROWB / 16;
    const int gl = threadIdx.x & (G - 1);
    const int64_t g0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngroups = (int64_t)gridDim.x * blockDim.x / G;
    uint32_t s = 0;
    for (int64_t r0 = g0 * UNROLL; r0 < n_gathers; r0 += ngroups * UNROLL) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int64_t row = (int64_t)(mix64((uint64_t)(r0 + u)) & (uint64_t)(rows - 1));
            v[u] = r0 + u < n_gathers ? *reinterpret_cast<const uint4*>(table + row * ROWB + gl * 16)
                                      : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) s ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (s == 0x12345678u) out[blockIdx.x] = s;
}

__global__ void fill_bytes(uint32_t* p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)mix64((uint64_t)i);
}

__global__ void make_perm(int32_t* perm, int64_t n) {
    // position i -> row (i * A + C) mod n with A coprime to n: a full-period permutation that
    // scatters consecutive positions far apart (good enough: every row exactly once, no locality)
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t A = 2654435761ull;  // odd prime; n below is 10,000,000 = 2^7 5^7, coprime to A
    perm[i] = (int32_t)(((uint64_t)i * A + 12345ull) % (uint64_t)n);
}

template <typename F>
float timed(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const int64_t rows = 10000000;
    const int64_t big = rows * 512;  // bytes: the 512-B table; the 256-B table is its first half
    unsigned char* table;
    int32_t* perm;
    uint32_t* out;
    CK(hipMalloc(&table, big));
    CK(hipMalloc(&perm, rows * 4));
    CK(hipMalloc(&out, 1 << 20));
    fill_bytes<<<4096, 256>>>(reinterpret_cast<uint32_t*>(table), big / 4);
    make_perm<<<(rows + 255) / 256, 256>>>(perm, rows);
    CK(hipDeviceSynchronize());
    const int grid = 256 * 32;  // 32 workgroups of 256 per CU
    const int64_t stream_bytes = 2ll << 30;
    float ms;
    ms = timed([&] { calib_stream<<<grid, 256>>>(reinterpret_cast<const uint4*>(table), stream_bytes / 16, out); }, reps);
    printf("stream    known_read_bytes %lld  %.3f ms  %.2f TB/s\n", (long long)stream_bytes, ms, stream_bytes / ms / 1e9);
    ms = timed([&] { calib_gather_once<256, 16><<<grid, 256>>>(table, perm, rows, out); }, reps);
    printf("once_256  known_read_bytes %lld  %.3f ms  %.2f TB/s (rows; + %lld B of row ids)\n",
           (long long)(rows * 256), ms, rows * 256 / ms / 1e9, (long long)(rows * 4));
    ms = timed([&] { calib_gather_once<512, 8><<<grid, 256>>>(table, perm, rows, out); }, reps);
    printf("once_512  known_read_bytes %lld  %.3f ms  %.2f TB/s (rows; + %lld B of row ids)\n",
           (long long)(rows * 512), ms, rows * 512 / ms / 1e9, (long long)(rows * 4));
    const int64_t ng = 40000000;
    const int64_t mall_rows = (128ll << 20) / 256, l2_rows = (2ll << 20) / 256;
    ms = timed([&] { calib_gather_hot<256, 16><<<grid, 256>>>(table, mall_rows, ng, out); }, reps);
    printf("hot_mall  gathered_bytes %lld unique_bytes %lld  %.3f ms  %.2f TB/s\n", (long long)(ng * 256),
           (long long)(mall_rows * 256), ms, ng * 256 / ms / 1e9);
    ms = timed([&] { calib_gather_hot<256, 16><<<grid, 256>>>(table, l2_rows, ng, out); }, reps);
    printf("hot_l2    gathered_bytes %lld unique_bytes %lld  %.3f ms  %.2f TB/s\n", (long long)(ng * 256),
           (long long)(l2_rows * 256), ms, ng * 256 / ms / 1e9);
    // gather ceiling by table size (uniform random 256-B rows), timing only
    for (int64_t mb = 1; mb <= 4096; mb *= 2) {
        const int64_t r = (mb << 20) / 256;
        ms = timed([&] { calib_gather_hot<256, 16><<<grid, 256>>>(table, r, ng, out); }, reps);
        printf("sweep_256 table_MiB %lld  %.3f ms  %.2f TB/s\n", (long long)mb, ms, ng * 256 / ms / 1e9);
    }
    for (int64_t mb = 1; mb <= 4096; mb *= 4) {
        const int64_t r = (mb << 20) / 512;
        ms = timed([&] { calib_gather_hot<512, 8><<<grid, 256>>>(table, r, ng / 2, out); }, reps);
        printf("sweep_512 table_MiB %lld  %.3f ms  %.2f TB/s\n", (long long)mb, ms, ng / 2 * 512 / ms / 1e9);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(table));
    CK(hipFree(perm));
    CK(hipFree(out));
    printf("done\n");
    return 0;
}
