// Development: the attainable bf16 MFMA rate on this device -- back-to-back
// v_mfma_f32_32x32x16_bf16 on random register operands, every CU, 8 waves per CU (the scoring
// kernel's occupancy), four independent accumulators per wave, operand bits flipped every
// iteration, no memory traffic in the loop; ~3 s of back-to-back launches so the clock settles.
//   make -C tools mfma_peak && tools/mfma_peak
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void mfma_loop(float* out, int iters, unsigned seed) {
    unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (__bf16)((float)(rnd() & 0xffff) / 65536.0f - 0.5f);
        b[i] = (__bf16)((float)(rnd() & 0xffff) / 65536.0f - 0.5f);
    }
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    for (int it = 0; it < iters; ++it) {
        // fresh operand bits every iteration (random-data switching, as in the scoring kernel)
        a = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, a) ^ 0x00450045u);
        b = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, b) ^ 0x00230023u);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


// same operand traffic, v_mfma_f32_16x16x32_bf16: 2x the instructions for the same FLOPs
__global__ __launch_bounds__(512) void mfma_loop16(float* out, int iters, unsigned seed) {
    unsigned x = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (__bf16)((float)(rnd() & 0xffff) / 65536.0f - 0.5f);
        b[i] = (__bf16)((float)(rnd() & 0xffff) / 65536.0f - 0.5f);
    }
    f32x4 c[8] = {};
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    for (int it = 0; it < iters; ++it) {
        a = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, a) ^ 0x00450045u);
        b = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, b) ^ 0x00230023u);
        c[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[0], 0, 0, 0);
        c[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c[1], 0, 0, 0);
        c[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c[2], 0, 0, 0);
        c[3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, c[3], 0, 0, 0);
        c[4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[4], 0, 0, 0);
        c[5] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c[5], 0, 0, 0);
        c[6] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, a, c[6], 0, 0, 0);
        c[7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, b, c[7], 0, 0, 0);
    }
    float s = 0.f;
    for (int j = 0; j < 8; ++j) for (int i = 0; i < 4; ++i) s += c[j][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount, threads = 512, iters = 400000;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    mfma_loop<<<blocks, threads>>>(out, 1000, 1);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 4; ++rep) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int j = 0; j < 10; ++j) mfma_loop<<<blocks, threads>>>(out, iters, 7 + rep * 10 + j);
        (void)hipDeviceSynchronize();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double flops = 10.0 * blocks * (threads / 64) * (double)iters * 4 * (2.0 * 32 * 32 * 16);
        std::printf("bare bf16 MFMA loop 32x32x16, %d CUs x 8 waves: %.0f TF/s (%.2f s)\n", blocks, flops / s / 1e12, s);
    }
    mfma_loop16<<<blocks, threads>>>(out, 1000, 1);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 4; ++rep) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int j = 0; j < 10; ++j) mfma_loop16<<<blocks, threads>>>(out, iters, 7 + rep * 10 + j);
        (void)hipDeviceSynchronize();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double flops = 10.0 * blocks * (threads / 64) * (double)iters * 8 * (2.0 * 16 * 16 * 32);
        std::printf("bare bf16 MFMA loop 16x16x32, %d CUs x 8 waves: %.0f TF/s (%.2f s)\n", blocks, flops / s / 1e12, s);
    }
    return 0;
}
