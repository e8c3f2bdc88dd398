// Whole-chip rate of v_mfma_i32_16x16x64_i8 against v_mfma_i32_32x32x32_i8 in dependent chains of 8
// (the headline kernel's K-loop shape), 1024-thread workgroups, G = 4 x 256 workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_16.hip -o mfma_i8_16
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(1024) void k_rate(int *out, int iters)
{
    const int l = threadIdx.x & 63;
    i32x4 a[8], b[8];
    for (int s = 0; s < 8; s++) {
        a[s] = i32x4{l + s, l * 3 + s, l ^ s, s};
        b[s] = i32x4{l * 5 + s, l + 7 * s, 3 * l ^ s, 2 * s};
    }
    int k1 = 0;
    if (SHAPE == 32) {
        i32x16 c;
        for (int i = 0; i < 16; i++) c[i] = i + l;
        for (int it = 0; it < iters; it++) {
            for (int s = 0; s < 8; s++) asm volatile("" : "+v"(a[s]));
            i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], b[0], c, 0, 0, 0);
#pragma unroll
            for (int s = 1; s < 8; s++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[s], acc, 0, 0, 0);
            k1 ^= acc[it & 15];
        }
    } else if (SHAPE == 33) {  // two independent 32x32 chains of 4 (the same MACs as one chain of 8)
        i32x16 c0, c1;
        for (int i = 0; i < 16; i++) {
            c0[i] = i + l;
            c1[i] = i - l;
        }
        for (int it = 0; it < iters; it++) {
            for (int s = 0; s < 8; s++) asm volatile("" : "+v"(a[s]));
            i32x16 x = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], b[0], c0, 0, 0, 0);
            i32x16 y = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[4], b[4], c1, 0, 0, 0);
#pragma unroll
            for (int s = 1; s < 4; s++) {
                x = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[s], x, 0, 0, 0);
                y = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s + 4], b[s + 4], y, 0, 0, 0);
            }
            k1 ^= x[it & 15] + y[(it + 3) & 15];
        }
    } else {  // two independent 16x16 chains per 32x32 chain: the same MACs
        i32x4 c0 = {l, 1, 2, 3}, c1 = {3, 2, 1, l};
        for (int it = 0; it < iters; it++) {
            for (int s = 0; s < 8; s++) asm volatile("" : "+v"(a[s]));
            i32x4 x = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[0], b[0], c0, 0, 0, 0);
            i32x4 y = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[1], b[1], c1, 0, 0, 0);
#pragma unroll
            for (int s = 1; s < 8; s++) {
                x = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[s], b[s], x, 0, 0, 0);
                y = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[(s + 1) & 7], b[(s + 1) & 7], y, 0, 0, 0);
            }
            k1 ^= x[it & 3] + y[(it + 1) & 3];
        }
    }
    out[blockIdx.x * 1024 + threadIdx.x] = k1;
}

template <int SHAPE>
double run(int *d, int iters, int G)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<SHAPE>, dim3(G), dim3(1024), 0, 0, d, iters);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_rate<SHAPE>, dim3(G), dim3(1024), 0, 0, d, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    const int G = 1024, iters = 256;
    int *d;
    (void)hipMalloc(&d, sizeof(int) * G * 1024);
    const double macs = (double)G * 16 * iters * 8 * 32768;  // per launch, both forms
    const double m32 = run<32>(d, iters, G), m16 = run<16>(d, iters, G), m33 = run<33>(d, iters, G);
    printf("{\"form\": \"32x32x32 chains\", \"ms\": %.4f, \"TOPS\": %.1f}\n", m32, macs * 2 / (m32 * 1e-3) / 1e12);
    printf("{\"form\": \"16x16x64 chains (2 per 32x32)\", \"ms\": %.4f, \"TOPS\": %.1f}\n", m16, macs * 2 / (m16 * 1e-3) / 1e12);
    printf("{\"form\": \"32x32x32, two chains of 4\", \"ms\": %.4f, \"TOPS\": %.1f}\n", m33, macs * 2 / (m33 * 1e-3) / 1e12);
    (void)hipFree(d);
    return 0;
}
