// Whole-chip rate of v_mfma_i32_32x32x32_i8 in the headline kernel's pattern (k_top2_mfma): per tile a
// dependent chain of 8 MFMAs, optionally followed by the 1.5-op-per-key top-2 update (28 VALU) of the
// previous tile's accumulator, operands in registers (no LDS) or re-read from LDS per K-step.
//   mode 0: MFMA chains only;  1: + update;  2: + LDS A reads;  3: + update + LDS A reads
// 1024-thread workgroups (16 waves, 4 per SIMD), one per CU at a time, G = 4 x 256 workgroups.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_rate.hip -o mfma_i8_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int med3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

template <int MODE>
__global__ __launch_bounds__(1024) void k_rate(int *out, int iters)
{
    __shared__ i32x4 s_a[32 * 17];
    const int l = threadIdx.x & 63;
    i32x4 a[8], b[8];
    for (int s = 0; s < 8; s++) {
        a[s] = i32x4{l + s, l * 3 + s, l ^ s, s};
        b[s] = i32x4{l * 5 + s, l + 7 * s, 3 * l ^ s, 2 * s};
    }
    for (int i = threadIdx.x; i < 32 * 17; i += 1024) s_a[i] = i32x4{i, 2 * i, 3 * i, 4 * i};
    __syncthreads();
    i32x16 c;
    for (int i = 0; i < 16; i++) c[i] = i + l;
    int k1 = 0x7fffffff, k2 = 0x7fffffff, k3 = 0x7fffffff, k4 = 0x7fffffff;
    i32x16 accp = c;
    for (int it = 0; it < iters; it++) {
        if (MODE & 2) {
            for (int s = 0; s < 8; s++) a[s] = s_a[(l & 31) * 17 + 2 * s + (l >> 5) + (it & 1)];
        } else {
            for (int s = 0; s < 8; s++) asm volatile("" : "+v"(a[s]));
        }
        i32x16 acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[0], b[0], c, 0, 0, 0);
#pragma unroll
        for (int s = 1; s < 8; s++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s], b[s], acc, 0, 0, 0);
        if (MODE & 1) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                int m = med3(k1, accp[i], accp[i + 1]);
                k1 = min(min(k1, accp[i]), accp[i + 1]);
                k2 = min(m, k2);
                m = med3(k3, accp[i + 8], accp[i + 9]);
                k3 = min(min(k3, accp[i + 8]), accp[i + 9]);
                k4 = min(m, k4);
            }
            k1 -= 32; k2 -= 32; k3 -= 32; k4 -= 32;
        } else {
            k1 ^= acc[it & 15];
        }
        accp = acc;
    }
    out[blockIdx.x * 1024 + threadIdx.x] = k1 + k2 + k3 + k4 + accp[l & 15];
}

template <int MODE>
double run(int *d, int iters, int G)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_rate<MODE>, dim3(G), dim3(1024), 0, 0, d, iters);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_rate<MODE>, dim3(G), dim3(1024), 0, 0, d, iters);
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
    const double mfma = (double)G * 16 * iters * 8;  // MFMAs per launch
    const double per_simd = mfma / 1024;
    double ms[4] = {run<0>(d, iters, G), run<1>(d, iters, G), run<2>(d, iters, G), run<3>(d, iters, G)};
    const char *nm[4] = {"mfma only", "mfma + update", "mfma + lds A", "mfma + update + lds A"};
    for (int m = 0; m < 4; m++)
        printf("{\"mode\": \"%s\", \"ms\": %.4f, \"ns_per_mfma_per_simd\": %.3f, \"cycles_at_2.4GHz\": %.2f, \"TOPS\": %.1f}\n",
               nm[m], ms[m], ms[m] * 1e6 / per_simd, ms[m] * 1e-3 / per_simd * 2.4e9,
               mfma * 32768 * 2 / (ms[m] * 1e-3) / 1e12);
    (void)hipFree(d);
    return 0;
}
