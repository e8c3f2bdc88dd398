// Whole-chip rate of the FP4 block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (cbsz = blgp = 4) in the
// headline kernel's pattern, beside the I8 form it would replace: per 32-row tile of 256-bit keys a
// dependent chain of 4 FP4 MFMAs (K = 64 each) against 8 I8 MFMAs (K = 32), optionally followed by the
// top-2 update (float min3 / med3 / min on the FP4 path's float keys).
//   mode 0: chains only;  1: + update on floats (fminf / med3 as written);  3: + update on the keys' bit
//   patterns with integer min3 / med3 (the form k_top2_fp4 uses since late r05);  4: that update alone, no
//   MFMA (the accumulators are opaque registers rewritten by an empty asm each iteration);  5: the chain with
//   the update's 28 ops on registers no MFMA writes (does VALU issue overlap a wave's own MFMAs?);  6: waves
//   specialised per SIMD, even waves the chain only, odd waves the update only (across waves?)
// 1024-thread workgroups (16 waves, 4 per SIMD), G = 1024 workgroups.  Random-ish operands: the clock the
// chip holds depends on the data, so both forms get nonzero patterns.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_fp4_rate.hip -o mfma_fp4_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float med3f(float a, float b, float c) { return fmaxf(fminf(a, b), fminf(fmaxf(a, b), c)); }
__device__ __forceinline__ int med3(int a, int b, int c) { return max(min(a, b), min(max(a, b), c)); }

template <int MODE>
__global__ __launch_bounds__(1024) void k_fp4(float *out, int iters)
{
    const int l = threadIdx.x & 63;
    i32x8 a[4], b[4];
    for (int s = 0; s < 4; s++)
        for (int r = 0; r < 8; r++) {
            // nibbles from {0x0, 0xC} (train: 0 / -2) and {0x2, 0xA} (query: +1 / -1)
            const unsigned x = (unsigned)(l * 2654435761u + s * 40503u + r * 977u);
            a[s][r] = r < 4 ? (int)((x & 0x44444444u) * 3u) : 0;
            b[s][r] = r < 4 ? (int)(0x22222222u | ((x >> 1) & 0x88888888u)) : 0;
        }
    f32x16 c;
    for (int i = 0; i < 16; i++) c[i] = (float)(i + l);
    float k1 = 3e38f, k2 = 3e38f, k3 = 3e38f, k4 = 3e38f;
    f32x16 accp = c;
    for (int it = 0; it < iters; it++) {
        for (int s = 0; s < 4; s++) asm volatile("" : "+v"(a[s]));
        f32x16 acc;
        if (MODE == 4 || (MODE == 6 && (threadIdx.x >> 6) % 2 == 1)) {
            acc = accp;
            asm volatile("" : "+v"(acc));
        } else {
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[0], b[0], c, 4, 4, 0, 139, 0, 127);
#pragma unroll
            for (int s = 1; s < 4; s++)
                acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[s], b[s], acc, 4, 4, 0, 139, 0, 127);
        }
        if (MODE == 5) {
            f32x16 z = c;
            asm volatile("" : "+v"(z));
            int j1 = __float_as_int(k1), j2 = __float_as_int(k2), j3 = __float_as_int(k3), j4 = __float_as_int(k4);
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const int x = __float_as_int(z[i]), y = __float_as_int(z[i + 1]);
                const int u = __float_as_int(z[i + 8]), v = __float_as_int(z[i + 9]);
                int m = med3(j1, x, y);
                j1 = min(min(j1, x), y);
                j2 = min(m, j2);
                m = med3(j3, u, v);
                j3 = min(min(j3, u), v);
                j4 = min(m, j4);
            }
            k1 = __int_as_float(j1 - 32); k2 = __int_as_float(j2 - 32);
            k3 = __int_as_float(j3 - 32); k4 = __int_as_float(j4 - 32);
            // keep every iteration's chain live (r05's first build of this mode let the compiler sink the
            // chain out of the loop, so it timed the update alone)
            asm volatile("" : : "v"(acc));
        } else if (MODE == 3 || MODE == 4 || (MODE == 6 && (threadIdx.x >> 6) % 2 == 1)) {
            int j1 = __float_as_int(k1), j2 = __float_as_int(k2), j3 = __float_as_int(k3), j4 = __float_as_int(k4);
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const int x = __float_as_int(accp[i]), y = __float_as_int(accp[i + 1]);
                const int u = __float_as_int(accp[i + 8]), v = __float_as_int(accp[i + 9]);
                int m = med3(j1, x, y);
                j1 = min(min(j1, x), y);
                j2 = min(m, j2);
                m = med3(j3, u, v);
                j3 = min(min(j3, u), v);
                j4 = min(m, j4);
            }
            k1 = __int_as_float(j1 - 32); k2 = __int_as_float(j2 - 32);
            k3 = __int_as_float(j3 - 32); k4 = __int_as_float(j4 - 32);
        } else if (MODE & 1) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                float m = med3f(k1, accp[i], accp[i + 1]);
                k1 = fminf(fminf(k1, accp[i]), accp[i + 1]);
                k2 = fminf(m, k2);
                m = med3f(k3, accp[i + 8], accp[i + 9]);
                k3 = fminf(fminf(k3, accp[i + 8]), accp[i + 9]);
                k4 = fminf(m, k4);
            }
            k1 -= 32.f; k2 -= 32.f; k3 -= 32.f; k4 -= 32.f;
        } else {
            k1 += acc[it & 15];
        }
        accp = acc;
    }
    out[blockIdx.x * 1024 + threadIdx.x] = k1 + k2 + k3 + k4 + accp[l & 15];
}

// 7: two tiles per iteration with two accumulator sets (no copy): the update of each tile's results runs
//    while the other tile's chain is in flight, reading MFMA results one chain old;  8: 7 with each MFMA's
//    A operand read from LDS (ds_read_b128 per MFMA, as k_top2_fp4's K-steps)
__device__ __forceinline__ void upd_bits(int &j1, int &j2, int &j3, int &j4, const f32x16 &v)
{
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        const int x = __float_as_int(v[i]), y = __float_as_int(v[i + 1]);
        const int u = __float_as_int(v[i + 8]), w = __float_as_int(v[i + 9]);
        int m = med3(j1, x, y);
        j1 = min(min(j1, x), y);
        j2 = min(m, j2);
        m = med3(j3, u, w);
        j3 = min(min(j3, u), w);
        j4 = min(m, j4);
    }
    j1 -= 32; j2 -= 32; j3 -= 32; j4 -= 32;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_fp4pp(float *out, int iters)
{
    const int l = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) int s_a[16][64][4];
    i32x8 a[4], b[4];
    for (int s = 0; s < 4; s++)
        for (int r = 0; r < 8; r++) {
            const unsigned x = (unsigned)(l * 2654435761u + s * 40503u + r * 977u);
            a[s][r] = r < 4 ? (int)((x & 0x44444444u) * 3u) : 0;
            b[s][r] = r < 4 ? (int)(0x22222222u | ((x >> 1) & 0x88888888u)) : 0;
        }
    for (int s = 0; s < 4; s++)
        for (int r = 0; r < 4; r++) s_a[(threadIdx.x >> 6) % 16][l][r] = a[s][r];
    __syncthreads();
    const int *sa = &s_a[(threadIdx.x >> 6) % 16][l][0];
    f32x16 c;
    for (int i = 0; i < 16; i++) c[i] = (float)(8388608 + i + l);
    int j1 = 0x7fffffff, j2 = j1, j3 = j1, j4 = j1;
    f32x16 accA = c, accB = c;
    auto chain = [&](f32x16 &acc) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            i32x8 av = a[s];
            if (MODE == 8) {
                const i32x4 v = *(const i32x4 *)(sa + 0);
                av = i32x8{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                asm volatile("" : "+v"(av));
            }
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, b[s], s ? acc : c, 4, 4, 0, 139, 0, 127);
        }
    };
    for (int it = 0; it < iters; it += 2) {
        for (int s = 0; s < 4; s++) asm volatile("" : "+v"(a[s]));
        chain(accA);
        upd_bits(j1, j2, j3, j4, accB);
        for (int s = 0; s < 4; s++) asm volatile("" : "+v"(a[s]));
        chain(accB);
        upd_bits(j1, j2, j3, j4, accA);
    }
    out[blockIdx.x * 1024 + threadIdx.x] = (float)(j1 + j2 + j3 + j4) + accA[l & 15] + accB[l & 15];
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_i8(float *out, int iters)
{
    const int l = threadIdx.x & 63;
    i32x4 a[8], b[8];
    for (int s = 0; s < 8; s++) {
        const unsigned x = (unsigned)(l * 2654435761u + s * 40503u);
        a[s] = i32x4{(int)(x & 0x80808080u), (int)((x >> 1) & 0x80808080u), (int)((x >> 2) & 0x80808080u),
                     (int)((x >> 3) & 0x80808080u)};
        b[s] = i32x4{(int)(0x40404040u | (x & 0x80808080u)), (int)(0x40404040u | ((x << 1) & 0x80808080u)),
                     (int)(0x40404040u | ((x << 2) & 0x80808080u)), (int)(0x40404040u | ((x << 3) & 0x80808080u))};
    }
    i32x16 c;
    for (int i = 0; i < 16; i++) c[i] = i + l;
    int k1 = 0x7fffffff, k2 = 0x7fffffff, k3 = 0x7fffffff, k4 = 0x7fffffff;
    i32x16 accp = c;
    for (int it = 0; it < iters; it++) {
        for (int s = 0; s < 8; s++) asm volatile("" : "+v"(a[s]));
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
    out[blockIdx.x * 1024 + threadIdx.x] = (float)(k1 + k2 + k3 + k4 + accp[l & 15]);
}

template <class K>
double run(K kern, float *d, int iters, int G)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(G), dim3(1024), 0, 0, d, iters);
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(G), dim3(1024), 0, 0, d, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    const int G = 1024, iters = 256;
    float *d;
    (void)hipMalloc(&d, sizeof(float) * G * 1024);
    // one tile = 32 rows x 32 queries x 256 bits: 262144 (query, row, bit) MACs
    const double tiles = (double)G * 16 * iters;
    const double ms[10] = {run(k_i8<0>, d, iters, G), run(k_i8<1>, d, iters, G), run(k_fp4<0>, d, iters, G),
                           run(k_fp4<1>, d, iters, G), run(k_fp4<3>, d, iters, G), run(k_fp4<4>, d, iters, G),
                           run(k_fp4<5>, d, iters, G), run(k_fp4<6>, d, iters, G), run(k_fp4pp<7>, d, iters, G),
                           run(k_fp4pp<8>, d, iters, G)};
    const char *nm[10] = {"i8 chain", "i8 chain + update", "fp4 chain", "fp4 chain + float update",
                         "fp4 chain + integer update on the bit patterns", "integer update alone (no MFMA)",
                         "fp4 chain + the update on registers no MFMA writes",
                         "even waves fp4 chain only, odd waves integer update only",
                         "two accumulator sets, the update one chain behind (no copies)",
                         "two accumulator sets, + the A operand from LDS per MFMA"};
    for (int m = 0; m < 10; m++)
        printf("{\"mode\": \"%s\", \"ms\": %.4f, \"ns_per_tile_per_simd\": %.3f, \"Tmatch_bits_per_s\": %.1f}\n", nm[m],
               ms[m], ms[m] * 1e6 / (tiles / 1024), tiles * 262144 / (ms[m] * 1e-3) / 1e12);
    (void)hipFree(d);
    return 0;
}
