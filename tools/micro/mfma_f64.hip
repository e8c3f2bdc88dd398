// FP64 MFMA on gfx950: operand layout of v_mfma_f64_4x4x4f64 (4 blocks) found by probing, and the
// whole-chip rate of v_mfma_f64_4x4x4f64 / v_mfma_f64_16x16x4f64 / v_fma_f64.
//   Layout: A[lane] = lane + 1, B one-hot at lane q; D[l] != 0 names the A lane that meets B lane q
//   in output lane l (so: which lanes share a block, row and column).
//   Rate: 4 independent accumulator chains per wave, full occupancy, N_IT iterations.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_f64.hip -o mfma_f64
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout4(double *out)
{  // out[q * 64 + l] = D[l] for B one-hot at lane q
    const int l = threadIdx.x;
    for (int q = 0; q < 64; q++) {
        const double a = l + 1.0, b = (l == q) ? 1.0 : 0.0;
        double d = 0.0;
        d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d, 0, 0, 0);
        out[q * 64 + l] = d;
    }
}

__global__ void k_layout16(double *out)
{  // out[(q * 64 + l) * 4 + r] = D[l][r] for B one-hot at lane q
    const int l = threadIdx.x;
    for (int q = 0; q < 64; q++) {
        const double a = l + 1.0, b = (l == q) ? 1.0 : 0.0;
        d4 d = {0, 0, 0, 0};
        d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
        for (int r = 0; r < 4; r++) out[(q * 64 + l) * 4 + r] = d[r];
    }
}

constexpr int N_IT = 2048;

__global__ __launch_bounds__(256) void k_rate4(double *out, double s)
{
    double a = threadIdx.x * 1e-3, b = s;
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < N_IT; i++) {
        c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
}

__global__ __launch_bounds__(256) void k_rate16(double *out, double s)
{
    double a = threadIdx.x * 1e-3, b = s;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < N_IT; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ __launch_bounds__(256) void k_ratefma(double *out, double s)
{
    double x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 1e-3 + u;
    for (int i = 0; i < N_IT; i++)
#pragma unroll
        for (int u = 0; u < 8; u++) x[u] = __builtin_fma(x[u], s, 1e-9);
    double r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main()
{
    double *d;
    const int NB = 4096;
    hipMalloc(&d, sizeof(double) * NB * 256 + sizeof(double) * 64 * 64 * 4);
    std::vector<double> h(64 * 64 * 4);
    hipLaunchKernelGGL(k_layout4, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h.data(), d, sizeof(double) * 64 * 64, hipMemcpyDeviceToHost);
    printf("4x4x4f64 layout: for B lane q, the output lanes l with D[l] = A[lane a] (printed l:a)\n");
    for (int q = 0; q < 64; q++) {
        printf("q=%2d:", q);
        for (int l = 0; l < 64; l++)
            if (h[q * 64 + l] != 0) printf(" %d:%d", l, (int)h[q * 64 + l] - 1);
        printf("\n");
    }
    hipLaunchKernelGGL(k_layout16, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h.data(), d, sizeof(double) * 64 * 64 * 4, hipMemcpyDeviceToHost);
    printf("16x16x4f64 layout: for B lane q, (l,r):a\n");
    for (int q = 0; q < 64; q += 17) {
        printf("q=%2d:", q);
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 4; r++)
                if (h[(q * 64 + l) * 4 + r] != 0) printf(" (%d,%d):%d", l, r, (int)h[(q * 64 + l) * 4 + r] - 1);
        printf("\n");
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K {
        const char *name;
        void (*f)(double *, double);
        double fma_per_wave_iter;
    } ks[] = {{"v_mfma_f64_4x4x4f64", k_rate4, 4 * 256.0},
              {"v_mfma_f64_16x16x4f64", k_rate16, 4 * 1024.0},
              {"v_fma_f64", k_ratefma, 8 * 64.0}};
    for (auto &k : ks) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(NB), dim3(256), 0, 0, d, 1.0000001);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double fma = k.fma_per_wave_iter * N_IT * (NB * 4.0);
            if (rep) printf("%-24s %8.3f ms  %7.2f TFLOP/s (FP64, 2 per FMA)\n", k.name, ms, 2 * fma / ms / 1e9);
        }
    }
    return 0;
}
