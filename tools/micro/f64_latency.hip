// Dependent-chain latency of FP64 VALU ops and LDS round trips on gfx950 (one wave), in shader
// cycles (s_memtime).  Build: hipcc --offload-arch=gfx950 -O3 f64_latency.hip -o f64_latency
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fma(double *out, long long *cyc, double a, double b, int n)
{
    double x = threadIdx.x * 1e-3;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 32)
#pragma unroll
        for (int u = 0; u < 32; u++) x = fma(x, a, b);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_add(double *out, long long *cyc, double a, int n)
{
    double x = threadIdx.x * 1e-3;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 32)
#pragma unroll
        for (int u = 0; u < 32; u++) x = x + a;
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_fma32(float *out, long long *cyc, float a, float b, int n)
{
    float x = threadIdx.x * 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 32)
#pragma unroll
        for (int u = 0; u < 32; u++) x = fmaf(x, a, b);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_lds(double *out, long long *cyc, int n)
{
    __shared__ double s[64];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    int idx = threadIdx.x;
    double acc = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const double v = s[idx];
            idx = ((int)v + 1) & 63;  // dependent address
            acc += v;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_bar(double *out, long long *cyc, int n)
{
    double x = 0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            __syncthreads();
            x += 1.0;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_rcp(double *out, long long *cyc, int n)
{
    double x = 1.0 + threadIdx.x * 1e-3;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 32)
#pragma unroll
        for (int u = 0; u < 32; u++) x = __builtin_amdgcn_rcp(x) + 1.0;
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void k_div(double *out, long long *cyc, int n)
{
    double x = 1.0 + threadIdx.x * 1e-3;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 32)
#pragma unroll
        for (int u = 0; u < 32; u++) x = 1.0 / x + 1.0;
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double *out; float *out32; long long *cyc, h;
    hipMalloc(&out, 1024 * 8); hipMalloc(&out32, 1024 * 4); hipMalloc(&cyc, 8);
    const int n = 4096;
    auto rep = [&](const char *name, int threads, auto launch) {
        for (int r = 0; r < 3; r++) launch(threads);
        hipDeviceSynchronize();
        hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-28s threads=%4d  %.1f cycles/iter\n", name, threads, (double)h / n);
    };
    for (int th : {64, 256, 1024}) {
        rep("fma_f64 chain", th, [&](int t) { hipLaunchKernelGGL(k_fma, dim3(1), dim3(t), 0, 0, out, cyc, 0.999, 1e-3, n); });
        rep("add_f64 chain", th, [&](int t) { hipLaunchKernelGGL(k_add, dim3(1), dim3(t), 0, 0, out, cyc, 1e-3, n); });
        rep("fma_f32 chain", th, [&](int t) { hipLaunchKernelGGL(k_fma32, dim3(1), dim3(t), 0, 0, out32, cyc, 0.999f, 1e-3f, n); });
        rep("rcp_f64+add chain", th, [&](int t) { hipLaunchKernelGGL(k_rcp, dim3(1), dim3(t), 0, 0, out, cyc, n); });
        rep("div_f64+add chain", th, [&](int t) { hipLaunchKernelGGL(k_div, dim3(1), dim3(t), 0, 0, out, cyc, n); });
        rep("syncthreads loop", th, [&](int t) { hipLaunchKernelGGL(k_bar, dim3(1), dim3(t), 0, 0, out, cyc, n); });
    }
    rep("lds dependent read", 64, [&](int t) { hipLaunchKernelGGL(k_lds, dim3(1), dim3(t), 0, 0, out, cyc, n); });
    return 0;
}
