// Whole-chip VALU throughput of the instruction classes the Hamming kernels issue (v_xor_b32,
// v_bcnt_u32_b32, v_med3_u32) against v_add_f32 / v_fma_f32, 8 independent chains per lane, full
// occupancy (2048 workgroups x 1024 threads).  Prints wave-instructions per SIMD-cycle at the
// measured clock and lane-ops/s.  Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N_IT = 4096;

#define CHAINS8(OP)                                                                                 \
    _Pragma("unroll") for (int u = 0; u < 8; u++) OP;

__global__ __launch_bounds__(1024) void k_xor(uint32_t *out, uint32_t s)
{
    uint32_t x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 7u + u;
    for (int i = 0; i < N_IT; i++) {
        CHAINS8(asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[u]) : "s"(s + u)))
    }
    uint32_t r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

__global__ __launch_bounds__(1024) void k_bcnt(uint32_t *out, uint32_t s)
{
    uint32_t x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 7u + u;
    for (int i = 0; i < N_IT; i++) {
        CHAINS8(asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(x[u]) : "s"(s + u)))
    }
    uint32_t r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

__global__ __launch_bounds__(1024) void k_med3(uint32_t *out, uint32_t s)
{
    uint32_t x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 7u + u;
    for (int i = 0; i < N_IT; i++) {
        CHAINS8(asm volatile("v_med3_u32 %0, %1, %0, %0" : "+v"(x[u]) : "s"(s + u)))
    }
    uint32_t r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

__global__ __launch_bounds__(1024) void k_addf(uint32_t *out, uint32_t s)
{
    float x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 7.f + u;
    const float a = __uint_as_float(s & 0x3F800000u);
    for (int i = 0; i < N_IT; i++) {
        CHAINS8(asm volatile("v_add_f32 %0, %1, %0" : "+v"(x[u]) : "s"(a)))
    }
    float r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 1024 + threadIdx.x] = __float_as_uint(r);
}

__global__ __launch_bounds__(1024) void k_addu(uint32_t *out, uint32_t s)
{
    uint32_t x[8];
    for (int u = 0; u < 8; u++) x[u] = threadIdx.x * 7u + u;
    for (int i = 0; i < N_IT; i++) {
        CHAINS8(asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[u]) : "s"(s + u)))
    }
    uint32_t r = 0;
    for (int u = 0; u < 8; u++) r += x[u];
    out[blockIdx.x * 1024 + threadIdx.x] = r;
}

int main()
{
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const int grid = 8 * cus;  // 2 workgroups of 16 waves per CU at a time, 4 rounds
    uint32_t *out;
    hipMalloc(&out, sizeof(uint32_t) * 1024 * (size_t)grid);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K { const char *name; void (*f)(uint32_t *, uint32_t); };
    const K ks[] = {{"v_xor_b32", k_xor}, {"v_bcnt_u32_b32", k_bcnt}, {"v_med3_u32", k_med3},
                    {"v_add_u32", k_addu}, {"v_add_f32", k_addf}};
    for (const K &k : ks) {
        for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(1024), 0, 0, out, 3u);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int R = 5;
        for (int rep = 0; rep < R; rep++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(1024), 0, 0, out, 3u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double lane_ops = (double)R * grid * 1024 * N_IT * 8;
        const double s = ms * 1e-3;
        const double per_simd_cycle_at_2p4 = lane_ops / 64.0 / (cus * 4.0) / (s * 2.4e9);
        printf("%-16s %8.3f ms  %7.2f T lane-ops/s  %.3f wave-instr per SIMD-cycle at 2.4 GHz\n", k.name, ms,
               lane_ops / s / 1e12, per_simd_cycle_at_2p4);
    }
    hipFree(out);
    return 0;
}
