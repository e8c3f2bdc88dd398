// Probe: the largest dynamic LDS a 1024-thread kernel launches with on this device, with and
// without hipFuncAttributeMaxDynamicSharedMemorySize.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(1024) void k_touch(int n, int *out)
{
    extern __shared__ int sm[];
    for (int i = threadIdx.x; i < n; i += blockDim.x) sm[i] = i;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = sm[n - 1];
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n",
           p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.sharedMemPerBlockOptin);
    int *d;
    (void)hipMalloc(&d, 4096);
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            hipError_t e = hipFuncSetAttribute((const void *)k_touch, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            printf("set attribute: %s\n", hipGetErrorString(e));
        }
        for (int kb : {32, 60, 64, 65, 96, 128, 150, 156, 160}) {
            const size_t bytes = (size_t)kb * 1024;
            hipLaunchKernelGGL(k_touch, dim3(1), dim3(1024), bytes, 0, (int)(bytes / 4), d);
            hipError_t e = hipGetLastError();
            hipError_t s = hipDeviceSynchronize();
            printf("pass %d  %3d KiB: launch %s, sync %s\n", pass, kb, hipGetErrorString(e), hipGetErrorString(s));
        }
    }
    return 0;
}
