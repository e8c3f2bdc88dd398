// row_newbcast semantics probe: out[j][lane] = update_dpp(row_newbcast:j) of in[lane] = lane
#include <hip/hip_runtime.h>
#include <cstdio>
template <int J>
__device__ int bc(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x150 + J, 0xF, 0xF, false); }
__global__ void k(int *out)
{
    const int l = threadIdx.x;
    const int v = 100 + l;
    out[0 * 64 + l] = bc<0>(v);
    out[1 * 64 + l] = bc<1>(v);
    out[2 * 64 + l] = bc<5>(v);
}
int main()
{
    int *d, h[192];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int r = 0; r < 3; r++) {
        for (int l = 0; l < 64; l++) printf("%d ", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
