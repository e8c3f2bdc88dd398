// Operand layout of v_mfma_i32_16x16x64_i8 on gfx950, found by probing (as mfma_i8.hip for 32x32x32):
// A slot (lane la, byte ja) set to 1, B bytes = (lane + 1) in pass 0 and (byte + 1) in pass 1; every
// nonzero D[lane][reg] then names the B slot holding B[k0][n] for the A slot's (m0, k0).  Prints one
// line per A slot: "la ja : (dl,di,bl,bj) ..." for all nonzero outputs.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_16_layout.hip -o mfma_i8_16_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(int *out)
{  // out[((slot * 2 + pass) * 64 + l) * 4 + i] = D[l][i]
    const int l = threadIdx.x;
    for (int slot = 0; slot < 1024; slot++) {
        const int la = slot / 16, ja = slot % 16;
        for (int pass = 0; pass < 2; pass++) {
            i32x4 a = {0, 0, 0, 0}, b;
            if (l == la) a[ja / 4] = 1 << (8 * (ja % 4));
            for (int w = 0; w < 4; w++) {
                unsigned v = 0;
                for (int y = 0; y < 4; y++) v |= (unsigned)(pass == 0 ? l + 1 : 4 * w + y + 1) << (8 * y);
                b[w] = (int)v;
            }
            i32x4 d = {0, 0, 0, 0};
            d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, d, 0, 0, 0);
            for (int i = 0; i < 4; i++) out[((slot * 2 + pass) * 64 + l) * 4 + i] = d[i];
        }
    }
}

int main()
{
    const size_t n = 1024 * 2 * 64 * 4;
    int *d;
    (void)hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d);
    std::vector<int> h(n);
    (void)hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    for (int slot = 0; slot < 1024; slot++) {
        printf("%d %d :", slot / 16, slot % 16);
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 4; i++) {
                const int v0 = h[((slot * 2 + 0) * 64 + l) * 4 + i], v1 = h[((slot * 2 + 1) * 64 + l) * 4 + i];
                if (v0) printf(" %d,%d,%d,%d", l, i, v0 - 1, v1 - 1);
            }
        printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
