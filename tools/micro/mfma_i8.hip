// I8 MFMA on gfx950: operand layout of v_mfma_i32_32x32x32_i8 found by probing.
//   For every A slot (lane la, byte ja) set to 1 (all other A bytes 0), B filled with byte value
//   (lane + 1) in pass 0 and (byte + 1) in pass 1: D[row m0][col n] is then the B slot holding
//   B[k0][n], where (m0, k0) is the element that A slot carries.  Printed per A slot: the output
//   (lane, register) pairs that are nonzero for column 0 and 1, and the B (lane, byte) they name.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8.hip -o mfma_i8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k_probe(int *out)
{  // out[((slot * 2 + pass) * 64 + l) * 16 + i] = D[l][i]
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
            i32x16 d = {};
            d = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, d, 0, 0, 0);
            for (int i = 0; i < 16; i++) out[((slot * 2 + pass) * 64 + l) * 16 + i] = d[i];
        }
    }
}

int main()
{
    const size_t n = 1024 * 2 * 64 * 16;
    int *d;
    hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d);
    std::vector<int> h(n);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    // per A slot: the (D lane, D reg) entries that are nonzero and the B slot they name
    int same = 0, total = 0;
    for (int slot = 0; slot < 1024; slot++) {
        const int la = slot / 16, ja = slot % 16;
        printf("A(l=%2d,j=%2d):", la, ja);
        int shown = 0;
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 16; i++) {
                const int v0 = h[((slot * 2 + 0) * 64 + l) * 16 + i], v1 = h[((slot * 2 + 1) * 64 + l) * 16 + i];
                if (!v0) continue;
                const int bl = v0 - 1, bj = v1 - 1;
                total++;
                if (bj == ja && (bl >> 5) == (la >> 5)) same++;
                if (shown < 3) printf(" D(l=%d,i=%d)<-B(l=%d,j=%d)", l, i, bl, bj);
                shown++;
            }
        printf(" [%d nonzero]\n", shown);
    }
    printf("B slot with the same (lane half, byte) as the A slot: %d of %d products\n", same, total);
    hipFree(d);
    return 0;
}
