// FP4 (e2m1) block-scaled MFMA on gfx950: the A / B operand lane maps of
// v_mfma_scale_f32_32x32x64_f8f6f4 (cbsz = blgp = 4) found by testing hypotheses with exact data.
//   Random A (32 x 64) and B (64 x 32) with entries in {-2, -1, 0, 1, 2} are packed on the host by a
//   candidate map (lane l holds row / column l & 31 and 32 nibbles j of K; k = f(l >> 5, j); nibble j in
//   register j >> 3, at bit 4 (j & 7) or 4 ((j & 7) ^ 1)), one MFMA runs, and D (the standard 32x32
//   C/D map: column l & 31, row (i & 3) + 8 (i >> 2) + 4 (l >> 5)) is compared with the host product.
//   The E8M0 scales: 127 = 1.0; a run with scale_a = 139 checks the x 4096 scaling.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_fp4_layout.hip -o mfma_fp4_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_one(const int *a, const int *b, float *d, int sa, int sb)
{
    const int l = threadIdx.x;
    i32x8 av = {}, bv = {};
    for (int r = 0; r < 4; r++) {
        av[r] = a[l * 4 + r];
        bv[r] = b[l * 4 + r];
    }
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 4, 4, 0, sa, 0, sb);
    for (int i = 0; i < 16; i++) d[l * 16 + i] = c[i];
}

static unsigned code(int v)  // e2m1
{
    switch (v) {
    case 0: return 0x0;
    case 1: return 0x2;
    case -1: return 0xA;
    case 2: return 0x4;
    case -2: return 0xC;
    }
    abort();
}

static int kmap(int hyp, int h, int j)
{
    switch (hyp) {
    case 0: return 32 * h + j;
    case 1: return 16 * h + (j & 15) + 32 * (j >> 4);
    case 2: return 8 * h + (j & 7) + 16 * (j >> 3);
    default: return 4 * h + (j & 3) + 8 * (j >> 2);
    }
}

int main()
{
    srand(7);
    int A[32][64], B[64][32];
    for (int m = 0; m < 32; m++)
        for (int k = 0; k < 64; k++) A[m][k] = rand() % 5 - 2;
    for (int k = 0; k < 64; k++)
        for (int n = 0; n < 32; n++) B[k][n] = rand() % 5 - 2;
    double ref[32][32];
    for (int m = 0; m < 32; m++)
        for (int n = 0; n < 32; n++) {
            double s = 0;
            for (int k = 0; k < 64; k++) s += A[m][k] * B[k][n];
            ref[m][n] = s;
        }
    int *da, *db;
    float *dd;
    hipMalloc(&da, 64 * 4 * 4);
    hipMalloc(&db, 64 * 4 * 4);
    hipMalloc(&dd, 64 * 16 * 4);
    for (int hyp = 0; hyp < 4; hyp++)
        for (int swap = 0; swap < 2; swap++)
            for (int scaled = 0; scaled < 2; scaled++) {
                std::vector<int> pa(64 * 4, 0), pb(64 * 4, 0);
                for (int l = 0; l < 64; l++)
                    for (int j = 0; j < 32; j++) {
                        const int k = kmap(hyp, l >> 5, j), sh = 4 * (swap ? ((j & 7) ^ 1) : (j & 7));
                        pa[l * 4 + (j >> 3)] |= (int)(code(A[l & 31][k]) << sh);
                        pb[l * 4 + (j >> 3)] |= (int)(code(B[k][l & 31]) << sh);
                    }
                hipMemcpy(da, pa.data(), pa.size() * 4, hipMemcpyHostToDevice);
                hipMemcpy(db, pb.data(), pb.size() * 4, hipMemcpyHostToDevice);
                hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, da, db, dd, scaled ? 139 : 127, 127);
                std::vector<float> h(64 * 16);
                hipMemcpy(h.data(), dd, h.size() * 4, hipMemcpyDeviceToHost);
                int bad = 0;
                for (int l = 0; l < 64; l++)
                    for (int i = 0; i < 16; i++) {
                        const int n = l & 31, m = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
                        if ((double)h[l * 16 + i] != ref[m][n] * (scaled ? 4096.0 : 1.0)) bad++;
                    }
                printf("hyp %d swap %d scale_a %d: %d of 1024 outputs differ\n", hyp, swap, scaled ? 139 : 127, bad);
            }
    hipFree(da);
    hipFree(db);
    hipFree(dd);
    return 0;
}
