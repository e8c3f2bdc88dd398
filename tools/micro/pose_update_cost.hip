// pose_update_cost.hip — cycles (s_memtime, one wave) of the pieces of one PoseOptimization LM trial's
// update chain: the FP64 sqrt / divide / add latencies, sincos_ref, se3_exp, se3_mul and the whole
// se3_oplus, with the operands in registers.  Each variant runs a dependent chain of REPS calls (the
// next input depends on the last output) and reports cycles per call, median of 9 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude tools/micro/pose_update_cost.hip -o tools/micro/pose_update_cost
#include <algorithm>
#include <cstdio>

#include "../../orb_slam3_comments_ghr_amd/csrc/ba_common.h"

using namespace osgba;

constexpr int REPS = 64;

template <int VAR>
__global__ __launch_bounds__(64) void k_cost(const double *in, unsigned long long *cyc, double *sink)
{
    double x = in[threadIdx.x];
    double upd[6] = {in[1] * 1e-3, in[2] * 1e-3, in[3] * 1e-3, in[4] * 1e-2, in[5] * 1e-2, in[6] * 1e-2};
    SE3 T = se3_from7(in + 8);
    double acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int r = 0; r < REPS; r++) {
        if (VAR == 0) {  // dependent FP64 add
#pragma unroll
            for (int u = 0; u < 16; u++) x = x + 1e-3;
        } else if (VAR == 1) {  // dependent FP64 fma
#pragma unroll
            for (int u = 0; u < 16; u++) x = fma(x, 0.999, 1e-3);
        } else if (VAR == 2) {  // dependent sqrt
#pragma unroll
            for (int u = 0; u < 4; u++) x = sqrt(x + 1.0);
        } else if (VAR == 3) {  // dependent divide
#pragma unroll
            for (int u = 0; u < 4; u++) x = 1.5 / (x + 1.0);
        } else if (VAR == 4) {  // sincos_ref at a typical LM rotation magnitude
            double s, c;
            osgx::sincos_ref(1e-3 * (1.0 + 1e-3 * x), s, c);
            x += s + c;
        } else if (VAR == 5) {  // se3_exp
            upd[0] += 1e-9 * x;
            const SE3 E = se3_exp(upd);
            x += E.q[0] + E.t[0];
        } else if (VAR == 6) {  // se3_mul
            T.t[0] += 1e-9 * x;
            const SE3 E = se3_mul(T, T);
            x += E.q[0] + E.t[0];
        } else if (VAR == 7) {  // se3_oplus (the LM update)
            upd[0] += 1e-12 * x;
            se3_oplus(T, upd);
            x += T.q[0];
        } else if (VAR == 8) {  // cube_rn
            x = osgx::cube_rn(x * 0.5 + 0.5);
        } else if (VAR == 9) {  // sincos_ref with the argument uniform across the wave (PoseOptimization)
            double s, c;
            osgx::sincos_ref<true>(1e-3 * (1.0 + 1e-3 * __shfl(x, 0)), s, c);
            x += s + c;
        } else if (VAR == 10) {  // se3_oplus<true>
            upd[0] += 1e-12 * __shfl(x, 0);
            se3_oplus<true>(T, upd);
            x += T.q[0];
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    acc += x + T.q[1];
    sink[threadIdx.x] = acc;
}

template <int VAR>
double run(const double *din, unsigned long long *dc, double *dsink)
{
    unsigned long long c[9];
    for (int i = 0; i < 9; i++) {
        hipLaunchKernelGGL(k_cost<VAR>, dim3(1), dim3(64), 0, 0, din, dc, dsink);
        hipMemcpy(&c[i], dc, 8, hipMemcpyDeviceToHost);
    }
    std::sort(c, c + 9);
    return (double)c[4] / REPS;
}

int main()
{
    double in[64];
    for (int i = 0; i < 64; i++) in[i] = 0.3 + 0.01 * i;
    in[8] = 0.01; in[9] = -0.02; in[10] = 0.005; in[11] = 0.9997; in[12] = 0.1; in[13] = 0.0; in[14] = -0.05;
    double *din, *dsink;
    unsigned long long *dc;
    (void)hipMalloc(&din, sizeof(in));
    (void)hipMalloc(&dc, 8);
    (void)hipMalloc(&dsink, 8 * 64);
    (void)hipMemcpy(din, in, sizeof(in), hipMemcpyHostToDevice);
    std::printf("{\"fp64_add\": %.1f, \"fp64_fma\": %.1f, \"sqrt\": %.1f, \"div\": %.1f, \"sincos_ref\": %.1f, "
                "\"se3_exp\": %.1f, \"se3_mul\": %.1f, \"se3_oplus\": %.1f, \"cube_rn\": %.1f, \"sincos_ref_uniform\": %.1f, "
                "\"se3_oplus_uniform\": %.1f}\n",
                run<0>(din, dc, dsink) / 16, run<1>(din, dc, dsink) / 16, run<2>(din, dc, dsink) / 4,
                run<3>(din, dc, dsink) / 4, run<4>(din, dc, dsink), run<5>(din, dc, dsink), run<6>(din, dc, dsink),
                run<7>(din, dc, dsink), run<8>(din, dc, dsink), run<9>(din, dc, dsink), run<10>(din, dc, dsink));
    return 0;
}
