// pose_edge_cost.hip — cycles of one PoseOptimization pass's per-edge work on one CU (8 waves), to
// locate k_pose_lat's pass cost: the buildSystem terms (error + Jacobian + 28 products) and the robust
// chi2 of one edge per lane, with the pose / camera in registers or read from LDS, and the 28-stream
// LDS tile writes.  Prints cycles (s_memtime, wave 0 lane 0) per variant, median of repetitions.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude tools/micro/pose_edge_cost.hip -o /tmp/pec \
//         -Lorb_slam3_comments_ghr_amd -lorbslam3_amd (the host entry points of pose.hip link against the library)
#include "../../orb_slam3_comments_ghr_amd/csrc/pose.hip"

#include <cstdio>

namespace {

template <int VAR>
__global__ __launch_bounds__(512) void k_cost(const int8_t *kind, const double *xw, const double *obs, const float *isig2,
                                              const double *pose7, osg_camera cam_in, unsigned long long *cyc, double *sink)
{
    __shared__ __attribute__((aligned(16))) double tile[8 * 29 * 66];
    __shared__ osg_camera cam_s;
    __shared__ SE3 T_s;
    __shared__ SE3 trl_s;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    if (threadIdx.x == 0) {
        cam_s = cam_in;
        T_s = se3_from7(pose7);
        trl_s = se3_from7(cam_in.trl);
    }
    __syncthreads();
    const PEdge E = load_edge(threadIdx.x, kind, xw, obs, isig2);
    const SE3 Treg = se3_from7(pose7);
    const SE3 trlreg = se3_from7(cam_in.trl);
    double *col = tile + wave * 29 * 66 + lane;
    double acc = 0;
    for (int rep = 0; rep < 8; rep++) {
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        const SE3 &T = (VAR & 1) ? T_s : Treg;
        const osg_camera &cam = (VAR & 1) ? cam_s : cam_in;
        const SE3 &Trl = (VAR & 1) ? trl_s : trlreg;
        if (VAR & 2) {  // robust chi2 only
            double ev[3];
            pose_edge_error(E, cam, cam, Trl, T, ev);
            const bool st = E.k == OSG_EDGE_STEREO;
            const double c = edge_chi2_of(ev, st, E.w);
            double v = c, r1;
            if (st) huber(c, 2.79, 7.815f, v, r1);
            else huber(c, 2.44, 5.991f, v, r1);
            col[0] = v;
        } else {
            double ev[3];
            pose_edge_error(E, cam, cam, Trl, T, ev);
            const bool st = E.k == OSG_EDGE_STEREO;
            const double chi = edge_chi2_of(ev, st, E.w);
            double r0 = chi, rho1 = 1.0;
            if (st) huber(chi, 2.79, 7.815f, r0, rho1);
            else huber(chi, 2.44, 5.991f, r0, rho1);
            col[27 * 66] = r0;
            double Jp[3][6];
            pose_edge_jac(E, cam, cam, Trl, T, Jp);
            const double ww = rho1 * E.w;
            int q = 0;
#pragma unroll
            for (int i = 0; i < 6; i++)
#pragma unroll
                for (int j = i; j < 6; j++) {
                    double h = 0;
                    h += Jp[0][i] * ww * Jp[0][j];
                    h += Jp[1][i] * ww * Jp[1][j];
                    if (st) h += Jp[2][i] * ww * Jp[2][j];
                    col[(q++) * 66] = h;
                }
#pragma unroll
            for (int i = 0; i < 6; i++) {
                double sb = 0;
                sb += rho1 * Jp[0][i] * (E.w * ev[0]);
                sb += rho1 * Jp[1][i] * (E.w * ev[1]);
                if (st) sb += rho1 * Jp[2][i] * (E.w * ev[2]);
                col[(21 + i) * 66] = -sb;
            }
        }
        __syncthreads();
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0) cyc[rep] = t1 - t0;
        acc += tile[threadIdx.x % 64];
    }
    sink[threadIdx.x] = acc;
}

}  // namespace

int main()
{
    const int n = 512;
    std::vector<int8_t> kind(n);
    std::vector<double> xw(3 * n), obs(3 * n);
    std::vector<float> isig(n, 1.0f);
    unsigned s = 12345;
    auto rnd = [&] { s = s * 1664525u + 1013904223u; return (s >> 8) / 16777216.0; };
    for (int i = 0; i < n; i++) {
        kind[i] = (i % 5 < 3) ? OSG_EDGE_STEREO : OSG_EDGE_MONO;
        const double z = 1 + 9 * rnd(), u = 20 + 700 * rnd(), v = 20 + 440 * rnd();
        xw[3 * i] = (u - 367) / 458 * z;
        xw[3 * i + 1] = (v - 248) / 457 * z;
        xw[3 * i + 2] = z;
        obs[3 * i] = u + rnd();
        obs[3 * i + 1] = v + rnd();
        obs[3 * i + 2] = u - 47.9 / z;
    }
    double pose[7] = {0.01, -0.02, 0.005, 0.9997, 0.1, 0.0, -0.05};
    osg_camera cam{};
    cam.type = OSG_CAM_PINHOLE;
    cam.fx = 458.654f;
    cam.fy = 457.296f;
    cam.cx = 367.215f;
    cam.cy = 248.375f;
    cam.bf = 47.9f;
    cam.trl[3] = 1.0;
    int8_t *dk;
    double *dx, *dobs, *dp, *dsink;
    float *di;
    unsigned long long *dc;
    hipMalloc(&dk, n);
    hipMalloc(&dx, 24 * n);
    hipMalloc(&dobs, 24 * n);
    hipMalloc(&di, 4 * n);
    hipMalloc(&dp, 56);
    hipMalloc(&dc, 8 * 8);
    hipMalloc(&dsink, 8 * 512);
    hipMemcpy(dk, kind.data(), n, hipMemcpyHostToDevice);
    hipMemcpy(dx, xw.data(), 24 * n, hipMemcpyHostToDevice);
    hipMemcpy(dobs, obs.data(), 24 * n, hipMemcpyHostToDevice);
    hipMemcpy(di, isig.data(), 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(dp, pose, 56, hipMemcpyHostToDevice);
    const char *names[4] = {"sys terms, pose+cam in registers", "sys terms, pose+cam in LDS",
                            "robust chi2, pose+cam in registers", "robust chi2, pose+cam in LDS"};
    for (int var = 0; var < 4; var++) {
        for (int threads : {512, 320, 64}) {
            unsigned long long c[8];
            switch (var) {
            case 0: hipLaunchKernelGGL(k_cost<0>, dim3(1), dim3(threads), 0, 0, dk, dx, dobs, di, dp, cam, dc, dsink); break;
            case 1: hipLaunchKernelGGL(k_cost<1>, dim3(1), dim3(threads), 0, 0, dk, dx, dobs, di, dp, cam, dc, dsink); break;
            case 2: hipLaunchKernelGGL(k_cost<2>, dim3(1), dim3(threads), 0, 0, dk, dx, dobs, di, dp, cam, dc, dsink); break;
            default: hipLaunchKernelGGL(k_cost<3>, dim3(1), dim3(threads), 0, 0, dk, dx, dobs, di, dp, cam, dc, dsink); break;
            }
            hipDeviceSynchronize();
            hipMemcpy(c, dc, 64, hipMemcpyDeviceToHost);
            std::sort(c, c + 8);
            std::printf("%-40s threads=%3d  %6llu cycles (median of 8; min %llu)\n", names[var], threads, c[4], c[0]);
        }
    }
    return 0;
}
