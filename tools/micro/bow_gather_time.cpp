// bow_gather_time.cpp — CPU-only timing of the adapter's gathers for the C3 stages (bench infrastructure):
// BowKfF::assign (SearchByBoW's gather from the KeyFrame and the Frame) and PoseGather::assign, on the
// problem pool bench.py's C3 wall stage uses (tools/wall_probe.py c3_pool), B frames per batch as the wall
// bench builds them.  No GPU and no C-ABI call: this is the host cost the wall rate pays per frame.
//
//   bow_gather_time pool.arrays B REPS          (the C3 pool: BowKfF, PoseGather)
//   bow_gather_time pool.arrays B REPS c5       (the C5 pool: LastGather, MpsGather, PoseGather)
#include <chrono>
#include <deque>

#include "../../tests/adapter/driver_common.h"

namespace oa = osg_orbslam3;
using Clock = std::chrono::steady_clock;

int main(int argc, char **argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s pool.arrays B REPS\n", argv[0]);
        return 2;
    }
    const Arrays in = read_arrays(argv[1]);
    const int B = atoi(argv[2]), reps = atoi(argv[3]);
    const int n = get(in, "pool.n").p<int32_t>()[0];
    if (argc > 4 && std::string(argv[4]) == "c5") {
        std::deque<Frame> Fl(n), LF(n), Fm(n), Fp5(n);
        std::deque<std::vector<MapPoint *>> Q(n);
        std::deque<Camera> c5(n), c25(n);
        std::vector<std::unique_ptr<MapPoint>> mp5;
        for (int i = 0; i < n; i++) {
            const std::string pre = "p" + std::to_string(i) + ".";
            build_last_problem(in, pre, Fl[i], LF[i], mp5);
            Fl[i].tlc_z_value = 0.f;
            build_mps_problem(in, pre, Fm[i], Q[i], mp5);
            build_pose_problem(in, pre, Fp5[i], c5[i], c25[i], mp5);
        }
        std::deque<Frame> fl, fm, fp5;
        std::vector<const Frame *> lfs;
        std::vector<const std::vector<MapPoint *> *> qs;
        for (int b = 0; b < B; b++) {
            fl.push_back(Fl[b % n]);
            fm.push_back(Fm[b % n]);
            fp5.push_back(Fp5[b % n]);
            lfs.push_back(&LF[b % n]);
            qs.push_back(&Q[b % n]);
        }
        double tl = 0, tm = 0, tp = 0;
        for (int r = 0; r < reps + 1; r++) {
            auto t0 = Clock::now();
            auto &gl = oa::gather_pool<oa::LastGather<MockHooks, Frame>>(B);
            for (int b = 0; b < B; b++) gl[b].assign(fl[b], *lfs[b]);
            auto t1 = Clock::now();
            auto &gm = oa::gather_pool<oa::MpsGather<Frame, MapPoint>>(B);
            for (int b = 0; b < B; b++) gm[b].assign(fm[b], *qs[b]);
            auto t2 = Clock::now();
            auto &gp = oa::gather_pool<oa::PoseGather<MockHooks, Frame>>(B);
            for (int b = 0; b < B; b++) gp[b].assign(&fp5[b], (oa::NoMutex *)nullptr);
            auto t3 = Clock::now();
            if (r == 0) continue;
            tl += std::chrono::duration<double>(t1 - t0).count();
            tm += std::chrono::duration<double>(t2 - t1).count();
            tp += std::chrono::duration<double>(t3 - t2).count();
        }
        if (getenv("OSG_GATHER_PARTS")) {  // FrameView and Slots of the LastF problem's current frame, alone
            std::deque<oa::FrameView<Frame>> fv(B);
            std::deque<oa::Slots<MapPoint>> sl(B);
            double a0 = 0, a1 = 0;
            for (int r = 0; r < reps + 1; r++) {
                auto t0 = Clock::now();
                for (int b = 0; b < B; b++) fv[b].assign(fl[b]);
                auto t1 = Clock::now();
                for (int b = 0; b < B; b++) sl[b].assign(fl[b].mvpMapPoints, lfs[b]->N, true);
                auto t2 = Clock::now();
                if (r == 0) continue;
                a0 += std::chrono::duration<double>(t1 - t0).count();
                a1 += std::chrono::duration<double>(t2 - t1).count();
            }
            std::printf("{\"frameview_us\": %.3f, \"slots_us\": %.3f}\n", a0 / B / reps * 1e6, a1 / B / reps * 1e6);
#ifndef GT_ORIG
            double a2 = 0, a3 = 0;
            std::vector<int32_t> gs, gi;
            std::vector<float> kx(4096), ka(4096);
            for (int r = 0; r < reps + 1; r++) {
                auto t0 = Clock::now();
                for (int b = 0; b < B; b++) {
                    oa::grid_csr(fl[b].mGrid, gs, gi, (size_t)(fl[b].Nleft == -1 ? fl[b].N : fl[b].Nleft));
                    if (fl[b].Nleft != -1) oa::grid_csr(fl[b].mGridRight, gs, gi, (size_t)(fl[b].N - fl[b].Nleft));
                }
                auto t1 = Clock::now();
                for (int b = 0; b < B; b++) {
                    const Frame &F = fl[b];
                    const int nl = F.Nleft;
                    for (int i = 0; i < F.N; i++) {
                        const auto &kp = nl == -1 ? F.mvKeysUn[i] : (i < nl ? F.mvKeys[i] : F.mvKeysRight[i - nl]);
                        kx[i & 4095] = kp.pt.x;
                        ka[i & 4095] = kp.angle;
                    }
                }
                auto t2 = Clock::now();
                if (r == 0) continue;
                a2 += std::chrono::duration<double>(t1 - t0).count();
                a3 += std::chrono::duration<double>(t2 - t1).count();
            }
            std::printf("{\"grids_us\": %.3f, \"keypoints_us\": %.3f, \"kx\": %f}\n", a2 / B / reps * 1e6, a3 / B / reps * 1e6, (double)kx[7] + ka[9]);
#endif
        }
        const double nf = (double)B * reps;
        std::printf("{\"frames\": %.0f, \"last_gather_us_per_frame\": %.3f, \"mps_gather_us_per_frame\": %.3f, "
                    "\"pose_gather_us_per_frame\": %.3f}\n", nf, tl / nf * 1e6, tm / nf * 1e6, tp / nf * 1e6);
        return 0;
    }
    std::deque<KeyFrame> K(n);
    std::deque<Frame> Fb(n), Fp(n);
    std::deque<Camera> c(n), c2(n);
    std::vector<std::unique_ptr<MapPoint>> mps;
    for (int i = 0; i < n; i++) {
        build_bow_kf_f_problem(in, "p" + std::to_string(i) + ".", K[i], Fb[i], mps);
        build_pose_problem(in, "p" + std::to_string(i) + ".", Fp[i], c[i], c2[i], mps);
    }
    std::vector<KeyFrame *> kfs;
    std::deque<Frame> fb, fp;
    for (int b = 0; b < B; b++) {
        kfs.push_back(&K[b % n]);
        fb.push_back(Fb[b % n]);
        fp.push_back(Fp[b % n]);
    }
    double t_bow = 0, t_pose = 0;
    for (int r = 0; r < reps + 1; r++) {
        auto t0 = Clock::now();
        auto &g = oa::gather_pool<oa::BowKfF<KeyFrame, Frame, MapPoint>>(B);
        for (int b = 0; b < B; b++) g[b].assign(kfs[b], fb[b]);
        auto t1 = Clock::now();
        auto &gp = oa::gather_pool<oa::PoseGather<MockHooks, Frame>>(B);
        for (int b = 0; b < B; b++) gp[b].assign(&fp[b], (oa::NoMutex *)nullptr);
        auto t2 = Clock::now();
        if (r == 0) continue;  // warm the pools
        t_bow += std::chrono::duration<double>(t1 - t0).count();
        t_pose += std::chrono::duration<double>(t2 - t1).count();
    }
    // the parts of BowKfF::assign, each over the whole batch (OSG_GATHER_PARTS=1)
    if (getenv("OSG_GATHER_PARTS")) {
        auto &g = oa::gather_pool<oa::BowKfF<KeyFrame, Frame, MapPoint>>(B);
        double tp[5] = {0, 0, 0, 0, 0};
        for (int r = 0; r < reps; r++) {
            auto a = Clock::now();
            for (int b = 0; b < B; b++) g[b].vpMPsKF = kfs[b]->GetMapPointMatches();
            auto b1 = Clock::now();
            for (int b = 0; b < B; b++) g[b].fk.assign(kfs[b]->mFeatVec);
            auto b2 = Clock::now();
            for (int b = 0; b < B; b++) g[b].ff.assign(fb[b].mFeatVec);
            auto b3 = Clock::now();
            for (int b = 0; b < B; b++) {
                auto &G = g[b];
                KeyFrame *pKF = kfs[b];
                const int nk = (int)G.vpMPsKF.size();
                G.good.resize(nk);
                G.ak.resize(nk);
                G.idk.assign(nk, -1);
                for (int i = 0; i < nk; i++) {
                    G.ak[i] = pKF->mvKeysUn[i].angle;
                    G.good[i] = G.vpMPsKF[i] && !G.vpMPsKF[i]->isBad();
                    if (G.vpMPsKF[i]) G.idk[i] = i;
                }
            }
            auto b4 = Clock::now();
            for (int b = 0; b < B; b++) {
                auto &G = g[b];
                const int nf = fb[b].N;
                G.af.resize(nf);
                for (int i = 0; i < nf; i++) G.af[i] = fb[b].mvKeysUn[i].angle;
            }
            auto b5 = Clock::now();
            tp[0] += std::chrono::duration<double>(b1 - a).count();
            tp[1] += std::chrono::duration<double>(b2 - b1).count();
            tp[2] += std::chrono::duration<double>(b3 - b2).count();
            tp[3] += std::chrono::duration<double>(b4 - b3).count();
            tp[4] += std::chrono::duration<double>(b5 - b4).count();
        }
        const double nfr = (double)B * reps;
        std::printf("{\"mp_copy\": %.3f, \"featvec_kf\": %.3f, \"featvec_f\": %.3f, \"kf_loop\": %.3f, \"f_loop\": %.3f}\n",
                    tp[0] / nfr * 1e6, tp[1] / nfr * 1e6, tp[2] / nfr * 1e6, tp[3] / nfr * 1e6, tp[4] / nfr * 1e6);
    }
    const double nf = (double)B * reps;
    std::printf("{\"frames\": %.0f, \"bow_gather_us_per_frame\": %.3f, \"pose_gather_us_per_frame\": %.3f}\n", nf,
                t_bow / nf * 1e6, t_pose / nf * 1e6);
    return 0;
}
