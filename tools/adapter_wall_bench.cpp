// adapter_wall_bench.cpp — the wall rate of the drop-in as ORB-SLAM3 runs it (bench infrastructure).
//
// Mock Frames, KeyFrames and MapPoints (tests/adapter/mock_orbslam3.h, the reference's member names)
// go through the batched entries of adapters/orbslam3/osg_orbslam3.h: the gather from the objects,
// the C-ABI call with host inputs (pack into pinned memory, upload, kernels, download) and the
// write-back into the objects, on T host threads with one osg_ctx (one HIP stream) each — T Tracking
// threads of independent sequences sharing one GPU (config C5 runs one sequence per thread).
//
//   adapter_wall_bench WORKLOAD pool.arrays B REPS THREADS        WORKLOAD: c3 c5 stereo dbow
//
//   c3      SearchByBoW(KF, F) then PoseOptimization (ref:src/Tracking.cc:3258-3300)
//   c5      SearchByProjection(F, LastF), SearchByProjection(F, local map), PoseOptimization on the
//           two-camera KannalaBrandt8 rig (ref:src/Tracking.cc:3482-3507, 3601-3640)
//   stereo  Frame::ComputeStereoMatches (ref:src/Frame.cc:1114-1290); the pyramid levels live in HBM,
//           built there by osg_orb_pyramid in the integrated ORBextractor, so no
//           pixels cross PCIe here: they are uploaded once before timing
//   dbow    Frame::ComputeBoW (ref:src/Frame.cc:995-1010)
//
// pool.arrays holds "pool.n" problems under "p0.", "p1.", ... (tools/adapter_arrays.py writes them,
// tests/adapter/driver_common.h reads them).  Thread t's frame b is a copy of problem (t*B + b) % n;
// KeyFrames, MapPoints and extractors are shared read-only, as the map's are.  Every repetition
// restores what the stages write (slots, pose, BowVector), as a new Frame would start.
//
// Prints one JSON line: frames / s = T * B * REPS / (wall time from a common start until the last
// thread ends), thread 0's seconds per stage, and thread 0's first-repetition per-frame results for
// frames 0 .. min(B, n) - 1 (bench.py checks them against the kernel-only path on the same problems).
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <thread>

#include "../tests/adapter/driver_common.h"

namespace oa = osg_orbslam3;
using Clock = std::chrono::steady_clock;

static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Barrier {
    std::mutex m;
    std::condition_variable cv;
    int n, waiting = 0, gen = 0;
    explicit Barrier(int n_) : n(n_) {}
    void wait()
    {
        std::unique_lock<std::mutex> l(m);
        const int g = gen;
        if (++waiting == n) {
            waiting = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g; });
        }
    }
};

static std::string pre(int i) { return "p" + std::to_string(i) + "."; }

// OSG_WALL_SPLIT=1 (probe runs only): before each repetition, thread 0 times the adapter's gathers of
// the same frames alone, per stage, and the JSON line carries them as "thread0_gather_s"
static const bool g_split = getenv("OSG_WALL_SPLIT") && atoi(getenv("OSG_WALL_SPLIT")) == 1;
static thread_local double g_split_s[4] = {0, 0, 0, 0};
static double g_split_t0[4] = {0, 0, 0, 0};

// The per-thread work of one workload: the constructor builds the thread's B frames; rep() runs one
// repetition of every stage, adds each stage's seconds to stage_s and, when `record` is given, keeps
// the per-frame results.
struct Workload {
    std::vector<std::string> stages, records;  // timed stages; names of the recorded per-frame results
    virtual ~Workload() = default;
    virtual void rep(std::vector<double> &stage_s, std::vector<std::vector<int32_t>> *record) = 0;
};

// ------------------------------------------------------------------------------------------ c3
struct C3Pool {
    int n;
    std::deque<KeyFrame> K;
    std::deque<Frame> Fb, Fp;
    std::deque<Camera> c, c2;
    std::vector<std::unique_ptr<MapPoint>> mps;
    explicit C3Pool(const Arrays &in) : n(get(in, "pool.n").p<int32_t>()[0]), K(n), Fb(n), Fp(n), c(n), c2(n)
    {
        for (int i = 0; i < n; i++) {
            build_bow_kf_f_problem(in, pre(i), K[i], Fb[i], mps);
            build_pose_problem(in, pre(i), Fp[i], c[i], c2[i], mps);
        }
    }
};

struct C3 : Workload {
    const C3Pool &P;
    std::vector<KeyFrame *> kfs;
    std::deque<Frame> fb, fp;
    std::vector<Frame *> fbp, fpp;
    std::vector<const Frame *> pristine;
    std::vector<int32_t> nm, ni;
    C3(const C3Pool &p, int t, int B) : P(p), nm(B), ni(B)
    {
        stages = records = {"SearchByBoW", "PoseOptimization"};
        for (int b = 0; b < B; b++) {
            const int i = (t * B + b) % P.n;
            kfs.push_back(const_cast<KeyFrame *>(&P.K[i]));
            fb.push_back(P.Fb[i]);
            fp.push_back(P.Fp[i]);
            pristine.push_back(&P.Fp[i]);
        }
        for (auto &f : fb) fbp.push_back(&f);
        for (auto &f : fp) fpp.push_back(&f);
    }
    void rep(std::vector<double> &st, std::vector<std::vector<int32_t>> *rec) override
    {
        if (g_split) {  // the adapter's gathers alone (no C-ABI call), timed apart from the stages
            auto g0 = Clock::now();
            {  // the entry points' own per-thread pools (warm buffers, as the stage's gather)
                auto &g = oa::gather_pool<oa::BowKfF<KeyFrame, Frame, MapPoint>>(kfs.size());
                for (size_t b = 0; b < kfs.size(); b++) g[b].assign(kfs[b], *fbp[b]);
            }
            auto g1 = Clock::now();
            {
                auto &g = oa::gather_pool<oa::PoseGather<MockHooks, Frame>>(fpp.size());
                for (size_t b = 0; b < fpp.size(); b++) g[b].assign(fpp[b], (oa::NoMutex *)nullptr);
            }
            g_split_s[0] += secs(g0, g1);
            g_split_s[1] += secs(g1, Clock::now());
        }
        auto t0 = Clock::now();
        std::vector<std::vector<MapPoint *>> matches;
        oa::search_by_bow_kf_f_batch<MockHooks>(kfs, fbp, matches, 0.7f, true, nm.data());
        auto t1 = Clock::now();
        for (size_t b = 0; b < fp.size(); b++) std::memcpy(fp[b].pose, pristine[b]->pose, sizeof fp[b].pose);
        oa::pose_optimization_batch<MockHooks>(fpp, ni.data());
        auto t2 = Clock::now();
        st[0] += secs(t0, t1);
        st[1] += secs(t1, t2);
        if (rec) *rec = {nm, ni};
    }
};

// ------------------------------------------------------------------------------------------ c5
struct C5Pool {
    int n;
    std::deque<Frame> Fl, LF, Fm, Fp;
    std::deque<std::vector<MapPoint *>> Q;
    std::deque<Camera> c, c2;
    std::vector<std::unique_ptr<MapPoint>> mps;
    explicit C5Pool(const Arrays &in)
        : n(get(in, "pool.n").p<int32_t>()[0]), Fl(n), LF(n), Fm(n), Fp(n), Q(n), c(n), c2(n)
    {
        for (int i = 0; i < n; i++) {
            build_last_problem(in, pre(i), Fl[i], LF[i], mps);
            Fl[i].tlc_z_value = 0.f;
            build_mps_problem(in, pre(i), Fm[i], Q[i], mps);
            build_pose_problem(in, pre(i), Fp[i], c[i], c2[i], mps);
        }
    }
};

struct C5 : Workload {
    const C5Pool &P;
    std::deque<Frame> fl, fm, fp;
    std::vector<Frame *> flp, fmp, fpp;
    std::vector<const Frame *> lfs, src_l, src_m, src_p;
    std::vector<const std::vector<MapPoint *> *> qs;
    std::vector<int32_t> nl, nq, ni;
    C5(const C5Pool &p, int t, int B) : P(p), nl(B), nq(B), ni(B)
    {
        stages = records = {"SearchByProjection(F,LastF)", "SearchByProjection(F,localMPs)", "PoseOptimization"};
        for (int b = 0; b < B; b++) {
            const int i = (t * B + b) % P.n;
            fl.push_back(P.Fl[i]);
            fm.push_back(P.Fm[i]);
            fp.push_back(P.Fp[i]);
            lfs.push_back(&P.LF[i]);
            qs.push_back(&P.Q[i]);
            src_l.push_back(&P.Fl[i]);
            src_m.push_back(&P.Fm[i]);
            src_p.push_back(&P.Fp[i]);
        }
        for (auto &f : fl) flp.push_back(&f);
        for (auto &f : fm) fmp.push_back(&f);
        for (auto &f : fp) fpp.push_back(&f);
    }
    void rep(std::vector<double> &st, std::vector<std::vector<int32_t>> *rec) override
    {
        const size_t B = fl.size();
        if (g_split) {  // the adapter's gathers alone (no C-ABI call), timed apart from the stages
            auto g0 = Clock::now();
            {
                auto &g = oa::gather_pool<oa::LastGather<MockHooks, Frame>>(B);
                for (size_t b = 0; b < B; b++) g[b].assign(*flp[b], *lfs[b]);
            }
            auto g1 = Clock::now();
            {
                auto &g = oa::gather_pool<oa::MpsGather<Frame, MapPoint>>(B);
                for (size_t b = 0; b < B; b++) g[b].assign(*fmp[b], *qs[b]);
            }
            auto g2 = Clock::now();
            {
                auto &g = oa::gather_pool<oa::PoseGather<MockHooks, Frame>>(fpp.size());
                for (size_t b = 0; b < fpp.size(); b++) g[b].assign(fpp[b], (oa::NoMutex *)nullptr);
            }
            g_split_s[0] += secs(g0, g1);
            g_split_s[1] += secs(g1, g2);
            g_split_s[2] += secs(g2, Clock::now());
        }
        auto t0 = Clock::now();
        for (size_t b = 0; b < B; b++) fl[b].mvpMapPoints = src_l[b]->mvpMapPoints;
        oa::search_by_projection_last_batch<MockHooks>(flp, lfs, 7.f, false, true, nl.data());
        auto t1 = Clock::now();
        for (size_t b = 0; b < B; b++) fm[b].mvpMapPoints = src_m[b]->mvpMapPoints;
        oa::search_by_projection_mps_batch<MockHooks>(fmp, qs, 3.f, false, 20.f, 0.9f, nq.data());
        auto t2 = Clock::now();
        for (size_t b = 0; b < B; b++) std::memcpy(fp[b].pose, src_p[b]->pose, sizeof fp[b].pose);
        oa::pose_optimization_batch<MockHooks>(fpp, ni.data());
        auto t3 = Clock::now();
        st[0] += secs(t0, t1);
        st[1] += secs(t1, t2);
        st[2] += secs(t2, t3);
        if (rec) *rec = {nl, nq, ni};
    }
};

// -------------------------------------------------------------------------------------- stereo
// One problem's levels in HBM and their on_device view (what the integrated ORBextractor keeps).
struct DevLevels {
    std::vector<const uint8_t *> data;
    std::vector<int32_t> rows, cols, step;
    osg_image_pyramid v{};
    explicit DevLevels(const ORBextractor &e)
    {
        for (const cv::Mat &m : e.mvImagePyramid) {
            void *d = nullptr;
            if (hipMalloc(&d, (size_t)m.rows * m.cols) != hipSuccess ||
                hipMemcpy2D(d, (size_t)m.cols, m.ptr<unsigned char>(0), m.step[0], (size_t)m.cols, (size_t)m.rows,
                            hipMemcpyHostToDevice) != hipSuccess)
                throw std::runtime_error("level upload failed");
            data.push_back((const uint8_t *)d);
            rows.push_back(m.rows);
            cols.push_back(m.cols);
            step.push_back(m.cols);
        }
        v.n_levels = (int32_t)data.size();
        v.on_device = 1;
        v.data = data.data();
        v.rows = rows.data();
        v.cols = cols.data();
        v.step = step.data();
    }
    ~DevLevels()
    {
        for (const uint8_t *d : data) (void)hipFree((void *)d);
    }
    DevLevels(const DevLevels &) = delete;
    DevLevels &operator=(const DevLevels &) = delete;
};

struct StereoPool {
    int n;
    std::deque<Frame> F;
    std::deque<ORBextractor> el, er;
    std::deque<DevLevels> dl, dr;
    explicit StereoPool(const Arrays &in) : n(get(in, "pool.n").p<int32_t>()[0]), F(n), el(n), er(n)
    {
        for (int i = 0; i < n; i++) {
            build_stereo_problem(in, pre(i), F[i], el[i], er[i]);
            dl.emplace_back(el[i]);
            dr.emplace_back(er[i]);
            el[i].mpOsgDeviceLevels = &dl.back().v;
            er[i].mpOsgDeviceLevels = &dr.back().v;
            el[i].mvImagePyramid.clear();  // the host levels are not read again
            er[i].mvImagePyramid.clear();
        }
    }
};

struct Stereo : Workload {
    std::deque<Frame> f;
    std::vector<Frame *> fp;
    std::vector<int32_t> nm;
    Stereo(const StereoPool &P, int t, int B) : nm(B)
    {
        stages = records = {"ComputeStereoMatches"};
        for (int b = 0; b < B; b++) f.push_back(P.F[(t * B + b) % P.n]);
        for (auto &x : f) fp.push_back(&x);
    }
    void rep(std::vector<double> &st, std::vector<std::vector<int32_t>> *rec) override
    {
        if (g_split) {  // the adapter's gather alone (no C-ABI call), timed apart from the stage
            auto g0 = Clock::now();
            auto &g = oa::gather_pool<oa::StereoGather<Frame>>(fp.size());
            for (size_t b = 0; b < fp.size(); b++) g[b].assign(*fp[b]);
            g_split_s[0] += secs(g0, Clock::now());
        }
        auto t0 = Clock::now();
        oa::compute_stereo_matches_batch(fp, nm.data());
        st[0] += secs(t0, Clock::now());
        if (rec) *rec = {nm};
    }
};

// ---------------------------------------------------------------------------------------- dbow
struct DbowPool {
    int n;
    std::deque<Frame> F;
    osg_vocabulary *voc;
    explicit DbowPool(const Arrays &in) : n(get(in, "pool.n").p<int32_t>()[0]), F(n), voc(build_vocabulary(in))
    {
        for (int i = 0; i < n; i++) build_bow_frame(in, pre(i), F[i]);
    }
    ~DbowPool() { osg_vocabulary_destroy(voc); }
};

struct Dbow : Workload {
    const osg_vocabulary *voc;
    std::deque<Frame> f;
    std::vector<Frame *> fp;
    Dbow(const DbowPool &P, int t, int B) : voc(P.voc)
    {
        stages = {"ComputeBoW"};
        records = {"n_words", "n_nodes"};
        for (int b = 0; b < B; b++) f.push_back(P.F[(t * B + b) % P.n]);
        for (auto &x : f) fp.push_back(&x);
    }
    void rep(std::vector<double> &st, std::vector<std::vector<int32_t>> *rec) override
    {
        auto t0 = Clock::now();
        for (auto &x : f) {  // a new Frame's BowVector / FeatureVector start empty
            x.mBowVec.clear();
            x.mFeatVec.clear();
        }
        oa::compute_bow_batch(fp, voc);
        st[0] += secs(t0, Clock::now());
        if (rec) {
            std::vector<int32_t> w, nodes;
            for (auto &x : f) {
                w.push_back((int32_t)x.mBowVec.size());
                nodes.push_back((int32_t)x.mFeatVec.size());
            }
            *rec = {w, nodes};
        }
    }
};

int main(int argc, char **argv)
{
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s c3|c5|stereo|dbow pool.arrays B REPS THREADS\n", argv[0]);
        return 2;
    }
    const std::string wl = argv[1];
    const int B = std::atoi(argv[3]), reps = std::atoi(argv[4]), T = std::atoi(argv[5]);
    if (B <= 0 || reps <= 0 || T <= 0 || T > 64) {
        std::fprintf(stderr, "bad B / REPS / THREADS\n");
        return 2;
    }
    try {
        const Arrays in = read_arrays(argv[2]);
        if (!oa::thread_ctx()) throw std::runtime_error("no gfx950 device (osg_ctx_create failed)");
        std::unique_ptr<C3Pool> c3;
        std::unique_ptr<C5Pool> c5;
        std::unique_ptr<StereoPool> sp;
        std::unique_ptr<DbowPool> dp;
        int n_pool = 0;
        if (wl == "c3") n_pool = (c3.reset(new C3Pool(in)), c3->n);
        else if (wl == "c5") n_pool = (c5.reset(new C5Pool(in)), c5->n);
        else if (wl == "stereo") n_pool = (sp.reset(new StereoPool(in)), sp->n);
        else if (wl == "dbow") n_pool = (dp.reset(new DbowPool(in)), dp->n);
        else throw std::runtime_error("unknown workload " + wl);

        Barrier ready(T + 1), go(T + 1);
        std::vector<Clock::time_point> end(T);
        std::vector<std::vector<double>> stage_s(T);
        std::vector<std::vector<int32_t>> first;
        std::vector<std::string> stages, records;
        std::vector<std::string> err(T);
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                std::unique_ptr<Workload> w;
                try {
                    if (c3) w.reset(new C3(*c3, t, B));
                    else if (c5) w.reset(new C5(*c5, t, B));
                    else if (sp) w.reset(new Stereo(*sp, t, B));
                    else w.reset(new Dbow(*dp, t, B));
                    stage_s[t].assign(w->stages.size(), 0.0);
                    std::vector<double> warm(w->stages.size(), 0.0);
                    w->rep(warm, t == 0 ? &first : nullptr);  // creates this thread's context, sizes its buffers
                    if (t == 0) {
                        stages = w->stages;
                        records = w->records;
                    }
                } catch (const std::exception &e) {
                    err[t] = e.what();
                }
                ready.wait();
                go.wait();
                if (err[t].empty())
                    for (int r = 0; r < reps; r++) w->rep(stage_s[t], nullptr);
                end[t] = Clock::now();
                if (t == 0)
                    for (int k = 0; k < 4; k++) g_split_t0[k] = g_split_s[k];
            });
        ready.wait();
        const auto t0 = Clock::now();
        go.wait();
        for (auto &x : th) x.join();
        for (int t = 0; t < T; t++)
            if (!err[t].empty()) throw std::runtime_error("thread " + std::to_string(t) + ": " + err[t]);
        Clock::time_point last = t0;
        for (auto &e : end) last = std::max(last, e);
        const double wall = secs(t0, last);
        const long frames = (long)T * B * reps;
        std::printf("{\"workload\": \"%s\", \"frames_per_call\": %d, \"reps\": %d, \"threads\": %d, \"distinct_problems\": %d, "
                    "\"frames\": %ld, \"wall_s\": %.6f, \"frames_per_s\": %.1f, \"thread0_stage_s\": {",
                    wl.c_str(), B, reps, T, n_pool, frames, wall, frames / wall);
        for (size_t s = 0; s < stages.size(); s++)
            std::printf("%s\"%s\": %.6f", s ? ", " : "", stages[s].c_str(), stage_s[0][s]);
        std::printf("}");
        if (g_split)
            std::printf(", \"thread0_gather_s\": [%.6f, %.6f, %.6f]", g_split_t0[0], g_split_t0[1], g_split_t0[2]);
        std::printf(", \"first_rep\": {");
        const int nrec = std::min(B, n_pool);
        for (size_t s = 0; s < first.size(); s++) {
            std::printf("%s\"%s\": [", s ? ", " : "", records[s].c_str());
            for (int i = 0; i < nrec; i++) std::printf("%s%d", i ? ", " : "", first[s][i]);
            std::printf("]");
        }
        std::printf("}}\n");
    } catch (const std::exception &e) {
        std::fprintf(stderr, "adapter_wall_bench: %s\n", e.what());
        return 1;
    }
    return 0;
}
