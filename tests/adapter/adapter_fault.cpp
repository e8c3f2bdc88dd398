// adapter_fault.cpp — the adapter's error contract on mock ORB-SLAM3 objects (test-only).
//
//   adapter_fault MODE      MODE: invalid   every ABI call returns OSG_E_INVALID (injected)
//                                 nodevice  the thread's context creation fails with OSG_E_NODEVICE (injected)
//                                 real      no injection: on a host without a gfx950 device the real
//                                           osg_ctx_create fails (prints "skip" when a device is present)
//
// Every adapter entry point runs on a small valid world; the test asserts that nothing is thrown,
// that each entry returns the reference's "nothing found" outcome (0 matches and the slots untouched,
// PoseOptimization 0 with the pose untouched, LBA / merge BA as on an abort, GBA writing the input
// state back, the ORBextractor stages without keypoints) and that the error is logged once per thread.
// Prints "ok <entry>" per check and "PASS <mode> reports=<n>"; exit status 1 on the first failure.
#define OSG_ADAPTER_FAULT_INJECTION 1
#include <cstdio>
#include <cstdlib>
#include <list>
#include <memory>
#include <string>
#include <thread>

#include "../../adapters/orbslam3/osg_orbslam3.h"
#include "mock_orbslam3.h"

using namespace mock;
namespace oa = osg_orbslam3;
using H = MockHooks;

static int g_fail = 0;
#define EXPECT(cond, what)                                                   \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stdout, "FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
            g_fail = 1;                                                      \
        } else {                                                             \
            std::fprintf(stdout, "ok %s\n", what);                           \
        }                                                                    \
    } while (0)

// ------------------------------------------------------------------------------- the world
static const int NKP = 6;

static void keypoints(std::vector<cv::KeyPoint> &kps, float dx)
{
    kps.resize(NKP);
    for (int i = 0; i < NKP; i++) {
        kps[i].pt.x = 40.f + 90.f * i + dx;
        kps[i].pt.y = 30.f + 60.f * i;
        kps[i].angle = 10.f * i;
        kps[i].octave = i % 2;
    }
}

static cv::Mat descriptors(int n, int salt)
{
    cv::Mat d(n, 32);
    for (int i = 0; i < n * 32; i++) d.buf[i] = (unsigned char)(i * 37 + salt);
    return d;
}

template <class GridT>
static void fill_grid(GridT &grid, const std::vector<cv::KeyPoint> &kps)
{
    for (size_t i = 0; i < kps.size(); i++) {
        const int ix = std::min(OSG_GRID_COLS - 1, (int)(kps[i].pt.x * OSG_GRID_COLS / 752.f));
        const int iy = std::min(OSG_GRID_ROWS - 1, (int)(kps[i].pt.y * OSG_GRID_ROWS / 480.f));
        grid[ix][iy].push_back(i);
    }
}

static std::vector<float> scales()
{
    std::vector<float> s(8, 1.f);
    for (int l = 1; l < 8; l++) s[l] = s[l - 1] * 1.2f;
    return s;
}

struct World {
    Map map;
    Camera cam, cam2;
    ORBextractor exl, exr;
    Frame F, F2;
    KeyFrame K1, K2;
    std::vector<std::unique_ptr<MapPoint>> pool;
    std::vector<MapPoint *> mps;

    MapPoint *new_mp(unsigned long id)
    {
        pool.emplace_back(new MapPoint());
        MapPoint *p = pool.back().get();
        p->mnId = id;
        p->map = &map;
        p->nobs = 2;
        for (int b = 0; b < 32; b++) p->desc.buf[b] = (unsigned char)(id * 11 + b);
        p->pos[0] = 0.1 * (double)id;
        p->pos[1] = -0.05 * (double)id;
        p->pos[2] = 4.0;
        p->mbTrackInView = true;
        p->mTrackProjX = 100.f + 50.f * (float)id;
        p->mTrackProjY = 80.f + 30.f * (float)id;
        p->mTrackViewCos = 0.99f;
        p->mnTrackScaleLevel = 1;
        p->proj_ok = true;
        p->proj_u = p->mTrackProjX;
        p->proj_v = p->mTrackProjY;
        p->proj_invz = 0.25f;
        p->proj_level = 1;
        p->s3_ok[0] = p->s3_ok[1] = true;
        p->s3_u[0] = p->s3_u[1] = p->mTrackProjX;
        p->s3_v[0] = p->s3_v[1] = p->mTrackProjY;
        p->s3_level[0] = p->s3_level[1] = 1;
        return p;
    }

    void frame(Frame &f, float dx, int salt)
    {
        f.N = NKP;
        keypoints(f.mvKeys, dx);
        f.mvKeysUn = f.mvKeys;
        keypoints(f.mvKeysRight, dx - 8.f);
        f.mDescriptors = descriptors(NKP, salt);
        f.mDescriptorsRight = descriptors(NKP, salt + 1);
        f.mvuRight.assign(NKP, -1.f);
        f.mvuRight[1] = f.mvKeys[1].pt.x - 8.f;
        f.mvDepth.assign(NKP, -1.f);
        fill_grid(f.mGrid, f.mvKeys);
        Frame::mnMinX = 0;
        Frame::mnMaxX = 752;
        Frame::mnMinY = 0;
        Frame::mnMaxY = 480;
        Frame::mfGridElementWidthInv = OSG_GRID_COLS / 752.f;
        Frame::mfGridElementHeightInv = OSG_GRID_ROWS / 480.f;
        f.mvScaleFactors = scales();
        f.mvInvScaleFactors.clear();
        for (float s : f.mvScaleFactors) f.mvInvScaleFactors.push_back(1.f / s);
        f.mvInvLevelSigma2.clear();
        f.mvLevelSigma2.clear();
        for (float s : f.mvScaleFactors) {
            f.mvLevelSigma2.push_back(s * s);
            f.mvInvLevelSigma2.push_back(1.f / (s * s));
        }
        f.mb = 0.11f;
        f.mbf = 47.9f;
        f.fx = f.fy = 458.f;
        f.cx = 367.f;
        f.cy = 248.f;
        f.mpCamera = &cam;
        f.mpORBextractorLeft = &exl;
        f.mpORBextractorRight = &exr;
        f.mvpMapPoints.assign(NKP, nullptr);
        f.mvbOutlier.assign(NKP, false);
        f.mFeatVec[7] = {0, 1, 2};
        f.mFeatVec[9] = {3, 4, 5};
        f.pose[6] = 0.5;
    }

    void keyframe(KeyFrame &k, unsigned long id, float dx, int salt)
    {
        k.mnId = id;
        k.map = &map;
        k.N = NKP;
        keypoints(k.mvKeys, dx);
        k.mvKeysUn = k.mvKeys;
        k.mDescriptors = descriptors(NKP, salt);
        k.mvuRight.assign(NKP, -1.f);
        k.mvScaleFactors = scales();
        for (float s : k.mvScaleFactors) {
            k.mvLevelSigma2.push_back(s * s);
            k.mvInvLevelSigma2.push_back(1.f / (s * s));
        }
        k.mGrid.assign(OSG_GRID_COLS, std::vector<std::vector<std::size_t>>(OSG_GRID_ROWS));
        k.mGridRight = k.mGrid;
        fill_grid(k.mGrid, k.mvKeys);
        k.mnMaxX = 752;
        k.mnMaxY = 480;
        k.mfGridElementWidthInv = OSG_GRID_COLS / 752.f;
        k.mfGridElementHeightInv = OSG_GRID_ROWS / 480.f;
        k.mpCamera = &cam;
        k.fx = k.fy = 458.f;
        k.cx = 367.f;
        k.cy = 248.f;
        k.mbf = 47.9f;
        k.mvpMapPoints.assign(NKP, nullptr);
        k.mFeatVec[7] = {0, 1, 2};
        k.mFeatVec[9] = {3, 4, 5};
        k.pose[4] = 0.1 * (double)id;
        k.triang_geom.pinhole = 1;
    }

    World()
    {
        cam.type = OSG_CAM_PINHOLE;
        cam.params = {458.f, 457.f, 367.f, 248.f};
        cam2.type = OSG_CAM_KB8;
        cam2.params = {190.f, 190.f, 254.f, 256.f, 0.003f, 0.0007f, -0.002f, 0.0002f};
        for (ORBextractor *e : {&exl, &exr}) {
            int r = 480, c = 752;
            for (int l = 0; l < 8; l++) {
                cv::Mat m(r, c);
                for (size_t i = 0; i < m.buf.size(); i++) m.buf[i] = (unsigned char)(i * 7);
                e->mvImagePyramid.push_back(m);
                r = (int)(r / 1.2f);
                c = (int)(c / 1.2f);
            }
            e->pattern.resize(512);
            for (int i = 0; i < 512; i++) e->pattern[i] = cv::Point{(i % 25) - 12, (i % 23) - 11};
            e->umax.assign(16, 15);
        }
        frame(F, 0.f, 3);
        frame(F2, 4.f, 5);
        keyframe(K1, 0, 0.f, 3);
        keyframe(K2, 1, 4.f, 5);
        for (unsigned long i = 0; i < 4; i++) mps.push_back(new_mp(100 + i));
        // slot occupants and observations: MapPoint i seen by K1 (keypoint i) and K2 (keypoint i + 1)
        for (int i = 0; i < 4; i++) {
            MapPoint *p = mps[i];
            K1.mvpMapPoints[i] = p;
            K2.mvpMapPoints[i + 1] = p;
            p->obs[&K1] = std::make_tuple(i, -1);
            p->obs[&K2] = std::make_tuple(i + 1, -1);
        }
        F.mvpMapPoints[2] = mps[2];
        F2.mvpMapPoints[0] = mps[0];
        F2.mvpMapPoints[3] = mps[3];
    }
};

// --------------------------------------------------------------------------- the entries
template <class V>
static bool same(const V &a, const V &b)
{
    return a == b;
}

static void run_all()
{
    World w;
    Sim3 S;
    MapPoint *const garbage = reinterpret_cast<MapPoint *>(0x1);

    {  // a5 SearchByProjection(Frame&, vector<MapPoint*>)
        const auto before = w.F.mvpMapPoints;
        const int n = oa::search_by_projection_mps<H>(w.F, w.mps, 1.f, false, 20.f, 0.8f);
        EXPECT(n == 0 && same(before, w.F.mvpMapPoints), "search_by_projection_mps: 0, slots untouched");
    }
    {  // a6 SearchByProjection(Frame&, const Frame&)
        const auto before = w.F.mvpMapPoints;
        const int n = oa::search_by_projection_last<H>(w.F, w.F2, 7.f, true, true);
        EXPECT(n == 0 && same(before, w.F.mvpMapPoints), "search_by_projection_last: 0, slots untouched");
    }
    {  // a7 SearchByProjection(Frame&, KeyFrame*, set)
        const auto before = w.F.mvpMapPoints;
        const std::set<MapPoint *> found;
        const int n = oa::search_by_projection_kf<H>(w.F, &w.K1, found, 10.f, 100, true);
        EXPECT(n == 0 && same(before, w.F.mvpMapPoints), "search_by_projection_kf: 0, slots untouched");
    }
    {  // Fuse(pKF, vpMapPoints)
        MapPoint *extra = w.new_mp(200);
        const auto before = w.K2.mvpMapPoints;
        const auto obs_before = extra->obs;
        const int n = oa::fuse<H>(&w.K2, std::vector<MapPoint *>{extra}, 3.f, false);
        EXPECT(n == 0 && same(before, w.K2.mvpMapPoints) && extra->obs == obs_before && !extra->isBad(),
               "fuse: 0, keyframe and MapPoints untouched");
    }
    {  // Fuse(pKF, Scw, vpPoints, vpReplacePoint)
        MapPoint *extra = w.new_mp(201);
        std::vector<MapPoint *> repl(1, garbage);
        const auto before = w.K2.mvpMapPoints;
        const int n = oa::fuse_sim3<H>(&w.K2, S, std::vector<MapPoint *>{extra}, 3.f, repl);
        EXPECT(n == 0 && same(before, w.K2.mvpMapPoints) && repl[0] == garbage,
               "fuse_sim3: 0, vpReplacePoint and keyframe untouched");
    }
    {  // a3 SearchByBoW(KF, F): the reference's vector<MapPoint*>(F.N, NULL)
        std::vector<MapPoint *> out(3, garbage);
        const int n = oa::search_by_bow_kf_f<H>(&w.K1, w.F, out, 0.7f, true);
        EXPECT(n == 0 && out == std::vector<MapPoint *>(w.F.N, nullptr), "search_by_bow_kf_f: 0, F.N NULLs");
    }
    {  // a4 SearchByBoW(KF, KF)
        std::vector<MapPoint *> out(2, garbage);
        const int n = oa::search_by_bow_kf_kf<H>(&w.K1, &w.K2, out, 0.75f, true);
        EXPECT(n == 0 && out == std::vector<MapPoint *>(w.K1.N, nullptr), "search_by_bow_kf_kf: 0, N1 NULLs");
    }
    {  // Sim3 SearchByProjection, both overloads
        std::vector<MapPoint *> matched(w.K2.N, nullptr);
        matched[5] = w.mps[0];
        const auto before = matched;
        const std::vector<MapPoint *> pts{w.new_mp(300), w.new_mp(301)};
        int n = oa::search_by_projection_sim3<H, KeyFrame>(&w.K2, S, pts, nullptr, matched, nullptr, 10, 1.f);
        EXPECT(n == 0 && matched == before, "search_by_projection_sim3: 0, vpMatched untouched");
        const std::vector<KeyFrame *> pkfs{&w.K1, &w.K1};
        std::vector<KeyFrame *> mkf(w.K2.N, nullptr);
        n = oa::search_by_projection_sim3<H, KeyFrame>(&w.K2, S, pts, &pkfs, matched, &mkf, 10, 1.f);
        EXPECT(n == 0 && matched == before && mkf == std::vector<KeyFrame *>(w.K2.N, nullptr),
               "search_by_projection_sim3 (vpPointsKFs): 0, vpMatched / vpMatchedKF untouched");
    }
    {  // SearchBySim3
        std::vector<MapPoint *> m12(w.K1.N, nullptr);
        m12[0] = w.mps[0];
        const auto before = m12;
        const int n = oa::search_by_sim3<H, KeyFrame>(&w.K1, &w.K2, m12, S, 7.5f);
        EXPECT(n == 0 && m12 == before, "search_by_sim3: 0, vpMatches12 untouched");
    }
    {  // SearchForInitialization: vnMatches12 = vector<int>(F1.mvKeysUn.size(), -1), vbPrevMatched untouched
        std::vector<cv::Point2f> prev(NKP);
        for (int i = 0; i < NKP; i++) prev[i] = w.F.mvKeysUn[i].pt;
        std::vector<int> m12(2, 7);
        const int n = oa::search_for_initialization<H>(w.F, w.F2, prev, m12, 100, 0.9f, true);
        bool prev_same = true;
        for (int i = 0; i < NKP; i++) prev_same &= prev[i].x == w.F.mvKeysUn[i].pt.x && prev[i].y == w.F.mvKeysUn[i].pt.y;
        EXPECT(n == 0 && m12 == std::vector<int>(NKP, -1) && prev_same,
               "search_for_initialization: 0, vnMatches12 all -1, vbPrevMatched untouched");
    }
    {  // ComputeStereoMatches: mvuRight / mvDepth = -1
        Frame f = w.F;
        f.mvuRight.assign(NKP, 3.f);
        f.mvDepth.assign(NKP, 3.f);
        const int n = oa::compute_stereo_matches(f);
        EXPECT(n == 0 && f.mvuRight == std::vector<float>(NKP, -1.f) && f.mvDepth == std::vector<float>(NKP, -1.f),
               "compute_stereo_matches: 0, mvuRight / mvDepth all -1");
    }
    {  // ComputeStereoFishEyeMatches: the :1558-1563 initial state
        Frame f = w.F;
        f.N = 2 * NKP;
        f.Nleft = NKP;
        f.Nright = NKP;
        f.monoLeft = 2;
        f.monoRight = 1;
        f.mpCamera = &w.cam2;
        f.mpCamera2 = &w.cam2;
        f.mDescriptors = descriptors(NKP, 9);
        f.mvLeftToRightMatch.assign(NKP, 4);
        f.mvRightToLeftMatch.assign(NKP, 4);
        f.mvDepth.assign(NKP, 2.f);
        const int n = oa::compute_stereo_fisheye_matches(f);
        EXPECT(n == 0 && f.mvLeftToRightMatch == std::vector<int>(NKP, -1) &&
                   f.mvRightToLeftMatch == std::vector<int>(NKP, -1) && f.mvDepth == std::vector<float>(NKP, -1.f) &&
                   f.mvuRight == std::vector<float>(NKP, -1.f) && (int)f.mvStereo3Dpoints.size() == NKP && f.mnCloseMPs == 0,
               "compute_stereo_fisheye_matches: 0, no stereo match");
    }
    {  // ORBextractor: ComputeKeyPointsOctTree -> no keypoints; describe -> zero rows
        std::vector<std::vector<cv::KeyPoint>> all(2, std::vector<cv::KeyPoint>(3));
        const std::vector<int> nf(8, 100);
        const int n = oa::compute_keypoints_oct_tree(w.exl.mvImagePyramid, all, nf, scales(), 20, 7);
        bool empty = all.size() == 8;
        for (const auto &l : all) empty &= l.empty();
        EXPECT(n == 0 && empty, "compute_keypoints_oct_tree: 0, no keypoints");
        std::vector<std::vector<cv::KeyPoint>> kps(8);
        for (int i = 0; i < 3; i++) {
            cv::KeyPoint kp;
            kp.pt.x = 100.f + 10.f * i;
            kp.pt.y = 100.f;
            kp.angle = 5.f;
            kps[0].push_back(kp);
        }
        std::vector<uint8_t> desc(7, 1);
        const int o = oa::orb_describe(w.exl.mvImagePyramid, w.exl.mvImagePyramid, kps, w.exl.pattern, w.exl.umax, desc);
        EXPECT(o == 0 && desc == std::vector<uint8_t>(3 * 32, 0) && kps[0][0].angle == 5.f,
               "orb_describe: 0, zero descriptors, angles untouched");
        std::vector<uint8_t> d2(7, 1);
        const int o2 = oa::orb_describe(w.exl.mvImagePyramid, w.exl.mvImagePyramid, kps, std::vector<cv::Point>(3),
                                        w.exl.umax, d2);
        EXPECT(o2 == 0 && d2 == std::vector<uint8_t>(3 * 32, 0), "orb_describe (bad pattern): 0, zero descriptors");
    }
    {  // SearchForTriangulation: vMatchedPairs cleared
        std::vector<std::pair<size_t, size_t>> pairs{{1, 2}};
        const int n = oa::search_for_triangulation<H>(&w.K1, &w.K2, pairs, false, false, true);
        EXPECT(n == 0 && pairs.empty(), "search_for_triangulation: 0, vMatchedPairs empty");
    }
    {  // ComputeDistinctiveDescriptors: descriptors unchanged
        std::vector<std::vector<unsigned char>> before;
        for (MapPoint *p : w.mps) before.push_back(p->desc.buf);
        oa::compute_distinctive_descriptors<H>(w.mps);
        bool same_desc = true;
        for (size_t i = 0; i < w.mps.size(); i++) same_desc &= w.mps[i]->desc.buf == before[i];
        EXPECT(same_desc, "compute_distinctive_descriptors: descriptors untouched");
    }
    {  // PoseOptimization: 0, pose untouched
        Frame f = w.F;
        for (int i = 0; i < 4; i++) f.mvpMapPoints[i] = w.mps[i];
        double pose_before[7];
        std::memcpy(pose_before, f.pose, sizeof pose_before);
        const int n = oa::pose_optimization<H>(&f);
        EXPECT(n == 0 && std::memcmp(pose_before, f.pose, sizeof pose_before) == 0, "pose_optimization: 0, pose untouched");
    }
    {  // LocalBundleAdjustment: as on an abort, nothing to write back
        std::list<KeyFrame *> local{&w.K2}, fixed{&w.K1};
        std::list<MapPoint *> lmps(w.mps.begin(), w.mps.end());
        bool stop = false;
        const auto out = oa::local_bundle_adjustment<H>(local, fixed, lmps, &w.map, 0ul, &stop, false);
        EXPECT(out.aborted && out.poses.empty() && out.points.empty() && out.to_erase.empty() && out.num_edges == 8 &&
                   out.num_MPs == 4 && out.num_fixedKF == 1 && out.num_OptKF == 1,
               "local_bundle_adjustment: aborted, nothing written back, window counts kept");
    }
    {  // global BA: the input state written back (0 iterations)
        bool stop = false;
        const auto out = oa::bundle_adjustment<H>(std::vector<KeyFrame *>{&w.K1, &w.K2}, w.mps, 0ul, 10, &stop, true);
        bool state_in = out.iterations == 0 && out.poses.size() == 2 && out.points.size() == 4;
        for (const auto &kp : out.poses) state_in &= std::memcmp(kp.second.data(), kp.first->pose, 56) == 0;
        for (const auto &mp : out.points) state_in &= std::memcmp(mp.second.data(), mp.first->pos, 24) == 0;
        EXPECT(state_in, "bundle_adjustment: the input state, 0 iterations");
        oa::apply_bundle_adjustment<H>(out, 42ul, false);
        EXPECT(w.K2.mnBAGlobalForKF == 42ul && std::memcmp(w.K2.pose_gba, w.K2.pose, 56) == 0 &&
                   w.mps[1]->mnBAGlobalForKF == 42ul,
               "apply_bundle_adjustment: mTcwGBA / mPosGBA = the input state");
    }
    {  // the merge BA: aborted, nothing to write back
        bool stop = false;
        const auto out = oa::merge_local_bundle_adjustment<H, KeyFrame, MapPoint>(&w.K2, std::vector<KeyFrame *>{&w.K2},
                                                                                 std::vector<KeyFrame *>{&w.K1}, &stop);
        EXPECT(out.aborted && out.poses.empty() && out.points.empty() && out.to_erase.empty(),
               "merge_local_bundle_adjustment: aborted, nothing written back");
    }
    {  // ComputeBoW: mBowVec / mFeatVec empty (no vocabulary reachable), single and batched
        Frame f = w.F;
        f.mDescriptors = descriptors(NKP, 3);
        f.mFeatVec[7] = {1, 2};
        oa::compute_bow(f, nullptr);
        EXPECT(f.mBowVec.empty() && f.mFeatVec.empty(), "compute_bow: mBowVec / mFeatVec empty");
        Frame g = f;
        g.mFeatVec[7] = {1};
        oa::compute_bow_batch(std::vector<Frame *>{&f, &g}, nullptr);
        EXPECT(f.mBowVec.empty() && g.mBowVec.empty() && g.mFeatVec.empty(), "compute_bow_batch: maps empty");
    }
    {  // the batched forms: each problem gets its single call's outcome
        Frame f1 = w.F, f2 = w.F;
        std::vector<std::vector<MapPoint *>> m;
        int32_t nm[2] = {5, 5};
        oa::search_by_bow_kf_f_batch<H>(std::vector<KeyFrame *>{&w.K1, &w.K1}, std::vector<Frame *>{&f1, &f2}, m, 0.7f,
                                        true, nm);
        EXPECT(nm[0] == 0 && nm[1] == 0 && m.size() == 2 && m[1] == std::vector<MapPoint *>(w.F.N, nullptr),
               "search_by_bow_kf_f_batch: 0 each, F.N NULLs");
        const auto before = f1.mvpMapPoints;
        nm[0] = nm[1] = 5;
        oa::search_by_projection_last_batch<H>(std::vector<Frame *>{&f1, &f2}, std::vector<const Frame *>{&w.F2, &w.F2},
                                               7.f, true, true, nm);
        EXPECT(nm[0] == 0 && nm[1] == 0 && f1.mvpMapPoints == before, "search_by_projection_last_batch: 0, slots untouched");
        nm[0] = nm[1] = 5;
        oa::search_by_projection_mps_batch<H>(std::vector<Frame *>{&f1, &f2},
                                              std::vector<const std::vector<MapPoint *> *>{&w.mps, &w.mps}, 1.f, false,
                                              20.f, 0.8f, nm);
        EXPECT(nm[0] == 0 && nm[1] == 0 && f2.mvpMapPoints == before, "search_by_projection_mps_batch: 0, slots untouched");
        for (int i = 0; i < 4; i++) f1.mvpMapPoints[i] = w.mps[i];
        double pose_before[7];
        std::memcpy(pose_before, f1.pose, sizeof pose_before);
        nm[0] = 5;
        oa::pose_optimization_batch<H>(std::vector<Frame *>{&f1}, nm);
        EXPECT(nm[0] == 0 && std::memcmp(pose_before, f1.pose, sizeof pose_before) == 0,
               "pose_optimization_batch: 0, pose untouched");
        f2.mvuRight.assign(NKP, 3.f);
        f2.mvDepth.assign(NKP, 3.f);
        nm[0] = 5;
        oa::compute_stereo_matches_batch(std::vector<Frame *>{&f2}, nm);
        EXPECT(nm[0] == 0 && f2.mvuRight == std::vector<float>(NKP, -1.f) && f2.mvDepth == std::vector<float>(NKP, -1.f),
               "compute_stereo_matches_batch: 0, mvuRight / mvDepth all -1");
    }
}

int main(int argc, char **argv)
{
    if (argc != 2) {
        std::fprintf(stderr, "usage: %s invalid|nodevice|real\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "real") {
        osg_ctx *c = nullptr;
        if (osg_ctx_create(0, &c) == OSG_OK) {
            osg_ctx_destroy(c);
            std::printf("skip: a gfx950 device is present\n");
            return 0;
        }
    } else if (mode != "invalid" && mode != "nodevice") {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    int reports = -1;
    bool threw = false;
    // a fresh thread: its own context slot and its own once-per-thread log state
    std::thread t([&] {
        try {
            if (mode == "invalid") oa::fault::call_rc = OSG_E_INVALID;
            if (mode == "nodevice") oa::fault::ctx_rc = OSG_E_NODEVICE;
            run_all();
        } catch (...) {
            threw = true;
        }
        reports = oa::fault::reports;
    });
    t.join();
    EXPECT(!threw, "no exception escaped");
    // each code once per thread: "invalid" logs OSG_E_INVALID; "nodevice" / "real" log OSG_E_NODEVICE and
    // the host-side pattern-shape check's OSG_E_INVALID
    EXPECT(reports == (mode == "invalid" ? 1 : 2), "each error code was logged once on this thread");
    if (g_fail) return 1;
    std::printf("PASS %s reports=%d\n", mode.c_str(), reports);
    return 0;
}
