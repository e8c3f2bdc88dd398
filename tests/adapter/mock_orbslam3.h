// mock_orbslam3.h — POD stand-ins for the ORB-SLAM3 types the adapter reads (test-only).
// Member names follow ref:include/Frame.h, KeyFrame.h, MapPoint.h so adapters/orbslam3/
// osg_orbslam3.h compiles unchanged against them; math the reference does with Sophus / Eigen is
// supplied through MockHooks from values stored on the objects.
#ifndef MOCK_ORBSLAM3_H
#define MOCK_ORBSLAM3_H

#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <thread>
#include <tuple>
#include <vector>

#include "osg.h"
#include "osg_ba.h"

namespace cv {
struct Point {
    int x = 0, y = 0;
};
struct Point2f {
    float x = 0, y = 0;
};
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = 0, response = 0;
    int octave = 0, class_id = -1;
};
struct Mat {  // CV_8UC1 rows x cols, step[0] bytes per row (an ROI of a wider buffer when > cols)
    int rows = 0, cols = 0;
    std::vector<unsigned char> buf;
    size_t step[2] = {0, 1};
    Mat() = default;
    Mat(int r, int c) : rows(r), cols(c), buf((size_t)r * c), step{(size_t)c, 1} {}
    Mat(int r, int c, size_t s) : rows(r), cols(c), buf((size_t)r * s), step{s, 1} {}
    template <class T>
    T *ptr(int i) { return reinterpret_cast<T *>(buf.data() + (size_t)i * step[0]); }
    template <class T>
    const T *ptr(int i) const { return reinterpret_cast<const T *>(buf.data() + (size_t)i * step[0]); }
};
}  // namespace cv

namespace mock {

struct Map {};
struct KeyFrame;

struct Camera {
    int type = OSG_CAM_PINHOLE;
    std::vector<float> params;
    std::vector<double> trl;  // test-only: GetRelativePoseTrl of a right camera {qx qy qz qw tx ty tz}; empty = identity
    float getParameter(const int i) const { return params[i]; }  // GeometricCamera::getParameter
};

// Eigen::Matrix3f / Vector3f as far as the adapters use them: m(r, c), v(k)
struct Mat3f {
    float a[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    float &operator()(int r, int c) { return a[3 * r + c]; }
    float operator()(int r, int c) const { return a[3 * r + c]; }
};
struct Vec3f {
    float a[3] = {0, 0, 0};
    float &operator()(int k) { return a[k]; }
    float operator()(int k) const { return a[k]; }
};

struct MapPoint {
    unsigned long mnId = 0;
    bool bad = false;
    int nobs = 0;
    cv::Mat desc{1, 32};
    double pos[3] = {0, 0, 0};
    // isInFrustum results (SearchByProjection(Frame&, vector<MapPoint*>))
    float mTrackProjX = 0, mTrackProjY = 0, mTrackDepth = 0, mTrackDepthR = 0, mTrackProjXR = 0, mTrackProjYR = 0;
    bool mbTrackInView = false, mbTrackInViewR = false;
    double pos_gba[3] = {0, 0, 0};  // mPosGBA
    unsigned long mnBAGlobalForKF = 0, mnBALocalForMerge = 0;
    Map *map = nullptr;
    Map *GetMap() const { return map; }
    int mnTrackScaleLevel = 0, mnTrackScaleLevelR = 0;
    float mTrackViewCos = 0, mTrackViewCosR = 0;
    // test-only: what MockHooks::project_last / kf_query return for this MapPoint
    bool proj_ok = false;
    float proj_u = 0, proj_v = 0, proj_invz = 0, proj_ur = 0, proj_vr = 0, proj_fuse_ur = 0;
    int proj_level = 0;
    // test-only: what MockHooks::sim3_pair_query returns, [0] KF1 -> KF2, [1] KF2 -> KF1
    bool s3_ok[2] = {false, false};
    float s3_u[2] = {0, 0}, s3_v[2] = {0, 0};
    int s3_level[2] = {0, 0};
    std::map<KeyFrame *, std::tuple<int, int>> obs;

    bool isBad() const { return bad; }
    int Observations() const { return nobs; }
    cv::Mat GetDescriptor() const { return desc; }
    // the integration's non-cloning accessor: the 32 bytes under the feature lock
    void GetDescriptorRow(unsigned char *dst) const { std::memcpy(dst, desc.buf.data(), 32); }
    std::map<KeyFrame *, std::tuple<int, int>> GetObservations() const { return obs; }
    void EraseObservation(KeyFrame *k) { obs.erase(k); }
    bool IsInKeyFrame(KeyFrame *k) const { return obs.count(k) != 0; }
    void AddObservation(KeyFrame *k, int idx)
    {
        obs[k] = std::make_tuple(idx, -1);
        nobs++;
    }
    // MapPoint::Replace (ref:src/MapPoint.cc:313-395) over the keyframes this test models; the
    // observations in other keyframes (nobs - obs.size()) move along; the survivor's descriptor
    // changes as ComputeDistinctiveDescriptors would (test-only: byte 0 ^= 0x5A)
    void Replace(MapPoint *p);
};

struct ORBextractor {
    std::vector<cv::Mat> mvImagePyramid;
    const osg_image_pyramid *mpOsgDeviceLevels = nullptr;  // the integration's device levels (osg_orb_pyramid)
    std::vector<cv::Point> pattern;  // ref:include/ORBextractor.h (512 points of bit_pattern_31_)
    std::vector<int> umax;           // HALF_PATCH_SIZE + 1 row half-widths
};

struct Frame {
    int N = 0, Nleft = -1;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn, mvKeysRight;
    cv::Mat mDescriptors, mDescriptorsRight;
    std::vector<float> mvuRight, mvDepth, mvInvScaleFactors;
    ORBextractor *mpORBextractorLeft = nullptr, *mpORBextractorRight = nullptr;
    std::vector<MapPoint *> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::vector<std::size_t> mGrid[OSG_GRID_COLS][OSG_GRID_ROWS];
    std::vector<std::size_t> mGridRight[OSG_GRID_COLS][OSG_GRID_ROWS];
    std::vector<int> mvLeftToRightMatch, mvRightToLeftMatch;
    static inline float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    static inline float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    int mnScaleLevels = 8;
    std::vector<float> mvScaleFactors, mvInvLevelSigma2;
    float mb = 0, mbf = 0, fx = 0, fy = 0, cx = 0, cy = 0;
    Camera *mpCamera = nullptr, *mpCamera2 = nullptr;
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;
    std::map<unsigned int, double> mBowVec;  // DBoW2::BowVector
    double pose[7] = {0, 0, 0, 1, 0, 0, 0};
    float tlc_z_value = 0;  // test-only: MockHooks::tlc_z
    // two-camera (KannalaBrandt8) Frame members of ComputeStereoFishEyeMatches (ref:include/Frame.h)
    int Nright = -1, monoLeft = -1, monoRight = -1, mnCloseMPs = -1;
    std::vector<float> mvLevelSigma2;
    Mat3f mRlr;
    Vec3f mtlr;
    std::vector<Vec3f> mvStereo3Dpoints;
};

struct KeyFrame {
    unsigned long mnId = 0;
    int N = 0, NLeft = -1;
    bool bad = false;
    Map *map = nullptr;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn, mvKeysRight;
    cv::Mat mDescriptors;
    std::vector<float> mvuRight, mvInvLevelSigma2;
    std::vector<MapPoint *> mvpMapPoints;
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;
    std::map<unsigned int, double> mBowVec;  // DBoW2::BowVector
    float mbf = 0, mb = 0, fx = 0, fy = 0, cx = 0, cy = 0;
    Camera *mpCamera = nullptr, *mpCamera2 = nullptr;
    double pose[7] = {0, 0, 0, 1, 0, 0, 0};
    // grid fields as in ref:include/KeyFrame.h:321-508 (mnMinX.. are int there)
    std::vector<std::vector<std::vector<std::size_t>>> mGrid, mGridRight;
    std::vector<int> mvLeftToRightMatch, mvRightToLeftMatch;
    int mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    int mnScaleLevels = 8;
    std::vector<float> mvScaleFactors, mvLevelSigma2;
    osg_triang_geom triang_geom{};  // test-only: MockHooks::triang_geom
    double pose_gba[7] = {0, 0, 0, 0, 0, 0, 0};  // mTcwGBA
    unsigned long mnBAGlobalForKF = 0, mnBALocalForMerge = 0;

    std::vector<MapPoint *> GetMapPointMatches() const { return mvpMapPoints; }
    bool isBad() const { return bad; }
    Map *GetMap() const { return map; }
    void EraseMapPointMatch(MapPoint *p)
    {
        for (auto &q : mvpMapPoints)
            if (q == p) q = nullptr;
    }
    MapPoint *GetMapPoint(std::size_t idx) const { return mvpMapPoints[idx]; }
    void AddMapPoint(MapPoint *p, std::size_t idx) { mvpMapPoints[idx] = p; }
    std::set<MapPoint *> GetMapPoints() const
    {  // ref:src/KeyFrame.cc GetMapPoints: the non-NULL, non-bad slot occupants
        std::set<MapPoint *> s;
        for (MapPoint *p : mvpMapPoints)
            if (p && !p->isBad()) s.insert(p);
        return s;
    }
};

inline void MapPoint::Replace(MapPoint *p)
{
    if (p->mnId == mnId) return;
    const int other = nobs - (int)obs.size();
    auto o = obs;
    obs.clear();
    bad = true;
    for (auto &kv : o) {
        KeyFrame *k = kv.first;
        const int li = std::get<0>(kv.second);
        if (!p->IsInKeyFrame(k)) {
            k->mvpMapPoints[li] = p;
            p->AddObservation(k, li);
        } else {
            k->mvpMapPoints[li] = nullptr;
        }
    }
    p->nobs += other;
    p->desc.buf[0] ^= 0x5A;
}

// test-only: a MapPoint::mGlobalMutex stand-in that records when it is held, and what the hooks saw
// (world_pos runs during the gather, set_pose during the write-back after the GPU solve)
struct ProbeMutex {
    std::mutex m;
    std::atomic<bool> held{false};
    int locks = 0;
    void lock()
    {
        m.lock();
        held = true;
        locks++;
    }
    void unlock()
    {
        held = false;
        m.unlock();
    }
};
inline ProbeMutex *g_probe = nullptr;
inline int g_gather_unlocked = 0, g_apply_locked = 0, g_apply_try_lock_failed = 0;

struct Sim3 {};  // Fuse(KeyFrame*, Sim3f&, ...): the projection is MockHooks' (test-only)

struct MockHooks {
    template <class T>
    static void pose(const T &o, double q[7]) { std::memcpy(q, o.pose, sizeof o.pose); }
    template <class T>
    static void set_pose(T &o, const double q[7])
    {
        if (g_probe) {  // another thread must be able to take the mutex while the result is applied
            g_apply_locked += g_probe->held ? 1 : 0;
            std::thread t([] {
                if (g_probe->m.try_lock()) g_probe->m.unlock();
                else g_apply_try_lock_failed++;
            });
            t.join();
        }
        std::memcpy(o.pose, q, sizeof o.pose);
    }
    static void world_pos(MapPoint *p, double x[3])
    {
        if (g_probe && !g_probe->held) g_gather_unlocked++;
        std::memcpy(x, p->pos, sizeof p->pos);
    }
    static void set_world_pos(MapPoint *p, const double x[3]) { std::memcpy(p->pos, x, sizeof p->pos); }
    static void set_gba_pose(KeyFrame &k, const double q[7], unsigned long n)
    {
        std::memcpy(k.pose_gba, q, sizeof k.pose_gba);
        k.mnBAGlobalForKF = n;
    }
    static void set_gba_pos(MapPoint *p, const double x[3], unsigned long n)
    {
        std::memcpy(p->pos_gba, x, sizeof p->pos_gba);
        p->mnBAGlobalForKF = n;
    }
    template <class T>
    static void camera(const T &o, bool right, osg_camera &c)
    {
        std::memset(&c, 0, sizeof c);
        const Camera *cam = right ? o.mpCamera2 : o.mpCamera;
        c.type = cam ? cam->type : OSG_CAM_PINHOLE;
        if (cam)
            for (size_t i = 0; i < cam->params.size() && i < 8; i++) c.p[i] = cam->params[i];
        c.fx = o.fx;
        c.fy = o.fy;
        c.cx = o.cx;
        c.cy = o.cy;
        c.bf = o.mbf;
        c.trl[3] = 1.0;
        if (right && cam && cam->trl.size() == 7)
            for (int i = 0; i < 7; i++) c.trl[i] = cam->trl[i];
    }
    static bool project_last(const Frame &, MapPoint *p, float &u, float &v, float &invz)
    {
        u = p->proj_u;
        v = p->proj_v;
        invz = p->proj_invz;
        return p->proj_ok;
    }
    static void project_last_right(const Frame &, MapPoint *p, float &u, float &v)
    {
        u = p->proj_ur;
        v = p->proj_vr;
    }
    static float tlc_z(const Frame &CF, const Frame &) { return CF.tlc_z_value; }
    static bool kf_query(const Frame &, MapPoint *p, float &u, float &v, int &level)
    {
        u = p->proj_u;
        v = p->proj_v;
        level = p->proj_level;
        return p->proj_ok;
    }
    static bool fuse_query(KeyFrame *, MapPoint *p, bool, float &u, float &v, float &ur, int &level)
    {
        u = p->proj_u;
        v = p->proj_v;
        ur = p->proj_fuse_ur;
        level = p->proj_level;
        return p->proj_ok;
    }
    static void triang_geom(KeyFrame *pKF1, KeyFrame *, osg_triang_geom &g) { g = pKF1->triang_geom; }
    static int index_in_keyframe(MapPoint *p, KeyFrame *k)
    {
        const auto it = p->obs.find(k);
        return it == p->obs.end() ? -1 : std::get<0>(it->second);
    }
    static bool sim3_pair_query(KeyFrame *, KeyFrame *, MapPoint *p, const Sim3 &, bool dir12, float &u, float &v,
                                int &level)
    {
        const int d = dir12 ? 0 : 1;
        u = p->s3_u[d];
        v = p->s3_v[d];
        level = p->s3_level[d];
        return p->s3_ok[d];
    }
    static bool sim3_query(KeyFrame *, const Sim3 &, MapPoint *p, bool, float &u, float &v, int &level)
    {
        u = p->proj_u;
        v = p->proj_v;
        level = p->proj_level;
        return p->proj_ok;
    }
    static void set_descriptor(MapPoint *p, const uint8_t *row) { std::memcpy(p->desc.buf.data(), row, 32); }
    static bool fuse_sim3_query(KeyFrame *, const Sim3 &, MapPoint *p, float &u, float &v, int &level)
    {
        u = p->proj_u;
        v = p->proj_v;
        level = p->proj_level;
        return p->proj_ok;
    }
};

}  // namespace mock
#endif
