// driver_common.h — mock ORB-SLAM3 objects from the array files tests/test_adapter.py and bench.py
// write (test / bench infrastructure): the array file I/O and the builders of mock Frames, KeyFrames
// and MapPoints shared by tests/adapter/adapter_driver.cpp and tools/adapter_wall_bench.cpp.
//
// Array file: repeated {u32 name_len, name, u8 dtype ('b' u8, 'i' i32, 'f' f32, 'd' f64), u64 count,
// data}.
#ifndef OSG_DRIVER_COMMON_H
#define OSG_DRIVER_COMMON_H
#include <cstdio>
#include <cstdlib>
#include <list>
#include <memory>
#include <string>
#include <unordered_map>

#include "../../adapters/orbslam3/osg_orbslam3.h"
#include "mock_orbslam3.h"

using namespace mock;

struct Arr {
    char t = 0;
    std::vector<unsigned char> b;
    size_t n = 0;
    template <class T>
    const T *p() const { return reinterpret_cast<const T *>(b.data()); }
};
using Arrays = std::unordered_map<std::string, Arr>;

inline Arrays read_arrays(const char *path)
{
    Arrays m;
    FILE *f = fopen(path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    for (;;) {
        uint32_t len;
        if (fread(&len, 4, 1, f) != 1) break;
        std::string name(len, '\0');
        Arr a;
        uint64_t n = 0;
        bool ok = fread(&name[0], 1, len, f) == len && fread(&a.t, 1, 1, f) == 1 && fread(&n, 8, 1, f) == 1;
        a.n = n;
        const size_t es = a.t == 'b' ? 1 : a.t == 'd' ? 8 : 4;
        a.b.resize(n * es);
        if (ok && n) ok = fread(a.b.data(), es, n, f) == n;
        if (!ok) {
            fclose(f);
            throw std::runtime_error(std::string("truncated array file ") + path);
        }
        m[name] = std::move(a);
    }
    fclose(f);
    return m;
}

inline void write_arrays(const char *path, const Arrays &m)
{
    FILE *f = fopen(path, "wb");
    for (const auto &kv : m) {
        const uint32_t len = (uint32_t)kv.first.size();
        fwrite(&len, 4, 1, f);
        fwrite(kv.first.data(), 1, len, f);
        fwrite(&kv.second.t, 1, 1, f);
        const uint64_t n = kv.second.n;
        fwrite(&n, 8, 1, f);
        fwrite(kv.second.b.data(), 1, kv.second.b.size(), f);
    }
    fclose(f);
}

template <class T>
inline Arr make(char t, const std::vector<T> &v)
{
    Arr a;
    a.t = t;
    a.n = v.size();
    a.b.resize(v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(a.b.data(), v.data(), a.b.size());
    return a;
}

inline const Arr &get(const Arrays &m, const std::string &k)
{
    auto it = m.find(k);
    if (it == m.end()) throw std::runtime_error("missing array " + k);
    return it->second;
}

inline bool has(const Arrays &m, const std::string &k) { return m.count(k) != 0; }

inline void fill_grid(const Arrays &m, const std::string &pre, std::vector<std::size_t> (&grid)[OSG_GRID_COLS][OSG_GRID_ROWS])
{
    const int32_t *gs = get(m, pre + "grid_start").p<int32_t>(), *gi = get(m, pre + "grid_idx").p<int32_t>();
    for (int ix = 0; ix < OSG_GRID_COLS; ix++)
        for (int iy = 0; iy < OSG_GRID_ROWS; iy++) {
            const int c = ix * OSG_GRID_ROWS + iy;
            for (int j = gs[c]; j < gs[c + 1]; j++) grid[ix][iy].push_back((size_t)gi[j]);
        }
}

// Frame from the FrameSoA arrays "F.*" (keypoints, descriptors, mvuRight, grid CSR, scales; for a
// two-camera rig "F.nleft", the right grid and the stereo-partner maps)
inline void build_frame(const Arrays &m, Frame &F, const std::string &P = "F.")
{
    const int n = (int)get(m, P + "kp_x").n;
    F.N = n;
    F.Nleft = has(m, P + "nleft") ? get(m, P + "nleft").p<int32_t>()[0] : -1;
    const int nl = F.Nleft == -1 ? n : F.Nleft;
    const float *x = get(m, P + "kp_x").p<float>(), *y = get(m, P + "kp_y").p<float>(), *a = get(m, P + "kp_angle").p<float>();
    const int32_t *o = get(m, P + "kp_octave").p<int32_t>();
    std::vector<cv::KeyPoint> kps(n);
    for (int i = 0; i < n; i++) {
        kps[i].pt.x = x[i];
        kps[i].pt.y = y[i];
        kps[i].angle = a[i];
        kps[i].octave = o[i];
    }
    F.mvKeys.assign(kps.begin(), kps.begin() + nl);
    F.mvKeysRight.assign(kps.begin() + nl, kps.end());
    F.mvKeysUn = F.mvKeys;  // left keypoints only on a two-camera rig (ref:src/Frame.cc:1022)
    if (F.Nleft != -1) {
        fill_grid(m, P, F.mGrid);
        fill_grid(m, P + "r_", F.mGridRight);
        const Arr &l2r = get(m, P + "left_to_right"), &r2l = get(m, P + "right_to_left");
        F.mvLeftToRightMatch.assign(l2r.p<int32_t>(), l2r.p<int32_t>() + l2r.n);
        F.mvRightToLeftMatch.assign(r2l.p<int32_t>(), r2l.p<int32_t>() + r2l.n);
    }
    F.mDescriptors = cv::Mat(n, 32);
    std::memcpy(F.mDescriptors.buf.data(), get(m, P + "desc").b.data(), (size_t)n * 32);
    F.mvuRight.assign(n, -1.0f);
    if (has(m, P + "u_right")) std::memcpy(F.mvuRight.data(), get(m, P + "u_right").b.data(), (size_t)n * 4);
    if (F.Nleft == -1) fill_grid(m, P, F.mGrid);
    const float *sc = get(m, P + "scalars").p<float>();  // min_x max_x min_y max_y inv_w inv_h mb mbf
    Frame::mnMinX = sc[0];
    Frame::mnMaxX = sc[1];
    Frame::mnMinY = sc[2];
    Frame::mnMaxY = sc[3];
    Frame::mfGridElementWidthInv = sc[4];
    Frame::mfGridElementHeightInv = sc[5];
    F.mb = sc[6];
    F.mbf = sc[7];
    const Arr &s = get(m, P + "scale");
    F.mvScaleFactors.assign(s.p<float>(), s.p<float>() + s.n);
    F.mnScaleLevels = (int)s.n;
    F.mvpMapPoints.assign(n, nullptr);
    F.mvbOutlier.assign(n, false);
}

// occupants of Frame::mvpMapPoints from "S.slot_mp" / "S.slot_taken"
inline void build_slots(const Arrays &m, const std::string &pre, Frame &F, std::vector<std::unique_ptr<MapPoint>> &pool)
{
    const int32_t *sm = get(m, pre + "S.slot_mp").p<int32_t>();
    const uint8_t *st = has(m, pre + "S.slot_taken") ? get(m, pre + "S.slot_taken").p<uint8_t>() : nullptr;
    for (int i = 0; i < F.N; i++)
        if (sm[i] >= 0) {
            pool.emplace_back(new MapPoint());
            pool.back()->mnId = (unsigned long)sm[i];
            pool.back()->nobs = st ? st[i] : 1;
            F.mvpMapPoints[i] = pool.back().get();
        }
}

inline std::vector<int32_t> slot_ids(const std::vector<MapPoint *> &v)
{
    std::vector<int32_t> r(v.size(), -1);
    for (size_t i = 0; i < v.size(); i++)
        if (v[i]) r[i] = (int32_t)v[i]->mnId;
    return r;
}

inline void fill_featvec(const Arrays &m, const std::string &pre, std::map<unsigned int, std::vector<unsigned int>> &fv)
{
    const Arr &nid = get(m, pre + "node_id"), &ns = get(m, pre + "node_start"), &ft = get(m, pre + "feat");
    for (size_t k = 0; k < nid.n; k++) {
        auto &v = fv[nid.p<uint32_t>()[k]];
        for (int j = ns.p<int32_t>()[k]; j < ns.p<int32_t>()[k + 1]; j++) v.push_back((unsigned)ft.p<int32_t>()[j]);
    }
}

// a BoW side "B1." / "B2." as a KeyFrame with MapPoints (mnId = mp_id, bad = !mp_good)
inline void build_bow_kf(const Arrays &m, const std::string &pre, KeyFrame &K, std::vector<std::unique_ptr<MapPoint>> &pool)
{
    const Arr &d = get(m, pre + "desc");
    const int n = (int)(d.n / 32);
    K.N = n;
    K.NLeft = has(m, pre + "nleft") ? get(m, pre + "nleft").p<int32_t>()[0] : -1;
    const int nl = K.NLeft == -1 ? n : K.NLeft;
    K.mDescriptors = cv::Mat(n, 32);
    std::memcpy(K.mDescriptors.buf.data(), d.b.data(), d.b.size());
    const float *ang = get(m, pre + "angle").p<float>();
    std::vector<cv::KeyPoint> kps(n);
    for (int i = 0; i < n; i++) kps[i].angle = ang[i];
    K.mvKeys.assign(kps.begin(), kps.begin() + nl);
    K.mvKeysRight.assign(kps.begin() + nl, kps.end());
    K.mvKeysUn = K.mvKeys;
    static Camera second;
    K.mpCamera2 = K.NLeft == -1 ? nullptr : &second;
    K.mvpMapPoints.assign(n, nullptr);
    const int32_t *id = get(m, pre + "mp_id").p<int32_t>();
    const uint8_t *good = get(m, pre + "mp_good").p<uint8_t>();
    for (int i = 0; i < n; i++)
        if (id[i] >= 0) {
            pool.emplace_back(new MapPoint());
            pool.back()->mnId = (unsigned long)id[i];
            pool.back()->bad = !good[i];
            K.mvpMapPoints[i] = pool.back().get();
        }
    fill_featvec(m, pre, K.mFeatVec);
}

// KeyFrame with keypoints / grid / scales from the FrameSoA arrays "F.*" (Fuse target)
inline void build_kf_frame(const Arrays &m, KeyFrame &K)
{
    Frame F;
    build_frame(m, F);
    K.N = F.N;
    K.NLeft = F.Nleft;
    K.mvKeys = F.mvKeys;
    K.mvKeysUn = F.mvKeysUn;
    K.mvKeysRight = F.mvKeysRight;
    K.mDescriptors = F.mDescriptors;
    K.mvuRight = F.mvuRight;
    K.mGrid.assign(OSG_GRID_COLS, std::vector<std::vector<std::size_t>>(OSG_GRID_ROWS));
    K.mGridRight.assign(OSG_GRID_COLS, std::vector<std::vector<std::size_t>>(OSG_GRID_ROWS));
    for (int ix = 0; ix < OSG_GRID_COLS; ix++)
        for (int iy = 0; iy < OSG_GRID_ROWS; iy++) {
            K.mGrid[ix][iy] = F.mGrid[ix][iy];
            K.mGridRight[ix][iy] = F.mGridRight[ix][iy];
        }
    K.mvLeftToRightMatch = F.mvLeftToRightMatch;
    K.mvRightToLeftMatch = F.mvRightToLeftMatch;
    K.mnMinX = (int)Frame::mnMinX;
    K.mnMaxX = (int)Frame::mnMaxX;
    K.mnMinY = (int)Frame::mnMinY;
    K.mnMaxY = (int)Frame::mnMaxY;
    K.mfGridElementWidthInv = Frame::mfGridElementWidthInv;
    K.mfGridElementHeightInv = Frame::mfGridElementHeightInv;
    K.mvScaleFactors = F.mvScaleFactors;
    K.mnScaleLevels = F.mnScaleLevels;
    K.mb = F.mb;
    K.mbf = F.mbf;
    K.mvpMapPoints.assign(K.N, nullptr);
}

// a SearchForTriangulation keyframe "A." / "B." (KFSide arrays); MapPoints where has_mp
inline void build_triang_kf(const Arrays &m, const std::string &pre, KeyFrame &K, std::vector<std::unique_ptr<MapPoint>> &pool)
{
    const Arr &d = get(m, pre + "desc");
    const int n = (int)(d.n / 32);
    K.N = n;
    K.NLeft = get(m, pre + "nleft").p<int32_t>()[0];
    static Camera second;
    K.mpCamera2 = get(m, pre + "two_cam").p<int32_t>()[0] ? &second : nullptr;
    K.mDescriptors = cv::Mat(n, 32);
    std::memcpy(K.mDescriptors.buf.data(), d.b.data(), d.b.size());
    std::vector<cv::KeyPoint> kps(n);
    for (int i = 0; i < n; i++) {
        kps[i].pt.x = get(m, pre + "kp_x").p<float>()[i];
        kps[i].pt.y = get(m, pre + "kp_y").p<float>()[i];
        kps[i].angle = get(m, pre + "kp_angle").p<float>()[i];
        kps[i].octave = get(m, pre + "kp_octave").p<int32_t>()[i];
    }
    const int nl = K.NLeft == -1 ? n : K.NLeft;
    if (K.NLeft == -1) {
        K.mvKeysUn = kps;
        K.mvKeys = kps;
    } else {  // mvKeysUn is not read on a rig: give it garbage positions to prove it
        K.mvKeys.assign(kps.begin(), kps.begin() + nl);
        K.mvKeysRight.assign(kps.begin() + nl, kps.end());
        K.mvKeysUn = K.mvKeys;
        for (auto &kp : K.mvKeysUn) kp.pt.x = -1e9f;
    }
    if (has(m, pre + "u_right")) {
        const Arr &u = get(m, pre + "u_right");
        K.mvuRight.assign(u.p<float>(), u.p<float>() + u.n);
    }
    const Arr &sc = get(m, pre + "scale"), &s2 = get(m, pre + "level_sigma2");
    K.mvScaleFactors.assign(sc.p<float>(), sc.p<float>() + sc.n);
    K.mvLevelSigma2.assign(s2.p<float>(), s2.p<float>() + s2.n);
    K.mvpMapPoints.assign(n, nullptr);
    for (int i = 0; i < n; i++)
        if (get(m, pre + "has_mp").p<uint8_t>()[i]) {
            pool.emplace_back(new MapPoint());
            pool.back()->mnId = (unsigned long)i;
            K.mvpMapPoints[i] = pool.back().get();
        }
    fill_featvec(m, pre, K.mFeatVec);
}

// A BA world from the graph arrays "G.*": one KeyFrame per pose (mnId = index, the shared camera
// "G.cam"), one MapPoint per point, one observation per edge (keypoint octave = its index in the
// KeyFrame, so mvInvLevelSigma2[octave] is the edge's weight; mvuRight = ur on stereo edges)
inline void build_ba_world(const Arrays &in, Map &map, Camera &c, std::vector<KeyFrame> &kf, std::vector<MapPoint> &mp)
{
    const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3), ne = (int)get(in, "G.e_pose").n;
    const float *cam = get(in, "G.cam").p<float>();
    c.type = (int)cam[0];
    c.params.assign(cam + 1, cam + 9);
    kf.resize(np);
    mp.resize(npt);
    for (int i = 0; i < np; i++) {
        kf[i].mnId = (unsigned long)i;
        kf[i].map = &map;
        std::memcpy(kf[i].pose, get(in, "G.pose").p<double>() + 7 * i, 56);
        kf[i].mpCamera = &c;
        kf[i].fx = cam[9];
        kf[i].fy = cam[10];
        kf[i].cx = cam[11];
        kf[i].cy = cam[12];
        kf[i].mbf = cam[13];
    }
    for (int j = 0; j < npt; j++) {
        mp[j].mnId = (unsigned long)j;
        mp[j].map = &map;
        std::memcpy(mp[j].pos, get(in, "G.point").p<double>() + 3 * j, 24);
    }
    for (int e = 0; e < ne; e++) {
        KeyFrame &k = kf[get(in, "G.e_pose").p<int32_t>()[e]];
        MapPoint &p = mp[get(in, "G.e_point").p<int32_t>()[e]];
        const double *o = get(in, "G.e_obs").p<double>() + 3 * e;
        cv::KeyPoint kp;
        kp.pt.x = (float)o[0];
        kp.pt.y = (float)o[1];
        kp.octave = (int)k.mvKeysUn.size();
        k.mvKeysUn.push_back(kp);
        k.mvInvLevelSigma2.push_back(get(in, "G.e_inv_sigma2").p<float>()[e]);
        k.mvuRight.push_back(get(in, "G.e_kind").p<uint8_t>()[e] == OSG_EDGE_STEREO ? (float)o[2] : -1.0f);
        k.mvpMapPoints.push_back(&p);
        p.obs[&k] = std::make_tuple(kp.octave, -1);
    }
}


// ------------------------------------------------------------- one problem per entry point
// Each reads the arrays of one problem under the name prefix `pre` (a batch file holds problems
// "b0.", "b1.", ...; a single-call file uses "").

// SearchByProjection(Frame&, vector<MapPoint*>): "F.*", "S.*", "Q.*"
inline void build_mps_problem(const Arrays &in, const std::string &pre, Frame &F, std::vector<MapPoint *> &q,
                              std::vector<std::unique_ptr<MapPoint>> &pool)
{
    build_frame(in, F, pre + "F.");
    build_slots(in, pre, F, pool);
    const std::string Q = pre + "Q.";
    const int nq = (int)get(in, Q + "mp_id").n;
    q.assign(nq, nullptr);
    for (int i = 0; i < nq; i++) {
        pool.emplace_back(new MapPoint());
        MapPoint *p = pool.back().get();
        p->mnId = (unsigned long)get(in, Q + "mp_id").p<int32_t>()[i];
        std::memcpy(p->desc.buf.data(), get(in, Q + "desc").p<uint8_t>() + 32 * i, 32);
        p->bad = !get(in, Q + "usable").p<uint8_t>()[i];
        p->nobs = get(in, Q + "has_obs").p<uint8_t>()[i];
        p->mbTrackInView = get(in, Q + "in_view").p<uint8_t>()[i];
        p->mTrackProjX = get(in, Q + "proj_x").p<float>()[i];
        p->mTrackProjY = get(in, Q + "proj_y").p<float>()[i];
        p->mTrackProjXR = get(in, Q + "proj_xr").p<float>()[i];
        p->mTrackViewCos = get(in, Q + "view_cos").p<float>()[i];
        p->mnTrackScaleLevel = get(in, Q + "pred_level").p<int32_t>()[i];
        p->mTrackDepth = get(in, Q + "track_depth").p<float>()[i];
        if (has(in, Q + "in_view_r")) {
            p->mbTrackInViewR = get(in, Q + "in_view_r").p<uint8_t>()[i];
            p->mTrackProjYR = get(in, Q + "proj_yr").p<float>()[i];
            p->mTrackViewCosR = get(in, Q + "view_cos_r").p<float>()[i];
            p->mnTrackScaleLevelR = get(in, Q + "pred_level_r").p<int32_t>()[i];
        }
        q[i] = p;
    }
}

// SearchByProjection(Frame&, const Frame&): "F.*", "S.*", "L.*"
inline void build_last_problem(const Arrays &in, const std::string &pre, Frame &CF, Frame &LF,
                               std::vector<std::unique_ptr<MapPoint>> &pool)
{
    build_frame(in, CF, pre + "F.");
    build_slots(in, pre, CF, pool);
    const std::string L = pre + "L.";
    const int n = (int)get(in, L + "mp_id").n;
    LF.N = n;
    LF.Nleft = -1;
    LF.mvKeysUn.resize(n);
    LF.mvpMapPoints.assign(n, nullptr);
    LF.mvbOutlier.assign(n, false);
    for (int i = 0; i < n; i++) {
        LF.mvKeysUn[i].octave = get(in, L + "octave").p<int32_t>()[i];
        LF.mvKeysUn[i].angle = get(in, L + "angle").p<float>()[i];
        const int id = get(in, L + "mp_id").p<int32_t>()[i];
        if (id < 0) continue;
        pool.emplace_back(new MapPoint());
        MapPoint *p = pool.back().get();
        p->mnId = (unsigned long)id;
        std::memcpy(p->desc.buf.data(), get(in, L + "desc").p<uint8_t>() + 32 * i, 32);
        p->nobs = get(in, L + "has_obs").p<uint8_t>()[i];
        p->proj_ok = true;
        p->proj_u = get(in, L + "u").p<float>()[i];
        p->proj_v = get(in, L + "v").p<float>()[i];
        p->proj_invz = get(in, L + "invz").p<float>()[i];
        if (has(in, L + "u_r")) {
            p->proj_ur = get(in, L + "u_r").p<float>()[i];
            p->proj_vr = get(in, L + "v_r").p<float>()[i];
        }
        LF.mvpMapPoints[i] = p;
        LF.mvbOutlier[i] = !get(in, L + "valid").p<uint8_t>()[i];
    }
    LF.mvKeys = LF.mvKeysUn;
}

// SearchByBoW(KeyFrame*, Frame&): "B1.*" (the KeyFrame), "B2.*" (the Frame side)
inline void build_bow_kf_f_problem(const Arrays &in, const std::string &pre, KeyFrame &K, Frame &F,
                                   std::vector<std::unique_ptr<MapPoint>> &pool)
{
    KeyFrame KF;
    build_bow_kf(in, pre + "B1.", K, pool);
    build_bow_kf(in, pre + "B2.", KF, pool);
    F.N = KF.N;  // the Frame side: descriptors, angles, FeatureVector
    F.Nleft = KF.NLeft;
    F.mDescriptors = KF.mDescriptors;
    F.mvKeys = KF.mvKeys;
    F.mvKeysUn = KF.mvKeysUn;
    F.mvKeysRight = KF.mvKeysRight;
    F.mpCamera2 = KF.mpCamera2;
    F.mFeatVec = KF.mFeatVec;
}

// PoseOptimization: "P.kind/xw/obs/inv_sigma2/pose/cam" (+ "P.cam2", "P.cam2_trl" with right-camera edges).  One
// slot per edge, octave = slot (one information level per keypoint).  A problem with right-camera
// (BODY) edges becomes a two-camera Frame: its other edges are the left slots, in edge order, then
// the BODY edges are the right slots.
inline void build_pose_problem(const Arrays &in, const std::string &pre, Frame &F, Camera &c, Camera &c2,
                               std::vector<std::unique_ptr<MapPoint>> &pool)
{
    const std::string P = pre + "P.";
    const int n = (int)get(in, P + "kind").n;
    const uint8_t *kind = get(in, P + "kind").p<uint8_t>();
    std::vector<int> order;
    for (int i = 0; i < n; i++)
        if (kind[i] != OSG_EDGE_BODY) order.push_back(i);
    const int nleft = (int)order.size();
    for (int i = 0; i < n; i++)
        if (kind[i] == OSG_EDGE_BODY) order.push_back(i);
    const bool two = nleft < n;
    F.N = n;
    F.Nleft = two ? nleft : -1;
    F.mvKeysUn.resize(two ? nleft : n);
    F.mvKeys.resize(two ? nleft : 0);
    F.mvKeysRight.resize(two ? n - nleft : 0);
    F.mvuRight.assign(n, -1.0f);
    F.mvInvLevelSigma2.resize(n);
    F.mvpMapPoints.assign(n, nullptr);
    F.mvbOutlier.assign(n, false);
    const double *obs = get(in, P + "obs").p<double>(), *xw = get(in, P + "xw").p<double>();
    for (int s = 0; s < n; s++) {
        const int i = order[s];
        pool.emplace_back(new MapPoint());
        std::memcpy(pool.back()->pos, xw + 3 * i, 24);
        F.mvpMapPoints[s] = pool.back().get();
        cv::KeyPoint kp;
        kp.pt.x = (float)obs[3 * i];
        kp.pt.y = (float)obs[3 * i + 1];
        kp.octave = s;
        if (!two) F.mvKeysUn[s] = kp;
        else if (s < nleft) F.mvKeys[s] = F.mvKeysUn[s] = kp;
        else F.mvKeysRight[s - nleft] = kp;
        F.mvInvLevelSigma2[s] = get(in, P + "inv_sigma2").p<float>()[i];
        if (kind[i] == OSG_EDGE_STEREO) F.mvuRight[s] = (float)obs[3 * i + 2];
    }
    std::memcpy(F.pose, get(in, P + "pose").b.data(), 56);
    const float *cam = get(in, P + "cam").p<float>();  // type p0..p7 fx fy cx cy bf
    c.type = (int)cam[0];
    c.params.assign(cam + 1, cam + 9);
    F.mpCamera = &c;
    F.fx = cam[9];
    F.fy = cam[10];
    F.cx = cam[11];
    F.cy = cam[12];
    F.mbf = cam[13];
    if (two) {
        const float *k2 = get(in, P + "cam2").p<float>();
        c2.type = (int)k2[0];
        c2.params.assign(k2 + 1, k2 + 9);
        if (has(in, P + "cam2_trl")) c2.trl.assign(get(in, P + "cam2_trl").p<double>(), get(in, P + "cam2_trl").p<double>() + 7);
        F.mpCamera2 = &c2;
    }
}

// ComputeStereoMatches: left "S.x/y/oct/desc", right "S.xr/yr/oct_r/desc_r", "S.scale", "S.inv_scale",
// "S.mb_mbf"; pyramids "PL.img" / "PR.img" (levels concatenated) with "PL.dims" / "PR.dims"
// (rows, cols) held as ROIs of wider rows (step = cols + 7), as ORBextractor's bordered levels are
inline void build_stereo_problem(const Arrays &in, const std::string &pre, Frame &F, ORBextractor &el,
                                 ORBextractor &er)
{
    const std::string S = pre + "S.";
    const int n = (int)get(in, S + "x").n, nr = (int)get(in, S + "xr").n;
    F.N = n;
    auto kps = [&](const std::string &x, const std::string &y, const std::string &o, int cnt) {
        std::vector<cv::KeyPoint> v(cnt);
        for (int i = 0; i < cnt; i++) {
            v[i].pt.x = get(in, x).p<float>()[i];
            v[i].pt.y = get(in, y).p<float>()[i];
            v[i].octave = get(in, o).p<int32_t>()[i];
        }
        return v;
    };
    F.mvKeys = kps(S + "x", S + "y", S + "oct", n);
    F.mvKeysRight = kps(S + "xr", S + "yr", S + "oct_r", nr);
    F.mDescriptors = cv::Mat(n, 32);
    std::memcpy(F.mDescriptors.buf.data(), get(in, S + "desc").b.data(), (size_t)n * 32);
    F.mDescriptorsRight = cv::Mat(nr, 32);
    std::memcpy(F.mDescriptorsRight.buf.data(), get(in, S + "desc_r").b.data(), (size_t)nr * 32);
    const Arr &sc = get(in, S + "scale"), &isc = get(in, S + "inv_scale");
    F.mvScaleFactors.assign(sc.p<float>(), sc.p<float>() + sc.n);
    F.mvInvScaleFactors.assign(isc.p<float>(), isc.p<float>() + isc.n);
    F.mnScaleLevels = (int)sc.n;
    F.mb = get(in, S + "mb_mbf").p<float>()[0];
    F.mbf = get(in, S + "mb_mbf").p<float>()[1];
    auto pyr = [&](const std::string &img, const std::string &dims, ORBextractor &e) {
        const uint8_t *src = get(in, img).p<uint8_t>();
        const int32_t *d = get(in, dims).p<int32_t>();
        e.mvImagePyramid.clear();
        for (size_t l = 0; l < sc.n; l++) {
            const int rows = d[2 * l], cols = d[2 * l + 1];
            cv::Mat m(rows, cols, (size_t)cols + 7);
            for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), src + (size_t)r * cols, cols);
            src += (size_t)rows * cols;
            e.mvImagePyramid.push_back(std::move(m));
        }
    };
    pyr(pre + "PL.img", pre + "PL.dims", el);
    pyr(pre + "PR.img", pre + "PR.dims", er);
    F.mpORBextractorLeft = &el;
    F.mpORBextractorRight = &er;
}

// ComputeBoW: a Frame whose mDescriptors are "D.desc" (n x 32)
inline void build_bow_frame(const Arrays &in, const std::string &pre, Frame &F)
{
    const Arr &d = get(in, pre + "D.desc");
    F.N = (int)(d.n / 32);
    F.mDescriptors = cv::Mat(F.N, 32);
    std::memcpy(F.mDescriptors.buf.data(), d.b.data(), d.b.size());
}

// the vocabulary "V.*" uploaded on this thread's context (the integration loads it once)
inline osg_vocabulary *build_vocabulary(const Arrays &in)
{
    const int32_t *kl = get(in, "V.kl").p<int32_t>();
    osg_vocabulary_desc v{};
    v.k = kl[0];
    v.L = kl[1];
    v.scoring = kl[2];
    v.weighting = kl[3];
    v.n_nodes = (int32_t)get(in, "V.parent").n;
    v.parent = get(in, "V.parent").p<int32_t>();
    v.is_leaf = get(in, "V.is_leaf").p<uint8_t>();
    v.desc = get(in, "V.desc").p<uint8_t>();
    v.weight = get(in, "V.weight").p<double>();
    osg_vocabulary *voc = nullptr;
    osg_ctx *ctx = osg_orbslam3::thread_ctx();
    if (!ctx || osg_vocabulary_create(ctx, &v, &voc) != OSG_OK) throw std::runtime_error("osg_vocabulary_create failed");
    return voc;
}

// mBowVec / mFeatVec of frames appended as flat arrays (word, value, node_id, node_start per frame
// with its own leading 0, feat) with per-frame counts
inline void append_bow(const Frame &F, std::vector<int32_t> &word, std::vector<double> &value,
                       std::vector<int32_t> &node_id, std::vector<int32_t> &node_start, std::vector<int32_t> &feat,
                       std::vector<int32_t> &counts)
{
    for (const auto &kv : F.mBowVec) {
        word.push_back((int32_t)kv.first);
        value.push_back(kv.second);
    }
    int s = 0;
    for (const auto &kv : F.mFeatVec) {
        node_id.push_back((int32_t)kv.first);
        node_start.push_back(s);
        for (unsigned f : kv.second) feat.push_back((int32_t)f);
        s += (int)kv.second.size();
    }
    node_start.push_back(s);
    counts.push_back((int32_t)F.mBowVec.size());
    counts.push_back((int32_t)F.mFeatVec.size());
}

#endif
