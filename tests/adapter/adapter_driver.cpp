// adapter_driver.cpp — runs adapters/orbslam3/osg_orbslam3.h on mock ORB-SLAM3 objects built from
// arrays written by tests/test_adapter.py, and writes the adapter's results back (test-only).
//
//   adapter_driver MODE in.arrays out.arrays      MODE: mps last kf bow_kf_f bow_kf_kf pose lba fuse fuse_sim3 triang distinct sim3 sim3_kfs sim3pair init stereo fisheye gba merge_lba orb
//
// Array file: repeated {u32 name_len, name, u8 dtype ('b' u8, 'i' i32, 'f' f32, 'd' f64), u64 count,
// data}.
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

static Arrays read_arrays(const char *path)
{
    Arrays m;
    FILE *f = fopen(path, "rb");
    if (!f) throw std::runtime_error(std::string("cannot open ") + path);
    for (;;) {
        uint32_t len;
        if (fread(&len, 4, 1, f) != 1) break;
        std::string name(len, '\0');
        fread(&name[0], 1, len, f);
        Arr a;
        fread(&a.t, 1, 1, f);
        uint64_t n;
        fread(&n, 8, 1, f);
        a.n = n;
        const size_t es = a.t == 'b' ? 1 : a.t == 'd' ? 8 : 4;
        a.b.resize(n * es);
        if (n) fread(a.b.data(), es, n, f);
        m[name] = std::move(a);
    }
    fclose(f);
    return m;
}

static void write_arrays(const char *path, const Arrays &m)
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
static Arr make(char t, const std::vector<T> &v)
{
    Arr a;
    a.t = t;
    a.n = v.size();
    a.b.resize(v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(a.b.data(), v.data(), a.b.size());
    return a;
}

static const Arr &get(const Arrays &m, const std::string &k)
{
    auto it = m.find(k);
    if (it == m.end()) throw std::runtime_error("missing array " + k);
    return it->second;
}

static bool has(const Arrays &m, const std::string &k) { return m.count(k) != 0; }

static void fill_grid(const Arrays &m, const std::string &pre, std::vector<std::size_t> (&grid)[OSG_GRID_COLS][OSG_GRID_ROWS])
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
static void build_frame(const Arrays &m, Frame &F, const std::string &P = "F.")
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
static void build_slots(const Arrays &m, Frame &F, std::vector<std::unique_ptr<MapPoint>> &pool)
{
    const int32_t *sm = get(m, "S.slot_mp").p<int32_t>();
    const uint8_t *st = has(m, "S.slot_taken") ? get(m, "S.slot_taken").p<uint8_t>() : nullptr;
    for (int i = 0; i < F.N; i++)
        if (sm[i] >= 0) {
            pool.emplace_back(new MapPoint());
            pool.back()->mnId = (unsigned long)sm[i];
            pool.back()->nobs = st ? st[i] : 1;
            F.mvpMapPoints[i] = pool.back().get();
        }
}

static std::vector<int32_t> slot_ids(const std::vector<MapPoint *> &v)
{
    std::vector<int32_t> r(v.size(), -1);
    for (size_t i = 0; i < v.size(); i++)
        if (v[i]) r[i] = (int32_t)v[i]->mnId;
    return r;
}

static void fill_featvec(const Arrays &m, const std::string &pre, std::map<unsigned int, std::vector<unsigned int>> &fv)
{
    const Arr &nid = get(m, pre + "node_id"), &ns = get(m, pre + "node_start"), &ft = get(m, pre + "feat");
    for (size_t k = 0; k < nid.n; k++) {
        auto &v = fv[nid.p<uint32_t>()[k]];
        for (int j = ns.p<int32_t>()[k]; j < ns.p<int32_t>()[k + 1]; j++) v.push_back((unsigned)ft.p<int32_t>()[j]);
    }
}

// a BoW side "B1." / "B2." as a KeyFrame with MapPoints (mnId = mp_id, bad = !mp_good)
static void build_bow_kf(const Arrays &m, const std::string &pre, KeyFrame &K, std::vector<std::unique_ptr<MapPoint>> &pool)
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
static void build_kf_frame(const Arrays &m, KeyFrame &K)
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
static void build_triang_kf(const Arrays &m, const std::string &pre, KeyFrame &K, std::vector<std::unique_ptr<MapPoint>> &pool)
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
static void build_ba_world(const Arrays &in, Map &map, Camera &c, std::vector<KeyFrame> &kf, std::vector<MapPoint> &mp)
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

int main(int argc, char **argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s MODE in out\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    try {
        const Arrays in = read_arrays(argv[2]);
        Arrays out;
        std::vector<std::unique_ptr<MapPoint>> pool;
        const float *prm = has(in, "params") ? get(in, "params").p<float>() : nullptr;
        if (mode == "mps") {
            Frame F;
            build_frame(in, F);
            build_slots(in, F, pool);
            const int nq = (int)get(in, "Q.mp_id").n;
            std::vector<MapPoint *> q(nq);
            for (int i = 0; i < nq; i++) {
                pool.emplace_back(new MapPoint());
                MapPoint *p = pool.back().get();
                p->mnId = (unsigned long)get(in, "Q.mp_id").p<int32_t>()[i];
                std::memcpy(p->desc.buf.data(), get(in, "Q.desc").p<uint8_t>() + 32 * i, 32);
                p->bad = !get(in, "Q.usable").p<uint8_t>()[i];
                p->nobs = get(in, "Q.has_obs").p<uint8_t>()[i];
                p->mbTrackInView = get(in, "Q.in_view").p<uint8_t>()[i];
                p->mTrackProjX = get(in, "Q.proj_x").p<float>()[i];
                p->mTrackProjY = get(in, "Q.proj_y").p<float>()[i];
                p->mTrackProjXR = get(in, "Q.proj_xr").p<float>()[i];
                p->mTrackViewCos = get(in, "Q.view_cos").p<float>()[i];
                p->mnTrackScaleLevel = get(in, "Q.pred_level").p<int32_t>()[i];
                p->mTrackDepth = get(in, "Q.track_depth").p<float>()[i];
                if (has(in, "Q.in_view_r")) {
                    p->mbTrackInViewR = get(in, "Q.in_view_r").p<uint8_t>()[i];
                    p->mTrackProjYR = get(in, "Q.proj_yr").p<float>()[i];
                    p->mTrackViewCosR = get(in, "Q.view_cos_r").p<float>()[i];
                    p->mnTrackScaleLevelR = get(in, "Q.pred_level_r").p<int32_t>()[i];
                }
                q[i] = p;
            }
            // params: nnratio th far thfar
            const int nm = osg_orbslam3::search_by_projection_mps<MockHooks>(F, q, prm[1], prm[2] != 0, prm[3], prm[0]);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(F.mvpMapPoints));
        } else if (mode == "last") {
            Frame CF, LF;
            build_frame(in, CF);
            build_slots(in, CF, pool);
            const int n = (int)get(in, "L.mp_id").n;
            LF.N = n;
            LF.Nleft = -1;
            LF.mvKeysUn.resize(n);
            LF.mvpMapPoints.assign(n, nullptr);
            LF.mvbOutlier.assign(n, false);
            for (int i = 0; i < n; i++) {
                LF.mvKeysUn[i].octave = get(in, "L.octave").p<int32_t>()[i];
                LF.mvKeysUn[i].angle = get(in, "L.angle").p<float>()[i];
                const int id = get(in, "L.mp_id").p<int32_t>()[i];
                if (id < 0) continue;
                pool.emplace_back(new MapPoint());
                MapPoint *p = pool.back().get();
                p->mnId = (unsigned long)id;
                std::memcpy(p->desc.buf.data(), get(in, "L.desc").p<uint8_t>() + 32 * i, 32);
                p->nobs = get(in, "L.has_obs").p<uint8_t>()[i];
                p->proj_ok = true;
                p->proj_u = get(in, "L.u").p<float>()[i];
                p->proj_v = get(in, "L.v").p<float>()[i];
                p->proj_invz = get(in, "L.invz").p<float>()[i];
                if (has(in, "L.u_r")) {
                    p->proj_ur = get(in, "L.u_r").p<float>()[i];
                    p->proj_vr = get(in, "L.v_r").p<float>()[i];
                }
                LF.mvpMapPoints[i] = p;
                LF.mvbOutlier[i] = !get(in, "L.valid").p<uint8_t>()[i];
            }
            LF.mvKeys = LF.mvKeysUn;
            CF.tlc_z_value = prm[3];
            // params: th mono ori tlc_z
            const int nm = osg_orbslam3::search_by_projection_last<MockHooks>(CF, LF, prm[0], prm[1] != 0, prm[2] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(CF.mvpMapPoints));
        } else if (mode == "kf") {
            Frame CF;
            build_frame(in, CF);
            build_slots(in, CF, pool);
            KeyFrame K;
            const int n = (int)get(in, "K.mp_id").n;
            K.N = n;
            K.mvKeysUn.resize(n);
            K.mvpMapPoints.assign(n, nullptr);
            for (int i = 0; i < n; i++) {
                K.mvKeysUn[i].angle = get(in, "K.angle").p<float>()[i];
                pool.emplace_back(new MapPoint());
                MapPoint *p = pool.back().get();
                p->mnId = (unsigned long)get(in, "K.mp_id").p<int32_t>()[i];
                std::memcpy(p->desc.buf.data(), get(in, "K.desc").p<uint8_t>() + 32 * i, 32);
                p->proj_ok = get(in, "K.valid").p<uint8_t>()[i];
                p->proj_u = get(in, "K.u").p<float>()[i];
                p->proj_v = get(in, "K.v").p<float>()[i];
                p->proj_level = get(in, "K.pred_level").p<int32_t>()[i];
                K.mvpMapPoints[i] = p;
            }
            std::set<MapPoint *> already;
            // params: th orbdist ori
            const int nm = osg_orbslam3::search_by_projection_kf<MockHooks>(CF, &K, already, prm[0], (int)prm[1], prm[2] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["slot_mp"] = make('i', slot_ids(CF.mvpMapPoints));
        } else if (mode == "bow_kf_f") {
            KeyFrame K, KF;
            build_bow_kf(in, "B1.", K, pool);
            build_bow_kf(in, "B2.", KF, pool);
            Frame F;  // the Frame side: descriptors, angles, FeatureVector
            F.N = KF.N;
            F.Nleft = KF.NLeft;
            F.mDescriptors = KF.mDescriptors;
            F.mvKeys = KF.mvKeys;
            F.mvKeysUn = KF.mvKeysUn;
            F.mvKeysRight = KF.mvKeysRight;
            F.mpCamera2 = KF.mpCamera2;
            F.mFeatVec = KF.mFeatVec;
            std::vector<MapPoint *> matches;
            // params: nnratio ori
            const int nm = osg_orbslam3::search_by_bow_kf_f<MockHooks>(&K, F, matches, prm[0], prm[1] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["out_mp"] = make('i', slot_ids(matches));
        } else if (mode == "bow_kf_kf") {
            KeyFrame K1, K2;
            build_bow_kf(in, "B1.", K1, pool);
            build_bow_kf(in, "B2.", K2, pool);
            std::vector<MapPoint *> matches;
            const int nm = osg_orbslam3::search_by_bow_kf_kf<MockHooks>(&K1, &K2, matches, prm[0], prm[1] != 0);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["out_mp"] = make('i', slot_ids(matches));
        } else if (mode == "pose") {
            Frame F;
            const int n = (int)get(in, "P.kind").n;
            F.N = n;
            F.Nleft = -1;
            F.mvKeysUn.resize(n);
            F.mvuRight.assign(n, -1.0f);
            F.mvInvLevelSigma2.resize(n);
            F.mvpMapPoints.assign(n, nullptr);
            F.mvbOutlier.assign(n, false);
            const double *obs = get(in, "P.obs").p<double>(), *xw = get(in, "P.xw").p<double>();
            for (int i = 0; i < n; i++) {
                pool.emplace_back(new MapPoint());
                std::memcpy(pool.back()->pos, xw + 3 * i, 24);
                F.mvpMapPoints[i] = pool.back().get();
                F.mvKeysUn[i].pt.x = (float)obs[3 * i];
                F.mvKeysUn[i].pt.y = (float)obs[3 * i + 1];
                F.mvKeysUn[i].octave = i;  // one information level per keypoint
                F.mvInvLevelSigma2[i] = get(in, "P.inv_sigma2").p<float>()[i];
                if (get(in, "P.kind").p<uint8_t>()[i] == OSG_EDGE_STEREO) F.mvuRight[i] = (float)obs[3 * i + 2];
            }
            std::memcpy(F.pose, get(in, "P.pose").b.data(), 56);
            const float *cam = get(in, "P.cam").p<float>();  // type p0..p7 fx fy cx cy bf
            Camera c;
            c.type = (int)cam[0];
            c.params.assign(cam + 1, cam + 9);
            F.mpCamera = &c;
            F.fx = cam[9];
            F.fy = cam[10];
            F.cx = cam[11];
            F.cy = cam[12];
            F.mbf = cam[13];
            ProbeMutex probe;  // params[0] != 0: pass a MapPoint::mGlobalMutex stand-in and report its use
            const bool use_probe = prm && prm[0] != 0;
            if (use_probe) g_probe = &probe;
            const int inl = use_probe ? osg_orbslam3::pose_optimization<MockHooks>(&F, &probe)
                                      : osg_orbslam3::pose_optimization<MockHooks>(&F);
            g_probe = nullptr;
            out["lock_stats"] = make('i', std::vector<int32_t>{probe.locks, g_gather_unlocked, g_apply_locked,
                                                               g_apply_try_lock_failed, (int32_t)probe.held});
            std::vector<uint8_t> outl(n);
            for (int i = 0; i < n; i++) outl[i] = F.mvbOutlier[i];
            out["n_inliers"] = make('i', std::vector<int32_t>{inl});
            out["pose"] = make('d', std::vector<double>(F.pose, F.pose + 7));
            out["outlier"] = make('b', outl);
        } else if (mode == "lba") {
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3), ne = (int)get(in, "G.e_pose").n;
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::list<KeyFrame *> local, fixedc;
            const uint8_t *fx = get(in, "G.pose_fixed").p<uint8_t>();
            for (int i = 0; i < np; i++) (fx[i] ? fixedc : local).push_back(&kf[i]);
            std::list<MapPoint *> mps;
            for (auto &p : mp) mps.push_back(&p);
            bool stop = false;
            // optional: params[0] = the map's init KeyFrame id (default none); "G.mp_bad" = MapPoints
            // another thread marks bad while the solve runs (in the graph, skipped at classification)
            const unsigned long init_id = prm ? (unsigned long)prm[0] : ~0ul;
            if (has(in, "G.mp_bad"))
                for (int j = 0; j < npt; j++) mp[j].bad = get(in, "G.mp_bad").p<uint8_t>()[j] != 0;
            auto o = osg_orbslam3::local_bundle_adjustment<MockHooks>(local, fixedc, mps, &map, init_id, &stop, false);
            std::vector<uint8_t> bad(ne, 0);
            std::vector<int32_t> erased;
            {
                std::map<std::pair<KeyFrame *, MapPoint *>, int> edge_of;
                for (int e = 0; e < ne; e++)
                    edge_of[{&kf[get(in, "G.e_pose").p<int32_t>()[e]], &mp[get(in, "G.e_point").p<int32_t>()[e]]}] = e;
                for (auto &km : o.to_erase) {
                    bad[edge_of[km]] = 1;
                    erased.push_back(edge_of[km]);
                }
            }
            out["erased"] = make('i', erased);
            out["counts"] = make('i', std::vector<int32_t>{o.num_fixedKF, o.num_OptKF, o.num_MPs, o.num_edges});
            osg_orbslam3::apply_local_bundle_adjustment<MockHooks>(o);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt);
            for (int i = 0; i < np; i++) std::memcpy(&pose[7 * i], kf[i].pose, 56);
            for (int j = 0; j < npt; j++) std::memcpy(&point[3 * j], mp[j].pos, 24);
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["edge_bad"] = make('b', bad);
            out["num_edges"] = make('i', std::vector<int32_t>{o.num_edges});
        } else if (mode == "merge_lba") {
            // the "lba" arrays; params: n_fixed stop.  vpFixedKF = KeyFrames [0, n_fixed), vpAdjustKF the
            // rest, pMainKF the last; out: poses, points, the erased (KeyFrame, MapPoint) pairs in order
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3);
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::vector<KeyFrame *> fixedk, adjust;
            for (int i = 0; i < np; i++) (i < (int)prm[0] ? fixedk : adjust).push_back(&kf[i]);
            bool stop = prm[1] != 0;
            auto o = osg_orbslam3::merge_local_bundle_adjustment<MockHooks, KeyFrame, MapPoint>(&kf[np - 1], adjust,
                                                                                             fixedk, &stop);
            std::vector<int32_t> erased;
            for (auto &km : o.to_erase) {
                erased.push_back((int32_t)(km.first - kf.data()));
                erased.push_back((int32_t)(km.second - mp.data()));
            }
            if (!o.aborted) osg_orbslam3::apply_merge_local_bundle_adjustment<MockHooks>(o);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt);
            for (int i = 0; i < np; i++) std::memcpy(&pose[7 * i], kf[i].pose, 56);
            for (int j = 0; j < npt; j++) std::memcpy(&point[3 * j], mp[j].pos, 24);
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["erased"] = make('i', erased);
            out["aborted"] = make('i', std::vector<int32_t>{(int32_t)o.aborted});
        } else if (mode == "gba") {
            // the "lba" arrays; params: nIterations bRobust nLoopKF.  KeyFrame 0 is the map's init and
            // origin KeyFrame: nLoopKF 0 writes into the map, anything else into mTcwGBA / mPosGBA
            const int np = (int)(get(in, "G.pose").n / 7), npt = (int)(get(in, "G.point").n / 3);
            Camera c;
            Map map;
            std::vector<KeyFrame> kf;
            std::vector<MapPoint> mp;
            build_ba_world(in, map, c, kf, mp);
            std::vector<KeyFrame *> vk;
            std::vector<MapPoint *> vm;
            for (auto &k : kf) vk.push_back(&k);
            for (auto &p : mp) vm.push_back(&p);
            bool stop = false;
            const unsigned long nLoop = (unsigned long)prm[2];
            auto o = osg_orbslam3::bundle_adjustment<MockHooks>(vk, vm, 0ul, (int)prm[0], &stop, prm[1] != 0);
            osg_orbslam3::apply_bundle_adjustment<MockHooks>(o, nLoop, nLoop == 0);
            std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)npt), pose_gba(7 * (size_t)np),
                point_gba(3 * (size_t)npt);
            std::vector<int32_t> ba_for;
            for (int i = 0; i < np; i++) {
                std::memcpy(&pose[7 * i], kf[i].pose, 56);
                std::memcpy(&pose_gba[7 * i], kf[i].pose_gba, 56);
                ba_for.push_back((int32_t)kf[i].mnBAGlobalForKF);
            }
            for (int j = 0; j < npt; j++) {
                std::memcpy(&point[3 * j], mp[j].pos, 24);
                std::memcpy(&point_gba[3 * j], mp[j].pos_gba, 24);
                ba_for.push_back((int32_t)mp[j].mnBAGlobalForKF);
            }
            out["pose"] = make('d', pose);
            out["point"] = make('d', point);
            out["pose_gba"] = make('d', pose_gba);
            out["point_gba"] = make('d', point_gba);
            out["ba_for"] = make('i', ba_for);
            out["iterations"] = make('i', std::vector<int32_t>{o.iterations});
        } else if (mode == "fuse" || mode == "fuse_sim3") {
            // pool of MapPoints "P.*" (index = id), the keyframe's slot occupants "K.slot_mp", the
            // list to fuse "L.list" (pool indices, -1 = NULL); params: th right
            KeyFrame K;
            build_kf_frame(in, K);
            const Arr &is2 = get(in, "K.inv_s2");
            K.mvInvLevelSigma2.assign(is2.p<float>(), is2.p<float>() + is2.n);
            const int np = (int)get(in, "P.nobs").n;
            std::vector<MapPoint> P(np);
            for (int i = 0; i < np; i++) {
                MapPoint &p = P[i];
                p.mnId = (unsigned long)i;
                std::memcpy(p.desc.buf.data(), get(in, "P.desc").p<uint8_t>() + 32 * i, 32);
                p.proj_ok = get(in, "P.ok").p<uint8_t>()[i];
                p.proj_u = get(in, "P.u").p<float>()[i];
                p.proj_v = get(in, "P.v").p<float>()[i];
                p.proj_fuse_ur = get(in, "P.ur").p<float>()[i];
                p.proj_level = get(in, "P.level").p<int32_t>()[i];
                p.bad = get(in, "P.bad").p<uint8_t>()[i];
                p.nobs = get(in, "P.nobs").p<int32_t>()[i];
            }
            const int32_t *sm = get(in, "K.slot_mp").p<int32_t>();
            for (int k = 0; k < K.N; k++)
                if (sm[k] >= 0) {
                    K.mvpMapPoints[k] = &P[sm[k]];
                    P[sm[k]].obs[&K] = std::make_tuple(k, -1);
                }
            const Arr &L = get(in, "L.list");
            std::vector<MapPoint *> list(L.n);
            for (size_t i = 0; i < L.n; i++) list[i] = L.p<int32_t>()[i] < 0 ? nullptr : &P[L.p<int32_t>()[i]];
            int nf;
            std::vector<int32_t> repl(L.n, -1);
            if (mode == "fuse") {
                nf = osg_orbslam3::fuse<MockHooks>(&K, list, prm[0], prm[1] != 0);
            } else {
                std::vector<MapPoint *> vpReplace(L.n, nullptr);
                nf = osg_orbslam3::fuse_sim3<MockHooks>(&K, Sim3{}, list, prm[0], vpReplace);
                for (size_t i = 0; i < L.n; i++) repl[i] = vpReplace[i] ? (int32_t)vpReplace[i]->mnId : -1;
            }
            std::vector<uint8_t> bad(np);
            std::vector<int32_t> nobs(np);
            for (int i = 0; i < np; i++) {
                bad[i] = P[i].bad;
                nobs[i] = P[i].nobs;
            }
            out["nfused"] = make('i', std::vector<int32_t>{nf});
            out["slot_mp"] = make('i', slot_ids(K.mvpMapPoints));
            out["bad"] = make('b', bad);
            out["nobs"] = make('i', nobs);
            out["replace"] = make('i', repl);
        } else if (mode == "triang") {
            // keyframes "A." / "B.", geometry "G.geom" {ep_x, ep_y, F12[36], pinhole}; params: only_stereo coarse ori
            KeyFrame A, B;
            build_triang_kf(in, "A.", A, pool);
            build_triang_kf(in, "B.", B, pool);
            const float *g = get(in, "G.geom").p<float>();
            A.triang_geom.ep_x = g[0];
            A.triang_geom.ep_y = g[1];
            std::memcpy(A.triang_geom.F12, g + 2, sizeof(float) * 36);
            A.triang_geom.pinhole = g[38] != 0;
            if (has(in, "G.kb8")) {  // KannalaBrandt8: R12[36] t12[12] kb[32]
                const float *k = get(in, "G.kb8").p<float>();
                std::memcpy(A.triang_geom.R12, k, sizeof(float) * 36);
                std::memcpy(A.triang_geom.t12, k + 36, sizeof(float) * 12);
                std::memcpy(A.triang_geom.kb, k + 48, sizeof(float) * 32);
            }
            std::vector<std::pair<size_t, size_t>> pairs;
            const int nm = osg_orbslam3::search_for_triangulation<MockHooks>(&A, &B, pairs, prm[0] != 0, prm[1] != 0,
                                                                              prm[2] != 0);
            std::vector<int32_t> flat;
            for (auto &pr : pairs) {
                flat.push_back((int32_t)pr.first);
                flat.push_back((int32_t)pr.second);
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["pairs"] = make('i', flat);
        } else if (mode == "sim3" || mode == "sim3_kfs") {
            // keyframe "F.*"; MapPoint pool "P.*" (desc ok u v level bad); "L.list" pool indices;
            // "V.matched" initial vpMatched (pool index, -1); params: th ratio
            KeyFrame K;
            build_kf_frame(in, K);
            const int np = (int)get(in, "P.bad").n;
            std::vector<MapPoint> P(np);
            for (int i = 0; i < np; i++) {
                MapPoint &p = P[i];
                p.mnId = (unsigned long)i;
                std::memcpy(p.desc.buf.data(), get(in, "P.desc").p<uint8_t>() + 32 * i, 32);
                p.proj_ok = get(in, "P.ok").p<uint8_t>()[i];
                p.proj_u = get(in, "P.u").p<float>()[i];
                p.proj_v = get(in, "P.v").p<float>()[i];
                p.proj_level = get(in, "P.level").p<int32_t>()[i];
                p.bad = get(in, "P.bad").p<uint8_t>()[i];
            }
            const Arr &L = get(in, "L.list");
            std::vector<MapPoint *> list(L.n);
            std::vector<KeyFrame> owners(7);
            std::vector<KeyFrame *> list_kfs(L.n);
            for (size_t i = 0; i < L.n; i++) {
                list[i] = &P[L.p<int32_t>()[i]];
                list_kfs[i] = &owners[i % 7];
            }
            std::vector<MapPoint *> matched(K.N, nullptr);
            std::vector<KeyFrame *> matched_kf(K.N, nullptr);
            for (int k = 0; k < K.N; k++) {
                const int32_t m = get(in, "V.matched").p<int32_t>()[k];
                if (m >= 0) matched[k] = &P[m];
            }
            int nm;
            if (mode == "sim3")
                nm = osg_orbslam3::search_by_projection_sim3<MockHooks, KeyFrame>(&K, Sim3{}, list, nullptr, matched,
                                                                                 nullptr, (int)prm[0], prm[1]);
            else
                nm = osg_orbslam3::search_by_projection_sim3<MockHooks, KeyFrame>(&K, Sim3{}, list, &list_kfs, matched,
                                                                                 &matched_kf, (int)prm[0], prm[1]);
            std::vector<int32_t> mo(K.N, -1), mk(K.N, -1);
            for (int k = 0; k < K.N; k++) {
                if (matched[k]) mo[k] = (int32_t)matched[k]->mnId;
                if (matched_kf[k]) mk[k] = (int32_t)(matched_kf[k] - owners.data());
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["matched"] = make('i', mo);
            out["matched_kf"] = make('i', mk);
        } else if (mode == "sim3pair") {
            // SearchBySim3: keyframes "F.*" (KF1) and "G.*" (KF2); per KF1 slot "A.*" (has desc ok u v level
            // bad) of its MapPoint projected into KF2, per KF2 slot "B.*" likewise into KF1; "V.matched":
            // initial vpMatches12 as KF2 slot indices (-1); params: th.  out: matched (KF2 slot or -1)
            KeyFrame K1, K2;
            build_kf_frame(in, K1);
            {
                Arrays g;
                for (auto &kv : in)
                    if (kv.first.rfind("G.", 0) == 0) g["F." + kv.first.substr(2)] = kv.second;
                build_kf_frame(g, K2);
            }
            std::vector<MapPoint> P1(K1.N), P2(K2.N);
            auto fill = [&](const char *pre, std::vector<MapPoint> &P, KeyFrame &K, KeyFrame &other, int d) {
                const std::string a(pre);
                for (int i = 0; i < K.N; i++) {
                    MapPoint &p = P[i];
                    if (!get(in, a + "has").p<uint8_t>()[i]) continue;
                    std::memcpy(p.desc.buf.data(), get(in, a + "desc").p<uint8_t>() + 32 * i, 32);
                    p.s3_ok[d] = get(in, a + "ok").p<uint8_t>()[i];
                    p.s3_u[d] = get(in, a + "u").p<float>()[i];
                    p.s3_v[d] = get(in, a + "v").p<float>()[i];
                    p.s3_level[d] = get(in, a + "level").p<int32_t>()[i];
                    p.bad = get(in, a + "bad").p<uint8_t>()[i];
                    p.obs[&K] = std::make_tuple(i, -1);
                    K.mvpMapPoints[i] = &p;
                }
                (void)other;
            };
            fill("A.", P1, K1, K2, 0);
            fill("B.", P2, K2, K1, 1);
            std::vector<MapPoint *> m12(K1.N, nullptr);
            for (int i = 0; i < K1.N; i++) {
                const int32_t j = get(in, "V.matched").p<int32_t>()[i];
                if (j >= 0) {
                    m12[i] = &P2[j];
                    P2[j].obs[&K2] = std::make_tuple(j, -1);
                }
            }
            const int nm = osg_orbslam3::search_by_sim3<MockHooks, KeyFrame>(&K1, &K2, m12, Sim3{}, prm[0]);
            std::vector<int32_t> mo(K1.N, -1);
            for (int i = 0; i < K1.N; i++)
                if (m12[i]) mo[i] = (int32_t)(m12[i] - P2.data());
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["matched"] = make('i', mo);
        } else if (mode == "init") {
            // F1 "F.*", F2 "G.*", vbPrevMatched "V.prev" (n1 x 2); params: windowSize nnratio checkOri
            Frame F1, F2;
            build_frame(in, F1, "F.");
            build_frame(in, F2, "G.");
            const Arr &pv = get(in, "V.prev");
            std::vector<cv::Point2f> prev(F1.N);
            for (int i = 0; i < F1.N; i++) {
                prev[i].x = pv.p<float>()[2 * i];
                prev[i].y = pv.p<float>()[2 * i + 1];
            }
            std::vector<int> m12;
            const int nm = osg_orbslam3::search_for_initialization<MockHooks>(F1, F2, prev, m12, (int)prm[0], prm[1],
                                                                               prm[2] != 0);
            std::vector<float> po(2 * (size_t)F1.N);
            for (int i = 0; i < F1.N; i++) {
                po[2 * i] = prev[i].x;
                po[2 * i + 1] = prev[i].y;
            }
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["m12"] = make('i', std::vector<int32_t>(m12.begin(), m12.end()));
            out["prev"] = make('f', po);
        } else if (mode == "stereo") {
            // left "S.x/y/oct/desc", right "S.xr/yr/oct_r/desc_r", "S.scale", "S.inv_scale", "S.mb_mbf";
            // pyramids "PL.img" / "PR.img" (levels concatenated) with "PL.dims" / "PR.dims" (rows, cols)
            // held as ROIs of wider rows (step = cols + 7), as ORBextractor's bordered levels are
            Frame F;
            const int n = (int)get(in, "S.x").n, nr = (int)get(in, "S.xr").n;
            F.N = n;
            auto kps = [&](const char *x, const char *y, const char *o, int cnt) {
                std::vector<cv::KeyPoint> v(cnt);
                for (int i = 0; i < cnt; i++) {
                    v[i].pt.x = get(in, x).p<float>()[i];
                    v[i].pt.y = get(in, y).p<float>()[i];
                    v[i].octave = get(in, o).p<int32_t>()[i];
                }
                return v;
            };
            F.mvKeys = kps("S.x", "S.y", "S.oct", n);
            F.mvKeysRight = kps("S.xr", "S.yr", "S.oct_r", nr);
            F.mDescriptors = cv::Mat(n, 32);
            std::memcpy(F.mDescriptors.buf.data(), get(in, "S.desc").b.data(), (size_t)n * 32);
            F.mDescriptorsRight = cv::Mat(nr, 32);
            std::memcpy(F.mDescriptorsRight.buf.data(), get(in, "S.desc_r").b.data(), (size_t)nr * 32);
            const Arr &sc = get(in, "S.scale"), &isc = get(in, "S.inv_scale");
            F.mvScaleFactors.assign(sc.p<float>(), sc.p<float>() + sc.n);
            F.mvInvScaleFactors.assign(isc.p<float>(), isc.p<float>() + isc.n);
            F.mnScaleLevels = (int)sc.n;
            F.mb = get(in, "S.mb_mbf").p<float>()[0];
            F.mbf = get(in, "S.mb_mbf").p<float>()[1];
            ORBextractor el, er;
            auto pyr = [&](const char *img, const char *dims, ORBextractor &e) {
                const uint8_t *src = get(in, img).p<uint8_t>();
                const int32_t *d = get(in, dims).p<int32_t>();
                for (size_t l = 0; l < sc.n; l++) {
                    const int rows = d[2 * l], cols = d[2 * l + 1];
                    cv::Mat m(rows, cols, (size_t)cols + 7);
                    for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), src + (size_t)r * cols, cols);
                    src += (size_t)rows * cols;
                    e.mvImagePyramid.push_back(std::move(m));
                }
            };
            pyr("PL.img", "PL.dims", el);
            pyr("PR.img", "PR.dims", er);
            F.mpORBextractorLeft = &el;
            F.mpORBextractorRight = &er;
            F.mvuRight.assign(n, 123.0f);  // overwritten, as the reference's are
            const int nm = osg_orbslam3::compute_stereo_matches(F);
            out["nmatches"] = make('i', std::vector<int32_t>{nm});
            out["ur"] = make('f', F.mvuRight);
            out["depth"] = make('f', F.mvDepth);
        } else if (mode == "fisheye") {
            // "FE.kl" / "FE.kr" (x, y), "FE.ol" / "FE.or", "FE.dl" / "FE.dr", "FE.mono" (monoLeft, monoRight),
            // "FE.sig2", "FE.cam" (2 x 8 KannalaBrandt8), "FE.R" (3x3), "FE.t"
            Frame F;
            const int nl = (int)get(in, "FE.ol").n, nr = (int)get(in, "FE.or").n;
            auto kps = [&](const char *k, const char *o, int cnt) {
                std::vector<cv::KeyPoint> v(cnt);
                for (int i = 0; i < cnt; i++) {
                    v[i].pt.x = get(in, k).p<float>()[2 * i];
                    v[i].pt.y = get(in, k).p<float>()[2 * i + 1];
                    v[i].octave = get(in, o).p<int32_t>()[i];
                }
                return v;
            };
            F.N = nl + nr;
            F.Nleft = nl;
            F.Nright = nr;
            F.mvKeys = kps("FE.kl", "FE.ol", nl);
            F.mvKeysRight = kps("FE.kr", "FE.or", nr);
            F.mDescriptors = cv::Mat(nl, 32);
            std::memcpy(F.mDescriptors.buf.data(), get(in, "FE.dl").b.data(), (size_t)nl * 32);
            F.mDescriptorsRight = cv::Mat(nr, 32);
            std::memcpy(F.mDescriptorsRight.buf.data(), get(in, "FE.dr").b.data(), (size_t)nr * 32);
            F.monoLeft = get(in, "FE.mono").p<int32_t>()[0];
            F.monoRight = get(in, "FE.mono").p<int32_t>()[1];
            const Arr &s2 = get(in, "FE.sig2");
            F.mvLevelSigma2.assign(s2.p<float>(), s2.p<float>() + s2.n);
            Camera c1, c2;
            c1.type = c2.type = OSG_CAM_KB8;
            c1.params.assign(get(in, "FE.cam").p<float>(), get(in, "FE.cam").p<float>() + 8);
            c2.params.assign(get(in, "FE.cam").p<float>() + 8, get(in, "FE.cam").p<float>() + 16);
            F.mpCamera = &c1;
            F.mpCamera2 = &c2;
            for (int k = 0; k < 9; k++) F.mRlr.a[k] = get(in, "FE.R").p<float>()[k];
            for (int k = 0; k < 3; k++) F.mtlr.a[k] = get(in, "FE.t").p<float>()[k];
            const int nm = osg_orbslam3::compute_stereo_fisheye_matches(F);
            std::vector<float> p3d(3 * (size_t)nl, 0.f);
            for (int i = 0; i < nl; i++)
                if (F.mvLeftToRightMatch[i] >= 0)
                    for (int k = 0; k < 3; k++) p3d[3 * (size_t)i + k] = F.mvStereo3Dpoints[i](k);
            out["nmatches"] = make('i', std::vector<int32_t>{nm, F.mnCloseMPs});
            out["l2r"] = make('i', std::vector<int32_t>(F.mvLeftToRightMatch.begin(), F.mvLeftToRightMatch.end()));
            out["r2l"] = make('i', std::vector<int32_t>(F.mvRightToLeftMatch.begin(), F.mvRightToLeftMatch.end()));
            out["depth"] = make('f', F.mvDepth);
            out["ur"] = make('f', F.mvuRight);
            out["p3d"] = make('f', p3d);
        } else if (mode == "orb") {
            // levels "O.raw" / "O.blur" concatenated with "O.dims" (rows, cols); keypoints "O.x", "O.y",
            // "O.level" (sorted by level); "O.pattern" (512 x 2), "O.umax" (16).  mvImagePyramid levels are
            // ROIs of wider rows (step = cols + 7); the blurred levels are continuous clones
            const Arr &dims = get(in, "O.dims");
            const int levels = (int)dims.n / 2;
            ORBextractor ex;
            std::vector<cv::Mat> blurred;
            const uint8_t *sr = get(in, "O.raw").p<uint8_t>(), *sb = get(in, "O.blur").p<uint8_t>();
            for (int l = 0; l < levels; l++) {
                const int rows = dims.p<int32_t>()[2 * l], cols = dims.p<int32_t>()[2 * l + 1];
                cv::Mat m(rows, cols, (size_t)cols + 7), b(rows, cols);
                for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), sr + (size_t)r * cols, cols);
                std::memcpy(b.buf.data(), sb, (size_t)rows * cols);
                sr += (size_t)rows * cols;
                sb += (size_t)rows * cols;
                ex.mvImagePyramid.push_back(std::move(m));
                blurred.push_back(std::move(b));
            }
            const Arr &pa = get(in, "O.pattern"), &um = get(in, "O.umax");
            for (size_t i = 0; i < pa.n / 2; i++) ex.pattern.push_back(cv::Point{pa.p<int32_t>()[2 * i], pa.p<int32_t>()[2 * i + 1]});
            ex.umax.assign(um.p<int32_t>(), um.p<int32_t>() + um.n);
            std::vector<std::vector<cv::KeyPoint>> all(levels);
            const Arr &kx = get(in, "O.x");
            for (size_t i = 0; i < kx.n; i++) {
                cv::KeyPoint kp;
                kp.pt.x = kx.p<float>()[i];
                kp.pt.y = get(in, "O.y").p<float>()[i];
                kp.angle = -7.0f;  // overwritten
                all[get(in, "O.level").p<int32_t>()[i]].push_back(kp);
            }
            std::vector<uint8_t> desc;
            const int n_out = osg_orbslam3::orb_describe(ex.mvImagePyramid, blurred, all, ex.pattern, ex.umax, desc);
            std::vector<float> ang;
            for (auto &lv : all)
                for (auto &kp : lv) ang.push_back(kp.angle);
            out["n_out"] = make('i', std::vector<int32_t>{n_out});
            out["angle"] = make('f', ang);
            out["desc"] = make('b', desc);
        } else if (mode == "detect") {
            // levels "D.raw" concatenated with "D.dims" (rows, cols), stored as ROIs (step = cols + 5);
            // "D.nf" mnFeaturesPerLevel, "D.scale" mvScaleFactor, "D.th" (iniThFAST, minThFAST)
            const Arr &dims = get(in, "D.dims");
            const int levels = (int)dims.n / 2;
            ORBextractor ex;
            const uint8_t *sr = get(in, "D.raw").p<uint8_t>();
            for (int l = 0; l < levels; l++) {
                const int rows = dims.p<int32_t>()[2 * l], cols = dims.p<int32_t>()[2 * l + 1];
                cv::Mat m(rows, cols, (size_t)cols + 5);
                for (int r = 0; r < rows; r++) std::memcpy(m.ptr<unsigned char>(r), sr + (size_t)r * cols, cols);
                sr += (size_t)rows * cols;
                ex.mvImagePyramid.push_back(std::move(m));
            }
            const Arr &nf = get(in, "D.nf"), &sc = get(in, "D.scale"), &th = get(in, "D.th");
            std::vector<int> nfl(nf.p<int32_t>(), nf.p<int32_t>() + nf.n);
            std::vector<float> scl(sc.p<float>(), sc.p<float>() + sc.n);
            std::vector<std::vector<cv::KeyPoint>> all;
            const int n = osg_orbslam3::compute_keypoints_oct_tree(ex.mvImagePyramid, all, nfl, scl, th.p<int32_t>()[0],
                                                                  th.p<int32_t>()[1]);
            std::vector<float> x, y, r, sz, a;
            std::vector<int32_t> oct;
            for (auto &lv : all)
                for (auto &kp : lv) {
                    x.push_back(kp.pt.x);
                    y.push_back(kp.pt.y);
                    r.push_back(kp.response);
                    sz.push_back(kp.size);
                    a.push_back(kp.angle);
                    oct.push_back(kp.octave);
                }
            out["n"] = make('i', std::vector<int32_t>{n});
            out["x"] = make('f', x);
            out["y"] = make('f', y);
            out["response"] = make('f', r);
            out["size"] = make('f', sz);
            out["angle"] = make('f', a);
            out["octave"] = make('i', oct);
        } else if (mode == "distinct") {
            // keyframes: "K.desc" (nk x nkp rows), "K.bad"; MapPoints: "M.bad", "M.desc" (initial);
            // observations CSR "O.start" / "O.kf" / "O.left" / "O.right"
            const int nk = (int)get(in, "K.bad").n, nm = (int)get(in, "M.bad").n;
            const int nkp = (int)(get(in, "K.desc").n / 32 / (nk ? nk : 1));
            std::vector<KeyFrame> K(nk);
            for (int k = 0; k < nk; k++) {
                K[k].N = nkp;
                K[k].bad = get(in, "K.bad").p<uint8_t>()[k];
                K[k].mDescriptors = cv::Mat(nkp, 32);
                std::memcpy(K[k].mDescriptors.buf.data(), get(in, "K.desc").p<uint8_t>() + (size_t)k * nkp * 32,
                            (size_t)nkp * 32);
            }
            std::vector<MapPoint> M(nm);
            std::vector<MapPoint *> list;
            const int32_t *os = get(in, "O.start").p<int32_t>();
            for (int i = 0; i < nm; i++) {
                M[i].mnId = (unsigned long)i;
                M[i].bad = get(in, "M.bad").p<uint8_t>()[i];
                std::memcpy(M[i].desc.buf.data(), get(in, "M.desc").p<uint8_t>() + 32 * (size_t)i, 32);
                for (int o = os[i]; o < os[i + 1]; o++)
                    M[i].obs[&K[get(in, "O.kf").p<int32_t>()[o]]] =
                        std::make_tuple(get(in, "O.left").p<int32_t>()[o], get(in, "O.right").p<int32_t>()[o]);
                list.push_back(i % 17 == 5 ? nullptr : &M[i]);  // a NULL entry now and then
            }
            osg_orbslam3::compute_distinctive_descriptors<MockHooks>(list);
            std::vector<uint8_t> d(32 * (size_t)nm);
            for (int i = 0; i < nm; i++) std::memcpy(&d[32 * (size_t)i], M[i].desc.buf.data(), 32);
            out["desc"] = make('b', d);
        } else {
            fprintf(stderr, "unknown mode %s\n", mode.c_str());
            return 2;
        }
        write_arrays(argv[3], out);
    } catch (const std::exception &e) {
        fprintf(stderr, "adapter_driver: %s\n", e.what());
        return 1;
    }
    return 0;
}
