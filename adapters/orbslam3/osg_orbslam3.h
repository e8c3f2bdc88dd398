// osg_orbslam3.h — ORB-SLAM3 side of the drop-in: gathers the reference's objects into the
// plain arrays of the C ABI (include/osg.h, include/osg_ba.h), calls it, and writes the results
// back the way the reference does.  Header-only C++17 templates over the reference's own member
// names (Frame, KeyFrame, MapPoint, cv::Mat, cv::KeyPoint, DBoW2::FeatureVector), so the same code
// compiles inside an ORB-SLAM3 tree (adapters/orbslam3/ORBmatcher_osg.cc, Optimizer_osg.cc) and
// against the POD mocks of tests/adapter/mock_orbslam3.h.
//
// The few places where the reference uses Sophus / Eigen / its camera classes go through a hook
// policy H (static member functions), defined by the integration with the reference's own code:
//
//   static void  H::pose(const Frame|KeyFrame&, double q[7])         GetPose() -> {qx qy qz qw tx ty tz}
//   static void  H::set_pose(Frame|KeyFrame&, const double q[7])     SetPose(SE3f(q, t))
//   static void  H::world_pos(MapPoint*, double x[3])                GetWorldPos().cast<double>()
//   static void  H::set_world_pos(MapPoint*, const double x[3])      SetWorldPos + UpdateNormalAndDepth
//   static void  H::camera(const Frame|KeyFrame&, bool right, osg_camera&)
//                mpCamera / mpCamera2 type + parameters, fx fy cx cy mbf, GetRelativePoseTrl()
//   static bool  H::project_last(const Frame& CF, MapPoint*, float& u, float& v, float& invz)
//                ref:src/ORBmatcher.cc:1993-2009 (Tcw * x3Dw, invzc, mpCamera->project); false = skip
//   static float H::tlc_z(const Frame& CF, const Frame& LF)          (Tlw * twc)(2), ref:src/ORBmatcher.cc:1972-1980
//   static bool  H::kf_query(const Frame& CF, MapPoint*, float& u, float& v, int& level)
//                ref:src/ORBmatcher.cc:2238-2262 (project, image bounds, distance range, PredictScale)
//   static bool  H::fuse_query / H::fuse_sim3_query   see b1/b2 Fuse below
//   static void  H::set_gba_pose(KeyFrame&, const double q[7], nLoopKF)   mTcwGBA, mnBAGlobalForKF
//   static void  H::set_gba_pos(MapPoint*, const double x[3], nLoopKF)   mPosGBA, mnBAGlobalForKF
#ifndef OSG_ORBSLAM3_H
#define OSG_ORBSLAM3_H

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <utility>
#include <unordered_map>
#include <utility>
#include <vector>

#include "osg.h"
#include "osg_ba.h"
#include "osg_dbow.h"

namespace osg_orbslam3 {

// The gather structs below hold ABI views that point into their own vectors: never copied or moved
// (batches keep them in a std::deque, which constructs in place).
#define OSG_PINNED_STRUCT(T) \
    T(const T &) = delete;  \
    T &operator=(const T &) = delete

// The entry points keep their per-frame gathers in a per-thread pool reused call to call: the vectors
// keep their capacity, so a 256-frame batch neither allocates nor pages in tens of MB of host memory
// again, and a one-frame call touches warm buffers.  A pooled type has a default constructor and an
// assign(...) that refills every member (measured: the allocation churn was half of the gather).
template <class T>
std::deque<T> &gather_pool(size_t n)
{
    thread_local std::deque<T> pool;
    while (pool.size() < n) pool.emplace_back();
    return pool;
}

// ------------------------------------------------------------------------------------ errors
// Nothing in this adapter throws: ORB-SLAM3's Tracking, LocalMapping and LoopClosing
// threads have no try / catch.  A failing ABI call (a negative OSG_E_* code) is logged once per
// thread and code, and the entry point then returns what the reference returns when it finds
// nothing:
//   * matchers: 0 matches, the caller's slots untouched (the output vectors the reference
//     re-initialises at its start -- SearchByBoW's, SearchForInitialization's vnMatches12,
//     SearchForTriangulation's vMatchedPairs, the stereo Frame members -- re-initialised the same way);
//   * PoseOptimization: 0, pose untouched (ref:src/Optimizer.cc:289-290);
//   * LocalBundleAdjustment / the merge BA: the early return of an abort, nothing written back
//     (ref:src/Optimizer.cc:1869-1873, 2112-2114, 5444-5446);
//   * global BA: the map's state written back unchanged, i.e. an optimize() that stopped before its
//     first iteration (LoopClosing then applies mTcwGBA / mPosGBA as after any GBA);
//   * ORBextractor stages: no keypoints (as for an empty image, ref:src/ORBextractor.cc:1586-1587).
//
// Built with -DOSG_ADAPTER_FAULT_INJECTION (tests/adapter/adapter_fault.cpp only), fault::ctx_rc makes
// the context creation fail and fault::call_rc replaces every ABI call's return code.
#ifdef OSG_ADAPTER_FAULT_INJECTION
namespace fault {
inline thread_local int ctx_rc = 0;
inline thread_local int call_rc = 0;
inline thread_local int reports = 0;  // log lines written by this thread
}  // namespace fault
#endif

inline void report(osg_ctx *ctx, int rc, const char *what)
{
    static thread_local std::set<int> seen;
    if (!seen.insert(rc).second) return;
#ifdef OSG_ADAPTER_FAULT_INJECTION
    fault::reports++;
    if (fault::call_rc) ctx = nullptr;  // the injected call never reached the context
#endif
    std::fprintf(stderr, "osg_orbslam3: %s: %s%s%s (later %s errors on this thread are not logged)\n", what,
                 osg_strerror(rc), ctx ? ": " : "", ctx ? osg_ctx_last_error(ctx) : "", osg_strerror(rc));
}

// One context per host thread: Tracking, LocalMapping and LoopClosing each get their own stream
// and scratch (ref:src/System.cc:234,254 start them as separate threads).  nullptr when no context
// can be created (no gfx950 device, ...); ctx_error() then holds the code, and every call() on this
// thread returns it.
struct ThreadCtx {
    osg_ctx *ctx = nullptr;
    int rc = 0;
    bool tried = false;
    ~ThreadCtx()
    {
        if (ctx) osg_ctx_destroy(ctx);
    }
};
inline ThreadCtx &thread_ctx_slot()
{
    static thread_local ThreadCtx h;
    return h;
}

inline osg_ctx *thread_ctx(int device = 0)
{
    ThreadCtx &h = thread_ctx_slot();
#ifdef OSG_ADAPTER_FAULT_INJECTION
    if (fault::ctx_rc) {
        report(nullptr, fault::ctx_rc, "osg_ctx_create");
        return nullptr;
    }
    if (fault::call_rc) return nullptr;  // call() returns the injected code before it needs a context
#endif
    if (!h.ctx && !h.tried) {
        h.tried = true;
        h.rc = osg_ctx_create(device, &h.ctx);
        if (h.rc < 0) {
            h.ctx = nullptr;
            report(nullptr, h.rc, "osg_ctx_create");
        }
    }
    return h.ctx;
}

inline int ctx_error()
{
#ifdef OSG_ADAPTER_FAULT_INJECTION
    if (fault::ctx_rc) return fault::ctx_rc;
#endif
    const int rc = thread_ctx_slot().rc;
    return rc < 0 ? rc : OSG_E_NODEVICE;
}

// Runs one ABI call f() on the thread's context; returns its code (>= 0) or a logged OSG_E_* code.
template <class F>
inline int call(osg_ctx *ctx, const char *what, F &&f)
{
#ifdef OSG_ADAPTER_FAULT_INJECTION
    if (fault::call_rc) {
        report(ctx, fault::call_rc, what);
        return fault::call_rc;
    }
#endif
    if (!ctx) return ctx_error();  // already logged by thread_ctx()
    const int rc = f();
    if (rc < 0) report(ctx, rc, what);
    return rc;
}

// ---------------------------------------------------------------------------------- gathering
template <class KeyPointT>
inline void push_kp(const KeyPointT &kp, std::vector<float> &x, std::vector<float> &y, std::vector<float> &a,
                    std::vector<int32_t> &o)
{
    x.push_back(kp.pt.x);
    y.push_back(kp.pt.y);
    a.push_back(kp.angle);
    o.push_back(kp.octave);
}

// A MapPoint's 256-bit descriptor into dst.  MapPoint::GetDescriptor() returns a clone (a heap
// allocation per call, ref:src/MapPoint.cc GetDescriptor); an integration that adds
// `void GetDescriptorRow(unsigned char *dst) const` (the 32 bytes copied under mMutexFeatures,
// INTEGRATION.md §2) is read through that instead -- measured 33 ns of the gather per MapPoint.
template <class MapPointT>
inline auto mp_descriptor_(MapPointT *p, uint8_t *dst, int) -> decltype(p->GetDescriptorRow(dst), void())
{
    p->GetDescriptorRow(dst);
}
template <class MapPointT>
inline void mp_descriptor_(MapPointT *p, uint8_t *dst, long)
{
    const auto d = p->GetDescriptor();
    std::memcpy(dst, d.template ptr<unsigned char>(0), 32);
}
template <class MapPointT>
inline void mp_descriptor(MapPointT *p, uint8_t *dst)
{
    mp_descriptor_(p, dst, 0);
}

template <class MatT>
inline void copy_desc_rows(const MatT &m, int n, std::vector<uint8_t> &out)
{
    out.resize((size_t)n * 32);
    for (int i = 0; i < n; i++) std::memcpy(&out[(size_t)32 * i], m.template ptr<unsigned char>(i), 32);
}

// The n descriptor rows as one contiguous block: the Mat's own storage when its rows are packed (an
// ORBextractor's N x 32 CV_8U output is), else a copy into `out`.  The ABI calls read it before they
// return, so pointing into the Frame's Mat is safe.
template <class MatT>
inline const uint8_t *desc_rows(const MatT &m, int n, std::vector<uint8_t> &out)
{
    if (n > 0 && m.rows >= n && (size_t)m.step[0] == 32) return m.template ptr<unsigned char>(0);
    copy_desc_rows(m, n, out);
    return out.data();
}

// 64 x 48 grid of vectors as CSR in GetFeaturesInArea's enumeration order (ix outer, iy inner,
// cell contents in insertion order)
template <class GridT>
inline void grid_csr(const GridT &grid, std::vector<int32_t> &gs, std::vector<int32_t> &gi, size_t cap)
{
    // one walk over the cells (separate heap blocks): sizes and indices together, into `gi` sized for
    // `cap` indices (a Frame's grid holds each of its keypoints at most once), trimmed after; the
    // two-walk form (count, then fill) below only if a grid holds more (a size walk first measured
    // 30 % slower, and a walk that reads every cell header twice costs as much again)
    gs.resize(OSG_GRID_CELLS + 1);
    gi.resize(cap);
    int32_t *g = gs.data(), *o = gi.data(), *const end = gi.data() + cap;
    g[0] = 0;
    bool fits = true;
    for (int ix = 0; ix < OSG_GRID_COLS && fits; ix++) {
        const auto *col = &grid[ix][0];
        for (int iy = 0; iy < OSG_GRID_ROWS; iy++) {
            const auto *b = col[iy].data();
            const int m = (int)col[iy].size();
            if (m > end - o) {
                fits = false;
                break;
            }
            for (int k = 0; k < m; k++) o[k] = (int32_t)b[k];
            o += m;
            g[ix * OSG_GRID_ROWS + iy + 1] = (int32_t)(o - gi.data());
        }
    }
    if (fits) {
        gi.resize((size_t)(o - gi.data()));
        return;
    }
    size_t total = 0;
    for (int ix = 0; ix < OSG_GRID_COLS; ix++)
        for (int iy = 0; iy < OSG_GRID_ROWS; iy++) total += grid[ix][iy].size();
    grid_csr(grid, gs, gi, total);
}

// The first `lines` 64-byte lines of a heap object (MapPoints: their state and the fields the hooks
// read lie past the first line)
template <class T>
inline void prefetch_obj(const T *p, int lines = 4)
{
    if (!p) return;
    for (int k = 0; k < lines; k++) __builtin_prefetch((const char *)p + 64 * k);
}

// Frame::Nleft / KeyFrame::NLeft (ref:include/Frame.h, include/KeyFrame.h spell it differently)
template <class T>
inline auto nleft_of(const T &F, int) -> decltype(F.Nleft, int())
{
    return F.Nleft;
}
template <class T>
inline auto nleft_of(const T &F, long) -> decltype(F.NLeft, int())
{
    return F.NLeft;
}

// osg_frame of a Frame or KeyFrame (ref:include/Frame.h:218-296, include/KeyFrame.h:321-508):
// keypoints (mvKeysUn, or mvKeys + mvKeysRight for a two-camera rig), descriptors, mvuRight, mGrid
// (+ mGridRight, mvLeftToRightMatch, mvRightToLeftMatch for a two-camera rig).
template <class FrameT>
struct FrameView {
    OSG_PINNED_STRUCT(FrameView);
    std::vector<float> kx, ky, ka, ur, scale;
    std::vector<int32_t> ko, gs, gi, gsr, gir, l2r, r2l;
    std::vector<uint8_t> desc;
    osg_frame v{};

    FrameView() = default;
    explicit FrameView(const FrameT &F) { assign(F); }
    void assign(const FrameT &F)
    {
        const int n = F.N, nleft = nleft_of(F, 0);
        v = osg_frame{};
        kx.resize(n);
        ky.resize(n);
        ka.resize(n);
        ko.resize(n);
        for (int i = 0; i < n; i++) {
            const auto &kp = nleft == -1 ? F.mvKeysUn[i] : (i < nleft ? F.mvKeys[i] : F.mvKeysRight[i - nleft]);
            kx[i] = kp.pt.x;
            ky[i] = kp.pt.y;
            ka[i] = kp.angle;
            ko[i] = kp.octave;
        }
        const uint8_t *dp = desc_rows(F.mDescriptors, n, desc);
        ur.assign(F.mvuRight.begin(), F.mvuRight.end());
        ur.resize(n, -1.0f);
        grid_csr(F.mGrid, gs, gi, (size_t)(nleft == -1 ? n : nleft));
        if (nleft != -1) {
            grid_csr(F.mGridRight, gsr, gir, (size_t)(n - nleft));
            l2r.assign(F.mvLeftToRightMatch.begin(), F.mvLeftToRightMatch.end());
            r2l.assign(F.mvRightToLeftMatch.begin(), F.mvRightToLeftMatch.end());
            l2r.resize(nleft, -1);
            r2l.resize(n - nleft, -1);
            v.grid_start_r = gsr.data();
            v.grid_idx_r = gir.data();
            v.left_to_right = l2r.data();
            v.right_to_left = r2l.data();
        }
        scale.assign(F.mvScaleFactors.begin(), F.mvScaleFactors.end());
        v.n = n;
        v.nleft = nleft;
        v.desc = dp;
        v.kp_x = kx.data();
        v.kp_y = ky.data();
        v.kp_angle = ka.data();
        v.kp_octave = ko.data();
        v.u_right = ur.data();
        v.grid_start = gs.data();
        v.grid_idx = gi.data();
        v.min_x = F.mnMinX;
        v.max_x = F.mnMaxX;
        v.min_y = F.mnMinY;
        v.max_y = F.mnMaxY;
        v.grid_inv_w = F.mfGridElementWidthInv;
        v.grid_inv_h = F.mfGridElementHeightInv;
        v.scale_factors = scale.data();
        v.n_levels = F.mnScaleLevels;
        v.mb = F.mb;
        v.mbf = F.mbf;
    }
};

// Slot state of Frame::mvpMapPoints with stable ids: ids [0, nq) are the caller's query MapPoints,
// a slot already holding another MapPoint gets id nq + slot.
template <class MapPointT>
struct Slots {
    std::vector<int32_t> mp;
    std::vector<uint8_t> taken;
    std::vector<MapPointT *> occupant;
    Slots() = default;
    Slots(const std::vector<MapPointT *> &slots, int nq, bool need_obs) { assign(slots, nq, need_obs); }
    void assign(const std::vector<MapPointT *> &slots, int nq, bool need_obs)
    {
        const int n = (int)slots.size();
        mp.assign(n, -1);
        taken.assign(n, 0);
        occupant = slots;
        for (int i = 0; i < n; i++)
            if (slots[i]) {
                mp[i] = nq + i;
                taken[i] = need_obs ? (slots[i]->Observations() > 0) : 1;
            }
    }
    // writes back the slots whose id changed; returns nothing (the count comes from the ABI)
    template <class QueryPtrVec>
    void apply(std::vector<MapPointT *> &slots, const QueryPtrVec &queries, int nq) const
    {
        for (size_t i = 0; i < slots.size(); i++) {
            const int id = mp[i];
            if (id < 0) slots[i] = nullptr;
            else if (id < nq) slots[i] = queries[id];
            else slots[i] = occupant[id - nq];
        }
    }
};

// ---------------------------------------------------------------------- a1 DescriptorDistance
template <class MatT>
inline int descriptor_distance(const MatT &a, const MatT &b)
{
    return osg_descriptor_distance(a.template ptr<unsigned char>(0), b.template ptr<unsigned char>(0));
}

// ---------------------------------------------- a5 SearchByProjection(Frame&, vector<MapPoint*>)
// ref:src/ORBmatcher.cc:44-242.  MpsGather: one problem (the Frame, the local MapPoints' isInFrustum
// results, the slot state), shared by the single and the batched entry points.
template <class FrameT, class MapPointT>
struct MpsGather {
    OSG_PINNED_STRUCT(MpsGather);
    FrameView<FrameT> fv;
    std::vector<int32_t> id, lvl, lvl_r;
    std::vector<uint8_t> desc, usable, has_obs, in_view, in_view_r;
    std::vector<float> px, py, pxr, pyr, vc, vcr, depth;
    osg_mp_queries q{};
    Slots<MapPointT> slots;
    MpsGather() = default;
    MpsGather(FrameT &F, const std::vector<MapPointT *> &vpMapPoints) { assign(F, vpMapPoints); }
    void assign(FrameT &F, const std::vector<MapPointT *> &vpMapPoints)
    {
        fv.assign(F);
        slots.assign(F.mvpMapPoints, (int)vpMapPoints.size(), true);
        const int nq = (int)vpMapPoints.size();
        q = osg_mp_queries{};
        id.assign(nq, 0);
        lvl.assign(nq, 0);
        lvl_r.assign(nq, 0);
        desc.assign((size_t)nq * 32, 0);
        usable.assign(nq, 0);
        has_obs.assign(nq, 0);
        in_view.assign(nq, 0);
        in_view_r.assign(nq, 0);
        for (auto *v : {&px, &py, &pxr, &pyr, &vc, &vcr, &depth}) v->assign(nq, 0.f);
        constexpr int PF = 8;  // MapPoints are scattered heap objects: fetch a few ahead
        for (int i = 0; i < std::min(PF, nq); i++) __builtin_prefetch(vpMapPoints[i]);
        for (int i = 0; i < nq; i++) {
            if (i + PF < nq) prefetch_obj(vpMapPoints[i + PF]);
            MapPointT *p = vpMapPoints[i];
            id[i] = i;
            in_view[i] = p->mbTrackInView;
            in_view_r[i] = p->mbTrackInViewR;
            if (!in_view[i] && !in_view_r[i]) continue;  // the reference skips before any other read
            usable[i] = !p->isBad();
            has_obs[i] = p->Observations() > 0;
            mp_descriptor(p, &desc[(size_t)32 * i]);
            px[i] = p->mTrackProjX;
            py[i] = p->mTrackProjY;
            pxr[i] = p->mTrackProjXR;
            pyr[i] = p->mTrackProjYR;
            vc[i] = p->mTrackViewCos;
            vcr[i] = p->mTrackViewCosR;
            lvl[i] = p->mnTrackScaleLevel;
            lvl_r[i] = p->mnTrackScaleLevelR;
            depth[i] = p->mTrackDepth;
        }
        q.n = nq;
        q.mp_id = id.data();
        q.desc = desc.data();
        q.usable = usable.data();
        q.has_obs = has_obs.data();
        q.in_view = in_view.data();
        q.proj_x = px.data();
        q.proj_y = py.data();
        q.proj_xr = pxr.data();
        q.view_cos = vc.data();
        q.pred_level = lvl.data();
        q.track_depth = depth.data();
        q.in_view_r = in_view_r.data();
        q.proj_yr = pyr.data();
        q.view_cos_r = vcr.data();
        q.pred_level_r = lvl_r.data();
    }
};

template <class H, class FrameT, class MapPointT>
int search_by_projection_mps(FrameT &F, const std::vector<MapPointT *> &vpMapPoints, float th, bool bFarPoints,
                             float thFarPoints, float nnratio)
{
    osg_ctx *ctx = thread_ctx();
    MpsGather<FrameT, MapPointT> &g = gather_pool<MpsGather<FrameT, MapPointT>>(1)[0];
    g.assign(F, vpMapPoints);
    const int nm = call(ctx, "osg_search_by_projection_mps", [&] {
        return osg_search_by_projection_mps(ctx, &g.fv.v, &g.q, nnratio, th, bFarPoints, thFarPoints, g.slots.mp.data(),
                                            g.slots.taken.data());
    });
    if (nm < 0) return 0;
    g.slots.apply(F.mvpMapPoints, vpMapPoints, (int)vpMapPoints.size());
    return nm;
}

// ------------------------------------------------- a6 SearchByProjection(Frame&, const Frame&)
// ref:src/ORBmatcher.cc:1957-2191.  LastGather: one (CurrentFrame, LastFrame) problem.
template <class H, class FrameT>
struct LastGather {
    OSG_PINNED_STRUCT(LastGather);
    using MapPointT = typename std::remove_pointer<typename std::decay<decltype(std::declval<FrameT &>().mvpMapPoints[0])>::type>::type;
    FrameView<FrameT> fv;
    std::vector<int32_t> id, oct;
    std::vector<uint8_t> desc, valid, has_obs;
    std::vector<float> u, v, invz, ang, ur, vr;
    std::vector<MapPointT *> queries;
    osg_last_queries q{};
    Slots<MapPointT> slots;
    LastGather() = default;
    LastGather(FrameT &CF, const FrameT &LF) { assign(CF, LF); }
    void assign(FrameT &CF, const FrameT &LF)
    {
        fv.assign(CF);
        slots.assign(CF.mvpMapPoints, LF.N, true);
        q = osg_last_queries{};
        const int n = LF.N;
        id.assign(n, -1);
        oct.assign(n, 0);
        desc.assign((size_t)n * 32, 0);
        valid.assign(n, 0);
        has_obs.assign(n, 0);
        for (auto *w : {&u, &v, &invz, &ang}) w->assign(n, 0.f);
        queries.assign(n, nullptr);
        const bool two = CF.Nleft != -1;
        if (two) {
            ur.assign(n, 0.f);
            vr.assign(n, 0.f);
        }
        constexpr int PF = 8;  // MapPoints are scattered heap objects: fetch a few ahead
        for (int i = 0; i < n; i++) {
            if (i + PF < n) prefetch_obj(LF.mvpMapPoints[i + PF]);
            MapPointT *p = LF.mvpMapPoints[i];
            const auto &kp = (LF.Nleft == -1) ? LF.mvKeysUn[i]
                                              : (i < LF.Nleft ? LF.mvKeys[i] : LF.mvKeysRight[i - LF.Nleft]);
            oct[i] = (LF.Nleft == -1 || i < LF.Nleft) ? LF.mvKeys[i].octave : LF.mvKeysRight[i - LF.Nleft].octave;
            ang[i] = kp.angle;
            if (!p || LF.mvbOutlier[i]) continue;
            if (!H::project_last(CF, p, u[i], v[i], invz[i])) continue;
            if (two) H::project_last_right(CF, p, ur[i], vr[i]);  // ref:src/ORBmatcher.cc:2096-2097
            valid[i] = 1;
            id[i] = i;
            queries[i] = p;
            has_obs[i] = p->Observations() > 0;
            mp_descriptor(p, &desc[(size_t)32 * i]);
        }
        q.n = n;
        q.mp_id = id.data();
        q.desc = desc.data();
        q.valid = valid.data();
        q.has_obs = has_obs.data();
        q.u = u.data();
        q.v = v.data();
        q.invz = invz.data();
        q.octave = oct.data();
        q.angle = ang.data();
        if (two) {
            q.u_r = ur.data();
            q.v_r = vr.data();
        }
        q.tlc_z = H::tlc_z(CF, LF);
    }
};

template <class H, class FrameT>
int search_by_projection_last(FrameT &CF, const FrameT &LF, float th, bool bMono, bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    LastGather<H, FrameT> &g = gather_pool<LastGather<H, FrameT>>(1)[0];
    g.assign(CF, LF);
    const int nm = call(ctx, "osg_search_by_projection_last", [&] {
        return osg_search_by_projection_last(ctx, &g.fv.v, &g.q, th, bMono, checkOri, g.slots.mp.data(),
                                             g.slots.taken.data());
    });
    if (nm < 0) return 0;
    g.slots.apply(CF.mvpMapPoints, g.queries, LF.N);
    return nm;
}

// ---------------------------------- a7 SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, ...)
// ref:src/ORBmatcher.cc:2203-2330
template <class H, class FrameT, class KeyFrameT, class MapPointT>
int search_by_projection_kf(FrameT &CF, KeyFrameT *pKF, const std::set<MapPointT *> &sAlreadyFound, float th,
                            int ORBdist, bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<FrameT> fv(CF);
    const std::vector<MapPointT *> vpMPs = pKF->GetMapPointMatches();
    const int n = (int)vpMPs.size();
    std::vector<int32_t> id(n, -1), lvl(n, 0);
    std::vector<uint8_t> desc((size_t)n * 32), valid(n, 0);
    std::vector<float> u(n), v(n), ang(n);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpMPs[i];
        ang[i] = pKF->mvKeysUn[i].angle;
        if (!p || p->isBad() || sAlreadyFound.count(p)) continue;
        if (!H::kf_query(CF, p, u[i], v[i], lvl[i])) continue;
        valid[i] = 1;
        id[i] = i;
        mp_descriptor(p, &desc[(size_t)32 * i]);
    }
    osg_kf_queries q{};
    q.n = n;
    q.mp_id = id.data();
    q.desc = desc.data();
    q.valid = valid.data();
    q.u = u.data();
    q.v = v.data();
    q.pred_level = lvl.data();
    q.angle = ang.data();
    Slots<MapPointT> slots(CF.mvpMapPoints, n, false);
    const int nm = call(ctx, "osg_search_by_projection_kf", [&] {
        return osg_search_by_projection_kf(ctx, &fv.v, &q, th, ORBdist, checkOri, slots.mp.data());
    });
    if (nm < 0) return 0;
    slots.apply(CF.mvpMapPoints, vpMPs, n);
    return nm;
}

// ---------------------------------------------------------------------------------- b1/b2 Fuse
// The reference's loop is "for each MapPoint in order: filters, search, then replace / add", and the
// replace / add mutates the map.  Here the search of every MapPoint runs first (one launch) and
// the replace / add runs after it, in order, re-checking the filters that can change inside the
// loop.  That is the same result because nothing a replace / add does changes the search of a
// MapPoint that still passes those checks:
//   * the search reads the KeyFrame's keypoints / grid (never mutated here) and the MapPoint's
//     position, normal, distances (unchanged by Replace / AddObservation) and descriptor;
//   * a descriptor changes only on the survivor of a Replace (MapPoint::Replace ->
//     ComputeDistinctiveDescriptors, ref:src/MapPoint.cc:313-395), and the survivor is in pKF
//     afterwards (it held, or took over, the slot bestIdx), so its own later turn is skipped by
//     IsInKeyFrame(pKF);
//   * isBad() / IsInKeyFrame(pKF) can only become true during the loop (Replace marks the
//     replaced point bad; AddObservation adds pKF), so the gather-time filter keeps a superset and
//     the apply-time re-check removes exactly the ones the reference skips.
// Fuse(pKF, vpMapPoints, th, bRight), ref:src/ORBmatcher.cc:1330-1541.  Hook:
//   static bool H::fuse_query(KeyFrame*, MapPoint*, bool right, float& u, float& v, float& ur, int& level)
//                ref:src/ORBmatcher.cc:1336-1347, 1385-1433 (Tcw * p3Dw, depth, project, IsInImage, ur, distance
//                range, viewing angle, PredictScale); false = skipped
template <class H, class KeyFrameT, class MapPointT>
int fuse(KeyFrameT *pKF, const std::vector<MapPointT *> &vpMapPoints, float th, bool bRight)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<KeyFrameT> fv(*pKF);
    const int n = (int)vpMapPoints.size();
    std::vector<uint8_t> desc((size_t)n * 32), valid(n, 0);
    std::vector<float> u(n, 0.f), v(n, 0.f), ur(n, 0.f);
    std::vector<int32_t> lvl(n, 0), best_idx(n, -1), best_dist(n, 256);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpMapPoints[i];
        if (!p || p->isBad() || p->IsInKeyFrame(pKF)) continue;  // ref:src/ORBmatcher.cc:1367-1382
        if (!H::fuse_query(pKF, p, bRight, u[i], v[i], ur[i], lvl[i])) continue;
        valid[i] = 1;
        mp_descriptor(p, &desc[(size_t)32 * i]);
    }
    std::vector<float> inv_s2(pKF->mvInvLevelSigma2.begin(), pKF->mvInvLevelSigma2.end());
    osg_fuse_queries q{};
    q.n = n;
    q.desc = desc.data();
    q.valid = valid.data();
    q.u = u.data();
    q.v = v.data();
    q.ur = ur.data();
    q.pred_level = lvl.data();
    q.inv_level_sigma2 = inv_s2.data();
    if (call(ctx, "osg_fuse_search", [&] {
            return osg_fuse_search(ctx, &fv.v, &q, th, bRight ? 1 : 0, 1, best_idx.data(), best_dist.data());
        }) < 0)
        return 0;
    int nFused = 0;
    for (int i = 0; i < n; i++) {  // ref:src/ORBmatcher.cc:1514-1539, in MapPoint order
        MapPointT *pMP = vpMapPoints[i];
        if (!valid[i] || best_idx[i] < 0) continue;
        if (pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;  // changed earlier in this loop
        const int bestIdx = best_idx[i];
        MapPointT *pMPinKF = pKF->GetMapPoint(bestIdx);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, bestIdx);
            pKF->AddMapPoint(pMP, bestIdx);
        }
        nFused++;
    }
    return nFused;
}

// Fuse(pKF, Scw, vpPoints, th, vpReplacePoint), ref:src/ORBmatcher.cc:1553-1694 (LoopClosing).
// Nothing in this loop makes a point bad, and spAlreadyFound is a snapshot, so the filters are
// static; only GetMapPoint(bestIdx) sees earlier iterations' AddMapPoint, and the apply reads it
// in order.  Hook:
//   static bool H::fuse_sim3_query(KeyFrame*, const Sim3&, MapPoint*, float& u, float& v, int& level)
//                ref:src/ORBmatcher.cc:1560-1562, 1587-1622; false = skipped
template <class H, class KeyFrameT, class Sim3T, class MapPointT>
int fuse_sim3(KeyFrameT *pKF, const Sim3T &Scw, const std::vector<MapPointT *> &vpPoints, float th,
              std::vector<MapPointT *> &vpReplacePoint)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<KeyFrameT> fv(*pKF);
    const auto spAlreadyFound = pKF->GetMapPoints();
    const int n = (int)vpPoints.size();
    std::vector<uint8_t> desc((size_t)n * 32), valid(n, 0);
    std::vector<float> u(n, 0.f), v(n, 0.f);
    std::vector<int32_t> lvl(n, 0), best_idx(n, -1), best_dist(n, 256);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpPoints[i];
        if (p->isBad() || spAlreadyFound.count(p)) continue;  // ref:src/ORBmatcher.cc:1582
        if (!H::fuse_sim3_query(pKF, Scw, p, u[i], v[i], lvl[i])) continue;
        valid[i] = 1;
        mp_descriptor(p, &desc[(size_t)32 * i]);
    }
    osg_fuse_queries q{};
    q.n = n;
    q.desc = desc.data();
    q.valid = valid.data();
    q.u = u.data();
    q.v = v.data();
    q.pred_level = lvl.data();
    if (call(ctx, "osg_fuse_search",
             [&] { return osg_fuse_search(ctx, &fv.v, &q, th, 0, 0, best_idx.data(), best_dist.data()); }) < 0)
        return 0;
    int nFused = 0;
    for (int i = 0; i < n; i++) {  // ref:src/ORBmatcher.cc:1661-1681
        if (!valid[i] || best_idx[i] < 0) continue;
        MapPointT *pMP = vpPoints[i];
        MapPointT *pMPinKF = pKF->GetMapPoint(best_idx[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, best_idx[i]);
            pKF->AddMapPoint(pMP, best_idx[i]);
        }
        nFused++;
    }
    return nFused;
}

// ------------------------------------------------------------------------------- a3/a4 BoW
// DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>) as CSR in key order.
template <class FeatVecT>
struct FeatVecCSR {
    std::vector<uint32_t> node;
    std::vector<int32_t> start, feat;
    FeatVecCSR() = default;
    explicit FeatVecCSR(const FeatVecT &fvec) { assign(fvec); }
    void assign(const FeatVecT &fvec)
    {
        // sized once, then written in place (push_back per feature measured ~2x slower)
        const size_t nn = fvec.size();
        size_t nf = 0;
        for (const auto &kv : fvec) nf += kv.second.size();
        node.resize(nn);
        start.resize(nn + 1);
        feat.resize(nf);
        uint32_t *pn = node.data();
        int32_t *ps = start.data(), *pf = feat.data();
        int32_t k = 0;
        ps[0] = 0;
        for (const auto &kv : fvec) {
            *pn++ = (uint32_t)kv.first;
            for (auto f : kv.second) pf[k++] = (int32_t)f;
            *++ps = k;
        }
    }
    osg_featvec view() const { return osg_featvec{(int32_t)node.size(), node.data(), start.data(), feat.data()}; }
};

// ref:src/ORBmatcher.cc:262-496.  vpMapPointMatches = vector<MapPoint*>(F.N, NULL) with the KF's
// MapPoints matched to Frame keypoints.  BowKfF gathers one (KeyFrame, Frame) problem; the single
// and the batched entry points share it.
template <class KeyFrameT, class FrameT, class MapPointT>
struct BowKfF {
    OSG_PINNED_STRUCT(BowKfF);
    std::vector<MapPointT *> vpMPsKF;
    std::vector<uint8_t> dk, df, good;
    std::vector<float> ak, af;
    std::vector<int32_t> idk;
    FeatVecCSR<decltype(std::declval<KeyFrameT &>().mFeatVec)> fk;
    FeatVecCSR<decltype(std::declval<FrameT &>().mFeatVec)> ff;
    osg_bow_side sk{}, sf{};
    BowKfF() = default;
    BowKfF(KeyFrameT *pKF, const FrameT &F) { assign(pKF, F); }
    void assign(KeyFrameT *pKF, const FrameT &F)
    {
        vpMPsKF = pKF->GetMapPointMatches();
        fk.assign(pKF->mFeatVec);
        ff.assign(F.mFeatVec);
        const int nk = (int)vpMPsKF.size(), nf = F.N;
        good.resize(nk);
        ak.resize(nk);
        af.resize(nf);
        idk.assign(nk, -1);
        const uint8_t *dkp = desc_rows(pKF->mDescriptors, nk, dk), *dfp = desc_rows(F.mDescriptors, nf, df);
        constexpr int PF = 8;  // isBad() reads each MapPoint, scattered heap objects: fetch a few ahead
        for (int i = 0; i < nk; i++) {
            if (i + PF < nk && vpMPsKF[i + PF]) __builtin_prefetch(vpMPsKF[i + PF]);
            // ref:src/ORBmatcher.cc:399-401
            ak[i] = (!pKF->mpCamera2) ? pKF->mvKeysUn[i].angle
                                      : (i >= pKF->NLeft ? pKF->mvKeysRight[i - pKF->NLeft].angle : pKF->mvKeys[i].angle);
            good[i] = vpMPsKF[i] && !vpMPsKF[i]->isBad();
            if (vpMPsKF[i]) idk[i] = i;
        }
        for (int i = 0; i < nf; i++)
            af[i] = (F.Nleft == -1) ? F.mvKeysUn[i].angle : (i < F.Nleft ? F.mvKeys[i].angle : F.mvKeysRight[i - F.Nleft].angle);
        sk = osg_bow_side{nk, pKF->NLeft, dkp, ak.data(), idk.data(), good.data(), fk.view()};
        sf = osg_bow_side{nf, F.Nleft, dfp, af.data(), nullptr, nullptr, ff.view()};
    }
    // ref:src/ORBmatcher.cc:268 (the vector is re-initialised whatever happens) + the matches
    void apply(const int32_t *out, int nf, std::vector<MapPointT *> &vpMapPointMatches, bool ok) const
    {
        vpMapPointMatches.assign(nf, nullptr);
        if (!ok) return;
        for (int i = 0; i < nf; i++)
            if (out[i] >= 0) vpMapPointMatches[i] = vpMPsKF[out[i]];
    }
};

template <class H, class KeyFrameT, class FrameT, class MapPointT>
int search_by_bow_kf_f(KeyFrameT *pKF, FrameT &F, std::vector<MapPointT *> &vpMapPointMatches, float nnratio,
                       bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    BowKfF<KeyFrameT, FrameT, MapPointT> &g = gather_pool<BowKfF<KeyFrameT, FrameT, MapPointT>>(1)[0];
    g.assign(pKF, F);
    std::vector<int32_t> out(F.N, -1);
    const int nm = call(ctx, "osg_search_by_bow_kf_f",
                        [&] { return osg_search_by_bow_kf_f(ctx, &g.sk, &g.sf, nnratio, checkOri, out.data()); });
    g.apply(out.data(), F.N, vpMapPointMatches, nm >= 0);
    return nm < 0 ? 0 : nm;
}

// ref:src/ORBmatcher.cc:890-1043.  vpMatches12[i] = KF2 MapPoint matched to KF1 keypoint i.
template <class H, class KeyFrameT, class MapPointT>
int search_by_bow_kf_kf(KeyFrameT *pKF1, KeyFrameT *pKF2, std::vector<MapPointT *> &vpMatches12, float nnratio,
                        bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    const std::vector<MapPointT *> v1 = pKF1->GetMapPointMatches(), v2 = pKF2->GetMapPointMatches();
    const int n1 = (int)v1.size(), n2 = (int)v2.size();
    std::vector<uint8_t> d1, d2, g1(n1), g2(n2);
    std::vector<float> a1(n1), a2(n2);
    std::vector<int32_t> id1(n1, -1), id2(n2, -1);
    copy_desc_rows(pKF1->mDescriptors, n1, d1);
    copy_desc_rows(pKF2->mDescriptors, n2, d2);
    // only keypoints below mvKeysUn.size() are ever matched (== NLeft on a two-camera rig)
    for (int i = 0; i < n1; i++) {
        a1[i] = i < (int)pKF1->mvKeysUn.size() ? pKF1->mvKeysUn[i].angle : 0.f;
        g1[i] = v1[i] && !v1[i]->isBad();
        if (v1[i]) id1[i] = i;
    }
    for (int i = 0; i < n2; i++) {
        a2[i] = i < (int)pKF2->mvKeysUn.size() ? pKF2->mvKeysUn[i].angle : 0.f;
        g2[i] = v2[i] && !v2[i]->isBad();
        if (v2[i]) id2[i] = i;
    }
    FeatVecCSR<decltype(pKF1->mFeatVec)> f1(pKF1->mFeatVec);
    FeatVecCSR<decltype(pKF2->mFeatVec)> f2(pKF2->mFeatVec);
    osg_bow_side s1{n1, pKF1->NLeft, d1.data(), a1.data(), id1.data(), g1.data(), f1.view()};
    osg_bow_side s2{n2, pKF2->NLeft, d2.data(), a2.data(), id2.data(), g2.data(), f2.view()};
    std::vector<int32_t> out(n1, -1);
    const int nm = call(ctx, "osg_search_by_bow_kf_kf",
                        [&] { return osg_search_by_bow_kf_kf(ctx, &s1, &s2, nnratio, checkOri, out.data()); });
    vpMatches12.assign(n1, nullptr);  // ref:src/ORBmatcher.cc:904
    if (nm < 0) return 0;
    for (int i = 0; i < n1; i++)
        if (out[i] >= 0) vpMatches12[i] = v2[out[i]];
    return nm;
}

// ------------------------------------------------- b5 SearchByProjection(KeyFrame*, Sim3f&, ...)
// ref:src/ORBmatcher.cc:498-621 (vpPointsKFs == nullptr) and :623-733 (with vpPointsKFs / vpMatchedKF).
// The pre-search part and the projection come from H::sim3_query; the GPU takes the greedy search.
template <class H, class KeyFrameT, class Sim3T, class MapPointT>
int search_by_projection_sim3(KeyFrameT *pKF, const Sim3T &Scw, const std::vector<MapPointT *> &vpPoints,
                              const std::vector<KeyFrameT *> *vpPointsKFs, std::vector<MapPointT *> &vpMatched,
                              std::vector<KeyFrameT *> *vpMatchedKF, int th, float ratioHamming)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<KeyFrameT> fv(*pKF);
    std::set<MapPointT *> spAlreadyFound(vpMatched.begin(), vpMatched.end());  // :515-516
    spAlreadyFound.erase(static_cast<MapPointT *>(nullptr));
    const int n = (int)vpPoints.size();
    std::vector<uint8_t> desc((size_t)n * 32), valid(n, 0);
    std::vector<float> u(n, 0.f), v(n, 0.f);
    std::vector<int32_t> lvl(n, 0);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpPoints[i];
        if (p->isBad() || spAlreadyFound.count(p)) continue;  // :528, :647
        if (!H::sim3_query(pKF, Scw, p, vpPointsKFs != nullptr, u[i], v[i], lvl[i])) continue;
        valid[i] = 1;
        mp_descriptor(p, &desc[(size_t)32 * i]);
    }
    std::vector<int32_t> slot_query(pKF->N);
    for (int i = 0; i < pKF->N; i++) slot_query[i] = vpMatched[i] ? -2 : -1;
    osg_fuse_queries q{};
    q.n = n;
    q.desc = desc.data();
    q.valid = valid.data();
    q.u = u.data();
    q.v = v.data();
    q.pred_level = lvl.data();
    const int nm = call(ctx, "osg_search_by_projection_sim3", [&] {
        return osg_search_by_projection_sim3(ctx, &fv.v, &q, (float)th, ratioHamming, slot_query.data());
    });
    if (nm < 0) return 0;
    for (int i = 0; i < pKF->N; i++)
        if (slot_query[i] >= 0) {  // vpMatched[bestIdx] = pMP (, vpMatchedKF[bestIdx] = pKFi), :614 / :726-727
            vpMatched[i] = vpPoints[slot_query[i]];
            if (vpMatchedKF) (*vpMatchedKF)[i] = (*vpPointsKFs)[slot_query[i]];
        }
    return nm;
}

// ------------------------------------------------------------------------- b7 SearchBySim3
// ref:src/ORBmatcher.cc:1696-1939: vbAlreadyMatched1/2 from vpMatches12 (the KF2 index through
// GetIndexInKeyFrame), each direction's projection and pre-search filters by the hook (S21 * T1w
// into KF2, S12 * T2w into KF1: depth, IsInImage, distance range, PredictScale), both searches in
// one GPU call, the mutual pairs written into vpMatches12.
template <class H, class KeyFrameT, class Sim3T, class MapPointT>
int search_by_sim3(KeyFrameT *pKF1, KeyFrameT *pKF2, std::vector<MapPointT *> &vpMatches12, const Sim3T &S12,
                   float th)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<KeyFrameT> f1(*pKF1), f2(*pKF2);
    const std::vector<MapPointT *> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPointT *> vpMapPoints2 = pKF2->GetMapPointMatches();
    const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
    std::vector<uint8_t> already1(N1, 0), already2(N2, 0);
    for (int i = 0; i < N1; i++) {  // :1715-1731
        MapPointT *pMP = vpMatches12[i];
        if (!pMP) continue;
        already1[i] = 1;
        const int idx2 = H::index_in_keyframe(pMP, pKF2);
        if (idx2 >= 0 && idx2 < N2) already2[idx2] = 1;
    }
    struct Q {
        std::vector<uint8_t> desc, valid;
        std::vector<float> u, v;
        std::vector<int32_t> lvl;
        osg_fuse_queries q{};
    } q12, q21;
    auto gather = [&](const std::vector<MapPointT *> &mps, const std::vector<uint8_t> &already, bool dir12, Q &Qd) {
        const int n = (int)mps.size();
        Qd.desc.assign((size_t)n * 32, 0);
        Qd.valid.assign(n, 0);
        Qd.u.assign(n, 0.f);
        Qd.v.assign(n, 0.f);
        Qd.lvl.assign(n, 0);
        for (int i = 0; i < n; i++) {
            MapPointT *pMP = mps[i];
            if (!pMP || already[i] || pMP->isBad()) continue;  // :1737-1742 / :1813-1818
            if (!H::sim3_pair_query(pKF1, pKF2, pMP, S12, dir12, Qd.u[i], Qd.v[i], Qd.lvl[i])) continue;
            Qd.valid[i] = 1;
            mp_descriptor(pMP, &Qd.desc[(size_t)32 * i]);
        }
        Qd.q.n = n;
        Qd.q.desc = Qd.desc.data();
        Qd.q.valid = Qd.valid.data();
        Qd.q.u = Qd.u.data();
        Qd.q.v = Qd.v.data();
        Qd.q.pred_level = Qd.lvl.data();
    };
    gather(vpMapPoints1, already1, true, q12);
    gather(vpMapPoints2, already2, false, q21);
    std::vector<int32_t> match12(N1, -1);
    const int nFound = call(ctx, "osg_search_by_sim3",
                            [&] { return osg_search_by_sim3(ctx, &f1.v, &f2.v, &q12.q, &q21.q, th, match12.data()); });
    if (nFound < 0) return 0;
    for (int i1 = 0; i1 < N1; i1++)  // :1920-1936
        if (match12[i1] >= 0) vpMatches12[i1] = vpMapPoints2[match12[i1]];
    return nFound;
}

// ---------------------------------------------------------------- b6 SearchForInitialization
// ref:src/ORBmatcher.cc:735-878: vnMatches12 sized F1.mvKeysUn.size(), vbPrevMatched updated for the
// surviving matches.
template <class H, class FrameT, class PointT>
int search_for_initialization(FrameT &F1, FrameT &F2, std::vector<PointT> &vbPrevMatched, std::vector<int> &vnMatches12,
                              int windowSize, float nnratio, bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    FrameView<FrameT> f1(F1), f2(F2);
    const int n1 = (int)F1.mvKeysUn.size();
    std::vector<float> prev(2 * (size_t)n1);
    for (int i = 0; i < n1; i++) {
        prev[2 * i] = vbPrevMatched[i].x;
        prev[2 * i + 1] = vbPrevMatched[i].y;
    }
    std::vector<int32_t> m12(n1, -1);
    const int nm = call(ctx, "osg_search_for_initialization", [&] {
        return osg_search_for_initialization(ctx, &f1.v, &f2.v, prev.data(), windowSize, nnratio, checkOri, m12.data());
    });
    if (nm < 0) {
        vnMatches12.assign(n1, -1);  // ref:src/ORBmatcher.cc:739
        return 0;
    }
    vnMatches12.assign(m12.begin(), m12.end());
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0) {
            vbPrevMatched[i].x = prev[2 * i];
            vbPrevMatched[i].y = prev[2 * i + 1];
        }
    return nm;
}

// ------------------------------------------------------------------ b7 ComputeStereoMatches
// ref:src/Frame.cc:1117-1373, called by the stereo Frame constructor (ref:src/Frame.cc:165).  Reads
// mvKeys / mvKeysRight, mDescriptors / mDescriptorsRight, mvScaleFactors / mvInvScaleFactors, mb,
// mbf and both ORBextractors' mvImagePyramid (ROI views: the row step comes from Mat::step[0]);
// writes mvuRight and mvDepth.  Returns the matches kept.
template <class MatT>
struct PyramidView {
    OSG_PINNED_STRUCT(PyramidView);
    std::vector<const uint8_t *> data;
    std::vector<int32_t> rows, cols, step;
    osg_image_pyramid v{};

    PyramidView() = default;
    PyramidView(const std::vector<MatT> &pyr, int n_levels, const osg_image_pyramid *on_device = nullptr)
    {
        assign(pyr, n_levels, on_device);
    }
    void assign(const std::vector<MatT> &pyr, int n_levels, const osg_image_pyramid *on_device = nullptr)
    {
        data.clear();
        rows.clear();
        cols.clear();
        step.clear();
        v = osg_image_pyramid{};
        if (on_device) {  // levels already in HBM: read in place, no pixels cross PCIe
            v = *on_device;
            return;
        }
        for (int l = 0; l < n_levels; l++) {
            data.push_back(pyr[l].template ptr<unsigned char>(0));
            rows.push_back(pyr[l].rows);
            cols.push_back(pyr[l].cols);
            step.push_back((int32_t)pyr[l].step[0]);
        }
        v.n_levels = n_levels;
        v.on_device = 0;
        v.data = data.data();
        v.rows = rows.data();
        v.cols = cols.data();
        v.step = step.data();
    }
};

// An ORBextractor whose levels were built on the device by osg_orb_pyramid (the
// pyramid section) keeps their view, on_device = 1, as `mpOsgDeviceLevels`; the stereo matcher then
// reads those levels in place.  Extractors without the member are gathered from mvImagePyramid.
template <class E>
inline auto device_levels(const E &e, int) -> decltype(e.mpOsgDeviceLevels, (const osg_image_pyramid *)nullptr)
{
    return e.mpOsgDeviceLevels;
}
template <class E>
inline const osg_image_pyramid *device_levels(const E &, long)
{
    return nullptr;
}

template <class FrameT>
struct StereoGather {
    OSG_PINNED_STRUCT(StereoGather);
    using MatT = typename std::decay<decltype(std::declval<FrameT &>().mpORBextractorLeft->mvImagePyramid[0])>::type;
    std::vector<float> x, y, xr, yr, ang, sc, isc;
    std::vector<int32_t> o, orr;
    std::vector<uint8_t> dl, dr;
    PyramidView<MatT> pl, pr;
    osg_stereo_frame s{};
    StereoGather() = default;
    explicit StereoGather(const FrameT &F) { assign(F); }
    void assign(const FrameT &F)
    {
        sc.assign(F.mvScaleFactors.begin(), F.mvScaleFactors.end());
        isc.assign(F.mvInvScaleFactors.begin(), F.mvInvScaleFactors.end());
        pl.assign(F.mpORBextractorLeft->mvImagePyramid, (int)F.mvScaleFactors.size(), device_levels(*F.mpORBextractorLeft, 0));
        pr.assign(F.mpORBextractorRight->mvImagePyramid, (int)F.mvScaleFactors.size(), device_levels(*F.mpORBextractorRight, 0));
        for (auto *w : {&x, &y, &xr, &yr, &ang}) w->clear();
        o.clear();
        orr.clear();
        s = osg_stereo_frame{};
        const int n = F.N, nr = (int)F.mvKeysRight.size();
        for (int i = 0; i < n; i++) push_kp(F.mvKeys[i], x, y, ang, o);
        for (int i = 0; i < nr; i++) push_kp(F.mvKeysRight[i], xr, yr, ang, orr);
        const uint8_t *dlp = desc_rows(F.mDescriptors, n, dl), *drp = desc_rows(F.mDescriptorsRight, nr, dr);
        s.n = n;
        s.x = x.data();
        s.y = y.data();
        s.octave = o.data();
        s.desc = dlp;
        s.n_right = nr;
        s.xr = xr.data();
        s.yr = yr.data();
        s.octave_r = orr.data();
        s.desc_r = drp;
        s.scale_factors = sc.data();
        s.inv_scale_factors = isc.data();
        s.n_levels = (int)sc.size();
        s.mb = F.mb;
        s.mbf = F.mbf;
        s.left = pl.v;
        s.right = pr.v;
    }
};

template <class FrameT>
int compute_stereo_matches(FrameT &F)
{
    osg_ctx *ctx = thread_ctx();
    StereoGather<FrameT> g(F);
    const int n = F.N;
    F.mvuRight.assign(n, -1.0f);  // :1134-1135
    F.mvDepth.assign(n, -1.0f);
    const int nm = call(ctx, "osg_compute_stereo_matches",
                        [&] { return osg_compute_stereo_matches(ctx, &g.s, F.mvuRight.data(), F.mvDepth.data()); });
    if (nm < 0) {  // no stereo match for any keypoint
        F.mvuRight.assign(n, -1.0f);
        F.mvDepth.assign(n, -1.0f);
        return 0;
    }
    return nm;
}

// ------------------------------------------------------- b7' ComputeStereoFishEyeMatches (KB8 rigs)
// ref:src/Frame.cc:1546-1603, called by the two-camera Frame constructor (:1523).  Reads mvKeys /
// mvKeysRight, mDescriptors / mDescriptorsRight, monoLeft / monoRight, mvLevelSigma2, both cameras'
// KannalaBrandt8 parameters (GeometricCamera::getParameter 0..7) and mRlr / mtlr; writes
// mvLeftToRightMatch, mvRightToLeftMatch, mvDepth, mvuRight (-1), mvStereo3Dpoints and mnCloseMPs = 0.
template <class FrameT>
int compute_stereo_fisheye_matches(FrameT &F)
{
    osg_ctx *ctx = thread_ctx();
    const int nl = F.Nleft, nr = F.Nright;
    std::vector<float> kl(2 * (size_t)nl), kr(2 * (size_t)nr);
    std::vector<int32_t> ol(nl), orr(nr);
    for (int i = 0; i < nl; i++) {
        kl[2 * i] = F.mvKeys[i].pt.x;
        kl[2 * i + 1] = F.mvKeys[i].pt.y;
        ol[i] = F.mvKeys[i].octave;
    }
    for (int j = 0; j < nr; j++) {
        kr[2 * j] = F.mvKeysRight[j].pt.x;
        kr[2 * j + 1] = F.mvKeysRight[j].pt.y;
        orr[j] = F.mvKeysRight[j].octave;
    }
    std::vector<uint8_t> dl, dr;
    copy_desc_rows(F.mDescriptors, nl, dl);
    copy_desc_rows(F.mDescriptorsRight, nr, dr);
    std::vector<float> s2(F.mvLevelSigma2.begin(), F.mvLevelSigma2.end());
    float c1[8], c2[8], R[9], t[3];
    for (int k = 0; k < 8; k++) {
        c1[k] = F.mpCamera->getParameter(k);
        c2[k] = F.mpCamera2->getParameter(k);
    }
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) R[3 * r + c] = F.mRlr(r, c);
        t[r] = F.mtlr(r);
    }
    std::vector<float> depth(nl), p3d(3 * (size_t)nl);
    F.mvLeftToRightMatch.assign(nl, -1);  // :1558-1563
    F.mvRightToLeftMatch.assign(nr, -1);
    F.mvuRight.assign(nl, -1.0f);
    F.mnCloseMPs = 0;
    const int n = call(ctx, "osg_compute_stereo_fisheye_matches", [&] {
        return osg_compute_stereo_fisheye_matches(ctx, nl, F.monoLeft, dl.data(), kl.data(), ol.data(), nr, F.monoRight,
                                                  dr.data(), kr.data(), orr.data(), s2.data(), (int32_t)s2.size(), c1,
                                                  c2, R, t, F.mvLeftToRightMatch.data(), F.mvRightToLeftMatch.data(),
                                                  depth.data(), p3d.data());
    });
    F.mvStereo3Dpoints.resize(nl);
    if (n < 0) {  // the :1558-1563 initial state: no stereo match
        F.mvLeftToRightMatch.assign(nl, -1);
        F.mvRightToLeftMatch.assign(nr, -1);
        F.mvDepth.assign(nl, -1.0f);
        return 0;
    }
    F.mvDepth.assign(depth.begin(), depth.end());
    for (int i = 0; i < nl; i++)
        if (F.mvLeftToRightMatch[i] >= 0)
            for (int k = 0; k < 3; k++) F.mvStereo3Dpoints[i](k) = p3d[3 * (size_t)i + k];
    return n;
}

// ----------------------------------------------------------------- b8 ORBextractor per-keypoint stages
// computeOrientation + computeDescriptors inside ORBextractor::operator() (ref:src/ORBextractor.cc:
// 585-597, 1534-1545, 1557-1652), for code that lives in ORBextractor.cc (pattern / umax are its
// members).  allKeypoints[level] in level coordinates, as ComputeKeyPointsOctTree leaves them;
// blurred[level] = the GaussianBlur'd clone of mvImagePyramid[level] (:1628-1640).  Writes
// KeyPoint::angle and the 32-byte rows in allKeypoints order (level by level) into `desc`; returns
// the keypoints whose rotated pattern left their level's buffer (the reference reads foreign heap).
template <class MatT, class KeyPointT, class PointT>
int orb_describe(const std::vector<MatT> &pyramid, const std::vector<MatT> &blurred,
                 std::vector<std::vector<KeyPointT>> &allKeypoints, const std::vector<PointT> &pattern,
                 const std::vector<int> &umax, std::vector<uint8_t> &desc)
{
    osg_ctx *ctx = thread_ctx();
    const int levels = (int)allKeypoints.size();
    std::vector<float> x, y;
    std::vector<int32_t> lev;
    for (int l = 0; l < levels; l++)
        for (const KeyPointT &kp : allKeypoints[l]) {
            x.push_back(kp.pt.x);
            y.push_back(kp.pt.y);
            lev.push_back(l);
        }
    const int n = (int)x.size();
    desc.assign((size_t)n * 32, 0);
    if (pattern.size() != 512 || umax.size() < 16) {
        report(ctx, OSG_E_INVALID, "orb_describe: pattern / umax shape");
        return 0;
    }
    std::vector<int32_t> pat(2 * pattern.size());
    for (size_t i = 0; i < pattern.size(); i++) {  // cv::Point -> (x, y) int pairs
        pat[2 * i] = pattern[i].x;
        pat[2 * i + 1] = pattern[i].y;
    }
    std::vector<int32_t> um(umax.begin(), umax.begin() + 16);
    PyramidView<MatT> raw(pyramid, levels), blur(blurred, levels);
    osg_orb_keypoints K{n, x.data(), y.data(), lev.data()};
    std::vector<float> angle(n);
    const int outside = call(ctx, "osg_orb_describe", [&] {
        return osg_orb_describe(ctx, &raw.v, &blur.v, &K, pat.data(), um.data(), 1, angle.data(), desc.data());
    });
    if (outside < 0) {
        desc.assign((size_t)n * 32, 0);
        return 0;
    }
    int i = 0;
    for (int l = 0; l < levels; l++)
        for (KeyPointT &kp : allKeypoints[l]) kp.angle = angle[i++];
    return outside;
}

// ------------------------------------------------- b9 ORBextractor::ComputeKeyPointsOctTree
// ref:src/ORBextractor.cc:1065-1198 over the extractor's members (mvImagePyramid, mnFeaturesPerLevel,
// mvScaleFactor, iniThFAST, minThFAST): FAST per cell + DistributeOctTree on the GPU path, then the
// :1190-1196 loop's fields (pt in level coordinates, octave, size).  KeyPoint::angle stays FAST's -1:
// computeOrientation runs with the descriptors in orb_describe (IC_Angle reads the raw level only,
// so the angles are the same as the reference's :1200-1204 pass).
template <class MatT, class KeyPointT>
int compute_keypoints_oct_tree(const std::vector<MatT> &pyramid, std::vector<std::vector<KeyPointT>> &allKeypoints,
                               const std::vector<int> &nFeaturesPerLevel, const std::vector<float> &scaleFactors,
                               int iniThFAST, int minThFAST)
{
    osg_ctx *ctx = thread_ctx();
    const int levels = (int)pyramid.size();
    allKeypoints.assign(levels, {});
    if ((int)nFeaturesPerLevel.size() < levels || (int)scaleFactors.size() < levels) {
        report(ctx, OSG_E_INVALID, "compute_keypoints_oct_tree: per-level tables");
        return 0;
    }
    PyramidView<MatT> raw(pyramid, levels);
    std::vector<int32_t> nf(nFeaturesPerLevel.begin(), nFeaturesPerLevel.begin() + levels);
    int cap = 64;
    for (int l = 0; l < levels; l++) cap += 2 * std::max(nf[l], 0) + 8;  // the octree stops within 3 of N
    std::vector<float> x(cap), y(cap), resp(cap), size(cap);
    std::vector<int32_t> ls(levels + 1);
    if (call(ctx, "osg_orb_detect", [&] {
            return osg_orb_detect(ctx, &raw.v, iniThFAST, minThFAST, nf.data(), scaleFactors.data(), cap, x.data(),
                                  y.data(), resp.data(), size.data(), ls.data());
        }) < 0)
        return 0;
    for (int l = 0; l < levels; l++) {
        allKeypoints[l].reserve(ls[l + 1] - ls[l]);
        for (int i = ls[l]; i < ls[l + 1]; i++) {
            KeyPointT kp;
            kp.pt.x = x[i];
            kp.pt.y = y[i];
            kp.size = size[i];
            kp.angle = -1.f;
            kp.response = resp[i];
            kp.octave = l;
            allKeypoints[l].push_back(kp);
        }
    }
    return ls[levels];
}

// ----------------------------------------------------------------- b3 SearchForTriangulation
// ref:src/ORBmatcher.cc:1045-1328.  vMatchedPairs = (KF1 index, KF2 index) in ascending KF1 index.
// The epipole and the F12 matrices come from the hook (the reference's Sophus / Eigen code).
template <class H, class KeyFrameT>
int search_for_triangulation(KeyFrameT *pKF1, KeyFrameT *pKF2, std::vector<std::pair<size_t, size_t>> &vMatchedPairs,
                             bool bOnlyStereo, bool bCoarse, bool checkOri)
{
    osg_ctx *ctx = thread_ctx();
    struct Side {
        std::vector<uint8_t> desc, has_mp;
        std::vector<float> x, y, a;
        std::vector<int32_t> oct;
    } s[2];
    KeyFrameT *K[2] = {pKF1, pKF2};
    osg_kf_side v[2];
    std::vector<std::unique_ptr<FeatVecCSR<decltype(pKF1->mFeatVec)>>> fv;
    for (int k = 0; k < 2; k++) {
        KeyFrameT *p = K[k];
        const int n = p->N;
        copy_desc_rows(p->mDescriptors, n, s[k].desc);
        s[k].has_mp.resize(n);
        for (int i = 0; i < n; i++) {
            // ref:src/ORBmatcher.cc:1142-1144 / 1184-1186: mvKeysUn, or mvKeys / mvKeysRight on a rig
            const auto &kp = (p->NLeft == -1) ? p->mvKeysUn[i] : (i < p->NLeft ? p->mvKeys[i] : p->mvKeysRight[i - p->NLeft]);
            s[k].x.push_back(kp.pt.x);
            s[k].y.push_back(kp.pt.y);
            s[k].a.push_back(kp.angle);
            s[k].oct.push_back(kp.octave);
            s[k].has_mp[i] = p->GetMapPoint(i) != nullptr;
        }
        fv.emplace_back(new FeatVecCSR<decltype(pKF1->mFeatVec)>(p->mFeatVec));
        v[k] = osg_kf_side{n, p->NLeft, p->mpCamera2 != nullptr, s[k].desc.data(), s[k].x.data(), s[k].y.data(),
                           s[k].a.data(), s[k].oct.data(), p->mvuRight.empty() ? nullptr : p->mvuRight.data(),
                           s[k].has_mp.data(), p->mvLevelSigma2.data(), p->mvScaleFactors.data(),
                           (int32_t)p->mvScaleFactors.size(), fv[k]->view()};
    }
    osg_triang_geom g;
    H::triang_geom(pKF1, pKF2, g);
    std::vector<int32_t> m12(pKF1->N, -1);
    const int nm = call(ctx, "osg_search_for_triangulation", [&] {
        return osg_search_for_triangulation(ctx, &v[0], &v[1], &g, bOnlyStereo, bCoarse, checkOri, m12.data());
    });
    vMatchedPairs.clear();  // ref:src/ORBmatcher.cc:1317
    if (nm < 0) return 0;
    vMatchedPairs.reserve(nm);
    for (int i = 0; i < pKF1->N; i++)
        if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
    return nm;
}

// ------------------------------------------------------ b4 MapPoint::ComputeDistinctiveDescriptors
// ref:src/MapPoint.cc:444-535 for a list of MapPoints in one launch (the loops of
// ref:src/LocalMapping.cc:421-436, 1066-1082).  Gathers each point's observation rows in the
// reference's order (mObservations map order; left row, then right row; bad keyframes skipped) and
// writes the chosen row back through H::set_descriptor (mDescriptor is protected: the hook is a
// friend of MapPoint).  Null / bad points and points without rows are left alone.
template <class H, class MapPointT>
void compute_distinctive_descriptors(const std::vector<MapPointT *> &vpMPs)
{
    osg_ctx *ctx = thread_ctx();
    const int np = (int)vpMPs.size();
    std::vector<uint8_t> rows;
    std::vector<int32_t> start(np + 1, 0);
    for (int p = 0; p < np; p++) {
        MapPointT *pMP = vpMPs[p];
        if (pMP && !pMP->isBad()) {
            const auto observations = pMP->GetObservations();
            for (const auto &kv : observations) {
                const auto *pKF = kv.first;
                if (pKF->isBad()) continue;
                const int l = std::get<0>(kv.second), r = std::get<1>(kv.second);
                for (int idx : {l, r}) {
                    if (idx == -1) continue;
                    const size_t o = rows.size();
                    rows.resize(o + 32);
                    std::memcpy(&rows[o], pKF->mDescriptors.template ptr<uint8_t>(idx), 32);
                }
            }
        }
        start[p + 1] = (int32_t)(rows.size() / 32);
    }
    std::vector<int32_t> best(np, -1);
    if (call(ctx, "osg_compute_distinctive_descriptors",
             [&] { return osg_compute_distinctive_descriptors(ctx, rows.data(), start.data(), np, best.data()); }) < 0)
        return;  // descriptors unchanged
    for (int p = 0; p < np; p++)
        if (best[p] >= 0) H::set_descriptor(vpMPs[p], &rows[32 * ((size_t)start[p] + best[p])]);
}

// ------------------------------------------------------------------- a10 PoseOptimization
// ref:src/Optimizer.cc:71-420: one edge per Frame slot holding a MapPoint, in slot order; the
// result sets mvbOutlier and the pose and returns nInitialCorrespondences - nBad.
// Locking as the reference: `gather_mutex` (MapPoint::mGlobalMutex in the ORB-SLAM3 tree) is held
// only while the edges are built from the MapPoints (ref:src/Optimizer.cc:128-286); the GPU solve
// and the write-back into the Frame run without it, so LocalMapping / LoopClosing's SetWorldPos
// are not blocked for the device round trip.
struct NoMutex {
    void lock() {}
    void unlock() {}
};

// PoseGather: one Frame's edges (the gather of ref:src/Optimizer.cc:128-286), shared by the single and
// the batched entry points.
template <class H, class FrameT>
struct PoseGather {
    OSG_PINNED_STRUCT(PoseGather);
    std::vector<int8_t> kind;
    std::vector<double> xw, obs;
    std::vector<float> isig;
    std::vector<int> slot;
    std::vector<uint8_t> outl;
    osg_pose_problem p{};
    PoseGather() = default;
    template <class MutexT>
    PoseGather(FrameT *pFrame, MutexT *gather_mutex) { assign(pFrame, gather_mutex); }
    template <class MutexT>
    void assign(FrameT *pFrame, MutexT *gather_mutex)
    {
        const int N = pFrame->N;
        p = osg_pose_problem{};
        // sized for every keypoint, written in place, trimmed to the edges found (push_back per edge
        // measured slower)
        kind.resize(N);
        xw.resize(3 * (size_t)N);
        obs.resize(3 * (size_t)N);
        isig.resize(N);
        slot.resize(N);
        int m = 0;
        const bool two = (bool)pFrame->mpCamera2;
        std::unique_lock<MutexT> gather_lock;
        if (gather_mutex) gather_lock = std::unique_lock<MutexT>(*gather_mutex);
        constexpr int PF = 8;  // world_pos reads scattered heap MapPoints: fetch a few ahead (two lines each)
        for (int i = 0; i < N; i++) {
            if (i + PF < N)
                if (const auto *q = pFrame->mvpMapPoints[i + PF]) {
                    __builtin_prefetch(q);
                    __builtin_prefetch((const char *)q + 64);
                }
            auto *pMP = pFrame->mvpMapPoints[i];
            if (!pMP) continue;
            double *X = &xw[3 * (size_t)m], *o = &obs[3 * (size_t)m];
            H::world_pos(pMP, X);
            int8_t k;
            o[0] = o[1] = o[2] = 0.0;
            int oct;
            if (!two) {
                const auto &kp = pFrame->mvKeysUn[i];
                k = pFrame->mvuRight[i] < 0 ? OSG_EDGE_MONO : OSG_EDGE_STEREO;
                o[0] = kp.pt.x;
                o[1] = kp.pt.y;
                if (k == OSG_EDGE_STEREO) o[2] = pFrame->mvuRight[i];
                oct = kp.octave;
            } else if (i < pFrame->Nleft) {
                const auto &kp = pFrame->mvKeys[i];
                k = OSG_EDGE_MONO;
                o[0] = kp.pt.x;
                o[1] = kp.pt.y;
                oct = kp.octave;
            } else {
                const auto &kp = pFrame->mvKeysRight[i - pFrame->Nleft];
                k = OSG_EDGE_BODY;
                o[0] = kp.pt.x;
                o[1] = kp.pt.y;
                oct = kp.octave;
            }
            pFrame->mvbOutlier[i] = false;
            kind[m] = k;
            isig[m] = pFrame->mvInvLevelSigma2[oct];
            slot[m] = i;
            m++;
        }
        kind.resize(m);
        xw.resize(3 * (size_t)m);
        obs.resize(3 * (size_t)m);
        isig.resize(m);
        slot.resize(m);
        if (gather_lock.owns_lock()) gather_lock.unlock();  // ref:src/Optimizer.cc:286, end of Step 3
        H::pose(*pFrame, p.pose);
        p.n_edges = (int32_t)kind.size();
        p.kind = kind.data();
        p.xw = xw.data();
        p.obs = obs.data();
        p.inv_sigma2 = isig.data();
        H::camera(*pFrame, false, p.cam);
        if (two) H::camera(*pFrame, true, p.cam2);
        outl.resize(kind.size());
    }
    // mvbOutlier and the pose, as ref:src/Optimizer.cc:405-419; a frame with < 3 edges keeps its pose
    int apply(FrameT *pFrame, const osg_pose_result &r) const
    {
        if (p.n_edges < 3) return 0;  // ref:src/Optimizer.cc:289-290 (pose untouched)
        for (size_t e = 0; e < slot.size(); e++) pFrame->mvbOutlier[slot[e]] = outl[e] != 0;
        H::set_pose(*pFrame, r.pose);
        return r.n_inliers;
    }
};

template <class H, class FrameT, class MutexT = NoMutex>
int pose_optimization(FrameT *pFrame, MutexT *gather_mutex = nullptr)
{
    osg_ctx *ctx = thread_ctx();
    PoseGather<H, FrameT> &g = gather_pool<PoseGather<H, FrameT>>(1)[0];
    g.assign(pFrame, gather_mutex);
    osg_pose_result r{};
    r.outlier = g.outl.data();
    if (call(ctx, "osg_pose_optimization", [&] { return osg_pose_optimization(ctx, &g.p, &r); }) < 0) return 0;
    return g.apply(pFrame, r);
}

// ---------------------------------------------------------- a11 LocalBundleAdjustment (g2o part)
// The local window (ref:src/Optimizer.cc:1762-1873: lLocalKeyFrames, lLocalMapPoints,
// lFixedCameras) is collected by the reference code unchanged; from the graph build on
// (ref:src/Optimizer.cc:1877-2203) this replaces g2o.  Vertex order = g2o id order (KeyFrames by
// mnId, MapPoints by mnId + maxKFid + 1); edges in the reference's insertion order (MapPoint list
// order x observation map order; left/stereo edge, then the right-camera edge).
template <class KeyFrameT, class MapPointT>
struct LbaOutcome {
    std::vector<std::pair<KeyFrameT *, MapPointT *>> to_erase;  // vToErase
    std::vector<std::pair<KeyFrameT *, std::vector<double>>> poses;   // optimised local KF poses (7)
    std::vector<std::pair<MapPointT *, std::vector<double>>> points;  // optimised MapPoints (3)
    int num_fixedKF = 0, num_OptKF = 0, num_MPs = 0, num_edges = 0;
    bool aborted = false;
};

template <class H, class KeyFrameT, class MapPointT, class MapT>
LbaOutcome<KeyFrameT, MapPointT> local_bundle_adjustment(const std::list<KeyFrameT *> &lLocalKeyFrames,
                                                         const std::list<KeyFrameT *> &lFixedCameras,
                                                         const std::list<MapPointT *> &lLocalMapPoints,
                                                         MapT *pCurrentMap, unsigned long initKFid,
                                                         bool *pbStopFlag, bool bInertial)
{
    osg_ctx *ctx = thread_ctx();
    LbaOutcome<KeyFrameT, MapPointT> out;
    // vertices sorted by g2o id
    std::vector<std::pair<unsigned long, KeyFrameT *>> kfs;
    std::unordered_map<KeyFrameT *, int> kf_fixed;
    unsigned long maxKFid = 0;
    for (auto *k : lLocalKeyFrames) {
        kfs.push_back({k->mnId, k});
        kf_fixed[k] = (k->mnId == initKFid);
        maxKFid = std::max(maxKFid, (unsigned long)k->mnId);
    }
    for (auto *k : lFixedCameras) {
        kfs.push_back({k->mnId, k});
        kf_fixed[k] = 1;
        maxKFid = std::max(maxKFid, (unsigned long)k->mnId);
    }
    std::sort(kfs.begin(), kfs.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::unordered_map<KeyFrameT *, int> kf_index;
    std::vector<double> pose(7 * kfs.size());
    std::vector<uint8_t> fixed(kfs.size());
    std::vector<osg_camera> cams(2 * kfs.size());
    for (size_t i = 0; i < kfs.size(); i++) {
        kf_index[kfs[i].second] = (int)i;
        H::pose(*kfs[i].second, &pose[7 * i]);
        fixed[i] = (uint8_t)kf_fixed[kfs[i].second];
        H::camera(*kfs[i].second, false, cams[2 * i]);
        if (kfs[i].second->mpCamera2) H::camera(*kfs[i].second, true, cams[2 * i + 1]);
    }
    out.num_OptKF = (int)lLocalKeyFrames.size();
    // ref:src/Optimizer.cc:1781-1790,1828: the fixed cameras plus the map's init KeyFrame when it is
    // one of the local KeyFrames (its vertex is fixed too, :1909)
    bool init_local = false;
    for (auto *k : lLocalKeyFrames) init_local |= (k->mnId == initKFid);
    out.num_fixedKF = (int)lFixedCameras.size() + (init_local ? 1 : 0);
    std::vector<std::pair<unsigned long, MapPointT *>> mps;
    for (auto *p : lLocalMapPoints) mps.push_back({p->mnId, p});
    std::sort(mps.begin(), mps.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::unordered_map<MapPointT *, int> mp_index;
    std::vector<double> point(3 * mps.size());
    for (size_t i = 0; i < mps.size(); i++) {
        mp_index[mps[i].second] = (int)i;
        H::world_pos(mps[i].second, &point[3 * i]);
    }
    out.num_MPs = (int)mps.size();
    std::vector<int32_t> e_point, e_pose, e_cam;
    std::vector<int8_t> e_kind;
    std::vector<double> e_obs;
    std::vector<float> e_isig;
    std::vector<std::pair<KeyFrameT *, MapPointT *>> e_pair;
    for (auto *pMP : lLocalMapPoints) {
        const auto observations = pMP->GetObservations();
        for (const auto &ob : observations) {
            KeyFrameT *pKFi = ob.first;
            if (pKFi->isBad() || pKFi->GetMap() != pCurrentMap) continue;
            const auto itk = kf_index.find(pKFi);
            if (itk == kf_index.end()) continue;
            const int leftIndex = std::get<0>(ob.second);
            auto add = [&](int8_t kind, int cam, const auto &kp, double ur) {
                e_point.push_back(mp_index[pMP]);
                e_pose.push_back(itk->second);
                e_kind.push_back(kind);
                e_cam.push_back(cam);
                e_obs.push_back(kp.pt.x);
                e_obs.push_back(kp.pt.y);
                e_obs.push_back(ur);
                e_isig.push_back(pKFi->mvInvLevelSigma2[kp.octave]);
                e_pair.push_back({pKFi, pMP});
            };
            if (leftIndex != -1 && pKFi->mvuRight[leftIndex] < 0)
                add(OSG_EDGE_MONO, 2 * itk->second, pKFi->mvKeysUn[leftIndex], 0.0);
            else if (leftIndex != -1 && pKFi->mvuRight[leftIndex] >= 0)
                add(OSG_EDGE_STEREO, 2 * itk->second, pKFi->mvKeysUn[leftIndex], pKFi->mvuRight[leftIndex]);
            if (pKFi->mpCamera2) {
                const int rightIndex = std::get<1>(ob.second);
                if (rightIndex != -1)
                    add(OSG_EDGE_BODY, 2 * itk->second + 1, pKFi->mvKeysRight[rightIndex - pKFi->NLeft], 0.0);
            }
        }
    }
    out.num_edges = (int)e_kind.size();
    if (pbStopFlag && *pbStopFlag) {
        out.aborted = true;
        return out;
    }
    osg_ba_graph g{};
    g.n_poses = (int32_t)kfs.size();
    g.pose = pose.data();
    g.pose_fixed = fixed.data();
    g.n_points = (int32_t)mps.size();
    g.point = point.data();
    g.n_edges = (int32_t)e_kind.size();
    g.e_point = e_point.data();
    g.e_pose = e_pose.data();
    g.e_kind = e_kind.data();
    g.e_cam = e_cam.data();
    g.e_obs = e_obs.data();
    g.e_inv_sigma2 = e_isig.data();
    g.n_cams = (int32_t)cams.size();
    g.cams = cams.data();
    g.iterations = 10;
    g.user_lambda_init = bInertial ? 100.0 : 0.0;
    std::vector<double> pose_out(pose.size()), point_out(point.size());
    std::vector<uint8_t> bad(e_kind.size());
    osg_ba_result r{};
    r.pose = pose_out.data();
    r.point = point_out.data();
    r.edge_bad = bad.data();
    static_assert(sizeof(bool) == 1, "pbStopFlag is passed as one byte");
    if (call(ctx, "osg_local_bundle_adjustment", [&] {
            return osg_local_bundle_adjustment(ctx, &g, &r, reinterpret_cast<const volatile uint8_t *>(pbStopFlag));
        }) < 0) {
        out.aborted = true;  // no poses: the caller returns as on an abort, nothing written back
        return out;
    }
    out.aborted = r.aborted != 0;
    // ref:src/Optimizer.cc:2123-2168: edges over the chi2 threshold or behind the camera, collected
    // in the reference's vToErase order (mono edges, then right-camera edges, then stereo edges),
    // skipping MapPoints another thread marked bad while the solve ran (:2130, :2145, :2160)
    for (int k : {OSG_EDGE_MONO, OSG_EDGE_BODY, OSG_EDGE_STEREO})
        for (size_t e = 0; e < bad.size(); e++)
            if (e_kind[e] == k && bad[e] && !e_pair[e].second->isBad()) out.to_erase.push_back(e_pair[e]);
    // only the local KeyFrames are written back (fixed cameras are not), ref:src/Optimizer.cc:2187-2203
    for (auto *k : lLocalKeyFrames) {
        const int i = kf_index[k];
        out.poses.push_back({k, std::vector<double>(&pose_out[7 * i], &pose_out[7 * i] + 7)});
    }
    for (size_t i = 0; i < mps.size(); i++)
        out.points.push_back({mps[i].second, std::vector<double>(&point_out[3 * i], &point_out[3 * i] + 3)});
    return out;
}

// Applies an LbaOutcome exactly as ref:src/Optimizer.cc:2171-2203 does; the caller holds
// pMap->mMutexMapUpdate.
template <class H, class KeyFrameT, class MapPointT>
void apply_local_bundle_adjustment(const LbaOutcome<KeyFrameT, MapPointT> &o)
{
    for (const auto &km : o.to_erase) {
        km.first->EraseMapPointMatch(km.second);
        km.second->EraseObservation(km.first);
    }
    for (const auto &kp : o.poses) H::set_pose(*kp.first, kp.second.data());
    for (const auto &mp : o.points) H::set_world_pos(mp.first, mp.second.data());
}

// ------------------------------------------------------- §8(f) rank 4: global BA (the g2o part)
// Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust)
// (ref:src/Optimizer.cc:2850-3237; GlobalBundleAdjustemnt hands it the whole map, :2831-2839).
// Vertices: every non-bad KeyFrame (only the map's init KeyFrame fixed, :2912-2930) and every
// non-bad MapPoint with a valid observation (:2939-3110), in g2o id order as for the local BA.
// Edges in the reference's insertion order (vpMP order x observation map order; left / stereo edge,
// then the right-camera edge behind the reference's `rightIndex < mvKeysRight.size()` test, which it
// applies before rightIndex -= NLeft, :3063-3097).  Mono / stereo edges carry Huber only with
// bRobust, body edges always; deltas sqrt(5.99) / sqrt(7.815) as floats (:2933-2934).
template <class KeyFrameT, class MapPointT>
struct GbaOutcome {
    std::vector<std::pair<KeyFrameT *, std::vector<double>>> poses;   // every non-bad KeyFrame (7)
    std::vector<std::pair<MapPointT *, std::vector<double>>> points;  // the graph's MapPoints (3)
    int iterations = 0;
};

template <class H, class KeyFrameT, class MapPointT>
GbaOutcome<KeyFrameT, MapPointT> bundle_adjustment(const std::vector<KeyFrameT *> &vpKFs,
                                                   const std::vector<MapPointT *> &vpMP, unsigned long initKFid,
                                                   int nIterations, bool *pbStopFlag, bool bRobust)
{
    osg_ctx *ctx = thread_ctx();
    GbaOutcome<KeyFrameT, MapPointT> out;
    std::vector<std::pair<unsigned long, KeyFrameT *>> kfs;
    unsigned long maxKFid = 0;
    for (auto *k : vpKFs) {
        if (k->isBad()) continue;
        kfs.push_back({k->mnId, k});
        maxKFid = std::max(maxKFid, (unsigned long)k->mnId);
    }
    std::sort(kfs.begin(), kfs.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::unordered_map<KeyFrameT *, int> kf_index;
    std::vector<double> pose(7 * kfs.size());
    std::vector<uint8_t> fixed(kfs.size());
    std::vector<osg_camera> cams(2 * kfs.size());
    for (size_t i = 0; i < kfs.size(); i++) {
        KeyFrameT *k = kfs[i].second;
        kf_index[k] = (int)i;
        H::pose(*k, &pose[7 * i]);
        fixed[i] = (uint8_t)(k->mnId == initKFid);
        H::camera(*k, false, cams[2 * i]);
        if (k->mpCamera2) H::camera(*k, true, cams[2 * i + 1]);
    }
    std::vector<MapPointT *> in_graph;  // vpMP order
    std::vector<int32_t> e_mp, e_pose, e_cam;
    std::vector<int8_t> e_kind;
    std::vector<uint8_t> e_rob;
    std::vector<double> e_obs;
    std::vector<float> e_isig;
    for (auto *pMP : vpMP) {
        if (pMP->isBad()) continue;
        const auto observations = pMP->GetObservations();
        int nEdges = 0;
        for (const auto &ob : observations) {
            KeyFrameT *pKF = ob.first;
            if (pKF->isBad() || pKF->mnId > maxKFid) continue;
            const auto itk = kf_index.find(pKF);
            if (itk == kf_index.end()) continue;
            nEdges++;
            const int leftIndex = std::get<0>(ob.second);
            auto add = [&](int8_t kind, int cam, const auto &kp, double ur, bool robust) {
                e_mp.push_back((int32_t)in_graph.size());
                e_pose.push_back(itk->second);
                e_kind.push_back(kind);
                e_cam.push_back(cam);
                e_rob.push_back((uint8_t)robust);
                e_obs.push_back(kp.pt.x);
                e_obs.push_back(kp.pt.y);
                e_obs.push_back(ur);
                e_isig.push_back(pKF->mvInvLevelSigma2[kp.octave]);
            };
            if (leftIndex != -1 && pKF->mvuRight[leftIndex] < 0)
                add(OSG_EDGE_MONO, 2 * itk->second, pKF->mvKeysUn[leftIndex], 0.0, bRobust);
            else if (leftIndex != -1 && pKF->mvuRight[leftIndex] >= 0)
                add(OSG_EDGE_STEREO, 2 * itk->second, pKF->mvKeysUn[leftIndex], pKF->mvuRight[leftIndex], bRobust);
            if (pKF->mpCamera2) {
                int rightIndex = std::get<1>(ob.second);
                if (rightIndex != -1 && rightIndex < (int)pKF->mvKeysRight.size()) {
                    rightIndex -= pKF->NLeft;
                    add(OSG_EDGE_BODY, 2 * itk->second + 1, pKF->mvKeysRight[rightIndex], 0.0, true);
                }
            }
        }
        if (nEdges > 0) in_graph.push_back(pMP);  // :3100-3110: a point without edges leaves the graph
    }
    // MapPoints in g2o id order (mnId + maxKFid + 1)
    std::vector<std::pair<unsigned long, int>> ord;
    for (size_t i = 0; i < in_graph.size(); i++) ord.push_back({(unsigned long)in_graph[i]->mnId, (int)i});
    std::sort(ord.begin(), ord.end());
    std::vector<int32_t> slot(in_graph.size());
    std::vector<double> point(3 * in_graph.size());
    for (size_t j = 0; j < ord.size(); j++) {
        slot[ord[j].second] = (int32_t)j;
        H::world_pos(in_graph[ord[j].second], &point[3 * j]);
    }
    std::vector<int32_t> e_point(e_mp.size());
    for (size_t e = 0; e < e_mp.size(); e++) e_point[e] = slot[e_mp[e]];
    osg_ba_graph g{};
    g.n_poses = (int32_t)kfs.size();
    g.pose = pose.data();
    g.pose_fixed = fixed.data();
    g.n_points = (int32_t)in_graph.size();
    g.point = point.data();
    g.n_edges = (int32_t)e_kind.size();
    g.e_point = e_point.data();
    g.e_pose = e_pose.data();
    g.e_kind = e_kind.data();
    g.e_cam = e_cam.data();
    g.e_obs = e_obs.data();
    g.e_inv_sigma2 = e_isig.data();
    g.n_cams = (int32_t)cams.size();
    g.cams = cams.data();
    g.iterations = nIterations;
    g.user_lambda_init = 0.0;
    g.e_robust = e_rob.data();
    g.huber_mono = (float)std::sqrt(5.99);   // const float thHuber2D = sqrt(5.99)
    g.huber_stereo = (float)std::sqrt(7.815);
    std::vector<double> pose_out(pose.size()), point_out(point.size());
    std::vector<uint8_t> bad(e_kind.size());
    osg_ba_result r{};
    r.pose = pose_out.data();
    r.point = point_out.data();
    r.edge_bad = bad.data();
    static_assert(sizeof(bool) == 1, "pbStopFlag is passed as one byte");
    if (call(ctx, "osg_bundle_adjustment", [&] {
            return osg_bundle_adjustment(ctx, &g, &r, reinterpret_cast<const volatile uint8_t *>(pbStopFlag));
        }) < 0) {  // an optimize() that stopped before its first iteration: the input state
        pose_out = pose;
        point_out = point;
        r.iterations = 0;
    }
    out.iterations = r.iterations;
    for (size_t i = 0; i < kfs.size(); i++)
        out.poses.push_back({kfs[i].second, std::vector<double>(&pose_out[7 * i], &pose_out[7 * i] + 7)});
    for (size_t j = 0; j < ord.size(); j++)
        out.points.push_back({in_graph[ord[j].second], std::vector<double>(&point_out[3 * j], &point_out[3 * j] + 3)});
    return out;
}

// Writes a GbaOutcome as ref:src/Optimizer.cc:3122-3236 does: straight into the map after the
// monocular initialisation (nLoopKF == the map's origin KeyFrame id), otherwise into mTcwGBA /
// mPosGBA with mnBAGlobalForKF = nLoopKF for LoopClosing to apply.
// KeyFrames and MapPoints another thread marked bad during the solve are skipped, as the reference's
// write-back loops re-check isBad() (:3127, :3219).
template <class H, class KeyFrameT, class MapPointT>
void apply_bundle_adjustment(const GbaOutcome<KeyFrameT, MapPointT> &o, unsigned long nLoopKF, bool into_map)
{
    for (const auto &kp : o.poses) {
        if (kp.first->isBad()) continue;
        if (into_map) H::set_pose(*kp.first, kp.second.data());
        else H::set_gba_pose(*kp.first, kp.second.data(), nLoopKF);
    }
    for (const auto &mp : o.points) {
        if (mp.first->isBad()) continue;
        if (into_map) H::set_world_pos(mp.first, mp.second.data());
        else H::set_gba_pos(mp.first, mp.second.data(), nLoopKF);
    }
}

// ------------------------------------------ §8(f) rank 4: the map-merge window BA (the g2o part)
// Optimizer::LocalBundleAdjustment(pMainKF, vpAdjustKF, vpFixedKF, pbStopFlag)
// (ref:src/Optimizer.cc:5211-5672), LoopClosing's merge.  Vertices: vpFixedKF (fixed) then
// vpAdjustKF, each non-bad and in pMainKF's map (a KeyFrame listed twice keeps its first, fixed
// vertex, as g2o's addVertex does), with their MapPoints (GetMapPoints() set order, deduplicated by
// mnBALocalForMerge, which is set on both as the reference does); edges per MapPoint in observation
// map order, mono or stereo by mvuRight, Huber sqrt(5.99) / sqrt(7.815).  Two passes through the C
// ABI: optimize(5) with the kernels; then (unless stopped) level-1 marking by chi2 / depth, every
// kernel dropped and a fresh optimize(10) over the level-0 edges; the final classification reads
// the level-1 edges' first-pass chi2 and the final depth.
template <class KeyFrameT, class MapPointT>
struct MergeLbaOutcome {
    std::vector<std::pair<KeyFrameT *, MapPointT *>> to_erase;        // vToErase, mono edges then stereo
    std::vector<std::pair<KeyFrameT *, std::vector<double>>> poses;   // vpAdjustKF (7)
    std::vector<std::pair<MapPointT *, std::vector<double>>> points;  // vpMPs (3)
    bool aborted = false;                                             // stopped before the first pass
};

inline bool depth_positive_se3(const double *q, const double *X)
{  // SE3Quat::map(X).z > 0 (Eigen's quaternion-vector product)
    const double uv[3] = {2 * (q[1] * X[2] - q[2] * X[1]), 2 * (q[2] * X[0] - q[0] * X[2]), 2 * (q[0] * X[1] - q[1] * X[0])};
    return X[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]) + q[6] > 0;
}

template <class H, class KeyFrameT, class MapPointT>
MergeLbaOutcome<KeyFrameT, MapPointT> merge_local_bundle_adjustment(KeyFrameT *pMainKF,
                                                                    const std::vector<KeyFrameT *> &vpAdjustKF,
                                                                    const std::vector<KeyFrameT *> &vpFixedKF,
                                                                    bool *pbStopFlag)
{
    osg_ctx *ctx = thread_ctx();
    MergeLbaOutcome<KeyFrameT, MapPointT> out;
    const auto *pCurrentMap = pMainKF->GetMap();
    const unsigned long mark = pMainKF->mnId;
    std::vector<std::pair<unsigned long, KeyFrameT *>> kfs;
    std::unordered_map<KeyFrameT *, int> kf_fixed;
    std::vector<MapPointT *> vpMPs;
    unsigned long maxKFid = 0;
    auto take = [&](KeyFrameT *k, bool fixed) {  // :5242-5315
        if (k->isBad() || k->GetMap() != pCurrentMap) return;
        k->mnBALocalForMerge = mark;
        if (kf_fixed.count(k)) return;
        kf_fixed[k] = fixed;
        kfs.push_back({k->mnId, k});
        maxKFid = std::max(maxKFid, (unsigned long)k->mnId);
        for (MapPointT *p : k->GetMapPoints())
            if (p && !p->isBad() && p->GetMap() == pCurrentMap && p->mnBALocalForMerge != mark) {
                vpMPs.push_back(p);
                p->mnBALocalForMerge = mark;
            }
    };
    for (auto *k : vpFixedKF) take(k, true);
    for (auto *k : vpAdjustKF) take(k, false);
    std::sort(kfs.begin(), kfs.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::unordered_map<KeyFrameT *, int> kf_index;
    std::vector<double> pose(7 * kfs.size());
    std::vector<uint8_t> fixed(kfs.size());
    std::vector<osg_camera> cams(kfs.size());
    for (size_t i = 0; i < kfs.size(); i++) {
        kf_index[kfs[i].second] = (int)i;
        H::pose(*kfs[i].second, &pose[7 * i]);
        fixed[i] = (uint8_t)kf_fixed[kfs[i].second];
        H::camera(*kfs[i].second, false, cams[i]);
    }
    // MapPoints (every non-bad one is a vertex, :5347-5358) in g2o id order
    std::vector<std::pair<unsigned long, MapPointT *>> mps;
    for (auto *p : vpMPs)
        if (!p->isBad()) mps.push_back({p->mnId, p});
    std::sort(mps.begin(), mps.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::unordered_map<MapPointT *, int> mp_index;
    std::vector<double> point(3 * mps.size());
    for (size_t j = 0; j < mps.size(); j++) {
        mp_index[mps[j].second] = (int)j;
        H::world_pos(mps[j].second, &point[3 * j]);
    }
    std::vector<int32_t> e_point, e_pose, e_cam;
    std::vector<int8_t> e_kind;
    std::vector<double> e_obs;
    std::vector<float> e_isig;
    std::vector<std::pair<KeyFrameT *, MapPointT *>> e_pair;
    for (auto *pMP : vpMPs) {  // :5347-5442
        if (pMP->isBad()) continue;
        for (const auto &ob : pMP->GetObservations()) {
            KeyFrameT *pKF = ob.first;
            const int li = std::get<0>(ob.second);
            if (pKF->isBad() || pKF->mnId > maxKFid || pKF->mnBALocalForMerge != mark || li < 0 || !pKF->GetMapPoint(li))
                continue;
            const auto itk = kf_index.find(pKF);
            if (itk == kf_index.end()) continue;
            const auto &kp = pKF->mvKeysUn[li];
            const bool mono = pKF->mvuRight[li] < 0;
            e_point.push_back(mp_index[pMP]);
            e_pose.push_back(itk->second);
            e_kind.push_back(mono ? OSG_EDGE_MONO : OSG_EDGE_STEREO);
            e_cam.push_back(itk->second);
            e_obs.push_back(kp.pt.x);
            e_obs.push_back(kp.pt.y);
            e_obs.push_back(mono ? 0.0 : pKF->mvuRight[li]);
            e_isig.push_back(pKF->mvInvLevelSigma2[kp.octave]);
            e_pair.push_back({pKF, pMP});
        }
    }
    if (pbStopFlag && *pbStopFlag) {  // :5444-5446
        out.aborted = true;
        return out;
    }
    const size_t ne = e_kind.size();
    auto pass = [&](const std::vector<size_t> &edges, const std::vector<uint8_t> &robust, int iters,
                    const std::vector<double> &p_in, const std::vector<double> &x_in, std::vector<double> &p_out,
                    std::vector<double> &x_out, std::vector<uint8_t> &bad, std::vector<double> &chi2) {
        std::vector<int32_t> ep, eo, ec;
        std::vector<int8_t> ek;
        std::vector<double> eobs;
        std::vector<float> eis;
        for (size_t e : edges) {
            ep.push_back(e_point[e]);
            eo.push_back(e_pose[e]);
            ec.push_back(e_cam[e]);
            ek.push_back(e_kind[e]);
            eobs.insert(eobs.end(), &e_obs[3 * e], &e_obs[3 * e] + 3);
            eis.push_back(e_isig[e]);
        }
        osg_ba_graph g{};
        g.n_poses = (int32_t)kfs.size();
        g.pose = p_in.data();
        g.pose_fixed = fixed.data();
        g.n_points = (int32_t)mps.size();
        g.point = x_in.data();
        g.n_edges = (int32_t)edges.size();
        g.e_point = ep.data();
        g.e_pose = eo.data();
        g.e_kind = ek.data();
        g.e_cam = ec.data();
        g.e_obs = eobs.data();
        g.e_inv_sigma2 = eis.data();
        g.n_cams = (int32_t)cams.size();
        g.cams = cams.data();
        g.iterations = iters;
        g.e_robust = robust.data();
        g.huber_mono = (float)std::sqrt(5.99);   // const float thHuber2D = sqrt(5.99), :5338
        g.huber_stereo = (float)std::sqrt(7.815);
        p_out.resize(p_in.size());
        x_out.resize(x_in.size());
        bad.assign(edges.size(), 0);
        chi2.assign(edges.size(), 0.0);
        osg_ba_result r{};
        r.pose = p_out.data();
        r.point = x_out.data();
        r.edge_bad = bad.data();
        r.edge_chi2 = chi2.data();
        return call(ctx, "osg_bundle_adjustment", [&] {
            return osg_bundle_adjustment(ctx, &g, &r, reinterpret_cast<const volatile uint8_t *>(pbStopFlag));
        });
    };
    std::vector<size_t> all(ne);
    for (size_t e = 0; e < ne; e++) all[e] = e;
    std::vector<double> p1, x1, p2, x2, chi1, chi2;
    std::vector<uint8_t> bad1, bad2;
    if (pass(all, std::vector<uint8_t>(ne, 1), 5, pose, point, p1, x1, bad1, chi1) < 0) {  // :5448-5449
        out.aborted = true;  // nothing written back
        return out;
    }
    std::vector<uint8_t> skip(ne), bad(ne, 0);
    for (size_t e = 0; e < ne; e++) skip[e] = e_pair[e].second->isBad();
    const double *pf = p1.data(), *xf = x1.data();
    if (!(pbStopFlag && *pbStopFlag)) {  // bDoMore, :5451-5498
        std::vector<size_t> keep;
        std::vector<uint8_t> rob;
        for (size_t e = 0; e < ne; e++)
            if (skip[e] || !bad1[e]) {  // level 0; a bad MapPoint's edges keep their kernel
                keep.push_back(e);
                rob.push_back(skip[e]);
            }
        if (pass(keep, rob, 10, p1, x1, p2, x2, bad2, chi2) < 0) {
            out.aborted = true;
            return out;
        }
        for (size_t i = 0; i < keep.size(); i++) bad[keep[i]] = bad2[i];
        for (size_t e = 0; e < ne; e++)
            if (!skip[e] && bad1[e]) {  // level 1: the first pass's chi2, the final depth
                const double th = e_kind[e] == OSG_EDGE_STEREO ? 7.815 : 5.991;
                bad[e] = chi1[e] > th || !depth_positive_se3(&p2[7 * e_pose[e]], &x2[3 * e_point[e]]);
            }
        pf = p2.data();
        xf = x2.data();
    } else {
        bad = bad1;
    }
    for (int kind : {OSG_EDGE_MONO, OSG_EDGE_STEREO})  // :5506-5546, vToErase order
        for (size_t e = 0; e < ne; e++)
            if (e_kind[e] == kind && !skip[e] && bad[e]) out.to_erase.push_back(e_pair[e]);
    for (auto *k : vpAdjustKF) {  // :5592-5660
        const auto it = kf_index.find(k);
        if (k->isBad() || it == kf_index.end()) continue;
        out.poses.push_back({k, std::vector<double>(pf + 7 * it->second, pf + 7 * it->second + 7)});
    }
    for (auto *p : vpMPs) {  // :5663-5671
        if (p->isBad()) continue;
        const int j = mp_index[p];
        out.points.push_back({p, std::vector<double>(xf + 3 * j, xf + 3 * j + 3)});
    }
    return out;
}

// Applies a MergeLbaOutcome as ref:src/Optimizer.cc:5550-5671 does; the caller holds the map's
// mMutexMapUpdate.
template <class H, class KeyFrameT, class MapPointT>
void apply_merge_local_bundle_adjustment(const MergeLbaOutcome<KeyFrameT, MapPointT> &o)
{
    for (const auto &km : o.to_erase) {
        km.first->EraseMapPointMatch(km.second);
        km.second->EraseObservation(km.first);
    }
    for (const auto &kp : o.poses) H::set_pose(*kp.first, kp.second.data());
    for (const auto &mp : o.points) H::set_world_pos(mp.first, mp.second.data());
}

// ------------------------------------------------------------------------------ batched forms
// B independent problems gathered from the reference's objects, solved in one launch (the
// osg_*_batch entry points: one workgroup or frame slice per problem), and written back exactly as
// B single calls would.  For hosts that hold several frames at once: the frames of several
// sequences' Tracking threads (config C5 runs one sequence per thread, ref:src/System.cc:234-273),
// a replayed sequence, or the neighbours of a new keyframe.  Gathering runs on the calling thread;
// nmatches[b] / n_inliers[b] receive what the single call returns for problem b.  On an ABI error
// every problem gets the single call's nothing-found outcome (logged once per thread).
template <class H, class KeyFrameT, class FrameT, class MapPointT>
int search_by_bow_kf_f_batch(const std::vector<KeyFrameT *> &kfs, const std::vector<FrameT *> &frames,
                             std::vector<std::vector<MapPointT *>> &matches, float nnratio, bool checkOri,
                             int32_t *nmatches)
{
    osg_ctx *ctx = thread_ctx();
    const int B = (int)frames.size();
    std::deque<BowKfF<KeyFrameT, FrameT, MapPointT>> &g = gather_pool<BowKfF<KeyFrameT, FrameT, MapPointT>>(B);
    thread_local std::vector<osg_bow_side> sk, sf;
    thread_local std::vector<size_t> off;
    thread_local std::vector<int32_t> out;
    sk.resize(B);
    sf.resize(B);
    off.assign(B + 1, 0);
    for (int b = 0; b < B; b++) {
        g[b].assign(kfs[b], *frames[b]);
        sk[b] = g[b].sk;
        sf[b] = g[b].sf;
        off[b + 1] = off[b] + (size_t)frames[b]->N;
    }
    out.assign(off[B], -1);
    const int rc = B == 0 ? OSG_OK : call(ctx, "osg_search_by_bow_kf_f_batch", [&] {
        return osg_search_by_bow_kf_f_batch(ctx, sk.data(), sf.data(), B, nnratio, checkOri, out.data(), nmatches);
    });
    matches.resize(B);
    for (int b = 0; b < B; b++) {
        g[b].apply(out.data() + off[b], frames[b]->N, matches[b], rc >= 0);
        if (rc < 0) nmatches[b] = 0;
    }
    return rc < 0 ? 0 : B;
}

template <class H, class FrameT, class MutexT = NoMutex>
int pose_optimization_batch(const std::vector<FrameT *> &frames, int32_t *n_inliers, MutexT *gather_mutex = nullptr)
{
    osg_ctx *ctx = thread_ctx();
    const int B = (int)frames.size();
    std::deque<PoseGather<H, FrameT>> &g = gather_pool<PoseGather<H, FrameT>>(B);
    thread_local std::vector<osg_pose_problem> p;
    thread_local std::vector<osg_pose_result> r;
    p.resize(B);
    r.resize(B);
    for (int b = 0; b < B; b++) {
        g[b].assign(frames[b], gather_mutex);
        p[b] = g[b].p;
        r[b] = osg_pose_result{};
        r[b].outlier = g[b].outl.data();
    }
    const int rc = B == 0 ? OSG_OK : call(ctx, "osg_pose_optimization_batch",
                                          [&] { return osg_pose_optimization_batch(ctx, p.data(), B, r.data()); });
    for (int b = 0; b < B; b++) n_inliers[b] = rc < 0 ? 0 : g[b].apply(frames[b], r[b]);
    return rc < 0 ? 0 : B;
}

template <class H, class FrameT>
int search_by_projection_last_batch(const std::vector<FrameT *> &CFs, const std::vector<const FrameT *> &LFs, float th,
                                    bool bMono, bool checkOri, int32_t *nmatches)
{
    osg_ctx *ctx = thread_ctx();
    const int B = (int)CFs.size();
    std::deque<LastGather<H, FrameT>> &g = gather_pool<LastGather<H, FrameT>>(B);
    thread_local std::vector<osg_frame> f;
    thread_local std::vector<osg_last_queries> q;
    thread_local std::vector<size_t> off;
    thread_local std::vector<int32_t> mp;
    thread_local std::vector<uint8_t> taken;
    f.resize(B);
    q.resize(B);
    off.assign(B + 1, 0);
    for (int b = 0; b < B; b++) {
        g[b].assign(*CFs[b], *LFs[b]);
        f[b] = g[b].fv.v;
        q[b] = g[b].q;
        off[b + 1] = off[b] + (size_t)CFs[b]->N;
    }
    mp.resize(off[B]);
    taken.resize(off[B]);
    for (int b = 0; b < B; b++) {
        std::copy(g[b].slots.mp.begin(), g[b].slots.mp.end(), mp.begin() + off[b]);
        std::copy(g[b].slots.taken.begin(), g[b].slots.taken.end(), taken.begin() + off[b]);
    }
    const int rc = B == 0 ? OSG_OK : call(ctx, "osg_search_by_projection_last_batch", [&] {
        return osg_search_by_projection_last_batch(ctx, f.data(), q.data(), B, th, bMono, checkOri, mp.data(),
                                                   taken.data(), nmatches);
    });
    for (int b = 0; b < B; b++) {
        if (rc < 0) {
            nmatches[b] = 0;
            continue;
        }
        std::copy(mp.begin() + off[b], mp.begin() + off[b + 1], g[b].slots.mp.begin());
        g[b].slots.apply(CFs[b]->mvpMapPoints, g[b].queries, LFs[b]->N);
    }
    return rc < 0 ? 0 : B;
}

template <class H, class FrameT, class MapPointT>
int search_by_projection_mps_batch(const std::vector<FrameT *> &Fs, const std::vector<const std::vector<MapPointT *> *> &mps,
                                   float th, bool bFarPoints, float thFarPoints, float nnratio, int32_t *nmatches)
{
    osg_ctx *ctx = thread_ctx();
    const int B = (int)Fs.size();
    std::deque<MpsGather<FrameT, MapPointT>> &g = gather_pool<MpsGather<FrameT, MapPointT>>(B);
    thread_local std::vector<osg_frame> f;
    thread_local std::vector<osg_mp_queries> q;
    thread_local std::vector<size_t> off;
    thread_local std::vector<int32_t> mp;
    thread_local std::vector<uint8_t> taken;
    f.resize(B);
    q.resize(B);
    off.assign(B + 1, 0);
    for (int b = 0; b < B; b++) {
        g[b].assign(*Fs[b], *mps[b]);
        f[b] = g[b].fv.v;
        q[b] = g[b].q;
        off[b + 1] = off[b] + (size_t)Fs[b]->N;
    }
    mp.resize(off[B]);
    taken.resize(off[B]);
    for (int b = 0; b < B; b++) {
        std::copy(g[b].slots.mp.begin(), g[b].slots.mp.end(), mp.begin() + off[b]);
        std::copy(g[b].slots.taken.begin(), g[b].slots.taken.end(), taken.begin() + off[b]);
    }
    const int rc = B == 0 ? OSG_OK : call(ctx, "osg_search_by_projection_mps_batch", [&] {
        return osg_search_by_projection_mps_batch(ctx, f.data(), q.data(), B, nnratio, th, bFarPoints, thFarPoints,
                                                  mp.data(), taken.data(), nmatches);
    });
    for (int b = 0; b < B; b++) {
        if (rc < 0) {
            nmatches[b] = 0;
            continue;
        }
        std::copy(mp.begin() + off[b], mp.begin() + off[b + 1], g[b].slots.mp.begin());
        g[b].slots.apply(Fs[b]->mvpMapPoints, *mps[b], (int)mps[b]->size());
    }
    return rc < 0 ? 0 : B;
}

template <class FrameT>
int compute_stereo_matches_batch(const std::vector<FrameT *> &frames, int32_t *nmatches)
{
    osg_ctx *ctx = thread_ctx();
    const int B = (int)frames.size();
    std::deque<StereoGather<FrameT>> &g = gather_pool<StereoGather<FrameT>>(B);
    thread_local std::vector<osg_stereo_frame> s;
    thread_local std::vector<size_t> off;
    thread_local std::vector<float> ur, depth;
    s.resize(B);
    off.assign(B + 1, 0);
    for (int b = 0; b < B; b++) {
        g[b].assign(*frames[b]);
        s[b] = g[b].s;
        off[b + 1] = off[b] + (size_t)frames[b]->N;
    }
    ur.assign(off[B], -1.0f);
    depth.assign(off[B], -1.0f);
    const int rc = B == 0 ? OSG_OK : call(ctx, "osg_compute_stereo_matches_batch", [&] {
        return osg_compute_stereo_matches_batch(ctx, s.data(), B, ur.data(), depth.data(), nmatches);
    });
    for (int b = 0; b < B; b++) {
        FrameT &F = *frames[b];
        F.mvuRight.assign(ur.begin() + off[b], ur.begin() + off[b + 1]);  // :1134-1135 when rc < 0 (all -1)
        F.mvDepth.assign(depth.begin() + off[b], depth.begin() + off[b + 1]);
        if (rc < 0) {
            F.mvuRight.assign(F.N, -1.0f);
            F.mvDepth.assign(F.N, -1.0f);
            nmatches[b] = 0;
        }
    }
    return rc < 0 ? 0 : B;
}

// ------------------------------------------------------ §8(f) rank 1: ComputeBoW (DBoW2 transform)
// Frame::ComputeBoW (ref:src/Frame.cc:995-1010) and KeyFrame::ComputeBoW (ref:src/KeyFrame.cc:102-116):
// when mBowVec is empty, transform(rows of mDescriptors, mBowVec, mFeatVec, levelsup = 4)
// (ref:Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1192) runs on the device.  `voc` is the
// vocabulary uploaded once with osg_vocabulary_load_text (next to System's ORBVocabulary load).
// KeyFrame's extra `|| mFeatVec.empty()` changes nothing: transform leaves both maps filled or both
// empty.  Both maps come back in key order, so every insert is an end-hint insert.  On an ABI error
// both maps stay empty, as for a frame without descriptors.
struct BowSet {
    OSG_PINNED_STRUCT(BowSet);
    std::vector<int32_t> word, node_start, feat;
    std::vector<double> value;
    std::vector<uint32_t> node_id;
    osg_bow_out o{};
    // (capacities of at least 1: a frame without descriptors still passes non-null arrays)
    explicit BowSet(int n)
        : word(std::max(n, 1)), node_start(n + 1), feat(std::max(n, 1)), value(std::max(n, 1)), node_id(std::max(n, 1))
    {
        o.word = word.data();
        o.value = value.data();
        o.node_id = node_id.data();
        o.node_start = node_start.data();
        o.feat = feat.data();
    }
    template <class T>
    void apply(T &F, bool ok) const
    {
        F.mBowVec.clear();
        F.mFeatVec.clear();
        if (!ok) return;
        for (int j = 0; j < o.n_words; j++) F.mBowVec.emplace_hint(F.mBowVec.end(), (unsigned)word[j], value[j]);
        for (int j = 0; j < o.n_nodes; j++)
            F.mFeatVec.emplace_hint(F.mFeatVec.end(), node_id[j],
                                    std::vector<unsigned int>(feat.begin() + node_start[j], feat.begin() + node_start[j + 1]));
    }
};

template <class T>
void compute_bow(T &F, const osg_vocabulary *voc)
{
    if (!F.mBowVec.empty()) return;
    osg_ctx *ctx = thread_ctx();
    const int n = F.mDescriptors.rows;
    std::vector<uint8_t> desc;
    copy_desc_rows(F.mDescriptors, n, desc);
    BowSet s(n);
    const int rc = call(ctx, "osg_vocabulary_transform",
                        [&] { return osg_vocabulary_transform(ctx, voc, desc.data(), n, 4, &s.o); });
    s.apply(F, rc >= 0);
}

// B frames or keyframes in one launch; those whose mBowVec is already filled are skipped, as the
// single call skips them.
template <class T>
void compute_bow_batch(const std::vector<T *> &frames, const osg_vocabulary *voc)
{
    osg_ctx *ctx = thread_ctx();
    std::vector<T *> todo;
    std::vector<int32_t> n;
    size_t rows = 0;
    for (T *F : frames)
        if (F->mBowVec.empty()) {
            todo.push_back(F);
            n.push_back(F->mDescriptors.rows);
            rows += (size_t)n.back();
        }
    const int B = (int)todo.size();
    if (B == 0) return;
    std::vector<uint8_t> desc(32 * rows);
    std::deque<BowSet> sets;
    std::vector<osg_bow_out> out(B);
    size_t r0 = 0;
    for (int b = 0; b < B; b++) {
        const auto &M = todo[b]->mDescriptors;
        for (int i = 0; i < n[b]; i++) std::memcpy(&desc[32 * (r0 + i)], M.template ptr<unsigned char>(i), 32);
        r0 += (size_t)n[b];
        sets.emplace_back(n[b]);
        out[b] = sets.back().o;
    }
    const int rc = call(ctx, "osg_vocabulary_transform_batch", [&] {
        return osg_vocabulary_transform_batch(ctx, voc, desc.data(), n.data(), B, 4, out.data());
    });
    for (int b = 0; b < B; b++) {
        sets[b].o.n_words = out[b].n_words;
        sets[b].o.n_nodes = out[b].n_nodes;
        sets[b].apply(*todo[b], rc >= 0);
    }
}

}  // namespace osg_orbslam3
#endif
