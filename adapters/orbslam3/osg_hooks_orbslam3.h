// osg_hooks_orbslam3.h — the hook policy of osg_orbslam3.h written with ORB-SLAM3's own Sophus /
// Eigen / GeometricCamera calls, so every float the reference computes before its matching and
// optimisation loops is computed by the same code.  Compiled only inside an ORB-SLAM3 tree.
#ifndef OSG_HOOKS_ORBSLAM3_H
#define OSG_HOOKS_ORBSLAM3_H

#include "Frame.h"
#include "KeyFrame.h"
#include "MapPoint.h"
#include "osg_orbslam3.h"

namespace ORB_SLAM3 {

struct OsgHooks {
    template <class T>
    static void pose(T &o, double q[7])
    {
        const Sophus::SE3<float> Tcw = const_cast<T &>(o).GetPose();
        const Eigen::Quaterniond qd = Tcw.unit_quaternion().cast<double>();
        const Eigen::Vector3d t = Tcw.translation().cast<double>();
        q[0] = qd.x(); q[1] = qd.y(); q[2] = qd.z(); q[3] = qd.w();
        q[4] = t.x(); q[5] = t.y(); q[6] = t.z();
    }
    template <class T>
    static void set_pose(T &o, const double q[7])
    {  // ref:src/Optimizer.cc:413-416 / 2187-2195: SE3Quat estimate -> SE3f
        const Eigen::Quaternionf qf(Eigen::Quaterniond(q[3], q[0], q[1], q[2]).cast<float>());
        o.SetPose(Sophus::SE3<float>(qf, Eigen::Vector3d(q[4], q[5], q[6]).cast<float>()));
    }
    static void world_pos(MapPoint *p, double x[3])
    {
        const Eigen::Vector3d X = p->GetWorldPos().cast<double>();
        x[0] = X.x(); x[1] = X.y(); x[2] = X.z();
    }
    static void set_world_pos(MapPoint *p, const double x[3])
    {  // ref:src/Optimizer.cc:2197-2203
        p->SetWorldPos(Eigen::Vector3d(x[0], x[1], x[2]).cast<float>());
        p->UpdateNormalAndDepth();
    }
    static void set_gba_pose(KeyFrame &k, const double q[7], unsigned long nLoopKF)
    {  // ref:src/Optimizer.cc:3144-3145: SE3d(SE3quat.rotation(), SE3quat.translation()).cast<float>()
        const Eigen::Quaterniond qd(q[3], q[0], q[1], q[2]);
        k.mTcwGBA = Sophus::SE3d(qd, Eigen::Vector3d(q[4], q[5], q[6])).cast<float>();
        k.mnBAGlobalForKF = nLoopKF;
    }
    static void set_gba_pos(MapPoint *p, const double x[3], unsigned long nLoopKF)
    {  // ref:src/Optimizer.cc:3233-3234
        p->mPosGBA = Eigen::Vector3d(x[0], x[1], x[2]).cast<float>();
        p->mnBAGlobalForKF = nLoopKF;
    }
    template <class T>
    static void camera(const T &o, bool right, osg_camera &c)
    {
        std::memset(&c, 0, sizeof c);
        GeometricCamera *cam = right ? o.mpCamera2 : o.mpCamera;
        c.type = (cam->GetType() == GeometricCamera::CAM_FISHEYE) ? OSG_CAM_KB8 : OSG_CAM_PINHOLE;
        for (size_t i = 0; i < cam->size() && i < 8; i++) c.p[i] = cam->getParameter((int)i);
        c.fx = o.fx; c.fy = o.fy; c.cx = o.cx; c.cy = o.cy; c.bf = o.mbf;
        c.trl[3] = 1.0;
        if (right) {
            const Sophus::SE3f Trl = const_cast<T &>(o).GetRelativePoseTrl();
            const Eigen::Quaterniond qd = Trl.unit_quaternion().cast<double>();
            const Eigen::Vector3d t = Trl.translation().cast<double>();
            c.trl[0] = qd.x(); c.trl[1] = qd.y(); c.trl[2] = qd.z(); c.trl[3] = qd.w();
            c.trl[4] = t.x(); c.trl[5] = t.y(); c.trl[6] = t.z();
        }
    }
    // ref:src/ORBmatcher.cc:1052-1083 and Pinhole.cpp:194-197: the epipole and F12 = K1^-T [t12]x R12 K2^-1
    // for each camera pair (ll, lr, rl, rr), evaluated with the reference's own Sophus / Eigen expressions
    static void triang_geom(KeyFrame *pKF1, KeyFrame *pKF2, osg_triang_geom &g)
    {
        std::memset(&g, 0, sizeof g);
        const Sophus::SE3f T1w = pKF1->GetPose(), T2w = pKF2->GetPose(), Tw2 = pKF2->GetPoseInverse();
        const Eigen::Vector3f Cw = pKF1->GetCameraCenter();
        const Eigen::Vector3f C2 = T2w * Cw;
        const Eigen::Vector2f ep = pKF2->mpCamera->project(C2);
        g.ep_x = ep(0);
        g.ep_y = ep(1);
        Sophus::SE3f T[4];
        int nk = 1;
        T[0] = T1w * Tw2;
        if (pKF1->mpCamera2 || pKF2->mpCamera2) {
            const Sophus::SE3f Tr1w = pKF1->GetRightPose(), Twr2 = pKF2->GetRightPoseInverse();
            T[1] = T1w * Twr2;
            T[2] = Tr1w * Tw2;
            T[3] = Tr1w * Twr2;
            nk = 4;
        }
        GeometricCamera *c1[2] = {pKF1->mpCamera, pKF1->mpCamera2}, *c2[2] = {pKF2->mpCamera, pKF2->mpCamera2};
        g.pinhole = 1;
        for (int k = 0; k < nk; k++)
            if (c1[k >> 1]->GetType() != GeometricCamera::CAM_PINHOLE ||
                c2[k & 1]->GetType() != GeometricCamera::CAM_PINHOLE)
                g.pinhole = 0;
        if (!g.pinhole) {  // KannalaBrandt8: R12 / t12 per pair and the four cameras' parameters
            for (int k = 0; k < nk; k++) {
                const Eigen::Matrix3f R12 = T[k].rotationMatrix();
                const Eigen::Vector3f t12 = T[k].translation();
                for (int r = 0; r < 3; r++) {
                    for (int c = 0; c < 3; c++) g.R12[k][3 * r + c] = R12(r, c);
                    g.t12[k][r] = t12(r);
                }
            }
            GeometricCamera *cams[4] = {c1[0], c1[1], c2[0], c2[1]};
            for (int i = 0; i < 4; i++)
                if (cams[i])
                    for (int j = 0; j < 8 && j < (int)cams[i]->size(); j++) g.kb[i][j] = cams[i]->getParameter(j);
            return;
        }
        for (int k = 0; k < nk; k++) {
            const Eigen::Matrix3f R12 = T[k].rotationMatrix();
            const Eigen::Vector3f t12 = T[k].translation();
            const Eigen::Matrix3f t12x = Sophus::SO3f::hat(t12);
            const Eigen::Matrix3f K1 = c1[k >> 1]->toK_();
            const Eigen::Matrix3f K2 = c2[k & 1]->toK_();
            const Eigen::Matrix3f F12 = K1.transpose().inverse() * t12x * R12 * K2.inverse();
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) g.F12[k][3 * r + c] = F12(r, c);
        }
    }
    // ref:src/MapPoint.cc:530-534: mDescriptor = vDescriptors[BestIdx].clone() under mMutexFeatures
    // (OsgHooks is a friend of MapPoint under ORB_SLAM3_OSG)
    static void set_descriptor(MapPoint *pMP, const uint8_t *row)
    {
        std::unique_lock<std::mutex> lock(pMP->mMutexFeatures);
        pMP->mDescriptor = cv::Mat(1, 32, CV_8UC1, const_cast<uint8_t *>(row)).clone();
    }
    // ref:src/ORBmatcher.cc:1993-2009; the invz < 0 and image-bounds tests stay in the kernel
    static bool project_last(const Frame &CF, MapPoint *pMP, float &u, float &v, float &invz)
    {
        const Sophus::SE3f Tcw = const_cast<Frame &>(CF).GetPose();
        const Eigen::Vector3f x3Dw = pMP->GetWorldPos();
        const Eigen::Vector3f x3Dc = Tcw * x3Dw;
        invz = 1.0 / x3Dc(2);
        const Eigen::Vector2f uv = CF.mpCamera->project(x3Dc);
        u = uv(0);
        v = uv(1);
        return true;
    }
    // ref:src/ORBmatcher.cc:2096-2097: right-camera projection of a two-camera current frame (the
    // reference projects Trl * x3Dc with mpCamera)
    static void project_last_right(const Frame &CF, MapPoint *pMP, float &u, float &v)
    {
        Frame &F = const_cast<Frame &>(CF);
        const Eigen::Vector3f x3Dc = F.GetPose() * pMP->GetWorldPos();
        const Eigen::Vector3f x3Dr = F.GetRelativePoseTrl() * x3Dc;
        const Eigen::Vector2f uv = CF.mpCamera->project(x3Dr);
        u = uv(0);
        v = uv(1);
    }
    // ref:src/ORBmatcher.cc:1972-1980
    static float tlc_z(const Frame &CF, const Frame &LF)
    {
        const Sophus::SE3f Tcw = const_cast<Frame &>(CF).GetPose();
        const Eigen::Vector3f twc = Tcw.inverse().translation();
        const Sophus::SE3f Tlw = const_cast<Frame &>(LF).GetPose();
        const Eigen::Vector3f tlc = Tlw * twc;
        return tlc(2);
    }
    // ref:src/ORBmatcher.cc:2238-2262: projection, image bounds, scale-invariance range, PredictScale
    static bool kf_query(const Frame &CF, MapPoint *pMP, float &u, float &v, int &level)
    {
        Frame &F = const_cast<Frame &>(CF);
        const Sophus::SE3f Tcw = F.GetPose();
        const Eigen::Vector3f Ow = Tcw.inverse().translation();
        const Eigen::Vector3f x3Dw = pMP->GetWorldPos();
        const Eigen::Vector3f x3Dc = Tcw * x3Dw;
        const Eigen::Vector2f uv = CF.mpCamera->project(x3Dc);
        if (uv(0) < CF.mnMinX || uv(0) > CF.mnMaxX) return false;
        if (uv(1) < CF.mnMinY || uv(1) > CF.mnMaxY) return false;
        const float dist3D = (x3Dw - Ow).norm();
        if (dist3D < pMP->GetMinDistanceInvariance() || dist3D > pMP->GetMaxDistanceInvariance()) return false;
        level = pMP->PredictScale(dist3D, &F);
        u = uv(0);
        v = uv(1);
        return true;
    }
    // ref:src/ORBmatcher.cc:1336-1347, 1385-1433 (Fuse): pose / centre / camera of the chosen side,
    // depth, projection, IsInImage, ur, scale-invariance range, viewing angle, PredictScale
    static bool fuse_query(KeyFrame *pKF, MapPoint *pMP, bool bRight, float &u, float &v, float &ur, int &level)
    {
        const Sophus::SE3f Tcw = bRight ? pKF->GetRightPose() : pKF->GetPose();
        const Eigen::Vector3f Ow = bRight ? pKF->GetRightCameraCenter() : pKF->GetCameraCenter();
        GeometricCamera *pCamera = bRight ? pKF->mpCamera2 : pKF->mpCamera;
        const float &bf = pKF->mbf;
        const Eigen::Vector3f p3Dw = pMP->GetWorldPos();
        const Eigen::Vector3f p3Dc = Tcw * p3Dw;
        if (p3Dc(2) < 0.0f) return false;
        const float invz = 1 / p3Dc(2);
        const Eigen::Vector2f uv = pCamera->project(p3Dc);
        if (!pKF->IsInImage(uv(0), uv(1))) return false;
        ur = uv(0) - bf * invz;
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        const Eigen::Vector3f PO = p3Dw - Ow;
        const float dist3D = PO.norm();
        if (dist3D < minDistance || dist3D > maxDistance) return false;
        const Eigen::Vector3f Pn = pMP->GetNormal();
        if (PO.dot(Pn) < 0.5 * dist3D) return false;
        level = pMP->PredictScale(dist3D, pKF);
        u = uv(0);
        v = uv(1);
        return true;
    }
    // ref:src/ORBmatcher.cc:1560-1562, 1587-1622 (Fuse with Sim3): the same tests with Tcw from Scw
    // ref:src/ORBmatcher.cc:1589-1622 (Fuse, Sim3) and :530-572 / :649-688 (SearchByProjection, Sim3):
    // depth, image, distance and viewing-angle tests, the projection and PredictScale.  The second
    // SearchByProjection overload projects with its own pinhole formula (invz = 1 / z; u = fx * x * invz
    // + cx, :661-667) instead of mpCamera->project — different float rounding, so it is kept apart.
    // ref:src/ORBmatcher.cc:1747-1772 (dir12: KF1's MapPoint into KF2 by S21 * T1w) and :1823-1850
    // (KF2's into KF1 by S12 * T2w); both directions use pKF1's intrinsics, as the reference does
    static int index_in_keyframe(MapPoint *pMP, KeyFrame *pKF) { return std::get<0>(pMP->GetIndexInKeyFrame(pKF)); }
    static bool sim3_pair_query(KeyFrame *pKF1, KeyFrame *pKF2, MapPoint *pMP, const Sophus::Sim3f &S12, bool dir12,
                                float &u, float &v, int &level)
    {
        KeyFrame *from = dir12 ? pKF1 : pKF2, *to = dir12 ? pKF2 : pKF1;
        const Sophus::Sim3f S = dir12 ? S12.inverse() : S12;
        const Eigen::Vector3f p3Dw = pMP->GetWorldPos();
        const Eigen::Vector3f pc = S * (from->GetPose() * p3Dw);
        if (pc(2) < 0.0) return false;
        const float invz = 1.0 / pc(2);
        const float x = pc(0) * invz;
        const float y = pc(1) * invz;
        u = pKF1->fx * x + pKF1->cx;
        v = pKF1->fy * y + pKF1->cy;
        if (!to->IsInImage(u, v)) return false;
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        const float dist3D = pc.norm();
        if (dist3D < minDistance || dist3D > maxDistance) return false;
        level = pMP->PredictScale(dist3D, to);
        return true;
    }
    static bool sim3_query(KeyFrame *pKF, const Sophus::Sim3f &Scw, MapPoint *pMP, bool pinhole_formula, float &u,
                           float &v, int &level)
    {
        const Sophus::SE3f Tcw = Sophus::SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale());
        const Eigen::Vector3f Ow = Tcw.inverse().translation();
        const Eigen::Vector3f p3Dw = pMP->GetWorldPos();
        const Eigen::Vector3f p3Dc = Tcw * p3Dw;
        if (p3Dc(2) < 0.0f) return false;
        if (pinhole_formula) {
            const float invz = 1 / p3Dc(2);
            const float x = p3Dc(0) * invz;
            const float y = p3Dc(1) * invz;
            u = pKF->fx * x + pKF->cx;
            v = pKF->fy * y + pKF->cy;
        } else {
            const Eigen::Vector2f uv = pKF->mpCamera->project(p3Dc);
            u = uv(0);
            v = uv(1);
        }
        if (!pKF->IsInImage(u, v)) return false;
        const float maxDistance = pMP->GetMaxDistanceInvariance();
        const float minDistance = pMP->GetMinDistanceInvariance();
        const Eigen::Vector3f PO = p3Dw - Ow;
        const float dist3D = PO.norm();
        if (dist3D < minDistance || dist3D > maxDistance) return false;
        const Eigen::Vector3f Pn = pMP->GetNormal();
        if (PO.dot(Pn) < 0.5 * dist3D) return false;
        level = pMP->PredictScale(dist3D, pKF);
        return true;
    }
    static bool fuse_sim3_query(KeyFrame *pKF, const Sophus::Sim3f &Scw, MapPoint *pMP, float &u, float &v,
                                int &level)
    {
        return sim3_query(pKF, Scw, pMP, false, u, v, level);
    }
};

}  // namespace ORB_SLAM3
#endif
