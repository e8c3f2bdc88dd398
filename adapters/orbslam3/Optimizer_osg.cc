// Optimizer_osg.cc — drop-in bodies for Optimizer::PoseOptimization, the g2o part of
// Optimizer::LocalBundleAdjustment (both overloads) and Optimizer::BundleAdjustment (global BA) on the
// MI355X path (ORB-SLAM3 tree built with -DORB_SLAM3_OSG;
// see INTEGRATION.md).  Signatures: ref:include/Optimizer.h:54-90.
#include "Optimizer.h"
#include "osg_hooks_orbslam3.h"

namespace ORB_SLAM3 {

int Optimizer::PoseOptimization(Frame *pFrame)
{  // ref:src/Optimizer.cc:71-420; MapPoint::mGlobalMutex is held only while the edges are gathered
   // (:128-286), released before the GPU solve and the write-back
    return osg_orbslam3::pose_optimization<OsgHooks>(pFrame, &MapPoint::mGlobalMutex);
}

// The local window (ref:src/Optimizer.cc:1762-1873) is the reference's code unchanged; it ends with
// lLocalKeyFrames, lLocalMapPoints, lFixedCameras and the no-fixed-KeyFrame early return.  Call
// this instead of the g2o graph build + optimize + classification (ref:src/Optimizer.cc:1877-2203).
void OsgLocalBundleAdjustmentTail(KeyFrame *pKF, bool *pbStopFlag, Map *pMap,
                                  std::list<KeyFrame *> &lLocalKeyFrames, std::list<KeyFrame *> &lFixedCameras,
                                  std::list<MapPoint *> &lLocalMapPoints, int &num_fixedKF, int &num_OptKF,
                                  int &num_MPs, int &num_edges)
{
    Map *pCurrentMap = pKF->GetMap();
    auto out = osg_orbslam3::local_bundle_adjustment<OsgHooks>(lLocalKeyFrames, lFixedCameras, lLocalMapPoints,
                                                               pCurrentMap, pMap->GetInitKFid(), pbStopFlag,
                                                               pMap->IsInertial());
    num_fixedKF = out.num_fixedKF;
    num_OptKF = out.num_OptKF;
    num_MPs = out.num_MPs;
    num_edges = out.num_edges;
    if (out.aborted && out.poses.empty()) return;  // stop flag before optimize (ref:src/Optimizer.cc:2112-2114)
    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);  // ref:src/Optimizer.cc:2171
    osg_orbslam3::apply_local_bundle_adjustment<OsgHooks>(out);
    pMap->IncreaseChangeIndex();
}

void Optimizer::BundleAdjustment(const std::vector<KeyFrame *> &vpKFs, const std::vector<MapPoint *> &vpMP,
                                 int nIterations, bool *pbStopFlag, const unsigned long nLoopKF, const bool bRobust)
{  // ref:src/Optimizer.cc:2850-3237 (GlobalBundleAdjustemnt, :2831-2839, passes the whole map)
    Map *pMap = vpKFs[0]->GetMap();
    auto out = osg_orbslam3::bundle_adjustment<OsgHooks>(vpKFs, vpMP, pMap->GetInitKFid(), nIterations, pbStopFlag,
                                                         bRobust);
    osg_orbslam3::apply_bundle_adjustment<OsgHooks>(out, nLoopKF, nLoopKF == pMap->GetOriginKF()->mnId);
}

void Optimizer::LocalBundleAdjustment(KeyFrame *pMainKF, std::vector<KeyFrame *> vpAdjustKF,
                                      std::vector<KeyFrame *> vpFixedKF, bool *pbStopFlag)
{  // ref:src/Optimizer.cc:5211-5672 (LoopClosing's map merge)
    auto out = osg_orbslam3::merge_local_bundle_adjustment<OsgHooks, KeyFrame, MapPoint>(pMainKF, vpAdjustKF, vpFixedKF,
                                                                                        pbStopFlag);
    if (out.aborted) return;  // :5444-5446
    std::unique_lock<std::mutex> lock(pMainKF->GetMap()->mMutexMapUpdate);  // :5551
    osg_orbslam3::apply_merge_local_bundle_adjustment<OsgHooks>(out);
}

}  // namespace ORB_SLAM3
