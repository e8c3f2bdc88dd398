// ORBmatcher_osg.cc — drop-in bodies for the ORBmatcher operators on the MI355X path, for an
// ORB-SLAM3 tree built with -DORB_SLAM3_OSG.  The reference's
// src/ORBmatcher.cc keeps every other member; the bodies below replace the six hot-path ones,
// the two Fuse overloads, SearchForTriangulation, the two Sim3
// SearchByProjection overloads, SearchBySim3 and SearchForInitialization
// under #ifdef ORB_SLAM3_OSG (signatures: ref:include/ORBmatcher.h:36-66).
#include "ORBmatcher.h"
#include "osg_hooks_orbslam3.h"

namespace ORB_SLAM3 {

using H = OsgHooks;

int ORBmatcher::DescriptorDistance(const cv::Mat &a, const cv::Mat &b)
{  // ref:src/ORBmatcher.cc:2388-2408 (host scalar; batched distances run on the GPU inside the searches)
    return osg_orbslam3::descriptor_distance(a, b);
}

int ORBmatcher::SearchByProjection(Frame &F, const std::vector<MapPoint *> &vpMapPoints, const float th,
                                   const bool bFarPoints, const float thFarPoints)
{  // ref:src/ORBmatcher.cc:44-242
    return osg_orbslam3::search_by_projection_mps<H>(F, vpMapPoints, th, bFarPoints, thFarPoints, mfNNratio);
}

int ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, const float th, const bool bMono)
{  // ref:src/ORBmatcher.cc:1957-2191
    return osg_orbslam3::search_by_projection_last<H>(CurrentFrame, LastFrame, th, bMono, mbCheckOrientation);
}

int ORBmatcher::SearchByProjection(Frame &CurrentFrame, KeyFrame *pKF, const std::set<MapPoint *> &sAlreadyFound,
                                   const float th, const int ORBdist)
{  // ref:src/ORBmatcher.cc:2203-2330
    return osg_orbslam3::search_by_projection_kf<H>(CurrentFrame, pKF, sAlreadyFound, th, ORBdist, mbCheckOrientation);
}

int ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, std::vector<MapPoint *> &vpMapPointMatches)
{  // ref:src/ORBmatcher.cc:262-496
    return osg_orbslam3::search_by_bow_kf_f<H>(pKF, F, vpMapPointMatches, mfNNratio, mbCheckOrientation);
}

int ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, std::vector<MapPoint *> &vpMatches12)
{  // ref:src/ORBmatcher.cc:890-1043
    return osg_orbslam3::search_by_bow_kf_kf<H>(pKF1, pKF2, vpMatches12, mfNNratio, mbCheckOrientation);
}

int ORBmatcher::Fuse(KeyFrame *pKF, const std::vector<MapPoint *> &vpMapPoints, const float th, const bool bRight)
{  // ref:src/ORBmatcher.cc:1330-1541
    return osg_orbslam3::fuse<H>(pKF, vpMapPoints, th, bRight);
}

int ORBmatcher::Fuse(KeyFrame *pKF, Sophus::Sim3f &Scw, const std::vector<MapPoint *> &vpPoints, float th,
                     std::vector<MapPoint *> &vpReplacePoint)
{  // ref:src/ORBmatcher.cc:1553-1694
    return osg_orbslam3::fuse_sim3<H>(pKF, Scw, vpPoints, th, vpReplacePoint);
}

int ORBmatcher::SearchForTriangulation(KeyFrame *pKF1, KeyFrame *pKF2, std::vector<std::pair<size_t, size_t>> &vMatchedPairs,
                                       const bool bOnlyStereo, const bool bCoarse)
{  // ref:src/ORBmatcher.cc:1045-1328
    return osg_orbslam3::search_for_triangulation<H>(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse, mbCheckOrientation);
}

int ORBmatcher::SearchByProjection(KeyFrame *pKF, Sophus::Sim3f &Scw, const std::vector<MapPoint *> &vpPoints,
                                   std::vector<MapPoint *> &vpMatched, int th, float ratioHamming)
{  // ref:src/ORBmatcher.cc:498-621
    return osg_orbslam3::search_by_projection_sim3<H, KeyFrame>(pKF, Scw, vpPoints, nullptr, vpMatched, nullptr, th,
                                                               ratioHamming);
}

int ORBmatcher::SearchByProjection(KeyFrame *pKF, Sophus::Sim3<float> &Scw, const std::vector<MapPoint *> &vpPoints,
                                   const std::vector<KeyFrame *> &vpPointsKFs, std::vector<MapPoint *> &vpMatched,
                                   std::vector<KeyFrame *> &vpMatchedKF, int th, float ratioHamming)
{  // ref:src/ORBmatcher.cc:623-733
    return osg_orbslam3::search_by_projection_sim3<H, KeyFrame>(pKF, Scw, vpPoints, &vpPointsKFs, vpMatched,
                                                               &vpMatchedKF, th, ratioHamming);
}

int ORBmatcher::SearchBySim3(KeyFrame *pKF1, KeyFrame *pKF2, std::vector<MapPoint *> &vpMatches12,
                             const Sophus::Sim3f &S12, const float th)
{  // ref:src/ORBmatcher.cc:1696-1939
    return osg_orbslam3::search_by_sim3<H, KeyFrame>(pKF1, pKF2, vpMatches12, S12, th);
}

int ORBmatcher::SearchForInitialization(Frame &F1, Frame &F2, std::vector<cv::Point2f> &vbPrevMatched,
                                        std::vector<int> &vnMatches12, int windowSize)
{  // ref:src/ORBmatcher.cc:735-878
    return osg_orbslam3::search_for_initialization<H>(F1, F2, vbPrevMatched, vnMatches12, windowSize, mfNNratio,
                                                      mbCheckOrientation);
}

}  // namespace ORB_SLAM3
