// Frame_osg.cc — drop-in bodies of Frame::ComputeStereoMatches and ComputeStereoFishEyeMatches on the MI355X path, for an ORB-SLAM3
// tree built with -DORB_SLAM3_OSG.  The reference's src/Frame.cc keeps every
// other member; its ComputeStereoMatches (ref:src/Frame.cc:1117-1373) goes under #ifndef
// ORB_SLAM3_OSG and this body replaces it.  The stereo Frame constructor calls it unchanged
// (ref:src/Frame.cc:165).
#include "Frame.h"
#include "ORBextractor.h"
#include "osg_hooks_orbslam3.h"

namespace ORB_SLAM3 {

void Frame::ComputeStereoMatches()
{  // mvuRight / mvDepth for every left keypoint (-1 = none)
    osg_orbslam3::compute_stereo_matches(*this);
}

void Frame::ComputeStereoFishEyeMatches()
{  // ref:src/Frame.cc:1546-1603 (the KannalaBrandt8 two-camera constructor, :1523)
    osg_orbslam3::compute_stereo_fisheye_matches(*this);
}

}  // namespace ORB_SLAM3
