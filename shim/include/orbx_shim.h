// orbx_shim.h -- the shim-wide device: the reference's constructors take no device, so
// ORBextractor, ORBmatcher, ORBVocabulary, MapPoint::ComputeDistinctiveDescriptors and
// Frame::ComputeImageBounds / UndistortKeyPoints, PnPsolver and Optimizer's graph forms run on device
// gOrbxDevice (default 0; set it before constructing the objects).
#pragma once

namespace ORB_SLAM2 {
extern int gOrbxDevice;
}  // namespace ORB_SLAM2
