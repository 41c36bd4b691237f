// orbx_shim.h -- shim-wide settings for the members that have no device of their own
// (MapPoint::ComputeDistinctiveDescriptors, Frame::ComputeImageBounds / UndistortKeyPoints):
// they run on device gOrbxDevice (default 0).  ORBmatcher, Optimizer, PnPsolver and
// ORBVocabulary keep their own device settings.
#pragma once

namespace ORB_SLAM2 {
extern int gOrbxDevice;
}  // namespace ORB_SLAM2
