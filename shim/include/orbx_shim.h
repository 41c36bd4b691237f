// orbx_shim.h -- the shim-wide device: the reference's constructors take no device, so
// ORBextractor, ORBmatcher, ORBVocabulary, MapPoint::ComputeDistinctiveDescriptors and
// Frame::ComputeImageBounds / UndistortKeyPoints, PnPsolver and Optimizer's graph forms run on device
// gOrbxDevice (default 0; set it before constructing the objects).
#pragma once

namespace ORB_SLAM2 {
extern int gOrbxDevice;
// The stereo Frame constructor runs its two ExtractORB calls and ComputeStereoMatches as one library
// call (orbx_frame_stereo) when both extractors have the same parameters (default true); false keeps
// the reference's two extraction threads followed by the matcher (same results).
extern bool gOrbxFrameStereoFused;
}  // namespace ORB_SLAM2
