// ORBextractor.h -- drop-in ORB_SLAM2::ORBextractor over liborbx.so.
// Public interface of the reference class (include/ORBextractor.h:51-104): the constructor
// (:61), operator() (:77-78), the level/scale getters (:81-103) and mvImagePyramid (:104).
// Extraction runs on the MI355X (orbx_extract); the handle owns one HIP stream, so Frame's two
// extraction threads (src/Frame.cc:80-84) drive two extractors concurrently, as in the reference.
#pragma once
#include <vector>

#include "opencv_min.hpp"
#include "orbx.h"

namespace ORB_SLAM2 {

class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  // Throws std::runtime_error (message carries the orbx_status) when no gfx950 device is usable.
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0);
  ~ORBextractor();
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // Mask is ignored, as in the reference.  An empty image returns silently (src/ORBextractor.cc:1141).
  void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                  cv::OutputArray descriptors);

  int inline GetLevels() { return nlevels; }
  float inline GetScaleFactor() { return scaleFactor; }
  std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  // The reference's only readers of mvImagePyramid are in Frame::ComputeStereoMatches
  // (src/Frame.cc:556,681,694,700), which here runs on the device copy; so by default the host
  // copy is NOT downloaded (eight synchronous copies per call).  A caller that reads the levels
  // on the host sets mbDownloadPyramid, and every operator() call then fills them.
  std::vector<cv::Mat> mvImagePyramid;
  bool mbDownloadPyramid = false;

  // The device handle (Frame::ComputeStereoMatches binds two of them).
  orbx_extractor* gpu() const { return mpGpu; }

 protected:
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;
  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;
  orbx_extractor* mpGpu = nullptr;
};

}  // namespace ORB_SLAM2
