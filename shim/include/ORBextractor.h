// ORBextractor.h -- drop-in ORB_SLAM2::ORBextractor over liborbx.so.
// Public interface of the reference class (include/ORBextractor.h:51-145): the constructor
// (:61), operator() (:77-78), the level/scale getters (:81-102) and mvImagePyramid (:104), and its
// protected members in the reference's order (:118-144), filled from the library's tables.
// Extraction runs on the MI355X (orbx_extract) on device gOrbxDevice (orbx_shim.h); the handle owns
// one HIP stream, so Frame's two extraction threads (src/Frame.cc:80-84) drive two extractors
// concurrently, as in the reference.
#pragma once
#include <vector>

#include "opencv_min.hpp"
#include "orbx.h"

namespace ORB_SLAM2 {

class Frame;

class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  // Throws std::runtime_error (message carries the orbx_status) when no gfx950 device is usable.
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
  ~ORBextractor();
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // Mask is ignored, as in the reference.  An empty image returns silently (src/ORBextractor.cc:1141).
  // Every call refreshes mvImagePyramid, as ComputePyramid does (src/ORBextractor.cc:1215-1250): the
  // levels leave the device in the same stream as the keypoints, before the call's one synchronisation.
  void operator()(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                  cv::OutputArray descriptors);

  int inline GetLevels() { return nlevels; }
  float inline GetScaleFactor() { return scaleFactor; }
  std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  // Level l of the last operator() call's image pyramid (level 0 = the input image).  The only
  // opt-out is this shim's own Frame (below), whose ComputeStereoMatches reads the device copy.
  std::vector<cv::Mat> mvImagePyramid;

  // The device handle (Frame::ComputeStereoMatches binds two of them).
  orbx_extractor* gpu() const { return mpGpu; }

 protected:
  friend class Frame;
  // operator() without the host pyramid: Frame's extraction threads (the stereo matcher reads the
  // levels on the device).  mvImagePyramid is emptied, so no stale levels outlive the call.
  void ExtractForFrame(const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints, cv::Mat& descriptors);
  void Extract(cv::InputArray image, std::vector<cv::KeyPoint>& keypoints, cv::OutputArray descriptors,
               bool pyramid);

  std::vector<cv::Point> pattern;  // the 256 rBRIEF pairs' 512 sample points (bit_pattern_31_)
  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;
  std::vector<int> mnFeaturesPerLevel;
  std::vector<int> umax;
  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;
  orbx_extractor* mpGpu = nullptr;  // the one member the reference does not have
};

}  // namespace ORB_SLAM2
