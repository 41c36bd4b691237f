// Objects.h -- the fields of ORB-SLAM2's Frame / KeyFrame / MapPoint (and DBoW2's FeatureVector)
// that the hot-path members read, with the reference's names.  Inside ORB-SLAM2 these are the
// real classes (include/Frame.h, include/KeyFrame.h, include/MapPoint.h); here they are the
// minimal stand-ins the shim's tests construct.
#pragma once
#include <map>
#include <vector>

#include "opencv_min.hpp"

namespace DBoW2 {
typedef unsigned int NodeId;
// Thirdparty/DBoW2/DBoW2/FeatureVector.h: node id -> indices of the features under it (ascending ids)
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2

namespace ORB_SLAM2 {

class ORBextractor;

class MapPoint {
 public:
  bool mbBad = false;
  bool isBad() const { return mbBad; }  // include/MapPoint.h: isBad()
};

class KeyFrame {
 public:
  int N = 0;
  std::vector<cv::KeyPoint> mvKeysUn;
  cv::Mat mDescriptors;            // N x 32 CV_8U
  DBoW2::FeatureVector mFeatVec;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }  // src/KeyFrame.cc
};

class Frame {
 public:
  Frame() = default;
  // Stereo constructor, ORB part (src/Frame.cc:62-100, without timestamp / vocabulary / grid):
  // left and right extraction on two threads, N, mb = mbf/fx, UndistortKeyPoints (a copy when
  // mDistCoef(0) == 0, :473-476, else cv::undistortPoints on the GPU), ComputeStereoMatches.
  // K: 3x3 CV_32F, distCoef: 4x1 or 5x1 CV_32F.
  Frame(const cv::Mat& imLeft, const cv::Mat& imRight, ORBextractor* extractorLeft, ORBextractor* extractorRight,
        const cv::Mat& K, const cv::Mat& distCoef, float bf, float thDepth);

  void ExtractORB(int flag, const cv::Mat& im);  // src/Frame.cc:273-279
  void UndistortKeyPoints();                     // src/Frame.cc:471-506
  void ComputeStereoMatches();                   // src/Frame.cc:547-788 (on the MI355X)

  cv::Mat mK, mDistCoef;

  ORBextractor* mpORBextractorLeft = nullptr;
  ORBextractor* mpORBextractorRight = nullptr;
  float mbf = 0.f, mb = 0.f, mThDepth = 0.f;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
  std::vector<float> mvuRight, mvDepth;
  cv::Mat mDescriptors, mDescriptorsRight;
  DBoW2::FeatureVector mFeatVec;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<bool> mvbOutlier;
};

// Free-function form of Frame::ComputeStereoMatches for callers without a Frame object:
// mvuRight / mvDepth (resized to kpsL.size()) from two extractors' last extraction.
void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, const std::vector<cv::KeyPoint>& kpsL,
                          const cv::Mat& descL, const std::vector<cv::KeyPoint>& kpsR, const cv::Mat& descR,
                          float mbf, float mb, std::vector<float>& mvuRight, std::vector<float>& mvDepth);

}  // namespace ORB_SLAM2
