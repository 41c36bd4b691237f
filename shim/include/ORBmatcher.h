// ORBmatcher.h -- drop-in ORB_SLAM2::ORBmatcher for the hot-path members over liborbx.so:
//   ORBmatcher(nnratio, checkOri)                 include/ORBmatcher.h:48
//   static DescriptorDistance(a, b)               include/ORBmatcher.h:50 (src/ORBmatcher.cc:1844-1860)
//   SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches)  include/ORBmatcher.h:114 (src/ORBmatcher.cc:175-325)
//   SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)     include/ORBmatcher.h:116 (src/ORBmatcher.cc:589-736)
// DescriptorDistance of one pair stays on the host (a GPU launch per pair would cost more than the
// popcounts); SearchByBoW runs on the MI355X (orbx_search_by_bow_kf_f / _kf_kf).
#pragma once
#include <vector>

#include "Objects.h"
#include "opencv_min.hpp"

namespace ORB_SLAM2 {

class ORBmatcher {
 public:
  ORBmatcher(float nnratio = 0.6, bool checkOri = true, int device = 0);

  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);

  int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
  int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);

  static const int TH_LOW;
  static const int TH_HIGH;
  static const int HISTO_LENGTH;

 protected:
  float mfNNratio;
  bool mbCheckOrientation;
  int mDevice;
};

}  // namespace ORB_SLAM2
