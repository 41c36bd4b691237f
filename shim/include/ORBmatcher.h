// ORBmatcher.h -- drop-in ORB_SLAM2::ORBmatcher for the hot-path members over liborbx.so:
//   ORBmatcher(nnratio, checkOri)                 include/ORBmatcher.h:47
//   static DescriptorDistance(a, b)               include/ORBmatcher.h:50 (src/ORBmatcher.cc:1844-1860)
//   SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches)  include/ORBmatcher.h:114 (src/ORBmatcher.cc:175-325)
//   SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)     include/ORBmatcher.h:116 (src/ORBmatcher.cc:589-736)
//   SearchByProjection(Frame&, const vector<MapPoint*>&, th)            include/ORBmatcher.h:64
//                                                       (src/ORBmatcher.cc:46-142)
//   SearchByProjection(Frame&, const Frame&, th, bMono)                 include/ORBmatcher.h:76
//                                                       (src/ORBmatcher.cc:1489-1646)
//   SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)   include/ORBmatcher.h:95
//                                                       (src/ORBmatcher.cc:1648-1795)
//   SearchForTriangulation(KeyFrame*, KeyFrame*, F12, vMatchedPairs, bOnlyStereo) include/ORBmatcher.h:134
//                                                       (src/ORBmatcher.cc:738-925)
//   Fuse(KeyFrame*, const vector<MapPoint*>&, th)                       include/ORBmatcher.h:148
//   SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, vector<MapPoint*>&, th)
//                                                                       include/ORBmatcher.h:99
//   Fuse(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&, th, vector<MapPoint*>&)  include/ORBmatcher.h:153
//   SearchBySim3(KeyFrame*, KeyFrame*, vector<MapPoint*>&, s12, R12, t12, th)     include/ORBmatcher.h:139
//   SearchForInitialization(Frame&, Frame&, vector<Point2f>&, vector<int>&, windowSize) include/ORBmatcher.h:130
//                                                       (src/ORBmatcher.cc:442-587)
// Every member runs on device gOrbxDevice (orbx_shim.h); the layout is the reference's two members.
// DescriptorDistance of one pair stays on the host (a GPU launch per pair would cost more than the
// popcounts); every other member runs its matching on the MI355X (orbx_search_by_bow_*,
// orbx_search_by_projection, orbx_search_for_triangulation) and applies the result to the object
// graph here, as the reference's own loops do.
#pragma once
#include <set>
#include <utility>
#include <vector>

#include "Objects.h"
#include "opencv_min.hpp"

namespace ORB_SLAM2 {

class ORBmatcher {
 public:
  ORBmatcher(float nnratio = 0.6, bool checkOri = true);

  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b);

  int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
  int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);

  // Tracking::SearchLocalPoints' local map (mbTrackInView / mTrackProj* set by Frame::isInFrustum)
  int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th = 3);
  // Tracking::TrackWithMotionModel: the last frame's MapPoints into the current frame
  int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);
  // Tracking::Relocalization: a candidate KeyFrame's MapPoints not found yet
  int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                         const float th, const int ORBdist);
  // LoopClosing::ComputeSim3: the loop MapPoints into the current KeyFrame through a Sim3
  int SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                         std::vector<MapPoint*>& vpMatched, int th);
  // LoopClosing::SearchAndFuse: the loop MapPoints into a corrected KeyFrame through its Sim3
  int Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
           std::vector<MapPoint*>& vpReplacePoint);
  // Tracking::MonocularInitialization: F1's level-0 keypoints in windows around vbPrevMatched in F2
  int SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                              std::vector<int>& vnMatches12, int windowSize = 10);
  // LoopClosing::ComputeSim3: matches between two KeyFrames' MapPoints through a Sim3, both ways
  int SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12, const float& s12,
                   const cv::Mat& R12, const cv::Mat& t12, const float th);
  // LocalMapping::CreateNewMapPoints
  int SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                             std::vector<std::pair<size_t, size_t>>& vMatchedPairs, const bool bOnlyStereo);
  // LocalMapping::SearchInNeighbors
  int Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th = 3.0);

  static const int TH_LOW;
  static const int TH_HIGH;
  static const int HISTO_LENGTH;

 protected:
  float mfNNratio;
  bool mbCheckOrientation;
};

}  // namespace ORB_SLAM2
