// Objects.h -- the fields and methods of ORB-SLAM2's Frame / KeyFrame / MapPoint / Map (and DBoW2's
// FeatureVector) that the hot-path members read or mutate, with the reference's names and
// signatures.  Inside ORB-SLAM2 these are the real classes (include/Frame.h, include/KeyFrame.h,
// include/MapPoint.h, include/Map.h) and shim.cc compiles against them unchanged; here they are
// minimal stand-ins the shim's tests build object graphs from.  Bodies restate the reference's
// (src/KeyFrame.cc, src/MapPoint.cc) for exactly the members LocalBundleAdjustment's gather and
// write-back use.
#pragma once
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "opencv_min.hpp"

namespace DBoW2 {
typedef unsigned int NodeId;
// Thirdparty/DBoW2/DBoW2/FeatureVector.h: node id -> indices of the features under it (ascending ids)
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2

namespace ORB_SLAM2 {

class ORBextractor;
class KeyFrame;
class Map;

class MapPoint {
 public:
  MapPoint() = default;
  MapPoint(const cv::Mat& Pos, KeyFrame* pRefKF, Map* pMap) : mpRefKF(pRefKF), mpMap(pMap) { SetWorldPos(Pos); }

  void SetWorldPos(const cv::Mat& Pos) {  // include/MapPoint.h:45
    std::unique_lock<std::mutex> lock(mMutexPos);
    Pos.copyTo(mWorldPos);
  }
  cv::Mat GetWorldPos() {  // include/MapPoint.h:46
    std::unique_lock<std::mutex> lock(mMutexPos);
    return mWorldPos.clone();
  }
  cv::Mat GetNormal() {
    std::unique_lock<std::mutex> lock(mMutexPos);
    return mNormalVector.clone();
  }
  std::map<KeyFrame*, size_t> GetObservations() {  // include/MapPoint.h:52
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mObservations;
  }
  int Observations() {
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return nObs;
  }
  void AddObservation(KeyFrame* pKF, size_t idx);  // src/MapPoint.cc AddObservation
  void EraseObservation(KeyFrame* pKF);            // src/MapPoint.cc EraseObservation
  int GetIndexInKeyFrame(KeyFrame* pKF) {          // include/MapPoint.h:66
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    auto it = mObservations.find(pKF);
    return it == mObservations.end() ? -1 : (int)it->second;
  }
  void SetBadFlag();                                // src/MapPoint.cc SetBadFlag
  bool isBad() {                                    // include/MapPoint.h: isBad()
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mbBad;
  }
  void UpdateNormalAndDepth();                      // src/MapPoint.cc UpdateNormalAndDepth
  float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }
  float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }

  long unsigned int mnId = 0;
  long unsigned int mnBALocalForKF = 0;
  int nObs = 0;
  bool mbBad = false;
  cv::Mat mWorldPos, mNormalVector;
  float mfMinDistance = 0.f, mfMaxDistance = 0.f;
  std::map<KeyFrame*, size_t> mObservations;
  KeyFrame* mpRefKF = nullptr;
  Map* mpMap = nullptr;
  std::mutex mMutexPos, mMutexFeatures;
};

class KeyFrame {
 public:
  void SetPose(const cv::Mat& Tcw_);  // src/KeyFrame.cc SetPose (Tcw, Ow)
  cv::Mat GetPose() {                  // include/KeyFrame.h:50
    std::unique_lock<std::mutex> lock(mMutexPose);
    return Tcw.clone();
  }
  cv::Mat GetCameraCenter() {          // include/KeyFrame.h:52
    std::unique_lock<std::mutex> lock(mMutexPose);
    return Ow.clone();
  }
  // covisibility graph order (weights descending), src/KeyFrame.cc GetVectorCovisibleKeyFrames
  std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() {
    std::unique_lock<std::mutex> lock(mMutexConnections);
    return mvpOrderedConnectedKeyFrames;
  }
  void EraseMapPointMatch(const size_t& idx) {  // include/KeyFrame.h:103
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    mvpMapPoints[idx] = nullptr;
  }
  void EraseMapPointMatch(MapPoint* pMP) {      // include/KeyFrame.h:104
    const int idx = pMP->GetIndexInKeyFrame(this);
    if (idx >= 0) mvpMapPoints[idx] = nullptr;
  }
  std::vector<MapPoint*> GetMapPointMatches() {  // src/KeyFrame.cc
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mvpMapPoints;
  }
  bool isBad() { return mbBad; }

  long unsigned int mnId = 0;
  long unsigned int mnBALocalForKF = 0, mnBAFixedForKF = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0, mThDepth = 0;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeysUn;
  std::vector<float> mvuRight, mvDepth;  // negative: monocular
  cv::Mat mDescriptors;                  // N x 32 CV_8U
  DBoW2::FeatureVector mFeatVec;
  int mnScaleLevels = 8;
  std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
  std::vector<MapPoint*> mvpMapPoints;
  std::vector<KeyFrame*> mvpOrderedConnectedKeyFrames;
  bool mbBad = false;
  cv::Mat Tcw, Ow;
  std::mutex mMutexPose, mMutexConnections, mMutexFeatures;
};

class Map {
 public:
  void EraseMapPoint(MapPoint* pMP) {  // src/Map.cc EraseMapPoint
    std::unique_lock<std::mutex> lock(mMutexMap);
    mspMapPoints.erase(pMP);
  }
  std::set<MapPoint*> mspMapPoints;
  std::mutex mMutexMapUpdate;  // include/Map.h:65
  std::mutex mMutexMap;
};

// ---- the reference bodies (src/MapPoint.cc, src/KeyFrame.cc), restated for the stand-ins
inline void MapPoint::AddObservation(KeyFrame* pKF, size_t idx) {
  std::unique_lock<std::mutex> lock(mMutexFeatures);
  if (mObservations.count(pKF)) return;
  mObservations[pKF] = idx;
  if (pKF->mvuRight[idx] >= 0)
    nObs += 2;
  else
    nObs++;
}

inline void MapPoint::EraseObservation(KeyFrame* pKF) {
  bool bBad = false;
  {
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    if (mObservations.count(pKF)) {
      const int idx = (int)mObservations[pKF];
      if (pKF->mvuRight[idx] >= 0)
        nObs -= 2;
      else
        nObs--;
      mObservations.erase(pKF);
      if (mpRefKF == pKF) mpRefKF = mObservations.empty() ? nullptr : mObservations.begin()->first;
      if (nObs <= 2) bBad = true;
    }
  }
  if (bBad) SetBadFlag();
}

inline void MapPoint::SetBadFlag() {
  std::map<KeyFrame*, size_t> obs;
  {
    std::unique_lock<std::mutex> lock1(mMutexFeatures);
    std::unique_lock<std::mutex> lock2(mMutexPos);
    mbBad = true;
    obs = mObservations;
    mObservations.clear();
  }
  for (auto& o : obs) o.first->EraseMapPointMatch(o.second);
  if (mpMap) mpMap->EraseMapPoint(this);
}

inline void MapPoint::UpdateNormalAndDepth() {
  std::map<KeyFrame*, size_t> observations;
  KeyFrame* pRefKF;
  cv::Mat Pos;
  {
    std::unique_lock<std::mutex> lock1(mMutexFeatures);
    std::unique_lock<std::mutex> lock2(mMutexPos);
    if (mbBad) return;
    observations = mObservations;
    pRefKF = mpRefKF;
    Pos = mWorldPos.clone();
  }
  if (observations.empty() || !pRefKF) return;
  float normal[3] = {0.f, 0.f, 0.f};
  int n = 0;
  for (auto& o : observations) {
    const cv::Mat Owi = o.first->GetCameraCenter();
    float d[3];
    double s = 0;
    for (int k = 0; k < 3; k++) {
      d[k] = Pos.at<float>(k, 0) - Owi.at<float>(k, 0);
      s += (double)d[k] * d[k];
    }
    const double nrm = std::sqrt(s);  // cv::norm (L2, accumulated in double)
    for (int k = 0; k < 3; k++) normal[k] = normal[k] + (float)(d[k] / nrm);
    n++;
  }
  const cv::Mat Oref = pRefKF->GetCameraCenter();
  double s = 0;
  for (int k = 0; k < 3; k++) {
    const float d = Pos.at<float>(k, 0) - Oref.at<float>(k, 0);
    s += (double)d * d;
  }
  const float dist = (float)std::sqrt(s);
  const int level = pRefKF->mvKeysUn[observations[pRefKF]].octave;
  const float levelScaleFactor = pRefKF->mvScaleFactors[level];
  const int nLevels = pRefKF->mnScaleLevels;
  std::unique_lock<std::mutex> lock3(mMutexPos);
  mfMaxDistance = dist * levelScaleFactor;
  mfMinDistance = mfMaxDistance / pRefKF->mvScaleFactors[nLevels - 1];
  mNormalVector.create(3, 1, CV_32F);
  for (int k = 0; k < 3; k++) mNormalVector.at<float>(k, 0) = normal[k] / (float)n;
}

inline void KeyFrame::SetPose(const cv::Mat& Tcw_) {
  std::unique_lock<std::mutex> lock(mMutexPose);
  Tcw_.copyTo(Tcw);
  Ow.create(3, 1, CV_32F);
  for (int r = 0; r < 3; r++) {  // Ow = -Rcw^T * tcw
    float acc = 0.f;
    for (int k = 0; k < 3; k++) acc += Tcw.at<float>(k, r) * Tcw.at<float>(k, 3);
    Ow.at<float>(r, 0) = -acc;
  }
}

class Frame {
 public:
  Frame() = default;
  // Stereo constructor, ORB part (src/Frame.cc:62-100, without timestamp / vocabulary / grid):
  // left and right extraction on two threads, N, the scale tables, the static intrinsics
  // (fx, fy, cx, cy, invfx, invfy from K, src/Frame.cc:111-126), mb = mbf/fx, UndistortKeyPoints
  // (a copy when mDistCoef(0) == 0, :473-476, else cv::undistortPoints on the GPU),
  // ComputeStereoMatches.  K: 3x3 CV_32F, distCoef: 4x1 or 5x1 CV_32F.
  Frame(const cv::Mat& imLeft, const cv::Mat& imRight, ORBextractor* extractorLeft, ORBextractor* extractorRight,
        const cv::Mat& K, const cv::Mat& distCoef, float bf, float thDepth);

  void ExtractORB(int flag, const cv::Mat& im);  // src/Frame.cc:273-279
  void UndistortKeyPoints();                     // src/Frame.cc:471-506
  void ComputeStereoMatches();                   // src/Frame.cc:547-788 (on the MI355X)

  cv::Mat mK, mDistCoef;
  static float fx, fy, cx, cy, invfx, invfy;  // include/Frame.h:135-140

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
  int mnScaleLevels = 0;
  float mfScaleFactor = 0.f;
  std::vector<float> mvScaleFactors, mvInvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;
};

// Free-function form of Frame::ComputeStereoMatches for callers without a Frame object:
// mvuRight / mvDepth (resized to kpsL.size()) from two extractors' last extraction.
void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, const std::vector<cv::KeyPoint>& kpsL,
                          const cv::Mat& descL, const std::vector<cv::KeyPoint>& kpsR, const cv::Mat& descR,
                          float mbf, float mb, std::vector<float>& mvuRight, std::vector<float>& mvDepth);

}  // namespace ORB_SLAM2
