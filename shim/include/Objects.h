// Objects.h -- the fields and methods of ORB-SLAM2's Frame / KeyFrame / MapPoint / Map (and DBoW2's
// FeatureVector) that the hot-path members read or mutate, with the reference's names and
// signatures.  Inside ORB-SLAM2 these are the real classes (include/Frame.h, include/KeyFrame.h,
// include/MapPoint.h, include/Map.h) and shim.cc compiles against them unchanged; here they are
// minimal stand-ins the shim's tests build object graphs from.  Bodies restate the reference's
// (src/KeyFrame.cc, src/MapPoint.cc, src/Frame.cc) for exactly the members the shim's hot-path
// bodies use: LocalBundleAdjustment's gather and write-back, SearchByProjection x3, Fuse's
// Replace/AddObservation, SearchForTriangulation, PoseOptimization, ComputeDistinctiveDescriptors
// and ComputeBoW.
#pragma once
#include <cmath>
#include <map>
#include <mutex>
#include <set>
#include <vector>

#include "opencv_min.hpp"

namespace DBoW2 {
typedef unsigned int NodeId;
typedef unsigned int WordId;
typedef double WordValue;
// Thirdparty/DBoW2/DBoW2/FeatureVector.h: node id -> indices of the features under it (ascending ids)
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
// Thirdparty/DBoW2/DBoW2/BowVector.h: word id -> weight (ascending ids)
class BowVector : public std::map<WordId, WordValue> {};
}  // namespace DBoW2

namespace ORB_SLAM2 {

class ORBextractor;
class ORBVocabulary;
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
  float GetMinDistanceInvariance() {
    std::unique_lock<std::mutex> lock(mMutexPos);
    return 0.8f * mfMinDistance;
  }
  float GetMaxDistanceInvariance() {
    std::unique_lock<std::mutex> lock(mMutexPos);
    return 1.2f * mfMaxDistance;
  }
  cv::Mat GetDescriptor() {                         // src/MapPoint.cc:323-327
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mDescriptor.clone();
  }
  bool IsInKeyFrame(KeyFrame* pKF) {                // src/MapPoint.cc IsInKeyFrame
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mObservations.count(pKF) > 0;
  }
  void IncreaseVisible(int n = 1) {
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    mnVisible += n;
  }
  void IncreaseFound(int n = 1) {
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    mnFound += n;
  }
  void Replace(MapPoint* pMP);                      // src/MapPoint.cc:179-221
  // MapPoint::ComputeDistinctiveDescriptors (include/MapPoint.h:85, src/MapPoint.cc:249-320): the
  // observed descriptor with the least median Hamming distance to the others, on the MI355X
  // (defined in shim.cc over orbx_distinctive_descriptors)
  void ComputeDistinctiveDescriptors();

  long unsigned int mnId = 0;
  long unsigned int mnBALocalForKF = 0, mnFuseCandidateForKF = 0;
  int nObs = 0;
  int mnVisible = 1, mnFound = 1;
  bool mbBad = false;
  MapPoint* mpReplaced = nullptr;
  cv::Mat mWorldPos, mNormalVector;
  cv::Mat mDescriptor;  // 1 x 32 CV_8U (the best descriptor)
  float mfMinDistance = 0.f, mfMaxDistance = 0.f;
  // Tracking::SearchLocalPoints' frustum test results read by SearchByProjection(Frame&, vector<MapPoint*>)
  bool mbTrackInView = false;
  float mTrackProjX = 0.f, mTrackProjY = 0.f, mTrackProjXR = 0.f, mTrackViewCos = 0.f;
  int mnTrackScaleLevel = 0;
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
  std::set<MapPoint*> GetMapPoints();           // src/KeyFrame.cc GetMapPoints: the non-bad MapPoints
  MapPoint* GetMapPoint(const size_t& idx) {     // src/KeyFrame.cc GetMapPoint
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    return mvpMapPoints[idx];
  }
  void AddMapPoint(MapPoint* pMP, const size_t& idx) {  // src/KeyFrame.cc AddMapPoint
    std::unique_lock<std::mutex> lock(mMutexFeatures);
    mvpMapPoints[idx] = pMP;
  }
  void ReplaceMapPointMatch(const size_t& idx, MapPoint* pMP) { mvpMapPoints[idx] = pMP; }
  cv::Mat GetRotation() {                        // Tcw.rowRange(0,3).colRange(0,3)
    std::unique_lock<std::mutex> lock(mMutexPose);
    cv::Mat R(3, 3, CV_32F);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) R.at<float>(r, c) = Tcw.at<float>(r, c);
    return R;
  }
  cv::Mat GetTranslation() {                     // Tcw.rowRange(0,3).col(3)
    std::unique_lock<std::mutex> lock(mMutexPose);
    cv::Mat t(3, 1, CV_32F);
    for (int r = 0; r < 3; r++) t.at<float>(r, 0) = Tcw.at<float>(r, 3);
    return t;
  }
  bool IsInImage(const float& x, const float& y) const {  // src/KeyFrame.cc:749-752
    return (x >= mnMinX && x < mnMaxX && y >= mnMinY && y < mnMaxY);
  }
  void ComputeBoW();                             // src/KeyFrame.cc ComputeBoW (defined in shim.cc)
  bool isBad() { return mbBad; }

  long unsigned int mnId = 0;
  long unsigned int mnBALocalForKF = 0, mnBAFixedForKF = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0, invfx = 0, invfy = 0, mbf = 0, mb = 0, mThDepth = 0;
  int N = 0;
  std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
  std::vector<float> mvuRight, mvDepth;  // negative: monocular
  cv::Mat mDescriptors;                  // N x 32 CV_8U
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  ORBVocabulary* mpORBvocabulary = nullptr;
  // the Frame's image bounds and grid, copied at KeyFrame creation (include/KeyFrame.h: const int mnMinX..)
  int mnMinX = 0, mnMinY = 0, mnMaxX = 0, mnMaxY = 0;
  float mfGridElementWidthInv = 0.f, mfGridElementHeightInv = 0.f;
  int mnScaleLevels = 8;
  float mfScaleFactor = 1.2f, mfLogScaleFactor = 0.f;
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

inline void MapPoint::Replace(MapPoint* pMP) {
  if (pMP->mnId == this->mnId) return;
  int nvisible, nfound;
  std::map<KeyFrame*, size_t> obs;
  {
    std::unique_lock<std::mutex> lock1(mMutexFeatures);
    std::unique_lock<std::mutex> lock2(mMutexPos);
    obs = mObservations;
    mObservations.clear();
    mbBad = true;
    nvisible = mnVisible;
    nfound = mnFound;
    mpReplaced = pMP;
  }
  for (auto& o : obs) {
    KeyFrame* pKF = o.first;
    if (!pMP->IsInKeyFrame(pKF)) {
      pKF->ReplaceMapPointMatch(o.second, pMP);
      pMP->AddObservation(pKF, o.second);
    } else {
      pKF->EraseMapPointMatch(o.second);
    }
  }
  pMP->IncreaseFound(nfound);
  pMP->IncreaseVisible(nvisible);
  pMP->ComputeDistinctiveDescriptors();
  if (mpMap) mpMap->EraseMapPoint(this);
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
  // The reference's stereo constructor with its own signature (include/Frame.h:55, src/Frame.cc:62-133):
  // as above, plus mnId / mTimeStamp / the vocabulary, mfLogScaleFactor, and on the first frame
  // ComputeImageBounds + the grid cell inverses (the statics mnMinX.., mfGridElementWidthInv..).
  Frame(const cv::Mat& imLeft, const cv::Mat& imRight, const double& timeStamp, ORBextractor* extractorLeft,
        ORBextractor* extractorRight, ORBVocabulary* voc, cv::Mat& K, cv::Mat& distCoef, const float& bf,
        const float& thDepth);

  void ExtractORB(int flag, const cv::Mat& im);  // src/Frame.cc:273-279
  void UndistortKeyPoints();                     // src/Frame.cc:471-506
  void ComputeImageBounds(const cv::Mat& imLeft);  // src/Frame.cc:508-537 (corners on the MI355X)
  void ComputeStereoMatches();                   // src/Frame.cc:547-788 (on the MI355X)
  void ComputeBoW();                             // src/Frame.cc:462-469 (ORBVocabulary::transform on the MI355X)
  void SetPose(const cv::Mat& Tcw);              // src/Frame.cc SetPose + UpdatePoseMatrices
  void UpdatePoseMatrices();
  cv::Mat GetCameraCenter() { return mOw.clone(); }

  cv::Mat mK, mDistCoef;
  static float fx, fy, cx, cy, invfx, invfy;  // include/Frame.h:135-140
  // image bounds and grid cell inverses, computed once (include/Frame.h: static float mnMinX ...)
  static float mnMinX, mnMaxX, mnMinY, mnMaxY;
  static float mfGridElementWidthInv, mfGridElementHeightInv;
  static bool mbInitialComputations;
  ORBVocabulary* mpORBvocabulary = nullptr;
  DBoW2::BowVector mBowVec;
  double mTimeStamp = 0.0;
  static long unsigned int nNextId;
  long unsigned int mnId = 0;
  cv::Mat mTcw, mRcw, mtcw, mRwc, mOw;
  float mfLogScaleFactor = 0.f;

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

 private:
  // src/Frame.cc:86-123 after the two ExtractORB calls; uR / dep: stereo results already computed by
  // orbx_frame_stereo (null: ComputeStereoMatches runs)
  void finish_stereo_frame(const std::vector<float>* uR, const std::vector<float>* dep);
};

// Free-function form of Frame::ComputeStereoMatches for callers without a Frame object:
// mvuRight / mvDepth (resized to kpsL.size()) from two extractors' last extraction.
void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, const std::vector<cv::KeyPoint>& kpsL,
                          const cv::Mat& descL, const std::vector<cv::KeyPoint>& kpsR, const cv::Mat& descR,
                          float mbf, float mb, std::vector<float>& mvuRight, std::vector<float>& mvDepth);

}  // namespace ORB_SLAM2
