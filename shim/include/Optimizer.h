// Optimizer.h -- Optimizer::LocalBundleAdjustment (include/Optimizer.h:61, src/Optimizer.cc:530-885)
// over liborbx.so.  Two forms:
//   * the reference signature LocalBundleAdjustment(KeyFrame*, bool*, Map*): the shim gathers the
//     local window from the object graph exactly as src/Optimizer.cc:532-745 does (covisible
//     KeyFrames, their MapPoints, the fixed cameras that observe them, one edge per observation in
//     GetObservations() order), runs it on the MI355X, and applies the result as :817-884 does
//     (EraseMapPointMatch / EraseObservation under Map::mMutexMapUpdate, SetPose, SetWorldPos,
//     UpdateNormalAndDepth);
//   * the same on an explicit problem (the caller gathers and applies).
// g2o semantics (BlockSolver_6_3, LinearSolverEigen, Levenberg, Huber kernels, optimize(5),
// outlier levels, optimize(10)) run in FP64 on the MI355X.
#pragma once
#include <array>
#include <vector>

#include "opencv_min.hpp"

namespace ORB_SLAM2 {

struct LocalBAProblem {
  struct Camera {
    cv::Mat Tcw;                    // 4x4 CV_32F, KeyFrame::GetPose()
    bool fixed = false;             // mnId == 0, or a member of lFixedCameras
    float fx = 0, fy = 0, cx = 0, cy = 0, bf = 0;
  };
  struct Observation {              // one edge per (KeyFrame, MapPoint) observation, in the reference's order
    int point = 0, camera = 0;
    float u = 0, v = 0;             // mvKeysUn[idx].pt
    float ur = -1;                  // mvuRight[idx]; < 0: monocular EdgeSE3ProjectXYZ
    float invSigma2 = 1;            // mvInvLevelSigma2[octave]
  };
  std::vector<Camera> cameras;
  std::vector<cv::Mat> points;      // 3x1 CV_32F, MapPoint::GetWorldPos()
  std::vector<Observation> observations;
};

struct LocalBAResult {
  std::vector<cv::Mat> Tcw;         // 4x4 CV_32F per camera (Converter::toCvMat of the optimised SE3Quat)
  std::vector<cv::Mat> points;      // 3x1 CV_32F per point
  std::vector<bool> erase;          // per observation: vToErase (:817-847)
  int iterations[2] = {0, 0};       // LM iterations of optimize(5) and optimize(10)
  int trials = 0;
  bool ran = false;                 // false: stopped before optimize(5), outputs are the inputs (:749-751)
};

class KeyFrame;
class Map;
class Frame;

class Optimizer {
 public:
  // include/Optimizer.h:71, src/Optimizer.cc:287-528: the pose of pFrame from its MapPoint matches
  // (four rounds of optimize(10) with outlier levels, on the MI355X).  Sets pFrame->mvbOutlier and,
  // with >= 3 correspondences, pFrame->SetPose; returns the inlier count (0 below 3 matches).
  int static PoseOptimization(Frame* pFrame);
  // include/Optimizer.h:61.  pbStopFlag: the reference's bool* (NULL allowed), polled before the
  // run and between LM trials.  Runs on device gOrbxDevice.  Throws std::runtime_error on a library
  // error (the object graph is then left as it was).
  void static LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap);
  // The explicit-problem form.  Throws std::runtime_error on a library error.
  void static LocalBundleAdjustment(const LocalBAProblem& problem, bool* pbStopFlag, LocalBAResult& result,
                                    int device = 0);

  // test hook: called with the window the graph form gathered, before it runs (NULL: none)
  static void (*mpfnGatheredHook)(const LocalBAProblem& problem, const std::vector<KeyFrame*>& cameras);
};

}  // namespace ORB_SLAM2
