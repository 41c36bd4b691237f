// Optimizer.h -- Optimizer::LocalBundleAdjustment (include/Optimizer.h:61, src/Optimizer.cc:530-885)
// over liborbx.so, taking the local window as an explicit problem: the caller gathers
// lLocalKeyFrames / lFixedCameras / lLocalMapPoints and their observations exactly as
// src/Optimizer.cc:532-650 does and applies the result under the map mutex (:817-885).
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
};

class Optimizer {
 public:
  // pbStopFlag: the reference's bool* (NULL allowed), polled before the run and between LM trials.
  // Throws std::runtime_error on a library error.
  void static LocalBundleAdjustment(const LocalBAProblem& problem, bool* pbStopFlag, LocalBAResult& result,
                                    int device = 0);
};

}  // namespace ORB_SLAM2
