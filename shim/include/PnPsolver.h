// PnPsolver.h -- drop-in ORB_SLAM2::PnPsolver over liborbx.so (include/PnPsolver.h:60-77): the
// constructor gathers the 2D-3D correspondences of a Frame's MapPoint matches exactly as
// src/PnPsolver.cc:67-125 does, SetRansacParameters derives the reference's RANSAC parameters
// (src/PnPsolver.cc:136-179), and iterate()/find() run the EPnP RANSAC + Refine on the MI355X
// (src/PnPsolver.cc:182-349), bit-exact with the reference's arithmetic.
//
// Random numbers: the reference draws DUtils::Random::RandomInt from the process rand() (glibc,
// never seeded on the stereo path: seed 1).  Every PnPsolver of the process draws from ONE shared
// glibc-rand() stream held by the shim (orbx_rand_state, seed 1), so a sequence of iterate()
// calls -- e.g. Tracking::Relocalization's round-robin over candidate KeyFrames,
// src/Tracking.cc:1738-1757 -- consumes the stream exactly as the reference does.
// SeedRandom() restarts it (DUtils::Random::SeedRand).
#pragma once
#include <vector>

#include "Objects.h"
#include "opencv_min.hpp"
#include "orbx.h"

namespace ORB_SLAM2 {

class PnPsolver {
 public:
  PnPsolver(const Frame& F, const std::vector<MapPoint*>& vpMapPointMatches);
  ~PnPsolver();
  PnPsolver(const PnPsolver&) = delete;
  PnPsolver& operator=(const PnPsolver&) = delete;

  // As the reference: may be called at any time; after iterate() the derived parameters are
  // recomputed in place and the iteration count / best set are kept (src/PnPsolver.cc:136-179).
  void SetRansacParameters(double probability = 0.99, int minInliers = 8, int maxIterations = 300, int minSet = 4,
                           float epsilon = 0.4, float th2 = 5.991);

  cv::Mat find(std::vector<bool>& vbInliers, int& nInliers);
  // Returns Tcw (4x4 CV_32F) or an empty Mat; vbInliers is indexed like vpMapPointMatches.
  cv::Mat iterate(int nIterations, bool& bNoMore, std::vector<bool>& vbInliers, int& nInliers);

  static void SeedRandom(unsigned int seed);  // the shared stream (srand)

 private:
  void ensure_solver();
  std::vector<MapPoint*> mvpMapPointMatches;
  std::vector<float> mvP2D, mvP3Dw, mvSigma2;  // x,y / x,y,z / sigma^2 per correspondence
  std::vector<size_t> mvKeyPointIndices;
  float fu = 0, fv = 0, uc = 0, vc = 0;
  orbx_pnp_params mParams{0.99, 8, 300, 4, 0.4f, 5.991f};
  int mRansacMaxIts = 0;
  orbx_pnp* mpGpu = nullptr;
};

}  // namespace ORB_SLAM2
