// mapping.cpp -- CPU ORACLE (test infrastructure only) of the two small
// per-KeyFrame / per-MapPoint routines of SURVEY §8(f) row 4:
//
//   MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:249-320
//   Frame::UndistortKeyPoints                src/Frame.cc:471-506 (and the
//                                            corner pass of ComputeImageBounds,
//                                            :508-537)
//
// UndistortKeyPoints delegates to cv::undistortPoints (OpenCV 3.2, absent from
// /root/reference): restated here from the published cvUndistortPoints
// (modules/imgproc/src/undistort.cpp): everything in double, x0 = (x-cx)*ifx
// with ifx = 1./fx, five fixed-point iterations of the inverse radial +
// tangential model, then P*R = K applied and the result narrowed to float.
// The tilt matrix is the identity and the rational / thin-prism coefficients
// are zero for the <= 5-coefficient mDistCoef ORB-SLAM2 builds
// (src/Tracking.cc:75-85), so those terms vanish exactly and are omitted.
// Parity against OpenCV itself is unpinned.
#include <climits>
#include <cstdint>
#include <cstring>

#include "orb_oracle.h"

namespace {

int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

// One MapPoint: descs = its observed descriptors in mObservations order (bad
// KeyFrames already dropped by the caller, :270-276).  Returns BestIdx.
int distinctive_one(const uint8_t* descs, int n) {
  if (n <= 0) return -1;  // vDescriptors.empty(): mDescriptor unchanged (:278-279)
  int* row = new int[n];
  int best_median = INT_MAX, best = 0;
  const size_t k = (size_t)(0.5 * (n - 1));  // vDists[0.5*(N-1)] (:306)
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) row[j] = i == j ? 0 : hamming(descs + 32 * (size_t)i, descs + 32 * (size_t)j);
    for (int a = 1; a < n; a++) {  // sort(vDists) (:304), insertion sort
      const int v = row[a];
      int b = a - 1;
      while (b >= 0 && row[b] > v) {
        row[b + 1] = row[b];
        b--;
      }
      row[b + 1] = v;
    }
    const int median = row[k];
    if (median < best_median) {
      best_median = median;
      best = i;
    }
  }
  delete[] row;
  return best;
}

}  // namespace

extern "C" void oracle_distinctive_descriptors(const uint8_t* desc, const int32_t* obs_off, int n_points,
                                               int32_t* best, uint8_t* out_desc) {
  for (int p = 0; p < n_points; p++) {
    const int b = distinctive_one(desc + 32 * (size_t)obs_off[p], obs_off[p + 1] - obs_off[p]);
    best[p] = b;
    if (out_desc && b >= 0) std::memcpy(out_desc + 32 * (size_t)p, desc + 32 * ((size_t)obs_off[p] + b), 32);
  }
}

// cvUndistortPoints for one point, K = mK (float 3x3 row-major), dist =
// mDistCoef (k1, k2, p1, p2[, k3]).
extern "C" void oracle_undistort_point(const float K[9], const float* dist, int n_dist, float x_in, float y_in,
                                       float* x_out, float* y_out) {
  double k[5] = {0, 0, 0, 0, 0};
  for (int i = 0; i < n_dist && i < 5; i++) k[i] = dist[i];
  double A[9];
  for (int i = 0; i < 9; i++) A[i] = K[i];
  const double fx = A[0], fy = A[4], ifx = 1. / fx, ify = 1. / fy, cx = A[2], cy = A[5];
  double x = x_in, y = y_in;
  const double x0 = x = (x - cx) * ifx;
  const double y0 = y = (y - cy) * ify;
  for (int j = 0; j < 5; j++) {
    const double r2 = x * x + y * y;
    const double icdist = 1 / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
    const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  // RR = P * I = K exactly; ww = 1/(K20 x + K21 y + K22)
  const double xx = A[0] * x + A[1] * y + A[2];
  const double yy = A[3] * x + A[4] * y + A[5];
  const double ww = 1. / (A[6] * x + A[7] * y + A[8]);
  *x_out = (float)(xx * ww);
  *y_out = (float)(yy * ww);
}

// Frame::UndistortKeyPoints: keys_un = keys with pt replaced (:498-505), or a
// plain copy when mDistCoef(0) == 0 (:474-478).
extern "C" void oracle_undistort_keypoints(const oracle_keypoint* keys, int n, const float K[9], const float* dist,
                                           int n_dist, oracle_keypoint* keys_un) {
  for (int i = 0; i < n; i++) {
    keys_un[i] = keys[i];
    if (dist[0] == 0.0f) continue;
    oracle_undistort_point(K, dist, n_dist, keys[i].x, keys[i].y, &keys_un[i].x, &keys_un[i].y);
  }
}
