// triangulation.cpp -- CPU ORACLE (test infrastructure only) of
// ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:738-925) with
// CheckDistEpipolarLine (:153-173) and ComputeThreeMaxima (:1797-1839).
//
// Behaviour kept from this reference commit: vbMatched2 is declared but never
// set (:760, :810), so every KF1 feature is matched independently; a
// candidate replaces the current best when dist <= bestDist (ties: the later
// one wins) and it passes the epipolar test; `3.84*mvLevelSigma2` and the
// comparison are double.  C2 = R2w*Cw + t2w is cv::gemm (double accumulation).
#include <cmath>
#include <cstdint>
#include <vector>

#include "orb_oracle.h"

namespace {

int hamming(const uint8_t* a, const uint8_t* b) {
  int d = 0;
  for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
  return d;
}

bool epipolar_ok(const oracle_keypoint& k1, const oracle_keypoint& k2, const float* F, float sigma2) {
  const float a = k1.x * F[0] + k1.y * F[3] + F[6];
  const float b = k1.x * F[1] + k1.y * F[4] + F[7];
  const float c = k1.x * F[2] + k1.y * F[5] + F[8];
  const float num = a * k2.x + b * k2.y + c;
  const float den = a * a + b * b;
  if (den == 0) return false;
  const float dsqr = num * num / den;
  return dsqr < 3.84 * sigma2;
}

int rot_bin(float a, float b) {
  float rot = a - b;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)std::round(rot * (1.0f / 30));
  if (bin == 30) bin = 0;
  return bin;
}

}  // namespace

extern "C" int oracle_search_for_triangulation(const oracle_tri_problem* P) {
  const oracle_tri_kf &K1 = P->kf1, &K2 = P->kf2;
  float C2[3];
  for (int r = 0; r < 3; r++) {  // R2w*Cw+t2w (src/ORBmatcher.cc:746-749): cv::gemm's small-matrix path
    const float t0 = P->T2w[4 * r] * P->C1w[0] + P->T2w[4 * r + 1] * P->C1w[1] + P->T2w[4 * r + 2] * P->C1w[2];
    C2[r] = (float)((double)t0 + (double)P->T2w[4 * r + 3]);
  }
  const float invz = 1.0f / C2[2];
  const float ex = P->fx * C2[0] * invz + P->cx;
  const float ey = P->fy * C2[1] * invz + P->cy;
  std::vector<int> m12(K1.n, -1);
  std::vector<int> rotHist[30];
  int nmatches = 0;
  int i = 0, j = 0;
  while (i < K1.n_nodes && j < K2.n_nodes) {  // FeatureVector merge walk
    if (K1.node_id[i] < K2.node_id[j]) { i++; continue; }
    if (K2.node_id[j] < K1.node_id[i]) { j++; continue; }
    for (int p1 = K1.node_off[i]; p1 < K1.node_off[i + 1]; p1++) {
      const int idx1 = K1.feat[p1];
      if (K1.has_mp && K1.has_mp[idx1]) continue;
      const bool bStereo1 = K1.u_right && K1.u_right[idx1] >= 0;
      if (P->only_stereo && !bStereo1) continue;
      const oracle_keypoint& kp1 = K1.keys_un[idx1];
      int bestDist = 50, bestIdx2 = -1;  // TH_LOW
      for (int p2 = K2.node_off[j]; p2 < K2.node_off[j + 1]; p2++) {
        const int idx2 = K2.feat[p2];
        if (K2.has_mp && K2.has_mp[idx2]) continue;  // vbMatched2[idx2] is always false
        const bool bStereo2 = K2.u_right && K2.u_right[idx2] >= 0;
        if (P->only_stereo && !bStereo2) continue;
        const int dist = hamming(K1.desc + 32 * (size_t)idx1, K2.desc + 32 * (size_t)idx2);
        if (dist > 50 || dist > bestDist) continue;
        const oracle_keypoint& kp2 = K2.keys_un[idx2];
        if (!bStereo1 && !bStereo2) {
          const float distex = ex - kp2.x, distey = ey - kp2.y;
          if (distex * distex + distey * distey < 100 * P->scale_factors2[kp2.octave]) continue;
        }
        if (epipolar_ok(kp1, kp2, P->F12, P->level_sigma2_2[kp2.octave])) {
          bestIdx2 = idx2;
          bestDist = dist;
        }
      }
      if (bestIdx2 >= 0) {
        m12[idx1] = bestIdx2;
        nmatches++;
        if (P->check_ori) rotHist[rot_bin(kp1.angle, K2.keys_un[bestIdx2].angle)].push_back(idx1);
      }
    }
    i++;
    j++;
  }
  if (P->check_ori) {
    int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int b = 0; b < 30; b++) {
      const int s = (int)rotHist[b].size();
      if (s > m1) {
        m3 = m2; m2 = m1; m1 = s;
        i3 = i2; i2 = i1; i1 = b;
      } else if (s > m2) {
        m3 = m2; m2 = s;
        i3 = i2; i2 = b;
      } else if (s > m3) {
        m3 = s;
        i3 = b;
      }
    }
    if (m2 < 0.1f * (float)m1) {
      i2 = -1;
      i3 = -1;
    } else if (m3 < 0.1f * (float)m1) {
      i3 = -1;
    }
    for (int b = 0; b < 30; b++) {
      if (b == i1 || b == i2 || b == i3) continue;
      for (int idx1 : rotHist[b]) {
        m12[idx1] = -1;
        nmatches--;
      }
    }
  }
  for (int k = 0; k < K1.n; k++) P->match12[k] = m12[k];
  *P->nmatches = nmatches;
  return nmatches;
}
