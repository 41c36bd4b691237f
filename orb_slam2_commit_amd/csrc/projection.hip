// projection.hip -- ORBmatcher::SearchByProjection, the three overloads run on
// every tracked frame (src/ORBmatcher.cc:46-142 local map, :1489-1646 last
// frame, :1648-1795 keyframe), the matching half of Fuse (:944-1054) and the
// loop-closing SearchByProjection(KeyFrame*, Scw, ...) (:327-440) and Fuse(KeyFrame*, Scw, ...)
// (:1094-1236, matching half), and both directions of SearchBySim3 (:1238-1487), with
// Frame::AssignFeaturesToGrid /
// GetFeaturesInArea (src/Frame.cc:254-271, 388-453) and, for the local map,
// Frame::isInFrustum (src/Frame.cc:315-375) fused in front.  One block per
// problem (a Frame plus the MapPoints projected into it), batched.
//
// The reference walks the MapPoints in order and each match it makes can
// hide a feature from every later MapPoint ("already has a MapPoint with
// observations", :90-92 / :1574-1576 / :1732-1733).  Point k's result is a
// function of the matches of points j < k only, so the sequential answer is
// the unique fixed point of
//     match_k = search(k, taken_k),  taken_k(f) = occ(f) || first_writer(f) < k
// where first_writer(f) is the smallest blocking point matched to f.  The
// block evaluates every point in parallel against the previous sweep's
// first_writer table and repeats until no match changes: after sweep s the
// first s points are final, so the loop ends, and an unchanged sweep is the
// fixed point -- bit-identical to the sequential scan, usually in 2-3 sweeps.
//
// Grid: the reference's 64x48 cells hold feature indices in ascending order
// and GetFeaturesInArea enumerates (cell x, cell y, index).  Sorting the keys
// (x*48 + y) << 13 | index makes that enumeration order the sorted position,
// and for one x the cells y0..y1 are one contiguous range.  Best/second-best
// with the reference's "first candidate wins" ties is then a min over 32-bit
// keys dist << 16 | position.
//
// Roofline: per candidate ~52 B (descriptor 32, keypoint x/y/octave 12,
// mvuRight 4, occ 1) from L2-resident frame arrays; per point 32 B descriptor
// + 16-40 B of geometry.  Latency-bound per block (a few hundred dependent
// loads per point group), so the batch is the unit of throughput.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "orbx_scratch.h"
#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_proj.h"

namespace orbx {

constexpr int PBS = 1024;         // threads per problem block
constexpr int kGroup = 16;        // lanes per MapPoint
constexpr int kCells = ORBX_GRID_COLS * ORBX_GRID_ROWS;
constexpr int kMaxF = ORBX_PROJ_MAX_FEATURES;  // 8192 = 2^13
constexpr int kThHigh = 100;

// Deterministic natural log rounded to float (same operation sequence as the
// oracle's log_det): frexp, 2*atanh series to s^25.
__device__ float log_det(float xf) {
  if (!(xf > 0.0f)) return xf == 0.0f ? -__builtin_inff() : __builtin_nanf("");
  if (__builtin_isinf(xf)) return __builtin_inff();
  int e;
  double m = __builtin_frexp((double)xf, &e);
  if (m < 0.70710678118654752440) {
    m = m * 2.0;
    e -= 1;
  }
  const double s = (m - 1.0) / (m + 1.0);
  const double s2 = s * s;
  double p = 1.0 / 25.0;
#pragma unroll
  for (int k = 23; k >= 1; k -= 2) p = p * s2 + 1.0 / (double)k;
  const double lm = 2.0 * s * p;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  return (float)((double)e * ln2_hi + ((double)e * ln2_lo + lm));
}

// MapPoint::PredictScale(dist, Frame*), src/MapPoint.cc:424-440
__device__ int predict_scale(float max_distance, float dist, float log_sf, int nlevels) {
  const float ratio = max_distance / dist;
  const float q = log_det(ratio) / log_sf;
  int n;
  if (q != q) n = 0;
  else if (q > 1e6f) n = nlevels - 1;
  else if (q < -1e6f) n = 0;
  else n = (int)__builtin_ceilf(q);
  if (n < 0) n = 0;
  else if (n >= nlevels) n = nlevels - 1;
  return n;
}

// `R*X + t` on 3x1 CV_32F Mats: cv::gemm(R, X, 1, t, 1) takes OpenCV 3.2's small-matrix path
// (matmul.cpp: flags == 0, 2 <= len <= 4): the dot product in float, left to right, then
// (float)(t0*alpha + c*beta) in double -- a correctly rounded float add of t.  (-R^T t, with
// GEMM_1_T set, is the general GEMMSingleMul<float,double> path: double accumulation, below.)
__device__ __forceinline__ void mat3x1(const float* T, const float* X, float* out) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const float t0 = T[4 * r + 0] * X[0] + T[4 * r + 1] * X[1] + T[4 * r + 2] * X[2];
    out[r] = (float)((double)t0 + (double)T[4 * r + 3]);
  }
}
// KeyFrame::GetCameraCenter (Fuse): Ow = -Rwc*tcw with Rwc a Mat -- cv::gemm's small-matrix path
__device__ __forceinline__ void camera_centre_kf(const float* T, float* Ow) {
#pragma unroll
  for (int c = 0; c < 3; c++) {
    const float t0 = T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11];
    Ow[c] = (float)((double)t0 * -1.0);
  }
}
// Frame's mOw = -mRcw.t()*mtcw: GEMM_1_T, the general GEMMSingleMul<float,double> path
__device__ __forceinline__ void camera_centre(const float* T, float* Ow) {
#pragma unroll
  for (int c = 0; c < 3; c++) {
    double s = (double)T[c] * T[3];
    s = s + (double)T[4 + c] * T[7];
    s = s + (double)T[8 + c] * T[11];
    Ow[c] = (float)(-s);
  }
}
__device__ __forceinline__ float norm3(const float* v) {
  double s = (double)v[0] * v[0];
  s = s + (double)v[1] * v[1];
  s = s + (double)v[2] * v[2];
  return (float)__builtin_sqrt(s);
}

__device__ __forceinline__ int rot_bin(float a, float b) {
  float rot = a - b;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)__builtin_roundf(rot * (1.0f / 30));
  if (bin == 30) bin = 0;
  return bin;
}

// The per-point search window (everything the reference derives before its
// candidate loop).
struct Query {
  bool active;
  float x, y, r;      // GetFeaturesInArea centre and half-size
  int min_level, max_level;
  float ur, ur_th;    // stereo check |ur - mvuRight| > ur_th (ur_th < 0: no check); FUSE: ur
  int th;             // accept bestDist <= th
};

__device__ Query setup_query(const ProjProblem& P, int i, const float* Tcw, const float* Ow, bool fwd, bool bwd) {
  Query q;
  q.active = false;
  const orbx_proj_frame& F = P.f;
  const uint8_t fl = P.flags[i];
  if (P.kind == ORBX_PROJ_LOCAL) {
    const int lvl = P.track_level[i];
    if (P.frustum ? lvl < 0 : !(fl & 1)) return q;
    if (lvl < 0 || lvl >= F.nlevels) return q;
    const float* tr = P.track + 4 * i;
    float r = tr[3] > 0.998f ? 2.5f : 4.0f;  // RadiusByViewingCos, src/ORBmatcher.cc:145-151
    if (P.th != 1.0f) r *= P.th;
    q.r = r * F.scale_factors[lvl];
    q.x = tr[0];
    q.y = tr[1];
    q.min_level = lvl - 1;
    q.max_level = lvl;
    q.ur = tr[2];
    q.ur_th = q.r;
    q.th = kThHigh;
    q.active = true;
    return q;
  }
  if (!(fl & 1)) return q;
  const float* X = P.pos + 3 * i;
  float c[3];
  if (P.kind == ORBX_PROJ_BY_SIM3) {  // one direction of SearchBySim3, src/ORBmatcher.cc:1283-1340
    float c1[3];
    mat3x1(Tcw, X, c1);          // R1w*p3Dw + t1w (the point's own KeyFrame)
    mat3x1(P.last_Tcw, c1, c);   // sR21*p3Dc1 + t21
    if (c[2] < 0.0f) return q;
    const float invz = (float)(1.0 / (double)c[2]);
    const float x = c[0] * invz, y = c[1] * invz;
    const float u = F.fx * x + F.cx, v = F.fy * y + F.cy;
    if (!(u >= F.min_x && u < F.max_x && v >= F.min_y && v < F.max_y)) return q;  // KeyFrame::IsInImage
    const float d3 = norm3(c);
    const float dmin = P.dist_minmax[2 * i], dmax = P.dist_minmax[2 * i + 1];
    if (d3 < 0.8f * dmin || d3 > 1.2f * dmax) return q;
    const int lvl = predict_scale(dmax, d3, F.log_scale_factor, F.nlevels);
    q.r = P.th * F.scale_factors[lvl];
    q.x = u;
    q.y = v;
    q.min_level = lvl - 1;
    q.max_level = lvl;
    q.ur_th = -1.0f;
    q.th = kThHigh;
    q.active = true;
    return q;
  }
  mat3x1(Tcw, X, c);
  if (P.kind == ORBX_PROJ_FUSE || P.kind == ORBX_PROJ_SIM3 || P.kind == ORBX_PROJ_FUSE_SIM3) {
    // src/ORBmatcher.cc:960-1006, :352-391, :1117-1160
    if (c[2] < 0.0f) return q;
    const float invz = P.kind == ORBX_PROJ_FUSE_SIM3 ? (float)(1.0 / (double)c[2]) : 1 / c[2];
    const float x = c[0] * invz, y = c[1] * invz;
    const float u = F.fx * x + F.cx, v = F.fy * y + F.cy;
    if (!(u >= F.min_x && u < F.max_x && v >= F.min_y && v < F.max_y)) return q;  // KeyFrame::IsInImage
    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
    const float d3 = norm3(PO);
    const float dmin = P.dist_minmax[2 * i], dmax = P.dist_minmax[2 * i + 1];
    if (d3 < 0.8f * dmin || d3 > 1.2f * dmax) return q;
    const float* Pn = P.normal + 3 * i;
    double dot = (double)PO[0] * Pn[0];
    dot = dot + (double)PO[1] * Pn[1];
    dot = dot + (double)PO[2] * Pn[2];
    if (dot < 0.5 * d3) return q;
    const int lvl = predict_scale(dmax, d3, F.log_scale_factor, F.nlevels);
    q.r = P.th * F.scale_factors[lvl];
    q.x = u;
    q.y = v;
    q.min_level = lvl - 1;  // the candidate loop's kpLevel window (:1015-1016)
    q.max_level = lvl;
    q.ur = u - F.bf * invz;
    q.ur_th = -1.0f;
    q.th = 50;  // TH_LOW
    q.active = true;
    return q;
  }
  const float invzc = (float)(1.0 / (double)c[2]);
  if (P.kind == ORBX_PROJ_LAST_FRAME && invzc < 0) return q;
  const float u = F.fx * c[0] * invzc + F.cx;
  const float v = F.fy * c[1] * invzc + F.cy;
  if (u != u || v != v) return q;  // 0 * inf: undefined in the reference
  if (u < F.min_x || u > F.max_x) return q;
  if (v < F.min_y || v > F.max_y) return q;
  q.x = u;
  q.y = v;
  if (P.kind == ORBX_PROJ_LAST_FRAME) {
    const int o = P.octave[i];
    if (o < 0 || o >= F.nlevels) return q;
    q.r = P.th * F.scale_factors[o];
    if (fwd) {
      q.min_level = o;
      q.max_level = -1;
    } else if (bwd) {
      q.min_level = 0;
      q.max_level = o;
    } else {
      q.min_level = o - 1;
      q.max_level = o + 1;
    }
    q.ur = u - F.bf * invzc;
    q.ur_th = q.r;
    q.th = kThHigh;
  } else {
    const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
    const float d3 = norm3(PO);
    const float dmin = P.dist_minmax[2 * i], dmax = P.dist_minmax[2 * i + 1];
    if (d3 < 0.8f * dmin || d3 > 1.2f * dmax) return q;
    const int lvl = predict_scale(dmax, d3, F.log_scale_factor, F.nlevels);
    q.r = P.th * F.scale_factors[lvl];
    q.min_level = lvl - 1;
    q.max_level = lvl + 1;
    q.ur_th = -1.0f;
    q.th = P.orb_dist;
  }
  q.active = true;
  return q;
}

__device__ __forceinline__ uint32_t group_min(uint32_t v) {
#pragma unroll
  for (int o = kGroup / 2; o > 0; o >>= 1) {
    const uint32_t w = __shfl_xor(v, o, kGroup);
    v = w < v ? w : v;
  }
  return v;
}

// ---- the kernel's phases as block-wide device functions (shared by the batched one-block-per-problem
// kernel and the split single-problem kernels below) ----

// the pose the points project with: Tcw, or for the Sim3 kinds [Rcw | tcw] = [sRcw | t] / scw
__device__ __forceinline__ void proj_pose(const ProjProblem& P, float* s_Tcw, int tid) {
  const orbx_proj_frame& F = P.f;
  if (tid < 16) {
    const float* S = P.Tcw_dev ? P.Tcw_dev : F.Tcw;
    if (P.kind == ORBX_PROJ_SIM3 || P.kind == ORBX_PROJ_FUSE_SIM3) {
      // Scw -> [Rcw | tcw] = [sRcw | t] / scw (src/ORBmatcher.cc:335-339): scw = sqrt(row0.dot(row0))
      // (double products summed left to right, rounded to float); Mat / double is convertTo(alpha =
      // 1/scw): x * (float)alpha + 0.0f in float.  Every one of the 16 threads derives scw itself.
      double d = (double)S[0] * S[0];
      d = d + (double)S[1] * S[1];
      d = d + (double)S[2] * S[2];
      const float a = (float)(1.0 / (double)(float)__builtin_sqrt(d));
      s_Tcw[tid] = tid < 12 ? S[tid] * a + 0.0f : (tid == 15 ? 1.0f : 0.0f);
    } else {
      s_Tcw[tid] = S[tid];
    }
  }
}

// camera centre and the last-frame direction flags (after proj_pose's writes are visible)
__device__ __forceinline__ void proj_centre(const ProjProblem& P, const float* s_Tcw, float* Ow, bool& fwd, bool& bwd) {
  if (P.kind == ORBX_PROJ_FUSE)
    camera_centre_kf(s_Tcw, Ow);  // pKF->GetCameraCenter() (src/ORBmatcher.cc:928)
  else
    camera_centre(s_Tcw, Ow);
  fwd = bwd = false;
  if (P.kind == ORBX_PROJ_LAST_FRAME) {
    float tlc[3];
    mat3x1(P.last_Tcw, Ow, tlc);  // twc = Ow
    fwd = tlc[2] > P.f.b && !P.mono;
    bwd = -tlc[2] > P.f.b && !P.mono;
  }
}

// Frame::AssignFeaturesToGrid as a sort of (cell << 13 | index): s_pos[sorted position] = feature,
// s_start[c] = first sorted position of cell c (s_keys is the sort's scratch); ends with a barrier
template <int NT>
__device__ void proj_grid(const orbx_proj_frame& F, int nF, uint32_t* s_keys, uint16_t* s_pos, int* s_start, int tid) {
  int nsort = 1;
  while (nsort < nF) nsort <<= 1;
  for (int i = tid; i < nsort; i += NT) {
    uint32_t key = 0xFFFFFFFFu;
    if (i < nF) {
      const orbx_keypoint kp = F.keys_un[i];
      const int px = (int)__builtin_roundf((kp.x - (F.grid_min_set ? F.grid_min_x : F.min_x)) * F.grid_inv_w);
      const int py = (int)__builtin_roundf((kp.y - (F.grid_min_set ? F.grid_min_y : F.min_y)) * F.grid_inv_h);
      if (px >= 0 && px < ORBX_GRID_COLS && py >= 0 && py < ORBX_GRID_ROWS)
        key = ((uint32_t)(px * ORBX_GRID_ROWS + py) << 13) | (uint32_t)i;
    }
    s_keys[i] = key;
  }
  __syncthreads();
  for (int k = 2; k <= nsort; k <<= 1) {  // bitonic sort, ascending
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < (nsort >> 1); t += NT) {
        const int lo = 2 * t - (t & (j - 1));
        const int hi = lo + j;
        const uint32_t a = s_keys[lo], b = s_keys[hi];
        const bool up = (lo & k) == 0;
        if ((a > b) == up) {
          s_keys[lo] = b;
          s_keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int c = tid; c <= kCells; c += NT) {  // s_start[c] = lower_bound(c << 13)
    const uint32_t target = (uint32_t)c << 13;
    int lo = 0, hi = nsort;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (s_keys[m] < target) lo = m + 1; else hi = m;
    }
    s_start[c] = lo;
  }
  for (int i = tid; i < nF; i += NT) s_pos[i] = (uint16_t)(s_keys[i] & 0x1FFF);
  __syncthreads();
}

// Tracking::SearchLocalPoints' isInFrustum(pMP, limit) for point i
__device__ __forceinline__ void proj_frustum(const ProjProblem& P, int i, const float* s_Tcw, const float* Ow) {
  const orbx_proj_frame& F = P.f;
  int lvl = -1;
  float* tr = P.track + 4 * i;
  if (P.flags[i] & 1) {
    const float* X = P.pos + 3 * i;
    float c[3];
    mat3x1(s_Tcw, X, c);
    if (!(c[2] < 0.0f)) {
      const float invz = 1.0f / c[2];
      const float u = F.fx * c[0] * invz + F.cx;
      const float v = F.fy * c[1] * invz + F.cy;
      if (!(u < F.min_x || u > F.max_x) && !(v < F.min_y || v > F.max_y) && u == u && v == v) {
        const float dmin = P.dist_minmax[2 * i], dmax = P.dist_minmax[2 * i + 1];
        const float PO[3] = {X[0] - Ow[0], X[1] - Ow[1], X[2] - Ow[2]};
        const float dist = norm3(PO);
        if (!(dist < 0.8f * dmin || dist > 1.2f * dmax)) {
          const float* Pn = P.normal + 3 * i;
          double dot = (double)PO[0] * Pn[0];
          dot = dot + (double)PO[1] * Pn[1];
          dot = dot + (double)PO[2] * Pn[2];
          const float vc = (float)(dot / dist);
          if (!(vc < P.view_cos_limit)) {
            lvl = predict_scale(dmax, dist, F.log_scale_factor, F.nlevels);
            tr[0] = u;
            tr[1] = v;
            tr[2] = u - F.bf * invz;
            tr[3] = vc;
          }
        }
      }
    }
  }
  P.track_level[i] = lvl;
}

struct ProjMode {
  bool local, kf, fuse, gate;
};
__device__ __forceinline__ ProjMode proj_mode(const ProjProblem& P) {
  ProjMode M;
  M.local = P.kind == ORBX_PROJ_LOCAL;
  // KEYFRAME and SIM3: any MapPoint on the feature blocks it, and every match blocks later points
  M.kf = P.kind == ORBX_PROJ_KEYFRAME || P.kind == ORBX_PROJ_SIM3;
  // no "already matched" state: one sweep (FUSE also gates candidates by reprojection error)
  M.fuse = P.kind == ORBX_PROJ_FUSE || P.kind == ORBX_PROJ_FUSE_SIM3 || P.kind == ORBX_PROJ_BY_SIM3;
  M.gate = P.kind == ORBX_PROJ_FUSE;
  return M;
}

// One point's match by a kGroup-lane group (the result is valid in every lane of the group) against
// the first-writer table fw of the previous sweep
__device__ __forceinline__ int proj_point(const ProjProblem& P, int i, int gl, const float* s_Tcw, const float* Ow,
                                          bool fwd, bool bwd, const uint16_t* s_pos, const int* s_start,
                                          const int* fw, const ProjMode& M) {
  const orbx_proj_frame& F = P.f;
  const Query q = setup_query(P, i, s_Tcw, Ow, fwd, bwd);
  int m = -1;
  if (!q.active) return m;
  uint64_t dq[4];
  {
    const uint64_t* d = (const uint64_t*)(P.desc + (size_t)i * 32);
    dq[0] = d[0]; dq[1] = d[1]; dq[2] = d[2]; dq[3] = d[3];
  }
  uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
  int x0 = 0, x1 = -1, y0 = 0, y1 = -1;
  {  // Frame::GetFeaturesInArea cell range, src/Frame.cc:395-413
    x0 = max(0, (int)__builtin_floorf((q.x - F.min_x - q.r) * F.grid_inv_w));
    x1 = min(ORBX_GRID_COLS - 1, (int)__builtin_ceilf((q.x - F.min_x + q.r) * F.grid_inv_w));
    y0 = max(0, (int)__builtin_floorf((q.y - F.min_y - q.r) * F.grid_inv_h));
    y1 = min(ORBX_GRID_ROWS - 1, (int)__builtin_ceilf((q.y - F.min_y + q.r) * F.grid_inv_h));
    if (x0 >= ORBX_GRID_COLS || x1 < 0 || y0 >= ORBX_GRID_ROWS || y1 < 0) x1 = x0 - 1;
  }
  const bool check = q.min_level > 0 || q.max_level >= 0;
  for (int ix = x0; ix <= x1; ix++) {
    const int c0 = ix * ORBX_GRID_ROWS;
    const int pend = s_start[c0 + y1 + 1];
    for (int p = s_start[c0 + y0] + gl; p < pend; p += kGroup) {
      const int idx = s_pos[p];
      const orbx_keypoint& kp = F.keys_un[idx];
      const int oct = kp.octave;
      if (check && (oct < q.min_level || (q.max_level >= 0 && oct > q.max_level))) continue;
      const float dx = kp.x - q.x, dy = kp.y - q.y;
      if (!(__builtin_fabsf(dx) < q.r && __builtin_fabsf(dy) < q.r)) continue;
      if (M.gate) {  // reprojection error gate, src/ORBmatcher.cc:1018-1042
        const float isg = F.inv_level_sigma2[oct];
        const float urf = F.u_right ? F.u_right[idx] : -1.0f;
        const float ex = q.x - kp.x, ey = q.y - kp.y;
        if (urf >= 0) {
          const float er = q.ur - urf;
          const float e2 = ex * ex + ey * ey + er * er;
          if (e2 * isg > 7.8) continue;
        } else {
          const float e2 = ex * ex + ey * ey;
          if (e2 * isg > 5.99) continue;
        }
      } else if (!M.fuse) {
        const int o = F.occ ? F.occ[idx] : 0;
        if ((M.kf ? o != 0 : o == 2) || fw[idx] < i) continue;
      }
      if (q.ur_th >= 0.0f && F.u_right) {
        const float urf = F.u_right[idx];
        if (urf > 0 && __builtin_fabsf(q.ur - urf) > q.ur_th) continue;
      }
      const uint64_t* d = (const uint64_t*)(F.desc + (size_t)idx * 32);
      const uint64_t x[4] = {d[0], d[1], d[2], d[3]};
      const uint32_t key = ((uint32_t)hamming256(dq, x) << 16) | (uint32_t)p;
      if (key < m1) {
        m2 = m1;
        m1 = key;
      } else if (key < m2) {
        m2 = key;
      }
    }
  }
  const uint32_t b1 = group_min(m1);
  const uint32_t b2 = group_min(m1 == b1 ? m2 : m1);
  if (b1 != 0xFFFFFFFFu) {
    const int d1 = (int)(b1 >> 16);
    if (d1 <= q.th) {
      const int i1 = s_pos[b1 & 0xFFFF];
      bool ok = true;
      if (M.local) {  // ratio only when best and second share a level, src/ORBmatcher.cc:127-131
        const int l1 = F.keys_un[i1].octave;
        const int l2 = b2 == 0xFFFFFFFFu ? -1 : F.keys_un[s_pos[b2 & 0xFFFF]].octave;
        const int d2 = b2 == 0xFFFFFFFFu ? 256 : (int)(b2 >> 16);
        if (l1 == l2 && (float)d1 > P.nnratio * (float)d2) ok = false;
      }
      if (ok) m = i1;
    }
  }
  return m;
}

// The sweeps to the sequential fixed point inside one block, from sweep `first` on, with the
// first-writer table s_fw already holding sweep `first`'s input
template <int NT>
__device__ void proj_sweeps(const ProjProblem& P, int nF, int nP, const float* s_Tcw, const float* Ow, bool fwd,
                            bool bwd, const uint16_t* s_pos, const int* s_start, int* s_fw, int* s_changed,
                            int first, int tid) {
  const ProjMode M = proj_mode(P);
  const int g = tid / kGroup, gl = tid % kGroup;
  constexpr int kGroups = NT / kGroup;
  for (int sweep = first; sweep <= nP + 1; sweep++) {
    if (tid == 0) *s_changed = 0;
    __syncthreads();
    int changed = 0;
    for (int i = g; i < nP; i += kGroups) {
      const int m = proj_point(P, i, gl, s_Tcw, Ow, fwd, bwd, s_pos, s_start, s_fw, M);
      if (gl == 0) {
        if (sweep == 0 || P.point_match[i] != m) changed = 1;
        P.point_match[i] = m;
      }
    }
    if (changed) *s_changed = 1;
    __threadfence_block();
    __syncthreads();
    if (!*s_changed || M.fuse) break;
    // first blocking writer per feature from this sweep's matches
    for (int f = tid; f < nF; f += NT) s_fw[f] = INT_MAX;
    __syncthreads();
    for (int i = tid; i < nP; i += NT) {
      const int m = P.point_match[i];
      if (m >= 0 && (M.kf || (P.flags[i] & 2))) atomicMin(&s_fw[m], i);
    }
    __syncthreads();
  }
}

// Final occupant (last writer), rotation consistency (ComputeThreeMaxima), frame_out and the count
template <int NT>
__device__ void proj_final(const ProjProblem& P, int nF, int nP, int* s_fw, int* s_hist, int* s_sel, int* s_count,
                           int* s_drop, int tid) {
  const orbx_proj_frame& F = P.f;
  const ProjMode M = proj_mode(P);
  for (int f = tid; f < nF; f += NT) s_fw[f] = -1;
  if (tid < 32) s_hist[tid] = 0;
  if (tid == 0) {
    *s_count = 0;
    *s_drop = 0;
  }
  __syncthreads();
  const bool rot = !M.local && !M.fuse && P.kind != ORBX_PROJ_SIM3 && P.check_ori;
  int cnt = 0;
  for (int i = tid; i < nP; i += NT) {
    const int m = P.point_match[i];
    if (m < 0) continue;
    cnt++;
    atomicMax(&s_fw[m], i);
    if (rot) atomicAdd(&s_hist[rot_bin(P.angle[i], F.keys_un[m].angle)], 1);
  }
  atomicAdd(s_count, cnt);
  __syncthreads();
  if (rot && tid == 0) {  // ComputeThreeMaxima, src/ORBmatcher.cc:1797-1839
    int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int b = 0; b < 30; b++) {
      const int s = s_hist[b];
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
    s_sel[0] = i1;
    s_sel[1] = i2;
    s_sel[2] = i3;
  }
  __syncthreads();
  if (rot) {
    int drop = 0;
    for (int i = tid; i < nP; i += NT) {
      const int m = P.point_match[i];
      if (m < 0) continue;
      const int b = rot_bin(P.angle[i], F.keys_un[m].angle);
      if (b != s_sel[0] && b != s_sel[1] && b != s_sel[2]) {
        s_fw[m] = -2;  // mvpMapPoints[bestIdx2] = NULL
        drop++;
      }
    }
    atomicAdd(s_drop, drop);
    __syncthreads();
  }
  for (int f = tid; f < nF; f += NT) P.frame_out[f] = s_fw[f];
  if (tid == 0) *P.nmatches = *s_count - *s_drop;
}

__device__ __forceinline__ int proj_nF(const ProjProblem& P) {
  return P.f_n_dev ? min(max(*P.f_n_dev, 0), P.f.n) : P.f.n;
}
__device__ __forceinline__ int proj_nP(const ProjProblem& P) {
  return P.n_points_dev ? min(max(*P.n_points_dev, 0), P.n_points) : P.n_points;
}

// One block per problem (batches: the chip fills with problems)
__global__ __launch_bounds__(PBS) void k_search_by_projection(const ProjProblem* __restrict__ probs) {
  __shared__ uint32_t s_keys[kMaxF];  // grid sort keys, then first-writer / final occupant table
  __shared__ uint16_t s_pos[kMaxF];   // sorted position -> feature index
  __shared__ int s_start[kCells + 1];
  __shared__ int s_hist[32];
  __shared__ int s_sel[3];
  __shared__ int s_changed, s_count, s_drop;
  __shared__ float s_Tcw[16];
  const ProjProblem& P = probs[blockIdx.x];
  const int tid = threadIdx.x;
  if (P.gate && !(*P.gate < P.gate_below)) return;  // block-uniform: the problem is skipped whole
  const int nF = proj_nF(P), nP = proj_nP(P);
  proj_pose(P, s_Tcw, tid);
  proj_grid<PBS>(P.f, nF, s_keys, s_pos, s_start, tid);
  int* s_fw = (int*)s_keys;
  float Ow[3];
  bool fwd, bwd;
  proj_centre(P, s_Tcw, Ow, fwd, bwd);
  if (P.kind == ORBX_PROJ_LOCAL && P.frustum) {
    for (int i = tid; i < nP; i += PBS) proj_frustum(P, i, s_Tcw, Ow);
    __threadfence_block();
  }
  for (int i = tid; i < nF; i += PBS) s_fw[i] = INT_MAX;
  __syncthreads();
  proj_sweeps<PBS>(P, nF, nP, s_Tcw, Ow, fwd, bwd, s_pos, s_start, s_fw, &s_changed, 0, tid);
  proj_final<PBS>(P, nF, nP, s_fw, s_hist, s_sel, &s_count, &s_drop, tid);
}

// ---- one problem split over many blocks (the host C-ABI's single call) ----
// A single problem in one block keeps one CU busy for the whole call (1 ms at 2,000 features /
// 3,000 points).  Split: k_proj_split_prep builds the grid once into global scratch (block 0) and
// runs isInFrustum over all blocks; each sweep is one launch of kProjSplitBlocks blocks, every block a
// slice of the points against the previous sweep's first-writer table (triple-buffered in global
// memory: sweep s reads fw[s % 3], takes atomicMin into fw[(s+1) % 3], clears fw[(s+2) % 3]); a sweep
// whose predecessor changed nothing returns at once.  k_proj_split_final (one block) finishes any
// sweeps still needed in the single-block way, then the final phase.  Same fixed point, so the
// same answer as k_search_by_projection bit for bit.
constexpr int kProjSplitSweeps = 3;  // sweep launches before the final kernel takes over
struct ProjSplit {
  uint16_t* pos;   // [kMaxF]
  int* start;      // [kCells + 1]
  int* fw;         // [3][kMaxF]
  int* changed;    // [kProjSplitSweeps]
};
// scratch bytes of one split problem (ProjSplit), 256-B aligned parts; problem z of a launch
// (blockIdx.z, the problems of one host call: SearchBySim3's two directions) at z * kProjSplitBytes
constexpr size_t kProjSplitBytes = 2 * kMaxF + 256 + (kCells + 1) * 4 + 256 + 3 * (size_t)kMaxF * 4 + 256 + 256;
__host__ __device__ inline ProjSplit proj_split_at(uint8_t* d) {
  ProjSplit S;
  S.pos = (uint16_t*)d;
  S.start = (int*)(d + 2 * kMaxF + 256);
  S.fw = (int*)(d + 2 * kMaxF + 256 + (kCells + 1) * 4 + 256);
  S.changed = (int*)(d + 2 * kMaxF + 256 + (kCells + 1) * 4 + 256 + 3 * (size_t)kMaxF * 4 + 256);
  return S;
}

__global__ __launch_bounds__(PBS) void k_proj_split_prep(const ProjProblem* __restrict__ probs, uint8_t* scratch) {
  __shared__ uint32_t s_keys[kMaxF];
  __shared__ uint16_t s_pos[kMaxF];
  __shared__ int s_start[kCells + 1];
  __shared__ float s_Tcw[16];
  const ProjProblem& P = probs[blockIdx.z];
  const ProjSplit S = proj_split_at(scratch + blockIdx.z * kProjSplitBytes);
  const int tid = threadIdx.x, nF = proj_nF(P), nP = proj_nP(P);
  const int gt = blockIdx.x * PBS + tid, gs = gridDim.x * PBS;
  for (int f = gt; f < nF; f += gs) {
    S.fw[f] = INT_MAX;
    S.fw[kMaxF + f] = INT_MAX;
  }
  if (gt < kProjSplitSweeps) S.changed[gt] = 0;
  if (P.kind == ORBX_PROJ_LOCAL && P.frustum) {
    proj_pose(P, s_Tcw, tid);
    __syncthreads();
    float Ow[3];
    bool fwd, bwd;
    proj_centre(P, s_Tcw, Ow, fwd, bwd);
    for (int i = gt; i < nP; i += gs) proj_frustum(P, i, s_Tcw, Ow);
  }
  if (blockIdx.x == 0) {
    proj_grid<PBS>(P.f, nF, s_keys, s_pos, s_start, tid);
    for (int i = tid; i < nF; i += PBS) S.pos[i] = s_pos[i];
    for (int c = tid; c <= kCells; c += PBS) S.start[c] = s_start[c];
  }
}

__global__ __launch_bounds__(PBS) void k_proj_split_sweep(const ProjProblem* __restrict__ probs, uint8_t* scratch,
                                                          int sweep) {
  __shared__ int s_fw[kMaxF];
  __shared__ uint16_t s_pos[kMaxF];
  __shared__ int s_start[kCells + 1];
  __shared__ float s_Tcw[16];
  const ProjProblem& P = probs[blockIdx.z];
  const ProjSplit S = proj_split_at(scratch + blockIdx.z * kProjSplitBytes);
  if (sweep > 0 && !__atomic_load_n(&S.changed[sweep - 1], __ATOMIC_RELAXED)) return;  // converged
  const int tid = threadIdx.x, nF = proj_nF(P), nP = proj_nP(P);
  const int* fwr = S.fw + (sweep % 3) * kMaxF;
  int* fwn = S.fw + ((sweep + 1) % 3) * kMaxF;
  int* fwc = S.fw + ((sweep + 2) % 3) * kMaxF;
  proj_pose(P, s_Tcw, tid);
  for (int i = tid; i < nF; i += PBS) {
    s_fw[i] = fwr[i];
    s_pos[i] = S.pos[i];
  }
  for (int c = tid; c <= kCells; c += PBS) s_start[c] = S.start[c];
  const int gt = blockIdx.x * PBS + tid, gs = gridDim.x * PBS;
  for (int f = gt; f < nF; f += gs) fwc[f] = INT_MAX;
  __syncthreads();
  float Ow[3];
  bool fwd, bwd;
  proj_centre(P, s_Tcw, Ow, fwd, bwd);
  const ProjMode M = proj_mode(P);
  const int g = blockIdx.x * (PBS / kGroup) + tid / kGroup, gl = tid % kGroup, G = gridDim.x * (PBS / kGroup);
  int changed = 0;
  for (int i = g; i < nP; i += G) {
    const int m = proj_point(P, i, gl, s_Tcw, Ow, fwd, bwd, s_pos, s_start, s_fw, M);
    if (gl == 0) {
      if (sweep == 0 || P.point_match[i] != m) changed = 1;
      P.point_match[i] = m;
      if (!M.fuse && m >= 0 && (M.kf || (P.flags[i] & 2))) atomicMin(&fwn[m], i);
    }
  }
  if (changed) S.changed[sweep] = 1;
}

__global__ __launch_bounds__(PBS) void k_proj_split_final(const ProjProblem* __restrict__ probs, uint8_t* scratch) {
  __shared__ int s_fw[kMaxF];
  __shared__ uint16_t s_pos[kMaxF];
  __shared__ int s_start[kCells + 1];
  __shared__ int s_hist[32];
  __shared__ int s_sel[3];
  __shared__ int s_changed, s_count, s_drop;
  __shared__ float s_Tcw[16];
  const ProjProblem& P = probs[blockIdx.z];
  const ProjSplit S = proj_split_at(scratch + blockIdx.z * kProjSplitBytes);
  const int tid = threadIdx.x, nF = proj_nF(P), nP = proj_nP(P);
  const ProjMode M = proj_mode(P);
  // the split sweeps stop at kProjSplitSweeps; a problem still changing goes on here, from the
  // state they left (point_match of the last sweep, its first writers in fw[kProjSplitSweeps % 3])
  if (!M.fuse && S.changed[kProjSplitSweeps - 1]) {  // block-uniform
    proj_pose(P, s_Tcw, tid);
    const int* fwr = S.fw + (kProjSplitSweeps % 3) * kMaxF;
    for (int i = tid; i < nF; i += PBS) {
      s_fw[i] = fwr[i];
      s_pos[i] = S.pos[i];
    }
    for (int c = tid; c <= kCells; c += PBS) s_start[c] = S.start[c];
    __syncthreads();
    float Ow[3];
    bool fwd, bwd;
    proj_centre(P, s_Tcw, Ow, fwd, bwd);
    proj_sweeps<PBS>(P, nF, nP, s_Tcw, Ow, fwd, bwd, s_pos, s_start, s_fw, &s_changed, kProjSplitSweeps, tid);
  }
  proj_final<PBS>(P, nF, nP, s_fw, s_hist, s_sel, &s_count, &s_drop, tid);
}

// ---- ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:442-587) ----
// The reference walks F1's level-0 keypoints in order; keypoint i1 skips every candidate i2 whose
// vMatchedDistance <= dist, and an accepted match takes i2 from its earlier holder (vnMatches21).
// vMatchedDistance before i1's turn is md_i1(f) = min{dist_j : j < i1 accepted at f} (a later
// acceptance at f needs a strictly smaller distance), so i1's choice is a function of the choices of
// j < i1 only and the sweeps of k_search_by_projection reach the sequential answer: every sweep
// evaluates all keypoints against the previous sweep's choices, held as a sorted (f << 13 | j) list
// with per-feature prefix minima of the distance (md lookup = one binary search, only for features
// with a chooser), until no choice changes.  The last chooser of a feature keeps it; the rotation
// histogram counts every acceptance (dropped ones included), as rotHist does.
// Dynamic LDS: sort keys (max(pow2(N1), pow2(N2)) x 4 B), cell starts, F2 grid positions, prefix
// minima (pow2(N1) x 2 B), has-chooser bitmap.
constexpr int IBS = 1024;
constexpr int kInitMaxHeld = kMaxF / IBS;  // sorted-list positions per thread in the final pass

__host__ __device__ inline int pow2_at_least(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}
__host__ __device__ inline size_t init_smem_bytes(int n1, int n2) {
  const int ns1 = pow2_at_least(n1), ns2 = pow2_at_least(n2), nk = ns1 > ns2 ? ns1 : ns2;
  return (size_t)nk * 4 + (size_t)(kCells + 1) * 4 + (size_t)((n2 + 1) & ~1) * 2 + (size_t)ns1 * 2 +
         (size_t)((n2 + 31) / 32) * 4;
}

template <class T>
__device__ void bitonic_asc(T* k, int n) {
  for (int size = 2; size <= n; size <<= 1)
    for (int j = size >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < (n >> 1); t += blockDim.x) {
        const int lo = 2 * t - (t & (j - 1)), hi = lo + j;
        const T a = k[lo], b = k[hi];
        if ((a > b) == ((lo & size) == 0)) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __syncthreads();
    }
}

// ---- its phases as block-wide device functions (the one-block kernel and the split single call) ----
struct InitLds {  // dynamic LDS views
  uint32_t* keys;   // grid sort scratch, then the sorted chooser list (ns1)
  int* start;       // [kCells + 1]
  uint16_t* pos;    // F2 sorted positions
  uint16_t* pmin;   // per list position: prefix minimum of the distance over the feature's choosers
  uint32_t* has;    // feature has a chooser
};
__device__ __forceinline__ InitLds init_lds(uint8_t* ismem, int n1, int n2) {
  const int ns1 = pow2_at_least(n1), ns2 = pow2_at_least(n2), nk = ns1 > ns2 ? ns1 : ns2;
  InitLds S;
  S.keys = (uint32_t*)ismem;
  S.start = (int*)(S.keys + nk);
  S.pos = (uint16_t*)(S.start + kCells + 1);
  S.pmin = S.pos + ((n2 + 1) & ~1);
  S.has = (uint32_t*)(S.pmin + ns1);
  return S;
}

// F2's level-0 keypoints into the grid (GetFeaturesInArea(x, y, w, 0, 0) sees only those)
__device__ void init_grid(const orbx_init_problem& P, const InitLds& S, int tid) {
  const orbx_proj_frame& F2 = P.f2;
  const int n2 = F2.n, ns2 = pow2_at_least(n2);
  for (int i = tid; i < ns2; i += IBS) {
    uint32_t key = 0xFFFFFFFFu;
    if (i < n2) {
      const orbx_keypoint kp = F2.keys_un[i];
      const int px = (int)__builtin_roundf((kp.x - (F2.grid_min_set ? F2.grid_min_x : F2.min_x)) * F2.grid_inv_w);
      const int py = (int)__builtin_roundf((kp.y - (F2.grid_min_set ? F2.grid_min_y : F2.min_y)) * F2.grid_inv_h);
      if (kp.octave == 0 && px >= 0 && px < ORBX_GRID_COLS && py >= 0 && py < ORBX_GRID_ROWS)
        key = ((uint32_t)(px * ORBX_GRID_ROWS + py) << 13) | (uint32_t)i;
    }
    S.keys[i] = key;
  }
  __syncthreads();
  bitonic_asc(S.keys, ns2);
  for (int c = tid; c <= kCells; c += IBS) {
    const uint32_t target = (uint32_t)c << 13;
    int lo = 0, hi = ns2;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (S.keys[m] < target) lo = m + 1; else hi = m;
    }
    S.start[c] = lo;
  }
  for (int i = tid; i < n2; i += IBS) S.pos[i] = (uint16_t)(S.keys[i] & 0x1FFF);
  __syncthreads();
}

// F1 keypoint i's choice (dist << 16 | i2, or -1) by a kGroup-lane group against the previous
// sweep's chooser list
__device__ __forceinline__ int init_point(const orbx_init_problem& P, const InitLds& S, int i, int gl) {
  const orbx_proj_frame& F1 = P.f1;
  const orbx_proj_frame& F2 = P.f2;
  const int ns1 = pow2_at_least(F1.n);
  const float r = (float)P.window;
  int m = -1;
  if (F1.keys_un[i].octave != 0) return m;
  const float x = P.prev_matched[2 * i], y = P.prev_matched[2 * i + 1];
  int x0 = max(0, (int)__builtin_floorf((x - F2.min_x - r) * F2.grid_inv_w));
  const int x1 = min(ORBX_GRID_COLS - 1, (int)__builtin_ceilf((x - F2.min_x + r) * F2.grid_inv_w));
  const int y0 = max(0, (int)__builtin_floorf((y - F2.min_y - r) * F2.grid_inv_h));
  const int y1 = min(ORBX_GRID_ROWS - 1, (int)__builtin_ceilf((y - F2.min_y + r) * F2.grid_inv_h));
  if (x0 >= ORBX_GRID_COLS || x1 < 0 || y0 >= ORBX_GRID_ROWS || y1 < 0) x0 = x1 + 1;
  uint64_t dq[4];
  {
    const uint64_t* d = (const uint64_t*)(F1.desc + (size_t)i * 32);
    dq[0] = d[0]; dq[1] = d[1]; dq[2] = d[2]; dq[3] = d[3];
  }
  uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
  for (int ix = x0; ix <= x1; ix++) {
    const int c0 = ix * ORBX_GRID_ROWS;
    const int pend = S.start[c0 + y1 + 1];
    for (int p = S.start[c0 + y0] + gl; p < pend; p += kGroup) {
      const int idx = S.pos[p];
      const orbx_keypoint& kp = F2.keys_un[idx];
      if (!(__builtin_fabsf(kp.x - x) < r && __builtin_fabsf(kp.y - y) < r)) continue;
      const uint64_t* d = (const uint64_t*)(F2.desc + (size_t)idx * 32);
      const uint64_t dd[4] = {d[0], d[1], d[2], d[3]};
      const int dist = hamming256(dq, dd);
      if ((S.has[idx >> 5] >> (idx & 31)) & 1) {  // vMatchedDistance[idx] <= dist: skip
        const uint32_t key = ((uint32_t)idx << 13) | (uint32_t)i;
        int lo = 0, hi = ns1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (S.keys[mid] < key) lo = mid + 1; else hi = mid;
        }
        if (lo > 0 && (S.keys[lo - 1] >> 13) == (uint32_t)idx && (int)S.pmin[lo - 1] <= dist) continue;
      }
      const uint32_t k = ((uint32_t)dist << 16) | (uint32_t)p;
      if (k < m1) {
        m2 = m1;
        m1 = k;
      } else if (k < m2) {
        m2 = k;
      }
    }
  }
  const uint32_t b1 = group_min(m1);
  const uint32_t b2 = group_min(m1 == b1 ? m2 : m1);
  if (b1 != 0xFFFFFFFFu) {
    const int d1 = (int)(b1 >> 16);
    const int d2 = b2 == 0xFFFFFFFFu ? INT_MAX : (int)(b2 >> 16);
    if (d1 <= 50 && (float)d1 < (float)d2 * P.nnratio) m = (d1 << 16) | (int)S.pos[b1 & 0xFFFF];
  }
  return m;
}

// the choosers of the current choices, sorted by (feature, keypoint), with per-feature prefix minima
__device__ void init_list(const orbx_init_problem& P, const InitLds& S, int tid) {
  const int n1 = P.f1.n, n2 = P.f2.n, ns1 = pow2_at_least(n1);
  const int32_t* choice = P.match12;
  for (int p = tid; p < ns1; p += IBS) {
    uint32_t key = 0xFFFFFFFFu;
    if (p < n1) {
      const int c = choice[p];
      if (c >= 0) key = ((uint32_t)(c & 0xFFFF) << 13) | (uint32_t)p;
    }
    S.keys[p] = key;
  }
  for (int w = tid; w < (n2 + 31) / 32; w += IBS) S.has[w] = 0;
  __syncthreads();
  bitonic_asc(S.keys, ns1);
  for (int p = tid; p < ns1; p += IBS) {
    const uint32_t key = S.keys[p];
    if (key == 0xFFFFFFFFu) continue;
    const uint32_t f = key >> 13;
    int d = choice[key & 0x1FFF] >> 16;
    for (int q = p - 1; q >= 0 && (S.keys[q] >> 13) == f; q--) d = min(d, choice[S.keys[q] & 0x1FFF] >> 16);
    S.pmin[p] = (uint16_t)d;
    atomicOr(&S.has[f >> 5], 1u << (f & 31));
  }
  __syncthreads();
}

// sweeps inside one block from sweep `first` on (S holds the list of the choices before it)
__device__ void init_sweeps(const orbx_init_problem& P, const InitLds& S, int* s_changed, int first, int tid) {
  const int n1 = P.f1.n;
  int32_t* choice = P.match12;
  const int g = tid / kGroup, gl = tid % kGroup;
  constexpr int kGroups = IBS / kGroup;
  for (int sweep = first; sweep <= n1 + 1; sweep++) {
    if (tid == 0) *s_changed = 0;
    __syncthreads();
    int changed = 0;
    for (int i = g; i < n1; i += kGroups) {
      const int m = init_point(P, S, i, gl);
      if (gl == 0) {
        if (choice[i] != m) changed = 1;
        choice[i] = m;
      }
    }
    if (changed) *s_changed = 1;
    __threadfence_block();
    __syncthreads();
    if (!*s_changed) break;
    init_list(P, S, tid);
  }
}

// final: a feature's last chooser keeps it; rotation histogram over every acceptance (S.keys holds
// the final choices' list: the last sweep changed nothing)
__device__ void init_final(const orbx_init_problem& P, const InitLds& S, int* s_hist, int* s_sel, int* s_count,
                           int tid) {
  const orbx_proj_frame& F1 = P.f1;
  const orbx_proj_frame& F2 = P.f2;
  const int ns1 = pow2_at_least(F1.n);
  const int32_t* choice = P.match12;
  int held_i[kInitMaxHeld], held_fin[kInitMaxHeld], held_bin[kInitMaxHeld];
  if (tid == 0) *s_count = 0;
  if (tid < 32) s_hist[tid] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kInitMaxHeld; k++) {
    const int p = tid + k * IBS;
    held_i[k] = -1;
    held_fin[k] = -1;
    held_bin[k] = -1;
    if (p < ns1) {
      const uint32_t key = S.keys[p];
      if (key != 0xFFFFFFFFu) {
        const int i = (int)(key & 0x1FFF), i2 = choice[i] & 0xFFFF;
        const bool last = p + 1 == ns1 || (S.keys[p + 1] >> 13) != (key >> 13);
        held_i[k] = i;
        held_fin[k] = last ? i2 : -1;
        if (P.check_ori) {
          held_bin[k] = rot_bin(F1.keys_un[i].angle, F2.keys_un[i2].angle);
          atomicAdd(&s_hist[held_bin[k]], 1);
        }
      }
    }
  }
  __syncthreads();
  if (P.check_ori && tid == 0) {  // ComputeThreeMaxima
    int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
    for (int b = 0; b < 30; b++) {
      const int sz = s_hist[b];
      if (sz > m1) {
        m3 = m2; m2 = m1; m1 = sz;
        i3 = i2; i2 = i1; i1 = b;
      } else if (sz > m2) {
        m3 = m2; m2 = sz;
        i3 = i2; i2 = b;
      } else if (sz > m3) {
        m3 = sz;
        i3 = b;
      }
    }
    if (m2 < 0.1f * (float)m1) {
      i2 = -1;
      i3 = -1;
    } else if (m3 < 0.1f * (float)m1) {
      i3 = -1;
    }
    s_sel[0] = i1;
    s_sel[1] = i2;
    s_sel[2] = i3;
  }
  __syncthreads();
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < kInitMaxHeld; k++) {
    const int i = held_i[k];
    if (i < 0) continue;
    int out = held_fin[k];
    if (P.check_ori && held_bin[k] != s_sel[0] && held_bin[k] != s_sel[1] && held_bin[k] != s_sel[2]) out = -1;
    P.match12[i] = out;
    if (out >= 0) {
      const orbx_keypoint kp = F2.keys_un[out];
      P.prev_matched[2 * i] = kp.x;
      P.prev_matched[2 * i + 1] = kp.y;
      cnt++;
    }
  }
  atomicAdd(s_count, cnt);
  __syncthreads();
  if (tid == 0) *P.nmatches = *s_count;
}

// no chooser before the first sweep
__device__ void init_clear(const orbx_init_problem& P, const InitLds& S, int tid) {
  const int n1 = P.f1.n, n2 = P.f2.n, ns1 = pow2_at_least(n1);
  for (int p = tid; p < ns1; p += IBS) S.keys[p] = 0xFFFFFFFFu;
  for (int w = tid; w < (n2 + 31) / 32; w += IBS) S.has[w] = 0;
  for (int i = tid; i < n1; i += IBS) P.match12[i] = -1;
  __threadfence_block();
  __syncthreads();
}

__global__ __launch_bounds__(IBS) void k_search_for_initialization(const orbx_init_problem* __restrict__ probs) {
  extern __shared__ __align__(16) uint8_t ismem[];
  __shared__ int s_changed, s_count;
  __shared__ int s_hist[32], s_sel[3];
  const orbx_init_problem& P = probs[blockIdx.x];
  const int tid = threadIdx.x;
  const InitLds S = init_lds(ismem, P.f1.n, P.f2.n);
  init_grid(P, S, tid);
  init_clear(P, S, tid);
  init_sweeps(P, S, &s_changed, 0, tid);
  init_final(P, S, s_hist, s_sel, &s_count, tid);
}

// ---- one problem over many blocks (the host single call): the F2 grid once (k_init_split_prep,
// one block), each sweep one launch over kInitSplitBlocks-sized slices of F1 against the chooser
// list in global memory, the list of a changed sweep rebuilt by one block (k_init_split_list); after
// kInitSplitSweeps sweeps k_init_split_final (one block) goes on in the single-block way where the
// choices still change, then the final phase.  Same fixed point: the same answer bit for bit.
constexpr int kInitSplitSweeps = 3;
struct InitSplit {
  uint32_t* keys;   // [kMaxF] the chooser list
  uint16_t* pmin;   // [kMaxF]
  uint32_t* has;    // [kMaxF / 32]
  uint16_t* pos;    // [kMaxF]
  int* start;       // [kCells + 1]
  int* changed;     // [kInitSplitSweeps]
};
constexpr size_t kInitSplitBytes = 4 * (size_t)kMaxF + 2 * kMaxF + kMaxF / 8 + 2 * kMaxF + 4 * (kCells + 1) + 64 + 6 * 256;
inline InitSplit init_split_at(uint8_t* d) {
  size_t o = 0;
  auto take = [&](size_t b) {
    uint8_t* p = d + o;
    o += (b + 255) & ~(size_t)255;
    return p;
  };
  InitSplit S;
  S.keys = (uint32_t*)take(4 * (size_t)kMaxF);
  S.pmin = (uint16_t*)take(2 * kMaxF);
  S.has = (uint32_t*)take(kMaxF / 8);
  S.pos = (uint16_t*)take(2 * kMaxF);
  S.start = (int*)take(4 * (kCells + 1));
  S.changed = (int*)take(64);
  return S;
}
// LDS view S <- global state G (the grid; the list when `list`)
__device__ void init_load(const orbx_init_problem& P, const InitLds& S, const InitSplit& G, bool list, int tid) {
  const int n1 = P.f1.n, n2 = P.f2.n, ns1 = pow2_at_least(n1);
  for (int c = tid; c <= kCells; c += IBS) S.start[c] = G.start[c];
  for (int i = tid; i < n2; i += IBS) S.pos[i] = G.pos[i];
  if (list) {
    for (int p = tid; p < ns1; p += IBS) {
      S.keys[p] = G.keys[p];
      S.pmin[p] = G.pmin[p];
    }
    for (int w = tid; w < (n2 + 31) / 32; w += IBS) S.has[w] = G.has[w];
  }
  __syncthreads();
}
__device__ void init_store_list(const orbx_init_problem& P, const InitLds& S, const InitSplit& G, int tid) {
  const int n1 = P.f1.n, n2 = P.f2.n, ns1 = pow2_at_least(n1);
  for (int p = tid; p < ns1; p += IBS) {
    G.keys[p] = S.keys[p];
    G.pmin[p] = S.pmin[p];
  }
  for (int w = tid; w < (n2 + 31) / 32; w += IBS) G.has[w] = S.has[w];
}

__global__ __launch_bounds__(IBS) void k_init_split_prep(const orbx_init_problem* __restrict__ probs, InitSplit G) {
  extern __shared__ __align__(16) uint8_t ismem[];
  const orbx_init_problem& P = probs[0];
  const int tid = threadIdx.x;
  const InitLds S = init_lds(ismem, P.f1.n, P.f2.n);
  init_grid(P, S, tid);
  for (int c = tid; c <= kCells; c += IBS) G.start[c] = S.start[c];
  for (int i = tid; i < P.f2.n; i += IBS) G.pos[i] = S.pos[i];
  init_clear(P, S, tid);
  init_store_list(P, S, G, tid);
  if (tid < kInitSplitSweeps) G.changed[tid] = 0;
}

__global__ __launch_bounds__(IBS) void k_init_split_sweep(const orbx_init_problem* __restrict__ probs, InitSplit G,
                                                          int sweep) {
  extern __shared__ __align__(16) uint8_t ismem[];
  const orbx_init_problem& P = probs[0];
  if (sweep > 0 && !G.changed[sweep - 1]) return;  // converged
  const int tid = threadIdx.x;
  const InitLds S = init_lds(ismem, P.f1.n, P.f2.n);
  init_load(P, S, G, true, tid);
  int32_t* choice = P.match12;
  const int g = blockIdx.x * (IBS / kGroup) + tid / kGroup, gl = tid % kGroup, NG = gridDim.x * (IBS / kGroup);
  int changed = 0;
  for (int i = g; i < P.f1.n; i += NG) {
    const int m = init_point(P, S, i, gl);
    if (gl == 0) {
      if (choice[i] != m) changed = 1;
      choice[i] = m;
    }
  }
  if (changed) G.changed[sweep] = 1;
}

__global__ __launch_bounds__(IBS) void k_init_split_list(const orbx_init_problem* __restrict__ probs, InitSplit G,
                                                         int sweep) {
  extern __shared__ __align__(16) uint8_t ismem[];
  const orbx_init_problem& P = probs[0];
  if (!G.changed[sweep]) return;  // unchanged: the stored list is this sweep's too
  const int tid = threadIdx.x;
  const InitLds S = init_lds(ismem, P.f1.n, P.f2.n);
  init_list(P, S, tid);
  init_store_list(P, S, G, tid);
}

__global__ __launch_bounds__(IBS) void k_init_split_final(const orbx_init_problem* __restrict__ probs, InitSplit G) {
  extern __shared__ __align__(16) uint8_t ismem[];
  __shared__ int s_changed, s_count;
  __shared__ int s_hist[32], s_sel[3];
  const orbx_init_problem& P = probs[0];
  const int tid = threadIdx.x;
  const InitLds S = init_lds(ismem, P.f1.n, P.f2.n);
  init_load(P, S, G, true, tid);
  if (G.changed[kInitSplitSweeps - 1]) init_sweeps(P, S, &s_changed, kInitSplitSweeps, tid);  // block-uniform
  init_final(P, S, s_hist, s_sel, &s_count, tid);
}

hipError_t launch_search_by_projection(const ProjProblem* d_probs, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_search_by_projection, dim3(n), dim3(PBS), 0, st, d_probs);
  return hipGetLastError();
}

// nprob problems (d_prob[0..nprob), scratch z at d_scratch + z * kProjSplitBytes), each split over
// many blocks: the host single calls.  kinds / nP from the host copies of the problems.
hipError_t launch_search_by_projection_split(const ProjProblem* d_prob, const int* kinds, const int* nPs, int nprob,
                                             uint8_t* d_scratch, hipStream_t st) {
  int nPmax = 0;
  bool fuse = true;
  for (int z = 0; z < nprob; z++) {
    nPmax = std::max(nPmax, nPs[z]);
    fuse = fuse && (kinds[z] == ORBX_PROJ_FUSE || kinds[z] == ORBX_PROJ_FUSE_SIM3 || kinds[z] == ORBX_PROJ_BY_SIM3);
  }
  const int nb = std::min(64, std::max(1, (nPmax + PBS / kGroup - 1) / (PBS / kGroup)));
  hipLaunchKernelGGL(k_proj_split_prep, dim3(nb, 1, nprob), dim3(PBS), 0, st, d_prob, d_scratch);
  for (int s = 0; s < (fuse ? 1 : kProjSplitSweeps); s++)
    hipLaunchKernelGGL(k_proj_split_sweep, dim3(nb, 1, nprob), dim3(PBS), 0, st, d_prob, d_scratch, s);
  hipLaunchKernelGGL(k_proj_split_final, dim3(1, 1, nprob), dim3(PBS), 0, st, d_prob, d_scratch);
  return hipGetLastError();
}

}  // namespace orbx

// ------------------------------------------------------------------ C ABI
namespace {

orbx_status proj_status(hipError_t e) { return e == hipSuccess ? ORBX_OK : ORBX_ERR_HIP; }

// Host-side argument checks shared by both entry points (the kernel assumes them).
orbx_status proj_check(const orbx_proj_problem& p, bool host) {
  if (p.kind < ORBX_PROJ_LOCAL || p.kind > ORBX_PROJ_BY_SIM3) return ORBX_ERR_ARG;
  if (p.f.n < 0 || p.n_points < 0) return ORBX_ERR_ARG;
  if (p.f.n > ORBX_PROJ_MAX_FEATURES) return ORBX_ERR_CAPACITY;
  if (p.f.nlevels < 1 || p.f.nlevels > 16) return ORBX_ERR_ARG;
  if (!p.frame_out || !p.point_match || !p.nmatches) return ORBX_ERR_ARG;
  if (host && (p.f_n_dev || p.n_points_dev || p.Tcw_dev || p.gate)) return ORBX_ERR_ARG;  // device batches only
  if (p.f.n > 0 && (!p.f.keys_un || !p.f.desc)) return ORBX_ERR_ARG;
  if (p.n_points > 0) {
    if (!p.desc || !p.flags) return ORBX_ERR_ARG;
    switch (p.kind) {
      case ORBX_PROJ_LOCAL:
        if (!p.track || !p.track_level) return ORBX_ERR_ARG;
        if (p.frustum && (!p.pos || !p.normal || !p.dist_minmax)) return ORBX_ERR_ARG;
        if (host && !p.frustum)
          for (int i = 0; i < p.n_points; i++)
            if ((p.flags[i] & 1) && (p.track_level[i] < 0 || p.track_level[i] >= p.f.nlevels)) return ORBX_ERR_ARG;
        break;
      case ORBX_PROJ_LAST_FRAME:
        if (!p.pos || !p.octave || (p.check_ori && !p.angle)) return ORBX_ERR_ARG;
        if (host)
          for (int i = 0; i < p.n_points; i++)
            if ((p.flags[i] & 1) && (p.octave[i] < 0 || p.octave[i] >= p.f.nlevels)) return ORBX_ERR_ARG;
        break;
      case ORBX_PROJ_BY_SIM3:
        if (!p.pos || !p.dist_minmax) return ORBX_ERR_ARG;
        break;
      case ORBX_PROJ_FUSE:
      case ORBX_PROJ_SIM3:
      case ORBX_PROJ_FUSE_SIM3:
        if (!p.pos || !p.normal || !p.dist_minmax) return ORBX_ERR_ARG;
        break;
      default:
        if (!p.pos || !p.dist_minmax || (p.check_ori && !p.angle)) return ORBX_ERR_ARG;
    }
  }
  return ORBX_OK;
}

}  // namespace

namespace {
// The host single calls: n problems (1, or SearchBySim3's two directions) staged in one pooled
// arena -- every problem's inputs, then every problem's outputs, then the n device descriptors,
// then the device-only split scratch -- one upload, one split launch set over blockIdx.z, one
// download of the outputs, one sync.
orbx_status proj_run_host(const orbx_proj_problem* const* ps, int n, int device) {
  if (n < 1 || n > 2) return ORBX_ERR_ARG;  // (one problem, or SearchBySim3's two directions)
  for (int z = 0; z < n; z++) {
    const orbx_status chk = proj_check(*ps[z], true);
    if (chk != ORBX_OK) return chk;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  size_t off = 0;
  struct Item { const void* src; size_t bytes; size_t at; };
  std::vector<Item> items;
  auto reserve = [&](const void* src, size_t bytes) -> size_t {
    off = (off + 255) & ~(size_t)255;
    items.push_back({src, bytes, off});
    const size_t at = off;
    off += bytes;
    return at;
  };
  struct Lay {
    size_t keys, fdesc, ur, occ, desc, flags, pos, nrm, dmm, ang, oct, trk, lvl, fout, pm, nm;
  };
  Lay L[2];
  for (int z = 0; z < n; z++) {  // inputs
    const orbx_proj_problem* p = ps[z];
    const size_t nF = (size_t)p->f.n, nP = (size_t)p->n_points;
    Lay& a = L[z];
    a.keys = reserve(p->f.keys_un, nF * sizeof(orbx_keypoint));
    a.fdesc = reserve(p->f.desc, nF * 32);
    a.ur = p->f.u_right ? reserve(p->f.u_right, nF * 4) : 0;
    a.occ = p->f.occ ? reserve(p->f.occ, nF) : 0;
    a.desc = reserve(p->desc, nP * 32);
    a.flags = reserve(p->flags, nP);
    a.pos = p->pos ? reserve(p->pos, nP * 12) : 0;
    a.nrm = p->normal ? reserve(p->normal, nP * 12) : 0;
    a.dmm = p->dist_minmax ? reserve(p->dist_minmax, nP * 8) : 0;
    a.ang = p->angle ? reserve(p->angle, nP * 4) : 0;
    a.oct = p->octave ? reserve(p->octave, nP * 4) : 0;
  }
  off = (off + 255) & ~(size_t)255;
  const size_t o_out = off;  // outputs are contiguous from here up to the descriptors
  for (int z = 0; z < n; z++) {
    const orbx_proj_problem* p = ps[z];
    const size_t nF = (size_t)p->f.n, nP = (size_t)p->n_points;
    const bool local = p->kind == ORBX_PROJ_LOCAL;
    Lay& a = L[z];
    a.trk = local ? reserve(p->frustum ? nullptr : p->track, nP * 16) : 0;  // (in / out)
    a.lvl = local ? reserve(p->frustum ? nullptr : p->track_level, nP * 4) : 0;
    a.fout = reserve(nullptr, nF * 4);
    a.pm = reserve(nullptr, nP * 4);
    a.nm = reserve(nullptr, 4);
  }
  const size_t a_prob = reserve(nullptr, sizeof(orbx_proj_problem) * n);
  const size_t a_split = reserve(nullptr, orbx::kProjSplitBytes * n);  // device-only scratch (not copied)
  orbx::ScratchGuard g(device);  // pooled lease: no per-call allocation (orbx_scratch.h)
  if (!g.l || g.l->reserve(off, off) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* hst = g.l->h;
  std::memset(hst, 0, a_split);
  for (const Item& it : items)
    if (it.src && it.bytes) std::memcpy(hst + it.at, it.src, it.bytes);
  uint8_t* d = g.l->d;
  int kinds[2], nPs[2];
  for (int z = 0; z < n; z++) {
    const orbx_proj_problem* p = ps[z];
    const Lay& a = L[z];
    const bool local = p->kind == ORBX_PROJ_LOCAL;
    orbx_proj_problem q = *p;
    q.f.keys_un = (const orbx_keypoint*)(d + a.keys);
    q.f.desc = d + a.fdesc;
    q.f.u_right = p->f.u_right ? (const float*)(d + a.ur) : nullptr;
    q.f.occ = p->f.occ ? (const int8_t*)(d + a.occ) : nullptr;
    q.desc = d + a.desc;
    q.flags = d + a.flags;
    q.pos = p->pos ? (const float*)(d + a.pos) : nullptr;
    q.normal = p->normal ? (const float*)(d + a.nrm) : nullptr;
    q.dist_minmax = p->dist_minmax ? (const float*)(d + a.dmm) : nullptr;
    q.angle = p->angle ? (const float*)(d + a.ang) : nullptr;
    q.octave = p->octave ? (const int32_t*)(d + a.oct) : nullptr;
    q.track = local ? (float*)(d + a.trk) : nullptr;
    q.track_level = local ? (int32_t*)(d + a.lvl) : nullptr;
    q.frame_out = (int32_t*)(d + a.fout);
    q.point_match = (int32_t*)(d + a.pm);
    q.nmatches = (int32_t*)(d + a.nm);
    std::memcpy(hst + a_prob + z * sizeof(orbx_proj_problem), &q, sizeof(q));
    kinds[z] = p->kind;
    nPs[z] = p->n_points;
  }
  hipStream_t st = g.l->st;
  hipError_t e = hipMemcpyAsync(d, hst, a_split, hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = orbx::launch_search_by_projection_split((const orbx::ProjProblem*)(d + a_prob), kinds, nPs, n, d + a_split, st);
  if (e == hipSuccess) e = hipMemcpyAsync(hst + o_out, d + o_out, a_prob - o_out, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = g.l->sync();
  if (e != hipSuccess) return proj_status(e);
  for (int z = 0; z < n; z++) {
    const orbx_proj_problem* p = ps[z];
    const Lay& a = L[z];
    const size_t nF = (size_t)p->f.n, nP = (size_t)p->n_points;
    if (nF) std::memcpy(p->frame_out, hst + a.fout, nF * 4);
    if (nP) std::memcpy(p->point_match, hst + a.pm, nP * 4);
    std::memcpy(p->nmatches, hst + a.nm, 4);
    if (p->kind == ORBX_PROJ_LOCAL && p->frustum && nP) {
      std::memcpy(p->track, hst + a.trk, nP * 16);
      std::memcpy(p->track_level, hst + a.lvl, nP * 4);
    }
  }
  return ORBX_OK;
}
}  // namespace

extern "C" orbx_status orbx_search_by_projection(const orbx_proj_problem* p, int device) {
  if (!p) return ORBX_ERR_ARG;
  return proj_run_host(&p, 1, device);
}

extern "C" orbx_status orbx_search_by_projection_device(const orbx_proj_problem* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++) {
    const orbx_status s = proj_check(problems[i], false);
    if (s != ORBX_OK) return s;
  }
  hipStream_t st = (hipStream_t)stream;
  orbx::ProjProblem* dP = nullptr;
  if (hipMallocAsync((void**)&dP, sizeof(orbx::ProjProblem) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(dP, problems, sizeof(orbx::ProjProblem) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = orbx::launch_search_by_projection(dP, n, st);
  const hipError_t e2 = hipFreeAsync(dP, st);
  return proj_status(e != hipSuccess ? e : e2);
}

namespace {
// sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(), t21 = -sR21*t12 (src/ORBmatcher.cc:1252-1254): a Mat times
// a scalar is convertTo(alpha) -- x * (float)alpha + 0.0f in float; R12.t() scaled is transpose then
// convertTo; -A*b is cv::gemm's small-matrix path (float dot, then (float)((double)t0 * -1.0))
void sim3_pair(float s12, const float* R12, const float* t12, float* sR12_t12, float* sR21_t21) {
  const float a12 = (float)(double)s12, a21 = (float)(1.0 / (double)s12);
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) {
      sR12_t12[4 * r + c] = R12[3 * r + c] * a12 + 0.0f;
      sR21_t21[4 * r + c] = R12[3 * c + r] * a21 + 0.0f;
    }
    sR12_t12[4 * r + 3] = t12[r];
  }
  for (int r = 0; r < 3; r++) {
    const float t0 = sR21_t21[4 * r] * t12[0] + sR21_t21[4 * r + 1] * t12[1] + sR21_t21[4 * r + 2] * t12[2];
    sR21_t21[4 * r + 3] = (float)((double)t0 * -1.0);
  }
  for (int k = 12; k < 16; k++) sR12_t12[k] = sR21_t21[k] = k == 15 ? 1.0f : 0.0f;
}
}  // namespace

extern "C" orbx_status orbx_search_by_sim3(const orbx_sim3_problem* p, int device) {
  if (!p || !p->match12 || !p->nfound) return ORBX_ERR_ARG;
  const int N1 = p->kf1.n, N2 = p->kf2.n;
  if (N1 < 0 || N2 < 0) return ORBX_ERR_ARG;
  if (!(p->s12 > 0.0f) && !(p->s12 < 0.0f)) return ORBX_ERR_ARG;  // 1/s12
  float A12[16], A21[16];
  sim3_pair(p->s12, p->R12, p->t12, A12, A21);
  // direction 1: KF1's MapPoints into KF2 (points = KF1 features), direction 2: KF2's into KF1
  std::vector<int32_t> m1(N1 > 0 ? N1 : 1, -1), m2(N2 > 0 ? N2 : 1, -1);
  std::vector<int32_t> fo1(N2 > 0 ? N2 : 1), fo2(N1 > 0 ? N1 : 1);
  int32_t n1 = 0, n2 = 0;
  orbx_proj_problem qs[2];
  for (int d = 0; d < 2; d++) {
    orbx_proj_problem& q = qs[d];
    std::memset(&q, 0, sizeof(q));
    q.kind = ORBX_PROJ_BY_SIM3;
    q.f = d == 0 ? p->kf2 : p->kf1;
    q.f.occ = nullptr;
    const orbx_proj_frame& own = d == 0 ? p->kf1 : p->kf2;  // the points' KeyFrame: R1w|t1w or R2w|t2w
    std::memcpy(q.f.Tcw, own.Tcw, sizeof(q.f.Tcw));
    std::memcpy(q.last_Tcw, d == 0 ? A21 : A12, sizeof(q.last_Tcw));
    q.n_points = d == 0 ? N1 : N2;
    q.desc = d == 0 ? p->desc1 : p->desc2;
    q.flags = d == 0 ? p->flags1 : p->flags2;
    q.pos = d == 0 ? p->pos1 : p->pos2;
    q.dist_minmax = d == 0 ? p->dist_minmax1 : p->dist_minmax2;
    q.th = p->th;
    q.frame_out = d == 0 ? fo1.data() : fo2.data();
    q.point_match = d == 0 ? m1.data() : m2.data();
    q.nmatches = d == 0 ? &n1 : &n2;
  }
  const orbx_proj_problem* qp[2] = {&qs[0], &qs[1]};
  const orbx_status st = proj_run_host(qp, 2, device);  // both directions in one upload / launch set
  if (st != ORBX_OK) return st;
  // mutual check (:1466-1482)
  int nFound = 0;
  for (int i1 = 0; i1 < N1; i1++) {
    const int idx2 = m1[i1];
    p->match12[i1] = -1;
    if (idx2 >= 0 && idx2 < N2 && m2[idx2] == i1) {
      p->match12[i1] = idx2;
      nFound++;
    }
  }
  *p->nfound = nFound;
  return ORBX_OK;
}

extern "C" orbx_status orbx_search_for_initialization(const orbx_init_problem* p, int device) {
  if (!p || !p->match12 || !p->nmatches || !p->prev_matched) return ORBX_ERR_ARG;
  const int n1 = p->f1.n, n2 = p->f2.n;
  if (n1 < 0 || n2 < 0) return ORBX_ERR_ARG;
  if (n1 > ORBX_PROJ_MAX_FEATURES || n2 > ORBX_PROJ_MAX_FEATURES) return ORBX_ERR_CAPACITY;
  if ((n1 > 0 && (!p->f1.keys_un || !p->f1.desc)) || (n2 > 0 && (!p->f2.keys_un || !p->f2.desc))) return ORBX_ERR_ARG;
  if (p->window < 0) return ORBX_ERR_ARG;
  for (int i = 0; i < n1; i++)
    if (p->f1.keys_un[i].octave < 0) return ORBX_ERR_ARG;  // GetFeaturesInArea(.., level1, level1) needs level1 >= 0
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  size_t off = 0;
  auto at = [&](size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    const size_t a = off;
    off += bytes;
    return a;
  };
  const size_t a_k1 = at((size_t)n1 * sizeof(orbx_keypoint)), a_d1 = at((size_t)n1 * 32);
  const size_t a_k2 = at((size_t)n2 * sizeof(orbx_keypoint)), a_d2 = at((size_t)n2 * 32);
  const size_t a_prev = at((size_t)n1 * 8), a_m = at((size_t)n1 * 4 + 4), a_nm = at(4);
  const size_t a_prob = at(sizeof(orbx_init_problem));
  const size_t a_split = at(orbx::kInitSplitBytes);  // device-only scratch
  orbx::ScratchGuard g(device);
  if (!g.l || g.l->reserve(off, off) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* h = g.l->h;
  uint8_t* d = g.l->d;
  std::memset(h, 0, a_split);
  if (n1) {
    std::memcpy(h + a_k1, p->f1.keys_un, (size_t)n1 * sizeof(orbx_keypoint));
    std::memcpy(h + a_d1, p->f1.desc, (size_t)n1 * 32);
    std::memcpy(h + a_prev, p->prev_matched, (size_t)n1 * 8);
  }
  if (n2) {
    std::memcpy(h + a_k2, p->f2.keys_un, (size_t)n2 * sizeof(orbx_keypoint));
    std::memcpy(h + a_d2, p->f2.desc, (size_t)n2 * 32);
  }
  orbx_init_problem q = *p;
  q.f1.keys_un = (const orbx_keypoint*)(d + a_k1);
  q.f1.desc = d + a_d1;
  q.f2.keys_un = (const orbx_keypoint*)(d + a_k2);
  q.f2.desc = d + a_d2;
  q.f1.u_right = q.f2.u_right = nullptr;
  q.f1.occ = q.f2.occ = nullptr;
  q.prev_matched = (float*)(d + a_prev);
  q.match12 = (int32_t*)(d + a_m);
  q.nmatches = (int32_t*)(d + a_nm);
  std::memcpy(h + a_prob, &q, sizeof(q));
  hipStream_t st = g.l->st;
  const size_t smem = orbx::init_smem_bytes(n1, n2);
  // the dynamic LDS reaches ~79 KB at 8192 features (above the 64 KB default)
  hipError_t e = hipSuccess;
  for (const void* k : {(const void*)orbx::k_init_split_prep, (const void*)orbx::k_init_split_sweep,
                        (const void*)orbx::k_init_split_list, (const void*)orbx::k_init_split_final})
    if (e == hipSuccess) e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e == hipSuccess) e = hipMemcpyAsync(d, h, a_split, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    // one problem over many blocks: ~64 F1 keypoints per block per sweep
    const orbx_init_problem* dp = (const orbx_init_problem*)(d + a_prob);
    const orbx::InitSplit S = orbx::init_split_at(d + a_split);
    const int nb = std::min(64, std::max(1, (n1 + orbx::IBS / orbx::kGroup - 1) / (orbx::IBS / orbx::kGroup)));
    hipLaunchKernelGGL(orbx::k_init_split_prep, dim3(1), dim3(orbx::IBS), smem, st, dp, S);
    for (int s = 0; s < orbx::kInitSplitSweeps; s++) {
      hipLaunchKernelGGL(orbx::k_init_split_sweep, dim3(nb), dim3(orbx::IBS), smem, st, dp, S, s);
      hipLaunchKernelGGL(orbx::k_init_split_list, dim3(1), dim3(orbx::IBS), smem, st, dp, S, s);
    }
    hipLaunchKernelGGL(orbx::k_init_split_final, dim3(1), dim3(orbx::IBS), smem, st, dp, S);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(h + a_prev, d + a_prev, a_prob - a_prev, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = g.l->sync();
  if (e != hipSuccess) return ORBX_ERR_HIP;
  if (n1) {
    std::memcpy(p->prev_matched, h + a_prev, (size_t)n1 * 8);
    std::memcpy(p->match12, h + a_m, (size_t)n1 * 4);
  }
  std::memcpy(p->nmatches, h + a_nm, 4);
  return ORBX_OK;
}
