// track.hip -- the gather between SearchByBoW and PoseOptimization in
// Tracking::TrackReferenceKeyFrame (src/Tracking.cc:910-969), on a device batch:
//
//   nmatches = matcher.SearchByBoW(mpReferenceKF, mCurrentFrame, vpMapPointMatches);  (:918-925)
//   mCurrentFrame.mvpMapPoints = vpMapPointMatches;                                     (:933)
//   Optimizer::PoseOptimization(&mCurrentFrame);                                        (:936)
//
// PoseOptimization adds one edge per current-frame feature with a MapPoint, in feature order
// (src/Optimizer.cc:318-410): the observation (mvKeysUn pt, mvuRight: monocular when < 0), the
// MapPoint's world position and mvInvLevelSigma2[octave].  Here the reference KeyFrame's MapPoints
// are its stereo points -- the map StereoInitialization / CreateNewKeyFrame build
// (src/Tracking.cc:640-668, 1515-1555): feature k has a MapPoint iff mvDepth[k] > 0, at
// Frame::UnprojectStereo(k) (src/Frame.cc:823-839: x3Dc = ((u-cx)*z*invfx, (v-cy)*z*invfy, z) from
// mvKeysUn, then mRwc*x3Dc+mOw -- cv::gemm with the addend on OpenCV 3.2's small-matrix path:
// the 3-term dot product in float, then one correctly rounded float add of mOw).
// One block per frame; the compaction is an ordered block scan, so edges keep feature order.
#include <hip/hip_runtime.h>

#include "../../include/orbx.h"

namespace orbx {
namespace track {

constexpr int TBS = 256;

__global__ __launch_bounds__(TBS) void k_track_gather(const orbx_track_gather* __restrict__ probs) {
  const orbx_track_gather& P = probs[blockIdx.x];
  __shared__ int wsum[TBS / 64];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = *P.f_count;
  const float invfx = 1.0f / P.fx, invfy = 1.0f / P.fy;  // Frame/KeyFrame invfx = 1.0f/fx
  if (tid == 0) base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < n; i0 += TBS) {
    const int i = i0 + tid;
    int k = -1;
    if (i < n) {
      k = P.match[i];
      if (k >= 0 && !(P.kf_depth[k] > 0.0f)) k = -1;  // no MapPoint behind that KeyFrame feature
    }
    const bool e = k >= 0;
    const unsigned long long b = __ballot(e);
    const int pre = __popcll(b & ((1ull << lane) - 1));
    if (lane == 0) wsum[wv] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (e) {
      const int o = off + pre;
      const orbx_keypoint kf = P.kf_kps[k];
      const float z = P.kf_depth[k];
      const float x = (kf.x - P.cx) * z * invfx;
      const float y = (kf.y - P.cy) * z * invfy;
      float X[3];
#pragma unroll
      for (int r = 0; r < 3; r++) {  // mRwc*x3Dc+mOw: cv::gemm's small-matrix path (float dot, then + Ow)
        const float t0 = P.Twc[4 * r] * x + P.Twc[4 * r + 1] * y + P.Twc[4 * r + 2] * z;
        X[r] = (float)((double)t0 + (double)P.Twc[4 * r + 3]);
      }
      const orbx_keypoint f = P.f_kps[i];
      P.obs[3 * o] = f.x;
      P.obs[3 * o + 1] = f.y;
      P.obs[3 * o + 2] = P.f_uright ? P.f_uright[i] : -1.0f;
      P.Xw[3 * o] = X[0];
      P.Xw[3 * o + 1] = X[1];
      P.Xw[3 * o + 2] = X[2];
      P.inv_sigma2[o] = P.inv_level_sigma2[f.octave];
      if (P.edge_feature) P.edge_feature[o] = i;
    }
    __syncthreads();
    if (tid == 0) {
      int t = base;
      for (int w = 0; w < TBS / 64; w++) t += wsum[w];
      base = t;
    }
    __syncthreads();
  }
  if (tid == 0) *P.n_edges = base;
}

// ---- the MapPoints of a stereo frame (orbx_frame_points) --------------------------------------
// Frame::UnprojectStereo then MapPoint::UpdateNormalAndDepth with the creating KeyFrame as the one
// observation, in OpenCV 3.2's float arithmetic: the gemm small-matrix path for Rwc*x3Dc+Ow,
// normali / cv::norm(normali) as Mat::convertTo with the scale (float)(1./norm) (x * scale in
// float), cv::norm as the sqrt of a double sum of squares.
__global__ __launch_bounds__(TBS) void k_frame_points(const orbx_frame_points* __restrict__ probs) {
  const orbx_frame_points& P = probs[blockIdx.y];
  const int i = blockIdx.x * TBS + threadIdx.x;
  const int n = min(max(*P.count, 0), P.cap);
  if (i >= n) return;
  const orbx_keypoint kp = P.kps[i];
  const float z = P.depth[i];
  P.angle[i] = kp.angle;
  P.octave[i] = kp.octave;
  if (!(z > 0.0f)) {
    P.flags[i] = 2;
    return;
  }
  P.flags[i] = 3;
  const float invfx = 1.0f / P.fx, invfy = 1.0f / P.fy;
  const float x = (kp.x - P.cx) * z * invfx;
  const float y = (kp.y - P.cy) * z * invfy;
  float X[3], PC[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const float t0 = P.Twc[4 * r] * x + P.Twc[4 * r + 1] * y + P.Twc[4 * r + 2] * z;
    X[r] = (float)((double)t0 + (double)P.Twc[4 * r + 3]);
    PC[r] = X[r] - P.Twc[4 * r + 3];
  }
  double ss = (double)PC[0] * PC[0];
  ss = ss + (double)PC[1] * PC[1];
  ss = ss + (double)PC[2] * PC[2];
  const double nrm = __builtin_sqrt(ss);
  const float sc = (float)(1.0 / nrm);
  const float dist = (float)nrm;
  const int lvl = min(max(kp.octave, 0), P.nlevels - 1);
  const float dmax = dist * P.scale_factors[lvl];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    P.pos[3 * i + r] = X[r];
    P.normal[3 * i + r] = PC[r] * sc;
  }
  P.dist_minmax[2 * i] = dmax / P.scale_factors[P.nlevels - 1];
  P.dist_minmax[2 * i + 1] = dmax;
}

// ---- TrackWithMotionModel / TrackLocalMap bookkeeping (orbx_track_step) ----------------------
// Edges of the frame's current MapPoint table, in feature order (src/Optimizer.cc:318-410): an
// ordered block compaction as in k_track_gather.
__device__ void track_edges(const orbx_track_step& P, int n, bool lost, int* wsum, int* base) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) *base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < (lost ? 0 : n); i0 += TBS) {
    const int i = i0 + tid;
    const int k = i < n ? P.fmap[i] : -1;
    const bool e = k >= 0;
    const unsigned long long b = __ballot(e);
    const int pre = __popcll(b & ((1ull << lane) - 1));
    if (lane == 0) wsum[wv] = __popcll(b);
    __syncthreads();
    int off = *base;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (e) {
      const int o = off + pre;
      const orbx_keypoint f = P.kps[i];
      P.obs[3 * o] = f.x;
      P.obs[3 * o + 1] = f.y;
      P.obs[3 * o + 2] = P.u_right ? P.u_right[i] : -1.0f;
#pragma unroll
      for (int c = 0; c < 3; c++) P.Xw[3 * o + c] = P.pos[3 * k + c];
      P.inv_sigma2[o] = P.inv_level_sigma2[f.octave];
      P.edge_feature[o] = i;
    }
    __syncthreads();
    if (tid == 0) {
      int t = *base;
      for (int w = 0; w < TBS / 64; w++) t += wsum[w];
      *base = t;
    }
    __syncthreads();
  }
  if (tid == 0) *P.n_edges = *base;
}

__global__ __launch_bounds__(TBS) void k_track_step(const orbx_track_step* __restrict__ probs) {
  const orbx_track_step& P = probs[blockIdx.x];
  __shared__ int wsum[TBS / 64];
  __shared__ int base;
  __shared__ int s_lost;
  const int tid = threadIdx.x;
  const int n = min(max(*P.count, 0), P.cap);
  const int np = min(max(*P.n_points, 0), P.cap);
  if (P.op == ORBX_TRACK_AFTER_MOTION) {
    // src/Tracking.cc:1066-1079: the search result is the frame's MapPoints; fewer than 20: lost
    if (tid == 0) s_lost = *P.nmatches < P.min_matches ? 1 : 0;
    for (int k = tid; k < np; k += TBS) P.seen[k] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += TBS) {
      const int k = P.frame_out[i];
      P.fmap[i] = k >= 0 ? k : -1;
      if (k >= 0) P.seen[k] = 1;  // mnLastFrameSeen = mCurrentFrame.mnId (:1101, :1413)
    }
    __syncthreads();
    if (tid == 0) *P.lost = s_lost;
    track_edges(P, n, s_lost != 0, wsum, &base);
  } else if (P.op == ORBX_TRACK_AFTER_POSE) {
    // :1093-1107 outliers leave the frame; :1135 nmatchesMap >= 10; :1408-1430 SearchLocalPoints' inputs
    if (tid == 0) s_lost = (*P.lost != 0 || *P.ngood < P.min_good) ? 1 : 0;
    const int ne = *P.n_edges;
    for (int e = tid; e < ne; e += TBS)
      if (P.outlier[e]) P.fmap[P.edge_feature[e]] = -1;
    __syncthreads();
    for (int i = tid; i < n; i += TBS) P.occ[i] = P.fmap[i] >= 0 ? 2 : 0;
    for (int k = tid; k < np; k += TBS)
      P.local_flags[k] = (uint8_t)(((P.flags[k] & 1) && !P.seen[k] && !s_lost ? 1 : 0) | 2);
    if (tid == 0) *P.lost = s_lost;
  } else {  // ORBX_TRACK_AFTER_LOCAL
    if (tid == 0) s_lost = *P.lost;
    __syncthreads();
    if (!s_lost)
      for (int i = tid; i < n; i += TBS) {
        const int k = P.frame_out[i];
        if (k >= 0) P.fmap[i] = k;
      }
    __syncthreads();
    track_edges(P, n, s_lost != 0, wsum, &base);
  }
}

}  // namespace track
}  // namespace orbx

extern "C" orbx_status orbx_track_gather_device(const orbx_track_gather* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++) {
    const orbx_track_gather& p = problems[i];
    if (!p.f_kps || !p.f_count || !p.match || !p.kf_kps || !p.kf_depth || !p.inv_level_sigma2 || !p.obs || !p.Xw ||
        !p.inv_sigma2 || !p.n_edges || p.fx == 0.0f || p.fy == 0.0f)
      return ORBX_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  orbx_track_gather* d = nullptr;
  if (hipMallocAsync((void**)&d, sizeof(orbx_track_gather) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(d, problems, sizeof(orbx_track_gather) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::track::k_track_gather, dim3(n), dim3(orbx::track::TBS), 0, st, d);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipFreeAsync(d, st);
  return (e == hipSuccess && e2 == hipSuccess) ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" orbx_status orbx_frame_points_device(const orbx_frame_points* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  int cap = 0;
  for (int i = 0; i < n; i++) {
    const orbx_frame_points& p = problems[i];
    if (!p.kps || !p.depth || !p.count || !p.pos || !p.normal || !p.dist_minmax || !p.angle || !p.octave ||
        !p.flags || p.cap <= 0 || p.nlevels < 1 || p.nlevels > 16 || p.fx == 0.0f || p.fy == 0.0f)
      return ORBX_ERR_ARG;
    cap = p.cap > cap ? p.cap : cap;
  }
  hipStream_t st = (hipStream_t)stream;
  orbx_frame_points* d = nullptr;
  if (hipMallocAsync((void**)&d, sizeof(orbx_frame_points) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(d, problems, sizeof(orbx_frame_points) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::track::k_frame_points, dim3((cap + orbx::track::TBS - 1) / orbx::track::TBS, n),
                       dim3(orbx::track::TBS), 0, st, d);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipFreeAsync(d, st);
  return (e == hipSuccess && e2 == hipSuccess) ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" orbx_status orbx_track_step_device(const orbx_track_step* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++) {
    const orbx_track_step& p = problems[i];
    if (p.op < ORBX_TRACK_AFTER_MOTION || p.op > ORBX_TRACK_AFTER_LOCAL || p.cap <= 0 || !p.count || !p.n_points ||
        !p.fmap || !p.lost || !p.n_edges)
      return ORBX_ERR_ARG;
    const bool edges = p.op != ORBX_TRACK_AFTER_POSE;
    if (edges && (!p.kps || !p.inv_level_sigma2 || !p.pos || !p.frame_out || !p.obs || !p.Xw || !p.inv_sigma2 ||
                  !p.edge_feature))
      return ORBX_ERR_ARG;
    if (p.op == ORBX_TRACK_AFTER_MOTION && (!p.nmatches || !p.seen)) return ORBX_ERR_ARG;
    if (p.op == ORBX_TRACK_AFTER_POSE &&
        (!p.outlier || !p.ngood || !p.edge_feature || !p.seen || !p.flags || !p.local_flags || !p.occ))
      return ORBX_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  orbx_track_step* d = nullptr;
  if (hipMallocAsync((void**)&d, sizeof(orbx_track_step) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(d, problems, sizeof(orbx_track_step) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::track::k_track_step, dim3(n), dim3(orbx::track::TBS), 0, st, d);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipFreeAsync(d, st);
  return (e == hipSuccess && e2 == hipSuccess) ? ORBX_OK : ORBX_ERR_HIP;
}
