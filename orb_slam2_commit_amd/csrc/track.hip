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
