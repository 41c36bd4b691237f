// mapping.hip -- the two small per-MapPoint / per-KeyFrame routines of
// SURVEY §8(f) row 4, batched:
//
//   k_distinctive  MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:249-320
//   k_undistort    Frame::UndistortKeyPoints               src/Frame.cc:471-506
//                  (cv::undistortPoints, OpenCV 3.2 cvUndistortPoints)
//
// k_distinctive: one wave per MapPoint.  The reference builds the N x N
// Hamming matrix, sorts every row and keeps the first row with the smallest
// vDists[(size_t)(0.5*(N-1))].  Here lane i owns row i and finds that order
// statistic without storing or sorting the row: the k-th smallest of N
// integers in [0,256] is the largest t with #{j : d(i,j) < t} <= k, built bit
// by bit in 9 counting passes over the point's descriptors (wave-uniform
// addresses, so the descriptor loads are scalar and shared by all lanes).
// The row winner is a wave min over (median << 16 | i): smallest median,
// first row on ties, as the reference's strict `median < BestMedian`.
// Bytes per point: 32 N read (L1/K$-resident after the first pass), 36 written.
//
// k_undistort: one thread per keypoint, all FP64 in cvUndistortPoints'
// operation order (-ffp-contract=off; AMDGPU f64 division is correctly
// rounded), so keys_un equals the oracle bit for bit.  28 B read + 28 B
// written per keypoint: HBM-bound when batched.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <vector>

#include "orbx_scratch.h"
#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {
namespace mapping {

constexpr int MBS = 256;  // 4 MapPoints per block
constexpr int UBS = 256;

__global__ __launch_bounds__(MBS) void k_distinctive(const uint8_t* __restrict__ desc,
                                                     const int32_t* __restrict__ obs_off, int n_points,
                                                     int32_t* __restrict__ best, uint8_t* __restrict__ out_desc) {
  const int lane = threadIdx.x & 63;
  const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * (MBS / 64) + (threadIdx.x >> 6));
  if (p >= n_points) return;  // whole wave
  const int o0 = obs_off[p], n = obs_off[p + 1] - o0;
  if (n <= 0) {
    if (lane == 0) best[p] = -1;
    return;
  }
  const uint64_t* D = (const uint64_t*)(desc + (size_t)o0 * 32);
  const int k = (n - 1) >> 1;  // (size_t)(0.5*(N-1)), src/MapPoint.cc:306
  uint32_t key = 0xFFFFFFFFu;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    uint64_t di[4] = {0, 0, 0, 0};
    if (i < n) {
      di[0] = D[4 * i];
      di[1] = D[4 * i + 1];
      di[2] = D[4 * i + 2];
      di[3] = D[4 * i + 3];
    }
    int t = 0;  // largest t with #{d < t} <= k  ==  the k-th smallest distance of row i
#pragma unroll 1
    for (int b = 256; b > 0; b >>= 1) {
      const int c = t + b;
      int cnt = 0;
      for (int j = 0; j < n; j++) cnt += hamming256(di, D + 4 * j) < c;
      if (cnt <= k) t = c;
    }
    if (i < n) {
      const uint32_t kk = ((uint32_t)t << 16) | (uint32_t)i;
      key = kk < key ? kk : key;
    }
  }
  key = wave_min_u32(key);
  const int bi = (int)(key & 0xFFFF);
  if (lane == 0) best[p] = bi;
  if (out_desc && lane < 8)
    ((uint32_t*)(out_desc + (size_t)p * 32))[lane] = ((const uint32_t*)(desc + ((size_t)o0 + bi) * 32))[lane];
}

__global__ __launch_bounds__(UBS) void k_undistort(const orbx_keypoint* __restrict__ keys,
                                                   const int32_t* __restrict__ frame_off,
                                                   const orbx_camera* __restrict__ cams,
                                                   orbx_keypoint* __restrict__ keys_un) {
  const int f = blockIdx.y;
  const int a = frame_off[f], n = frame_off[f + 1] - a;
  const int i = blockIdx.x * UBS + threadIdx.x;
  if (i >= n) return;
  orbx_keypoint kp = keys[a + i];
  const orbx_camera& cam = cams[f];
  if (cam.dist[0] != 0.0f) {  // mDistCoef.at<float>(0)==0.0: plain copy (src/Frame.cc:474-478)
    double kc[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 5; j++)
      if (j < cam.n_dist) kc[j] = cam.dist[j];
    double A[9];
#pragma unroll
    for (int j = 0; j < 9; j++) A[j] = cam.K[j];
    const double ifx = 1. / A[0], ify = 1. / A[4], cx = A[2], cy = A[5];
    double x = kp.x, y = kp.y;
    const double x0 = x = (x - cx) * ifx;
    const double y0 = y = (y - cy) * ify;
#pragma unroll
    for (int it = 0; it < 5; it++) {  // cvUndistortPoints: iters = 5 with distortion
      const double r2 = x * x + y * y;
      const double icdist = 1 / (1 + ((kc[4] * r2 + kc[1]) * r2 + kc[0]) * r2);
      const double deltaX = 2 * kc[2] * x * y + kc[3] * (r2 + 2 * x * x);
      const double deltaY = kc[2] * (r2 + 2 * y * y) + 2 * kc[3] * x * y;
      x = (x0 - deltaX) * icdist;
      y = (y0 - deltaY) * icdist;
    }
    const double xx = A[0] * x + A[1] * y + A[2];
    const double yy = A[3] * x + A[4] * y + A[5];
    const double ww = 1. / (A[6] * x + A[7] * y + A[8]);
    kp.x = (float)(xx * ww);
    kp.y = (float)(yy * ww);
  }
  keys_un[a + i] = kp;
}

}  // namespace mapping
}  // namespace orbx

// ------------------------------------------------------------------ C ABI
namespace {

orbx_status set_device(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  return ORBX_OK;
}

bool camera_ok(const orbx_camera& c) { return c.n_dist >= 4 && c.n_dist <= 5 && c.K[0] != 0.0f && c.K[4] != 0.0f; }

}  // namespace

extern "C" orbx_status orbx_distinctive_descriptors_device(const uint8_t* desc, const int32_t* obs_off, int n_points,
                                                           int32_t* best, uint8_t* out_desc, void* stream) {
  if (n_points < 0 || (n_points > 0 && (!desc || !obs_off || !best))) return ORBX_ERR_ARG;
  if (n_points == 0) return ORBX_OK;
  const int grid = (n_points + orbx::mapping::MBS / 64 - 1) / (orbx::mapping::MBS / 64);
  hipLaunchKernelGGL(orbx::mapping::k_distinctive, dim3(grid), dim3(orbx::mapping::MBS), 0, (hipStream_t)stream,
                     desc, obs_off, n_points, best, out_desc);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" orbx_status orbx_distinctive_descriptors(const uint8_t* desc, const int32_t* obs_off, int n_points,
                                                    int32_t* best, uint8_t* out_desc, int device) {
  if (n_points < 0 || (n_points > 0 && (!desc || !obs_off || !best))) return ORBX_ERR_ARG;
  if (n_points == 0) return ORBX_OK;
  if (obs_off[0] != 0) return ORBX_ERR_ARG;
  for (int p = 0; p < n_points; p++)  // host check of the CSR the kernel trusts (row index fits 16 bits)
    if (obs_off[p + 1] < obs_off[p] || obs_off[p + 1] - obs_off[p] > 65535) return ORBX_ERR_ARG;
  const orbx_status ds = set_device(device);
  if (ds != ORBX_OK) return ds;
  const size_t nd = (size_t)obs_off[n_points];
  const size_t b_desc = (nd * 32 + 255) & ~(size_t)255, b_off = ((size_t)(n_points + 1) * 4 + 255) & ~(size_t)255;
  const size_t b_best = ((size_t)n_points * 4 + 255) & ~(size_t)255;
  // pooled lease (orbx_scratch.h): inputs staged in pinned memory, one stream, no allocation
  const size_t total = b_desc + b_off + b_best + (size_t)n_points * 32;
  orbx::ScratchGuard g(device);
  if (!g.l || g.l->reserve(total, total) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* d = g.l->d;
  uint8_t* h = g.l->h;
  uint8_t *d_desc = d, *d_off = d + b_desc, *d_best = d_off + b_off, *d_out = d_best + b_best;
  if (nd) std::memcpy(h, desc, nd * 32);
  std::memcpy(h + b_desc, obs_off, (size_t)(n_points + 1) * 4);
  hipStream_t sm = g.l->st;
  hipError_t e = hipMemcpyAsync(d, h, b_desc + (size_t)(n_points + 1) * 4, hipMemcpyHostToDevice, sm);
  orbx_status st = ORBX_ERR_HIP;
  if (e == hipSuccess)
    st = orbx_distinctive_descriptors_device(d_desc, (const int32_t*)d_off, n_points, (int32_t*)d_best,
                                             out_desc ? d_out : nullptr, sm);
  if (st == ORBX_OK) {
    // best and the descriptors are adjacent: one copy back
    e = hipMemcpyAsync(h + (d_best - d), d_best, out_desc ? b_best + (size_t)n_points * 32 : (size_t)n_points * 4,
                       hipMemcpyDeviceToHost, sm);
    if (e == hipSuccess) e = g.l->sync();
    if (e != hipSuccess) {
      st = ORBX_ERR_HIP;
    } else {
      std::memcpy(best, h + (d_best - d), (size_t)n_points * 4);
      if (out_desc) std::memcpy(out_desc, h + (d_out - d), (size_t)n_points * 32);
    }
  }
  return st;
}

extern "C" orbx_status orbx_undistort_keypoints_device(const orbx_keypoint* keys, const int32_t* frame_off,
                                                       int n_frames, int max_keys, const orbx_camera* cams,
                                                       orbx_keypoint* keys_un, void* stream) {
  if (n_frames < 0 || max_keys < 0 || (n_frames > 0 && (!keys || !frame_off || !cams || !keys_un)))
    return ORBX_ERR_ARG;
  if (n_frames == 0 || max_keys == 0) return ORBX_OK;
  if (n_frames > 65535) return ORBX_ERR_SIZE;
  const dim3 grid((max_keys + orbx::mapping::UBS - 1) / orbx::mapping::UBS, n_frames);
  hipLaunchKernelGGL(orbx::mapping::k_undistort, grid, dim3(orbx::mapping::UBS), 0, (hipStream_t)stream, keys,
                     frame_off, cams, keys_un);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" orbx_status orbx_undistort_keypoints(const orbx_keypoint* keys, int n, const orbx_camera* cam,
                                                orbx_keypoint* keys_un, int device) {
  if (n < 0 || !cam || (n > 0 && (!keys || !keys_un))) return ORBX_ERR_ARG;
  if (!camera_ok(*cam)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  const orbx_status ds = set_device(device);
  if (ds != ORBX_OK) return ds;
  const size_t bk = ((size_t)n * sizeof(orbx_keypoint) + 255) & ~(size_t)255;
  const size_t total = 2 * bk + 256 + sizeof(orbx_camera);
  orbx::ScratchGuard g(device);  // pooled lease (orbx_scratch.h)
  if (!g.l || g.l->reserve(total, total) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* d = g.l->d;
  uint8_t* h = g.l->h;
  orbx_keypoint *d_in = (orbx_keypoint*)d, *d_out = (orbx_keypoint*)(d + bk);
  int32_t* d_off = (int32_t*)(d + 2 * bk);
  orbx_camera* d_cam = (orbx_camera*)(d + 2 * bk + 256);
  const int32_t off[2] = {0, n};
  std::memcpy(h, keys, (size_t)n * sizeof(orbx_keypoint));
  std::memcpy(h + 2 * bk, off, sizeof(off));
  std::memcpy(h + 2 * bk + 256, cam, sizeof(orbx_camera));
  hipStream_t sm = g.l->st;
  // inputs in two copies (keypoints; offsets + camera), the output in one
  hipError_t e = hipMemcpyAsync(d, h, (size_t)n * sizeof(orbx_keypoint), hipMemcpyHostToDevice, sm);
  if (e == hipSuccess) e = hipMemcpyAsync(d + 2 * bk, h + 2 * bk, 256 + sizeof(orbx_camera), hipMemcpyHostToDevice, sm);
  orbx_status st = ORBX_ERR_HIP;
  if (e == hipSuccess) st = orbx_undistort_keypoints_device(d_in, d_off, 1, n, d_cam, d_out, sm);
  if (st == ORBX_OK) {
    e = hipMemcpyAsync(h + bk, d_out, (size_t)n * sizeof(orbx_keypoint), hipMemcpyDeviceToHost, sm);
    if (e == hipSuccess) e = g.l->sync();
    if (e != hipSuccess)
      st = ORBX_ERR_HIP;
    else
      std::memcpy(keys_un, h + bk, (size_t)n * sizeof(orbx_keypoint));
  }
  return st;
}
