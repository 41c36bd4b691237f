// orbx_stereo.h -- argument block of the batched stereo matcher (stereo.hip).
#pragma once
#include "orbx_internal.h"

namespace orbx {

constexpr int kMaxStereoKps = 4096;  // right keypoints per frame (12-bit index in sort keys)

struct StereoArgs {
  const orbx_keypoint* kpL;
  const uint8_t* dL;
  const int32_t* nL;
  long long kL_stride;   // entries between frames
  long long n_stride_L;  // stride of nL between frames
  const orbx_keypoint* kpR;
  const uint8_t* dR;
  const int32_t* nR;
  long long kR_stride;
  long long n_stride_R;
  BatchPtrs BL, BR;       // pyramids
  int l_step, l_off, r_step, r_off;  // frame f -> image indices
  int nlevels;
  int maxL;
  float inv_scale[kMaxLevelsPlan];
  float bf, minZ, minD, maxD;
  float* uR;
  float* depth;
  int* sad;
  long long out_stride;
  uint64_t* rkeys;  // [n_frames * kMaxStereoKps]
  int* oct_start;   // [n_frames * (kMaxLevelsPlan+1)]
  int2* rxi;        // [n_frames * kMaxStereoKps]: (float bits of x, index) in (octave, y) order
  uint4* rdesc;     // [n_frames * kMaxStereoKps * 2]: right descriptors in the same sorted order
  uint32_t* rtab;   // [n_frames * nlevels * rows]: candidate range start | end << 16 per (octave, row)
  uint4* lrange;    // [n_frames * maxL]: per left keypoint its rtab entries of octaves level-1..level+1 (0: none)
  int rows;         // rows of the row table = level-0 image height (vRowIndices size)
  int32_t* nmatches;
};

struct StageTimer;
hipError_t launch_stereo(const StereoArgs& A, const Geometry* Gd, int n_frames, int maxL, hipStream_t st,
                         StageTimer* T);
hipError_t launch_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out, hipStream_t st);

}  // namespace orbx
