// orbx_device.h -- device-side numerics shared by the HIP kernels.
//
// Everything here is compiled with -ffp-contract=off: every float/double
// expression rounds exactly as written, so results equal the CPU restatement
// of the reference (oracle/) bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbx {

constexpr int kHalfPatch = 15;      // HALF_PATCH_SIZE, src/ORBextractor.cc:73
constexpr int kEdgeThreshold = 19;  // EDGE_THRESHOLD, src/ORBextractor.cc:74
constexpr int kMaxLevels = 16;

// cvRound (SSE2 cvtss2si): round half to even.
// XCD-aware block order.  MI355X deals blocks round-robin over its 8 XCDs,
// each with a private L2, so neighbouring blocks -- cells, tiles, keypoints
// that read overlapping image rows -- would each pull the shared lines into a
// different L2.  xcd_block maps the hardware linear block id so that the
// blocks sharing an XCD take one contiguous range of the logical grid.
// Bijective for any grid size (q + 1 blocks for the first total % 8 groups);
// affects speed only, never results.
__device__ __forceinline__ int xcd_block(int hw, int total) {
  const int x = hw & 7, i = hw >> 3, q = total >> 3, r = total & 7;
  return x * q + min(x, r) + i;
}
// logical (x, y) of a 2-D grid, x fastest
// (unsigned divisions: the block-uniform quotients are scalar instruction sequences, and the signed
// forms' abs / sign fix-ups made them a large part of a short kernel's scalar work)
__device__ __forceinline__ int2 xcd_block2() {
  const unsigned gx = gridDim.x;
  const unsigned l = (unsigned)xcd_block(blockIdx.x + gx * blockIdx.y, gx * gridDim.y);
  const unsigned q = l / gx;
  return make_int2((int)(l - q * gx), (int)q);
}
// logical (x, y, z) of a 3-D grid, x fastest
__device__ __forceinline__ int3 xcd_block3() {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned l = (unsigned)xcd_block(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const unsigned q = l / gx, z = q / gy;
  return make_int3((int)(l - q * gx), (int)(q - z * gy), (int)z);
}

__device__ __forceinline__ int round_even(float v) { return (int)__builtin_rintf(v); }

// fastAtan2 (OpenCV 3.2 core): degrees in [0,360).
__device__ __forceinline__ float fast_atan2(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / 3.14159265358979323846);
  const float p3 = -0.3258083974640975f * (float)(180 / 3.14159265358979323846);
  const float p5 = 0.1555786518463281f * (float)(180 / 3.14159265358979323846);
  const float p7 = -0.04432655554792128f * (float)(180 / 3.14159265358979323846);
  const float eps = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON
  float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

// Deterministic float sin/cos: double-precision Cody-Waite reduction + Taylor
// polynomials, rounded once to float (same operation sequence as the CPU
// restatement).  The 23 constants sit in a constant-memory
// table: a few wide scalar loads instead of two s_mov_b32 per double on the
// (scalar-issue-bound) describe path.  x - c is x + (-c) exactly, so the table
// holds the polynomial coefficients with their signs.
// K: the 23 constants in this order (extract.hip's c_sincos).
__device__ __forceinline__ void sincos_det(float xf, const double* __restrict__ K, float* s_out, float* c_out) {
  const double x = (double)xf;
  double kd = __builtin_rint(x * K[0]);
  int q = (int)kd;
  double r = (x - kd * K[1]) - kd * K[2];
  double r2 = r * r;
  double ps = K[3];
#pragma unroll
  for (int i = 4; i < 13; i++) ps = ps * r2 + K[i];
  double sr = r + r * (r2 * ps);
  double pc = K[13];
#pragma unroll
  for (int i = 14; i < 23; i++) pc = pc * r2 + K[i];
  double cr = 1.0 + r2 * pc;
  double s, c;
  switch (q & 3) {
    case 0: s = sr; c = cr; break;
    case 1: s = cr; c = -sr; break;
    case 2: s = -sr; c = -cr; break;
    default: s = -cr; c = sr; break;
  }
  *s_out = (float)s;
  *c_out = (float)c;
}

// Hamming distance of two 256-bit descriptors held as 4 x u64.
__device__ __forceinline__ int hamming256(const uint64_t a[4], const uint64_t b[4]) {
  return __popcll(a[0] ^ b[0]) + __popcll(a[1] ^ b[1]) + __popcll(a[2] ^ b[2]) + __popcll(a[3] ^ b[3]);
}

// Wave (64-lane) reductions.
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

}  // namespace orbx
