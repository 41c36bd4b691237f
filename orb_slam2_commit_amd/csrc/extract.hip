// extract.hip -- ORB extraction (ORBextractor::operator(), src/ORBextractor.cc:1138-1211)
// as a batched chain of gfx950 kernels.  One launch per stage covers every
// image of the batch:
//
//   k_resize   x(nlevels-1)  ComputePyramid            src/ORBextractor.cc:1215-1250
//   k_fast                   per-cell FAST + fallback  src/ORBextractor.cc:843-915
//   k_octree                 DistributeOctTree         src/ORBextractor.cc:562-815
//   k_describe               IC_Angle + rBRIEF on the blurred level + scale
//                                                      src/ORBextractor.cc:77-152,1186-1207
//   k_blur                   whole-level GaussianBlur 7x7 s=2 into 8 x 16-B tiles (k_describe samples them)
//
// Integer/byte work throughout (HBM-bound); the only float math is the
// orientation/rotation and it is compiled without FP contraction so it rounds
// exactly like the CPU path.
#include <hip/hip_runtime.h>

#include <utility>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_prof.h"

namespace orbx {

__constant__ float c_pattern_f[1024] = {  // bit_pattern_31_ as floats (exact small integers)
#include "brief_pattern_31.inc"
};
// IC_Angle's circle (umax, src/ORBextractor.cc:77-105) as per-lane byte masks over the 31x31
// box: lane = (row r = lane >> 1, half h = lane & 1) keeps byte b (column 16h + b) iff that
// column is inside row r - 15's span; lanes 62, 63 keep nothing
__constant__ uint4 c_icmask[64];
// sincos_det constants (orbx_device.h); external linkage keeps them loads, not folded immediates
__constant__ double c_sincos[23] = {
    6.36619772367581382433e-01,  // 2/pi
    1.57079632673412561417e+00,  // pi/2 hi
    6.07710050650619224932e-11,  // pi/2 lo
    1.0 / 51090942171709440000.0, -1.0 / 121645100408832000.0, 1.0 / 355687428096000.0,
    -1.0 / 1307674368000.0,       1.0 / 6227020800.0,           -1.0 / 39916800.0,
    1.0 / 362880.0,               -1.0 / 5040.0,                1.0 / 120.0,
    -1.0 / 6.0,  // sin: x^19 .. x^3
    1.0 / 2432902008176640000.0,  -1.0 / 6402373705728000.0,    1.0 / 20922789888000.0,
    -1.0 / 87178291200.0,         1.0 / 479001600.0,            -1.0 / 3628800.0,
    1.0 / 40320.0,                -1.0 / 720.0,                 1.0 / 24.0,
    -0.5};  // cos: x^20 .. x^2


constexpr int BS = 256;

typedef float float2v __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------- block scan
// Exclusive scan of a[0..n) in LDS (in place); returns the total. All NT threads call.
// Two barriers: after the wave totals are published every thread adds up the
// NT/64 totals below its own wave itself (no serial pass + second barrier);
// the trailing barrier orders the in-place writes before any other reader.
template <int NT, class T>
__device__ T block_scan_excl(T* a, int n) {
  __shared__ T wsum[NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = (n + NT - 1) / NT;
  const int b = tid * chunk, e = min(n, b + chunk);
  T local = 0;
  for (int i = b; i < e; i++) local += a[i];
  T incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  T before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    const T t = wsum[w];
    before += w < wid ? t : 0;
    total += t;
  }
  T run = before + incl - local;
  for (int i = b; i < e; i++) {
    const T v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

template <int NT>
__device__ int block_exclusive_scan(int* a, int n) {
  return block_scan_excl<NT, int>(a, n);
}

template <int NT>
__device__ int block_sum(int v) {
  __shared__ int red[NT / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int s = 0;
  for (int w = 0; w < NT / 64; w++) s += red[w];
  __syncthreads();
  return s;
}

// ------------------------------------------------------------ LDS staging
// Copy an nrows x ncols byte window (row stride `stride`, any alignment) into
// LDS (row stride ls).  Every load is an aligned dword and all MAXK loads of a
// thread are issued before the first LDS write, so the window costs one
// memory latency instead of one per row.  Needs ncols+6 <= 4*dwpr and the
// dword-rounded span to stay inside the buffer (true for level windows that
// start >= 3 bytes into a row and end >= 3 bytes before its end).
template <int MAXK>
__device__ __forceinline__ void window_to_lds(const uint8_t* base, size_t stride, int nrows, int ncols, uint8_t* lds,
                                              int ls, int tid, int nth) {
  const int dwpr = (ncols + 6) / 4 + 1;
  const int total = nrows * dwpr;
  uint32_t v[MAXK];
  int rr[MAXK], cc[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; k++) {
    const int q = tid + k * nth;
    v[k] = 0;
    rr[k] = -1;
    cc[k] = 0;
    if (q < total) {
      const int r = q / dwpr, j = q - r * dwpr;
      const uintptr_t a = (uintptr_t)(base + (size_t)r * stride);
      const int sh = (int)(a & 3);
      if (4 * j < sh + ncols) {
        v[k] = *((const uint32_t*)(a & ~(uintptr_t)3) + j);
        rr[k] = r;
        cc[k] = 4 * j - sh;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXK; k++) {
    if (rr[k] < 0) continue;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int c = cc[k] + b;
      if (c >= 0 && c < ncols) lds[rr[k] * ls + c] = (uint8_t)(v[k] >> (8 * b));
    }
  }
}

// ------------------------------------------------------------------ resize
// cv::resize INTER_LINEAR 8U (OpenCV 3.2 fixed point, coefficient tables built
// on the host exactly as resizeGeneric_ does).  One block per 128x16 output
// tile, in three LDS phases:
//   1. the tile's source footprint (rows sy0(first)..sy1(last), cols
//      sx0(first)..sx1(last)) arrives as 16-B buffer loads at the unaligned row
//      positions, stored to 16-B aligned LDS rows (byte loads only for a chunk
//      straddling the level's last byte);
//   2. the horizontal pass once per footprint row and output column:
//      (S[sx0]*a0 + S[sx1]*a1) >> 4 as int16 (shared by the <= 2 output rows that
//      read each source row);
//   3. the vertical pass for 4 output columns per item:
//      ((b0*h0)>>16 + (b1*h1)>>16 + 2) >> 2 with v_mul_hi_u32_u24(b<<8, h<<8), packed
//      into one dword store.
__global__ __launch_bounds__(BS) void k_resize(const Geometry* __restrict__ G, const ResizeX* __restrict__ xt,
                                               const ResizeY* __restrict__ yt, BatchPtrs B, int l) {
  extern __shared__ __align__(16) uint8_t rz_smem[];
  const LevelGeom& L = G->lv[l];
  const LevelGeom& S = G->lv[l - 1];
  const int3 bi = xcd_block3();
  const int img = bi.z, tid = threadIdx.x;
  const int ox0 = bi.x * kRzTW, oy0 = bi.y * kRzTH;
  const int nx = min(kRzTW, L.w - ox0), ny = min(kRzTH, L.h - oy0);
  const ResizeX* X = xt + L.xtab_off + ox0;
  const ResizeY* Y = yt + L.ytab_off + oy0;
  const int cx0 = X[0].sx0, span = X[nx - 1].sx1 - cx0 + 1;
  const int ry0 = Y[0].sy0, nrows = Y[ny - 1].sy1 - ry0 + 1;
  const int stride = G->rz_stride;
  uint8_t* tin = rz_smem;
  int16_t* hb = (int16_t*)(rz_smem + G->rz_rows * stride);  // [rows][kRzTW]
  const uint8_t* src = level_ptr(*G, B, img, l - 1);
  const int swh = S.w * S.h;
  // the coefficient entries this thread needs later load first, beside the footprint: every
  // global load of the block is then in flight before the first wait (they used to trail the
  // barriers, one round trip each)
  const int hc = tid & (kRzTW - 1);
  const ResizeX xc = X[hc < nx ? hc : 0];
  constexpr int kVIt = kRzTH * (kRzTW / 4) / BS;  // vertical items per thread
  ResizeY yv[kVIt];
#pragma unroll
  for (int k = 0; k < kVIt; k++) {
    const int i = (tid + k * BS) / (kRzTW / 4);
    yv[k] = Y[i < ny ? i : 0];
  }
  // 1. footprint -> LDS: lane = (row, 16-B chunk) with a power-of-two lane count per row (the
  //    widest span's chunks; no division), all of a thread's chunk loads issued before their stores
  {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, swh, 0x00020000);
    const int nch = (span + 15) >> 4;
    const int lc = G->rz_lc;  // log2(chunk lanes per row)
    const int c = tid & ((1 << lc) - 1), r0 = tid >> lc, rstep = BS >> lc;
    constexpr int kRzLd = (kRzMaxRows + 15) / 16;  // >= rows per thread when >= 16 rows per step
    uint4 v[kRzLd];
#pragma unroll
    for (int u = 0; u < kRzLd; u++) {
      const int r = r0 + u * rstep;
      const int o = (ry0 + r) * S.w + cx0 + 16 * c;
      v[u] = make_uint4(0, 0, 0, 0);
      if (r < nrows && c < nch) {
        if (o + 16 <= swh) {
          const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
          v[u] = make_uint4(t[0], t[1], t[2], t[3]);
        } else {  // last bytes of the level: byte loads, each range-checked (outside -> 0, never used)
          uint32_t w4[4] = {0, 0, 0, 0};
#pragma unroll
          for (int b = 0; b < 16; b++)
            w4[b >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, o + b, 0, 0) << (8 * (b & 3));
          v[u] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kRzLd; u++) {
      const int r = r0 + u * rstep;
      if (r < nrows && c < nch) *(uint4*)&tin[r * stride + 16 * c] = v[u];
    }
  }
  __syncthreads();
  // 2. horizontal pass: thread = one output column, rows strided by BS / kRzTW
  if (hc < nx) {
    const int s0 = xc.sx0 - cx0, s1 = xc.sx1 - cx0, a0 = xc.a0, a1 = xc.a1;
    // (the first row is wave-uniform: a scalar loop, no exec-mask bookkeeping per row)
    for (int r = __builtin_amdgcn_readfirstlane(tid / kRzTW); r < nrows; r += BS / kRzTW) {
      const uint8_t* t = tin + r * stride;
      hb[r * kRzTW + hc] = (int16_t)((t[s0] * a0 + t[s1] * a1) >> 4);
    }
  }
  __syncthreads();
  // 3. vertical pass: item = (output row, group of 4 columns)
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(B.pyr + (size_t)img * G->pyr_bytes + L.off), (short)0, L.w * L.h, 0x00020000);
#pragma unroll
  for (int k = 0; k < kVIt; k++) {
    const int it = tid + k * BS;
    const int i = it / (kRzTW / 4), g = it - i * (kRzTW / 4);
    if (i >= ny || 4 * g >= nx) continue;
    const ResizeY y = yv[k];
    // (b * h) >> 16 as v_mul_hi_u32_u24(b << 8, h << 8): both factors stay below 2^24 (b <= 2048,
    // 0 <= h <= 32640), so the full-rate 24-bit high multiply gives the same bits as the
    // quarter-rate v_mul_hi_u32(b << 16, h); h << 8 comes straight out of its packed pair (v_perm)
    const uint32_t B0 = (uint32_t)y.b0 << 8, B1 = (uint32_t)y.b1 << 8;
    const uint2 p0 = *(const uint2*)&hb[(y.sy0 - ry0) * kRzTW + 4 * g];
    const uint2 p1 = *(const uint2*)&hb[(y.sy1 - ry0) * kRzTW + 4 * g];
    constexpr uint32_t kLo = 0x0C01000Cu, kHi = 0x0C03020Cu;  // bytes 0-1 / 2-3 -> bits 8..23
    const uint32_t h0[4] = {__builtin_amdgcn_perm(0u, p0.x, kLo), __builtin_amdgcn_perm(0u, p0.x, kHi),
                            __builtin_amdgcn_perm(0u, p0.y, kLo), __builtin_amdgcn_perm(0u, p0.y, kHi)};
    const uint32_t h1[4] = {__builtin_amdgcn_perm(0u, p1.x, kLo), __builtin_amdgcn_perm(0u, p1.x, kHi),
                            __builtin_amdgcn_perm(0u, p1.y, kLo), __builtin_amdgcn_perm(0u, p1.y, kHi)};
    auto mulhi24 = [](uint32_t x, uint32_t z) {
      return (uint32_t)(((uint64_t)(x & 0xFFFFFFu) * (z & 0xFFFFFFu)) >> 32);
    };
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t v = (mulhi24(B0, h0[j]) + mulhi24(B1, h1[j]) + 2) >> 2;
      packed |= v << (8 * j);
    }
    const int o = (oy0 + i) * L.w + ox0 + 4 * g;
    if (4 * g + 4 <= nx) {
      __builtin_amdgcn_raw_buffer_store_b32(packed, rd, o, 0, 0);
    } else {
      for (int j = 0; j < nx - 4 * g; j++) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(packed >> (8 * j)), rd, o + j, 0, 0);
    }
  }
}

// ----------------------------------------------------------------- blur
// GaussianBlur(7x7, sigma=2, BORDER_REFLECT_101), OpenCV 3.2 8U fixed point:
// integer kernel {k0..k6} (x256), exact integer row+column sums, then
// rint(acc/65536) on SIMD column groups (x < w&~3) and (acc+2^15)>>16 on the
// scalar tail; saturate to u8 (the integer kernel {18,34,49,55,49,34,18} sums to 257).  128x128 output tile per block, staged in LDS.
__constant__ int c_gauss[7];

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

// Tile of kBlurTileW x kBlurTileH (128 x 128) outputs per 256-thread block.
// Input tile col 0 = x0-4 so that every 4-output group reads 3 aligned LDS
// dwords.  The tile arrives as 16-B buffer loads at the (unaligned) source row
// positions, stored to 16-B aligned LDS rows (rows reflected per row index;
// the <= 3 reflected columns each side are patched from LDS afterwards).
// Thread = 4 columns x a 16-row strip: row sums (byte dot products) go into a
// 7-row register window that slides down the strip; the column taps are exact
// packed-f32 FMAs on the row sums with the weights pre-scaled by 2^-16 (every
// partial sum is an integer multiple of 2^-16 below 2^8, exact in f32), rounded
// by the 1.5*2^23 add and packed by byte permutes: ~10 VALU per output (18.6
// with per-column byte aligns, v_rndne / v_med3 / v_cvt_pk_u8 per output; the
// kernel is VALU-issue-bound).  A strip's 16 packed output dwords stay in
// registers until the whole tile is done, then go through the (no longer
// needed) input tile in LDS in the tiled blurred-level order (8x16-B tiles)
// and out as whole 128-B tiles of b128 stores.  7 waves per SIMD: 68 VGPRs,
// no scratch (8 spills 12 B per lane for the same time, profiles/r04/ab_blur_tiled.txt).
constexpr int kBIn = kBlurTileW + 16;  // input tile row stride (bytes, 16-B multiple)
constexpr int kBStrip = 16;            // output rows per thread
#ifndef ORBX_BLUR_WPE
#define ORBX_BLUR_WPE 7
#endif
__global__ __launch_bounds__(BS, ORBX_BLUR_WPE) void k_blur(const Geometry* __restrict__ G, const int* __restrict__ tile_level,
                                             BatchPtrs B) {
  constexpr int TR = kBlurTileH + 6;
  __shared__ __align__(16) uint8_t tin[(TR + 1) * kBIn];
  const int2 bi = xcd_block2();
  const int tile = bi.x, img = bi.y, tid = threadIdx.x;
  const int l = tile_level[tile];
  const LevelGeom& L = G->lv[l];
  const int t = tile - L.tile_begin;
  const int x0 = (t % L.tiles_x) * kBlurTileW, y0 = (t / L.tiles_x) * kBlurTileH;
  const uint8_t* src = level_ptr(*G, B, img, l);
  uint8_t* dst = B.blur + (size_t)img * G->blur_bytes + L.boff;
  const int w = L.w, h = L.h, bs = L.bstride;
  // input tile rows y0-3 .. y0+H+2 (REFLECT_101), cols x0-4 .. x0+W+11
  {
    constexpr int CPR = kBIn / 16, NQ = TR * CPR, KQ = (NQ + BS - 1) / BS;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, w * h, 0x00020000);
    uint32_t v[KQ][4];
#pragma unroll
    for (int k = 0; k < KQ; k++) {
      const int q = k * BS + tid;
      const int ty = q / CPR, j = q - ty * CPR;
      v[k][0] = v[k][1] = v[k][2] = v[k][3] = 0;
      if (q < NQ) {
        const int sy = reflect101(y0 - 3 + ty, h);
        const int o = sy * w + x0 - 4 + 16 * j;
        if (o >= 0 && o + 16 <= w * h) {
          const auto r = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
          v[k][0] = r[0];
          v[k][1] = r[1];
          v[k][2] = r[2];
          v[k][3] = r[3];
        } else {
          // a chunk straddling the level's first or last byte (a range check covers the whole
          // 16-B access): byte loads, each range-checked on its own (outside -> 0, patched below)
#pragma unroll
          for (int b = 0; b < 16; b++)
            v[k][b >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, o + b, 0, 0) << (8 * (b & 3));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KQ; k++) {
      const int q = k * BS + tid;
      const int ty = q / CPR, j = q - ty * CPR;
      if (q < NQ) *(uint4*)&tin[ty * kBIn + 16 * j] = make_uint4(v[k][0], v[k][1], v[k][2], v[k][3]);
    }
  }
  const bool left = x0 < 3, right = x0 + kBlurTileW + 3 > w;
  if (left || right) {
    // patch the reflected columns x in [-3, -1] and [w, w+2] of every tile row (read after a barrier:
    // the source columns are inside the row and were stored by other threads)
    __syncthreads();
    // two-phase (read all, then write) so no patched byte feeds another patch
    const int nfix = TR * 6;
    uint8_t vals[(TR * 6 + BS - 1) / BS];
#pragma unroll
    for (int k = 0; k < (TR * 6 + BS - 1) / BS; k++) {
      const int q = k * BS + tid;
      vals[k] = 0;
      if (q < nfix) {
        const int ty = q / 6, s = q - ty * 6;
        const int x = s < 3 ? -3 + s : w + (s - 3);
        const int c = x - (x0 - 4);
        if (c >= 0 && c < kBIn && (s < 3 ? left : right)) vals[k] = tin[ty * kBIn + reflect101(x, w) - (x0 - 4)];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < (TR * 6 + BS - 1) / BS; k++) {
      const int q = k * BS + tid;
      if (q < nfix) {
        const int ty = q / 6, s = q - ty * 6;
        const int x = s < 3 ? -3 + s : w + (s - 3);
        const int c = x - (x0 - 4);
        if (c >= 0 && c < kBIn && (s < 3 ? left : right)) tin[ty * kBIn + c] = vals[k];
      }
    }
  }
  __syncthreads();
  const int g = tid & (kBlurTileW / 4 - 1);
  const int ys = (tid / (kBlurTileW / 4)) * kBStrip;  // strip's first output row in the tile
  const int xg = x0 + 4 * g;
  // (threads past the level compute nothing but stay for the barriers of the tile write-out)
  const bool active = xg < w && y0 + ys < h;
  uint32_t outv[kBStrip];
  const uint32_t k0 = c_gauss[0], k1 = c_gauss[1], k2 = c_gauss[2], k3 = c_gauss[3];
  // horizontal taps as byte dot products (exact integers, weights < 256) straight on the three
  // aligned dwords [a b c] = tile bytes 4g .. 4g+11: output col j of the group takes bytes
  // j+1 .. j+7, i.e. ten v_dot4_u32_u8 with the taps pre-shifted into the word each byte sits in
  // (no byte-align step).  The accumulator starts at 0x4B000000, so the sum comes out as the f32
  // bits of 2^23 + s (s <= 257*255 < 2^23) and one packed subtract per two columns converts it.
  auto W4 = [](uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) { return b0 | b1 << 8 | b2 << 16 | b3 << 24; };
  const uint32_t wa0 = W4(0, k0, k1, k2), wb0 = W4(k3, k2, k1, k0);
  const uint32_t wa1 = W4(0, 0, k0, k1), wb1 = W4(k2, k3, k2, k1), wc1 = W4(k0, 0, 0, 0);
  const uint32_t wa2 = W4(0, 0, 0, k0), wb2 = W4(k1, k2, k3, k2), wc2 = W4(k1, k0, 0, 0);
  const uint32_t wb3 = W4(k0, k1, k2, k3), wc3 = W4(k2, k1, k0, 0);
  const float f0 = (float)k0 * (1.f / 65536.f), f1 = (float)k1 * (1.f / 65536.f), f2 = (float)k2 * (1.f / 65536.f),
              f3 = (float)k3 * (1.f / 65536.f);
  const float2v F0 = {f0, f0}, F1 = {f1, f1}, F2 = {f2, f2}, F3 = {f3, f3};
  const float2v two23 = {8388608.0f, 8388608.0f}, magic = {12582912.0f, 12582912.0f};
  // row sums (<= 257*255, exact in f32) of output cols xg..xg+3 on tile row ty, as two f32 pairs
  auto rowsum = [&](int ty, float2v (&o)[2]) {
    const uint32_t* r32 = (const uint32_t*)&tin[ty * kBIn + 4 * g];
    const uint32_t a = r32[0], b = r32[1], c = r32[2];
    constexpr uint32_t bias = 0x4B000000u;  // f32 2^23
    const uint32_t s0 = __builtin_amdgcn_udot4(b, wb0, __builtin_amdgcn_udot4(a, wa0, bias, false), false);
    const uint32_t s1 = __builtin_amdgcn_udot4(
        c, wc1, __builtin_amdgcn_udot4(b, wb1, __builtin_amdgcn_udot4(a, wa1, bias, false), false), false);
    const uint32_t s2 = __builtin_amdgcn_udot4(
        c, wc2, __builtin_amdgcn_udot4(b, wb2, __builtin_amdgcn_udot4(a, wa2, bias, false), false), false);
    const uint32_t s3 = __builtin_amdgcn_udot4(c, wc3, __builtin_amdgcn_udot4(b, wb3, bias, false), false);
    o[0] = (float2v){__uint_as_float(s0), __uint_as_float(s1)} - two23;
    o[1] = (float2v){__uint_as_float(s2), __uint_as_float(s3)} - two23;
  };
  // 7-row ring indexed by compile-time (r + i) % 7 in the unrolled loop: no register moves
  float2v win[7][2];
  if (active) {
#pragma unroll
  for (int r = 0; r < 6; r++) rowsum(ys + r, win[r]);
  const int simd_w = w & ~3;
  const bool all_simd = xg + 3 < simd_w;  // the whole group takes the SSE2 rounding
  // wave-uniform: the per-row tail fix-up below is a scalar branch (no exec-mask juggling per row)
  const bool wave_tail = __builtin_amdgcn_ballot_w64(!all_simd) != 0;

#pragma unroll
  for (int r = 0; r < kBStrip; r++) {
    rowsum(ys + r + 6, win[(r + 6) % 7]);
    // column taps on packed f32 pairs, each element exactly the scalar chain
    // fma(f3, w3, fma(f2, w2+w4, fma(f1, w1+w5, f0*(w0+w6)))) = acc / 2^16 (integer sums below
    // 2^24 scaled by a power of two); + 1.5*2^23 rounds it half-to-even (the SSE2 groups'
    // rint), leaving the integer in the low bits
    float2v acc[2];
    uint32_t rb[4];
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
      const float2v w0 = win[r % 7][hh], w1 = win[(r + 1) % 7][hh], w2 = win[(r + 2) % 7][hh],
                    w3 = win[(r + 3) % 7][hh], w4 = win[(r + 4) % 7][hh], w5 = win[(r + 5) % 7][hh],
                    w6 = win[(r + 6) % 7][hh];
      acc[hh] = __builtin_elementwise_fma(
          F3, w3, __builtin_elementwise_fma(F2, w2 + w4, __builtin_elementwise_fma(F1, w1 + w5, F0 * (w0 + w6))));
      const float2v rr = acc[hh] + magic;
      rb[2 * hh] = __float_as_uint(rr.x);
      rb[2 * hh + 1] = __float_as_uint(rr.y);
    }
    // low halves as u16 pairs, saturated to 255 (the kernel sums to 257), then the low bytes
    u16x2 p01 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(rb[1], rb[0], 0x05040100u));
    u16x2 p23 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(rb[3], rb[2], 0x05040100u));
    const u16x2 cap = {255, 255};
    p01 = __builtin_elementwise_min(p01, cap);
    p23 = __builtin_elementwise_min(p23, cap);
    uint32_t packed = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, p23), __builtin_bit_cast(uint32_t, p01), 0x06040200u);
    if (wave_tail) {
      // the row's scalar tail (x >= w & ~3): (acc + 2^15) >> 16, selected per lane and column
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const float aj = j == 0 ? acc[0].x : j == 1 ? acc[0].y : j == 2 ? acc[1].x : acc[1].y;
        const int v = min(((int)(aj * 65536.f) + (1 << 15)) >> 16, 255);
        const uint32_t fixed = (packed & ~(0xFFu << (8 * j))) | ((uint32_t)v << (8 * j));
        packed = xg + j >= simd_w ? fixed : packed;
      }
    }
    outv[r] = packed;
  }
  }  // active
  // Write-out in the level's tile layout (8 rows x 16 bytes = 128-B tiles, the layout k_describe
  // gathers from): the outputs go to LDS (the input tile is no longer read) in tile order, then
  // leave as whole 128-B lines, 16 B per lane: the block's 128 x 128 outputs are 16 tile rows of
  // 8 consecutive tiles (1 KB each).  Columns past w and rows past h land in the level's padding.
  __syncthreads();
  if (active) {
#pragma unroll
    for (int r = 0; r < kBStrip; r++) {
      const int yr = ys + r, c = 4 * g;
      *(uint32_t*)&tin[((yr >> 3) * (kBlurTileW / 16) + (c >> 4)) * 128 + (yr & 7) * 16 + (c & 15)] = outv[r];
    }
  }
  __syncthreads();
  {
    const int ntx = bs >> 4, nty = (h + 7) >> 3;
    const int tx0 = x0 >> 4, ty0 = y0 >> 3;
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, nty * ntx * 128, 0x00020000);
    constexpr int kTiles = (kBlurTileW / 16) * (kBlurTileH / 8), kChunks = kTiles * 8;  // 16-B chunks
#pragma unroll
    for (int k = 0; k < kChunks / BS; k++) {
      const int q = tid + k * BS, t = q >> 3, tr = t / (kBlurTileW / 16), tc = t - tr * (kBlurTileW / 16);
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = *(const u32x4*)&tin[q * 16];
      if (tx0 + tc < ntx && ty0 + tr < nty)
        __builtin_amdgcn_raw_buffer_store_b128(v, rd, (uint32_t)(((ty0 + tr) * ntx + tx0 + tc) * 128 + (q & 7) * 16), 0, 0);
    }
  }
}

// ------------------------------------------------------------------- FAST
// One wavefront per kFastCPW (2) FAST cell windows, one after the other (block = 1 wave); the next
// cell's window loads are issued before the current cell's work (0.733 -> 0.726 ms per step against
// one cell per wave, profiles/r04/ab_fast_cells_per_wave.txt).
// cv::FAST(window, th, nonmax) semantics (OpenCV 3.2 FAST_t<16>): a pixel of
// the detection region is a corner at threshold t iff >= 9 contiguous ring
// pixels are all > v+t or all < v-t; its cornerScore<16> S satisfies
// corner_t <=> S >= t, so one score map serves both thresholds.  NMS is strict
// against the 8 neighbours inside the region (0 outside).  The cell runs FAST at
// iniThFAST; only if nothing survives does it run again at minThFAST (a
// wave-uniform second pass, src/ORBextractor.cc:892-900).  Survivors are written
// in row-major order.
//
// The kernel is VALU-issue-bound, so every phase is shaped for few vector
// instructions per pixel:
//   1. window -> LDS: 16-B buffer loads at the (unaligned) row positions land on
//      16-B aligned LDS rows of compile-time stride S, so every ring / map
//      access below is an LDS read with an immediate offset (no address VALU);
//   2. compass quick test (two adjacent of ring pixels 0,4,8,12 beyond t), as
//      min(max(p0,p8), max(p4,p12)) > c+t or max(min(p0,p8), min(p4,p12)) < c-t
//      (six min/max on the raw bytes; 0.855 -> 0.820 ms against the earlier packed
//      sign-bit form), survivors compacted by ballot rank as tile offsets e = y*S + x
//      (the 7x7 neighbourhood's top-left);
//   3. cornerScore and the corner test in ONE pass on the compacted list:
//      ring pixel p is packed as the f16 pair (1024+p, 1279-p) (one v_mad_i32_i24:
//      bits 0x6400+p / 0x64FF-p), the 9-arc maximum of both halves is two rounds
//      of v_pk_maximum3_f16 and the minimum over the 16 arcs three rounds of
//      v_pk_minimum3_f16, giving (min_k max_arc p, 255 - max_k min_arc p), so
//      S+1 = max(v - min_k max_arc p, max_k min_arc p - v) (= cornerScore<16> + 1)
//      and corner_t <=> S+1 > t; corners are compacted in place, the map holds S+1;
//   4. NMS at iniThFAST -> count (steps 2-3 ran at iniThFAST; an empty cell repeats
//      them at minThFAST); 5. NMS at the chosen threshold -> ballot-ranked row-major
//      writes.
constexpr int kMaxCell = 60;  // wCell,hCell <= 60 (checked on the host)

__device__ __forceinline__ uint32_t pk_max3_f16(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint32_t pk_min3_f16(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// cornerScore<16> + 1 of the pixel whose 7x7 neighbourhood starts at t (row stride S): the
// ring in OpenCV's makeOffsets order, offsets relative to the top-left (centre at 3S+3)
template <int S>
__device__ __forceinline__ int ring_score1(const uint8_t* t) {
  constexpr int o[16] = {6 * S + 3, 6 * S + 4, 5 * S + 5, 4 * S + 6, 3 * S + 6, 2 * S + 6, S + 5, 4,
                         3,         2,         S + 1,     2 * S,     3 * S,     4 * S,     5 * S + 1, 6 * S + 2};
  const int v = t[3 * S + 3];
  uint32_t P[16];
#pragma unroll
  for (int k = 0; k < 16; k++) P[k] = (uint32_t)((int)t[o[k]] * -65535 + 0x64FF6400);  // (0x64FF-p)<<16 | 0x6400+p
  uint32_t M3[16], M9[16];
#pragma unroll
  for (int k = 0; k < 16; k++) M3[k] = pk_max3_f16(P[k], P[(k + 1) & 15], P[(k + 2) & 15]);
#pragma unroll
  for (int k = 0; k < 16; k++) M9[k] = pk_max3_f16(M3[k], M3[(k + 3) & 15], M3[(k + 6) & 15]);
  const uint32_t a0 = pk_min3_f16(M9[0], M9[1], M9[2]), a1 = pk_min3_f16(M9[3], M9[4], M9[5]),
                 a2 = pk_min3_f16(M9[6], M9[7], M9[8]), a3 = pk_min3_f16(M9[9], M9[10], M9[11]),
                 a4 = pk_min3_f16(M9[12], M9[13], M9[14]);
  const uint32_t R = pk_min3_f16(pk_min3_f16(a0, a1, a2), pk_min3_f16(a3, a4, M9[15]), M9[15]);
  const int a = (v + 0x6400) - (int)(R & 0xFFFF);  // v - min_k max_arc p
  const int b = (0x64FF - v) - (int)(R >> 16);     // max_k min_arc p - v
  return max(a, b);
}

#ifdef ORBX_FAST_PROBE
// probe only: the necessary condition "4 contiguous of the 8 even ring points beyond t" (a 9-arc
// always holds 4 or 5 consecutive even positions), counted on the compass survivors
template <int S>
__device__ __forceinline__ bool even8_test(const uint8_t* t, int th) {
  constexpr int o[8] = {6 * S + 3, 5 * S + 5, 3 * S + 6, S + 5, 3, S + 1, 3 * S, 5 * S + 1};
  const int v = t[3 * S + 3];
  int p[8], lo2[8], hi2[8];
#pragma unroll
  for (int k = 0; k < 8; k++) p[k] = t[o[k]];
#pragma unroll
  for (int k = 0; k < 8; k++) lo2[k] = min(p[k], p[(k + 1) & 7]), hi2[k] = max(p[k], p[(k + 1) & 7]);
  int bl = 0, bh = 255;
#pragma unroll
  for (int k = 0; k < 8; k++) bl = max(bl, min(lo2[k], lo2[(k + 2) & 7])), bh = min(bh, max(hi2[k], hi2[(k + 2) & 7]));
  return bl > v + th || bh < v - th;
}
#endif

typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s16x2(int v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ int as_int(s16x2 v) { return __builtin_bit_cast(int, v); }

__device__ __forceinline__ int lane_rank(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Phase probe (build with -DORBX_FAST_PROBE only; tools/fast_probe.py): per-phase s_memtime
// deltas of every cell wave, stored (plain vector stores, no contention) to a host-provided
// buffer of 8 words per wave, indexed img * ncells + cell.
#ifdef ORBX_FAST_PROBE
__device__ unsigned int* fast_probe_buf;
#define FAST_TS(k) const unsigned long long ts##k = __builtin_amdgcn_s_memtime()
#else
#define FAST_TS(k)
#endif

// S: LDS row stride of the window tile and the score map (multiple of 16, >= window width);
// RP: region rows per compass instruction (2 when the widest cell fits 32 lanes)
#ifndef ORBX_FAST_CPW
#define ORBX_FAST_CPW 2
#endif
constexpr int kFastCPW = ORBX_FAST_CPW;  // FAST cells per wave
template <int S, int RP>
__global__ __launch_bounds__(64) void k_fast(const Geometry* __restrict__ G, const CellInfo* __restrict__ cells,
                                             BatchPtrs B, int grp) {
  // dynamic LDS sized by the launch group's largest cell (G->fg[grp])
  extern __shared__ __align__(16) uint8_t fast_smem[];
  const int tile_bytes = G->fg[grp].tile_bytes, map_bytes = G->fg[grp].map_bytes;
  uint8_t* tile = fast_smem;
  uint8_t* smap = fast_smem + tile_bytes;
  uint16_t* list = (uint16_t*)(fast_smem + tile_bytes + map_bytes);
  const int2 bi = xcd_block2();
  const int img = bi.y, lane = threadIdx.x;
  // 1. window -> registers -> LDS: lane = (row, 16-B chunk); window pixel (r, col) lands at tile[r*S + col]
  constexpr int CPR = (S + 15) / 16, RPI = 64 / CPR;
  constexpr int KMAX = (kMaxCell + 6 + RPI - 1) / RPI;
  const int lr = lane / CPR, lj = lane - lr * CPR;
  const bool lane_ok = lr < RPI;
  // every load unconditional (a lane outside the window reads past num_records and gets zeros): no
  // branch between them, so all KMAX are in flight before the first wait
  auto load_window = [&](const CellInfo& cc, uint32_t (&w)[KMAX][4]) {
    const uint8_t* lvl =
        cc.level == 0 ? B.in + (size_t)img * B.in_pitch : B.pyr + (size_t)img * G->pyr_bytes + cc.loff;
    const uint8_t* base = lvl + (size_t)(cc.y0 - 3) * cc.lw + (cc.x0 - 3);
    const int th = cc.y1 - cc.y0 + 7;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, th * cc.lw + S, 0x00020000);
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      const int r = k * RPI + lr;
      const uint32_t off = (lane_ok && r < th) ? (uint32_t)(r * cc.lw + 16 * lj) : 0x80000000u;
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      w[k][0] = q[0];
      w[k][1] = q[1];
      w[k][2] = q[2];
      w[k][3] = q[3];
    }
  };
  // kFastCPW cells per wave, one after another; the next cell's window loads are issued before the
  // current cell's work, so their latency hides behind it
  const int cell0 = G->fg[grp].c0 + bi.x * kFastCPW, cend = G->fg[grp].c1;
  CellInfo cn = cells[cell0];
  uint32_t vn[KMAX][4];
  load_window(cn, vn);
#pragma unroll
  for (int q = 0; q < kFastCPW; q++) {
  const int cell = cell0 + q;
  if (cell >= cend) break;  // wave-uniform
  const CellInfo c = cn;
  uint32_t v[KMAX][4];
#pragma unroll
  for (int k = 0; k < KMAX; k++)
#pragma unroll
    for (int e = 0; e < 4; e++) v[k][e] = vn[k][e];
  if (q + 1 < kFastCPW && cell + 1 < cend) {
    cn = cells[cell + 1];
    load_window(cn, vn);
  }
  const int W = c.x1 - c.x0 + 1, H = c.y1 - c.y0 + 1, TH = H + 6;
  FAST_TS(0);
  if (q > 0) __syncthreads();  // the previous cell's tile / map / list reads are done
  {
    // zero the score map (its border row/column stands for "outside the region")
    for (int i = lane * 16; i < map_bytes; i += 64 * 16) *(uint4*)(smap + i) = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      const int r = k * RPI + lr;
      if (k * RPI < TH && lane_ok && r < TH) {
        if constexpr (S % 16 == 0) {
          *(uint4*)(tile + r * S + 16 * lj) = make_uint4(v[k][0], v[k][1], v[k][2], v[k][3]);
        } else {  // 8-B aligned rows: the chunk as two halves, the part past the stride dropped
          if (16 * lj + 8 <= S) *(uint2*)(tile + r * S + 16 * lj) = make_uint2(v[k][0], v[k][1]);
          if (16 * lj + 16 <= S) *(uint2*)(tile + r * S + 16 * lj + 8) = make_uint2(v[k][2], v[k][3]);
        }
      }
    }
  }
  __syncthreads();
  const int ini = min(max(G->ini_th, 0), 255), mint = min(max(G->min_th, 0), 255);
  const int ly = RP == 2 ? (lane >> 5) : 0, lx = RP == 2 ? (lane & 31) : lane;
  const int cw = lx - W;
  constexpr int QU = 8 / RP;
#ifdef ORBX_FAST_PROBE
  unsigned long long ts_mid = 0;
  int n_compass = 0, n_even8 = 0, n_corner_ini = 0;
#endif
  // 2.+3. FAST(window, th): compass quick test at th, row-major compaction of tile offsets, then
  // cornerScore + the corner test at th on the compass list, corners compacted in place and their
  // S+1 written to the map (the score does not depend on th, so a second pass at another threshold
  // rewrites the same values).  Returns the corner count.
  auto detect = [&](int th) -> int {
    int n = 0;
    for (int y0r = 0; y0r < H; y0r += QU * RP) {
      const int eb = (y0r + ly) * S + lx;
      int cv[QU], c0[QU], c4[QU], c8[QU], c12[QU];
#pragma unroll
      for (int u = 0; u < QU; u++) {
        const uint8_t* t = tile + eb + u * RP * S;
        cv[u] = t[3 * S + 3];
        c0[u] = t[6 * S + 3];
        c4[u] = t[3 * S + 6];
        c8[u] = t[3];
        c12[u] = t[3 * S];
      }
#pragma unroll
      for (int u = 0; u < QU; u++) {
        // two ADJACENT compass points beyond the threshold <=> (p0 | p8) & (p4 | p12) per
        // polarity, i.e. min(max(p0,p8), max(p4,p12)) > c+t or max(min(p0,p8), min(p4,p12)) < c-t:
        // min/max on the raw bytes, one difference per polarity
        const int hi = min(max(c0[u], c8[u]), max(c4[u], c12[u]));
        const int lo = max(min(c0[u], c8[u]), min(c4[u], c12[u]));
        const int v = max(hi - cv[u], cv[u] - lo) - (th + 1);  // >= 0 <=> compass hit
        // lane inside the region: (col - W) and (row - H) both negative, and v >= 0
        const bool hit = (~v & cw & (y0r + u * RP + ly - H)) < 0;
        const uint64_t m = __ballot(hit);
        if (hit) list[n + lane_rank(m)] = (uint16_t)(eb + u * RP * S);
        n += __popcll(m);
      }
    }
    __syncthreads();
#ifdef ORBX_FAST_PROBE
    if (th == ini) ts_mid = __builtin_amdgcn_s_memtime(), n_compass = n;
#endif
    int nc = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
      const int i = i0 + lane;
      int e = 0, sc1 = 0;
      bool corner = false;
      if (i < n) {
        e = list[i];
        sc1 = ring_score1<S>(tile + e);
        corner = sc1 > th;
      }
#ifdef ORBX_FAST_PROBE
      if (th == ini) n_even8 += __popcll(__ballot(i < n && even8_test<S>(tile + e, th)));
#endif
      const uint64_t m = __ballot(corner);
      __syncthreads();
      if (corner) {
        list[nc + lane_rank(m)] = (uint16_t)e;
        smap[e + S + 1] = (uint8_t)sc1;
      }
      nc += __popcll(m);
    }
    __syncthreads();
    return nc;
  };
  // strict NMS inside the region; the map's zero border stands for "outside"
  auto keep = [&](int e, int thr) -> bool {  // thr = t + 1 in map units (S + 1)
    const uint8_t* m = smap + e;              // centre at m[S + 1]
    const int s = m[S + 1];
    const int n0 = m[0], n1 = m[1], n2 = m[2], n3 = m[S], n4 = m[S + 2], n5 = m[2 * S], n6 = m[2 * S + 1],
              n7 = m[2 * S + 2];
    // a neighbour beats the centre iff nv >= thr and nv >= s: one max over the eight
    const int mx = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
    const bool lost = mx >= max(thr, s);
    return s >= thr && s > 1 && !lost;
  };
  // FAST at iniThFAST only (src/ORBextractor.cc:892): the map then holds exactly the corners at
  // iniThFAST, which is all NMS at iniThFAST looks at (a weaker neighbour never beats a centre)
  FAST_TS(1);
  int nc = detect(ini);
  FAST_TS(2);
#ifdef ORBX_FAST_PROBE
  n_corner_ini = nc;
#endif
  // 4. survivors at iniThFAST (verdict kept in bit 15 of the list entry)
  int cnt = 0;
  for (int i0 = 0; i0 < nc; i0 += 64) {
    const int i = i0 + lane;
    bool k = false;
    if (i < nc) {
      const int e = list[i];
      k = keep(e, ini + 1);
      if (k) list[i] = (uint16_t)(e | 0x8000);
    }
    cnt += __popcll(__ballot(k));
  }
  // an empty cell runs FAST(window, minThFAST) (src/ORBextractor.cc:894-900): a wave-uniform
  // second pass, taken by ~10 % of the cells on the bench images
  FAST_TS(3);
  if (cnt == 0 && mint != ini) nc = detect(mint);
  FAST_TS(4);
  const int thr = (cnt > 0 ? ini : mint) + 1;
  // 5. row-major writes at the chosen threshold
  // survivor p goes to the cell's inline slot p (p < kin) or overflow slot p - kin (cell_slot)
  // (as one offset, no select between two pointers: the pointer select made the compiler give up
  // duplicating the cell loop, +7 % VALU per wave)
  uint32_t* const out = B.cand + (size_t)img * G->cand_total + c.ovf_off - c.kin;
  uint32_t* const out_in = B.cand + (size_t)img * G->cand_total + c.cand_off;
  const int kin = c.kin;
  int pos = 0;
  for (int i0 = 0; i0 < nc; i0 += 64) {
    const int i = i0 + lane;
    int e = 0;
    bool k = false;
    if (i < nc) {
      const int le = list[i];
      e = le & 0x7FFF;
      k = cnt > 0 ? (le >> 15) != 0 : keep(e, thr);  // at iniThFAST the verdict is already known
    }
    const uint64_t m = __ballot(k);
    if (k) {
      const int p = pos + lane_rank(m);
      const int y = e / S, x = e - y * S;
      if (p < c.cap)
      {
        const uint32_t v = ((uint32_t)(smap[e + S + 1] - 1) << 24) | ((uint32_t)(c.y0 + y) << 12) | (uint32_t)(c.x0 + x);
        if (p < kin) out_in[p]= v; else out[p] = v;
      }
    }
    pos += __popcll(m);
  }
  if (lane == 0) B.cell_count[(size_t)img * G->ncells + cell] = min(pos, c.cap);
#ifdef ORBX_FAST_PROBE
  FAST_TS(5);
  if (lane < 8 && fast_probe_buf) {
    // word 6: empty-cell flag | corners at iniThFAST << 1 | survivors at iniThFAST << 16;
    // word 7: compass survivors | even-8 survivors << 16 (both at iniThFAST)
    const unsigned long long t[8] = {ts1 - ts0, ts_mid - ts1, ts2 - ts_mid, ts3 - ts2, ts4 - ts3, ts5 - ts4,
                                     (unsigned long long)((cnt == 0) | (n_corner_ini << 1) | (cnt << 16)),
                                     (unsigned long long)(n_compass | (n_even8 << 16))};
    fast_probe_buf[((size_t)img * G->ncells + cell) * 8 + lane] = (unsigned int)t[lane];
  }
#endif
  }  // cells of this wave
}

// ----------------------------------------------------------------- octree
// One block per (level, image).  Restates DistributeOctTree as rounds over an
// explicit node list held in LDS (list order == the reference's std::list
// order): each round splits the selected nodes, pushes their non-empty
// children to the front (reversed, as successive push_front do) and keeps the
// rest in order.  Keypoints never move; each keeps the index of its node.
// Phase 2 sorts (size, creation sequence) descending -- the reference sorts
// by (size, heap pointer); DESIGN.md §Parity documents the tie-break.
struct OctSmem {
  int16_t* x0;  // [2*NC] double-buffered node list
  int16_t* y0;
  int16_t* x1;
  int16_t* y1;
  int* cnt;
  int* seq;
  int* ccnt;       // [NC*4]
  int16_t* cidx;   // [NC*4]
  int16_t* nidx;   // [NC]
  int* sa;         // [NC]
  int* sb;         // [NC]
  uint64_t* key;   // [NP2] (also best)
  int* cpre;       // [cell_cap+1]
  int* ctrl;       // [8]
  uint32_t* kp;    // [kcap] candidate positions
  uint16_t* kn;    // [kcap] candidate node | digit << 14
};

__host__ __device__ inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

__host__ __device__ inline size_t octree_smem_bytes(int NC, int cell_cap, int kcap) {
  const int NP2 = next_pow2(NC);
  size_t b = 0;
  b += 2 * 4 * NC * sizeof(int16_t);
  b += 2 * 2 * NC * sizeof(int);
  b += NC * 4 * sizeof(int);
  b += NC * 4 * sizeof(int16_t);
  b += NC * sizeof(int16_t);
  b += 2 * NC * sizeof(int);
  b = (b + 7) & ~(size_t)7;
  b += (size_t)NP2 * sizeof(uint64_t);
  b += (cell_cap + 1) * sizeof(int);
  b += 8 * sizeof(int);
  b += (size_t)kcap * (sizeof(uint32_t) + sizeof(uint16_t));
  return b;
}

// octree block size NT per launch group (Geometry::og): the split rounds loop over every candidate
// of the level (thousands at levels 0-2: 512 threads there, 512 beat 256 for a single launch, 0.42
// -> 0.38 ms per 256 frames, and 1024 halved the resident blocks per CU, 0.71); the upper levels
// run as 256-thread blocks with a smaller LDS footprint, so more of them share a CU
// phase 2 sorts up to this many splittable nodes by rank (M^2 / NT compares per thread), more by
// the bitonic network
constexpr int kOctRankSortMax = 1024;

template <int NT>
__device__ __forceinline__ void bitonic_sort_desc(uint64_t* k, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n / 2; i += NT) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t a = k[lo], b = k[hi];
        if (desc ? (a < b) : (a > b)) {
          k[lo] = b;
          k[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// Per-candidate state across the split rounds: the packed position (score<<24 |
// y<<12 | x, level-relative) and node | child digit<<14.  The first G->oct_kcap
// candidates of a level live in LDS for the whole kernel (sized on the host so
// the block still fits three per CU); only a level with more candidates keeps
// the rest in the global kpos/knode scratch.  Every round walks all candidates
// of the level, so keeping them out of memory removes the per-round L2/HBM
// round trips (counter traffic 240 -> ~100 MB per 512 images).
struct OctCands {
  uint32_t* lpos;
  uint16_t* lnd;
  int kcap;
  uint32_t* gpos;
  uint32_t* gnd;
  __device__ __forceinline__ uint32_t pos(int k) const { return k < kcap ? lpos[k] : gpos[k]; }
  __device__ __forceinline__ uint32_t nd(int k) const { return k < kcap ? (uint32_t)lnd[k] : gnd[k]; }
  __device__ __forceinline__ void set(int k, uint32_t p, uint32_t n) const {
    if (k < kcap) {
      lpos[k] = p;
      lnd[k] = (uint16_t)n;
    } else {
      gpos[k] = p;
      gnd[k] = n;
    }
  }
  __device__ __forceinline__ void set_nd(int k, uint32_t n) const {
    if (k < kcap) lnd[k] = (uint16_t)n; else gnd[k] = n;
  }
};

template <int NT, class F>
__device__ __forceinline__ void oct_cands(int T, const OctCands& c, F f) {
  for (int k = threadIdx.x; k < T; k += NT) {
    const uint32_t n0 = c.nd(k);
    uint32_t n = n0;
    f(k, c.pos(k), n);
    if (n != n0) c.set_nd(k, n);
  }
}

// Phase probe (build with -DORBX_OCT_PROBE only; tools/oct_probe.py): per block, s_memtime ticks
// of the candidate load, the roots, the phase-1 and phase-2 rounds (with their counts) and the
// best-response pass, plus the level's candidate count; 8 words per block, indexed img * nlevels + l.
#ifdef ORBX_OCT_PROBE
__device__ unsigned int* oct_probe_buf;
#define OCT_TS(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define OCT_TS(v)
#endif

template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(6))) void k_octree(const Geometry* __restrict__ G, const CellInfo* __restrict__ cells,
                                               BatchPtrs B, OctGroup grp) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  // level-major grid (images fastest): every image's level-0 block (the longest) is dispatched
  // first and the short top levels last, so the kernel's tail is short blocks (longest first;
  // image-major order left one level-0 block per image until the end: 0.302 -> 0.232 ms per step)
  const int img = blockIdx.x, l = grp.l0 + blockIdx.y, tid = threadIdx.x;
  const LevelGeom& L = G->lv[l];
  const int NC = grp.node_cap;
  const int NP2 = next_pow2(NC);
  OctSmem s;
  {
    unsigned char* p = smem_raw;
    s.x0 = (int16_t*)p; p += NC * 4;
    s.y0 = (int16_t*)p; p += NC * 4;
    s.x1 = (int16_t*)p; p += NC * 4;
    s.y1 = (int16_t*)p; p += NC * 4;
    s.cnt = (int*)p; p += NC * 8;
    s.seq = (int*)p; p += NC * 8;
    s.ccnt = (int*)p; p += NC * 16;
    s.cidx = (int16_t*)p; p += NC * 8;
    s.nidx = (int16_t*)p; p += NC * 2;
    s.sa = (int*)p; p += NC * 4;
    s.sb = (int*)p; p += NC * 4;
    p = (unsigned char*)(((uintptr_t)p + 7) & ~(uintptr_t)7);
    s.key = (uint64_t*)p; p += (size_t)NP2 * 8;
    s.cpre = (int*)p; p += (grp.cell_cap + 1) * 4;
    s.ctrl = (int*)p; p += 8 * 4;
    s.kp = (uint32_t*)p; p += (size_t)grp.kcap * 4;
    s.kn = (uint16_t*)p;
  }
  uint32_t* oct_out = B.oct + (size_t)img * G->oct_total + L.oct_off;
  int* oct_cnt = B.oct_count + (size_t)img * G->nlevels + l;
  const size_t kbase = (size_t)img * G->cand_total + L.cand_begin;
  OctCands oc{s.kp, s.kn, grp.kcap, B.kpos + kbase, (uint32_t*)B.knode + kbase};

  OCT_TS(ot0);
#ifdef ORBX_OCT_PROBE
  unsigned long long ot_p1 = 0, ot_p2 = 0;
  int n_p1 = 0, n_p2 = 0;
#endif
  // 1. candidates of this level in vToDistributeKeys order (cells row-major)
  const int ncl = L.cell_end - L.cell_begin;
  for (int c = tid; c < ncl; c += NT) s.cpre[c] = B.cell_count[(size_t)img * G->ncells + L.cell_begin + c];
  __syncthreads();
  const int T = block_exclusive_scan<NT>(s.cpre, ncl);
  if (tid == 0) s.cpre[ncl] = T;
  if (T == 0) {
    if (tid == 0) *oct_cnt = 0;
    return;
  }
  const int nIni = L.nIni;
  const float hX = L.hX;
  const int minBX = L.minBX, minBY = L.minBY;
  for (int i = tid; i < nIni; i += NT) s.ccnt[i] = 0;
  __syncthreads();
  const uint32_t* cand = B.cand + (size_t)img * G->cand_total;
  auto put_cand = [&](int k, uint32_t v) {
    const int xr = (int)(v & 0xFFF) - minBX, yr = (int)((v >> 12) & 0xFFF) - minBY;
    const uint32_t pos = (v & 0xFF000000u) | ((uint32_t)yr << 12) | (uint32_t)xr;
    int root = (int)((float)xr / hX);
    root = min(max(root, 0), nIni - 1);
    oc.set(k, pos, (uint32_t)root);
    atomicAdd(&s.ccnt[root], 1);
  };
  if (ncl >= NT / 2) {
    // many cells (the dense levels): one thread per cell walks its survivors (candidate
    // k = cpre[c] + i), four loads in flight at a time
    for (int c = tid; c < ncl; c += NT) {
      const int k0 = s.cpre[c], n = s.cpre[c + 1] - k0;
      const CellInfo& ci = cells[L.cell_begin + c];
      const int kin = ci.kin, off = ci.cand_off, ovf = ci.ovf_off - kin;  // slot i: i < kin ? off + i : ovf + i
      int i = 0;
      for (; i + 4 <= n; i += 4) {
        const uint32_t v0 = cand[(i < kin ? off : ovf) + i], v1 = cand[(i + 1 < kin ? off : ovf) + i + 1],
                       v2 = cand[(i + 2 < kin ? off : ovf) + i + 2], v3 = cand[(i + 3 < kin ? off : ovf) + i + 3];
        put_cand(k0 + i, v0);
        put_cand(k0 + i + 1, v1);
        put_cand(k0 + i + 2, v2);
        put_cand(k0 + i + 3, v3);
      }
      for (; i < n; i++) put_cand(k0 + i, cand[(i < kin ? off : ovf) + i]);
    }
  } else {
    // few cells with many survivors each: one thread per candidate, its cell by binary search
    for (int k = tid; k < T; k += NT) {
      int lo = 0, hi = ncl - 1;  // last c with cpre[c] <= k
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s.cpre[mid] <= k) lo = mid; else hi = mid - 1;
      }
      put_cand(k, cand[cell_slot(cells[L.cell_begin + lo], k - s.cpre[lo])]);
    }
  }
  __syncthreads();
  OCT_TS(ot1);
  // 2. roots -> list (empty roots erased, src/ORBextractor.cc:604-615)
  for (int i = tid; i < nIni; i += NT) s.sa[i] = s.ccnt[i] > 0 ? 1 : 0;
  __syncthreads();
  int S = block_exclusive_scan<NT>(s.sa, nIni);
  for (int i = tid; i < nIni; i += NT) {
    if (s.ccnt[i] > 0) {
      const int ni = s.sa[i];
      s.x0[ni] = (int16_t)(int)(hX * (float)i);
      s.x1[ni] = (int16_t)(int)(hX * (float)(i + 1));
      s.y0[ni] = 0;
      s.y1[ni] = (int16_t)(L.maxBY - minBY);
      s.cnt[ni] = s.ccnt[i];
      s.seq[ni] = i;
      s.nidx[i] = (int16_t)ni;
    }
  }
  __syncthreads();
  oct_cands<NT>(T, oc, [&](int, uint32_t, uint32_t& nd) { nd = (uint32_t)s.nidx[nd]; });
  // child counters of the next round are cleared by the pass that precedes that
  // round's opening barrier (here, and after each round's remap): one barrier
  // per round fewer than a separate clear
  for (int i = tid; i < S * 4; i += NT) s.ccnt[i] = 0;
  OCT_TS(ot2);
  int cur = 0;
  int seqBase = nIni;
  int phase = 1;
  const int N = L.nfeat;
  for (int round = 0; round < 256; round++) {
    __syncthreads();
#ifdef ORBX_OCT_PROBE
    const unsigned long long rt0 = __builtin_amdgcn_s_memtime();
    const int rphase = phase;
    struct RoundStamp {
      unsigned long long t0;
      int ph;
      unsigned long long *p1, *p2;
      int *n1, *n2;
      __device__ ~RoundStamp() {
        const unsigned long long d = __builtin_amdgcn_s_memtime() - t0;
        if (ph == 1) { *p1 += d; ++*n1; } else { *p2 += d; ++*n2; }
      }
    } rstamp{rt0, rphase, &ot_p1, &ot_p2, &n_p1, &n_p2};
#endif
    const int nb = cur ^ 1;
    // kp pass A: child digit of every keypoint whose node splits (count > 1)
    oct_cands<NT>(T, oc, [&](int, uint32_t v, uint32_t& nd) {
      const int n = (int)(nd & 0x3FFF);
      if ((s.cnt + cur * NC)[n] > 1) {
        const int nx0 = (s.x0 + cur * NC)[n], ny0 = (s.y0 + cur * NC)[n];
        const int hx = (int)__builtin_ceilf((float)((s.x1 + cur * NC)[n] - nx0) / 2);
        const int hy = (int)__builtin_ceilf((float)((s.y1 + cur * NC)[n] - ny0) / 2);
        const float fx = (float)(int)(v & 0xFFF), fy = (float)(int)((v >> 12) & 0xFFF);
        const int d = (fx < (float)(nx0 + hx) ? 0 : 1) + (fy < (float)(ny0 + hy) ? 0 : 2);
        nd = (uint32_t)n | ((uint32_t)d << 14);
        atomicAdd(&s.ccnt[n * 4 + d], 1);
      }
    });
    __syncthreads();
    int C, Snew;
    if (phase == 1) {
      // split every node with > 1 keypoint, in list order.  One scan of packed
      // (children | kept << 16 | expandable children << 32) gives each node its
      // child and kept positions and the round's totals.
      for (int i = tid; i < S; i += NT) {
        const bool split = (s.cnt + cur * NC)[i] > 1;
        uint64_t v = split ? 0 : (1ull << 16);
        if (split)
          for (int d = 0; d < 4; d++) {
            const int cc = s.ccnt[i * 4 + d];
            v += (cc > 0 ? 1ull : 0ull) + (cc > 1 ? (1ull << 32) : 0ull);
          }
        s.key[i] = v;
      }
      __syncthreads();
      const uint64_t tot = block_scan_excl<NT, uint64_t>(s.key, S);
      C = (int)(tot & 0xFFFF);
      const int Sg = (int)((tot >> 16) & 0xFFFF);
      const int nexp = (int)(tot >> 32);
      for (int i = tid; i < S; i += NT) {
        const uint64_t pre = s.key[i];
        if ((s.cnt + cur * NC)[i] > 1) {
          const int nx0 = (s.x0 + cur * NC)[i], ny0 = (s.y0 + cur * NC)[i], nx1 = (s.x1 + cur * NC)[i], ny1 = (s.y1 + cur * NC)[i];
          const int hx = (int)__builtin_ceilf((float)(nx1 - nx0) / 2);
          const int hy = (int)__builtin_ceilf((float)(ny1 - ny0) / 2);
          int rank = 0;
          for (int d = 0; d < 4; d++) {
            const int cc = s.ccnt[i * 4 + d];
            if (cc == 0) continue;
            const int p = (int)(pre & 0xFFFF) + rank++;
            const int ni = C - 1 - p;
            (s.x0 + nb * NC)[ni] = (int16_t)((d & 1) ? nx0 + hx : nx0);
            (s.x1 + nb * NC)[ni] = (int16_t)((d & 1) ? nx1 : nx0 + hx);
            (s.y0 + nb * NC)[ni] = (int16_t)((d & 2) ? ny0 + hy : ny0);
            (s.y1 + nb * NC)[ni] = (int16_t)((d & 2) ? ny1 : ny0 + hy);
            (s.cnt + nb * NC)[ni] = cc;
            (s.seq + nb * NC)[ni] = seqBase + p;
            s.cidx[i * 4 + d] = (int16_t)ni;
          }
        } else {
          const int ni = C + (int)((pre >> 16) & 0xFFFF);
          (s.x0 + nb * NC)[ni] = (s.x0 + cur * NC)[i];
          (s.x1 + nb * NC)[ni] = (s.x1 + cur * NC)[i];
          (s.y0 + nb * NC)[ni] = (s.y0 + cur * NC)[i];
          (s.y1 + nb * NC)[ni] = (s.y1 + cur * NC)[i];
          (s.cnt + nb * NC)[ni] = (s.cnt + cur * NC)[i];
          (s.seq + nb * NC)[ni] = (s.seq + cur * NC)[i];
          s.nidx[i] = (int16_t)ni;
        }
      }
      __syncthreads();  // children / cidx / nidx written before the candidates remap
      oct_cands<NT>(T, oc, [&](int, uint32_t, uint32_t& nd) {
        const int n = (int)(nd & 0x3FFF);
        nd = (uint32_t)((s.cnt + cur * NC)[n] > 1 ? s.cidx[n * 4 + (nd >> 14)] : s.nidx[n]);
      });
      Snew = C + Sg;
      for (int i = tid; i < Snew * 4; i += NT) s.ccnt[i] = 0;
      seqBase += C;
      const bool finish = Snew >= N || Snew == S;
      S = Snew;
      cur = nb;
      if (finish) break;
      if (Snew + 3 * nexp > N) phase = 2;
    } else {
      // phase 2: split the largest (size, seq) first until the list reaches N
      for (int i = tid; i < S; i += NT) s.sa[i] = (s.cnt + cur * NC)[i] > 1 ? 1 : 0;
      __syncthreads();
      const int M = block_exclusive_scan<NT>(s.sa, S);
      const int P2 = next_pow2(max(M, 2));
      for (int i = tid; i < P2; i += NT) s.key[i] = 0;
      __syncthreads();
      for (int i = tid; i < S; i += NT)
        if ((s.cnt + cur * NC)[i] > 1)
          s.key[s.sa[i]] = ((uint64_t)(s.cnt + cur * NC)[i] << 43) | ((uint64_t)(s.seq + cur * NC)[i] << 13) | (uint64_t)i;
      __syncthreads();
      if (M <= kOctRankSortMax) {
        // descending order by rank (keys are distinct: they carry the node index): key j goes to
        // #{keys > key j}; one pass over the M keys per key instead of log2(P2)^2/2 barrier stages
        uint64_t* tmp = reinterpret_cast<uint64_t*>(s.cidx);  // cidx is rewritten below
        for (int j = tid; j < M; j += NT) {
          const uint64_t x = s.key[j];
          int r = 0;
#pragma unroll 4
          for (int y = 0; y < M; y++) r += s.key[y] > x ? 1 : 0;
          tmp[r] = x;
        }
        __syncthreads();
        for (int j = tid; j < M; j += NT) s.key[j] = tmp[j];
        __syncthreads();
      } else {
        bitonic_sort_desc<NT>(s.key, P2);
      }
      if (tid == 0) s.ctrl[1] = M - 1;
      for (int j = tid; j < M; j += NT) {
        const int n = (int)(s.key[j] & 0x1FFF);
        int nc = 0;
        for (int d = 0; d < 4; d++) nc += s.ccnt[n * 4 + d] > 0;
        s.sb[j] = nc - 1;
      }
      __syncthreads();
      // inclusive prefix of growth; first j reaching N
      block_exclusive_scan<NT>(s.sb, M);  // exclusive
      for (int j = tid; j < M; j += NT) {
        const int n = (int)(s.key[j] & 0x1FFF);
        int nc = 0;
        for (int d = 0; d < 4; d++) nc += s.ccnt[n * 4 + d] > 0;
        if (S + s.sb[j] + (nc - 1) >= N) atomicMin(&s.ctrl[1], j);
      }
      __syncthreads();
      const int m = s.ctrl[1];
      // children positions in processing order j = 0..m
      for (int j = tid; j < M; j += NT) {
        int nc = 0;
        if (j <= m) {
          const int n = (int)(s.key[j] & 0x1FFF);
          for (int d = 0; d < 4; d++) nc += s.ccnt[n * 4 + d] > 0;
        }
        s.sb[j] = nc;
      }
      for (int i = tid; i < S; i += NT) s.nidx[i] = -1;  // -1: processed marker set below
      __syncthreads();
      C = block_exclusive_scan<NT>(s.sb, M);
      for (int j = tid; j <= m; j += NT) {
        const int n = (int)(s.key[j] & 0x1FFF);
        s.nidx[n] = -2;  // processed
      }
      __syncthreads();
      for (int i = tid; i < S; i += NT) s.sa[i] = s.nidx[i] == -2 ? 0 : 1;
      __syncthreads();
      const int rest = block_exclusive_scan<NT>(s.sa, S);
      for (int j = tid; j <= m; j += NT) {
        const int i = (int)(s.key[j] & 0x1FFF);
        const int nx0 = (s.x0 + cur * NC)[i], ny0 = (s.y0 + cur * NC)[i], nx1 = (s.x1 + cur * NC)[i], ny1 = (s.y1 + cur * NC)[i];
        const int hx = (int)__builtin_ceilf((float)(nx1 - nx0) / 2);
        const int hy = (int)__builtin_ceilf((float)(ny1 - ny0) / 2);
        int rank = 0;
        for (int d = 0; d < 4; d++) {
          const int cc = s.ccnt[i * 4 + d];
          if (cc == 0) continue;
          const int p = s.sb[j] + rank++;
          const int ni = C - 1 - p;
          (s.x0 + nb * NC)[ni] = (int16_t)((d & 1) ? nx0 + hx : nx0);
          (s.x1 + nb * NC)[ni] = (int16_t)((d & 1) ? nx1 : nx0 + hx);
          (s.y0 + nb * NC)[ni] = (int16_t)((d & 2) ? ny0 + hy : ny0);
          (s.y1 + nb * NC)[ni] = (int16_t)((d & 2) ? ny1 : ny0 + hy);
          (s.cnt + nb * NC)[ni] = cc;
          (s.seq + nb * NC)[ni] = seqBase + p;
          s.cidx[i * 4 + d] = (int16_t)ni;
        }
      }
      for (int i = tid; i < S; i += NT) {
        if (s.nidx[i] == -2) continue;
        const int ni = C + s.sa[i];
        (s.x0 + nb * NC)[ni] = (s.x0 + cur * NC)[i];
        (s.x1 + nb * NC)[ni] = (s.x1 + cur * NC)[i];
        (s.y0 + nb * NC)[ni] = (s.y0 + cur * NC)[i];
        (s.y1 + nb * NC)[ni] = (s.y1 + cur * NC)[i];
        (s.cnt + nb * NC)[ni] = (s.cnt + cur * NC)[i];
        (s.seq + nb * NC)[ni] = (s.seq + cur * NC)[i];
        s.nidx[i] = (int16_t)ni;
      }
      __syncthreads();
      oct_cands<NT>(T, oc, [&](int, uint32_t, uint32_t& nd) {
        const int n = (int)(nd & 0x3FFF);
        const int ni = s.nidx[n];  // -2: n was split this round
        nd = (uint32_t)(ni == -2 ? s.cidx[n * 4 + (nd >> 14)] : ni);
      });
      Snew = C + rest;
      for (int i = tid; i < Snew * 4; i += NT) s.ccnt[i] = 0;
      seqBase += C;
      const bool finish = Snew >= N || Snew == S;
      S = Snew;
      cur = nb;
      if (finish) break;
    }
  }
  __syncthreads();
  // 3. best response per node: max score, then lowest candidate index
  for (int i = tid; i < S; i += NT) s.key[i] = 0;
  __syncthreads();
  oct_cands<NT>(T, oc, [&](int k, uint32_t v, uint32_t& nd) {
    const uint32_t x = (v & 0xFFF) + minBX, y = ((v >> 12) & 0xFFF) + minBY;
    const uint64_t key = ((uint64_t)(v >> 24) << 56) | ((uint64_t)(0xFFFFFFu - (uint32_t)k) << 24) |
                         (uint64_t)((y << 12) | x);
    atomicMax((unsigned long long*)&s.key[nd & 0x3FFF], (unsigned long long)key);
  });
  __syncthreads();
  const int nout = min(S, L.oct_cap);
  for (int i = tid; i < nout; i += NT) {
    const uint64_t key = s.key[i];
    oct_out[i] = ((uint32_t)(key >> 56) << 24) | (uint32_t)(key & 0xFFFFFF);
  }
  if (tid == 0) *oct_cnt = nout;
#ifdef ORBX_OCT_PROBE
  if (tid == 0 && oct_probe_buf) {
    const unsigned long long ot3 = __builtin_amdgcn_s_memtime();
    unsigned int* o = oct_probe_buf + ((size_t)img * G->nlevels + l) * 8;
    o[0] = (unsigned int)(ot1 - ot0);
    o[1] = (unsigned int)(ot2 - ot1);
    o[2] = (unsigned int)ot_p1;
    o[3] = (unsigned int)n_p1;
    o[4] = (unsigned int)ot_p2;
    o[5] = (unsigned int)n_p2;
    o[6] = (unsigned int)(ot3 - ot0);
    o[7] = (unsigned int)T;
  }
#endif
}

// --------------------------------------------------------------- describe
// One wave per keypoint: IC_Angle on the raw level (src/ORBextractor.cc:77-105),
// computeOrbDescriptor on the blurred level (:110-152), then the keypoint
// record in level-major output order with pt *= mvScaleFactor[l] (:1201-1207).
// Sum over the 64 lanes (all active), returned wave-uniform: DPP row_shr 1/2/4/8
// prefix sums leave each 16-lane row's total in its last lane, then four readlanes.
// (Integer adds: the order is immaterial.)
__device__ __forceinline__ int wave_sum_dpp(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
  return __builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31) + __builtin_amdgcn_readlane(v, 47) +
         __builtin_amdgcn_readlane(v, 63);
}


// describe's blurred patch: rotated bit_pattern_31_ points stay within radius 18.39, so
// |row|, |col| <= 18 after cvRound: a 37 x 37 patch around the keypoint
constexpr int kPatchR = 18;
constexpr int kPatchRows = 2 * kPatchR + 1;  // 37
constexpr int kPS = 80;  // LDS row stride of the staged patches (bytes): 20 dwords, so the rotated
                         // samples' rows spread over the banks (a 64-B stride folds every 4th row)
// bytes per wave: the blurred patch + the descriptor words
constexpr int kDescLds = kPatchRows * kPS + 256;
// half-width hw(r) of patch row r = 0..36 (row offset r - 18) the rotated pattern can reach
// describe patch slots: slot s -> (row << 2 | k-th chunk of the row's span), 2 / 3 / 4 slots per row
// (the most 16-B chunks the row's span covers over the 16 alignments), 124 slots, 0xFF past them
__constant__ uint8_t c_patch_slot[128] = {0,1,4,5,8,9,10,12,13,14,16,17,18,20,21,22,24,25,26,28,29,30,32,33,34,36,37,38,40,41,42,43,44,45,46,47,48,49,50,51,52,53,54,55,56,57,58,59,60,61,62,63,64,65,66,67,68,69,70,71,72,73,74,75,76,77,78,79,80,81,82,83,84,85,86,87,88,89,90,91,92,93,94,95,96,97,98,99,100,101,102,103,104,105,106,107,108,109,110,112,113,114,116,117,118,120,121,122,124,125,126,128,129,130,132,133,134,136,137,138,140,141,144,145,255,255,255,255};
__constant__ int c_patch_hw[kPatchRows] = {6,  8,  10, 11, 12, 13, 14, 15, 16, 16, 17, 17, 18, 18, 18, 18, 18, 18, 18,
                                           18, 18, 18, 18, 18, 18, 17, 17, 16, 16, 15, 14, 13, 12, 11, 10, 8,  6};

#ifndef ORBX_DESC_K
#define ORBX_DESC_K 8
#endif
constexpr int kDescK = ORBX_DESC_K;  // keypoints per wave
static_assert(kDescK * 8 <= 64, "one descriptor dword per lane");

// f(std::integral_constant<int, 0>{}) ... f(<N-1>): compile-time lane indices in an unrolled loop
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ const uint8_t* lane_ptr(const uint8_t* p, int j) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)a, j), hi = __builtin_amdgcn_readlane((uint32_t)(a >> 32), j);
  return (const uint8_t*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float lane_f(float v, int j) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), j));
}

// k_describe: IC_Angle (src/ORBextractor.cc:77-105), computeOrbDescriptor (:110-152) on the blurred
// level k_blur wrote (:1186-1190), and the keypoint record in level-major output order with
// pt *= mvScaleFactor[l] (:1201-1207).
//
// kDescK keypoints per wave (consecutive output indices):
//   1. lane j finds keypoint i0 + j's level and loads its octree entry and level record;
//   2. the IC_Angle boxes of all kDescK keypoints and the blurred patches of the first two are
//      issued together; the moments are wave sums per keypoint (v_dot4 on circle-masked 16-B rows);
//   3. fastAtan2 and the deterministic sin/cos run once, lane j for keypoint j;
//   4. per keypoint: the blurred patch (only the pixels a rotated pair can reach) -> LDS, the patch
//      two ahead issued, then the 256 rotated pairs with pair p in lane p & 63: ballot k =
//      descriptor bits 64k .. 64k+63, staged in LDS;
//   5. one coalesced store of the kDescK descriptors (lane = dword) and the keypoint records.
__global__ __launch_bounds__(BS) void k_describe(const Geometry* __restrict__ G, BatchPtrs B,
                                                 orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                 int32_t* __restrict__ counts, int kp_cap) {
  __shared__ __align__(16) uint8_t s_desc[BS / 64][kDescLds];
  const int2 bi = xcd_block2();
  const int img = bi.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i0 = __builtin_amdgcn_readfirstlane((bi.x * (BS / 64) + wv) * kDescK);
  const int nl = G->nlevels;
  // per-level counts as independent scalar loads
  const int* oc = B.oct_count + (size_t)img * nl;
  int cnt[kMaxLevelsPlan];
#pragma unroll
  for (int ll = 0; ll < kMaxLevelsPlan; ll++) cnt[ll] = ll < nl ? oc[ll] : 0;
  int total = 0;
#pragma unroll
  for (int ll = 0; ll < kMaxLevelsPlan; ll++) total += cnt[ll];
  if (bi.x == 0 && threadIdx.x == 0) counts[img] = total;
  // the rBRIEF pairs of this lane (p = lane + 64k), reused for every keypoint of the wave
  float4 pat[4];
#pragma unroll
  for (int k = 0; k < 4; k++) pat[k] = reinterpret_cast<const float4*>(c_pattern_f)[lane + 64 * k];
  if (i0 >= total) return;  // wave-uniform: the DPP sums below see a full wave
  const int nk = min(kDescK, total - i0);
  // 1. lane j: keypoint i0 + min(j, nk - 1) (lanes past nk repeat the last one; never written)
  const int i = i0 + min(lane, nk - 1);
  int l = 0, first = 0, acc = 0;
#pragma unroll
  for (int ll = 0; ll < kMaxLevelsPlan; ll++) {
    if (i >= acc) {  // last level whose start is <= i
      l = ll;
      first = acc;
    }
    acc += cnt[ll];
  }
  const LevelGeom& L = G->lv[l];
  const uint32_t v = B.oct[(size_t)img * G->oct_total + L.oct_off + (i - first)];
  const int w = L.w, h = L.h;
  const float lscale = L.scale, lsize = L.kp_size;
  const int x = v & 0xFFF, y = (v >> 12) & 0xFFF, score = v >> 24;
  const uint8_t* lvl = level_ptr(*G, B, img, l);
  // IC box origin (x - 15, y - 15); keypoints sit >= 19 px inside the level, so the box is too
  const uint8_t* icp = lvl + (size_t)(y - 15) * w + (x - 15);

  // 2. IC boxes of every keypoint, then the first two blurred patches
  const int r = lane >> 1, hh = lane & 1;
  uint32_t q[kDescK][4];
#pragma unroll
  for (int j = 0; j < kDescK; j++) {
    const int wj = __builtin_amdgcn_readlane(w, j);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)lane_ptr(icp, j), (short)0, 31 * wj, 0x00020000);
    const uint32_t off = lane < 62 ? (uint32_t)(r * wj + 16 * hh) : 0x80000000u;
    const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    q[j][0] = t[0];
    q[j][1] = t[1];
    q[j][2] = t[2];
    q[j][3] = t[3];
  }
  constexpr int kPatchLd = 2;  // 16-B loads per lane per patch
  // the blurred level's patch: rows y-18..y+18, 16-B chunks from the 16-aligned column x0
  const int bs = L.bstride;
  const int x0 = (x - kPatchR) & ~15;
  const uint8_t* pbl = B.blur + (size_t)img * G->blur_bytes + L.boff;  // the level's tiles
  constexpr int PS = kPS;
  const uint32_t corr_l = (uint32_t)(kPatchR * PS + (x - x0)) - (0x400000u * (uint32_t)PS + 0x4B400000u);
  // Only the blurred pixels a rotated pattern point can land on are loaded: a point of radius rho
  // rounds to (r, c) with (|r| - 1/2)^2 + (|c| - 1/2)^2 <= rho^2 <= 338 (the pattern's largest
  // rho^2), so row r needs |c| <= hw(r) (c_patch_hw; equal to the brute-force reach of the pattern
  // over all angles).  Each row's span [18+a-hw, 18+a+hw] (a = (x-18) & 15, patch column 0 = the
  // 16-aligned level column x0) covers 2-4 16-B chunks: slot s = lane + 64k is (row, k-th chunk of
  // its span) (c_patch_slot), 124 slots, 99-112 of them valid by a -- two 16-B loads per lane
  // instead of three, 25-33 % fewer bytes than the full 37 x 64.
  int srow[kPatchLd], skk[kPatchLd], shw[kPatchLd];
#pragma unroll
  for (int k = 0; k < kPatchLd; k++) {
    const int e = c_patch_slot[lane + 64 * k];
    srow[k] = e == 0xFF ? -1 : e >> 2;
    skk[k] = e & 3;
    shw[k] = c_patch_hw[e == 0xFF ? 0 : e >> 2];
  }
  uint32_t pv[2][kPatchLd][4];
  int pdst[2][kPatchLd];  // LDS byte offset of each loaded chunk (-1: none)
  auto load_patch = [&](int j, uint32_t (&dst)[kPatchLd][4], int (&dofs)[kPatchLd]) {
    const int bt8 = __builtin_amdgcn_readlane(bs, j) * 8, hj = __builtin_amdgcn_readlane(h, j);
    const int xj = __builtin_amdgcn_readlane(x, j), y0j = __builtin_amdgcn_readlane(y, j) - kPatchR;
    const int aj = (xj - kPatchR) & 15, tx0 = (xj - kPatchR) >> 4;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)lane_ptr(pbl, j), (short)0, ((hj + 7) >> 3) * bt8, 0x00020000);
#pragma unroll
    for (int k = 0; k < kPatchLd; k++) {
      // 16-B chunks at 16-aligned columns: each is one row of an 8 x 16 tile (blur_tile_off), so the
      // chunks of eight patch rows in a column share one 128-B line
      const int lo = (kPatchR + aj - shw[k]) >> 4, hi = (kPatchR + aj + shw[k]) >> 4;
      const int ch = lo + skk[k];
      const bool ok = srow[k] >= 0 && ch <= hi;
      const int yy = y0j + srow[k];
      const uint32_t off = ok ? (uint32_t)((yy >> 3) * bt8 + (tx0 + ch) * 128 + (yy & 7) * 16) : 0x80000000u;
      dofs[k] = ok ? srow[k] * kPS + 16 * ch : -1;
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
      dst[k][0] = t[0];
      dst[k][1] = t[1];
      dst[k][2] = t[2];
      dst[k][3] = t[3];
    }
  };
  load_patch(0, pv[0], pdst[0]);
  if (kDescK > 1) load_patch(1, pv[1], pdst[1]);
  // moments: lane (r, hh) holds the 16 bytes at columns 16hh .. 16hh + 15 of box row r, masked to
  // the circle; s0 = sum I, s1 = sum b * I, m01 = (r - 15) s0, m10 = s1 + (16hh - 15) s0 (integers:
  // exact in any order).  Keypoint j's sums land in lane j.
  int M01 = 0, M10 = 0;
  {
    const uint4 mk = c_icmask[lane];
    static_for<kDescK>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const uint32_t I0 = q[j][0] & mk.x, I1 = q[j][1] & mk.y, I2 = q[j][2] & mk.z, I3 = q[j][3] & mk.w;
      uint32_t s0 = __builtin_amdgcn_udot4(I0, 0x01010101u, 0u, false);
      s0 = __builtin_amdgcn_udot4(I1, 0x01010101u, s0, false);
      s0 = __builtin_amdgcn_udot4(I2, 0x01010101u, s0, false);
      s0 = __builtin_amdgcn_udot4(I3, 0x01010101u, s0, false);
      uint32_t s1 = __builtin_amdgcn_udot4(I0, 0x03020100u, 0u, false);
      s1 = __builtin_amdgcn_udot4(I1, 0x07060504u, s1, false);
      s1 = __builtin_amdgcn_udot4(I2, 0x0B0A0908u, s1, false);
      s1 = __builtin_amdgcn_udot4(I3, 0x0F0E0D0Cu, s1, false);
      const int m01 = wave_sum_dpp((r - 15) * (int)s0);
      const int m10 = wave_sum_dpp((int)s1 + (16 * hh - 15) * (int)s0);
      M01 = lane == j ? m01 : M01;
      M10 = lane == j ? m10 : M10;
    });
  }
  // 3. orientation of keypoint j in lane j
  const float angle = fast_atan2((float)M01, (float)M10);
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float sn, cs;
  sincos_det(angle * factorPI, c_sincos, &sn, &cs);

  const float2v magic = {12582912.0f, 12582912.0f};  // 1.5 * 2^23: round half to even

  // 4. per keypoint
  uint8_t* pb = s_desc[wv];
  // the descriptors' 64-bit words, staged per wave and stored by lane = dword at the end
  uint64_t* sdw = reinterpret_cast<uint64_t*>(s_desc[wv] + kDescLds - 256);
  static_for<kDescK>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    if (j >= nk) return;  // wave-uniform
    uint32_t (&cur)[kPatchLd][4] = pv[j & 1];
    int (&cdst)[kPatchLd] = pdst[j & 1];
#pragma unroll
    for (int k = 0; k < kPatchLd; k++)
      if (cdst[k] >= 0) *(uint4*)(pb + cdst[k]) = make_uint4(cur[k][0], cur[k][1], cur[k][2], cur[k][3]);
    if (j + 2 < kDescK && j + 2 < nk) load_patch(j + 2, cur, cdst);
    const uint32_t corr = __builtin_amdgcn_readlane(corr_l, j);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // rotated pattern point (px, py) -> patch pixel (18 + r, 18 + c) with
    //   r = cvRound(px*b + py*a), c = cvRound(px*a - py*b)    (src/ORBextractor.cc:119-125)
    // Both coordinates ride in packed-f32 lanes.  Each sum is rounded exactly as the scalar
    // expression (products, then the add / subtract); adding 1.5*2^23 rounds it to an integer
    // half-to-even (|sum| < 2^22), leaving 0x4B400000 + r in the bits.  A 24-bit mad on the raw
    // bits ((0x400000 + r) * kPS, low 24 bits sign-extended) plus a constant gives the offset.
    const float a = lane_f(cs, j), b = lane_f(sn, j);
    const float2v ba = {b, a}, ab = {a, b};
    static_for<4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      int t[2];
#pragma unroll
      for (int e = 0; e < 2; e++) {
        const float px = e ? pat[k].z : pat[k].x, py = e ? pat[k].w : pat[k].y;
        const float2v P = (float2v){px, px} * ba;   // {px*b, px*a}
        const float2v Q = (float2v){py, -py} * ab;  // {py*a, -(py*b)}: negation is exact
        const float2v M = (P + Q) + magic;
        const uint32_t mr = __float_as_uint(M.x), mc = __float_as_uint(M.y);
        t[e] = pb[(uint32_t)__mul24((int)mr, kPS) + mc + corr];
      }
      // bits 64k .. 64k + 63 of the descriptor: every lane stores the same wave-uniform word
      sdw[4 * j + k] = __ballot(t[0] < t[1]);
    });
    // the next keypoint's patches overwrite these: every lane's reads come first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  });
  // 5. output: descriptors (lane = dword) and keypoint records (lane = keypoint)
  const size_t o0 = (size_t)img * kp_cap + i0;
  if (lane < 8 * nk) reinterpret_cast<uint32_t*>(desc + o0 * 32)[lane] = reinterpret_cast<const uint32_t*>(sdw)[lane];
  if (lane < nk) {
    orbx_keypoint kp;
    float fx = (float)x, fy = (float)y;
    if (l != 0) {
      fx *= lscale;
      fy *= lscale;
    }
    kp.x = fx;
    kp.y = fy;
    kp.size = lsize;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    kps[o0 + lane] = kp;
  }
}

// ------------------------------------------------------------------ launch
hipError_t upload_constants(const int* umax16, const int* gauss7) {
  uint32_t mask[64][4] = {};
  for (int lane = 0; lane < 62; lane++) {
    const int r = lane >> 1, h = lane & 1, v = r - 15, um = umax16[v < 0 ? -v : v];
    for (int b = 0; b < 16; b++) {
      const int u = 16 * h + b - 15;
      if (u <= 15 && u >= -um && u <= um) mask[lane][b >> 2] |= 0xFFu << (8 * (b & 3));
    }
  }
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_icmask), mask, sizeof(mask));
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(c_gauss), gauss7, 7 * sizeof(int));
}

hipError_t launch_extract_stages(const Geometry& Gh, const Geometry* Gd, const CellInfo* cells,
                                 const int* tile_level, const ResizeX* xt, const ResizeY* yt, const BatchPtrs& B,
                                 int n_img, orbx_keypoint* kps, uint8_t* desc, int32_t* counts, int kp_cap,
                                 hipStream_t st, StageTimer* T) {
  for (int l = 1; l < Gh.nlevels; l++) {
    dim3 grid((Gh.lv[l].w + kRzTW - 1) / kRzTW, (Gh.lv[l].h + kRzTH - 1) / kRzTH, n_img);
    T->begin(st);
    hipLaunchKernelGGL(k_resize, grid, dim3(BS), (size_t)Gh.rz_rows * (Gh.rz_stride + 2 * kRzTW), st, Gd, xt, yt, B, l);
    T->end(ST_RESIZE, st);
  }
  if (Gh.ncells > 0) {
    T->begin(st);
    for (int g = 0; g < Gh.n_fg; g++) {
      const Geometry::FastGroup& F = Gh.fg[g];
      if (F.c1 <= F.c0) continue;
      auto kf = F.s == 40   ? (F.rp == 2 ? k_fast<40, 2> : k_fast<40, 1>)
                : F.s == 48 ? (F.rp == 2 ? k_fast<48, 2> : k_fast<48, 1>)
                            : k_fast<80, 1>;
      hipLaunchKernelGGL(kf, dim3((F.c1 - F.c0 + kFastCPW - 1) / kFastCPW, n_img), dim3(64), F.smem, st, Gd, cells, B, g);
    }
    T->end(ST_FAST, st);
  } else {
    (void)hipMemsetAsync(B.oct_count, 0, sizeof(int) * Gh.nlevels * n_img, st);
  }
  {
    T->begin(st);
    hipLaunchKernelGGL(k_blur, dim3(Gh.ntiles, n_img), dim3(BS), 0, st, Gd, tile_level, B);
    T->end(ST_BLUR, st);
  }
  if (Gh.ncells > 0) {
    T->begin(st);
    // (launch order of the groups measured flat).  One or two images: all levels in one launch
    // (the groups' launches would run one after the other with a few blocks each)
    const bool one = n_img <= kOctOneLaunch;
    for (int gi = 0; gi < (one ? 1 : Gh.n_og); gi++) {
      const OctGroup& og = one ? Gh.og_all : Gh.og[gi];
      const size_t smem = octree_smem_bytes(og.node_cap, og.cell_cap, og.kcap);
      if (og.nt == 512)
        hipLaunchKernelGGL(k_octree<512>, dim3(n_img, og.l1 - og.l0), dim3(512), smem, st, Gd, cells, B, og);
      else
        hipLaunchKernelGGL(k_octree<256>, dim3(n_img, og.l1 - og.l0), dim3(256), smem, st, Gd, cells, B, og);
    }
    T->end(ST_OCTREE, st);
  }
  const int nb = (Gh.max_kps + BS / 64 * kDescK - 1) / (BS / 64 * kDescK);  // kDescK keypoints per wave
  T->begin(st);
  hipLaunchKernelGGL(k_describe, dim3(max(nb, 1), n_img), dim3(BS), 0, st, Gd, B, kps, desc, counts, kp_cap);
  T->end(ST_DESCRIBE, st);
  return hipGetLastError();
}

// The blurred levels of n_img images (ORBX_DBG_BLUR_LEVEL; the extraction itself never writes them)
hipError_t launch_blur(const Geometry& Gh, const Geometry* Gd, const int* tile_level, const BatchPtrs& B, int n_img,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_blur, dim3(Gh.ntiles, n_img), dim3(BS), 0, st, Gd, tile_level, B);
  return hipGetLastError();
}

size_t octree_smem_host(int NC, int cell_cap, int kcap) { return octree_smem_bytes(NC, cell_cap, kcap); }

hipError_t octree_set_smem_limit(size_t bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)k_octree<512>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)k_octree<256>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace orbx

#ifdef ORBX_OCT_PROBE
extern "C" int orbx_debug_oct_probe(void* d_buf) {  // device buffer of 8 u32 per (image, level) block, or NULL
  unsigned int* p = (unsigned int*)d_buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(orbx::oct_probe_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
#ifdef ORBX_FAST_PROBE
extern "C" int orbx_debug_fast_probe(void* d_buf) {  // device buffer of 8 u32 per cell wave, or NULL
  unsigned int* p = (unsigned int*)d_buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(orbx::fast_probe_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
