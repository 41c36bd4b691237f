// stereo.hip -- Frame::ComputeStereoMatches (src/Frame.cc:547-788) batched over
// stereo frames, plus batched ORBmatcher::DescriptorDistance
// (src/ORBmatcher.cc:1844-1860).
//
//   k_stereo_prep     per frame: right keypoints sorted by (octave, y) -- replaces
//                     the reference's row-band table (:564-590); the candidate
//                     set of a left keypoint is then 3 contiguous ranges.
//   k_stereo_match    16 lanes per left keypoint (four per wave in parallel): band
//                     Hamming argmin (strict <, lowest index), 11x11 SAD over +-5 px
//                     on the unblurred pyramid level, parabola, depth (:600-770).
//   k_stereo_finalize per frame: median SAD by 2-pass radix select, reject
//                     SAD >= 1.5*1.4*median (:774-787).
#include <hip/hip_runtime.h>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_stereo.h"
#include "orbx_prof.h"

namespace orbx {

constexpr int SBS = 256;
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }

// Sorts the right keypoints by (octave, y) and builds, per (octave, row Y), the
// candidate range [start, end) of right keypoints whose band
// [floor(y - 2 s_o), ceil(y + 2 s_o)] contains Y -- the reference's
// vRowIndices[Y] (src/Frame.cc:572-590) split by octave, in iR order within
// equal y.  Also writes (x, index) in sorted order for the match kernel.
// one 1024-thread block per frame: the bitonic stages and the per-(octave,row)
// binary searches are the serial part, spread over 4x the threads of SBS
constexpr int PBS = 1024;
__global__ __launch_bounds__(PBS) void k_stereo_prep(StereoArgs A, const Geometry* __restrict__ G) {
  __shared__ uint64_t keys[kMaxStereoKps];
  __shared__ int ost[kMaxLevelsPlan + 1];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int nR = min(A.nR[(size_t)f * A.n_stride_R], kMaxStereoKps);
  const orbx_keypoint* kR = A.kpR + (size_t)f * A.kR_stride;
  int P2 = 2;
  while (P2 < nR) P2 <<= 1;
  for (int i = tid; i < P2; i += PBS) {
    uint64_t k = ~0ull;
    if (i < nR) {
      const orbx_keypoint kp = kR[i];
      k = ((uint64_t)(uint32_t)kp.octave << 44) | ((uint64_t)fbits(kp.y) << 12) | (uint64_t)i;
    }
    keys[i] = k;
  }
  __syncthreads();
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P2 / 2; i += PBS) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool asc = (lo & size) == 0;
        const uint64_t a = keys[lo], b = keys[hi];
        if (asc ? (a > b) : (a < b)) {
          keys[lo] = b;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  uint64_t* out = A.rkeys + (size_t)f * kMaxStereoKps;
  int2* rxi = A.rxi + (size_t)f * kMaxStereoKps;
  for (int i = tid; i < nR; i += PBS) {
    const uint64_t k = keys[i];
    out[i] = k;
    const int idx = (int)(k & 0xFFF);
    rxi[i] = make_int2(__float_as_int(kR[idx].x), idx);
  }
  // descriptors in sorted order, so the match kernel loads a candidate's
  // descriptor beside its (x, index) instead of after it
  {
    const uint4* dR = (const uint4*)(A.dR + (size_t)f * A.kR_stride * 32);
    uint4* rd = A.rdesc + (size_t)f * kMaxStereoKps * 2;
    for (int e = tid; e < 2 * nR; e += PBS) rd[e] = dR[2 * (int)(keys[e >> 1] & 0xFFF) + (e & 1)];
  }
  // octave starts
  int* os = A.oct_start + (size_t)f * (kMaxLevelsPlan + 1);
  for (int o = tid; o <= A.nlevels; o += PBS) {
    int lo = 0, hi = nR;  // first i with octave >= o
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((int)(keys[mid] >> 44) < o) lo = mid + 1; else hi = mid;
    }
    os[o] = lo;
    ost[o] = lo;
  }
  __syncthreads();
  // row table: first with ceil(y + r) >= Y, then first (from there) with floor(y - r) > Y
  uint32_t* tab = A.rtab + (size_t)f * A.nlevels * A.rows;
  for (int e = tid; e < A.nlevels * A.rows; e += PBS) {
    const int o = e / A.rows, Y = e - o * A.rows;
    const float r = 2.0f * G->lv[o].scale;
    const int lo = ost[o], hi = ost[o + 1];
    int a = lo, b = hi;
    while (a < b) {
      const int m = (a + b) >> 1;
      if ((int)__builtin_ceilf(__uint_as_float((uint32_t)(keys[m] >> 12)) + r) >= Y) b = m; else a = m + 1;
    }
    int c = a, d = hi;
    while (c < d) {
      const int m = (c + d) >> 1;
      if ((int)__builtin_floorf(__uint_as_float((uint32_t)(keys[m] >> 12)) - r) > Y) d = m; else c = m + 1;
    }
    tab[e] = (uint32_t)a | ((uint32_t)c << 16);
  }
  // each left keypoint's three candidate ranges (vRowIndices[vL] of octaves level-1..level+1), so
  // the match kernel loads them beside the keypoint instead of after it (one dependent round trip
  // fewer per keypoint)
  __syncthreads();
  const int nL = min(A.nL[(size_t)f * A.n_stride_L], A.maxL);
  const orbx_keypoint* kL = A.kpL + (size_t)f * A.kL_stride;
  uint4* lr = A.lrange + (size_t)f * A.maxL;
  for (int i = tid; i < nL; i += PBS) {
    const orbx_keypoint kp = kL[i];
    const int Y = (int)kp.y;
    uint32_t t[3];
#pragma unroll
    for (int q = 0; q < 3; q++) {
      const int o = kp.octave - 1 + q;
      t[q] = (o >= 0 && o < A.nlevels && Y >= 0 && Y < A.rows) ? tab[(size_t)o * A.rows + Y] : 0u;
    }
    lr[i] = make_uint4(t[0], t[1], t[2], 0u);
  }
}

// 16 left keypoints per 4-wave block (one per 16-lane quarter)
constexpr int kKpsPerBlock = SBS / 16;
// SAD staging per keypoint: 11 rows x (4 left + 6 right) dwords
constexpr int kSadDwL = 4, kSadDwR = 6, kSadDw = kSadDwL + kSadDwR;

// k_stereo_match: the four left keypoints of a wave run in PARALLEL, one per 16-lane quarter
// (q = lane >> 4), 16 per 256-thread block: each keypoint's chain of dependent round trips
// (keypoint + candidate ranges -> candidates' (x, index) and descriptors -> SAD rows) overlaps the
// other three.  One keypoint per wave, four in series, took 0.388 ms per step against 0.225 here
// (profiles/r04/ab_stereo_quarters.txt).  Per keypoint (src/Frame.cc:600-770): strict-min Hamming
// over the candidate ranges (key dist<<12 | index, the winner's x carried by the key's lane); the
// 11x11 left patch and 11x21 right strip staged in the quarter's LDS slot; SAD term
// |(L - Lc) - (R - Rc)| = |(L + Rc) - (R + Lc)| on u16 pairs (two pixels per v_sad_u16), lane
// s < 11 of the quarter summing offset s - 5 over the 11 rows; parabola; depth.  Quarter
// reductions are DPP row rotations (a DPP row is 16 lanes); a quarter leaves early on its own
// (its lanes agree).  LDS 19.0 KB per block: 8 blocks (32 waves) per CU.
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {  // min over the lane's 16-lane row
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, false));  // row_ror:2
  v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false));  // row_ror:1
  return v;
}

#ifdef ORBX_STEREO_ROWS_PROBE
// Probe build only (tools/stereo_floor.py): the row origins of every keypoint that reaches the SAD
// staging (k_stereo_match records them), then
//   k_stereo_rows_only  the staging loads alone, in k_stereo_match's grid, block order and lane
//                       pattern (its FETCH_SIZE: what those reads cost as the match kernel issues them)
//   k_stereo_rows_mark  every 64-B sector those reads touch, marked once in per-buffer bitmaps, and
//   k_stereo_rows_count the marked sectors and 128-B lines counted: the unique-sector floor of the
//                       refinement's reads (orbx_debug_stereo_floor reads the totals).
constexpr int kProbeFrames = 512, kProbeKps = 2048;
__device__ uint2 g_rows_probe[kProbeFrames * kProbeKps];  // (rowL0 - imL, rowR0 - imR + 1), 0: not staged
constexpr int kProbeWords = 1 << 20;                      // per bitmap: 32M sectors (2 GiB of image)
__device__ uint32_t g_probe_bits[4][kProbeWords];         // L input, L pyramid, R input, R pyramid
__device__ unsigned long long g_probe_count[3];           // sectors, lines, staged keypoints
#endif

__global__ __launch_bounds__(SBS, 8) void k_stereo_match(StereoArgs A, const Geometry* __restrict__ G) {
  constexpr int NQ = SBS / 16;                // quarters (keypoints) per block
  __shared__ uint32_t s_raw[NQ][11 * kSadDw];  // per quarter: 11 rows x (4 left + 6 right) dwords
  __shared__ uint32_t s_sw[NQ][66 + 121];  // per quarter: u16-pair forms of the patch and strip
  const int2 bi = xcd_block2();
  const int f = bi.y, tid = threadIdx.x, lane = tid & 63, ql = lane & 15, qb = tid >> 4;
  const int nL = min(A.nL[(size_t)f * A.n_stride_L], A.maxL);
  const int iL = bi.x * NQ + qb;
  if (iL >= nL) return;
  const int2* rxi = A.rxi + (size_t)f * kMaxStereoKps;
  const uint4* rdR = A.rdesc + (size_t)f * kMaxStereoKps * 2;
  const orbx_keypoint* kL = A.kpL + (size_t)f * A.kL_stride;
  const int limg = f * A.l_step + A.l_off, rimg = f * A.r_step + A.r_off;
  const orbx_keypoint kp = kL[iL];
  const uint4 lrg = A.lrange[(size_t)f * A.maxL + iL];
  uint64_t ld[4];
  {
    const uint64_t* p = (const uint64_t*)(A.dL + ((size_t)f * A.kL_stride + iL) * 32);
    ld[0] = p[0]; ld[1] = p[1]; ld[2] = p[2]; ld[3] = p[3];
  }
  const int levelL = kp.octave;
  const float uL = kp.x;
  const float minU = uL - A.maxD, maxU = uL - A.minD;
  float* outU = A.uR + (size_t)f * A.out_stride + iL;
  float* outD = A.depth + (size_t)f * A.out_stride + iL;
  int* outS = A.sad + (size_t)f * A.out_stride + iL;
  if (ql == 0) {
    *outU = -1.0f;
    *outD = -1.0f;
    *outS = -1;
  }
#ifdef ORBX_STEREO_ROWS_PROBE
  if (ql == 0 && f < kProbeFrames && iL < kProbeKps) g_rows_probe[f * kProbeKps + iL] = make_uint2(0u, 0u);
#endif
  if (maxU < 0) return;
  const uint32_t t3[3] = {lrg.x, lrg.y, lrg.z};
  int rb[3], re[3];
#pragma unroll
  for (int q = 0; q < 3; q++) {
    rb[q] = (int)(t3[q] & 0xFFFF);
    re[q] = (int)(t3[q] >> 16);
  }
  const int n0 = re[0] - rb[0], n1 = re[1] - rb[1], n2 = re[2] - rb[2];
  const int K = n0 + n1 + n2;
  uint32_t best = 0xFFFFFFFFu;
  float bestX = 0.f;
  for (int j = ql; j < K; j += 16) {
    const int pos = j < n0 ? rb[0] + j : (j < n0 + n1 ? rb[1] + (j - n0) : rb[2] + (j - n0 - n1));
    const int2 xi = rxi[pos];
    const uint4 r0 = rdR[2 * pos], r1 = rdR[2 * pos + 1];
    const float uR = __int_as_float(xi.x);
    if (!(uR >= minU && uR <= maxU)) continue;
    const uint64_t rd[4] = {(uint64_t)r0.x | ((uint64_t)r0.y << 32), (uint64_t)r0.z | ((uint64_t)r0.w << 32),
                            (uint64_t)r1.x | ((uint64_t)r1.y << 32), (uint64_t)r1.z | ((uint64_t)r1.w << 32)};
    const int dist = hamming256(ld, rd);
    const uint32_t key = ((uint32_t)dist << 12) | (uint32_t)xi.y;
    if (key < best) {
      best = key;
      bestX = uR;
    }
  }
  const uint32_t wbest = row_min_u32(best);
  const int bestDist = wbest == 0xFFFFFFFFu ? 100 : (int)(wbest >> 12);
  if (bestDist >= 75) return;  // thOrbDist = (TH_HIGH+TH_LOW)/2 (also < TH_HIGH)
  const LevelGeom& Lv = G->lv[levelL];
  const uint64_t om = __ballot(best == wbest) >> (lane & 48);
  const int owner = (lane & 48) + __builtin_ctzll(om & 0xFFFF);
  const float uR0 = __shfl(bestX, owner, 64);
  const float sf = A.inv_scale[levelL];
  const float scaleduL = __builtin_roundf(kp.x * sf);
  const float scaledvL = __builtin_roundf(kp.y * sf);
  const float scaleduR0 = __builtin_roundf(uR0 * sf);
  const int w = 5, L = 5;
  const float iniu = scaleduR0 + L - w;
  const float endu = scaleduR0 + L + w + 1;
  if (iniu < 0 || endu >= Lv.w) return;
  if (scaleduR0 - 2 * w < 0 || scaledvL - w < 0 || scaledvL + w >= Lv.h || scaleduL - w < 0 ||
      scaleduL + w >= Lv.w)
    return;
  const uint8_t* imL = level_ptr(*G, A.BL, limg, levelL);
  const uint8_t* imR = level_ptr(*G, A.BR, rimg, levelL);
  const int lw = Lv.w;
  const int cy = (int)scaledvL, cxL = (int)scaleduL, cxR0 = (int)scaleduR0;
  uint32_t* sp = s_raw[qb];
  const uint8_t* rowL0 = imL + (size_t)(cy - w) * lw + (cxL - w);
  const uint8_t* rowR0 = imR + (size_t)(cy - w) * lw + (cxR0 - 2 * w);
#ifdef ORBX_STEREO_ROWS_PROBE
  if (ql == 0 && f < kProbeFrames && iL < kProbeKps)
    g_rows_probe[f * kProbeKps + iL] = make_uint2((uint32_t)(rowL0 - imL), (uint32_t)(rowR0 - imR) + 1u);
#endif
  {
    constexpr int IT = (11 * kSadDw + 15) / 16;
    uint32_t sv[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
      const int q = ql + 16 * k, r = q / kSadDw, j = q - r * kSadDw;
      const bool left = j < kSadDwL;
      const uintptr_t a = (uintptr_t)((left ? rowL0 : rowR0) + (size_t)r * lw);
      const int jj = left ? j : j - kSadDwL, need = left ? 2 * w + 1 : 4 * w + 1;
      sv[k] = 0;
      if (q < 11 * kSadDw && 4 * jj < (int)(a & 3) + need) sv[k] = *((const uint32_t*)(a & ~(uintptr_t)3) + jj);
    }
#pragma unroll
    for (int k = 0; k < IT; k++)
      if (ql + 16 * k < 11 * kSadDw) sp[ql + 16 * k] = sv[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(sp);
  const uint32_t aL0 = (uint32_t)(uintptr_t)rowL0, aR0 = (uint32_t)(uintptr_t)rowR0;
  auto lpix = [&](int dy, int dx) -> int { return sb[4 * kSadDw * dy + ((aL0 + (uint32_t)(dy * lw)) & 3) + dx]; };
  auto rpix = [&](int dy, int dx) -> int {
    return sb[4 * (kSadDw * dy + kSadDwL) + ((aR0 + (uint32_t)(dy * lw)) & 3) + dx];
  };
  uint32_t* l16 = s_sw[qb];
  uint32_t* re16 = l16 + 66;
  const uint32_t Lc = (uint32_t)lpix(w, w);
  for (int q = ql; q < 66; q += 16) {
    const int r = q / 6, k = q - r * 6;
    l16[q] = (uint32_t)lpix(r, 2 * k) | (2 * k + 1 <= 2 * w ? (uint32_t)lpix(r, 2 * k + 1) << 16 : 0u);
  }
  for (int q = ql; q < 121; q += 16) {
    const int r = q / 11, k = q - r * 11;
    const uint32_t a = (uint32_t)rpix(r, 2 * k) + Lc;
    const uint32_t b = (2 * k + 1 <= 4 * w ? (uint32_t)rpix(r, 2 * k + 1) : 0u) + Lc;
    re16[q] = a | b << 16;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int so = ql < 11 ? ql : 0;
  const uint32_t rc = (uint32_t)rpix(w, so + w);  // Rc = strip column inc + 2w
  const u16x2 rc2 = {(uint16_t)rc, (uint16_t)rc};
  // strip pairs (so + 2p, so + 2p + 1): the even-aligned pairs re16[so/2 + p] themselves, or for an odd
  // offset the middle halves of two neighbours (one v_alignbyte; the odd-aligned copy is not stored)
  const uint32_t* rrow = re16 + (so >> 1);
  const uint32_t sh = (uint32_t)(so & 1) * 2;
  uint32_t acc = 0;
#pragma unroll
  for (int dy = 0; dy < 2 * w + 1; dy++) {
    uint32_t wv[7];
#pragma unroll
    for (int t = 0; t < 7; t++) wv[t] = rrow[dy * 11 + t];  // (the 7th may run into the next row: used only when odd)
#pragma unroll
    for (int p2 = 0; p2 < 6; p2++) {
      uint32_t lp = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, l16[dy * 6 + p2]) + rc2);
      uint32_t rp = __builtin_amdgcn_alignbyte(wv[p2 + 1], wv[p2], sh);
      if (p2 == 5) {
        lp &= 0xFFFFu;
        rp &= 0xFFFFu;
      }
      acc = __builtin_amdgcn_sad_u16(lp, rp, acc);
    }
  }
  const int sad = (int)acc;
  // first strict minimum over inc = -5..5 (quarter lanes 0..10)
  const uint32_t skey = row_min_u32(ql < 11 ? ((uint32_t)sad << 4) | (uint32_t)ql : 0xFFFFFFFFu);
  const int bix = (int)(skey & 15);
  const int bestSad = (int)(skey >> 4);
  const int bestinc = bix - L;
  const int qbase = lane & 48;
  const float d1 = (float)__shfl(sad, qbase + max(bix - 1, 0), 64);
  const float d3 = (float)__shfl(sad, qbase + min(bix + 1, 15), 64);
  if (bestinc == -L || bestinc == L) return;
  const float d2 = (float)bestSad;
  const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
  if (deltaR < -1 || deltaR > 1) return;
  float bestuR = Lv.scale * ((float)scaleduR0 + (float)bestinc + deltaR);
  float disparity = uL - bestuR;
  if (disparity >= A.minD && disparity < A.maxD) {
    if (disparity <= 0) {
      disparity = 0.01f;
      bestuR = uL - 0.01f;
    }
    if (ql == 0) {
      *outD = A.bf / disparity;
      *outU = bestuR;
      *outS = bestSad;
    }
  }
}

__global__ __launch_bounds__(SBS) void k_stereo_finalize(StereoArgs A) {
  __shared__ int hist[256];
  __shared__ int sel[4];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int nL = min(A.nL[(size_t)f * A.n_stride_L], A.maxL);
  const int* sad = A.sad + (size_t)f * A.out_stride;
  float* uR = A.uR + (size_t)f * A.out_stride;
  float* depth = A.depth + (size_t)f * A.out_stride;
  for (int i = tid; i < 256; i += SBS) hist[i] = 0;
  __syncthreads();
  for (int i = tid; i < nL; i += SBS) {
    const int s = sad[i];
    if (s >= 0) atomicAdd(&hist[(s >> 8) & 255], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int b = 0; b < 256; b++) n += hist[b];
    sel[0] = n;
    const int k = n / 2;
    int acc = 0, b = 0;
    for (; b < 256; b++) {
      if (acc + hist[b] > k) break;
      acc += hist[b];
    }
    sel[1] = b;
    sel[2] = k - acc;
  }
  __syncthreads();
  const int n = sel[0];
  if (n == 0) {
    if (tid == 0) A.nmatches[f] = 0;
    return;
  }
  const int hb = sel[1], k2 = sel[2];
  __syncthreads();
  for (int i = tid; i < 256; i += SBS) hist[i] = 0;
  __syncthreads();
  for (int i = tid; i < nL; i += SBS) {
    const int s = sad[i];
    if (s >= 0 && ((s >> 8) & 255) == hb) atomicAdd(&hist[s & 255], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0, b = 0;
    for (; b < 256; b++) {
      if (acc + hist[b] > k2) break;
      acc += hist[b];
    }
    sel[3] = (hb << 8) | b;
  }
  __syncthreads();
  const float median = (float)sel[3];
  const float th = 1.5f * 1.4f * median;
  int kept = 0;
  for (int i = tid; i < nL; i += SBS) {
    const int s = sad[i];
    if (s < 0) continue;
    if ((float)s >= th) {
      uR[i] = -1.0f;
      depth[i] = -1.0f;
    } else {
      kept++;
    }
  }
  kept = wave_sum(kept);
  __shared__ int ksum;
  if (tid == 0) ksum = 0;
  __syncthreads();
  if ((tid & 63) == 0) atomicAdd(&ksum, kept);
  __syncthreads();
  if (tid == 0) A.nmatches[f] = ksum;
}

__global__ __launch_bounds__(SBS) void k_hamming(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int n,
                                                 int32_t* __restrict__ out) {
  const int i = blockIdx.x * SBS + threadIdx.x;
  if (i >= n) return;
  const uint64_t* pa = (const uint64_t*)(a + (size_t)i * 32);
  const uint64_t* pb = (const uint64_t*)(b + (size_t)i * 32);
  uint64_t x[4] = {pa[0], pa[1], pa[2], pa[3]};
  uint64_t y[4] = {pb[0], pb[1], pb[2], pb[3]};
  out[i] = hamming256(x, y);
}

#ifdef ORBX_STEREO_ROWS_PROBE
// the staged reads of keypoint (f, iL): calls fn(side, level 0?, dword address) for each dword k_stereo_match
// loads (11 rows x 4 left / 6 right dwords at the 4-aligned row starts, dwords past the span skipped)
template <typename Fn>
__device__ inline void probe_rows(const StereoArgs& A, const Geometry* G, int f, int iL, int ql, Fn fn) {
  const uint2 rec = g_rows_probe[f * kProbeKps + iL];
  if (rec.y == 0) return;
  const orbx_keypoint kp = (A.kpL + (size_t)f * A.kL_stride)[iL];
  const int limg = f * A.l_step + A.l_off, rimg = f * A.r_step + A.r_off;
  const uint8_t* rowL0 = level_ptr(*G, A.BL, limg, kp.octave) + rec.x;
  const uint8_t* rowR0 = level_ptr(*G, A.BR, rimg, kp.octave) + (rec.y - 1u);
  const int lw = G->lv[kp.octave].w, w = 5;
  constexpr int IT = (11 * kSadDw + 15) / 16;
#pragma unroll
  for (int k = 0; k < IT; k++) {
    const int q = ql + 16 * k, r = q / kSadDw, j = q - r * kSadDw;
    const bool left = j < kSadDwL;
    const uintptr_t a = (uintptr_t)((left ? rowL0 : rowR0) + (size_t)r * lw);
    const int jj = left ? j : j - kSadDwL, need = left ? 2 * w + 1 : 4 * w + 1;
    if (q < 11 * kSadDw && 4 * jj < (int)(a & 3) + need)
      fn(left ? 0 : 1, kp.octave == 0, (a & ~(uintptr_t)3) + 4 * (uintptr_t)jj);
  }
}

__global__ __launch_bounds__(SBS) void k_stereo_rows_only(StereoArgs A, const Geometry* __restrict__ G, uint32_t* sink) {
  constexpr int NQ = SBS / 16;
  const int2 bi = xcd_block2();
  const int f = bi.y, tid = threadIdx.x, ql = tid & 15, qb = tid >> 4;
  const int nL = min(A.nL[(size_t)f * A.n_stride_L], A.maxL);
  const int iL = bi.x * NQ + qb;
  if (iL >= nL || f >= kProbeFrames || iL >= kProbeKps) return;
  uint32_t x = 0;
  probe_rows(A, G, f, iL, ql, [&](int, bool, uintptr_t a) { x ^= *(const uint32_t*)a; });
  if (x == 0x9E3779B9u) sink[0] = x;  // keeps the loads
}

// bitmap slot of a dword address: which buffer (level 0 = the input images, else the pyramid) of
// which side, and the 64-B sector index from the buffer's start
__device__ inline void probe_mark(const StereoArgs& A, int side, bool l0, uintptr_t a) {
  const BatchPtrs& B = side ? A.BR : A.BL;
  const int m = 2 * side + (l0 ? 0 : 1);
  const uintptr_t off = a - (l0 ? (uintptr_t)B.in : (uintptr_t)B.pyr);
  const unsigned long long sec = off >> 6;
  if (sec < 32ull * kProbeWords) atomicOr(&g_probe_bits[m][sec >> 5], 1u << (sec & 31));
}

__global__ __launch_bounds__(SBS) void k_stereo_rows_mark(StereoArgs A, const Geometry* __restrict__ G) {
  constexpr int NQ = SBS / 16;
  const int f = blockIdx.y, tid = threadIdx.x, ql = tid & 15, qb = tid >> 4;
  const int nL = min(A.nL[(size_t)f * A.n_stride_L], A.maxL);
  const int iL = blockIdx.x * NQ + qb;
  if (iL >= nL || f >= kProbeFrames || iL >= kProbeKps) return;
  if (ql == 0 && g_rows_probe[f * kProbeKps + iL].y) atomicAdd(&g_probe_count[2], 1ull);
  probe_rows(A, G, f, iL, ql, [&](int side, bool l0, uintptr_t a) { probe_mark(A, side, l0, a); });
}

// counts the marked sectors and 128-B lines and clears the bitmaps for the next call
__global__ __launch_bounds__(256) void k_stereo_rows_count() {
  unsigned long long s = 0, l = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < 4 * kProbeWords; i += gridDim.x * 256) {
    uint32_t* wp = &g_probe_bits[i / kProbeWords][i % kProbeWords];
    const uint32_t v = *wp;
    if (v) {
      s += __popc(v);
      l += __popc((v | (v >> 1)) & 0x55555555u);
      *wp = 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {  // wave sums, one atomic per wave
    s += __shfl_down(s, o, 64);
    l += __shfl_down(l, o, 64);
  }
  if ((threadIdx.x & 63) == 0 && (s || l)) {
    atomicAdd(&g_probe_count[0], s);
    atomicAdd(&g_probe_count[1], l);
  }
}
#endif

hipError_t launch_stereo(const StereoArgs& A, const Geometry* Gd, int n_frames, int maxL, hipStream_t st,
                         StageTimer* T) {
  T->begin(st);
  hipLaunchKernelGGL(k_stereo_prep, dim3(n_frames), dim3(PBS), 0, st, A, Gd);
  T->end(ST_STEREO_PREP, st);
  const int nb = (maxL + kKpsPerBlock - 1) / kKpsPerBlock;
  T->begin(st);
  hipLaunchKernelGGL(k_stereo_match, dim3(max(nb, 1), n_frames), dim3(SBS), 0, st, A, Gd);
  T->end(ST_STEREO_MATCH, st);
  T->begin(st);
  hipLaunchKernelGGL(k_stereo_finalize, dim3(n_frames), dim3(SBS), 0, st, A);
  T->end(ST_STEREO_FINAL, st);
#ifdef ORBX_STEREO_ROWS_PROBE
  hipLaunchKernelGGL(k_stereo_rows_only, dim3(max(nb, 1), n_frames), dim3(SBS), 0, st, A, Gd, (uint32_t*)A.nmatches);
  hipLaunchKernelGGL(k_stereo_rows_mark, dim3(max(nb, 1), n_frames), dim3(SBS), 0, st, A, Gd);
  hipLaunchKernelGGL(k_stereo_rows_count, dim3(1024), dim3(256), 0, st);
#endif
  return hipGetLastError();
}

hipError_t launch_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hamming, dim3((n + SBS - 1) / SBS), dim3(SBS), 0, st, a, b, n, out);
  return hipGetLastError();
}

}  // namespace orbx

#ifdef ORBX_STEREO_ROWS_PROBE
// probe builds only: totals since the last call (64-B sectors, 128-B lines, staged keypoints), reset
extern "C" int orbx_debug_stereo_floor(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  unsigned long long h[3] = {0, 0, 0};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(orbx::g_probe_count), sizeof(h)) != hipSuccess) return -1;
  const unsigned long long z[3] = {0, 0, 0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(orbx::g_probe_count), z, sizeof(z)) != hipSuccess) return -1;
  for (int i = 0; i < 3; i++) out[i] = h[i];
  return 0;
}
#endif
