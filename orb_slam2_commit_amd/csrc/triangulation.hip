// triangulation.hip -- ORBmatcher::SearchForTriangulation
// (src/ORBmatcher.cc:738-925) with CheckDistEpipolarLine (:153-173) and
// ComputeThreeMaxima (:1797-1839), batched: one block per KeyFrame pair.
//
// In this reference commit vbMatched2 is never set (:760, :810), so each KF1
// feature's match depends only on its own FeatureVector node: waves take the
// nodes, lanes the KF2 features of a node.  The reference's scan keeps a
// candidate when dist <= bestDist and the epipolar test passes, i.e. the
// minimum distance with the LAST passing candidate on ties: a min over keys
// dist << 16 | (0xFFFF - position).
//
// Roofline: per KF2 node feature 32 B descriptor + 20 B geometry loaded once
// per node (register cache of 256 features), per KF1 feature 32 B + 12 B;
// latency-bound per node, throughput from the batch.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "orbx_scratch.h"
#include "orbx_device.h"
#include "orbx_internal.h"

namespace orbx {
namespace tri {

constexpr int TBS = 256;
constexpr int kOwn = 4;  // KF2 node features per lane held in registers

__device__ __forceinline__ int rot_bin(float a, float b) {
  float rot = a - b;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)__builtin_roundf(rot * (1.0f / 30));
  if (bin == 30) bin = 0;
  return bin;
}

__global__ __launch_bounds__(TBS) void k_search_for_triangulation(const orbx_tri_problem* __restrict__ probs) {
  __shared__ int s_hist[32];
  __shared__ int s_sel[3];
  __shared__ int s_count, s_drop;
  const orbx_tri_problem& P = probs[blockIdx.x];
  const orbx_tri_kf &K1 = P.kf1, &K2 = P.kf2;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < K1.n; i += TBS) P.match12[i] = -1;
  if (tid < 32) s_hist[tid] = 0;
  if (tid == 0) {
    s_count = 0;
    s_drop = 0;
  }
  // epipole of KF1 in KF2 (src/ORBmatcher.cc:748-756)
  float C2[3];
#pragma unroll
  for (int r = 0; r < 3; r++) {  // R2w*Cw+t2w: cv::gemm's small-matrix path (float dot, then + t)
    const float t0 = P.T2w[4 * r] * P.C1w[0] + P.T2w[4 * r + 1] * P.C1w[1] + P.T2w[4 * r + 2] * P.C1w[2];
    C2[r] = (float)((double)t0 + (double)P.T2w[4 * r + 3]);
  }
  const float invz = 1.0f / C2[2];
  const float ex = P.fx * C2[0] * invz + P.cx;
  const float ey = P.fy * C2[1] * invz + P.cy;
  __syncthreads();
  int cnt = 0;
  for (int jb = wid; jb < K2.n_nodes; jb += TBS / 64) {
    const uint32_t id = K2.node_id[jb];
    int lo = 0, hi = K1.n_nodes;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (K1.node_id[m] < id) lo = m + 1; else hi = m;
    }
    if (lo >= K1.n_nodes || K1.node_id[lo] != id) continue;
    const int b0 = K2.node_off[jb], nb = K2.node_off[jb + 1] - b0;
    // lane-owned KF2 candidates (positions lane + 64 t)
    uint64_t rd[kOwn][4];
    float rx[kOwn], ry[kOwn], rang[kOwn];
    int roct[kOwn], ridx[kOwn];
    uint32_t ok2 = 0, st2 = 0;
#pragma unroll
    for (int t = 0; t < kOwn; t++) {
      const int pos = lane + 64 * t;
      ridx[t] = -1;
      rx[t] = ry[t] = rang[t] = 0.f;
      roct[t] = 0;
      rd[t][0] = rd[t][1] = rd[t][2] = rd[t][3] = 0;
      if (pos < nb) {
        const int idx = K2.feat[b0 + pos];
        ridx[t] = idx;
        const uint64_t* d = (const uint64_t*)(K2.desc + (size_t)idx * 32);
        rd[t][0] = d[0]; rd[t][1] = d[1]; rd[t][2] = d[2]; rd[t][3] = d[3];
        const orbx_keypoint kp = K2.keys_un[idx];
        rx[t] = kp.x;
        ry[t] = kp.y;
        roct[t] = kp.octave;
        rang[t] = kp.angle;
        const bool stereo = K2.u_right && K2.u_right[idx] >= 0;
        const bool usable = !(K2.has_mp && K2.has_mp[idx]) && (!P.only_stereo || stereo);
        ok2 |= (uint32_t)usable << t;
        st2 |= (uint32_t)stereo << t;
      }
    }
    const int a0 = K1.node_off[lo], na = K1.node_off[lo + 1] - a0;
    for (int pa = 0; pa < na; pa++) {
      const int idx1 = K1.feat[a0 + pa];
      if (K1.has_mp && K1.has_mp[idx1]) continue;
      const bool st1 = K1.u_right && K1.u_right[idx1] >= 0;
      if (P.only_stereo && !st1) continue;
      const orbx_keypoint kp1 = K1.keys_un[idx1];
      uint64_t da[4];
      {
        const uint64_t* d = (const uint64_t*)(K1.desc + (size_t)idx1 * 32);
        da[0] = d[0]; da[1] = d[1]; da[2] = d[2]; da[3] = d[3];
      }
      // epipolar line of kp1 in KF2: l = x1' F12 (CheckDistEpipolarLine, :156-158)
      const float* F = P.F12;
      const float la = kp1.x * F[0] + kp1.y * F[3] + F[6];
      const float lb = kp1.x * F[1] + kp1.y * F[4] + F[7];
      const float lc = kp1.x * F[2] + kp1.y * F[5] + F[8];
      const float den = la * la + lb * lb;
      uint32_t best = 0xFFFFFFFFu;
      auto consider = [&](int pos, const uint64_t* d2, float x2, float y2, int o2, bool stereo2) {
        const int dist = hamming256(da, d2);
        if (dist > 50) return;  // TH_LOW (bestDist only ever decreases from TH_LOW)
        if (!st1 && !stereo2) {
          const float dx = ex - x2, dy = ey - y2;
          if (dx * dx + dy * dy < 100 * P.scale_factors2[o2]) return;
        }
        if (den == 0) return;
        const float num = la * x2 + lb * y2 + lc;
        const float dsqr = num * num / den;
        if (!(dsqr < 3.84 * P.level_sigma2_2[o2])) return;
        const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)(0xFFFF - pos);
        best = key < best ? key : best;
      };
#pragma unroll
      for (int t = 0; t < kOwn; t++)
        if ((ok2 >> t) & 1) consider(lane + 64 * t, rd[t], rx[t], ry[t], roct[t], (st2 >> t) & 1);
      for (int pos = lane + 64 * kOwn; pos < nb; pos += 64) {  // nodes beyond the register cache
        const int idx = K2.feat[b0 + pos];
        const bool stereo = K2.u_right && K2.u_right[idx] >= 0;
        if ((K2.has_mp && K2.has_mp[idx]) || (P.only_stereo && !stereo)) continue;
        const uint64_t* d = (const uint64_t*)(K2.desc + (size_t)idx * 32);
        const uint64_t x[4] = {d[0], d[1], d[2], d[3]};
        const orbx_keypoint kp = K2.keys_un[idx];
        consider(pos, x, kp.x, kp.y, kp.octave, stereo);
      }
      const uint32_t b = wave_min_u32(best);
      if (b == 0xFFFFFFFFu) continue;
      const int bpos = 0xFFFF - (int)(b & 0xFFFF);
      if (lane == 0) {
        const int idx2 = K2.feat[b0 + bpos];
        P.match12[idx1] = idx2;
        cnt++;
        if (P.check_ori) atomicAdd(&s_hist[rot_bin(kp1.angle, K2.keys_un[idx2].angle)], 1);
      }
    }
  }
  if (lane == 0) atomicAdd(&s_count, cnt);
  __threadfence_block();
  __syncthreads();
  if (P.check_ori) {
    if (tid == 0) {
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
    int drop = 0;
    for (int i = tid; i < K1.n; i += TBS) {
      const int m = P.match12[i];
      if (m < 0) continue;
      const int b = rot_bin(K1.keys_un[i].angle, K2.keys_un[m].angle);
      if (b != s_sel[0] && b != s_sel[1] && b != s_sel[2]) {
        P.match12[i] = -1;
        drop++;
      }
    }
    atomicAdd(&s_drop, drop);
    __syncthreads();
  }
  if (tid == 0) *P.nmatches = s_count - s_drop;
}

}  // namespace tri
}  // namespace orbx

// ------------------------------------------------------------------ C ABI
namespace {

bool tri_kf_ok(const orbx_tri_kf& k) {
  if (k.n < 0 || k.n_nodes < 0) return false;
  if (k.n > 0 && (!k.keys_un || !k.desc)) return false;
  if (k.n_nodes > 0 && (!k.node_id || !k.node_off || !k.feat)) return false;
  return true;
}

orbx_status tri_check(const orbx_tri_problem& p) {
  if (!tri_kf_ok(p.kf1) || !tri_kf_ok(p.kf2) || !p.nmatches || (p.kf1.n > 0 && !p.match12)) return ORBX_ERR_ARG;
  return ORBX_OK;
}

}  // namespace

extern "C" orbx_status orbx_search_for_triangulation(const orbx_tri_problem* p, int device) {
  if (!p) return ORBX_ERR_ARG;
  const orbx_status chk = tri_check(*p);
  if (chk != ORBX_OK) return chk;
  for (int s = 0; s < 2; s++) {  // host-side check of the CSR the kernel trusts
    const orbx_tri_kf& k = s ? p->kf2 : p->kf1;
    if (k.n_nodes > 0 && (k.node_off[0] != 0 || k.node_off[k.n_nodes] < 0)) return ORBX_ERR_ARG;
    for (int j = 0; j < k.n_nodes; j++)
      if (k.node_off[j + 1] < k.node_off[j]) return ORBX_ERR_ARG;
    const int nf = k.n_nodes ? k.node_off[k.n_nodes] : 0;
    for (int j = 0; j < nf; j++)
      if (k.feat[j] < 0 || k.feat[j] >= k.n) return ORBX_ERR_ARG;
    for (int i = 0; i < k.n; i++)
      if (k.keys_un[i].octave < 0 || k.keys_un[i].octave > 15) return ORBX_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  size_t off = 0;
  struct Item { const void* src; size_t bytes; size_t at; };
  std::vector<Item> items;
  auto put = [&](const void* src, size_t bytes) -> size_t {
    off = (off + 255) & ~(size_t)255;
    items.push_back({src, bytes, off});
    const size_t at = off;
    off += bytes;
    return at;
  };
  size_t a[2][8];
  for (int s = 0; s < 2; s++) {
    const orbx_tri_kf& k = s ? p->kf2 : p->kf1;
    const size_t nf = k.n_nodes ? (size_t)k.node_off[k.n_nodes] : 0;
    a[s][0] = put(k.keys_un, (size_t)k.n * sizeof(orbx_keypoint));
    a[s][1] = put(k.desc, (size_t)k.n * 32);
    a[s][2] = k.u_right ? put(k.u_right, (size_t)k.n * 4) : 0;
    a[s][3] = k.has_mp ? put(k.has_mp, (size_t)k.n) : 0;
    a[s][4] = put(k.node_id, (size_t)k.n_nodes * 4);
    a[s][5] = put(k.node_off, (size_t)(k.n_nodes + 1) * 4);
    a[s][6] = put(k.feat, nf * 4);
  }
  const size_t a_m = put(nullptr, (size_t)p->kf1.n * 4), a_n = put(nullptr, 4);
  const size_t a_p = put(nullptr, sizeof(orbx_tri_problem));
  orbx::ScratchGuard g(device);  // pooled lease: no per-call allocation (orbx_scratch.h)
  if (!g.l || g.l->reserve(off, off) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* hst = g.l->h;
  std::memset(hst, 0, off);
  for (const Item& it : items)
    if (it.src && it.bytes) std::memcpy(hst + it.at, it.src, it.bytes);
  uint8_t* d = g.l->d;
  orbx_tri_problem q = *p;
  for (int s = 0; s < 2; s++) {
    const orbx_tri_kf& k = s ? p->kf2 : p->kf1;
    orbx_tri_kf& o = s ? q.kf2 : q.kf1;
    o.keys_un = (const orbx_keypoint*)(d + a[s][0]);
    o.desc = d + a[s][1];
    o.u_right = k.u_right ? (const float*)(d + a[s][2]) : nullptr;
    o.has_mp = k.has_mp ? d + a[s][3] : nullptr;
    o.node_id = (const uint32_t*)(d + a[s][4]);
    o.node_off = (const int32_t*)(d + a[s][5]);
    o.feat = (const int32_t*)(d + a[s][6]);
  }
  q.match12 = (int32_t*)(d + a_m);
  q.nmatches = (int32_t*)(d + a_n);
  std::memcpy(hst + a_p, &q, sizeof(q));
  hipStream_t st = g.l->st;
  hipError_t e = hipMemcpyAsync(d, hst, off, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::tri::k_search_for_triangulation, dim3(1), dim3(orbx::tri::TBS), 0, st,
                       (const orbx_tri_problem*)(d + a_p));
    e = hipGetLastError();
  }
  // match12 and the count are adjacent: one copy back
  if (e == hipSuccess) e = hipMemcpyAsync(hst + a_m, d + a_m, a_p - a_m, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = g.l->sync();
  if (e != hipSuccess) return ORBX_ERR_HIP;
  if (p->kf1.n) std::memcpy(p->match12, hst + a_m, (size_t)p->kf1.n * 4);
  std::memcpy(p->nmatches, hst + a_n, 4);
  return ORBX_OK;
}

extern "C" orbx_status orbx_search_for_triangulation_device(const orbx_tri_problem* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++)
    if (tri_check(problems[i]) != ORBX_OK) return ORBX_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  orbx_tri_problem* dP = nullptr;
  if (hipMallocAsync((void**)&dP, sizeof(orbx_tri_problem) * n, st) != hipSuccess) return ORBX_ERR_HIP;
  hipError_t e = hipMemcpyAsync(dP, problems, sizeof(orbx_tri_problem) * n, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::tri::k_search_for_triangulation, dim3(n), dim3(orbx::tri::TBS), 0, st, dP);
    e = hipGetLastError();
  }
  const hipError_t e2 = hipFreeAsync(dP, st);
  return (e != hipSuccess || e2 != hipSuccess) ? ORBX_ERR_HIP : ORBX_OK;
}
