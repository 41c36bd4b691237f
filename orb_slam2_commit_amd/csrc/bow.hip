// bow.hip -- ORBmatcher::SearchByBoW (src/ORBmatcher.cc:175-325 KF-Frame,
// :589-736 KF-KF) and ComputeThreeMaxima (:1797-1839), batched: one block per
// problem.
//
// Every feature belongs to exactly one FeatureVector node, so the "already
// matched" state is node-local: nodes run in parallel (one wave each), the
// first side's features of a node run sequentially, and the second side's
// features of the node are spread over the lanes.  best1 = min key and
// best2 = second-smallest key over (dist << 16 | position) reproduce the
// reference's sequential best/second-best scan exactly (first position wins
// ties; best2 counts duplicates).
#include <hip/hip_runtime.h>

#include "orbx_device.h"
#include "orbx_internal.h"
#include "orbx_bow.h"

namespace orbx {

constexpr int BBS = 256;
constexpr int kOwn = 4;  // second-side features per lane held in registers (256 per node)

__device__ __forceinline__ int rot_bin(float a, float b) {
  const float factor = 1.0f / 30;
  float rot = a - b;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)__builtin_roundf(rot * factor);
  if (bin == 30) bin = 0;
  return bin;
}

__global__ __launch_bounds__(BBS) void k_search_by_bow(const BowProblem* __restrict__ probs) {
  __shared__ int32_t smatch[kMaxBowFeatures];
  __shared__ uint32_t bmatched[kMaxBowFeatures / 32];  // second-side features matched so far
  __shared__ int hist[32];
  __shared__ int sel[4];
  BowProblem P = probs[blockIdx.x];
  // device-sized sides: the counts an earlier kernel of the stream wrote, capped by the capacities
  if (P.a_n_dev) P.a.n = min(max(*P.a_n_dev, 0), P.a.n);
  if (P.a_nodes_dev) P.a.n_nodes = min(max(*P.a_nodes_dev, 0), P.a.n_nodes);
  if (P.b_n_dev) P.b.n = min(max(*P.b_n_dev, 0), P.b.n);
  if (P.b_nodes_dev) P.b.n_nodes = min(max(*P.b_nodes_dev, 0), P.b.n_nodes);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool kfkf = P.mode == 1;
  const int nout = kfkf ? P.a.n : P.b.n;
  for (int i = tid; i < nout; i += BBS) smatch[i] = -1;
  for (int i = tid; i < kMaxBowFeatures / 32; i += BBS) bmatched[i] = 0;
  if (tid < 32) hist[tid] = 0;
  __syncthreads();
  for (int jb = wid; jb < P.b.n_nodes; jb += BBS / 64) {
    const uint32_t id = P.b.node_id[jb];
    int lo = 0, hi = P.a.n_nodes;  // lower_bound in the first side's node ids
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (P.a.node_id[m] < id) lo = m + 1; else hi = m;
    }
    if (lo >= P.a.n_nodes || P.a.node_id[lo] != id) continue;
    const int ia = lo;
    const int b0 = P.b.node_off[jb], nb = P.b.node_off[jb + 1] - b0;
    // lane-owned second-side features (positions lane + 64*t)
    uint64_t rd[kOwn][4];
    int ridx[kOwn];
    uint32_t avail = 0;  // bit t: position usable (valid, not yet matched)
#pragma unroll
    for (int t = 0; t < kOwn; t++) {
      const int pos = lane + 64 * t;
      ridx[t] = -1;
      if (pos < nb) {
        const int idx = P.b.feat[b0 + pos];
        ridx[t] = idx;
        const uint64_t* d = (const uint64_t*)(P.b.desc + (size_t)idx * 32);
        rd[t][0] = d[0]; rd[t][1] = d[1]; rd[t][2] = d[2]; rd[t][3] = d[3];
        const bool ok = !kfkf || !P.b.valid || P.b.valid[idx];
        avail |= (uint32_t)ok << t;
      }
    }
    const int a0 = P.a.node_off[ia], na = P.a.node_off[ia + 1] - a0;
    for (int pa = 0; pa < na; pa++) {
      const int idxA = P.a.feat[a0 + pa];
      if (P.a.valid && !P.a.valid[idxA]) continue;
      uint64_t da[4];
      {
        const uint64_t* d = (const uint64_t*)(P.a.desc + (size_t)idxA * 32);
        da[0] = d[0]; da[1] = d[1]; da[2] = d[2]; da[3] = d[3];
      }
      uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;  // two smallest own keys
#pragma unroll
      for (int t = 0; t < kOwn; t++) {
        if (!((avail >> t) & 1)) continue;
        const uint32_t key = ((uint32_t)hamming256(da, rd[t]) << 16) | (uint32_t)(lane + 64 * t);
        if (key < m1) {
          m2 = m1;
          m1 = key;
        } else if (key < m2) {
          m2 = key;
        }
      }
      // nodes larger than kOwn*64: remaining positions straight from memory
      for (int pos = lane + 64 * kOwn; pos < nb; pos += 64) {
        const int idx = P.b.feat[b0 + pos];
        const bool ok = (!kfkf || !P.b.valid || P.b.valid[idx]) && !((bmatched[idx >> 5] >> (idx & 31)) & 1);
        if (!ok) continue;
        const uint64_t* d = (const uint64_t*)(P.b.desc + (size_t)idx * 32);
        uint64_t x[4] = {d[0], d[1], d[2], d[3]};
        const uint32_t key = ((uint32_t)hamming256(da, x) << 16) | (uint32_t)pos;
        if (key < m1) {
          m2 = m1;
          m1 = key;
        } else if (key < m2) {
          m2 = key;
        }
      }
      const uint32_t b1 = wave_min_u32(m1);
      const uint32_t b2 = wave_min_u32(m1 == b1 ? m2 : m1);
      const int dist1 = b1 == 0xFFFFFFFFu ? 256 : (int)(b1 >> 16);
      const int dist2 = b2 == 0xFFFFFFFFu ? 256 : (int)(b2 >> 16);
      const bool pass = kfkf ? dist1 < 50 : dist1 <= 50;  // TH_LOW, src/ORBmatcher.cc:260 / :672
      if (!pass || !((float)dist1 < P.nnratio * (float)dist2)) continue;
      const int bpos = (int)(b1 & 0xFFFF);
      int idxB;
      if (bpos < 64 * kOwn) {
        const int owner = bpos & 63, t = bpos >> 6;
        int v = -1;
#pragma unroll
        for (int u = 0; u < kOwn; u++)
          if (u == t) v = ridx[u];
        idxB = __shfl(v, owner, 64);
        if (lane == owner) avail &= ~(1u << t);
      } else {
        idxB = P.b.feat[b0 + bpos];
      }
      if (lane == 0) {
        const int out = kfkf ? idxA : idxB;
        int bin = 0;
        if (P.check_ori) {
          bin = rot_bin(P.a.angle[idxA], P.b.angle[idxB]);
          atomicAdd(&hist[bin], 1);
        }
        smatch[out] = (kfkf ? idxB : idxA) | (bin << 24);
        atomicOr(&bmatched[idxB >> 5], 1u << (idxB & 31));
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int ind1 = -1, ind2 = -1, ind3 = -1;
    if (P.check_ori) {
      int max1 = 0, max2 = 0, max3 = 0;
      for (int i = 0; i < 30; i++) {
        const int s = hist[i];
        if (s > max1) {
          max3 = max2; max2 = max1; max1 = s;
          ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
          max3 = max2; max2 = s;
          ind3 = ind2; ind2 = i;
        } else if (s > max3) {
          max3 = s;
          ind3 = i;
        }
      }
      if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
      } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
      }
    }
    sel[0] = ind1;
    sel[1] = ind2;
    sel[2] = ind3;
    sel[3] = 0;
  }
  __syncthreads();
  int kept = 0;
  for (int i = tid; i < nout; i += BBS) {
    int v = smatch[i];
    if (v >= 0) {
      const int bin = v >> 24;
      v &= 0xFFFFFF;
      if (P.check_ori && bin != sel[0] && bin != sel[1] && bin != sel[2]) v = -1;
    }
    P.match[i] = v;
    kept += v >= 0;
  }
  kept = wave_sum(kept);
  if (lane == 0) atomicAdd(&sel[3], kept);
  __syncthreads();
  if (tid == 0) *P.nmatches = sel[3];
}

hipError_t launch_search_by_bow(const BowProblem* d_probs, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_search_by_bow, dim3(n), dim3(BBS), 0, st, d_probs);
  return hipGetLastError();
}

}  // namespace orbx
