// poseopt.hip -- Optimizer::PoseOptimization (src/Optimizer.cc:287-528), one
// block per frame, the whole four-round g2o Levenberg schedule on the device.
//
// Per frame the problem is a single 6-DoF vertex with n ~ 10^2..10^3 unary
// edges (EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose, Huber),
// so the unit of parallelism is the frame batch: a block per frame keeps the
// LM state in LDS and never returns to the host between rounds, trials or
// iterations.  Inside a block the per-edge work (errors, Jacobians, the 27
// quadratic-form terms) is spread over the threads; the sums that g2o forms
// in edge insertion order (activeRobustChi2, buildSystem's H and b) are then
// taken in exactly that order, one FP64 chain per H/b entry on its own lane,
// from contiguous scratch rows.  With the deterministic sin/cos of
// SE3Quat::exp and the same Eigen-LDLT restatement as the oracle
// (oracle/poseopt.cpp), the GPU reproduces the oracle bit for bit: pose, outlier
// flags, return value and per-round iteration counts.
//
// Bound: latency (dependent FP64 chains of length n per LM iteration, ~10
// cycles per link); throughput comes from thousands of frames in flight.
// Algorithmic bytes per LM trial: 28 B of edge input + 24 B stored error +
// 8 B chi term per active edge, + 216 B of quadratic-form terms written and
// read once per iteration.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "orbx_device.h"
#include "orbx_scratch.h"
#include "orbx_internal.h"

namespace orbx {
namespace pose {

constexpr int PBS = 256;
constexpr int kRow = 32;  // scratch doubles per edge: 27 terms | err[3] | chi term | pad

struct Quat {
  double x, y, z, w;
};
struct SE3 {
  Quat q;
  double t[3];
};

__device__ __forceinline__ Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - (a.x * b.x + a.y * b.y + a.z * b.z);
  r.x = a.w * b.x + b.w * a.x + (a.y * b.z - a.z * b.y);
  r.y = a.w * b.y + b.w * a.y + (a.z * b.x - a.x * b.z);
  r.z = a.w * b.z + b.w * a.z + (a.x * b.y - a.y * b.x);
  return r;
}
__device__ __forceinline__ void qrot(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
#pragma unroll
  for (int i = 0; i < 3; i++) out[i] = v[i] + q.w * uv[i] + c[i];
}
__device__ __forceinline__ void qmat(const Quat& q, double R[9]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
__device__ __forceinline__ Quat mat2q(const double m[9]) {
  Quat q;
  double t = m[0] + m[4] + m[8];
  if (t > 0) {
    t = __builtin_sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m[7] - m[5]) * t;
    q.y = (m[2] - m[6]) * t;
    q.z = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > (i == 0 ? m[0] : m[4])) i = 2;
    // the three cases spelled out on named entries: no array indexed at run time (which put the
    // matrix in scratch memory); same arithmetic as c[i], c[j], c[k] with (i, j, k) cyclic
    if (i == 0) {  // (0, 1, 2)
      t = __builtin_sqrt(m[0] - m[4] - m[8] + 1.0);
      const double ci = 0.5 * t;
      t = 0.5 / t;
      q.w = (m[7] - m[5]) * t;
      q.x = ci;
      q.y = (m[3] + m[1]) * t;
      q.z = (m[6] + m[2]) * t;
    } else if (i == 1) {  // (1, 2, 0)
      t = __builtin_sqrt(m[4] - m[8] - m[0] + 1.0);
      const double ci = 0.5 * t;
      t = 0.5 / t;
      q.w = (m[2] - m[6]) * t;
      q.y = ci;
      q.z = (m[7] + m[5]) * t;
      q.x = (m[1] + m[3]) * t;
    } else {  // (2, 0, 1)
      t = __builtin_sqrt(m[8] - m[0] - m[4] + 1.0);
      const double ci = 0.5 * t;
      t = 0.5 / t;
      q.w = (m[3] - m[1]) * t;
      q.z = ci;
      q.x = (m[2] + m[6]) * t;
      q.y = (m[5] + m[7]) * t;
    }
  }
  return q;
}
__device__ __forceinline__ void qnormalize(Quat& q) {
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double n = __builtin_sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

__device__ __forceinline__ void sincos_d(double x, double* s_out, double* c_out) {
  const double kInvPio2 = 6.36619772367581382433e-01;
  const double kPio2Hi = 1.57079632673412561417e+00;
  const double kPio2Lo = 6.07710050650619224932e-11;
  const double kd = __builtin_rint(x * kInvPio2);
  const int q = (int)kd;
  const double r = (x - kd * kPio2Hi) - kd * kPio2Lo;
  const double r2 = r * r;
  double ps = 1.0 / 51090942171709440000.0;
  ps = ps * r2 - 1.0 / 121645100408832000.0;
  ps = ps * r2 + 1.0 / 355687428096000.0;
  ps = ps * r2 - 1.0 / 1307674368000.0;
  ps = ps * r2 + 1.0 / 6227020800.0;
  ps = ps * r2 - 1.0 / 39916800.0;
  ps = ps * r2 + 1.0 / 362880.0;
  ps = ps * r2 - 1.0 / 5040.0;
  ps = ps * r2 + 1.0 / 120.0;
  ps = ps * r2 - 1.0 / 6.0;
  const double sr = r + r * (r2 * ps);
  double pc = 1.0 / 2432902008176640000.0;
  pc = pc * r2 - 1.0 / 6402373705728000.0;
  pc = pc * r2 + 1.0 / 20922789888000.0;
  pc = pc * r2 - 1.0 / 87178291200.0;
  pc = pc * r2 + 1.0 / 479001600.0;
  pc = pc * r2 - 1.0 / 3628800.0;
  pc = pc * r2 + 1.0 / 40320.0;
  pc = pc * r2 - 1.0 / 720.0;
  pc = pc * r2 + 1.0 / 24.0;
  pc = pc * r2 - 0.5;
  const double cr = 1.0 + r2 * pc;
  double s, c;
  switch (q & 3) {
    case 0: s = sr; c = cr; break;
    case 1: s = cr; c = -sr; break;
    case 2: s = -sr; c = -cr; break;
    default: s = -cr; c = sr; break;
  }
  *s_out = s;
  *c_out = c;
}

// SE3Quat::exp(update), types/se3quat.h:223-257 (then operator* with T)
__device__ __forceinline__ SE3 se3_exp(const double u[6]) {
  const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
  const double theta = __builtin_sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double O2[9];
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
  double R[9], V[9];
  if (theta < 0.00001) {
#pragma unroll
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + O[i] + O2[i];
#pragma unroll
    for (int i = 0; i < 9; i++) V[i] = R[i];
  } else {
    double s, c;
    sincos_d(theta, &s, &c);
    const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / (theta * theta * theta);
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const double I = (i % 4) == 0 ? 1.0 : 0.0;
      R[i] = I + a * O[i] + b * O2[i];
      V[i] = I + b * O[i] + d * O2[i];
    }
  }
  SE3 T;
  T.q = mat2q(R);
#pragma unroll
  for (int r = 0; r < 3; r++) T.t[r] = V[3 * r] * up[0] + V[3 * r + 1] * up[1] + V[3 * r + 2] * up[2];
  qnormalize(T.q);
  return T;
}
__device__ __forceinline__ SE3 se3_mul(const SE3& a, const SE3& b) {
  SE3 r = a;
  double rt[3];
  qrot(a.q, b.t, rt);
#pragma unroll
  for (int i = 0; i < 3; i++) r.t[i] += rt[i];
  r.q = qmul(a.q, b.q);
  qnormalize(r.q);
  return r;
}

// Eigen::LDLT<MatrixXd> (diagonal pivoting) + solve; false when !isPositive().
// Every loop is unrolled and the pivot swaps / the permutation of the right-hand side run as
// unrolled compare-and-swap over the candidate rows, so every index is a compile-time constant:
// the matrix lives in registers (a runtime index put it in scratch memory, ~25k cycles per call
// on the LM's serial path).  Same operations in the same order as before.
// conditional exchange of two registers by value selects (a branch per candidate let the
// compiler merge the paths into pointer phis, which sends the array to scratch memory)
__device__ __forceinline__ void cswap(bool sw, double& a, double& b) {
  const double x = a, y = b;
  a = sw ? y : x;
  b = sw ? x : y;
}
template <int K, int C>
__device__ __forceinline__ void ldlt6_swap(double (&m)[36], bool sw) {  // transpositions k <-> c (c > k)
#pragma unroll
  for (int j = 0; j < K; j++) cswap(sw, m[6 * K + j], m[6 * C + j]);
#pragma unroll
  for (int i = C + 1; i < 6; i++) cswap(sw, m[6 * i + K], m[6 * i + C]);
  cswap(sw, m[7 * K], m[7 * C]);
#pragma unroll
  for (int i = K + 1; i < C; i++) cswap(sw, m[6 * i + K], m[6 * C + i]);
}
template <int K, int C>
__device__ __forceinline__ void ldlt6_swap_to(double (&m)[36], int big) {
  if constexpr (C < 6) {
    ldlt6_swap<K, C>(m, big == C);
    ldlt6_swap_to<K, C + 1>(m, big);
  }
}
template <int K>
__device__ __forceinline__ void ldlt6_step(double (&m)[36], int (&tr)[6], int& sign, bool& zero) {
  if constexpr (K < 6) {
    if (!zero) {
      int big = K;
      double bv = __builtin_fabs(m[7 * K]);
#pragma unroll
      for (int i = K + 1; i < 6; i++)
        if (__builtin_fabs(m[7 * i]) > bv) {
          bv = __builtin_fabs(m[7 * i]);
          big = i;
        }
      if (K == 0 && !(bv > 0.0)) {
#pragma unroll
        for (int j = 0; j < 6; j++) tr[j] = j;
#pragma unroll
        for (int j = 0; j < 6; j++) m[7 * j] = 0.0;
        sign = 0;
        zero = true;
      } else {
        tr[K] = big;
        ldlt6_swap_to<K, K + 1>(m, big);
        if constexpr (K > 0) {
          double temp[6];
#pragma unroll
          for (int j = 0; j < K; j++) temp[j] = m[7 * j] * m[6 * K + j];
          double dot = m[6 * K] * temp[0];
#pragma unroll
          for (int j = 1; j < K; j++) dot = dot + m[6 * K + j] * temp[j];
          m[7 * K] -= dot;
#pragma unroll
          for (int i = K + 1; i < 6; i++) {
            double sv = m[6 * i] * temp[0];
#pragma unroll
            for (int j = 1; j < K; j++) sv = sv + m[6 * i + j] * temp[j];
            m[6 * i + K] -= sv;
          }
        }
        const double akk = m[7 * K];
        if (__builtin_fabs(akk) > 0.0) {
#pragma unroll
          for (int i = K + 1; i < 6; i++) m[6 * i + K] /= akk;
        }
        if (akk > 0) sign = (sign == 2 || sign == 3) ? 3 : 1;
        else if (akk < 0) sign = (sign == 1 || sign == 3) ? 3 : 2;
      }
    }
    ldlt6_step<K + 1>(m, tr, sign, zero);
  }
}
// y[k] <-> y[t] for the unrolled k, t >= k (the transposition's other row)
template <int K>
__device__ __forceinline__ void perm_swap(double (&y)[6], int t) {
#pragma unroll
  for (int c = K + 1; c < 6; c++) cswap(t == c, y[K], y[c]);
}
__device__ __forceinline__ bool ldlt6(const double* Hin, const double* b, double* x) {
  double m[36];
#pragma unroll
  for (int i = 0; i < 36; i++) m[i] = Hin[i];
  int tr[6] = {0, 1, 2, 3, 4, 5};
  int sign = 0;
  bool zero = false;
  ldlt6_step<0>(m, tr, sign, zero);
  if (!(sign == 1 || sign == 0)) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; i++) y[i] = b[i];
  perm_swap<0>(y, tr[0]);
  perm_swap<1>(y, tr[1]);
  perm_swap<2>(y, tr[2]);
  perm_swap<3>(y, tr[3]);
  perm_swap<4>(y, tr[4]);
  perm_swap<5>(y, tr[5]);
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < i; j++) y[i] -= m[6 * i + j] * y[j];
  const double tol = 2.2250738585072014e-308;  // numeric_limits<double>::min()
#pragma unroll
  for (int i = 0; i < 6; i++) y[i] = __builtin_fabs(m[7 * i]) > tol ? y[i] / m[7 * i] : 0.0;
#pragma unroll
  for (int i = 5; i >= 0; i--)
#pragma unroll
    for (int j = i + 1; j < 6; j++) y[i] -= m[6 * j + i] * y[j];
  perm_swap<5>(y, tr[5]);
  perm_swap<4>(y, tr[4]);
  perm_swap<3>(y, tr[3]);
  perm_swap<2>(y, tr[2]);
  perm_swap<1>(y, tr[1]);
  perm_swap<0>(y, tr[0]);
#pragma unroll
  for (int i = 0; i < 6; i++) x[i] = y[i];
  return true;
}

struct PoseDev {
  orbx_pose_problem p;
  double* scratch;  // n x kRow doubles
  int* act;         // n: active edge ids in insertion order
};

struct Edge {
  bool stereo;
  double obs[3], X[3], info;
};

__device__ __forceinline__ Edge load_edge(const orbx_pose_problem& P, int i) {
  Edge e;
  e.stereo = P.obs[3 * i + 2] >= 0;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    e.obs[k] = P.obs[3 * i + k];
    e.X[k] = P.Xw[3 * i + k];
  }
  e.info = P.inv_sigma2[i];
  return e;
}

__device__ __forceinline__ void edge_error(const SE3& T, const orbx_pose_problem& P, const Edge& e, double err[3]) {
  double Pc[3];
  qrot(T.q, e.X, Pc);
#pragma unroll
  for (int i = 0; i < 3; i++) Pc[i] += T.t[i];
  const double fx = P.fx, fy = P.fy, cx = P.cx, cy = P.cy;
  if (!e.stereo) {
    const double u = Pc[0] / Pc[2] * fx + cx, v = Pc[1] / Pc[2] * fy + cy;
    err[0] = e.obs[0] - u;
    err[1] = e.obs[1] - v;
    err[2] = 0;
  } else {
    const float invz = (float)(1.0 / Pc[2]);
    const double u = Pc[0] * invz * fx + cx, v = Pc[1] * invz * fy + cy;
    const double ur = u - (double)P.bf * invz;
    err[0] = e.obs[0] - u;
    err[1] = e.obs[1] - v;
    err[2] = e.obs[2] - ur;
  }
}

__device__ __forceinline__ double chi2_of(const Edge& e, const double err[3]) {
  double s = err[0] * (e.info * err[0]);
  s += err[1] * (e.info * err[1]);
  if (e.stereo) s += err[2] * (e.info * err[2]);
  return s;
}

__device__ __forceinline__ void huber(bool stereo, double chi, double rho[3]) {
  const float dm = __builtin_sqrtf(5.991f), ds = __builtin_sqrtf(7.815f);
  const double delta = stereo ? ds : dm;
  const float dsqr = (float)(delta * delta);
  if (chi <= dsqr) {
    rho[0] = chi;
    rho[1] = 1.;
    rho[2] = 0.;
  } else {
    const double sq = __builtin_sqrt(chi);
    rho[0] = 2 * sq * delta - dsqr;
    rho[1] = delta / sq;
    rho[2] = -0.5 * rho[1] / chi;
  }
}

__device__ __forceinline__ void jacobian(const SE3& T, const orbx_pose_problem& P, const Edge& e, double J[18]) {
  double Pc[3];
  qrot(T.q, e.X, Pc);
#pragma unroll
  for (int i = 0; i < 3; i++) Pc[i] += T.t[i];
  const double fx = P.fx, fy = P.fy, bf = P.bf;
  const double x = Pc[0], y = Pc[1], iz = 1.0 / Pc[2], iz2 = iz * iz;
  J[0] = x * y * iz2 * fx;
  J[1] = -(1 + (x * x * iz2)) * fx;
  J[2] = y * iz * fx;
  J[3] = -iz * fx;
  J[4] = 0;
  J[5] = x * iz2 * fx;
  J[6] = (1 + y * y * iz2) * fy;
  J[7] = -x * y * iz2 * fy;
  J[8] = -x * iz * fy;
  J[9] = 0;
  J[10] = -iz * fy;
  J[11] = y * iz2 * fy;
  J[12] = J[0] - bf * y * iz2;
  J[13] = J[1] + bf * x * iz2;
  J[14] = J[2];
  J[15] = J[3];
  J[16] = 0;
  J[17] = J[5] - bf * iz2;
}

// LDS staging of the per-edge terms for the insertion-order sums: a chunk of kCh edges' 21 H
// (upper) + 6 b terms + the chi term at an odd row stride (kTs: lanes of the summing wave read
// consecutive doubles; the writers' 29-double stride spreads over the banks), summed chunk by
// chunk by one lane per entry.  The sums used to read the rows back from global scratch, 8 loads
// in flight per lane: ~700 cycles per 8 links of the chain.
constexpr int kCh = PBS;
constexpr int kTerm = 28, kTs = 29;
constexpr int kChiCh = kCh * kTs;  // chi terms per trial pass (one double each)

// sequential sum of m LDS values at stride st (insertion order kept), software-pipelined: the next
// 8 values load while the current 8 are added, so the chain runs at the add latency
__device__ __forceinline__ double lds_chain(const double* base, int m, int st, double s, bool sub) {
  const int m8 = m & ~7;
  double v[8];
  if (m8 > 0) {
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = base[u * st];
  }
  for (int k = 0; k < m8; k += 8) {
    double w[8];
    const int kn = k + 8 < m8 ? k + 8 : k;  // last batch: a harmless reload
#pragma unroll
    for (int u = 0; u < 8; u++) w[u] = base[(kn + u) * st];
#pragma unroll
    for (int u = 0; u < 8; u++) s = sub ? s - v[u] : s + v[u];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = w[u];
  }
  for (int k = m8; k < m; k++) s = sub ? s - base[k * st] : s + base[k * st];
  return s;
}

struct Shared {
  SE3 T, T0, bak;
  double H[36], b[6], x[6];
  double lambda, ni, currentChi, iniChi, tempChi, rho;
  int nact, qmax, ok2, nbad_lm, go, term, robust, nbad_cls;
  int scan[PBS / 64];
};

// Phase probe (build with -DORBX_POSE_PROBE only): s_memtime ticks per phase of each block, taken
// by thread 0 after the phase's closing barrier, into a host-provided buffer of 16 words per block.
#ifdef ORBX_POSE_PROBE
__device__ unsigned long long* pose_probe_buf;
#define POSE_TS(k)                                                    \
  do {                                                                \
    if (tid == 0) {                                                   \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
      pacc[k] += t_ - plast;                                          \
      plast = t_;                                                     \
    }                                                                 \
  } while (0)
#else
#define POSE_TS(k)
#endif

__global__ __launch_bounds__(PBS) void k_pose_optimization(const PoseDev* __restrict__ probs) {
  __shared__ Shared S;
  __shared__ double sterm[kCh * kTs];
#ifdef ORBX_POSE_PROBE
  unsigned long long pacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, plast = __builtin_amdgcn_s_memtime();
#endif
  const PoseDev& D = probs[blockIdx.x];
  const orbx_pose_problem& P = D.p;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = P.n_dev ? min(max(*P.n_dev, 0), P.n) : P.n;  // device-sized: P.n is the capacity
  double* scr = D.scratch;
  int* act = D.act;
  const float* Tin = P.Tcw_dev ? P.Tcw_dev : P.Tcw;

  for (int i = tid; i < n; i += PBS) P.outlier[i] = 0;
  if (tid < 16) P.Tcw_out[tid] = Tin[tid];
  if (P.iterations && tid < 4) P.iterations[tid] = 0;
  if (n < 3) {  // nInitialCorrespondences < 3: return 0, pose untouched
    if (tid == 0) *P.ngood = 0;
    return;
  }
  if (tid == 0) {  // Converter::toSE3Quat(pFrame->mTcw)
    const float* T = Tin;
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    S.T0.q = mat2q(R);
    qnormalize(S.T0.q);
    S.T0.t[0] = T[3];
    S.T0.t[1] = T[7];
    S.T0.t[2] = T[11];
    S.robust = 1;
  }
  __syncthreads();
  int nBad = 0;
  for (int it = 0; it < 4; it++) {
    // ---- initializeOptimization(0): active = level-0 edges, insertion order ----
    if (tid == 0) S.T = S.T0;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += PBS) {
      const int i = c0 + tid;
      const int a = (i < n && !P.outlier[i]) ? 1 : 0;
      const uint64_t m = __ballot(a);
      const int pre = __popcll(m & ((1ull << lane) - 1));
      if (lane == 0) S.scan[wid] = __popcll(m);
      __syncthreads();
      int off = base;
      for (int w = 0; w < wid; w++) off += S.scan[w];
      if (a) act[off + pre] = i;
      int tot = 0;
      for (int w = 0; w < PBS / 64; w++) tot += S.scan[w];
      base += tot;
      __syncthreads();
    }
    const int nact = base;
    __threadfence_block();
    __syncthreads();
    POSE_TS(0);
    int its = 0;
    if (nact > 0) {
      for (int iter = 0; iter < 10; iter++) {
        its++;
        // computeActiveErrors + activeRobustChi2 (currentChi) and buildSystem's terms, a chunk of
        // kCh active edges at a time into LDS, each summed in insertion order by its own lane
        const bool robust = S.robust;
        const SE3 T = S.T;
        double acc = 0.0;  // wave 0, lanes 0..27: H upper (0..20), b (21..26, -= terms), chi (27)
        for (int c0 = 0; c0 < nact; c0 += kCh) {
          const int k = c0 + tid;
          if (k < nact) {
            const int i = act[k];
            const Edge e = load_edge(P, i);
            double err[3];
            edge_error(T, P, e, err);
            double* row = scr + (size_t)k * kRow;  // errors kept for the outlier pass
            row[27] = err[0];
            row[28] = err[1];
            row[29] = err[2];
            double* tr = sterm + tid * kTs;
            const double c = chi2_of(e, err);
            double rho[3];
            if (robust) huber(e.stereo, c, rho);
            tr[27] = robust ? rho[0] : c;
            // buildSystem terms (linearizeOplus + constructQuadraticForm)
            double J[18];
            jacobian(T, P, e, J);
            const int Dm = e.stereo ? 3 : 2;
            double w = e.info, r1 = 1.0;
            if (robust) {
              r1 = rho[1];
              w = rho[1] * e.info;
            }
            int q = 0;
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
              for (int cc = r; cc < 6; cc++) {
                double sv = (J[r] * w) * J[cc];
                sv = sv + (J[6 + r] * w) * J[6 + cc];
                if (Dm == 3) sv = sv + (J[12 + r] * w) * J[12 + cc];
                tr[q++] = sv;
              }
#pragma unroll
            for (int r = 0; r < 6; r++) {
              double sv = ((r1 * J[r]) * e.info) * err[0];
              sv = sv + ((r1 * J[6 + r]) * e.info) * err[1];
              if (Dm == 3) sv = sv + ((r1 * J[12 + r]) * e.info) * err[2];
              tr[21 + r] = sv;
            }
          }
          __syncthreads();
          POSE_TS(1);
          if (wid == 0 && lane < kTerm)
            acc = lds_chain(sterm + lane, min(kCh, nact - c0), kTs, acc, lane >= 21 && lane < 27);
          __syncthreads();
          POSE_TS(2);
        }
        if (wid == 0 && lane < kTerm) {
          if (lane < 21) {
            int r = 0, c = lane;
            while (c >= 6 - r) {
              c -= 6 - r;
              r++;
            }
            c += r;
            S.H[6 * r + c] = acc;
            S.H[6 * c + r] = acc;
          } else if (lane < 27) {
            S.b[lane - 21] = acc;
          } else {
            S.currentChi = acc;
            S.iniChi = acc;
          }
        }
        __syncthreads();
        POSE_TS(2);
        if (tid == 0) {
          if (iter == 0) {
            double m = 0;
            for (int j = 0; j < 6; j++) {
              const double a = __builtin_fabs(S.H[7 * j]);
              m = (a < m) ? m : a;  // std::max(|H_jj|, m)
            }
            S.lambda = 1e-5 * m;
            S.ni = 2;
            S.nbad_lm = 0;
          }
          S.qmax = 0;
        }
        __syncthreads();
        POSE_TS(3);
        // ---- trials ----
        for (;;) {
          if (tid == 0) {
            S.bak = S.T;
            double Hd[36];  // registers: every index static
#pragma unroll
            for (int j = 0; j < 36; j++) Hd[j] = S.H[j];
#pragma unroll
            for (int j = 0; j < 6; j++) Hd[7 * j] += S.lambda;
            const bool ok2 = ldlt6(Hd, S.b, S.x);
            S.ok2 = ok2;
            POSE_TS(9);
            if (ok2) S.T = se3_mul(se3_exp(S.x), S.T);
          }
          __syncthreads();
          POSE_TS(4);
          double tempChi = 0.0;  // thread 0: activeRobustChi2 at the trial pose, insertion order
          {
            const SE3 Tt = S.T;
            const bool rb = S.robust;
            for (int c0 = 0; c0 < nact; c0 += kChiCh) {
              for (int k = c0 + tid; k < min(nact, c0 + kChiCh); k += PBS) {
                const int i = act[k];
                const Edge e = load_edge(P, i);
                double err[3];
                edge_error(Tt, P, e, err);
                double* row = scr + (size_t)k * kRow;
                row[27] = err[0];
                row[28] = err[1];
                row[29] = err[2];
                const double c = chi2_of(e, err);
                double rho[3];
                if (rb) huber(e.stereo, c, rho);
                sterm[k - c0] = rb ? rho[0] : c;
              }
              __syncthreads();
              POSE_TS(5);
              if (tid == 0) tempChi = lds_chain(sterm, min(kChiCh, nact - c0), 1, tempChi, false);
              __syncthreads();
              POSE_TS(6);
            }
          }
          if (tid == 0) {
            const bool ok2 = S.ok2;
            if (!ok2) tempChi = 1.7976931348623157e308;
            double rho = S.currentChi - tempChi;
            double scale = 0.0;
            if (ok2)
              for (int j = 0; j < 6; j++) scale += S.x[j] * (S.lambda * S.x[j] + S.b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && __builtin_isfinite(tempChi)) {
              const double t3 = 2 * rho - 1;
              double alpha = 1. - t3 * t3 * t3;
              alpha = (2. / 3. < alpha) ? 2. / 3. : alpha;       // std::min(alpha, 2/3)
              S.lambda *= (1. / 3. < alpha) ? alpha : 1. / 3.;    // std::max(1/3, alpha)
              S.ni = 2;
              S.currentChi = tempChi;
            } else {
              S.lambda *= S.ni;
              S.ni *= 2;
              S.T = S.bak;
            }
            S.qmax++;
            S.rho = rho;
            S.go = (rho < 0 && S.qmax < 10);
          }
          __syncthreads();
          POSE_TS(7);
          if (!S.go) break;
        }
        if (tid == 0) {
          int term = 0;
          if (S.qmax == 10 || S.rho == 0) term = 1;
          else {
            if ((S.iniChi - S.currentChi) * 1e3 < S.iniChi) S.nbad_lm++;
            else S.nbad_lm = 0;
            if (S.nbad_lm >= 3) term = 1;
          }
          S.term = term;
        }
        __syncthreads();
        POSE_TS(7);
        if (S.term) break;
      }
    }
    if (P.iterations && tid == 0) P.iterations[it] = its;
    // ---- outlier classification, src/Optimizer.cc:433-497 ----
    // stored errors of active edges sit in the scratch rows of their active position
    if (tid == 0) S.nbad_cls = 0;
    __syncthreads();
    {
      const SE3 T = S.T;
      // map edge -> active position: act[] is ascending, binary search
      int cnt = 0;
      for (int i = tid; i < n; i += PBS) {
        const Edge e = load_edge(P, i);
        double err[3];
        if (P.outlier[i]) {
          edge_error(T, P, e, err);  // e->computeError()
        } else {
          int lo = 0, hi = nact;
          while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (act[m] < i) lo = m + 1; else hi = m;
          }
          const double* row = scr + (size_t)lo * kRow;
          err[0] = row[27];
          err[1] = row[28];
          err[2] = row[29];
        }
        const float chi2 = (float)chi2_of(e, err);
        const bool bad = chi2 > (e.stereo ? 7.815f : 5.991f);
        cnt += bad;
        // written after every thread has read the old flags (barrier below)
        scr[(size_t)i * kRow + 31] = bad ? 1.0 : 0.0;
      }
      atomicAdd(&S.nbad_cls, cnt);
    }
    __threadfence_block();
    __syncthreads();
    POSE_TS(8);
    for (int i = tid; i < n; i += PBS) P.outlier[i] = scr[(size_t)i * kRow + 31] != 0.0 ? 1 : 0;
    nBad = S.nbad_cls;
    if (it == 2 && tid == 0) S.robust = 0;
    __threadfence_block();
    __syncthreads();
    POSE_TS(8);
    if (n < 10) break;
  }
#ifdef ORBX_POSE_PROBE
  if (tid == 0 && pose_probe_buf)
    for (int k = 0; k < 10; k++) pose_probe_buf[(size_t)blockIdx.x * 16 + k] = pacc[k];
#endif
  if (tid == 0) {
    double R[9];
    qmat(S.T.q, R);
    for (int r = 0; r < 3; r++) {
      for (int k = 0; k < 3; k++) P.Tcw_out[4 * r + k] = (float)R[3 * r + k];
      P.Tcw_out[4 * r + 3] = (float)S.T.t[r];
    }
    P.Tcw_out[12] = P.Tcw_out[13] = P.Tcw_out[14] = 0.0f;
    P.Tcw_out[15] = 1.0f;
    *P.ngood = n - nBad;
  }
}

}  // namespace pose
}  // namespace orbx

#ifdef ORBX_POSE_PROBE
extern "C" int orbx_debug_pose_probe(void* d_buf) {  // device buffer of 16 u64 per block, or NULL
  unsigned long long* p = (unsigned long long*)d_buf;
  return hipMemcpyToSymbol(HIP_SYMBOL(orbx::pose::pose_probe_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif

// ------------------------------------------------------------------ C ABI
namespace {

orbx_status pose_check(const orbx_pose_problem& p) {
  if (p.n < 0) return ORBX_ERR_ARG;
  if (!p.Tcw_out || !p.ngood) return ORBX_ERR_ARG;
  if (p.n > 0 && (!p.obs || !p.Xw || !p.inv_sigma2 || !p.outlier)) return ORBX_ERR_ARG;
  return ORBX_OK;
}

}  // namespace

extern "C" orbx_status orbx_pose_optimization(const orbx_pose_problem* p, int device) {
  if (!p) return ORBX_ERR_ARG;
  const orbx_status chk = pose_check(*p);
  if (chk != ORBX_OK) return chk;
  if (p->n_dev || p->Tcw_dev) return ORBX_ERR_ARG;  // device batches only
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= ndev || hipSetDevice(device) != hipSuccess) return ORBX_ERR_ARG;
  const size_t n = (size_t)p->n;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_obs = 0, o_X = o_obs + al(n * 12), o_s2 = o_X + al(n * 12), o_Tout = o_s2 + al(n * 4),
               o_out = o_Tout + al(64), o_ng = o_out + al(n), o_it = o_ng + al(4),
               o_scr = o_it + al(16), o_act = o_scr + al(n * orbx::pose::kRow * 8), o_dev = o_act + al(n * 4),
               total = o_dev + al(sizeof(orbx::pose::PoseDev));
  orbx::ScratchGuard g(device);  // pooled lease: no per-call allocation (orbx_scratch.h)
  if (!g.l || g.l->reserve(total, o_scr + sizeof(orbx::pose::PoseDev)) != hipSuccess) return ORBX_ERR_HIP;
  uint8_t* host = g.l->h;
  std::memset(host, 0, o_scr);  // outputs start zeroed, as before
  if (n) {
    std::memcpy(host + o_obs, p->obs, n * 12);
    std::memcpy(host + o_X, p->Xw, n * 12);
    std::memcpy(host + o_s2, p->inv_sigma2, n * 4);
  }
  uint8_t* d = g.l->d;
  orbx::pose::PoseDev pd;
  pd.p = *p;
  pd.p.obs = (const float*)(d + o_obs);
  pd.p.Xw = (const float*)(d + o_X);
  pd.p.inv_sigma2 = (const float*)(d + o_s2);
  pd.p.Tcw_out = (float*)(d + o_Tout);
  pd.p.outlier = (uint8_t*)(d + o_out);
  pd.p.ngood = (int32_t*)(d + o_ng);
  pd.p.iterations = (int32_t*)(d + o_it);
  pd.scratch = (double*)(d + o_scr);
  pd.act = (int*)(d + o_act);
  std::memcpy(host + o_scr, &pd, sizeof(pd));  // the record rides in the staging block's tail
  hipStream_t st = g.l->st;
  hipError_t e = hipMemcpyAsync(d, host, o_scr, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + o_dev, host + o_scr, sizeof(pd), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::pose::k_pose_optimization, dim3(1), dim3(orbx::pose::PBS), 0, st,
                       (const orbx::pose::PoseDev*)(d + o_dev));
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(host + o_Tout, d + o_Tout, o_scr - o_Tout, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = g.l->sync();
  if (e != hipSuccess) return ORBX_ERR_HIP;
  std::memcpy(p->Tcw_out, host + o_Tout, 64);
  if (n) std::memcpy(p->outlier, host + o_out, n);
  std::memcpy(p->ngood, host + o_ng, 4);
  if (p->iterations) std::memcpy(p->iterations, host + o_it, 16);
  return ORBX_OK;
}

extern "C" orbx_status orbx_pose_optimization_device(const orbx_pose_problem* problems, int n, void* stream) {
  if (n < 0 || (n > 0 && !problems)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  size_t rows = 0;
  for (int i = 0; i < n; i++) {
    const orbx_status s = pose_check(problems[i]);
    if (s != ORBX_OK) return s;
    rows += (size_t)problems[i].n;
  }
  hipStream_t st = (hipStream_t)stream;
  const size_t dev_bytes = sizeof(orbx::pose::PoseDev) * n;
  const size_t scr_off = (dev_bytes + 255) & ~(size_t)255;
  const size_t act_off = scr_off + rows * orbx::pose::kRow * 8;
  uint8_t* d = nullptr;
  if (hipMallocAsync((void**)&d, act_off + rows * 4 + 16, st) != hipSuccess) return ORBX_ERR_HIP;
  std::vector<orbx::pose::PoseDev> pd(n);
  size_t r = 0;
  for (int i = 0; i < n; i++) {
    pd[i].p = problems[i];
    pd[i].scratch = (double*)(d + scr_off) + r * orbx::pose::kRow;
    pd[i].act = (int*)(d + act_off) + r;
    r += (size_t)problems[i].n;
  }
  hipError_t e = hipMemcpyAsync(d, pd.data(), dev_bytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(orbx::pose::k_pose_optimization, dim3(n), dim3(orbx::pose::PBS), 0, st,
                       (const orbx::pose::PoseDev*)d);
    e = hipGetLastError();
  }
  // pageable source: hipMemcpyAsync returns once pd is staged, so pd may go
  const hipError_t e2 = hipFreeAsync(d, st);
  return e != hipSuccess ? ORBX_ERR_HIP : (e2 != hipSuccess ? ORBX_ERR_HIP : ORBX_OK);
}
