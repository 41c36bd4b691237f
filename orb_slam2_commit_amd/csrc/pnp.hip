// pnp.hip -- PnPsolver (src/PnPsolver.cc:67-1101) on the GPU: RANSAC
// hypotheses evaluated in parallel, resolved in the reference's order.
//
//   k_pnp_hyp     one 256-thread block per hypothesis: EPnP compute_pose on
//                 its minimal set (DUtils::Random::RandomInt + swap-remove
//                 sampling replayed on the host from the caller's rand()
//                 values), everything in LDS
//   k_pnp_check   one block per hypothesis: CheckInliers (float/double mix
//                 exactly as :352-384) -> inlier bytes + count
//   k_pnp_refine  one block: Refine() (:303-349) = EPnP on every inlier of
//                 the best hypothesis (staged in LDS) + CheckInliers
// The host walks hypotheses in order (best = first strict maximum, Refine at
// each hypothesis reaching minInliers, return on the first successful
// Refine), which is iterate() (:182-301) including its
// `mnIterations<maxIts || nCurrent<nIterations` loop condition.
//
// EPnP and the OpenCV 3.2 helpers it calls (cvMulTransposed, Jacobi cvSVD,
// cvInvert/cvSolve through SVBkSb) use only IEEE + - * / sqrt in the same
// order as the oracle, with every reduction sequential in the reference's
// order, so poses and masks are bit-identical to the CPU restatement.  The
// parallelism is only where it cannot change a bit: per-point terms, the
// 12x12 Jacobi's independent rotations (wavefront schedule), the three
// independent beta approximations (one wave each), and loads/terms of the
// sequential sums computed ahead of the additions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/orbx.h"

namespace orbx {

constexpr int kPnpMaxSet = 16;


struct PnpIn {
  const float* p3d;
  const float* p2d;
  const float* max_error;
  int N;
  double fu, fv, uc, vc;
};

// ------------------------------------------------------------ OpenCV 3.2 math
struct CvRng {
  unsigned long long state;
  __device__ unsigned next() {
    state = (unsigned long long)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
    return (unsigned)state;
  }
};

__device__ inline void swap_d(double& a, double& b) {
  const double t = a;
  a = b;
  b = t;
}

// JacobiSVDImpl_<double> (see oracle/pnp.cpp) on N rows of length M in At
// (row stride M), n1 = N.  Sizes are compile-time so the small systems live
// in registers; kV = false skips the V rotations -- they never feed back into
// At or W, so U and W are unchanged (EPnP's 12x12 SVD only reads Ut).
// One Jacobi rotation of rows i < j (At row stride M, W the squared row
// norms); returns false when the pair is already orthogonal (skipped).
template <int M, int N, bool kV>
__device__ __forceinline__ bool jacobi_rotate(double* At, double* W, double* Vt, int i, int j) {
  const double eps = DBL_EPSILON * 10;
  double* Ai = At + i * M;
  double* Aj = At + j * M;
  double a = W[i], p = 0, b = W[j];
  double xi[M], xj[M];
#pragma unroll
  for (int k = 0; k < M; k++) {
    xi[k] = Ai[k];
    xj[k] = Aj[k];
  }
#pragma unroll
  for (int k = 0; k < M; k++) p += xi[k] * xj[k];
  if (fabs(p) <= eps * sqrt(a * b)) return false;
  p *= 2;
  const double beta = a - b, gamma = sqrt(p * p + beta * beta);
  double c, s;
  if (beta < 0) {
    const double delta = (gamma - beta) * 0.5;
    s = sqrt(delta / gamma);
    c = p / (gamma * s * 2);
  } else {
    c = sqrt((gamma + beta) / (gamma * 2));
    s = p / (gamma * c * 2);
  }
  a = b = 0;
#pragma unroll
  for (int k = 0; k < M; k++) {
    const double t0 = c * xi[k] + s * xj[k];
    const double t1 = -s * xi[k] + c * xj[k];
    Ai[k] = t0;
    Aj[k] = t1;
    a += t0 * t0;
    b += t1 * t1;
  }
  W[i] = a;
  W[j] = b;
  if (kV) {
    double* Vi = Vt + i * N;
    double* Vj = Vt + j * N;
#pragma unroll
    for (int k = 0; k < N; k++) {
      const double t0 = c * Vi[k] + s * Vj[k];
      const double t1 = -s * Vi[k] + c * Vj[k];
      Vi[k] = t0;
      Vj[k] = t1;
    }
  }
  return true;
}

// After the sweeps: singular values, descending sort (rows of At and Vt
// swapped along), and the cv::RNG(0x12345678) completion of null rows.
template <int M, int N, bool kV, bool kSmall>
__device__ __forceinline__ void jacobi_tail(double* At, double* W, double* Wout, double* Vt) {
  const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < M; k++) {
      const double t = At[i * M + k];
      sd += t * t;
    }
    W[i] = sqrt(sd);
  }
#pragma unroll
  for (int i = 0; i < N - 1; i++) {
    int j = i;
#pragma unroll
    for (int k = i + 1; k < N; k++)
      if (W[j] < W[k]) j = k;
    if (i != j) {
      if constexpr (kSmall) {  // W[j] with j runtime: select chains keep W in registers
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < N; k++)
          if (k == j) wj = W[k];
#pragma unroll
        for (int k = i + 1; k < N; k++)
          if (k == j) W[k] = W[i];
        W[i] = wj;
      } else {
        swap_d(W[i], W[j]);
      }
      if constexpr (kSmall) {  // rows of register arrays: swap with every candidate row under a
                               // select (static indices), never a runtime-indexed (scratch) access
#pragma unroll
        for (int r = i + 1; r < N; r++) {
          const bool sw = r == j;
#pragma unroll
          for (int k = 0; k < M; k++) {
            const double a = At[i * M + k], b = At[r * M + k];
            At[i * M + k] = sw ? b : a;
            At[r * M + k] = sw ? a : b;
          }
          if (kV) {
#pragma unroll
            for (int k = 0; k < N; k++) {
              const double a = Vt[i * N + k], b = Vt[r * N + k];
              Vt[i * N + k] = sw ? b : a;
              Vt[r * N + k] = sw ? a : b;
            }
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < M; k++) swap_d(At[i * M + k], At[j * M + k]);
        if (kV) {
#pragma unroll
          for (int k = 0; k < N; k++) swap_d(Vt[i * N + k], Vt[j * N + k]);
        }
      }
    }
  }
  if (kSmall) {
#pragma unroll
    for (int i = 0; i < N; i++) Wout[i] = W[i];
  }
  CvRng rng{0x12345678};
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = W[i];
    for (int ii = 0; ii < 100 && sd <= minval; ii++) {
      const double val0 = 1. / M;
#pragma unroll
      for (int k = 0; k < M; k++) At[i * M + k] = (rng.next() & 256) != 0 ? val0 : -val0;
      for (int iter = 0; iter < 2; iter++)
        for (int j = 0; j < i; j++) {
          sd = 0;
#pragma unroll
          for (int k = 0; k < M; k++) sd += At[i * M + k] * At[j * M + k];
          double asum = 0;
#pragma unroll
          for (int k = 0; k < M; k++) {
            const double t = At[i * M + k] - sd * At[j * M + k];
            At[i * M + k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
          for (int k = 0; k < M; k++) At[i * M + k] *= asum;
        }
      sd = 0;
#pragma unroll
      for (int k = 0; k < M; k++) {
        const double t = At[i * M + k];
        sd += t * t;
      }
      sd = sqrt(sd);
    }
    const double s = sd > minval ? 1 / sd : 0.;
#pragma unroll
    for (int k = 0; k < M; k++) At[i * M + k] *= s;
  }
}

// JacobiSVDImpl_<double> (see oracle/pnp.cpp) on N rows of length M in At
// (row stride M), n1 = N, one thread.  Sizes are compile-time so the small
// systems live in registers; kV = false skips the V rotations -- they never
// feed back into At or W, so U and W are unchanged.
template <int M, int N, bool kV>
__device__ __forceinline__ void jacobi_svd(double* At, double* Wout, double* Vt) {
  constexpr bool kSmall = N <= 6;  // else W works in Wout and the pair loops stay rolled
  double Wreg[kSmall ? N : 1];
  double* W = kSmall ? Wreg : Wout;
  constexpr int max_iter = M > 30 ? M : 30;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < M; k++) {
      const double t = At[i * M + k];
      sd += t * t;
    }
    W[i] = sd;
    if (kV) {
#pragma unroll
      for (int k = 0; k < N; k++) Vt[i * N + k] = 0;
      Vt[i * N + i] = 1;
    }
  }
  for (int iter = 0; iter < max_iter; iter++) {
    bool changed = false;
    if constexpr (kSmall) {
#pragma unroll
      for (int i = 0; i < N - 1; i++)
#pragma unroll
        for (int j = i + 1; j < N; j++) changed |= jacobi_rotate<M, N, kV>(At, W, Vt, i, j);
    } else {
#pragma unroll 1
      for (int i = 0; i < N - 1; i++)
#pragma unroll 1
        for (int j = i + 1; j < N; j++) changed |= jacobi_rotate<M, N, kV>(At, W, Vt, i, j);
    }
    if (!changed) break;
  }
  jacobi_tail<M, N, kV, kSmall>(At, W, Wout, Vt);
}

// The same SVD (no V) run by one wave on LDS data: rotation (i, j) only
// touches rows i, j, and in the cyclic order each row's rotations come in
// increasing i + j, so step t = i + j runs every pair (lane i, t - i) at once
// -- disjoint rows, each row's rotations in the reference order, so the
// result is bit-identical -- 2N-3 steps per sweep instead of N(N-1)/2.  The
// sort and null-row completion stay on lane 0.
template <int M, int N>
__device__ __forceinline__ void jacobi_svd_wave(double* At, double* W) {
  constexpr int max_iter = M > 30 ? M : 30;
  const int lane = threadIdx.x & 63;
  if (lane < N) {
    double sd = 0;
#pragma unroll
    for (int k = 0; k < M; k++) {
      const double t = At[lane * M + k];
      sd += t * t;
    }
    W[lane] = sd;
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): LDS writes visible wave-wide
  __builtin_amdgcn_wave_barrier();
  for (int iter = 0; iter < max_iter; iter++) {
    bool changed = false;
    for (int t = 1; t <= 2 * N - 3; t++) {
      const int j = t - lane;
      if (lane < j && j < N) changed |= jacobi_rotate<M, N, false>(At, W, nullptr, lane, j);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
    }
    if (__ballot(changed) == 0) break;
  }
  if (lane == 0) jacobi_tail<M, N, false, false>(At, W, W, nullptr);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_wave_barrier();
}

// _SVDcompute, m >= n: left singular vectors as rows Ut (n x m), w, Vt.
template <int M, int N, bool kV = true>
__device__ __forceinline__ void svd_rows(const double* A, double* Ut, double* w, double* Vt) {
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int k = 0; k < M; k++) Ut[i * M + k] = A[k * N + i];
  jacobi_svd<M, N, kV>(Ut, w, Vt);
}

// SVBkSbImpl_ (kInv: b = identity, i.e. the inverse)
template <int M, int N, bool kInv>
__device__ __forceinline__ void svd_backsubst(const double* Ut, const double* w, const double* Vt, const double* b, double* x) {
  constexpr int nb = kInv ? M : 1;
#pragma unroll
  for (int i = 0; i < N * nb; i++) x[i] = 0;
  double threshold = 0;
#pragma unroll
  for (int i = 0; i < N; i++) threshold += w[i];
  threshold *= DBL_EPSILON * 2;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double wi = w[i];
    if (fabs(wi) <= threshold) continue;
    wi = 1 / wi;
    const double* u = Ut + i * M;
    const double* v = Vt + i * N;
    if (!kInv) {
      double s = 0;
#pragma unroll
      for (int j = 0; j < M; j++) s += u[j] * b[j];
      s *= wi;
#pragma unroll
      for (int j = 0; j < N; j++) x[j] = x[j] + s * v[j];
    } else {
      double buffer[nb];
#pragma unroll
      for (int j = 0; j < nb; j++) buffer[j] = u[j] * wi;
#pragma unroll
      for (int j = 0; j < N; j++)
#pragma unroll
        for (int k = 0; k < nb; k++) x[j * nb + k] += buffer[k] * v[j];
    }
  }
}

__device__ inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ inline double dist2(const double* p1, const double* p2) {
  return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

// find_betas_approx_{1,2,3}, compute_L_6x10, compute_rho, gauss_newton, qr_solve
template <int K>
__device__ __forceinline__ void solve6(const double* L, const double* rho, double* x) {
  double ut[6 * K], w[K], vt[K * K];
  svd_rows<6, K>(L, ut, w, vt);
  svd_backsubst<6, K, false>(ut, w, vt, rho, x);
}

__device__ __forceinline__ void find_betas_approx_1(const double* l_6x10, const double* rho, double* betas) {
  double l_6x4[24], b4[4];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    l_6x4[4 * i] = l_6x10[10 * i];
    l_6x4[4 * i + 1] = l_6x10[10 * i + 1];
    l_6x4[4 * i + 2] = l_6x10[10 * i + 3];
    l_6x4[4 * i + 3] = l_6x10[10 * i + 6];
  }
  solve6<4>(l_6x4, rho, b4);
  if (b4[0] < 0) {
    betas[0] = sqrt(-b4[0]);
    betas[1] = -b4[1] / betas[0];
    betas[2] = -b4[2] / betas[0];
    betas[3] = -b4[3] / betas[0];
  } else {
    betas[0] = sqrt(b4[0]);
    betas[1] = b4[1] / betas[0];
    betas[2] = b4[2] / betas[0];
    betas[3] = b4[3] / betas[0];
  }
}

__device__ __forceinline__ void find_betas_approx_2(const double* l_6x10, const double* rho, double* betas) {
  double l_6x3[18], b3[3];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) l_6x3[3 * i + j] = l_6x10[10 * i + j];
  solve6<3>(l_6x3, rho, b3);
  if (b3[0] < 0) {
    betas[0] = sqrt(-b3[0]);
    betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
  } else {
    betas[0] = sqrt(b3[0]);
    betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
  }
  if (b3[1] < 0) betas[0] = -betas[0];
  betas[2] = 0.0;
  betas[3] = 0.0;
}

__device__ __forceinline__ void find_betas_approx_3(const double* l_6x10, const double* rho, double* betas) {
  double l_6x5[30], b5[5];
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) l_6x5[5 * i + j] = l_6x10[10 * i + j];
  solve6<5>(l_6x5, rho, b5);
  if (b5[0] < 0) {
    betas[0] = sqrt(-b5[0]);
    betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
  } else {
    betas[0] = sqrt(b5[0]);
    betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
  }
  if (b5[1] < 0) betas[0] = -betas[0];
  betas[2] = b5[3] / betas[0];
  betas[3] = 0.0;
}

__device__ __forceinline__ void compute_L_6x10(const double* ut, double* l_6x10) {
  double dv[4][6][3];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const double* v = ut + 12 * (11 - i);
    int a = 0, b = 1;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      dv[i][j][0] = v[3 * a] - v[3 * b];
      dv[i][j][1] = v[3 * a + 1] - v[3 * b + 1];
      dv[i][j][2] = v[3 * a + 2] - v[3 * b + 2];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double* row = l_6x10 + 10 * i;
    row[0] = dot3(dv[0][i], dv[0][i]);
    row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
    row[2] = dot3(dv[1][i], dv[1][i]);
    row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
    row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
    row[5] = dot3(dv[2][i], dv[2][i]);
    row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
    row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
    row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
    row[9] = dot3(dv[3][i], dv[3][i]);
  }
}

// Householder QR solve of the 6x4 Gauss-Newton system (the reference's
// qr_solve, pointer walks replaced by indices; same operation order).
__device__ __forceinline__ void qr_solve(double* A, double* b, double* X) {
  constexpr int nr = 6, nc = 4;
  double A1[nc], A2[nc];
#pragma unroll
  for (int k = 0; k < nc; k++) {
    // the reference's scan reads rows k .. nr-2 (its pointer advances after
    // the read), so row nr-1 never enters eta -- kept as is
    double eta = fabs(A[k * nc + k]);
#pragma unroll
    for (int i = k + 1; i < nr; i++) {
      const double elt = fabs(A[(i - 1) * nc + k]);
      if (eta < elt) eta = elt;
    }
    if (eta == 0) return;
    double sum = 0.0;
    const double inv_eta = 1. / eta;
#pragma unroll
    for (int i = k; i < nr; i++) {
      A[i * nc + k] *= inv_eta;
      sum += A[i * nc + k] * A[i * nc + k];
    }
    double sigma = sqrt(sum);
    if (A[k * nc + k] < 0) sigma = -sigma;
    A[k * nc + k] += sigma;
    A1[k] = sigma * A[k * nc + k];
    A2[k] = -eta * sigma;
#pragma unroll
    for (int j = k + 1; j < nc; j++) {
      double s = 0;
#pragma unroll
      for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
      const double tau = s / A1[k];
#pragma unroll
      for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
    }
  }
#pragma unroll
  for (int j = 0; j < nc; j++) {
    double tau = 0;
#pragma unroll
    for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
    tau /= A1[j];
#pragma unroll
    for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
  }
  X[nc - 1] = b[nc - 1] / A2[nc - 1];
#pragma unroll
  for (int i = nc - 2; i >= 0; i--) {
    double s = 0;
#pragma unroll
    for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * X[j];
    X[i] = (b[i] - s) / A2[i];
  }
}

__device__ __forceinline__ void gauss_newton(const double* l_6x10, const double* rho, double betas[4]) {
  double a[24], b[6], x[4] = {0, 0, 0, 0};
  for (int k = 0; k < 5; k++) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const double* rowL = l_6x10 + i * 10;
      double* rowA = a + i * 4;
      rowA[0] = 2 * rowL[0] * betas[0] + rowL[1] * betas[1] + rowL[3] * betas[2] + rowL[6] * betas[3];
      rowA[1] = rowL[1] * betas[0] + 2 * rowL[2] * betas[1] + rowL[4] * betas[2] + rowL[7] * betas[3];
      rowA[2] = rowL[3] * betas[0] + rowL[4] * betas[1] + 2 * rowL[5] * betas[2] + rowL[8] * betas[3];
      rowA[3] = rowL[6] * betas[0] + rowL[7] * betas[1] + rowL[8] * betas[2] + 2 * rowL[9] * betas[3];
      b[i] = rho[i] - (rowL[0] * betas[0] * betas[0] + rowL[1] * betas[0] * betas[1] + rowL[2] * betas[1] * betas[1] +
                       rowL[3] * betas[0] * betas[2] + rowL[4] * betas[1] * betas[2] + rowL[5] * betas[2] * betas[2] +
                       rowL[6] * betas[0] * betas[3] + rowL[7] * betas[1] * betas[3] + rowL[8] * betas[2] * betas[3] +
                       rowL[9] * betas[3] * betas[3]);
    }
    qr_solve(a, b, x);
#pragma unroll
    for (int i = 0; i < 4; i++) betas[i] += x[i];
  }
}

// ------------------------------------------------------------ EPnP on a block
// One block computes one EPnP (a RANSAC hypothesis on its minimal set, or
// Refine on the inlier set): per-point work is spread over the threads, every
// reduction runs on thread 0 (or one thread per output) in point order, and
// the SVDs run on thread 0 -- the reference's sequential order, so results
// are bit-identical to the oracle.  The matrices live in LDS (EpnpSmall) and
// so do the points when they fit (EpnpPts); M is never materialised: MtM
// recomputes the entries of fill_M on the fly (same expressions).

struct EpnpSmall {
  double cws[4][3], ccs[4][3], ci[9], pw0tpw0[9], mtm[144], ut[144], d[12];
  double l_6x10[60], rho[6], betas[4][4], rep[4], Rs[4][3][3], ts[4][3];
  double pw0[3], ccs_ap[4][4][3], pc0_ap[4][3], abt_ap[4][9];
};

struct EpnpPts {   // per-correspondence arrays of one problem (n entries)
  const float* pw;  // 3n
  const float* uv;  // 2n
  double* alphas;   // 4n
  double* tmp;      // 3n: pcs (compute_pcs), later the reprojection errors
};

// s = ((0 + t(0)) + t(1)) + ... + t(n-1): the reference's sequential sum,
// with the terms of each group of 8 computed (and loaded) independently so
// their latencies overlap; only the additions form the chain.
template <class F>
__device__ __forceinline__ double seq_sum(int n, F term) {
  double s = 0;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    double t[8];
#pragma unroll
    for (int u = 0; u < 8; u++) t[u] = term(i + u);
#pragma unroll
    for (int u = 0; u < 8; u++) s += t[u];
  }
  for (; i < n; i++) s += term(i);
  return s;
}

template <int NT>
__device__ __forceinline__ void epnp_compute_pose(const PnpIn& in, const EpnpPts P, const int n, EpnpSmall* S) {
  const int tid = threadIdx.x;
  auto pw = [&](int k, int j) { return (double)P.pw[3 * k + j]; };
  auto uv = [&](int k, int j) { return (double)P.uv[2 * k + j]; };
  // choose_control_points
  if (tid < 3)  // the three coordinate sums are independent chains
    S->cws[0][tid] = seq_sum(n, [&](int i) { return pw(i, tid); }) / n;
  __syncthreads();
  if (tid < 6) {
    const int i = tid < 3 ? 0 : (tid < 5 ? 1 : 2), j = tid < 3 ? tid : (tid < 5 ? tid - 2 : 2);
    const double ci0 = S->cws[0][i], cj0 = S->cws[0][j];
    S->pw0tpw0[3 * i + j] = seq_sum(n, [&](int k) { return (pw(k, i) - ci0) * (pw(k, j) - cj0); });
  }
  __syncthreads();
  if (tid == 0) {
    double P9[9];
#pragma unroll
    for (int e = 0; e < 9; e++) P9[e] = S->pw0tpw0[e];
    P9[3] = P9[1];
    P9[6] = P9[2];
    P9[7] = P9[5];
    double uct[9], dc[3], vt[9];
    svd_rows<3, 3>(P9, uct, dc, vt);
#pragma unroll
    for (int i = 1; i < 4; i++) {
      const double k = sqrt(dc[i - 1] / n);
#pragma unroll
      for (int j = 0; j < 3; j++) S->cws[i][j] = S->cws[0][j] + k * uct[3 * (i - 1) + j];
    }
    double cc[9], ut[9], w[3], ci[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = S->cws[j][i] - S->cws[0][i];
    svd_rows<3, 3>(cc, ut, w, vt);
    svd_backsubst<3, 3, true>(ut, w, vt, nullptr, ci);
#pragma unroll
    for (int e = 0; e < 9; e++) S->ci[e] = ci[e];
  }
  __syncthreads();
  // compute_barycentric_coordinates
  for (int i = tid; i < n; i += NT) {
    double ci[9];
#pragma unroll
    for (int e = 0; e < 9; e++) ci[e] = S->ci[e];
    const double p0 = pw(i, 0), p1 = pw(i, 1), p2 = pw(i, 2);
    double a[4];
#pragma unroll
    for (int j = 0; j < 3; j++)
      a[1 + j] = ci[3 * j] * (p0 - S->cws[0][0]) + ci[3 * j + 1] * (p1 - S->cws[0][1]) + ci[3 * j + 2] * (p2 - S->cws[0][2]);
    a[0] = 1.0f - a[1] - a[2] - a[3];
#pragma unroll
    for (int j = 0; j < 4; j++) P.alphas[4 * i + j] = a[j];
  }
  __syncthreads();
  // MtM = M^T M, M = fill_M rows (2 per point, M1 then M2), upper triangle
  // sums over rows in order, mirrored
  for (int e = tid; e < 78; e += NT) {
    int i = 0, r = e;
    while (r >= 12 - i) {
      r -= 12 - i;
      i++;
    }
    const int j = i + r;
    const int qi = i / 3, ci = i % 3, qj = j / 3, cj = j % 3;
    // rows 2k (M1) and 2k+1 (M2) of point k, summed in row order; the fill_M
    // entry of column c is selected branch-free (c % 3: fu / 0 / (uc - u))
    // Branch-free: the factor is w_fu*fu + w_du*du with 0/1 weights, which is
    // exactly fu, du or +-0 (a +-0 entry where fill_M holds +0 yields a +-0
    // term, which never changes the sum).
    const double i0 = ci == 0, i2 = ci == 2, j0 = cj == 0, j2 = cj == 2;
    const double i1 = ci == 1, j1 = cj == 1;
    double s = 0;
    int k = 0;
    for (; k + 4 <= n; k += 4) {
      double t[8];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const double ai = P.alphas[4 * (k + u) + qi], aj = P.alphas[4 * (k + u) + qj];
        const double du = in.uc - uv(k + u, 0), dv = in.vc - uv(k + u, 1);
        t[2 * u] = (ai * (i0 * in.fu + i2 * du)) * (aj * (j0 * in.fu + j2 * du));
        t[2 * u + 1] = (ai * (i1 * in.fv + i2 * dv)) * (aj * (j1 * in.fv + j2 * dv));
      }
#pragma unroll
      for (int u = 0; u < 8; u++) s += t[u];
    }
    for (; k < n; k++) {
      const double ai = P.alphas[4 * k + qi], aj = P.alphas[4 * k + qj];
      const double du = in.uc - uv(k, 0), dv = in.vc - uv(k, 1);
      s += (ai * (i0 * in.fu + i2 * du)) * (aj * (j0 * in.fu + j2 * du));
      s += (ai * (i1 * in.fv + i2 * dv)) * (aj * (j1 * in.fv + j2 * dv));
    }
    S->mtm[12 * i + j] = s;
  }
  __syncthreads();
  if (tid < 64) {  // wave 0: Ut = MtM^T of the mirrored MtM, then the wave-parallel Jacobi
    for (int e = tid; e < 144; e += 64) {
      const int i = e / 12, k = e % 12;  // Ut[i][k] = MtM[k][i]; MtM[k][i] = upper (min, max)
      S->ut[e] = S->mtm[12 * min(i, k) + max(i, k)];
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    jacobi_svd_wave<12, 12>(S->ut, S->d);
  }
  __syncthreads();
  if (tid == 0) {
    compute_L_6x10(S->ut, S->l_6x10);
    S->rho[0] = dist2(S->cws[0], S->cws[1]);
    S->rho[1] = dist2(S->cws[0], S->cws[2]);
    S->rho[2] = dist2(S->cws[0], S->cws[3]);
    S->rho[3] = dist2(S->cws[1], S->cws[2]);
    S->rho[4] = dist2(S->cws[1], S->cws[3]);
    S->rho[5] = dist2(S->cws[2], S->cws[3]);
  }
  __syncthreads();
  // estimate_R_and_t's pw0 is the same for every approximation: once
  if (tid < 3) S->pw0[tid] = seq_sum(n, [&](int i) { return pw(i, tid); }) / n;
  __syncthreads();
  // The three beta approximations are independent: with >= 3 waves, wave w
  // runs approximation w+1 (its own ccs/pc0/abt/error scratch), so their
  // serial FP64 chains overlap; each keeps the reference's operation order.
  const int wv = tid >> 6, lane = tid & 63;
  constexpr bool kApPar = NT >= 192;
  auto wave_sync = [] {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
  };
  if (kApPar ? wv < 3 : wv == 0) {
    for (int ap = kApPar ? wv + 1 : 1; ap <= (kApPar ? wv + 1 : 3); ap++) {
      double* ccs_s = &S->ccs_ap[ap][0][0];
      if (lane == 0) {
        const double* l = S->l_6x10;
        const double* rho = S->rho;
        double betas[4];
        if (ap == 1) find_betas_approx_1(l, rho, betas);
        if (ap == 2) find_betas_approx_2(l, rho, betas);
        if (ap == 3) find_betas_approx_3(l, rho, betas);
        gauss_newton(l, rho, betas);
#pragma unroll
        for (int e = 0; e < 4; e++) S->betas[ap][e] = betas[e];
        // compute_ccs
        double ccs[4][3];
#pragma unroll
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const double* v = S->ut + 12 * (11 - i);
#pragma unroll
          for (int j = 0; j < 4; j++)
#pragma unroll
            for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
        }
        // solve_for_sign on point 0's compute_pcs value; the flipped pcs are
        // the pcs of the negated ccs, exactly
        const double* a0 = P.alphas;
        const double z0 = a0[0] * ccs[0][2] + a0[1] * ccs[1][2] + a0[2] * ccs[2][2] + a0[3] * ccs[3][2];
        const int flip = z0 < 0.0;
#pragma unroll
        for (int e = 0; e < 12; e++) ccs_s[e] = flip ? -ccs[e / 3][e % 3] : ccs[e / 3][e % 3];
      }
      wave_sync();
      // compute_pcs on the fly: pcs(i, j) from the point's alphas
      double cj[4] = {0, 0, 0, 0};
      const int jl = lane < 3 ? lane : (lane < 12 ? (lane - 3) / 3 : 0);
#pragma unroll
      for (int q = 0; q < 4; q++) cj[q] = ccs_s[3 * q + jl];
      auto pcs = [&](int i) {
        const double* a = P.alphas + 4 * i;
        return a[0] * cj[0] + a[1] * cj[1] + a[2] * cj[2] + a[3] * cj[3];
      };
      // estimate_R_and_t: centroid sums (lanes 0-2), then ABt sums (lanes 3-11), in point order
      if (lane < 3) S->pc0_ap[ap][lane] = seq_sum(n, pcs) / n;
      wave_sync();
      if (lane >= 3 && lane < 12) {
        const int c = (lane - 3) % 3;
        const double pc0 = S->pc0_ap[ap][jl], pw0 = S->pw0[c];
        S->abt_ap[ap][lane - 3] = seq_sum(n, [&](int i) { return (pcs(i) - pc0) * (pw(i, c) - pw0); });
      }
      wave_sync();
      if (lane == 0) {
        double abt[9], ut[9], w[3], vt[9], U[9], V[9];
#pragma unroll
        for (int e = 0; e < 9; e++) abt[e] = S->abt_ap[ap][e];
        svd_rows<3, 3>(abt, ut, w, vt);
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int k = 0; k < 3; k++) {
            U[3 * i + k] = ut[3 * k + i];
            V[3 * i + k] = vt[3 * k + i];
          }
        double R[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int j = 0; j < 3; j++) R[i][j] = dot3(U + 3 * i, V + 3 * j);
        const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                           R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
        if (det < 0) {
          R[2][0] = -R[2][0];
          R[2][1] = -R[2][1];
          R[2][2] = -R[2][2];
        }
        const double pc0[3] = {S->pc0_ap[ap][0], S->pc0_ap[ap][1], S->pc0_ap[ap][2]};
        const double pw0[3] = {S->pw0[0], S->pw0[1], S->pw0[2]};
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
          for (int j = 0; j < 3; j++) S->Rs[ap][i][j] = R[i][j];
#pragma unroll
        for (int r = 0; r < 3; r++) S->ts[ap][r] = pc0[r] - dot3(R[r], pw0);
      }
      wave_sync();
      double* err = P.tmp + (size_t)(ap - 1) * n;
      {
        double R[9], t[3];
#pragma unroll
        for (int e = 0; e < 9; e++) R[e] = S->Rs[ap][e / 3][e % 3];
#pragma unroll
        for (int e = 0; e < 3; e++) t[e] = S->ts[ap][e];
        for (int i = lane; i < n; i += (kApPar ? 64 : NT)) {  // reprojection_error terms
          const double p[3] = {pw(i, 0), pw(i, 1), pw(i, 2)};
          const double Xc = dot3(R, p) + t[0];
          const double Yc = dot3(R + 3, p) + t[1];
          const double inv_Zc = 1.0 / (dot3(R + 6, p) + t[2]);
          const double ue = in.uc + in.fu * Xc * inv_Zc;
          const double ve = in.vc + in.fv * Yc * inv_Zc;
          const double u = uv(i, 0), v = uv(i, 1);
          err[i] = sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
      }
      wave_sync();
      if (lane == 0) S->rep[ap] = seq_sum(n, [&](int i) { return err[i]; }) / n;
      wave_sync();
    }
  }
  __syncthreads();
  if (tid == 0) {
    int N = 1;
    if (S->rep[2] < S->rep[1]) N = 2;
    if (S->rep[3] < S->rep[N]) N = 3;
    S->rep[0] = (double)N;
  }
  __syncthreads();
}

// CheckInliers (:352-384) of one point
__device__ inline bool check_inlier(const PnpIn& in, const double* R, const double* t, int i) {
  const float X = in.p3d[3 * i], Y = in.p3d[3 * i + 1], Z = in.p3d[3 * i + 2];
  const float Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
  const float Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
  const float invZc = 1 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]);
  const double ue = in.uc + in.fu * Xc * invZc;
  const double ve = in.vc + in.fv * Yc * invZc;
  const float distX = in.p2d[2 * i] - ue;
  const float distY = in.p2d[2 * i + 1] - ve;
  const float error2 = distX * distX + distY * distY;
  return error2 < in.max_error[i];
}

// ------------------------------------------------------------ kernels
constexpr int kHypThreads = 256;  // 4 waves: the beta approximations run one per wave
constexpr int kRefThreads = 256;
constexpr int kRefineLdsPts = 2000;  // Refine stages up to this many inliers in LDS
constexpr size_t kRefinePtBytes = 4 * 8 + 3 * 8 + 3 * 4 + 2 * 4;  // alphas, pcs/errors, pw, uv

// One block per hypothesis: its minimal set staged in LDS, EPnP, pose record
// R (9, row-major) + t (3).
template <int NT>
__device__ __forceinline__ void pnp_hyp_body(const PnpIn& in, const int* __restrict__ idx, int set_size,
                                             double* __restrict__ pose) {
  __shared__ EpnpSmall S;
  __shared__ float spw[3 * kPnpMaxSet], suv[2 * kPnpMaxSet];
  __shared__ double salpha[4 * kPnpMaxSet], stmp[3 * kPnpMaxSet];
  const int tid = threadIdx.x;
  if (tid < set_size) {
    const int i = idx[tid];
#pragma unroll
    for (int j = 0; j < 3; j++) spw[3 * tid + j] = in.p3d[3 * i + j];
    suv[2 * tid] = in.p2d[2 * i];
    suv[2 * tid + 1] = in.p2d[2 * i + 1];
  }
  __syncthreads();
  epnp_compute_pose<NT>(in, EpnpPts{spw, suv, salpha, stmp}, set_size, &S);
  if (tid < 12) {
    const int b = (int)S.rep[0];
    pose[tid] = tid < 9 ? S.Rs[b][tid / 3][tid % 3] : S.ts[b][tid - 9];
  }
}

__global__ __launch_bounds__(kHypThreads) void k_pnp_hyp(PnpIn in, const int* __restrict__ sets, int set_size,
                                                         double* __restrict__ poses) {
  const int h = blockIdx.x;
  pnp_hyp_body<kHypThreads>(in, sets + (size_t)h * set_size, set_size, poses + 12 * (size_t)h);
}

// CheckInliers (src/PnPsolver.cc:352-384) of one hypothesis -> mask + count.
__device__ __forceinline__ void pnp_check_body(const PnpIn& in, const double* __restrict__ P,
                                               uint8_t* __restrict__ m, int* __restrict__ count) {
  __shared__ int red[4];
  double R[9], t[3];
  for (int i = 0; i < 9; i++) R[i] = P[i];
  for (int i = 0; i < 3; i++) t[i] = P[9 + i];
  int c = 0;
  for (int i = threadIdx.x; i < in.N; i += 256) {
    const bool ok = check_inlier(in, R, t, i);
    m[i] = ok;
    c += ok;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) *count = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_pnp_check(PnpIn in, const double* __restrict__ poses,
                                                   uint8_t* __restrict__ masks, int* __restrict__ counts) {
  const int h = blockIdx.x;
  pnp_check_body(in, poses + 12 * (size_t)h, masks + (size_t)h * in.N, counts + h);
}

// Many solvers in one launch (orbx_pnp_iterate_candidates / _many): grid (hypotheses
// of the largest job, jobs); job j runs its hypotheses h0 .. h0+H-1 (their minimal
// sets at sets[(h0 + h) * set_size], results at index h0 + h of its own arrays).
struct PnpHypJob {
  PnpIn in;
  const int* sets;
  double* poses;
  uint8_t* masks;
  int* counts;
  int h0, H, set_size;
};

// throughput form: one wave per hypothesis (the three beta approximations in series on it), so
// four hypotheses share a CU where the 4-wave latency form (whose VGPR budget allows one
// block per CU) runs one
constexpr int kHypManyThreads = 64;
__global__ __launch_bounds__(kHypManyThreads) __attribute__((amdgpu_waves_per_eu(2))) void k_pnp_hyp_many(const PnpHypJob* __restrict__ jobs) {
  const PnpHypJob& J = jobs[blockIdx.y];
  if ((int)blockIdx.x >= J.H) return;  // block-uniform
  const int h = J.h0 + blockIdx.x;
  pnp_hyp_body<kHypManyThreads>(J.in, J.sets + (size_t)h * J.set_size, J.set_size, J.poses + 12 * (size_t)h);
}

__global__ __launch_bounds__(256) void k_pnp_check_many(const PnpHypJob* __restrict__ jobs) {
  const PnpHypJob& J = jobs[blockIdx.y];
  if ((int)blockIdx.x >= J.H) return;
  const int h = J.h0 + blockIdx.x;
  pnp_check_body(J.in, J.poses + 12 * (size_t)h, J.masks + (size_t)h * J.in.N, J.counts + h);
}

// Refine(): EPnP on the inliers of `best` (ascending index), then CheckInliers.
// The inliers are compacted in order and staged in LDS (dynamic: kLds, up to
// kRefineLdsPts) or in the global work buffer.  out: [0..8] R, [9..11] t;
// *count; mask_out.
struct PnpRefJob {
  PnpIn in;
  const uint8_t* best;
  int* idx;
  double* work;
  double* out;
  uint8_t* mask_out;
  int* count;
};

template <bool kLds>
__device__ __forceinline__ void pnp_refine_body(const PnpRefJob& J) {
  __shared__ EpnpSmall S;
  __shared__ int wsum[4], base;
  extern __shared__ __attribute__((aligned(16))) double dyn[];
  const PnpIn& in = J.in;
  const int tid = threadIdx.x;
  // ordered compaction of the best inlier set
  if (tid == 0) base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < in.N; i0 += 256) {
    const int i = i0 + tid;
    const int f = (i < in.N && J.best[i]) ? 1 : 0;
    const unsigned long long bal = __ballot(f);
    const int lane = tid & 63, wv = tid >> 6;
    const int pre = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (f) J.idx[off + pre] = i;
    __syncthreads();
    if (tid == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  const int n = base;
  const int cap = kLds ? kRefineLdsPts : in.N;
  double* alphas = kLds ? dyn : J.work;
  double* tmp = alphas + 4 * (size_t)cap;
  float* spw = reinterpret_cast<float*>(tmp + 3 * (size_t)cap);
  float* suv = spw + 3 * (size_t)cap;
  for (int k = tid; k < n; k += kRefThreads) {
    const int i = J.idx[k];
#pragma unroll
    for (int j = 0; j < 3; j++) spw[3 * k + j] = in.p3d[3 * i + j];
    suv[2 * k] = in.p2d[2 * i];
    suv[2 * k + 1] = in.p2d[2 * i + 1];
  }
  __syncthreads();
  epnp_compute_pose<kRefThreads>(in, EpnpPts{spw, suv, alphas, tmp}, n, &S);
  const int b = (int)S.rep[0];
  double R[9], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[3 * i + j] = S.Rs[b][i][j];
    t[i] = S.ts[b][i];
  }
  int c = 0;
  for (int i = tid; i < in.N; i += kRefThreads) {
    const bool ok = check_inlier(in, R, t, i);
    J.mask_out[i] = ok;
    c += ok;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) wsum[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) {
    *J.count = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    for (int i = 0; i < 9; i++) J.out[i] = R[i];
    for (int i = 0; i < 3; i++) J.out[9 + i] = t[i];
  }
}

template <bool kLds>
__global__ __launch_bounds__(kRefThreads) void k_pnp_refine(PnpIn in, const uint8_t* __restrict__ best,
                                                            int* __restrict__ idx, double* __restrict__ work,
                                                            double* __restrict__ out, uint8_t* __restrict__ mask_out,
                                                            int* __restrict__ count) {
  pnp_refine_body<kLds>(PnpRefJob{in, best, idx, work, out, mask_out, count});
}

// one block per job
template <bool kLds>
__global__ __launch_bounds__(kRefThreads) void k_pnp_refine_many(const PnpRefJob* __restrict__ jobs) {
  pnp_refine_body<kLds>(jobs[blockIdx.x]);
}

// byte ranges of several solvers' buffers into one staging block (one readback for all)
struct PnpGatherJob {
  const uint8_t* src;
  uint8_t* dst;
  int n;
};
__global__ __launch_bounds__(256) void k_pnp_gather(const PnpGatherJob* __restrict__ jobs) {
  const PnpGatherJob J = jobs[blockIdx.x];
  for (int i = threadIdx.x; i < J.n; i += 256) J.dst[i] = J.src[i];
}

// correspondences of device-resident problems into their solvers' blocks (orbx_pnp_create_many_device):
// p3d, p2d copied, maxError = sigma2 * th2 (src/PnPsolver.cc:107, the float product of the host path)
struct PnpSetupJob {
  const float* p3d;
  const float* p2d;
  const float* sigma2;
  float* d_p3d;
  float* d_p2d;
  float* d_maxerr;
  int n;
};
__global__ __launch_bounds__(256) void k_pnp_setup(const PnpSetupJob* __restrict__ jobs, float th2) {
  const PnpSetupJob J = jobs[blockIdx.x];
  for (int i = threadIdx.x; i < J.n; i += 256) {
    J.d_p3d[3 * i] = J.p3d[3 * i];
    J.d_p3d[3 * i + 1] = J.p3d[3 * i + 1];
    J.d_p3d[3 * i + 2] = J.p3d[3 * i + 2];
    J.d_p2d[2 * i] = J.p2d[2 * i];
    J.d_p2d[2 * i + 1] = J.p2d[2 * i + 1];
    J.d_maxerr[i] = J.sigma2[i] * th2;
  }
}

}  // namespace orbx

// ------------------------------------------------------------------ host / C ABI
// One stream and one pinned readback block per device, shared by every
// solver (the reference creates a PnPsolver per relocalisation candidate, so
// creation must be cheap); each solver owns one stream-ordered allocation
// (hipMallocAsync) holding all of its arrays.
namespace {

struct PnpDevice {
  std::once_flag once;
  hipError_t init_err = hipSuccess;
  hipStream_t st = nullptr;
  std::mutex mu;  // serialises iterate() calls that share the stream and readback block
  void* pinned = nullptr;
  size_t pinned_cap = 0;
  void* dstage = nullptr;  // device staging of the batched calls: job records, minimal sets, counts
  size_t dstage_cap = 0;
  hipError_t dstage_reserve(size_t bytes) {
    if (bytes <= dstage_cap) return hipSuccess;
    if (dstage) (void)hipFree(dstage);
    dstage = nullptr;
    dstage_cap = 0;
    hipError_t e = hipMalloc(&dstage, bytes);
    if (e == hipSuccess) dstage_cap = bytes;
    return e;
  }
  hipError_t pinned_reserve(size_t bytes) {
    if (bytes <= pinned_cap) return hipSuccess;
    if (pinned) (void)hipHostFree(pinned);
    pinned = nullptr;
    pinned_cap = 0;
    hipError_t e = hipHostMalloc(&pinned, bytes, hipHostMallocDefault);
    if (e == hipSuccess) pinned_cap = bytes;
    return e;
  }
};
PnpDevice g_pnp_dev[64];

hipError_t pnp_device_init(int device) {
  PnpDevice& d = g_pnp_dev[device];
  std::call_once(d.once, [&] {
    d.init_err = hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking);
    if (d.init_err == hipSuccess)
      d.init_err = hipFuncSetAttribute((const void*)orbx::k_pnp_refine<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(orbx::kRefineLdsPts * orbx::kRefinePtBytes));
    if (d.init_err == hipSuccess)
      d.init_err = hipFuncSetAttribute((const void*)orbx::k_pnp_refine_many<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)(orbx::kRefineLdsPts * orbx::kRefinePtBytes));
    if (d.init_err == hipSuccess) d.init_err = d.pinned_reserve(1 << 16);
  });
  return d.init_err;
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

struct orbx_pnp {
  int device = 0;
  hipStream_t st = nullptr;
  int N = 0;
  double fu, fv, uc, vc;
  double prob;
  int min_inliers, max_its, min_set;
  float epsilon;
  // device (one allocation): correspondences, refine buffers, per-hypothesis buffers
  uint8_t* d_mem = nullptr;
  float *d_p3d = nullptr, *d_p2d = nullptr, *d_maxerr = nullptr;
  uint8_t *d_best = nullptr, *d_refmask = nullptr;
  int* d_idx = nullptr;
  double* d_rwork = nullptr;
  double* d_res = nullptr;  // refine result: R t (12) + count; best pose (12)
  int* d_sets = nullptr;
  double* d_poses = nullptr;
  uint8_t* d_masks = nullptr;
  int* d_counts = nullptr;
  int cap_hyp = 0;
  // iterate() state
  int iterations = 0, best_inliers = 0;
  float best_Tcw[16];
  bool refine_valid = false;  // Refine() of the current best set already known to fail
  orbx::PnpIn in() const {
    return orbx::PnpIn{d_p3d, d_p2d, d_maxerr, N, fu, fv, uc, vc};
  }
  // lays the arrays out in d_mem for cap hypotheses; returns the byte size
  size_t layout(int cap, uint8_t* base) {
    const size_t nn = std::max(N, 1);
    size_t o = 0;
    auto take = [&](size_t bytes) {
      uint8_t* p = base ? base + o : nullptr;
      o += align256(bytes);
      return p;
    };
    d_p3d = (float*)take(12 * nn);
    d_p2d = (float*)take(8 * nn);
    d_maxerr = (float*)take(4 * nn);
    d_best = take(nn);
    d_refmask = take(nn);
    d_idx = (int*)take(4 * nn);
    d_rwork = (double*)take(orbx::kRefinePtBytes * nn);  // global-fallback refine: same per-point layout
    d_res = (double*)take(8 * 32);
    d_sets = (int*)take(sizeof(int) * (size_t)cap * orbx::kPnpMaxSet);
    d_poses = (double*)take(sizeof(double) * 12 * (size_t)cap);
    d_masks = take((size_t)cap * nn);
    d_counts = (int*)take(sizeof(int) * (size_t)cap);
    return o;
  }
  // grows the per-hypothesis buffers to H, keeping correspondences, best mask and results
  hipError_t ensure_cap(int H) {
    if (H <= cap_hyp) return hipSuccess;
    uint8_t* old = d_mem;
    const size_t keep = (uint8_t*)d_best - (uint8_t*)d_p3d;
    const size_t best_off = (uint8_t*)d_best - old, res_off = (uint8_t*)d_res - old;
    d_mem = nullptr;
    const size_t bytes = layout(H, nullptr);
    hipError_t e = hipMallocAsync((void**)&d_mem, bytes, st);
    if (e != hipSuccess) return e;
    layout(H, d_mem);
    cap_hyp = H;
    if ((e = hipMemcpyAsync(d_p3d, old, keep, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(d_best, old + best_off, std::max(N, 1), hipMemcpyDeviceToDevice, st)) != hipSuccess)
      return e;
    if ((e = hipMemcpyAsync(d_res, old + res_off, 8 * 32, hipMemcpyDeviceToDevice, st)) != hipSuccess) return e;
    return hipFreeAsync(old, st);
  }
  hipError_t alloc(int cap) {  // (re)allocates d_mem; the correspondences are re-uploaded by the caller
    if (d_mem) (void)hipFreeAsync(d_mem, st);
    d_mem = nullptr;
    const size_t bytes = layout(cap, nullptr);
    hipError_t e = hipMallocAsync((void**)&d_mem, bytes, st);
    if (e != hipSuccess) return e;
    layout(cap, d_mem);
    cap_hyp = cap;
    return hipSuccess;
  }
};

namespace {

void pose_to_Tcw(const double* P, float T[16]) {  // Rcw/tcw convertTo(CV_32F) into eye(4)
  for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.f : 0.f;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = (float)P[3 * r + c];
    T[4 * r + 3] = (float)P[9 + r];
  }
}

#define PNP_CHECK(x)                             \
  do {                                           \
    if ((x) != hipSuccess) return ORBX_ERR_HIP;  \
  } while (0)

}  // namespace

extern "C" {

}  // extern "C"

namespace {

orbx_status pnp_check_problem(const orbx_pnp_problem* p, const orbx_pnp_params* prm) {
  if (!p || !prm || p->n < 0 || (p->n > 0 && (!p->p3d || !p->p2d || !p->sigma2))) return ORBX_ERR_ARG;
  if (prm->min_set < 1 || prm->min_set > orbx::kPnpMaxSet) return ORBX_ERR_ARG;
  return ORBX_OK;
}

orbx_status pnp_device_check(int device) {
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= nd || device >= 64) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  if (pnp_device_init(device) != hipSuccess) return ORBX_ERR_HIP;
  return ORBX_OK;
}

// SetRansacParameters' derived values (src/PnPsolver.cc:136-179) from the handle's N
void pnp_derive(orbx_pnp* h, const orbx_pnp_params* prm) {
  const int n = h->N;
  h->prob = prm->probability;
  h->min_inliers = prm->min_inliers;
  h->max_its = prm->max_iterations;
  h->epsilon = prm->epsilon;
  h->min_set = prm->min_set;
  int nMinInliers = n * h->epsilon;
  if (nMinInliers < h->min_inliers) nMinInliers = h->min_inliers;
  if (nMinInliers < prm->min_set) nMinInliers = prm->min_set;
  h->min_inliers = nMinInliers;
  if (n > 0 && h->epsilon < (float)h->min_inliers / n) h->epsilon = (float)h->min_inliers / n;
  int nIterations;
  if (h->min_inliers == n)
    nIterations = 1;
  else
    nIterations = (int)std::ceil(std::log(1 - h->prob) / std::log(1 - std::pow(h->epsilon, 3)));
  h->max_its = std::max(1, std::min(nIterations, h->max_its));
}

// PnPsolver ctor + SetRansacParameters (src/PnPsolver.cc:67-179) without the upload
orbx_pnp* pnp_new(const orbx_pnp_problem* p, const orbx_pnp_params* prm, int device) {
  orbx_pnp* h = new (std::nothrow) orbx_pnp();
  if (!h) return nullptr;
  h->device = device;
  h->st = g_pnp_dev[device].st;
  const int n = p->n;
  h->N = n;
  h->fu = p->fx;
  h->fv = p->fy;
  h->uc = p->cx;
  h->vc = p->cy;
  pnp_derive(h, prm);
  for (int i = 0; i < 16; i++) h->best_Tcw[i] = 0;
  return h;
}

// p3d | p2d | maxerr (= sigma2 * th2) of one solver, laid out as in its device block
void pnp_stage_problem(const orbx_pnp* h, const orbx_pnp_problem* p, const orbx_pnp_params* prm, uint8_t* dst) {
  const int n = p->n;
  std::memcpy(dst, p->p3d, 12 * (size_t)n);
  std::memcpy(dst + ((uint8_t*)h->d_p2d - (uint8_t*)h->d_p3d), p->p2d, 8 * (size_t)n);
  float* me = (float*)(dst + ((uint8_t*)h->d_maxerr - (uint8_t*)h->d_p3d));
  for (int i = 0; i < n; i++) me[i] = p->sigma2[i] * prm->th2;
}

}  // namespace

extern "C" {

orbx_status orbx_pnp_create(const orbx_pnp_problem* p, const orbx_pnp_params* prm, int device, orbx_pnp** out) {
  orbx_status s = pnp_check_problem(p, prm);
  if (s != ORBX_OK || !out) return s != ORBX_OK ? s : ORBX_ERR_ARG;
  *out = nullptr;
  if ((s = pnp_device_check(device)) != ORBX_OK) return s;
  orbx_pnp* h = pnp_new(p, prm, device);
  if (!h) return ORBX_ERR_HIP;
  const int n = p->n;
  hipError_t e = h->alloc(std::max(h->max_its, 8));
  if (e == hipSuccess && n > 0) {
    // one upload: p3d | p2d | maxerr are consecutive in the layout
    std::vector<uint8_t> stage((uint8_t*)h->d_best - (uint8_t*)h->d_p3d);
    pnp_stage_problem(h, p, prm, stage.data());
    e = hipMemcpyAsync(h->d_p3d, stage.data(), stage.size(), hipMemcpyHostToDevice, h->st);
    if (e == hipSuccess) e = hipStreamSynchronize(h->st);  // stage is pageable and local
  }
  if (e != hipSuccess) {
    if (h->d_mem) (void)hipFreeAsync(h->d_mem, h->st);
    delete h;
    return ORBX_ERR_HIP;
  }
  *out = h;
  return ORBX_OK;
}

orbx_status orbx_pnp_create_many(const orbx_pnp_problem* problems, int n, const orbx_pnp_params* prm, int device,
                                 orbx_pnp** out) {
  if (n < 0 || (n > 0 && (!problems || !out))) return ORBX_ERR_ARG;
  for (int i = 0; i < n; i++) {
    const orbx_status s = pnp_check_problem(&problems[i], prm);
    if (s != ORBX_OK) return s;
    out[i] = nullptr;
  }
  if (n == 0) return ORBX_OK;
  orbx_status s = pnp_device_check(device);
  if (s != ORBX_OK) return s;
  PnpDevice& dev = g_pnp_dev[device];
  std::lock_guard<std::mutex> lock(dev.mu);
  std::vector<orbx_pnp*> hs(n, nullptr);
  auto fail = [&](orbx_status code) {
    for (orbx_pnp* h : hs)
      if (h) {
        if (h->d_mem) (void)hipFreeAsync(h->d_mem, h->st);
        delete h;
      }
    return code;
  };
  size_t stage = 0;
  for (int i = 0; i < n; i++) {
    hs[i] = pnp_new(&problems[i], prm, device);
    if (!hs[i]) return fail(ORBX_ERR_HIP);
    if (hs[i]->alloc(std::max(hs[i]->max_its, 8)) != hipSuccess) return fail(ORBX_ERR_HIP);
    stage += align256((uint8_t*)hs[i]->d_best - (uint8_t*)hs[i]->d_p3d);
  }
  // all correspondences in one pinned block, one upload, one gather launch into the solvers' blocks
  const size_t off_data = align256(n * sizeof(orbx::PnpGatherJob));
  const size_t bytes = off_data + stage;
  if (dev.pinned_reserve(bytes) != hipSuccess || dev.dstage_reserve(bytes) != hipSuccess) return fail(ORBX_ERR_HIP);
  uint8_t* hp = (uint8_t*)dev.pinned;
  uint8_t* dp = (uint8_t*)dev.dstage;
  orbx::PnpGatherJob* jobs = (orbx::PnpGatherJob*)hp;
  size_t o = off_data;
  for (int i = 0; i < n; i++) {
    orbx_pnp* h = hs[i];
    const size_t len = (uint8_t*)h->d_best - (uint8_t*)h->d_p3d;
    if (problems[i].n > 0) pnp_stage_problem(h, &problems[i], prm, hp + o);
    jobs[i] = orbx::PnpGatherJob{dp + o, (uint8_t*)h->d_p3d, problems[i].n > 0 ? (int)len : 0};
    o += align256(len);
  }
  hipStream_t st = dev.st;
  if (hipMemcpyAsync(dp, hp, bytes, hipMemcpyHostToDevice, st) != hipSuccess) return fail(ORBX_ERR_HIP);
  hipLaunchKernelGGL(orbx::k_pnp_gather, dim3(n), dim3(256), 0, st, (const orbx::PnpGatherJob*)dp);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return fail(ORBX_ERR_HIP);
  for (int i = 0; i < n; i++) out[i] = hs[i];
  return ORBX_OK;
}

orbx_status orbx_pnp_create_many_device(const float* d_p3d, const float* d_p2d, const float* d_sigma2,
                                        const int32_t* offsets, const float* intr, int n,
                                        const orbx_pnp_params* prm, int device, orbx_pnp** out) {
  if (n < 0 || (n > 0 && (!offsets || !intr || !out || !prm))) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  if (!d_p3d || !d_p2d || !d_sigma2 || prm->min_set < 1 || prm->min_set > orbx::kPnpMaxSet) return ORBX_ERR_ARG;
  for (int i = 0; i < n; i++) {
    if (offsets[i + 1] < offsets[i]) return ORBX_ERR_ARG;
    out[i] = nullptr;
  }
  orbx_status s = pnp_device_check(device);
  if (s != ORBX_OK) return s;
  PnpDevice& dev = g_pnp_dev[device];
  std::lock_guard<std::mutex> lock(dev.mu);
  std::vector<orbx_pnp*> hs(n, nullptr);
  auto fail = [&](orbx_status code) {
    for (orbx_pnp* h : hs)
      if (h) {
        if (h->d_mem) (void)hipFreeAsync(h->d_mem, h->st);
        delete h;
      }
    return code;
  };
  const size_t bytes = n * sizeof(orbx::PnpSetupJob);
  if (dev.pinned_reserve(bytes) != hipSuccess || dev.dstage_reserve(bytes) != hipSuccess) return fail(ORBX_ERR_HIP);
  orbx::PnpSetupJob* jobs = (orbx::PnpSetupJob*)dev.pinned;
  for (int i = 0; i < n; i++) {
    const orbx_pnp_problem p{offsets[i + 1] - offsets[i], nullptr, nullptr, nullptr, intr[4 * i], intr[4 * i + 1],
                             intr[4 * i + 2], intr[4 * i + 3]};
    hs[i] = pnp_new(&p, prm, device);
    if (!hs[i]) return fail(ORBX_ERR_HIP);
    if (hs[i]->alloc(std::max(hs[i]->max_its, 8)) != hipSuccess) return fail(ORBX_ERR_HIP);
    const size_t o = (size_t)offsets[i];
    jobs[i] = orbx::PnpSetupJob{d_p3d + 3 * o, d_p2d + 2 * o, d_sigma2 + o, hs[i]->d_p3d, hs[i]->d_p2d,
                                hs[i]->d_maxerr, p.n};
  }
  hipStream_t st = dev.st;
  if (hipMemcpyAsync(dev.dstage, dev.pinned, bytes, hipMemcpyHostToDevice, st) != hipSuccess) return fail(ORBX_ERR_HIP);
  hipLaunchKernelGGL(orbx::k_pnp_setup, dim3(n), dim3(256), 0, st, (const orbx::PnpSetupJob*)dev.dstage, prm->th2);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return fail(ORBX_ERR_HIP);
  for (int i = 0; i < n; i++) out[i] = hs[i];
  return ORBX_OK;
}

orbx_status orbx_pnp_destroy(orbx_pnp* h) {
  if (!h) return ORBX_ERR_ARG;
  (void)hipSetDevice(h->device);
  if (h->d_mem) (void)hipFreeAsync(h->d_mem, h->st);
  delete h;
  return ORBX_OK;
}

orbx_status orbx_pnp_set_ransac_parameters(orbx_pnp* h, const float* sigma2, const orbx_pnp_params* prm) {
  if (!h || !prm || (h->N > 0 && !sigma2)) return ORBX_ERR_ARG;
  if (prm->min_set < 1 || prm->min_set > orbx::kPnpMaxSet) return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  PnpDevice& dev = g_pnp_dev[h->device];
  std::lock_guard<std::mutex> lock(dev.mu);
  // src/PnPsolver.cc:136-179 recomputes the parameters in place: mnIterations, mnBestInliers and
  // mvbBestInliers (and the best pose) are kept; mvMaxError = sigma2 * th2 is rebuilt
  pnp_derive(h, prm);
  h->refine_valid = false;  // Refine() succeeds on "> mRansacMinInliers", which may have changed
  if (h->N > 0) {
    PNP_CHECK(dev.pinned_reserve(4 * (size_t)h->N));
    float* me = (float*)dev.pinned;
    for (int i = 0; i < h->N; i++) me[i] = sigma2[i] * prm->th2;
    PNP_CHECK(hipMemcpyAsync(h->d_maxerr, me, 4 * (size_t)h->N, hipMemcpyHostToDevice, h->st));
    PNP_CHECK(hipStreamSynchronize(h->st));  // the pinned block is reused by the next call
  }
  return ORBX_OK;
}

orbx_status orbx_pnp_get_params(const orbx_pnp* h, int* min_inliers, int* max_iterations, float* epsilon) {
  if (!h) return ORBX_ERR_ARG;
  if (min_inliers) *min_inliers = h->min_inliers;
  if (max_iterations) *max_iterations = h->max_its;
  if (epsilon) *epsilon = h->epsilon;
  return ORBX_OK;
}

orbx_status orbx_pnp_iterate(orbx_pnp* h, int n_iterations, const int32_t* rand_vals, int n_rand, int* used,
                             int* no_more, float Tcw[16], uint8_t* inliers, int* n_inliers, int* found) {
  if (!h || !used || !no_more || !Tcw || !n_inliers || !found || (h->N > 0 && !inliers) || n_rand < 0 ||
      (n_rand > 0 && !rand_vals))
    return ORBX_ERR_ARG;
  *used = 0;
  *no_more = 0;
  *n_inliers = 0;
  *found = 0;
  const int N = h->N, ms = h->min_set;
  if (N < h->min_inliers) {
    *no_more = 1;
    return ORBX_OK;
  }
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  // hypotheses this call may run: while (iterations < maxIts || current < nIterations)
  const int H = std::max(h->max_its - h->iterations, n_iterations);
  if (H <= 0) return ORBX_OK;
  if ((long long)H * ms > n_rand) return ORBX_ERR_CAPACITY;
  PnpDevice& dev = g_pnp_dev[h->device];
  std::lock_guard<std::mutex> lock(dev.mu);
  const size_t pin_bytes = std::max(sizeof(int) * (size_t)H * ms, sizeof(int) * (size_t)H) + 8 * 32;
  PNP_CHECK(dev.pinned_reserve(pin_bytes));
  PNP_CHECK(h->ensure_cap(H));  // keeps the correspondences
  // DUtils::Random::RandomInt(0, size-1) on the rand() stream + swap-remove
  int* sets = (int*)dev.pinned;
  std::vector<int> avail(N);
  for (int k = 0; k < H; k++) {
    for (int i = 0; i < N; i++) avail[i] = i;
    int size = N;
    for (int i = 0; i < ms; i++) {
      const int randi = (int)(((double)rand_vals[k * ms + i] / ((double)RAND_MAX + 1.0)) * size);
      sets[(size_t)k * ms + i] = avail[randi];
      avail[randi] = avail[size - 1];
      size--;
    }
  }
  hipStream_t st = h->st;
  PNP_CHECK(hipMemcpyAsync(h->d_sets, sets, sizeof(int) * (size_t)H * ms, hipMemcpyHostToDevice, st));
  const orbx::PnpIn in = h->in();
  hipLaunchKernelGGL(orbx::k_pnp_hyp, dim3(H), dim3(orbx::kHypThreads), 0, st, in, h->d_sets, ms, h->d_poses);
  hipLaunchKernelGGL(orbx::k_pnp_check, dim3(H), dim3(256), 0, st, in, h->d_poses, h->d_masks, h->d_counts);
  PNP_CHECK(hipGetLastError());
  int* counts = (int*)dev.pinned;  // the sets were consumed by the copy above (stream order)
  PNP_CHECK(hipMemcpyAsync(counts, h->d_counts, sizeof(int) * H, hipMemcpyDeviceToHost, st));
  PNP_CHECK(hipStreamSynchronize(st));
  double* res = (double*)((uint8_t*)dev.pinned + align256(sizeof(int) * (size_t)H));
  int cur = 0;
  for (int k = 0; k < H && (h->iterations < h->max_its || cur < n_iterations); k++) {
    cur++;
    h->iterations++;
    *used += ms;
    if (counts[k] < h->min_inliers) continue;
    if (counts[k] > h->best_inliers) {  // new best: mask + pose stay on the device
      h->best_inliers = counts[k];
      PNP_CHECK(hipMemcpyAsync(h->d_best, h->d_masks + (size_t)k * N, N, hipMemcpyDeviceToDevice, st));
      PNP_CHECK(hipMemcpyAsync(h->d_res + 16, h->d_poses + 12 * (size_t)k, 12 * sizeof(double),
                               hipMemcpyDeviceToDevice, st));
      h->refine_valid = false;
    }
    if (h->refine_valid) continue;  // same best set: Refine() fails again
    if (h->best_inliers <= orbx::kRefineLdsPts)  // the refined set is the best mask
      hipLaunchKernelGGL(orbx::k_pnp_refine<true>, dim3(1), dim3(orbx::kRefThreads),
                         orbx::kRefineLdsPts * orbx::kRefinePtBytes, st, in, h->d_best, h->d_idx, h->d_rwork,
                         h->d_res, h->d_refmask, (int*)(h->d_res + 12));
    else
      hipLaunchKernelGGL(orbx::k_pnp_refine<false>, dim3(1), dim3(orbx::kRefThreads), 0, st, in, h->d_best, h->d_idx,
                         h->d_rwork, h->d_res, h->d_refmask, (int*)(h->d_res + 12));
    PNP_CHECK(hipGetLastError());
    PNP_CHECK(hipMemcpyAsync(res, h->d_res, 13 * sizeof(double), hipMemcpyDeviceToHost, st));
    PNP_CHECK(hipStreamSynchronize(st));
    const int rc = *(const int*)(res + 12);
    if (rc > h->min_inliers) {
      PNP_CHECK(hipMemcpyAsync(inliers, h->d_refmask, N, hipMemcpyDeviceToHost, st));
      PNP_CHECK(hipStreamSynchronize(st));
      pose_to_Tcw(res, Tcw);
      *n_inliers = rc;
      *found = 1;
      return ORBX_OK;
    }
    h->refine_valid = true;
  }
  if (h->iterations >= h->max_its) {
    *no_more = 1;
    if (h->best_inliers >= h->min_inliers) {
      PNP_CHECK(hipMemcpyAsync(res, h->d_res + 16, 12 * sizeof(double), hipMemcpyDeviceToHost, st));
      PNP_CHECK(hipMemcpyAsync(inliers, h->d_best, N, hipMemcpyDeviceToHost, st));
      PNP_CHECK(hipStreamSynchronize(st));
      pose_to_Tcw(res, h->best_Tcw);
      std::memcpy(Tcw, h->best_Tcw, sizeof(float) * 16);
      *n_inliers = h->best_inliers;
      *found = 1;
    }
  }
  return ORBX_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- many solvers
// The walk of PnPsolver::iterate (the loop above) over several solvers at once.
// Hypotheses are computed a chunk at a time for every solver that needs them
// (one k_pnp_hyp_many + one k_pnp_check_many launch per round, minimal sets and
// job records in one upload, counts in one readback), each solver's walk runs on
// the host exactly as in orbx_pnp_iterate, and the Refine() calls the walks ask
// for in the same round go out as one k_pnp_refine_many launch.
namespace {

struct PnpRun {
  orbx_pnp* h = nullptr;
  const int32_t* rv = nullptr;  // rand values this call may consume (H * min_set)
  int H = 0;                    // hypotheses this call may run
  int k = 0;                    // next hypothesis to walk
  int launched = 0;             // hypotheses [0, launched) have counts
  int cur = 0, used = 0;
  bool eligible = true, done = false, pending = false, read_best = false;
  int best_k = -1;  // hypothesis of this call holding the best set (-1: d_best / d_res+16 of an earlier call)
  const uint8_t* best_mask() const { return best_k >= 0 ? h->d_masks + (size_t)best_k * h->N : h->d_best; }
  const double* best_pose() const { return best_k >= 0 ? h->d_poses + 12 * (size_t)best_k : h->d_res + 16; }
  std::vector<int> counts;
  orbx_pnp_result* out = nullptr;
  uint8_t* inliers = nullptr;
};

constexpr int kPnpFirstChunk = 16;  // RANSAC at ~60 % inliers usually stops within its first hypotheses

orbx_status pnp_begin(PnpRun& r, int n_iterations) {
  orbx_pnp* h = r.h;
  r.out->no_more = r.out->found = r.out->n_inliers = r.out->used = 0;
  if (h->N < h->min_inliers) {
    r.out->no_more = 1;
    r.done = true;
    return ORBX_OK;
  }
  r.H = std::max(h->max_its - h->iterations, n_iterations);
  if (r.H <= 0) {
    r.H = 0;
    r.done = true;
    return ORBX_OK;
  }
  r.counts.assign(r.H, 0);
  return h->ensure_cap(r.H) == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

// hypotheses [launched, launched + c) of every run in `rs` with c > 0
orbx_status pnp_launch_chunks(PnpDevice& dev, hipStream_t st, std::vector<std::pair<PnpRun*, int>>& rs) {
  if (rs.empty()) return ORBX_OK;
  const size_t nj = rs.size();
  size_t nsets = 0, ncounts = 0;
  int maxc = 0;
  for (auto& q : rs) {
    nsets += (size_t)q.second * q.first->h->min_set;
    ncounts += q.second;
    maxc = std::max(maxc, q.second);
  }
  const size_t off_sets = align256(nj * sizeof(orbx::PnpHypJob));
  const size_t off_counts = off_sets + align256(nsets * sizeof(int));
  const size_t bytes = off_counts + align256(ncounts * sizeof(int));
  PNP_CHECK(dev.pinned_reserve(bytes));
  PNP_CHECK(dev.dstage_reserve(bytes));
  uint8_t* hp = (uint8_t*)dev.pinned;
  uint8_t* dp = (uint8_t*)dev.dstage;
  orbx::PnpHypJob* jobs = (orbx::PnpHypJob*)hp;
  int* sets = (int*)(hp + off_sets);
  size_t so = 0, co = 0;
  for (size_t j = 0; j < nj; j++) {
    PnpRun& r = *rs[j].first;
    orbx_pnp* h = r.h;
    const int c = rs[j].second, ms = h->min_set, N = h->N, h0 = r.launched;
    // DUtils::Random::RandomInt(0, size-1) on the rand() stream + swap-remove (src/PnPsolver.cc:214-229)
    std::vector<int> avail(N);
    for (int k = 0; k < c; k++) {
      for (int i = 0; i < N; i++) avail[i] = i;
      int size = N;
      for (int i = 0; i < ms; i++) {
        const int32_t v = r.rv[(size_t)(h0 + k) * ms + i];
        const int randi = (int)(((double)v / ((double)RAND_MAX + 1.0)) * size);
        sets[so + (size_t)k * ms + i] = avail[randi];
        avail[randi] = avail[size - 1];
        size--;
      }
    }
    orbx::PnpHypJob& J = jobs[j];
    J.in = h->in();
    J.sets = (const int*)(dp + off_sets) + so - (size_t)h0 * ms;  // indexed by absolute hypothesis
    J.poses = h->d_poses;
    J.masks = h->d_masks;
    J.counts = (int*)(dp + off_counts) + co - h0;
    J.h0 = h0;
    J.H = c;
    J.set_size = ms;
    so += (size_t)c * ms;
    co += c;
  }
  PNP_CHECK(hipMemcpyAsync(dp, hp, off_counts, hipMemcpyHostToDevice, st));
  const orbx::PnpHypJob* dj = (const orbx::PnpHypJob*)dp;
  hipLaunchKernelGGL(orbx::k_pnp_hyp_many, dim3(maxc, nj), dim3(orbx::kHypManyThreads), 0, st, dj);
  hipLaunchKernelGGL(orbx::k_pnp_check_many, dim3(maxc, nj), dim3(256), 0, st, dj);
  PNP_CHECK(hipGetLastError());
  int* hc = (int*)(hp + off_counts);
  PNP_CHECK(hipMemcpyAsync(hc, dp + off_counts, ncounts * sizeof(int), hipMemcpyDeviceToHost, st));
  PNP_CHECK(hipStreamSynchronize(st));
  co = 0;
  for (auto& q : rs) {
    PnpRun& r = *q.first;
    for (int k = 0; k < q.second; k++) r.counts[r.launched + k] = hc[co + k];
    co += q.second;
    r.launched += q.second;
  }
  return ORBX_OK;
}

// the walk of orbx_pnp_iterate from hypothesis r.k: stops at a Refine() request,
// at the end of the launched hypotheses, or at the end of the call
orbx_status pnp_walk(PnpRun& r) {
  orbx_pnp* h = r.h;
  while (!r.pending && r.k < r.launched) {
    const int k = r.k++;
    r.cur++;
    h->iterations++;
    r.used += h->min_set;
    if (r.counts[k] < h->min_inliers) continue;
    if (r.counts[k] > h->best_inliers) {  // new best: its mask and pose stay where they are
      h->best_inliers = r.counts[k];
      r.best_k = k;
      h->refine_valid = false;
    }
    if (h->refine_valid) continue;  // same best set: Refine() fails again
    r.pending = true;
  }
  return ORBX_OK;
}

// the end of iterate() once all H hypotheses were walked without a refined pose
// (the best pose and mask are read back by pnp_read_best, batched)
void pnp_finish(PnpRun& r) {
  orbx_pnp* h = r.h;
  r.done = true;
  if (h->iterations >= h->max_its) {
    r.out->no_more = 1;
    if (h->best_inliers >= h->min_inliers) {
      r.out->n_inliers = h->best_inliers;
      r.out->found = 1;
      r.read_best = true;
    }
  }
}

// best pose (12 doubles) + best mask of every run in `rs`: one gather launch, one readback
orbx_status pnp_read_best(PnpDevice& dev, hipStream_t st, std::vector<PnpRun*>& rs) {
  if (rs.empty()) return ORBX_OK;
  const size_t nj = 2 * rs.size();
  size_t data = 0;
  for (PnpRun* r : rs) data += 96 + align256((size_t)r->h->N);
  const size_t off_data = align256(nj * sizeof(orbx::PnpGatherJob));
  const size_t bytes = off_data + data;
  PNP_CHECK(dev.pinned_reserve(bytes));
  PNP_CHECK(dev.dstage_reserve(bytes));
  uint8_t* hp = (uint8_t*)dev.pinned;
  uint8_t* dp = (uint8_t*)dev.dstage;
  orbx::PnpGatherJob* jobs = (orbx::PnpGatherJob*)hp;
  size_t o = off_data;
  for (size_t j = 0; j < rs.size(); j++) {
    orbx_pnp* h = rs[j]->h;
    jobs[2 * j] = orbx::PnpGatherJob{(const uint8_t*)rs[j]->best_pose(), dp + o, 96};
    jobs[2 * j + 1] = orbx::PnpGatherJob{rs[j]->best_mask(), dp + o + 96, h->N};
    o += 96 + align256((size_t)h->N);
  }
  PNP_CHECK(hipMemcpyAsync(dp, hp, nj * sizeof(orbx::PnpGatherJob), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(orbx::k_pnp_gather, dim3(nj), dim3(256), 0, st, (const orbx::PnpGatherJob*)dp);
  PNP_CHECK(hipGetLastError());
  PNP_CHECK(hipMemcpyAsync(hp + off_data, dp + off_data, data, hipMemcpyDeviceToHost, st));
  PNP_CHECK(hipStreamSynchronize(st));
  o = off_data;
  for (PnpRun* r : rs) {
    orbx_pnp* h = r->h;
    pose_to_Tcw((const double*)(hp + o), h->best_Tcw);
    std::memcpy(r->out->Tcw, h->best_Tcw, sizeof(float) * 16);
    if (r->inliers) std::memcpy(r->inliers, hp + o + 96, h->N);
    r->read_best = false;
    o += 96 + align256((size_t)h->N);
  }
  rs.clear();
  return ORBX_OK;
}

orbx_status pnp_refine_round(PnpDevice& dev, hipStream_t st, std::vector<PnpRun*>& pend) {
  if (pend.empty()) return ORBX_OK;
  const size_t nj = pend.size();
  // staging: job records | per job 16 doubles (R t, count) | per job its refined mask
  size_t masks = 0;
  for (PnpRun* r : pend) masks += align256((size_t)r->h->N);
  const size_t off_res = align256(nj * sizeof(orbx::PnpRefJob));
  const size_t off_mask = off_res + align256(nj * 16 * sizeof(double));
  const size_t bytes = off_mask + masks;
  PNP_CHECK(dev.pinned_reserve(bytes));
  PNP_CHECK(dev.dstage_reserve(bytes));
  uint8_t* hp = (uint8_t*)dev.pinned;
  uint8_t* dp = (uint8_t*)dev.dstage;
  orbx::PnpRefJob* jobs = (orbx::PnpRefJob*)hp;
  // LDS-staged jobs first, then the (rare) jobs whose best set exceeds the LDS stage
  std::vector<PnpRun*> order;
  for (PnpRun* r : pend)
    if (r->h->best_inliers <= orbx::kRefineLdsPts) order.push_back(r);
  const int n_lds = (int)order.size();
  for (PnpRun* r : pend)
    if (r->h->best_inliers > orbx::kRefineLdsPts) order.push_back(r);
  std::vector<size_t> moff(nj);
  size_t mo = off_mask;
  for (size_t j = 0; j < nj; j++) {
    orbx_pnp* h = order[j]->h;
    double* out = (double*)(dp + off_res) + 16 * j;
    moff[j] = mo;
    jobs[j] = orbx::PnpRefJob{h->in(), order[j]->best_mask(), h->d_idx, h->d_rwork, out, dp + mo, (int*)(out + 12)};
    mo += align256((size_t)h->N);
  }
  PNP_CHECK(hipMemcpyAsync(dp, hp, nj * sizeof(orbx::PnpRefJob), hipMemcpyHostToDevice, st));
  const orbx::PnpRefJob* dj = (const orbx::PnpRefJob*)dp;
  if (n_lds > 0)
    hipLaunchKernelGGL(orbx::k_pnp_refine_many<true>, dim3(n_lds), dim3(orbx::kRefThreads),
                       orbx::kRefineLdsPts * orbx::kRefinePtBytes, st, dj);
  if ((int)nj > n_lds)
    hipLaunchKernelGGL(orbx::k_pnp_refine_many<false>, dim3((int)nj - n_lds), dim3(orbx::kRefThreads), 0, st,
                       dj + n_lds);
  PNP_CHECK(hipGetLastError());
  PNP_CHECK(hipMemcpyAsync(hp + off_res, dp + off_res, bytes - off_res, hipMemcpyDeviceToHost, st));
  PNP_CHECK(hipStreamSynchronize(st));
  const double* res = (const double*)(hp + off_res);
  for (size_t j = 0; j < nj; j++) {
    PnpRun& r = *order[j];
    orbx_pnp* h = r.h;
    r.pending = false;
    const int rc = *(const int*)(res + 16 * j + 12);
    if (rc > h->min_inliers) {  // Refine() succeeded: the call returns mRefinedTcw
      if (r.inliers) std::memcpy(r.inliers, hp + moff[j], h->N);
      pose_to_Tcw(res + 16 * j, r.out->Tcw);
      r.out->n_inliers = rc;
      r.out->found = 1;
      r.done = true;
    } else {
      h->refine_valid = true;
    }
  }
  return ORBX_OK;
}

// shared: all runs draw from one stream in order and the call stops at the first run
// that returns a pose (Tracking::Relocalization's candidate loop); otherwise the runs
// are independent and all of them complete.
orbx_status pnp_run_many(std::vector<PnpRun>& runs, bool shared, int* stopped) {
  if (runs.empty()) return ORBX_OK;
  const int device = runs[0].h->device;
  PnpDevice& dev = g_pnp_dev[device];
  hipStream_t st = dev.st;
  std::vector<PnpRun*> best_reads;
  const int nr = (int)runs.size();
  int active = 0;  // shared mode: the run whose walk is committed
  bool first_round = true;
  if (stopped) *stopped = nr;
  while (true) {
    if (shared) {
      while (active < nr && runs[active].done) {
        if (runs[active].out->found) break;
        active++;
      }
      if (active >= nr || runs[active].out->found) {
        if (stopped && active < nr) *stopped = active;
        break;
      }
    }
    // 1. hypotheses: every eligible run whose walk reached the end of its launched ones
    std::vector<std::pair<PnpRun*, int>> chunk;
    for (int i = 0; i < nr; i++) {
      PnpRun& r = runs[i];
      const bool eligible = shared ? (first_round || i == active) : true;
      if (!eligible || r.done || r.pending || r.k < r.launched || r.launched >= r.H) continue;
      // the first chunk, then everything left: a solver still without a pose after its first
      // hypotheses most often runs all of them (no set reaches minInliers), and one launch of
      // them beats a chain of doubling rounds
      const int c = r.launched == 0 ? std::min(r.H, kPnpFirstChunk) : r.H - r.launched;
      chunk.push_back({&r, c});
    }
    first_round = false;
    orbx_status s = pnp_launch_chunks(dev, st, chunk);
    if (s != ORBX_OK) return s;
    // 2. walks (shared: only the committed run)
    std::vector<PnpRun*> pend;
    for (int i = 0; i < nr; i++) {
      PnpRun& r = runs[i];
      if (r.done || (shared && i != active)) continue;
      if ((s = pnp_walk(r)) != ORBX_OK) return s;
      if (r.pending) {
        pend.push_back(&r);
      } else if (r.k >= r.H) {
        pnp_finish(r);
        if (r.read_best) best_reads.push_back(&r);
      }
    }
    // 3. the Refine() calls of this round, then the best poses of the runs that ended
    if ((s = pnp_refine_round(dev, st, pend)) != ORBX_OK) return s;
    for (PnpRun* r : pend)
      if (!r->done && r->k >= r->H) {
        pnp_finish(*r);
        if (r->read_best) best_reads.push_back(r);
      }
    if ((s = pnp_read_best(dev, st, best_reads)) != ORBX_OK) return s;
    bool all_done = true;
    for (int i = 0; i < nr; i++) all_done = all_done && runs[i].done;
    if (!shared && all_done) break;
    if (shared && all_done) {
      // fall through to the stop scan at the top
    }
  }
  // persist the best set of every solver whose best now comes from this call (the next call
  // reuses the hypothesis buffers): one gather launch
  std::vector<orbx::PnpGatherJob> keep;
  for (PnpRun& r : runs)
    if (r.best_k >= 0) {
      keep.push_back(orbx::PnpGatherJob{r.best_mask(), r.h->d_best, r.h->N});
      keep.push_back(orbx::PnpGatherJob{(const uint8_t*)r.best_pose(), (uint8_t*)(r.h->d_res + 16), 96});
      r.best_k = -1;
    }
  if (!keep.empty()) {
    const size_t bytes = keep.size() * sizeof(orbx::PnpGatherJob);
    PNP_CHECK(dev.pinned_reserve(bytes));
    PNP_CHECK(dev.dstage_reserve(bytes));
    std::memcpy(dev.pinned, keep.data(), bytes);
    PNP_CHECK(hipMemcpyAsync(dev.dstage, dev.pinned, bytes, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(orbx::k_pnp_gather, dim3((unsigned)keep.size()), dim3(256), 0, st,
                       (const orbx::PnpGatherJob*)dev.dstage);
    PNP_CHECK(hipGetLastError());
    PNP_CHECK(hipStreamSynchronize(st));
  }
  return ORBX_OK;
}

orbx_status pnp_check_solvers(orbx_pnp* const* solvers, int n, const orbx_pnp_result* results) {
  if (n < 0 || (n > 0 && (!solvers || !results))) return ORBX_ERR_ARG;
  for (int i = 0; i < n; i++) {
    if (!solvers[i]) return ORBX_ERR_ARG;
    if (solvers[i]->device != solvers[0]->device) return ORBX_ERR_ARG;
    for (int j = 0; j < i; j++)
      if (solvers[j] == solvers[i]) return ORBX_ERR_ARG;  // one walk per solver and call
  }
  return ORBX_OK;
}

}  // namespace

extern "C" {

orbx_status orbx_pnp_iterate_candidates(orbx_pnp* const* solvers, int n, int n_iterations, orbx_rand_state* rng,
                                        orbx_pnp_result* results, uint8_t* const* inliers, int* stopped) {
  orbx_status s = pnp_check_solvers(solvers, n, results);
  if (s != ORBX_OK || !rng || !stopped) return s != ORBX_OK ? s : ORBX_ERR_ARG;
  *stopped = n;
  if (n == 0) return ORBX_OK;
  if (hipSetDevice(solvers[0]->device) != hipSuccess) return ORBX_ERR_HIP;
  std::lock_guard<std::mutex> lock(g_pnp_dev[solvers[0]->device].mu);
  std::vector<PnpRun> runs(n);
  size_t total = 0;
  for (int i = 0; i < n; i++) {
    runs[i].h = solvers[i];
    runs[i].out = &results[i];
    runs[i].inliers = inliers ? inliers[i] : nullptr;
    if ((s = pnp_begin(runs[i], n_iterations)) != ORBX_OK) return s;
    total += (size_t)runs[i].H * solvers[i]->min_set;
  }
  // run i draws from where run i-1 would end without a pose (all of its hypotheses)
  orbx_rand_state peek = *rng;
  std::vector<int32_t> vals(std::max(total, (size_t)1));
  for (size_t k = 0; k < total; k++) vals[k] = orbx_rand_next(&peek);
  size_t o = 0;
  for (int i = 0; i < n; i++) {
    runs[i].rv = vals.data() + o;
    o += (size_t)runs[i].H * solvers[i]->min_set;
  }
  if ((s = pnp_run_many(runs, true, stopped)) != ORBX_OK) return s;
  for (int i = 0; i < n; i++) results[i].used = runs[i].used;
  // the reference never reaches the candidates after the one that returned a pose: their
  // results are all zero (pnp_begin above already set bNoMore for N < minInliers on them)
  for (int i = *stopped + 1; i < n; i++) std::memset(&results[i], 0, sizeof(results[i]));
  size_t used = 0;
  for (int i = 0; i < n && i <= *stopped; i++) used += runs[i].used;
  for (size_t k = 0; k < used; k++) (void)orbx_rand_next(rng);
  return ORBX_OK;
}

orbx_status orbx_pnp_iterate_many(orbx_pnp* const* solvers, int n, int n_iterations, orbx_rand_state* const* rngs,
                                  orbx_pnp_result* results, uint8_t* const* inliers) {
  orbx_status s = pnp_check_solvers(solvers, n, results);
  if (s != ORBX_OK) return s;
  if (n == 0) return ORBX_OK;
  if (!rngs) return ORBX_ERR_ARG;
  for (int i = 0; i < n; i++) {
    if (!rngs[i]) return ORBX_ERR_ARG;
    for (int j = 0; j < i; j++)
      if (rngs[j] == rngs[i]) return ORBX_ERR_ARG;  // independent streams only (shared: _candidates)
  }
  if (hipSetDevice(solvers[0]->device) != hipSuccess) return ORBX_ERR_HIP;
  std::lock_guard<std::mutex> lock(g_pnp_dev[solvers[0]->device].mu);
  std::vector<PnpRun> runs(n);
  std::vector<std::vector<int32_t>> vals(n);
  for (int i = 0; i < n; i++) {
    runs[i].h = solvers[i];
    runs[i].out = &results[i];
    runs[i].inliers = inliers ? inliers[i] : nullptr;
    if ((s = pnp_begin(runs[i], n_iterations)) != ORBX_OK) return s;
    const size_t need = (size_t)runs[i].H * solvers[i]->min_set;
    orbx_rand_state peek = *rngs[i];
    vals[i].resize(std::max(need, (size_t)1));
    for (size_t k = 0; k < need; k++) vals[i][k] = orbx_rand_next(&peek);
    runs[i].rv = vals[i].data();
  }
  if ((s = pnp_run_many(runs, false, nullptr)) != ORBX_OK) return s;
  for (int i = 0; i < n; i++) {
    results[i].used = runs[i].used;
    for (int k = 0; k < runs[i].used; k++) (void)orbx_rand_next(rngs[i]);
  }
  return ORBX_OK;
}

void orbx_rand_seed(orbx_rand_state* s, uint32_t seed) {
  // glibc __srandom_r: r[0] = seed (0 -> 1), r[i] = 16807 r[i-1] mod (2^31 - 1) (Schrage),
  // r[31..33] = r[0..2], then 310 outputs discarded
  if (!s) return;
  int32_t r[34];
  r[0] = (int32_t)(seed == 0 ? 1 : seed);
  for (int i = 1; i < 31; i++) {
    const int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
    int32_t word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[i] = word;
  }
  for (int i = 31; i < 34; i++) r[i] = r[i - 31];
  for (int i = 0; i < 34; i++) s->r[i] = (uint32_t)r[i];
  s->i = 34;
  for (int k = 0; k < 310; k++) (void)orbx_rand_next(s);
}

int32_t orbx_rand_next(orbx_rand_state* s) {
  const int i = s->i;
  const uint32_t v = s->r[(i - 31) % 34] + s->r[(i - 3) % 34];
  s->r[i % 34] = v;
  s->i = i + 1 >= 34 * 1024 ? i + 1 - 34 * 1000 : i + 1;  // keep the index bounded (multiple of 34)
  return (int32_t)(v >> 1);
}

orbx_status orbx_pnp_iterate_stream(orbx_pnp* h, int n_iterations, orbx_rand_state* rng, int* no_more, float Tcw[16],
                                    uint8_t* inliers, int* n_inliers, int* found) {
  if (!h || !rng) return ORBX_ERR_ARG;
  const int need = h->min_set * std::max(std::max(h->max_its - h->iterations, n_iterations), 0);
  orbx_rand_state peek = *rng;
  std::vector<int32_t> vals(need);
  for (int k = 0; k < need; k++) vals[k] = orbx_rand_next(&peek);
  int used = 0;
  const orbx_status st =
      orbx_pnp_iterate(h, n_iterations, vals.data(), need, &used, no_more, Tcw, inliers, n_inliers, found);
  if (st != ORBX_OK) return st;
  for (int k = 0; k < used; k++) (void)orbx_rand_next(rng);
  return ORBX_OK;
}

}  // extern "C"
