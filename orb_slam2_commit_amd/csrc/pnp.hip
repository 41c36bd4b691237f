// pnp.hip -- PnPsolver (src/PnPsolver.cc:67-1101) on the GPU: RANSAC
// hypotheses evaluated in parallel, resolved in the reference's order.
//
//   k_pnp_hyp     one thread per hypothesis: EPnP compute_pose on its
//                 minimal set (DUtils::Random::RandomInt + swap-remove
//                 sampling replayed on the host from the caller's rand()
//                 values)
//   k_pnp_check   one block per hypothesis: CheckInliers (float/double mix
//                 exactly as :352-384) -> inlier bytes + count
//   k_pnp_refine  one block: Refine() (:303-349) = EPnP on every inlier of
//                 the best hypothesis + CheckInliers
// The host walks hypotheses in order (best = first strict maximum, Refine at
// each hypothesis reaching minInliers, return on the first successful
// Refine), which is iterate() (:182-301) including its
// `mnIterations<maxIts || nCurrent<nIterations` loop condition.
//
// EPnP and the OpenCV 3.2 helpers it calls (cvMulTransposed, Jacobi cvSVD,
// cvInvert/cvSolve through SVBkSb) use only IEEE + - * / sqrt in the same
// order as the oracle, with every reduction sequential in the reference's
// order, so poses and masks are bit-identical to the CPU restatement.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
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

// JacobiSVDImpl_<double> (see oracle/pnp.cpp): n rows of length m in At.
__device__ void jacobi_svd(double* At, int astep, double* Wout, double* Vt, int vstep, int m, int n, int n1) {
  const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
  double W[16];
  const int max_iter = m > 30 ? m : 30;
  for (int i = 0; i < n; i++) {
    double sd = 0;
    for (int k = 0; k < m; k++) {
      const double t = At[i * astep + k];
      sd += t * t;
    }
    W[i] = sd;
    for (int k = 0; k < n; k++) Vt[i * vstep + k] = 0;
    Vt[i * vstep + i] = 1;
  }
  for (int iter = 0; iter < max_iter; iter++) {
    bool changed = false;
    for (int i = 0; i < n - 1; i++)
      for (int j = i + 1; j < n; j++) {
        double* Ai = At + i * astep;
        double* Aj = At + j * astep;
        double a = W[i], p = 0, b = W[j];
        for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
        if (fabs(p) <= eps * sqrt(a * b)) continue;
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
        for (int k = 0; k < m; k++) {
          const double t0 = c * Ai[k] + s * Aj[k];
          const double t1 = -s * Ai[k] + c * Aj[k];
          Ai[k] = t0;
          Aj[k] = t1;
          a += t0 * t0;
          b += t1 * t1;
        }
        W[i] = a;
        W[j] = b;
        changed = true;
        double* Vi = Vt + i * vstep;
        double* Vj = Vt + j * vstep;
        for (int k = 0; k < n; k++) {
          const double t0 = c * Vi[k] + s * Vj[k];
          const double t1 = -s * Vi[k] + c * Vj[k];
          Vi[k] = t0;
          Vj[k] = t1;
        }
      }
    if (!changed) break;
  }
  for (int i = 0; i < n; i++) {
    double sd = 0;
    for (int k = 0; k < m; k++) {
      const double t = At[i * astep + k];
      sd += t * t;
    }
    W[i] = sqrt(sd);
  }
  for (int i = 0; i < n - 1; i++) {
    int j = i;
    for (int k = i + 1; k < n; k++)
      if (W[j] < W[k]) j = k;
    if (i != j) {
      swap_d(W[i], W[j]);
      for (int k = 0; k < m; k++) swap_d(At[i * astep + k], At[j * astep + k]);
      for (int k = 0; k < n; k++) swap_d(Vt[i * vstep + k], Vt[j * vstep + k]);
    }
  }
  for (int i = 0; i < n; i++) Wout[i] = W[i];
  CvRng rng{0x12345678};
  for (int i = 0; i < n1; i++) {
    double sd = i < n ? W[i] : 0;
    for (int ii = 0; ii < 100 && sd <= minval; ii++) {
      const double val0 = 1. / m;
      for (int k = 0; k < m; k++) At[i * astep + k] = (rng.next() & 256) != 0 ? val0 : -val0;
      for (int iter = 0; iter < 2; iter++)
        for (int j = 0; j < i; j++) {
          sd = 0;
          for (int k = 0; k < m; k++) sd += At[i * astep + k] * At[j * astep + k];
          double asum = 0;
          for (int k = 0; k < m; k++) {
            const double t = At[i * astep + k] - sd * At[j * astep + k];
            At[i * astep + k] = t;
            asum += fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
          for (int k = 0; k < m; k++) At[i * astep + k] *= asum;
        }
      sd = 0;
      for (int k = 0; k < m; k++) {
        const double t = At[i * astep + k];
        sd += t * t;
      }
      sd = sqrt(sd);
    }
    const double s = sd > minval ? 1 / sd : 0.;
    for (int k = 0; k < m; k++) At[i * astep + k] *= s;
  }
}

// _SVDcompute, m >= n: left singular vectors as rows Ut (n x m), w, Vt.
__device__ void svd_rows(const double* A, int m, int n, double* Ut, double* w, double* Vt) {
  for (int i = 0; i < n; i++)
    for (int k = 0; k < m; k++) Ut[i * m + k] = A[k * n + i];
  jacobi_svd(Ut, m, w, Vt, n, m, n, n);
}

// SVBkSbImpl_ (b == nullptr: inverse)
__device__ void svd_backsubst(const double* Ut, const double* w, const double* Vt, int m, int n, const double* b,
                              double* x) {
  const int nb = b ? 1 : m;
  for (int i = 0; i < n * nb; i++) x[i] = 0;
  double threshold = 0;
  for (int i = 0; i < n; i++) threshold += w[i];
  threshold *= DBL_EPSILON * 2;
  double buffer[16];
  for (int i = 0; i < n; i++) {
    double wi = w[i];
    if (fabs(wi) <= threshold) continue;
    wi = 1 / wi;
    const double* u = Ut + i * m;
    const double* v = Vt + i * n;
    if (nb == 1) {
      double s = 0;
      for (int j = 0; j < m; j++) s += u[j] * b[j];
      s *= wi;
      for (int j = 0; j < n; j++) x[j] = x[j] + s * v[j];
    } else {
      for (int j = 0; j < nb; j++) buffer[j] = u[j] * wi;
      for (int j = 0; j < n; j++)
        for (int k = 0; k < nb; k++) x[j * nb + k] += buffer[k] * v[j];
    }
  }
}

__device__ inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ inline double dist2(const double* p1, const double* p2) {
  return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

// find_betas_approx_{1,2,3}, compute_L_6x10, compute_rho, gauss_newton, qr_solve
__device__ void solve6(const double* L, int k, const double* rho, double* x) {
  double ut[6 * 5], w[5], vt[25];
  svd_rows(L, 6, k, ut, w, vt);
  svd_backsubst(ut, w, vt, 6, k, rho, x);
}

__device__ void find_betas_approx_1(const double* l_6x10, const double* rho, double* betas) {
  double l_6x4[24], b4[4];
  for (int i = 0; i < 6; i++) {
    l_6x4[4 * i] = l_6x10[10 * i];
    l_6x4[4 * i + 1] = l_6x10[10 * i + 1];
    l_6x4[4 * i + 2] = l_6x10[10 * i + 3];
    l_6x4[4 * i + 3] = l_6x10[10 * i + 6];
  }
  solve6(l_6x4, 4, rho, b4);
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

__device__ void find_betas_approx_2(const double* l_6x10, const double* rho, double* betas) {
  double l_6x3[18], b3[3];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 3; j++) l_6x3[3 * i + j] = l_6x10[10 * i + j];
  solve6(l_6x3, 3, rho, b3);
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

__device__ void find_betas_approx_3(const double* l_6x10, const double* rho, double* betas) {
  double l_6x5[30], b5[5];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 5; j++) l_6x5[5 * i + j] = l_6x10[10 * i + j];
  solve6(l_6x5, 5, rho, b5);
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

__device__ void compute_L_6x10(const double* ut, double* l_6x10) {
  const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
  double dv[4][6][3];
  for (int i = 0; i < 4; i++) {
    int a = 0, b = 1;
    for (int j = 0; j < 6; j++) {
      dv[i][j][0] = v[i][3 * a] - v[i][3 * b];
      dv[i][j][1] = v[i][3 * a + 1] - v[i][3 * b + 1];
      dv[i][j][2] = v[i][3 * a + 2] - v[i][3 * b + 2];
      b++;
      if (b > 3) {
        a++;
        b = a + 1;
      }
    }
  }
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

__device__ void qr_solve(double* A, double* b, double* X) {
  const int nr = 6, nc = 4;
  double A1[6], A2[6];
  double* pA = A;
  double* ppAkk = pA;
  for (int k = 0; k < nc; k++) {
    double* ppAik = ppAkk;
    double eta = fabs(*ppAik);
    for (int i = k + 1; i < nr; i++) {
      const double elt = fabs(*ppAik);
      if (eta < elt) eta = elt;
      ppAik += nc;
    }
    if (eta == 0) return;
    double sum = 0.0;
    const double inv_eta = 1. / eta;
    ppAik = ppAkk;
    for (int i = k; i < nr; i++) {
      *ppAik *= inv_eta;
      sum += *ppAik * *ppAik;
      ppAik += nc;
    }
    double sigma = sqrt(sum);
    if (*ppAkk < 0) sigma = -sigma;
    *ppAkk += sigma;
    A1[k] = sigma * *ppAkk;
    A2[k] = -eta * sigma;
    for (int j = k + 1; j < nc; j++) {
      double* p = ppAkk;
      double s = 0;
      for (int i = k; i < nr; i++) {
        s += *p * p[j - k];
        p += nc;
      }
      const double tau = s / A1[k];
      p = ppAkk;
      for (int i = k; i < nr; i++) {
        p[j - k] -= tau * *p;
        p += nc;
      }
    }
    ppAkk += nc + 1;
  }
  double* ppAjj = pA;
  for (int j = 0; j < nc; j++) {
    double* ppAij = ppAjj;
    double tau = 0;
    for (int i = j; i < nr; i++) {
      tau += *ppAij * b[i];
      ppAij += nc;
    }
    tau /= A1[j];
    ppAij = ppAjj;
    for (int i = j; i < nr; i++) {
      b[i] -= tau * *ppAij;
      ppAij += nc;
    }
    ppAjj += nc + 1;
  }
  X[nc - 1] = b[nc - 1] / A2[nc - 1];
  for (int i = nc - 2; i >= 0; i--) {
    double* ppAij = pA + i * nc + (i + 1);
    double s = 0;
    for (int j = i + 1; j < nc; j++) {
      s += *ppAij * X[j];
      ppAij++;
    }
    X[i] = (b[i] - s) / A2[i];
  }
}

__device__ void gauss_newton(const double* l_6x10, const double* rho, double betas[4]) {
  double a[24], b[6], x[4] = {0, 0, 0, 0};
  for (int k = 0; k < 5; k++) {
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
    for (int i = 0; i < 4; i++) betas[i] += x[i];
  }
}

// ------------------------------------------------------------ EPnP on a group
// Group = one thread (hypotheses) or one block (Refine).  Per-point work is
// spread over the group; every reduction runs on one thread in point order.
struct GroupThread {
  __device__ int tid() const { return 0; }
  __device__ int nt() const { return 1; }
  __device__ void sync() const {}
};
struct GroupBlock {
  __device__ int tid() const { return threadIdx.x; }
  __device__ int nt() const { return blockDim.x; }
  __device__ void sync() const { __syncthreads(); }
};

struct EpnpSmall {
  double cws[4][3], ccs[4][3], ci[9], pw0tpw0[9], mtm[144], ut[144], vt[144], d[12];
  double l_6x10[60], rho[6], betas[4][4], rep[4], Rs[4][3][3], ts[4][3];
  double pc0[3], pw0[3], abt[9];
  int flip;
};

struct EpnpWork {  // per-correspondence arrays (n entries)
  double* alphas;  // 4n
  double* pcs;     // 3n
  double* M;       // 24n
  double* tmp;     // n
};

template <class G>
__device__ void epnp_compute_pose(const G& g, const PnpIn& in, const int* idx, int n, EpnpSmall* S, EpnpWork W) {
  const int tid = g.tid(), nt = g.nt();
  auto pw = [&](int k, int j) { return (double)in.p3d[3 * idx[k] + j]; };
  auto uv = [&](int k, int j) { return (double)in.p2d[2 * idx[k] + j]; };
  // choose_control_points
  if (tid == 0) {
    S->cws[0][0] = S->cws[0][1] = S->cws[0][2] = 0;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) S->cws[0][j] += pw(i, j);
    for (int j = 0; j < 3; j++) S->cws[0][j] /= n;
  }
  g.sync();
  for (int e = tid; e < 6; e += nt) {
    const int i = e < 3 ? 0 : (e < 5 ? 1 : 2), j = e < 3 ? e : (e < 5 ? e - 2 : 2);
    double s = 0;
    for (int k = 0; k < n; k++) s += (pw(k, i) - S->cws[0][i]) * (pw(k, j) - S->cws[0][j]);
    S->pw0tpw0[3 * i + j] = s;
  }
  g.sync();
  if (tid == 0) {
    double* P = S->pw0tpw0;
    P[3] = P[1];
    P[6] = P[2];
    P[7] = P[5];
    double uct[9], dc[3], vt[9];
    svd_rows(P, 3, 3, uct, dc, vt);
    for (int i = 1; i < 4; i++) {
      const double k = sqrt(dc[i - 1] / n);
      for (int j = 0; j < 3; j++) S->cws[i][j] = S->cws[0][j] + k * uct[3 * (i - 1) + j];
    }
    double cc[9], ut[9], w[3];
    for (int i = 0; i < 3; i++)
      for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = S->cws[j][i] - S->cws[0][i];
    svd_rows(cc, 3, 3, ut, w, vt);
    svd_backsubst(ut, w, vt, 3, 3, nullptr, S->ci);
  }
  g.sync();
  // compute_barycentric_coordinates + fill_M
  for (int i = tid; i < n; i += nt) {
    double* a = W.alphas + 4 * i;
    const double* ci = S->ci;
    const double p0 = pw(i, 0), p1 = pw(i, 1), p2 = pw(i, 2);
    for (int j = 0; j < 3; j++)
      a[1 + j] = ci[3 * j] * (p0 - S->cws[0][0]) + ci[3 * j + 1] * (p1 - S->cws[0][1]) + ci[3 * j + 2] * (p2 - S->cws[0][2]);
    a[0] = 1.0f - a[1] - a[2] - a[3];
    double* M1 = W.M + 24 * i;
    double* M2 = M1 + 12;
    const double u = uv(i, 0), v = uv(i, 1);
    for (int q = 0; q < 4; q++) {
      M1[3 * q] = a[q] * in.fu;
      M1[3 * q + 1] = 0.0;
      M1[3 * q + 2] = a[q] * (in.uc - u);
      M2[3 * q] = 0.0;
      M2[3 * q + 1] = a[q] * in.fv;
      M2[3 * q + 2] = a[q] * (in.vc - v);
    }
  }
  g.sync();
  // MtM = M^T M (upper triangle sums over rows in order), mirrored
  for (int e = tid; e < 78; e += nt) {
    int i = 0, r = e;
    while (r >= 12 - i) {
      r -= 12 - i;
      i++;
    }
    const int j = i + r;
    double s = 0;
    for (int k = 0; k < 2 * n; k++) s += W.M[12 * k + i] * W.M[12 * k + j];
    S->mtm[12 * i + j] = s;
  }
  g.sync();
  if (tid == 0) {
    for (int i = 0; i < 12; i++)
      for (int j = 0; j < i; j++) S->mtm[12 * i + j] = S->mtm[12 * j + i];
    svd_rows(S->mtm, 12, 12, S->ut, S->d, S->vt);
    compute_L_6x10(S->ut, S->l_6x10);
    S->rho[0] = dist2(S->cws[0], S->cws[1]);
    S->rho[1] = dist2(S->cws[0], S->cws[2]);
    S->rho[2] = dist2(S->cws[0], S->cws[3]);
    S->rho[3] = dist2(S->cws[1], S->cws[2]);
    S->rho[4] = dist2(S->cws[1], S->cws[3]);
    S->rho[5] = dist2(S->cws[2], S->cws[3]);
  }
  g.sync();
  for (int ap = 1; ap <= 3; ap++) {
    if (tid == 0) {
      double* betas = S->betas[ap];
      if (ap == 1) find_betas_approx_1(S->l_6x10, S->rho, betas);
      if (ap == 2) find_betas_approx_2(S->l_6x10, S->rho, betas);
      if (ap == 3) find_betas_approx_3(S->l_6x10, S->rho, betas);
      gauss_newton(S->l_6x10, S->rho, betas);
      // compute_ccs
      for (int i = 0; i < 4; i++) S->ccs[i][0] = S->ccs[i][1] = S->ccs[i][2] = 0.0f;
      for (int i = 0; i < 4; i++) {
        const double* v = S->ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
          for (int k = 0; k < 3; k++) S->ccs[j][k] += betas[i] * v[3 * j + k];
      }
    }
    g.sync();
    for (int i = tid; i < n; i += nt) {  // compute_pcs
      const double* a = W.alphas + 4 * i;
      double* pc = W.pcs + 3 * i;
      for (int j = 0; j < 3; j++)
        pc[j] = a[0] * S->ccs[0][j] + a[1] * S->ccs[1][j] + a[2] * S->ccs[2][j] + a[3] * S->ccs[3][j];
    }
    g.sync();
    if (tid == 0) S->flip = W.pcs[2] < 0.0;  // solve_for_sign
    g.sync();
    if (S->flip) {
      for (int i = tid; i < n; i += nt) {
        W.pcs[3 * i] = -W.pcs[3 * i];
        W.pcs[3 * i + 1] = -W.pcs[3 * i + 1];
        W.pcs[3 * i + 2] = -W.pcs[3 * i + 2];
      }
      if (tid == 0)
        for (int i = 0; i < 4; i++)
          for (int j = 0; j < 3; j++) S->ccs[i][j] = -S->ccs[i][j];
    }
    g.sync();
    // estimate_R_and_t: centroid sums, then ABt sums, in point order
    for (int e = tid; e < 6; e += nt) {
      double s = 0;
      for (int i = 0; i < n; i++) s += e < 3 ? W.pcs[3 * i + e] : pw(i, e - 3);
      if (e < 3)
        S->pc0[e] = s / n;
      else
        S->pw0[e - 3] = s / n;
    }
    g.sync();
    for (int e = tid; e < 9; e += nt) {
      const int j = e / 3, c = e % 3;
      double s = 0;
      for (int i = 0; i < n; i++) s += (W.pcs[3 * i + j] - S->pc0[j]) * (pw(i, c) - S->pw0[c]);
      S->abt[e] = s;
    }
    g.sync();
    if (tid == 0) {
      double ut[9], w[3], vt[9], U[9], V[9];
      svd_rows(S->abt, 3, 3, ut, w, vt);
      for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) {
          U[3 * i + k] = ut[3 * k + i];
          V[3 * i + k] = vt[3 * k + i];
        }
      double(*R)[3] = S->Rs[ap];
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = dot3(U + 3 * i, V + 3 * j);
      const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                         R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
      if (det < 0) {
        R[2][0] = -R[2][0];
        R[2][1] = -R[2][1];
        R[2][2] = -R[2][2];
      }
      for (int r = 0; r < 3; r++) S->ts[ap][r] = S->pc0[r] - dot3(R[r], S->pw0);
    }
    g.sync();
    for (int i = tid; i < n; i += nt) {  // reprojection_error terms
      const double(*R)[3] = S->Rs[ap];
      const double* t = S->ts[ap];
      const double p[3] = {pw(i, 0), pw(i, 1), pw(i, 2)};
      const double Xc = dot3(R[0], p) + t[0];
      const double Yc = dot3(R[1], p) + t[1];
      const double inv_Zc = 1.0 / (dot3(R[2], p) + t[2]);
      const double ue = in.uc + in.fu * Xc * inv_Zc;
      const double ve = in.vc + in.fv * Yc * inv_Zc;
      const double u = uv(i, 0), v = uv(i, 1);
      W.tmp[i] = sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    g.sync();
    if (tid == 0) {
      double sum2 = 0.0;
      for (int i = 0; i < n; i++) sum2 += W.tmp[i];
      S->rep[ap] = sum2 / n;
    }
    g.sync();
  }
  if (tid == 0) {
    int N = 1;
    if (S->rep[2] < S->rep[1]) N = 2;
    if (S->rep[3] < S->rep[N]) N = 3;
    S->rep[0] = (double)N;
  }
  g.sync();
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
// pose record per hypothesis: R (9, row-major) + t (3)
__global__ __launch_bounds__(64) void k_pnp_hyp(PnpIn in, const int* __restrict__ sets, int set_size, int n_hyp,
                                                double* __restrict__ poses, double* __restrict__ work) {
  const int h = blockIdx.x * 64 + threadIdx.x;
  if (h >= n_hyp) return;
  EpnpSmall S;
  double* w = work + (size_t)h * (32 * kPnpMaxSet);
  EpnpWork W{w, w + 4 * kPnpMaxSet, w + 7 * kPnpMaxSet, w + 31 * kPnpMaxSet};
  epnp_compute_pose(GroupThread{}, in, sets + (size_t)h * set_size, set_size, &S, W);
  const int b = (int)S.rep[0];
  double* P = poses + 12 * (size_t)h;
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) P[3 * i + j] = S.Rs[b][i][j];
    P[9 + i] = S.ts[b][i];
  }
}

__global__ __launch_bounds__(256) void k_pnp_check(PnpIn in, const double* __restrict__ poses,
                                                   uint8_t* __restrict__ masks, int* __restrict__ counts) {
  __shared__ int red[4];
  const int h = blockIdx.x;
  const double* P = poses + 12 * (size_t)h;
  double R[9], t[3];
  for (int i = 0; i < 9; i++) R[i] = P[i];
  for (int i = 0; i < 3; i++) t[i] = P[9 + i];
  int c = 0;
  uint8_t* m = masks + (size_t)h * in.N;
  for (int i = threadIdx.x; i < in.N; i += 256) {
    const bool ok = check_inlier(in, R, t, i);
    m[i] = ok;
    c += ok;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[h] = red[0] + red[1] + red[2] + red[3];
}

// Refine(): EPnP on the inliers of `best` (ascending index), then CheckInliers.
// out: [0..8] R, [9..11] t; *count; mask_out.
__global__ __launch_bounds__(256) void k_pnp_refine(PnpIn in, const uint8_t* __restrict__ best, int* __restrict__ idx,
                                                    double* __restrict__ work, double* __restrict__ out,
                                                    uint8_t* __restrict__ mask_out, int* __restrict__ count) {
  __shared__ EpnpSmall S;
  __shared__ int wsum[4], base;
  const int tid = threadIdx.x;
  // ordered compaction of the best inlier set
  if (tid == 0) base = 0;
  __syncthreads();
  for (int i0 = 0; i0 < in.N; i0 += 256) {
    const int i = i0 + tid;
    const int f = (i < in.N && best[i]) ? 1 : 0;
    const unsigned long long bal = __ballot(f);
    const int lane = tid & 63, wv = tid >> 6;
    const int pre = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wv; w++) off += wsum[w];
    if (f) idx[off + pre] = i;
    __syncthreads();
    if (tid == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  const int n = base;
  EpnpWork W{work, work + 4 * (size_t)in.N, work + 7 * (size_t)in.N, work + 31 * (size_t)in.N};
  epnp_compute_pose(GroupBlock{}, in, idx, n, &S, W);
  const int b = (int)S.rep[0];
  double R[9], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[3 * i + j] = S.Rs[b][i][j];
    t[i] = S.ts[b][i];
  }
  int c = 0;
  for (int i = tid; i < in.N; i += 256) {
    const bool ok = check_inlier(in, R, t, i);
    mask_out[i] = ok;
    c += ok;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) wsum[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) {
    *count = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    for (int i = 0; i < 9; i++) out[i] = R[i];
    for (int i = 0; i < 3; i++) out[9 + i] = t[i];
  }
}

}  // namespace orbx

// ------------------------------------------------------------------ host / C ABI
struct orbx_pnp {
  int device = 0;
  hipStream_t st = nullptr;
  int N = 0;
  double fu, fv, uc, vc;
  double prob;
  int min_inliers, max_its, min_set;
  float epsilon;
  // device: correspondences, per-hypothesis buffers, refine buffers
  float *d_p3d = nullptr, *d_p2d = nullptr, *d_maxerr = nullptr;
  int* d_sets = nullptr;
  double* d_poses = nullptr;
  double* d_hwork = nullptr;
  uint8_t* d_masks = nullptr;
  int* d_counts = nullptr;
  uint8_t *d_best = nullptr, *d_refmask = nullptr;
  int* d_idx = nullptr;
  double* d_rwork = nullptr;
  double* d_rout = nullptr;
  int* d_rcount = nullptr;
  int cap_hyp = 0;
  // iterate() state
  int iterations = 0, best_inliers = 0;
  float best_Tcw[16];
  bool refine_valid = false;  // Refine() of the current best set already known to fail
  orbx::PnpIn in() const {
    return orbx::PnpIn{d_p3d, d_p2d, d_maxerr, N, fu, fv, uc, vc};
  }
};

namespace {

void free_pnp(orbx_pnp* h) {
  void* ptrs[] = {h->d_p3d,  h->d_p2d,     h->d_maxerr, h->d_sets,  h->d_poses, h->d_hwork, h->d_masks,
                  h->d_counts, h->d_best, h->d_refmask, h->d_idx,   h->d_rwork, h->d_rout,  h->d_rcount};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
}

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

orbx_status orbx_pnp_create(const orbx_pnp_problem* p, const orbx_pnp_params* prm, int device, orbx_pnp** out) {
  if (!p || !prm || !out || p->n < 0 || (p->n > 0 && (!p->p3d || !p->p2d || !p->sigma2))) return ORBX_ERR_ARG;
  if (prm->min_set < 1 || prm->min_set > orbx::kPnpMaxSet) return ORBX_ERR_ARG;
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= nd) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  orbx_pnp* h = new (std::nothrow) orbx_pnp();
  if (!h) return ORBX_ERR_HIP;
  h->device = device;
  const int n = p->n;
  h->N = n;
  h->fu = p->fx;
  h->fv = p->fy;
  h->uc = p->cx;
  h->vc = p->cy;
  // SetRansacParameters (src/PnPsolver.cc:136-179)
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
  std::vector<float> maxerr(n);
  for (int i = 0; i < n; i++) maxerr[i] = p->sigma2[i] * prm->th2;
  const size_t nn = std::max(n, 1);
  hipError_t e = hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_p3d, 12 * nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_p2d, 8 * nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_maxerr, 4 * nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_best, nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_refmask, nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_idx, 4 * nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_rwork, 32 * 8 * nn);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_rout, 12 * 8);
  if (e == hipSuccess) e = hipMalloc((void**)&h->d_rcount, 4);
  if (e == hipSuccess && n > 0) e = hipMemcpy(h->d_p3d, p->p3d, 12 * (size_t)n, hipMemcpyHostToDevice);
  if (e == hipSuccess && n > 0) e = hipMemcpy(h->d_p2d, p->p2d, 8 * (size_t)n, hipMemcpyHostToDevice);
  if (e == hipSuccess && n > 0) e = hipMemcpy(h->d_maxerr, maxerr.data(), 4 * (size_t)n, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_pnp(h);
    if (h->st) (void)hipStreamDestroy(h->st);
    delete h;
    return ORBX_ERR_HIP;
  }
  for (int i = 0; i < 16; i++) h->best_Tcw[i] = 0;
  *out = h;
  return ORBX_OK;
}

orbx_status orbx_pnp_destroy(orbx_pnp* h) {
  if (!h) return ORBX_ERR_ARG;
  (void)hipSetDevice(h->device);
  free_pnp(h);
  if (h->st) (void)hipStreamDestroy(h->st);
  delete h;
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
  // DUtils::Random::RandomInt(0, size-1) on the rand() stream + swap-remove
  std::vector<int> sets((size_t)H * ms), avail(N);
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
  if (H > h->cap_hyp) {
    if (h->d_sets) (void)hipFree(h->d_sets);
    if (h->d_poses) (void)hipFree(h->d_poses);
    if (h->d_hwork) (void)hipFree(h->d_hwork);
    if (h->d_masks) (void)hipFree(h->d_masks);
    if (h->d_counts) (void)hipFree(h->d_counts);
    h->d_sets = nullptr;
    h->d_poses = h->d_hwork = nullptr;
    h->d_masks = nullptr;
    h->d_counts = nullptr;
    h->cap_hyp = 0;
    PNP_CHECK(hipMalloc((void**)&h->d_sets, sizeof(int) * (size_t)H * orbx::kPnpMaxSet));
    PNP_CHECK(hipMalloc((void**)&h->d_poses, sizeof(double) * 12 * (size_t)H));
    PNP_CHECK(hipMalloc((void**)&h->d_hwork, sizeof(double) * 32 * orbx::kPnpMaxSet * (size_t)H));
    PNP_CHECK(hipMalloc((void**)&h->d_masks, (size_t)H * std::max(N, 1)));
    PNP_CHECK(hipMalloc((void**)&h->d_counts, sizeof(int) * (size_t)H));
    h->cap_hyp = H;
  }
  hipStream_t st = h->st;
  PNP_CHECK(hipMemcpyAsync(h->d_sets, sets.data(), sizeof(int) * sets.size(), hipMemcpyHostToDevice, st));
  const orbx::PnpIn in = h->in();
  hipLaunchKernelGGL(orbx::k_pnp_hyp, dim3((H + 63) / 64), dim3(64), 0, st, in, h->d_sets, ms, H, h->d_poses,
                     h->d_hwork);
  hipLaunchKernelGGL(orbx::k_pnp_check, dim3(H), dim3(256), 0, st, in, h->d_poses, h->d_masks, h->d_counts);
  PNP_CHECK(hipGetLastError());
  std::vector<int> counts(H);
  PNP_CHECK(hipMemcpyAsync(counts.data(), h->d_counts, sizeof(int) * H, hipMemcpyDeviceToHost, st));
  PNP_CHECK(hipStreamSynchronize(st));
  int cur = 0;
  for (int k = 0; k < H && (h->iterations < h->max_its || cur < n_iterations); k++) {
    cur++;
    h->iterations++;
    *used += ms;
    if (counts[k] < h->min_inliers) continue;
    if (counts[k] > h->best_inliers) {
      h->best_inliers = counts[k];
      PNP_CHECK(hipMemcpyAsync(h->d_best, h->d_masks + (size_t)k * N, N, hipMemcpyDeviceToDevice, st));
      double P[12];
      PNP_CHECK(hipMemcpyAsync(P, h->d_poses + 12 * (size_t)k, sizeof(P), hipMemcpyDeviceToHost, st));
      PNP_CHECK(hipStreamSynchronize(st));
      pose_to_Tcw(P, h->best_Tcw);
      h->refine_valid = false;
    }
    if (h->refine_valid) continue;  // same best set: Refine() fails again
    hipLaunchKernelGGL(orbx::k_pnp_refine, dim3(1), dim3(256), 0, st, in, h->d_best, h->d_idx, h->d_rwork,
                       h->d_rout, h->d_refmask, h->d_rcount);
    PNP_CHECK(hipGetLastError());
    int rc = 0;
    double P[12];
    PNP_CHECK(hipMemcpyAsync(&rc, h->d_rcount, sizeof(int), hipMemcpyDeviceToHost, st));
    PNP_CHECK(hipMemcpyAsync(P, h->d_rout, sizeof(P), hipMemcpyDeviceToHost, st));
    PNP_CHECK(hipStreamSynchronize(st));
    if (rc > h->min_inliers) {
      PNP_CHECK(hipMemcpy(inliers, h->d_refmask, N, hipMemcpyDeviceToHost));
      pose_to_Tcw(P, Tcw);
      *n_inliers = rc;
      *found = 1;
      return ORBX_OK;
    }
    h->refine_valid = true;
  }
  if (h->iterations >= h->max_its) {
    *no_more = 1;
    if (h->best_inliers >= h->min_inliers) {
      PNP_CHECK(hipMemcpy(inliers, h->d_best, N, hipMemcpyDeviceToHost));
      std::memcpy(Tcw, h->best_Tcw, sizeof(float) * 16);
      *n_inliers = h->best_inliers;
      *found = 1;
    }
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
