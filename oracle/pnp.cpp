// pnp.cpp -- CPU ORACLE (test infrastructure only) for PnPsolver
// (src/PnPsolver.cc:67-1101): SetRansacParameters, iterate() RANSAC with
// DUtils::Random::RandomInt over caller-supplied rand() values, EPnP
// compute_pose, CheckInliers and Refine.
//
// The OpenCV 3.2 calls EPnP makes (cvMulTransposed, cvSVD, cvInvert(CV_SVD),
// cvSolve(CV_SVD)) are restated from OpenCV 3.2 modules/core (matmul.cpp
// MulTransposedR, lapack.cpp JacobiSVDImpl_/SVBkSbImpl_/_SVDcompute) on the
// generic (non-SIMD) path.  One deliberate deviation: std::hypot(p, beta) in
// the Jacobi rotation is written sqrt(p*p + beta*beta), so that every
// operation is an IEEE basic op (+ - * / sqrt) that the GPU reproduces
// bit-for-bit.  OpenCV itself is not in the container: parity against the
// genuine library is unpinned.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "orb_oracle.h"

namespace {

// cv::RNG (core.hpp): state = (uint64)(unsigned)state * 4164903690 + (state >> 32)
struct CvRng {
  uint64_t state;
  unsigned next() {
    state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
    return (unsigned)state;
  }
};

// JacobiSVDImpl_<double> (lapack.cpp): At holds n rows of length m; on exit its
// first n1 rows are the left singular vectors (sorted by descending W), Vt the
// right ones.  minval = DBL_MIN, eps = 10 * DBL_EPSILON.
void jacobi_svd(double* At, int astep, double* Wout, double* Vt, int vstep, int m, int n, int n1) {
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
    if (Vt) {
      for (int k = 0; k < n; k++) Vt[i * vstep + k] = 0;
      Vt[i * vstep + i] = 1;
    }
  }
  for (int iter = 0; iter < max_iter; iter++) {
    bool changed = false;
    for (int i = 0; i < n - 1; i++)
      for (int j = i + 1; j < n; j++) {
        double* Ai = At + i * astep;
        double* Aj = At + j * astep;
        double a = W[i], p = 0, b = W[j];
        for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
        if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
        p *= 2;
        const double beta = a - b, gamma = std::sqrt(p * p + beta * beta);
        double c, s;
        if (beta < 0) {
          const double delta = (gamma - beta) * 0.5;
          s = std::sqrt(delta / gamma);
          c = p / (gamma * s * 2);
        } else {
          c = std::sqrt((gamma + beta) / (gamma * 2));
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
        if (Vt) {
          double* Vi = Vt + i * vstep;
          double* Vj = Vt + j * vstep;
          for (int k = 0; k < n; k++) {
            const double t0 = c * Vi[k] + s * Vj[k];
            const double t1 = -s * Vi[k] + c * Vj[k];
            Vi[k] = t0;
            Vj[k] = t1;
          }
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
    W[i] = std::sqrt(sd);
  }
  for (int i = 0; i < n - 1; i++) {
    int j = i;
    for (int k = i + 1; k < n; k++)
      if (W[j] < W[k]) j = k;
    if (i != j) {
      std::swap(W[i], W[j]);
      if (Vt) {
        for (int k = 0; k < m; k++) std::swap(At[i * astep + k], At[j * astep + k]);
        for (int k = 0; k < n; k++) std::swap(Vt[i * vstep + k], Vt[j * vstep + k]);
      }
    }
  }
  for (int i = 0; i < n; i++) Wout[i] = W[i];
  if (!Vt) return;
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
            asum += std::fabs(t);
          }
          asum = asum > eps * 100 ? 1 / asum : 0;
          for (int k = 0; k < m; k++) At[i * astep + k] *= asum;
        }
      sd = 0;
      for (int k = 0; k < m; k++) {
        const double t = At[i * astep + k];
        sd += t * t;
      }
      sd = std::sqrt(sd);
    }
    const double s = sd > minval ? 1 / sd : 0.;
    for (int k = 0; k < m; k++) At[i * astep + k] *= s;
  }
}

// _SVDcompute for an m x n row-major A with m >= n (never transposed here):
// temp_a = A^T (n rows of length m), Jacobi with n1 = n; outputs the left
// singular vectors as ROWS (U^T, n x m), w (n), and Vt (n x n).
void svd_rows(const double* A, int m, int n, double* Ut, double* w, double* Vt) {
  for (int i = 0; i < n; i++)
    for (int k = 0; k < m; k++) Ut[i * m + k] = A[k * n + i];
  jacobi_svd(Ut, m, w, Vt, n, m, n, n);
}

// SVBkSbImpl_ with u given as rows Ut (n x m), vt rows (n x n), w (n):
// x = sum_i [|w_i| > thr] (1/w_i) (u_i . b) v_i, thr = 2 DBL_EPSILON sum w.
// b == nullptr: the inverse (nb = m columns of the identity).
void svd_backsubst(const double* Ut, const double* w, const double* Vt, int m, int n, const double* b, double* x) {
  const int nb = b ? 1 : m;
  for (int i = 0; i < n * nb; i++) x[i] = 0;
  double threshold = 0;
  for (int i = 0; i < n; i++) threshold += w[i];
  threshold *= DBL_EPSILON * 2;
  double buffer[16];
  for (int i = 0; i < n; i++) {
    double wi = w[i];
    if (std::fabs(wi) <= threshold) continue;
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
      for (int j = 0; j < n; j++)  // MatrAXPY(n, nb, buffer, 0, v, 1, x, nb)
        for (int k = 0; k < nb; k++) x[j * nb + k] += buffer[k] * v[j];
    }
  }
}

// cvMulTransposed(src, dst, order=1): dst = src^T src, upper triangle by
// column sums over rows in ascending order, mirrored (MulTransposedR).
void mul_transposed(const double* src, int rows, int cols, double* dst) {
  for (int i = 0; i < cols; i++)
    for (int j = i; j < cols; j++) {
      double s = 0;
      for (int k = 0; k < rows; k++) s += src[k * cols + i] * src[k * cols + j];
      dst[i * cols + j] = s;
    }
  for (int i = 0; i < cols; i++)
    for (int j = 0; j < i; j++) dst[i * cols + j] = dst[j * cols + i];
}

double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
double dist2(const double* p1, const double* p2) {
  return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

// EPnP of the reference (src/PnPsolver.cc:426-1050) on n correspondences.
struct Epnp {
  double fu, fv, uc, vc;
  int n = 0;
  std::vector<double> pws, us, alphas, pcs;
  double cws[4][3], ccs[4][3];

  void choose_control_points() {
    cws[0][0] = cws[0][1] = cws[0][2] = 0;
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
    for (int j = 0; j < 3; j++) cws[0][j] /= n;
    std::vector<double> PW0(3 * (size_t)n);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) PW0[3 * i + j] = pws[3 * i + j] - cws[0][j];
    double pw0tpw0[9], dc[3], uct[9], vt[9];
    mul_transposed(PW0.data(), n, 3, pw0tpw0);
    svd_rows(pw0tpw0, 3, 3, uct, dc, vt);  // cvSVD(.., U_T): rows of UCt
    for (int i = 1; i < 4; i++) {
      const double k = std::sqrt(dc[i - 1] / n);
      for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
    }
  }

  void compute_barycentric_coordinates() {
    double cc[9], ut[9], w[3], vt[9], ci[9];
    for (int i = 0; i < 3; i++)
      for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    svd_rows(cc, 3, 3, ut, w, vt);  // cvInvert(CV_SVD) = SVD + backSubst(identity)
    svd_backsubst(ut, w, vt, 3, 3, nullptr, ci);
    alphas.resize(4 * (size_t)n);
    for (int i = 0; i < n; i++) {
      const double* pi = &pws[3 * i];
      double* a = &alphas[4 * i];
      for (int j = 0; j < 3; j++)
        a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                   ci[3 * j + 2] * (pi[2] - cws[0][2]);
      a[0] = 1.0f - a[1] - a[2] - a[3];
    }
  }

  void fill_M(double* M, int row, const double* as, double u, double v) const {
    double* M1 = M + row * 12;
    double* M2 = M1 + 12;
    for (int i = 0; i < 4; i++) {
      M1[3 * i] = as[i] * fu;
      M1[3 * i + 1] = 0.0;
      M1[3 * i + 2] = as[i] * (uc - u);
      M2[3 * i] = 0.0;
      M2[3 * i + 1] = as[i] * fv;
      M2[3 * i + 2] = as[i] * (vc - v);
    }
  }

  void compute_ccs(const double* betas, const double* ut) {
    for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; i++) {
      const double* v = ut + 12 * (11 - i);
      for (int j = 0; j < 4; j++)
        for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
    }
  }

  void compute_pcs() {
    pcs.resize(3 * (size_t)n);
    for (int i = 0; i < n; i++) {
      const double* a = &alphas[4 * i];
      double* pc = &pcs[3 * i];
      for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
  }

  double reprojection_error(const double R[3][3], const double t[3]) const {
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
      const double* pw = &pws[3 * i];
      const double Xc = dot3(R[0], pw) + t[0];
      const double Yc = dot3(R[1], pw) + t[1];
      const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
      const double ue = uc + fu * Xc * inv_Zc;
      const double ve = vc + fv * Yc * inv_Zc;
      const double u = us[2 * i], v = us[2 * i + 1];
      sum2 += std::sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
  }

  void estimate_R_and_t(double R[3][3], double t[3]) const {
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
      for (int j = 0; j < 3; j++) {
        pc0[j] += pcs[3 * i + j];
        pw0[j] += pws[3 * i + j];
      }
    for (int j = 0; j < 3; j++) {
      pc0[j] /= n;
      pw0[j] /= n;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
      const double* pc = &pcs[3 * i];
      const double* pw = &pws[3 * i];
      for (int j = 0; j < 3; j++) {
        abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
        abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
        abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
      }
    }
    // cvSVD(ABt, D, U, V, MODIFY_A): U = columns of left vectors, V = columns of right vectors
    double ut[9], w[3], vt[9], U[9], V[9];
    svd_rows(abt, 3, 3, ut, w, vt);
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 3; k++) {
        U[3 * i + k] = ut[3 * k + i];
        V[3 * i + k] = vt[3 * k + i];
      }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i][j] = dot3(U + 3 * i, V + 3 * j);
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                       R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
      R[2][0] = -R[2][0];
      R[2][1] = -R[2][1];
      R[2][2] = -R[2][2];
    }
    t[0] = pc0[0] - dot3(R[0], pw0);
    t[1] = pc0[1] - dot3(R[1], pw0);
    t[2] = pc0[2] - dot3(R[2], pw0);
  }

  void solve_for_sign() {
    if (pcs[2] < 0.0) {
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
      for (int i = 0; i < n; i++) {
        pcs[3 * i] = -pcs[3 * i];
        pcs[3 * i + 1] = -pcs[3 * i + 1];
        pcs[3 * i + 2] = -pcs[3 * i + 2];
      }
    }
  }

  double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
    compute_ccs(betas, ut);
    compute_pcs();
    solve_for_sign();
    estimate_R_and_t(R, t);
    return reprojection_error(R, t);
  }

  // cvSolve(L_6xk, Rho, B, CV_SVD): least squares through the thin SVD
  static void solve6(const double* L, int k, const double* rho, double* x) {
    double ut[6 * 5], w[5], vt[25];
    svd_rows(L, 6, k, ut, w, vt);
    svd_backsubst(ut, w, vt, 6, k, rho, x);
  }

  static void find_betas_approx_1(const double* l_6x10, const double* rho, double* betas) {
    double l_6x4[24], b4[4];
    for (int i = 0; i < 6; i++) {
      l_6x4[4 * i] = l_6x10[10 * i];
      l_6x4[4 * i + 1] = l_6x10[10 * i + 1];
      l_6x4[4 * i + 2] = l_6x10[10 * i + 3];
      l_6x4[4 * i + 3] = l_6x10[10 * i + 6];
    }
    solve6(l_6x4, 4, rho, b4);
    if (b4[0] < 0) {
      betas[0] = std::sqrt(-b4[0]);
      betas[1] = -b4[1] / betas[0];
      betas[2] = -b4[2] / betas[0];
      betas[3] = -b4[3] / betas[0];
    } else {
      betas[0] = std::sqrt(b4[0]);
      betas[1] = b4[1] / betas[0];
      betas[2] = b4[2] / betas[0];
      betas[3] = b4[3] / betas[0];
    }
  }

  static void find_betas_approx_2(const double* l_6x10, const double* rho, double* betas) {
    double l_6x3[18], b3[3];
    for (int i = 0; i < 6; i++)
      for (int j = 0; j < 3; j++) l_6x3[3 * i + j] = l_6x10[10 * i + j];
    solve6(l_6x3, 3, rho, b3);
    if (b3[0] < 0) {
      betas[0] = std::sqrt(-b3[0]);
      betas[1] = (b3[2] < 0) ? std::sqrt(-b3[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b3[0]);
      betas[1] = (b3[2] > 0) ? std::sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
  }

  static void find_betas_approx_3(const double* l_6x10, const double* rho, double* betas) {
    double l_6x5[30], b5[5];
    for (int i = 0; i < 6; i++)
      for (int j = 0; j < 5; j++) l_6x5[5 * i + j] = l_6x10[10 * i + j];
    solve6(l_6x5, 5, rho, b5);
    if (b5[0] < 0) {
      betas[0] = std::sqrt(-b5[0]);
      betas[1] = (b5[2] < 0) ? std::sqrt(-b5[2]) : 0.0;
    } else {
      betas[0] = std::sqrt(b5[0]);
      betas[1] = (b5[2] > 0) ? std::sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
  }

  static void compute_L_6x10(const double* ut, double* l_6x10) {
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

  void compute_rho(double* rho) const {
    rho[0] = dist2(cws[0], cws[1]);
    rho[1] = dist2(cws[0], cws[2]);
    rho[2] = dist2(cws[0], cws[3]);
    rho[3] = dist2(cws[1], cws[2]);
    rho[4] = dist2(cws[1], cws[3]);
    rho[5] = dist2(cws[2], cws[3]);
  }

  static void compute_A_and_b_gauss_newton(const double* l_6x10, const double* rho, const double betas[4], double* A,
                                           double* b) {
    for (int i = 0; i < 6; i++) {
      const double* rowL = l_6x10 + i * 10;
      double* rowA = A + i * 4;
      rowA[0] = 2 * rowL[0] * betas[0] + rowL[1] * betas[1] + rowL[3] * betas[2] + rowL[6] * betas[3];
      rowA[1] = rowL[1] * betas[0] + 2 * rowL[2] * betas[1] + rowL[4] * betas[2] + rowL[7] * betas[3];
      rowA[2] = rowL[3] * betas[0] + rowL[4] * betas[1] + 2 * rowL[5] * betas[2] + rowL[8] * betas[3];
      rowA[3] = rowL[6] * betas[0] + rowL[7] * betas[1] + rowL[8] * betas[2] + 2 * rowL[9] * betas[3];
      b[i] = rho[i] - (rowL[0] * betas[0] * betas[0] + rowL[1] * betas[0] * betas[1] + rowL[2] * betas[1] * betas[1] +
                       rowL[3] * betas[0] * betas[2] + rowL[4] * betas[1] * betas[2] + rowL[5] * betas[2] * betas[2] +
                       rowL[6] * betas[0] * betas[3] + rowL[7] * betas[1] * betas[3] + rowL[8] * betas[2] * betas[3] +
                       rowL[9] * betas[3] * betas[3]);
    }
  }

  // qr_solve (src/PnPsolver.cc:922-1001): Householder QR of the 6 x 4 system.
  // A singular column returns early leaving X untouched (the reference prints
  // and returns).
  static void qr_solve(double* A, double* b, double* X) {
    const int nr = 6, nc = 4;
    double A1[6], A2[6];
    double* pA = A;
    double* ppAkk = pA;
    for (int k = 0; k < nc; k++) {
      double* ppAik = ppAkk;
      double eta = std::fabs(*ppAik);
      for (int i = k + 1; i < nr; i++) {
        const double elt = std::fabs(*ppAik);
        if (eta < elt) eta = elt;
        ppAik += nc;
      }
      if (eta == 0) {
        A1[k] = A2[k] = 0.0;
        return;
      }
      double sum = 0.0, inv_eta = 1. / eta;
      ppAik = ppAkk;
      for (int i = k; i < nr; i++) {
        *ppAik *= inv_eta;
        sum += *ppAik * *ppAik;
        ppAik += nc;
      }
      double sigma = std::sqrt(sum);
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
    double* pb = b;
    for (int j = 0; j < nc; j++) {
      double* ppAij = ppAjj;
      double tau = 0;
      for (int i = j; i < nr; i++) {
        tau += *ppAij * pb[i];
        ppAij += nc;
      }
      tau /= A1[j];
      ppAij = ppAjj;
      for (int i = j; i < nr; i++) {
        pb[i] -= tau * *ppAij;
        ppAij += nc;
      }
      ppAjj += nc + 1;
    }
    double* pX = X;
    pX[nc - 1] = pb[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
      double* ppAij = pA + i * nc + (i + 1);
      double s = 0;
      for (int j = i + 1; j < nc; j++) {
        s += *ppAij * pX[j];
        ppAij++;
      }
      pX[i] = (pb[i] - s) / A2[i];
    }
  }

  static void gauss_newton(const double* l_6x10, const double* rho, double betas[4]) {
    double a[24], b[6], x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
      compute_A_and_b_gauss_newton(l_6x10, rho, betas, a, b);
      qr_solve(a, b, x);
      for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
  }

  double compute_pose(double R[3][3], double t[3]) {
    choose_control_points();
    compute_barycentric_coordinates();
    std::vector<double> M(2 * (size_t)n * 12);
    for (int i = 0; i < n; i++) fill_M(M.data(), 2 * i, &alphas[4 * i], us[2 * i], us[2 * i + 1]);
    double mtm[144], d[12], ut[144], vt[144];
    mul_transposed(M.data(), 2 * n, 12, mtm);
    svd_rows(mtm, 12, 12, ut, d, vt);
    double l_6x10[60], rho[6];
    compute_L_6x10(ut, l_6x10);
    compute_rho(rho);
    double Betas[4][4], rep_errors[4], Rs[4][3][3], ts[4][3];
    find_betas_approx_1(l_6x10, rho, Betas[1]);
    gauss_newton(l_6x10, rho, Betas[1]);
    rep_errors[1] = compute_R_and_t(ut, Betas[1], Rs[1], ts[1]);
    find_betas_approx_2(l_6x10, rho, Betas[2]);
    gauss_newton(l_6x10, rho, Betas[2]);
    rep_errors[2] = compute_R_and_t(ut, Betas[2], Rs[2], ts[2]);
    find_betas_approx_3(l_6x10, rho, Betas[3]);
    gauss_newton(l_6x10, rho, Betas[3]);
    rep_errors[3] = compute_R_and_t(ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep_errors[2] < rep_errors[1]) N = 2;
    if (rep_errors[3] < rep_errors[N]) N = 3;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) R[i][j] = Rs[N][i][j];
      t[i] = ts[N][i];
    }
    return rep_errors[N];
  }
};

}  // namespace

struct oracle_pnp {
  // correspondences (PnPsolver ctor gather order)
  int N = 0;
  std::vector<float> p3d, p2d, sigma2, max_error;
  double fu, fv, uc, vc;
  // SetRansacParameters
  double prob;
  int min_inliers, max_its, min_set;
  float epsilon;
  // iterate() state
  int iterations = 0, best_inliers = 0, refined_inliers = 0;
  std::vector<uint8_t> inl, best, refined;
  int inliers_i = 0;
  double R[3][3], t[3];
  float best_Tcw[16], refined_Tcw[16];

  void check_inliers() {  // :352-384
    inliers_i = 0;
    for (int i = 0; i < N; i++) {
      const float X = p3d[3 * i], Y = p3d[3 * i + 1], Z = p3d[3 * i + 2];
      const float Xc = R[0][0] * X + R[0][1] * Y + R[0][2] * Z + t[0];
      const float Yc = R[1][0] * X + R[1][1] * Y + R[1][2] * Z + t[1];
      const float invZc = 1 / (R[2][0] * X + R[2][1] * Y + R[2][2] * Z + t[2]);
      const double ue = uc + fu * Xc * invZc;
      const double ve = vc + fv * Yc * invZc;
      const float distX = p2d[2 * i] - ue;
      const float distY = p2d[2 * i + 1] - ve;
      const float error2 = distX * distX + distY * distY;
      inl[i] = error2 < max_error[i] ? 1 : 0;
      inliers_i += inl[i];
    }
  }

  void pose_to_Tcw(float T[16]) const {  // Rcw/tcw convertTo(CV_32F) into eye(4)
    for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.f : 0.f;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[r][c];
      T[4 * r + 3] = (float)t[r];
    }
  }

  void pose_from(const std::vector<int>& idx) {
    Epnp e;
    e.fu = fu;
    e.fv = fv;
    e.uc = uc;
    e.vc = vc;
    e.n = (int)idx.size();
    e.pws.resize(3 * idx.size());
    e.us.resize(2 * idx.size());
    for (size_t k = 0; k < idx.size(); k++) {
      const int i = idx[k];
      for (int j = 0; j < 3; j++) e.pws[3 * k + j] = p3d[3 * i + j];  // add_correspondence(double X, ...)
      e.us[2 * k] = p2d[2 * i];
      e.us[2 * k + 1] = p2d[2 * i + 1];
    }
    e.compute_pose(R, t);
  }

  bool refine() {  // :303-349
    std::vector<int> idx;
    for (int i = 0; i < N; i++)
      if (best[i]) idx.push_back(i);
    pose_from(idx);
    check_inliers();
    refined_inliers = inliers_i;
    refined = inl;
    if (inliers_i > min_inliers) {
      pose_to_Tcw(refined_Tcw);
      return true;
    }
    return false;
  }
};

extern "C" {

// SetRansacParameters (src/PnPsolver.cc:136-179): the derived parameters and mvMaxError, in place
// (mnIterations, mnBestInliers and mvbBestInliers are kept, as in the reference)
void oracle_pnp_set_params(oracle_pnp* h, double probability, int min_inliers, int max_iterations, int min_set,
                           float epsilon, float th2) {
  const int n = h->N;
  h->prob = probability;
  h->min_inliers = min_inliers;
  h->max_its = max_iterations;
  h->epsilon = epsilon;
  h->min_set = min_set;
  int nMinInliers = n * h->epsilon;
  if (nMinInliers < h->min_inliers) nMinInliers = h->min_inliers;
  if (nMinInliers < min_set) nMinInliers = min_set;
  h->min_inliers = nMinInliers;
  if (h->epsilon < (float)h->min_inliers / n) h->epsilon = (float)h->min_inliers / n;
  int nIterations;
  if (h->min_inliers == n)
    nIterations = 1;
  else
    nIterations = (int)std::ceil(std::log(1 - h->prob) / std::log(1 - std::pow(h->epsilon, 3)));
  h->max_its = std::max(1, std::min(nIterations, h->max_its));
  h->max_error.resize(n);
  for (int i = 0; i < n; i++) h->max_error[i] = h->sigma2[i] * th2;
}

oracle_pnp* oracle_pnp_create(int n, const float* p3d, const float* p2d, const float* sigma2, float fx, float fy,
                              float cx, float cy, double probability, int min_inliers, int max_iterations,
                              int min_set, float epsilon, float th2) {
  oracle_pnp* h = new oracle_pnp();
  h->N = n;
  h->p3d.assign(p3d, p3d + 3 * (size_t)n);
  h->p2d.assign(p2d, p2d + 2 * (size_t)n);
  h->sigma2.assign(sigma2, sigma2 + n);
  h->fu = fx;
  h->fv = fy;
  h->uc = cx;
  h->vc = cy;
  oracle_pnp_set_params(h, probability, min_inliers, max_iterations, min_set, epsilon, th2);
  h->inl.assign(n, 0);
  h->best.assign(n, 0);
  h->refined.assign(n, 0);
  return h;
}

void oracle_pnp_destroy(oracle_pnp* h) { delete h; }

void oracle_pnp_params(const oracle_pnp* h, int* min_inliers, int* max_its, float* epsilon) {
  *min_inliers = h->min_inliers;
  *max_its = h->max_its;
  *epsilon = h->epsilon;
}

// PnPsolver::iterate (:182-301).  rand_vals: the process's rand() outputs in
// draw order (RandomInt(min,max) = min + int(rand()/(RAND_MAX+1.0) * (max-min+1)));
// *used = values consumed.  Returns 1 with Tcw/inliers when a pose is returned.
int oracle_pnp_iterate(oracle_pnp* h, int nIterations, const int32_t* rand_vals, int n_rand, int* used,
                       int* bNoMore, float Tcw[16], uint8_t* inliers, int* nInliers) {
  *bNoMore = 0;
  *nInliers = 0;
  *used = 0;
  const int N = h->N;
  if (N < h->min_inliers) {
    *bNoMore = 1;
    return 0;
  }
  int nCurrentIterations = 0;
  std::vector<int> avail;
  while (h->iterations < h->max_its || nCurrentIterations < nIterations) {
    if (*used + h->min_set > n_rand) return -1;  // caller supplied too few rand() values
    nCurrentIterations++;
    h->iterations++;
    avail.resize(N);
    for (int i = 0; i < N; i++) avail[i] = i;
    std::vector<int> idx;
    for (int i = 0; i < h->min_set; ++i) {
      const int mx = (int)avail.size() - 1;
      const int randi = (int)(((double)rand_vals[(*used)++] / ((double)RAND_MAX + 1.0)) * (mx + 1));
      idx.push_back(avail[randi]);
      avail[randi] = avail.back();
      avail.pop_back();
    }
    h->pose_from(idx);
    h->check_inliers();
    if (h->inliers_i >= h->min_inliers) {
      if (h->inliers_i > h->best_inliers) {
        h->best = h->inl;
        h->best_inliers = h->inliers_i;
        h->pose_to_Tcw(h->best_Tcw);
      }
      if (h->refine()) {
        *nInliers = h->refined_inliers;
        std::memcpy(inliers, h->refined.data(), N);
        std::memcpy(Tcw, h->refined_Tcw, sizeof(float) * 16);
        return 1;
      }
    }
  }
  if (h->iterations >= h->max_its) {
    *bNoMore = 1;
    if (h->best_inliers >= h->min_inliers) {
      *nInliers = h->best_inliers;
      std::memcpy(inliers, h->best.data(), N);
      std::memcpy(Tcw, h->best_Tcw, sizeof(float) * 16);
      return 1;
    }
  }
  return 0;
}

// EPnP probe: compute_pose on n correspondences (double), R row-major 3x3.
double oracle_epnp(const double* pws, const double* us, int n, double fu, double fv, double uc, double vc, double* R,
                   double* t) {
  Epnp e;
  e.fu = fu;
  e.fv = fv;
  e.uc = uc;
  e.vc = vc;
  e.n = n;
  e.pws.assign(pws, pws + 3 * (size_t)n);
  e.us.assign(us, us + 2 * (size_t)n);
  double Rm[3][3];
  const double err = e.compute_pose(Rm, t);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = Rm[i][j];
  return err;
}

// Jacobi SVD probe (cvSVD semantics on an m x n matrix, m >= n): Ut rows, w, Vt.
void oracle_svd(const double* A, int m, int n, double* Ut, double* w, double* Vt) { svd_rows(A, m, n, Ut, w, Vt); }

}  // extern "C"
