// poseopt.cpp -- CPU ORACLE (test infrastructure only) for
// Optimizer::PoseOptimization (src/Optimizer.cc:287-528): one VertexSE3Expmap,
// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose unary edges with
// Huber kernels (delta sqrt(5.991) / sqrt(7.815)), four rounds of
// optimize(10) that each restart from pFrame->mTcw, outlier levels between
// rounds, robust kernels dropped after round 2.
//
// g2o bodies absent from /root/reference, restated from upstream ORB-SLAM2 g2o:
//   EdgeSE3ProjectXYZOnlyPose / EdgeStereo... cam_project + linearizeOplus
//       (types_six_dof_expmap.cpp; declarations types_six_dof_expmap.h:143-202):
//       mono   u = x/z*fx + cx (project2d), stereo invz = (float)(1/z),
//              u = x*invz*fx + cx, ur = u - bf*invz (bf double member)
//       J row0 = [x*y*iz2*fx, -(1+x*x*iz2)*fx, y*iz*fx, -iz*fx, 0, x*iz2*fx]
//       J row1 = [(1+y*y*iz2)*fy, -x*y*iz2*fy, -x*iz*fy, 0, -iz*fy, y*iz2*fy]
//       J row2 = row0 + [-bf*y*iz2, +bf*x*iz2, 0, 0, 0, -bf*iz2]   (iz = 1/z, iz2 = iz*iz)
//   BaseUnaryEdge::constructQuadraticForm (core/base_unary_edge.hpp:43-72):
//       b -= rho1 * A^T * Omega * e;  H += A^T * (rho1*Omega) * A
//   LinearSolverDense (solvers/linear_solver_dense.h:65-112): Eigen::LDLT with
//       diagonal pivoting, isPositive() gate; restated below (sequential dots).
//   OptimizationAlgorithmLevenberg incl. the ORB-SLAM2 _nBad rule, the same
//       loop as oracle/localba.cpp.
// Transcendentals: SE3Quat::exp's sin/cos are a deterministic double
// evaluation (Cody-Waite + Taylor, basic IEEE ops), pow(theta,3) is
// theta*theta*theta and LM's pow(2rho-1, 3) a cube -- shared operation sequences with the GPU, so the HIP path
// reproduces this oracle bit for bit (sums run in the same edge order there).
// Parity vs the genuine g2o/Eigen binary is unpinned.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "orb_oracle.h"

namespace {

struct Quat {
  double x, y, z, w;
};

Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - (a.x * b.x + a.y * b.y + a.z * b.z);
  r.x = a.w * b.x + b.w * a.x + (a.y * b.z - a.z * b.y);
  r.y = a.w * b.y + b.w * a.y + (a.z * b.x - a.x * b.z);
  r.z = a.w * b.z + b.w * a.z + (a.x * b.y - a.y * b.x);
  return r;
}

void qrot(const Quat& q, const double v[3], double out[3]) {  // Eigen _transformVector
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  for (int i = 0; i < 3; i++) out[i] = v[i] + q.w * uv[i] + c[i];
}

void qmat(const Quat& q, double R[9]) {  // QuaternionBase::toRotationMatrix
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

Quat mat2q(const double m[9]) {  // quaternionbase_assign_impl
  Quat q;
  double t = m[0] + m[4] + m[8];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m[7] - m[5]) * t;
    q.y = (m[2] - m[6]) * t;
    q.z = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[3 * i + i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double c[3];
    t = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (m[3 * k + j] - m[3 * j + k]) * t;
    c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
    c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
  }
  return q;
}

void qnormalize(Quat& q) {  // SE3Quat::normalizeRotation
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

struct SE3 {
  Quat q;
  double t[3];
};

// Deterministic double sin/cos (same sequence on the GPU).
void sincos_d(double x, double* s_out, double* c_out) {
  const double kInvPio2 = 6.36619772367581382433e-01;
  const double kPio2Hi = 1.57079632673412561417e+00;
  const double kPio2Lo = 6.07710050650619224932e-11;
  const double kd = std::rint(x * kInvPio2);
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

SE3 se3_exp(const double u[6]) {  // SE3Quat::exp, types/se3quat.h:223-257
  const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
  const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double O2[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
  double R[9], V[9];
  if (theta < 0.00001) {
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + O[i] + O2[i];
    for (int i = 0; i < 9; i++) V[i] = R[i];
  } else {
    double s, c;
    sincos_d(theta, &s, &c);
    const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / (theta * theta * theta);
    for (int i = 0; i < 9; i++) {
      const double I = (i % 4) == 0 ? 1.0 : 0.0;
      R[i] = I + a * O[i] + b * O2[i];
      V[i] = I + b * O[i] + d * O2[i];
    }
  }
  SE3 T;
  T.q = mat2q(R);
  for (int r = 0; r < 3; r++) T.t[r] = V[3 * r] * up[0] + V[3 * r + 1] * up[1] + V[3 * r + 2] * up[2];
  qnormalize(T.q);
  return T;
}

SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
  SE3 r = a;
  double rt[3];
  qrot(a.q, b.t, rt);
  for (int i = 0; i < 3; i++) r.t[i] += rt[i];
  r.q = qmul(a.q, b.q);
  qnormalize(r.q);
  return r;
}

SE3 from_tcw(const float* T) {  // Converter::toSE3Quat
  const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
  SE3 s;
  s.q = mat2q(R);
  qnormalize(s.q);
  s.t[0] = T[3];
  s.t[1] = T[7];
  s.t[2] = T[11];
  return s;
}

struct Edge {
  bool stereo;
  double obs[3], X[3], info;
  double delta;
  float dsqr;
  int level = 0;
  double err[3] = {0, 0, 0};
};

struct Cam {
  double fx, fy, cx, cy, bf;
};

void compute_error(const SE3& T, const Cam& K, Edge& e) {
  double Pc[3];
  qrot(T.q, e.X, Pc);
  for (int i = 0; i < 3; i++) Pc[i] += T.t[i];
  if (!e.stereo) {
    const double u = Pc[0] / Pc[2] * K.fx + K.cx, v = Pc[1] / Pc[2] * K.fy + K.cy;
    e.err[0] = e.obs[0] - u;
    e.err[1] = e.obs[1] - v;
  } else {
    const float invz = (float)(1.0 / Pc[2]);
    const double u = Pc[0] * invz * K.fx + K.cx, v = Pc[1] * invz * K.fy + K.cy;
    const double ur = u - K.bf * invz;
    e.err[0] = e.obs[0] - u;
    e.err[1] = e.obs[1] - v;
    e.err[2] = e.obs[2] - ur;
  }
}

double edge_chi2(const Edge& e) {
  const int D = e.stereo ? 3 : 2;
  double s = 0;
  for (int i = 0; i < D; i++) s += e.err[i] * (e.info * e.err[i]);
  return s;
}

void huber(const Edge& e, double chi, double rho[3]) {  // RobustKernelHuber::robustify
  if (chi <= e.dsqr) {
    rho[0] = chi;
    rho[1] = 1.;
    rho[2] = 0.;
  } else {
    const double sq = std::sqrt(chi);
    rho[0] = 2 * sq * e.delta - e.dsqr;
    rho[1] = e.delta / sq;
    rho[2] = -0.5 * rho[1] / chi;
  }
}

void jacobian(const SE3& T, const Cam& K, const Edge& e, double J[18]) {
  double Pc[3];
  qrot(T.q, e.X, Pc);
  for (int i = 0; i < 3; i++) Pc[i] += T.t[i];
  const double x = Pc[0], y = Pc[1], iz = 1.0 / Pc[2], iz2 = iz * iz;
  J[0] = x * y * iz2 * K.fx;
  J[1] = -(1 + (x * x * iz2)) * K.fx;
  J[2] = y * iz * K.fx;
  J[3] = -iz * K.fx;
  J[4] = 0;
  J[5] = x * iz2 * K.fx;
  J[6] = (1 + y * y * iz2) * K.fy;
  J[7] = -x * y * iz2 * K.fy;
  J[8] = -x * iz * K.fy;
  J[9] = 0;
  J[10] = -iz * K.fy;
  J[11] = y * iz2 * K.fy;
  if (e.stereo) {
    J[12] = J[0] - K.bf * y * iz2;
    J[13] = J[1] + K.bf * x * iz2;
    J[14] = J[2];
    J[15] = J[3];
    J[16] = 0;
    J[17] = J[5] - K.bf * iz2;
  }
}

// One edge's quadratic-form terms: c[0..20] = upper triangle of A^T W A
// (row-major (r, c >= r)), c[21..26] = rho1 * A^T Omega e (subtracted from b).
void edge_terms(const Edge& e, const double J[18], bool robust, double c[27]) {
  const int D = e.stereo ? 3 : 2;
  double w = e.info, r1 = 1.0;
  if (robust) {
    double rho[3];
    huber(e, edge_chi2(e), rho);
    r1 = rho[1];
    w = rho[1] * e.info;  // robustInformation
  }
  int k = 0;
  for (int r = 0; r < 6; r++)
    for (int cc = r; cc < 6; cc++) {
      double s = (J[r] * w) * J[cc];
      for (int d = 1; d < D; d++) s = s + (J[6 * d + r] * w) * J[6 * d + cc];
      c[k++] = s;
    }
  for (int r = 0; r < 6; r++) {
    double s = ((r1 * J[r]) * e.info) * e.err[0];
    for (int d = 1; d < D; d++) s = s + ((r1 * J[6 * d + r]) * e.info) * e.err[d];
    c[21 + r] = s;
  }
}

// Eigen::LDLT<MatrixXd> (diagonal pivoting, lower storage) + solve; false when
// !isPositive().
bool ldlt6(const double Hin[36], const double b[6], double x[6]) {
  double m[36];
  std::memcpy(m, Hin, sizeof(m));
  int tr[6];
  int sign = 0;  // 0 zero, 1 PositiveSemiDef, 2 NegativeSemiDef, 3 Indefinite
  const int n = 6;
  for (int k = 0; k < n; k++) {
    int big = k;
    double bv = std::fabs(m[7 * k]);
    for (int i = k + 1; i < n; i++)
      if (std::fabs(m[7 * i]) > bv) {
        bv = std::fabs(m[7 * i]);
        big = i;
      }
    if (k == 0 && !(bv > 0.0)) {  // the entire diagonal is zero: ZeroSign
      for (int j = 0; j < n; j++) tr[j] = j;
      for (int j = 0; j < n; j++) m[7 * j] = 0.0;
      sign = 0;
      break;
    }
    tr[k] = big;
    if (k != big) {
      for (int j = 0; j < k; j++) std::swap(m[6 * k + j], m[6 * big + j]);
      for (int i = big + 1; i < n; i++) std::swap(m[6 * i + k], m[6 * i + big]);
      std::swap(m[7 * k], m[7 * big]);
      for (int i = k + 1; i < big; i++) {
        const double t = m[6 * i + k];
        m[6 * i + k] = m[6 * big + i];
        m[6 * big + i] = t;
      }
    }
    double temp[6];
    if (k > 0) {
      for (int j = 0; j < k; j++) temp[j] = m[7 * j] * m[6 * k + j];
      double dot = m[6 * k] * temp[0];
      for (int j = 1; j < k; j++) dot = dot + m[6 * k + j] * temp[j];
      m[7 * k] -= dot;
      for (int i = k + 1; i < n; i++) {
        double s = m[6 * i] * temp[0];
        for (int j = 1; j < k; j++) s = s + m[6 * i + j] * temp[j];
        m[6 * i + k] -= s;
      }
    }
    const double akk = m[7 * k];
    const bool valid = std::fabs(akk) > 0.0;
    if (valid)
      for (int i = k + 1; i < n; i++) m[6 * i + k] /= akk;
    if (akk > 0) sign = (sign == 2 || sign == 3) ? 3 : 1;
    else if (akk < 0) sign = (sign == 1 || sign == 3) ? 3 : 2;
  }
  if (!(sign == 1 || sign == 0)) return false;  // isPositive()
  double y[6];
  for (int i = 0; i < n; i++) y[i] = b[i];
  for (int k = 0; k < n; k++) std::swap(y[k], y[tr[k]]);  // P b
  for (int i = 0; i < n; i++)                              // L^-1 (unit lower)
    for (int j = 0; j < i; j++) y[i] -= m[6 * i + j] * y[j];
  const double tol = std::numeric_limits<double>::min();
  for (int i = 0; i < n; i++) y[i] = std::fabs(m[7 * i]) > tol ? y[i] / m[7 * i] : 0.0;
  for (int i = n - 1; i >= 0; i--)  // L^-T
    for (int j = i + 1; j < n; j++) y[i] -= m[6 * j + i] * y[j];
  for (int k = n - 1; k >= 0; k--) std::swap(y[k], y[tr[k]]);  // P^T
  for (int i = 0; i < n; i++) x[i] = y[i];
  return true;
}

struct PoseOpt {
  std::vector<Edge>& E;
  const Cam& K;
  SE3 T;
  std::vector<int> act;
  bool robust = true;
  double H[36], b[6], x[6];
  double lambda = 0, ni = 2;
  int nBad = 0, trials = 0;

  PoseOpt(std::vector<Edge>& e, const Cam& k) : E(e), K(k) {}

  void errors() {
    for (int i : act) compute_error(T, K, E[i]);
  }
  double chi2() const {  // activeRobustChi2, active edges in insertion order
    double s = 0;
    for (int i : act) {
      const double c = edge_chi2(E[i]);
      if (robust) {
        double rho[3];
        huber(E[i], c, rho);
        s += rho[0];
      } else {
        s += c;
      }
    }
    return s;
  }
  void build() {  // BlockSolver::buildSystem for one pose vertex
    double up[21] = {0}, bb[6] = {0};
    for (int i : act) {
      double J[18], c[27];
      jacobian(T, K, E[i], J);
      edge_terms(E[i], J, robust, c);
      for (int k = 0; k < 21; k++) up[k] += c[k];
      for (int k = 0; k < 6; k++) bb[k] -= c[21 + k];
    }
    int k = 0;
    for (int r = 0; r < 6; r++)
      for (int c = r; c < 6; c++) {
        H[6 * r + c] = up[k];
        H[6 * c + r] = up[k];
        k++;
      }
    for (int r = 0; r < 6; r++) b[r] = bb[r];
  }
  enum { OK, TERMINATE };
  int iteration(int it) {  // OptimizationAlgorithmLevenberg::solve
    errors();
    double currentChi = chi2();
    const double iniChi = currentChi;
    build();
    if (it == 0) {
      double m = 0;
      for (int j = 0; j < 6; j++) m = std::max(std::fabs(H[7 * j]), m);
      lambda = 1e-5 * m;
      ni = 2;
      nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      const SE3 bak = T;
      double Hd[36];
      std::memcpy(Hd, H, sizeof(Hd));
      for (int j = 0; j < 6; j++) Hd[7 * j] += lambda;
      const bool ok2 = ldlt6(Hd, b, x);
      trials++;
      if (ok2) T = se3_mul(se3_exp(x), T);
      errors();
      double tempChi = chi2();
      if (!ok2) tempChi = std::numeric_limits<double>::max();
      rho = currentChi - tempChi;
      double scale = 0.0;
      if (ok2)
        for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        const double t3 = 2 * rho - 1;
        double alpha = 1. - t3 * t3 * t3;  // pow(2*rho-1, 3), deterministic
        alpha = std::min(alpha, 2. / 3.);
        lambda *= std::max(1. / 3., alpha);
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        T = bak;  // pop; the rejected trial's errors stay in the edges
      }
      qmax++;
    } while (rho < 0 && qmax < 10);
    if (qmax == 10 || rho == 0) return TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
    else nBad = 0;
    if (nBad >= 3) return TERMINATE;
    return OK;
  }
  int optimize(int its) {
    if (act.empty()) return 0;  // no active edge: the vertex is not optimised
    int n = 0;
    for (int i = 0; i < its; i++) {
      n++;
      if (iteration(i) != OK) break;
    }
    return n;
  }
};

}  // namespace

extern "C" int oracle_pose_optimization(const oracle_pose_problem* p) {
  const int n = p->n;
  Cam K{p->fx, p->fy, p->cx, p->cy, p->bf};
  std::vector<Edge> E(n);
  const float dMono = std::sqrt(5.991f), dStereo = std::sqrt(7.815f);  // src/Optimizer.cc:325-326 (float)
  for (int i = 0; i < n; i++) {
    Edge& e = E[i];
    e.stereo = p->obs[3 * i + 2] >= 0;  // mvuRight < 0: monocular edge (src/Optimizer.cc:337)
    for (int k = 0; k < 3; k++) {
      e.obs[k] = p->obs[3 * i + k];
      e.X[k] = p->Xw[3 * i + k];
    }
    e.info = p->inv_sigma2[i];
    e.delta = e.stereo ? dStereo : dMono;
    e.dsqr = (float)(e.delta * e.delta);
  }
  std::memcpy(p->Tcw_out, p->Tcw, sizeof(float) * 16);
  for (int i = 0; i < n; i++) p->outlier[i] = 0;
  if (p->iterations)
    for (int r = 0; r < 4; r++) p->iterations[r] = 0;
  if (n < 3) {  // nInitialCorrespondences < 3
    *p->ngood = 0;
    return 0;
  }
  const SE3 T0 = from_tcw(p->Tcw);
  PoseOpt opt(E, K);
  const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
  int nBad = 0;
  for (int it = 0; it < 4; it++) {
    opt.T = T0;  // vSE3->setEstimate(Converter::toSE3Quat(pFrame->mTcw))
    opt.act.clear();
    for (int i = 0; i < n; i++)
      if (E[i].level == 0) opt.act.push_back(i);
    const int its = opt.optimize(10);
    if (p->iterations) p->iterations[it] = its;
    nBad = 0;
    for (int i = 0; i < n; i++) {
      Edge& e = E[i];
      if (p->outlier[i]) compute_error(opt.T, K, e);
      const float chi2 = (float)edge_chi2(e);
      if (chi2 > (e.stereo ? chi2Stereo : chi2Mono)) {
        p->outlier[i] = 1;
        e.level = 1;
        nBad++;
      } else {
        p->outlier[i] = 0;
        e.level = 0;
      }
    }
    if (it == 2) opt.robust = false;  // e->setRobustKernel(0)
    if (n < 10) break;                // optimizer.edges().size() < 10
  }
  double R[9];
  qmat(opt.T.q, R);
  for (int r = 0; r < 3; r++) {  // Converter::toCvMat(SE3Quat)
    for (int k = 0; k < 3; k++) p->Tcw_out[4 * r + k] = (float)R[3 * r + k];
    p->Tcw_out[4 * r + 3] = (float)opt.T.t[r];
  }
  p->Tcw_out[12] = p->Tcw_out[13] = p->Tcw_out[14] = 0.0f;
  p->Tcw_out[15] = 1.0f;
  *p->ngood = n - nBad;
  return 0;
}

extern "C" void oracle_pose_edge_probe(const double q[4], const double t[3], const double X[3], const double intr[5],
                                       int stereo, const double obs[3], double err[3], double J[18]) {
  SE3 T;
  T.q = {q[0], q[1], q[2], q[3]};
  for (int i = 0; i < 3; i++) T.t[i] = t[i];
  Cam K{intr[0], intr[1], intr[2], intr[3], intr[4]};
  Edge e;
  e.stereo = stereo != 0;
  for (int i = 0; i < 3; i++) {
    e.obs[i] = obs[i];
    e.X[i] = X[i];
  }
  e.info = 1;
  compute_error(T, K, e);
  for (int i = 0; i < 3; i++) err[i] = e.err[i];
  for (int i = 0; i < 18; i++) J[i] = 0;
  jacobian(T, K, e, J);
}

extern "C" int oracle_ldlt6(const double* H, const double* b, double* x) { return ldlt6(H, b, x) ? 1 : 0; }
