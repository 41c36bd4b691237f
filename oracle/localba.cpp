// localba.cpp -- CPU ORACLE for Optimizer::LocalBundleAdjustment
// (src/Optimizer.cc:530-885) on g2o semantics.  TEST INFRASTRUCTURE ONLY.
//
// The g2o .cpp bodies are absent from /root/reference; they are
// restated from upstream g2o / ORB-SLAM2:
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ  computeError, cam_project,
//       linearizeOplus, isDepthPositive  (types_six_dof_expmap.h:80-141)
//   BaseBinaryEdge::constructQuadraticForm       (core/base_binary_edge.hpp:55-120)
//   RobustKernelHuber::robustify (dsqr is float) (core/robust_kernel_impl.h:76-85)
//   BlockSolver<6,3> buildSystem / setLambda / restoreDiagonal / solve (Schur)
//                                                (core/block_solver.hpp:354-604)
//   LinearSolverEigen: SPD solve; failure -> LM rejects the step (solvers/linear_solver_eigen.h:94-124)
//   OptimizationAlgorithmLevenberg::solve incl. the ORB-SLAM2 _nBad rule
//                                                (core/optimization_algorithm_levenberg.h:37-88)
//   SparseOptimizer initializeOptimization(level) / optimize / push / pop / update
//   VertexSE3Expmap::oplusImpl = exp(d)*T, SE3Quat exp/map/operator*  (types/se3quat.h)
// The reduced camera system is solved with a dense LDLT (no pivoting); the
// reference uses a sparse LDLT with AMD ordering -- same solution to rounding.
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "orb_oracle.h"

namespace {

struct Quat {
  double x, y, z, w;  // Eigen coeffs order
};

Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - (a.x * b.x + a.y * b.y + a.z * b.z);
  r.x = a.w * b.x + b.w * a.x + (a.y * b.z - a.z * b.y);
  r.y = a.w * b.y + b.w * a.y + (a.z * b.x - a.x * b.z);
  r.z = a.w * b.z + b.w * a.z + (a.x * b.y - a.y * b.x);
  return r;
}

// Eigen Quaternion * Vector3 (_transformVector): v + w*uv + q x uv, uv = 2 q x v
void qrot(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  for (int i = 0; i < 3; i++) out[i] = v[i] + q.w * uv[i] + c[i];
}

// Eigen QuaternionBase::toRotationMatrix
void qmat(const Quat& q, double R[9]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// Eigen Quaternion from a rotation matrix (quaternionbase_assign_impl)
Quat mat2q(const double m[9]) {
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

void se3_map(const SE3& T, const double X[3], double out[3]) {
  qrot(T.q, X, out);
  for (int i = 0; i < 3; i++) out[i] += T.t[i];
}

// SE3Quat::exp(update), update = (omega, upsilon)
SE3 se3_exp(const double u[6]) {
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
    const double s = std::sin(theta), c = std::cos(theta);
    const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / std::pow(theta, 3);
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

struct Edge {
  int point, cam;
  bool stereo;
  double obs[3];
  double info;      // invSigma2 (information = info * I)
  double fx, fy, cx, cy, bf;
  double delta;     // Huber delta (double, from float sqrt)
  float dsqr;       // Huber delta^2 stored as float
  bool robust = true;
  int level = 0;
  double err[3] = {0, 0, 0};  // _error from the last computeError
};

double edge_chi2(const Edge& e) {
  const int D = e.stereo ? 3 : 2;
  double s = 0;
  for (int i = 0; i < D; i++) s += e.err[i] * (e.info * e.err[i]);
  return s;
}

void huber(const Edge& e, double chi, double rho[3]) {
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

struct Problem {
  std::vector<SE3> cams;
  std::vector<char> cam_fixed;
  std::vector<double> pts;  // 3 per point
  std::vector<Edge> edges;
};

void compute_error(const Problem& P, Edge& e) {
  double Pc[3];
  se3_map(P.cams[e.cam], &P.pts[3 * e.point], Pc);
  if (!e.stereo) {
    const double u = Pc[0] / Pc[2] * e.fx + e.cx, v = Pc[1] / Pc[2] * e.fy + e.cy;
    e.err[0] = e.obs[0] - u;
    e.err[1] = e.obs[1] - v;
  } else {
    const float invz = (float)(1.0 / Pc[2]);
    const float bff = (float)e.bf;
    const double u = Pc[0] * invz * e.fx + e.cx, v = Pc[1] * invz * e.fy + e.cy;
    const double ur = u - (double)(bff * invz);
    e.err[0] = e.obs[0] - u;
    e.err[1] = e.obs[1] - v;
    e.err[2] = e.obs[2] - ur;
  }
}

bool depth_positive(const Problem& P, const Edge& e) {
  double Pc[3];
  se3_map(P.cams[e.cam], &P.pts[3 * e.point], Pc);
  return Pc[2] > 0.0;
}

// linearizeOplus: A = d err / d point (D x 3), B = d err / d pose (D x 6)
void linearize(const Problem& P, const Edge& e, double A[9], double B[18]) {
  const SE3& T = P.cams[e.cam];
  double Pc[3];
  se3_map(T, &P.pts[3 * e.point], Pc);
  const double x = Pc[0], y = Pc[1], z = Pc[2], z_2 = z * z;
  double R[9];
  qmat(T.q, R);
  const double fx = e.fx, fy = e.fy, bf = e.bf;
  if (!e.stereo) {
    const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
    for (int r = 0; r < 2; r++)
      for (int c = 0; c < 3; c++)
        A[3 * r + c] = -1. / z * (tmp[3 * r] * R[c] + tmp[3 * r + 1] * R[3 + c] + tmp[3 * r + 2] * R[6 + c]);
  } else {
    for (int c = 0; c < 3; c++) {
      A[c] = -fx * R[c] / z + fx * x * R[6 + c] / z_2;
      A[3 + c] = -fy * R[3 + c] / z + fy * y * R[6 + c] / z_2;
      A[6 + c] = A[c] - bf * R[6 + c] / z_2;
    }
  }
  B[0] = x * y / z_2 * fx;
  B[1] = -(1 + (x * x / z_2)) * fx;
  B[2] = y / z * fx;
  B[3] = -1. / z * fx;
  B[4] = 0;
  B[5] = x / z_2 * fx;
  B[6] = (1 + y * y / z_2) * fy;
  B[7] = -x * y / z_2 * fy;
  B[8] = -x / z * fy;
  B[9] = 0;
  B[10] = -1. / z * fy;
  B[11] = y / z_2 * fy;
  if (e.stereo) {
    B[12] = B[0] - bf * y / z_2;
    B[13] = B[1] + bf * x / z_2;
    B[14] = B[2];
    B[15] = B[3];
    B[16] = 0;
    B[17] = B[5] - bf / z_2;
  }
}

// Dense LDLT without pivoting; false on a zero pivot (Eigen SimplicialLDLT's failure mode).
bool ldlt_solve(std::vector<double> H, int n, const std::vector<double>& b, std::vector<double>& x) {
  std::vector<double> L(n * (size_t)n, 0.0), D(n, 0.0);
  for (int j = 0; j < n; j++) {
    double d = H[(size_t)j * n + j];
    for (int k = 0; k < j; k++) d -= L[(size_t)j * n + k] * L[(size_t)j * n + k] * D[k];
    if (d == 0.0) return false;
    D[j] = d;
    for (int i = j + 1; i < n; i++) {
      double s = H[(size_t)i * n + j];
      for (int k = 0; k < j; k++) s -= L[(size_t)i * n + k] * L[(size_t)j * n + k] * D[k];
      L[(size_t)i * n + j] = s / d;
    }
  }
  x.assign(n, 0.0);
  std::vector<double> y(n);
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[(size_t)i * n + k] * y[k];
    y[i] = s;
  }
  for (int i = 0; i < n; i++) y[i] /= D[i];
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < n; k++) s -= L[(size_t)k * n + i] * x[k];
    x[i] = s;
  }
  return true;
}

void inv3(const double m[9], double out[9]) {  // Matrix3d::inverse (cofactors)
  const double c00 = m[4] * m[8] - m[5] * m[7], c01 = m[5] * m[6] - m[3] * m[8], c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  const double id = 1.0 / det;
  out[0] = c00 * id;
  out[1] = (m[2] * m[7] - m[1] * m[8]) * id;
  out[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  out[3] = c01 * id;
  out[4] = (m[0] * m[8] - m[2] * m[6]) * id;
  out[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  out[6] = c02 * id;
  out[7] = (m[1] * m[6] - m[0] * m[7]) * id;
  out[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

struct Optimizer {
  Problem& P;
  std::vector<int> active_edges;
  std::vector<int> cam_idx, pt_idx;  // hessian index (-1 = inactive/fixed)
  int nposes = 0, npts = 0;
  // system
  std::vector<double> Hpp, Hll, bp, bl;      // Hpp dense (6n)^2; Hll 9 per point
  std::vector<double> Hpl;                   // per active edge: 6x3 (pose rows, point cols)
  std::vector<double> x;                     // poses then points
  std::vector<double> diagBackP, diagBackL;
  double lambda = 0, ni = 2;
  int nBad = 0;
  const volatile int* stop;
  int trials = 0;
  explicit Optimizer(Problem& p, const volatile int* s) : P(p), stop(s) {}

  bool terminate() const { return stop && *stop; }

  // SparseOptimizer::initializeOptimization(level) + buildIndexMapping
  void initialize(int level) {
    active_edges.clear();
    std::vector<char> cam_used(P.cams.size(), 0), pt_used(P.pts.size() / 3, 0);
    for (size_t i = 0; i < P.edges.size(); i++) {
      const Edge& e = P.edges[i];
      if (level >= 0 && e.level != level) continue;
      active_edges.push_back((int)i);  // a point vertex is never fixed: !allVerticesFixed
      cam_used[e.cam] = 1;
      pt_used[e.point] = 1;
    }
    cam_idx.assign(P.cams.size(), -1);
    pt_idx.assign(P.pts.size() / 3, -1);
    nposes = npts = 0;
    for (size_t c = 0; c < P.cams.size(); c++)
      if (cam_used[c] && !P.cam_fixed[c]) cam_idx[c] = nposes++;
    for (size_t p = 0; p < pt_idx.size(); p++)
      if (pt_used[p]) pt_idx[p] = npts++;
  }

  void compute_active_errors() {
    for (int i : active_edges) compute_error(P, P.edges[i]);
  }

  double active_robust_chi2() const {
    double chi = 0;
    for (int i : active_edges) {
      const Edge& e = P.edges[i];
      if (e.robust) {
        double rho[3];
        huber(e, edge_chi2(e), rho);
        chi += rho[0];
      } else {
        chi += edge_chi2(e);
      }
    }
    return chi;
  }

  void build_system() {
    const int N = 6 * nposes;
    Hpp.assign((size_t)N * N, 0.0);
    bp.assign(N, 0.0);
    Hll.assign(9 * (size_t)npts, 0.0);
    bl.assign(3 * (size_t)npts, 0.0);
    Hpl.assign(18 * active_edges.size(), 0.0);
    for (size_t k = 0; k < active_edges.size(); k++) {
      Edge& e = P.edges[active_edges[k]];
      const int D = e.stereo ? 3 : 2;
      double A[9], B[18];
      linearize(P, e, A, B);
      double omega_r[3], W = e.info;
      for (int i = 0; i < D; i++) omega_r[i] = -e.info * e.err[i];
      if (e.robust) {
        double rho[3];
        huber(e, edge_chi2(e), rho);
        W = rho[1] * e.info;
        for (int i = 0; i < D; i++) omega_r[i] *= rho[1];
      }
      const int pi = pt_idx[e.point], ci = cam_idx[e.cam];
      // point (always active, never fixed)
      for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int d = 0; d < D; d++) s += A[3 * d + r] * omega_r[d];
        bl[3 * pi + r] += s;
        for (int c = 0; c < 3; c++) {
          double h = 0;
          for (int d = 0; d < D; d++) h += A[3 * d + r] * W * A[3 * d + c];
          Hll[9 * pi + 3 * r + c] += h;
        }
      }
      if (ci >= 0) {
        for (int r = 0; r < 6; r++) {
          double s = 0;
          for (int d = 0; d < D; d++) s += B[6 * d + r] * omega_r[d];
          bp[6 * ci + r] += s;
          for (int c = 0; c < 6; c++) {
            double h = 0;
            for (int d = 0; d < D; d++) h += B[6 * d + r] * W * B[6 * d + c];
            Hpp[(size_t)(6 * ci + r) * N + 6 * ci + c] += h;
          }
          for (int c = 0; c < 3; c++) {  // Hpl = B^T W A (pose x point)
            double h = 0;
            for (int d = 0; d < D; d++) h += B[6 * d + r] * W * A[3 * d + c];
            Hpl[18 * k + 3 * r + c] = h;
          }
        }
      }
    }
  }

  double lambda_init() const {  // computeLambdaInit: tau * max |H_jj| over active vertices
    double m = 0;
    const int N = 6 * nposes;
    for (int i = 0; i < N; i++) m = std::max(std::fabs(Hpp[(size_t)i * N + i]), m);
    for (int p = 0; p < npts; p++)
      for (int j = 0; j < 3; j++) m = std::max(std::fabs(Hll[9 * p + 4 * j]), m);
    return 1e-5 * m;
  }

  // setLambda + Schur + linear solve + back substitution (BlockSolver::solve)
  bool solve_damped(double lam) {
    const int N = 6 * nposes;
    std::vector<double> S((size_t)N * N);
    for (size_t i = 0; i < S.size(); i++) S[i] = Hpp[i];
    for (int i = 0; i < N; i++) S[(size_t)i * N + i] += lam;
    std::vector<double> coef(N, 0.0);
    std::vector<double> Dinv(9 * (size_t)npts);
    // edges grouped by point
    std::vector<std::vector<int>> pe(npts);
    for (size_t k = 0; k < active_edges.size(); k++) {
      const Edge& e = P.edges[active_edges[k]];
      if (cam_idx[e.cam] >= 0) pe[pt_idx[e.point]].push_back((int)k);
    }
    for (int p = 0; p < npts; p++) {
      double D[9];
      for (int i = 0; i < 9; i++) D[i] = Hll[9 * p + i];
      D[0] += lam;
      D[4] += lam;
      D[8] += lam;
      inv3(D, &Dinv[9 * p]);
      const double* Di = &Dinv[9 * p];
      double db[3];
      for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * bl[3 * p] + Di[3 * r + 1] * bl[3 * p + 1] + Di[3 * r + 2] * bl[3 * p + 2];
      for (int k1 : pe[p]) {
        const int c1 = cam_idx[P.edges[active_edges[k1]].cam];
        const double* B1 = &Hpl[18 * k1];
        double BD[18];
        for (int r = 0; r < 6; r++)
          for (int c = 0; c < 3; c++) BD[3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
        for (int r = 0; r < 6; r++) coef[6 * c1 + r] += B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
        for (int k2 : pe[p]) {
          const int c2 = cam_idx[P.edges[active_edges[k2]].cam];
          if (c2 < c1) continue;  // upper triangle
          const double* B2 = &Hpl[18 * k2];
          for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++) {
              const double v = BD[3 * r] * B2[3 * c] + BD[3 * r + 1] * B2[3 * c + 1] + BD[3 * r + 2] * B2[3 * c + 2];
              S[(size_t)(6 * c1 + r) * N + 6 * c2 + c] -= v;
              if (c1 != c2) S[(size_t)(6 * c2 + c) * N + 6 * c1 + r] -= v;
            }
        }
      }
    }
    std::vector<double> bs(N);
    for (int i = 0; i < N; i++) bs[i] = bp[i] - coef[i];
    std::vector<double> xp;
    if (N > 0) {
      if (!ldlt_solve(S, N, bs, xp)) return false;
    }
    x.assign(N + 3 * (size_t)npts, 0.0);
    for (int i = 0; i < N; i++) x[i] = xp[i];
    for (int p = 0; p < npts; p++) {
      double c[3] = {bl[3 * p], bl[3 * p + 1], bl[3 * p + 2]};
      for (int k : pe[p]) {
        const int ci = cam_idx[P.edges[active_edges[k]].cam];
        const double* B = &Hpl[18 * k];
        for (int j = 0; j < 3; j++)
          for (int r = 0; r < 6; r++) c[j] -= B[3 * r + j] * x[6 * ci + r];
      }
      const double* Di = &Dinv[9 * p];
      for (int r = 0; r < 3; r++) x[N + 3 * p + r] = Di[3 * r] * c[0] + Di[3 * r + 1] * c[1] + Di[3 * r + 2] * c[2];
    }
    return true;
  }

  void update() {  // SparseOptimizer::update: oplus on every active vertex
    const int N = 6 * nposes;
    for (size_t c = 0; c < P.cams.size(); c++) {
      if (cam_idx[c] < 0) continue;
      P.cams[c] = se3_mul(se3_exp(&x[6 * cam_idx[c]]), P.cams[c]);
    }
    for (size_t p = 0; p < pt_idx.size(); p++) {
      if (pt_idx[p] < 0) continue;
      for (int r = 0; r < 3; r++) P.pts[3 * p + r] += x[N + 3 * pt_idx[p] + r];
    }
  }

  double compute_scale(double lam) const {
    double s = 0;
    const int N = 6 * nposes;
    for (int i = 0; i < N; i++) s += x[i] * (lam * x[i] + bp[i]);
    for (int i = 0; i < 3 * npts; i++) s += x[N + i] * (lam * x[N + i] + bl[i]);
    return s;
  }

  enum Result { OK, TERMINATE };

  // OptimizationAlgorithmLevenberg::solve(iteration)
  Result lm_iteration(int iteration) {
    compute_active_errors();
    double currentChi = active_robust_chi2();
    const double iniChi = currentChi;
    build_system();
    if (iteration == 0) {
      lambda = lambda_init();
      ni = 2;
      nBad = 0;
    }
    double rho = 0;
    int qmax = 0;
    do {
      std::vector<SE3> cams_bak = P.cams;
      std::vector<double> pts_bak = P.pts;
      const bool ok2 = solve_damped(lambda);
      trials++;
      if (ok2) update();
      compute_active_errors();
      double tempChi = active_robust_chi2();
      if (nan_trial >= 0 && phase_trial == nan_trial) tempChi = std::nan("");  // test hook (ORBX_BA_NAN_TRIAL)
      phase_trial++;
      if (!ok2) tempChi = std::numeric_limits<double>::max();
      rho = currentChi - tempChi;
      double scale = ok2 ? compute_scale(lambda) : 0.0;
      scale += 1e-3;
      rho /= scale;
      if (rho > 0 && std::isfinite(tempChi)) {
        double alpha = 1. - std::pow((2 * rho - 1), 3);
        alpha = std::min(alpha, 2. / 3.);
        const double scaleFactor = std::max(1. / 3., alpha);
        lambda *= scaleFactor;
        ni = 2;
        currentChi = tempChi;
      } else {
        lambda *= ni;
        ni *= 2;
        P.cams = cams_bak;  // pop (errors of the rejected estimate stay)
        P.pts = pts_bak;
      }
      qmax++;
    } while (rho < 0 && qmax < 10 && !terminate());
    if (qmax == 10 || rho == 0) return TERMINATE;
    if ((iniChi - currentChi) * 1e3 < iniChi)
      nBad++;
    else
      nBad = 0;
    if (nBad >= 3) return TERMINATE;
    return OK;
  }

  // test hook: the given trial of each optimize() call computes a NaN chi (rho NaN), as the GPU
  // library's ORBX_BA_NAN_TRIAL does
  int nan_trial = std::getenv("ORBX_BA_NAN_TRIAL") ? std::atoi(std::getenv("ORBX_BA_NAN_TRIAL")) : -1;
  int phase_trial = 0;

  int optimize(int iterations, double* final_chi) {
    int it = 0;
    phase_trial = 0;
    for (int i = 0; i < iterations && !terminate(); i++) {
      Result r = lm_iteration(i);
      ++it;
      if (r != OK) break;
    }
    if (final_chi) *final_chi = active_robust_chi2();
    return it;
  }
};

}  // namespace

extern "C" int oracle_local_ba(const oracle_ba_problem* pb, oracle_ba_result* res, const volatile int* stop_flag) {
  Problem P;
  const int nc = pb->n_cams, np = pb->n_points, ne = pb->n_edges;
  P.cams.resize(nc);
  P.cam_fixed.resize(nc);
  for (int c = 0; c < nc; c++) {  // Converter::toSE3Quat (float -> double)
    const float* T = pb->Tcw + 12 * c;
    double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    P.cams[c].q = mat2q(R);
    qnormalize(P.cams[c].q);
    P.cams[c].t[0] = T[3];
    P.cams[c].t[1] = T[7];
    P.cams[c].t[2] = T[11];
    P.cam_fixed[c] = pb->fixed ? pb->fixed[c] : 0;
  }
  P.pts.resize(3 * (size_t)np);
  for (int i = 0; i < 3 * np; i++) P.pts[i] = pb->Xw[i];
  const float thMono = std::sqrt(5.991f), thStereo = std::sqrt(7.815f);  // src/Optimizer.cc:653-654
  P.edges.resize(ne);
  for (int i = 0; i < ne; i++) {
    Edge& e = P.edges[i];
    e.point = pb->edge_point[i];
    e.cam = pb->edge_cam[i];
    e.stereo = pb->obs[3 * i + 2] >= 0;
    for (int k = 0; k < 3; k++) e.obs[k] = pb->obs[3 * i + k];
    e.info = pb->inv_sigma2[i];
    const float* in = pb->intr + 5 * e.cam;
    e.fx = in[0];
    e.fy = in[1];
    e.cx = in[2];
    e.cy = in[3];
    e.bf = in[4];
    e.delta = e.stereo ? thStereo : thMono;
    e.dsqr = (float)(e.delta * e.delta);
  }
  Optimizer opt(P, stop_flag);
  res->iterations[0] = res->iterations[1] = 0;
  res->trials = 0;
  res->chi2[0] = res->chi2[1] = 0;
  if (stop_flag && *stop_flag) {  // src/Optimizer.cc:749-751: return before any write-back
    std::memcpy(res->Tcw, pb->Tcw, sizeof(float) * 12 * nc);
    std::memcpy(res->Xw, pb->Xw, sizeof(float) * 3 * np);
    std::memset(res->edge_outlier, 0, ne);
    if (res->Tcw_d)
      for (int i = 0; i < 12 * nc; i++) res->Tcw_d[i] = pb->Tcw[i];
    if (res->Xw_d)
      for (int i = 0; i < 3 * np; i++) res->Xw_d[i] = pb->Xw[i];
    return 0;
  }
  opt.initialize(-1);
  res->iterations[0] = opt.optimize(5, &res->chi2[0]);
  bool doMore = !(stop_flag && *stop_flag);
  if (doMore) {
    for (Edge& e : P.edges) {  // :764-802 (errors as left by the last computeActiveErrors)
      const double th = e.stereo ? 7.815 : 5.991;
      if (edge_chi2(e) > th || !depth_positive(P, e)) e.level = 1;
      e.robust = false;
    }
    opt.initialize(0);
    res->iterations[1] = opt.optimize(10, &res->chi2[1]);
  }
  res->trials = opt.trials;
  for (int i = 0; i < ne; i++) {  // :817-847 vToErase
    const Edge& e = P.edges[i];
    const double th = e.stereo ? 7.815 : 5.991;
    res->edge_outlier[i] = (edge_chi2(e) > th || !depth_positive(P, e)) ? 1 : 0;
  }
  for (int c = 0; c < nc; c++) {  // Converter::toCvMat(SE3Quat) -> float
    double R[9];
    qmat(P.cams[c].q, R);
    float* T = res->Tcw + 12 * c;
    for (int r = 0; r < 3; r++) {
      for (int k = 0; k < 3; k++) T[4 * r + k] = (float)R[3 * r + k];
      T[4 * r + 3] = (float)P.cams[c].t[r];
    }
  }
  for (int i = 0; i < 3 * np; i++) res->Xw[i] = (float)P.pts[i];
  if (res->Tcw_d) {
    for (int c = 0; c < nc; c++) {
      double R[9];
      qmat(P.cams[c].q, R);
      for (int r = 0; r < 3; r++) {
        for (int k = 0; k < 3; k++) res->Tcw_d[12 * c + 4 * r + k] = R[3 * r + k];
        res->Tcw_d[12 * c + 4 * r + 3] = P.cams[c].t[r];
      }
    }
  }
  if (res->Xw_d)
    for (int i = 0; i < 3 * np; i++) res->Xw_d[i] = P.pts[i];
  return 0;
}

/* Probes for the unit tests: edge error + analytic Jacobians at an explicit
 * state, and SE3Quat::exp / operator* as the optimizer applies them. */
extern "C" void oracle_ba_edge_probe(const double q[4], const double t[3], const double X[3], const double intr[5],
                                     int stereo, const double obs[3], double err[3], double A[9], double B[18]) {
  Problem P;
  P.cams.resize(1);
  P.cams[0].q = {q[0], q[1], q[2], q[3]};
  for (int i = 0; i < 3; i++) P.cams[0].t[i] = t[i];
  P.pts.assign(X, X + 3);
  Edge e;
  e.point = 0;
  e.cam = 0;
  e.stereo = stereo != 0;
  for (int i = 0; i < 3; i++) e.obs[i] = obs[i];
  e.info = 1;
  e.fx = intr[0];
  e.fy = intr[1];
  e.cx = intr[2];
  e.cy = intr[3];
  e.bf = intr[4];
  compute_error(P, e);
  for (int i = 0; i < 3; i++) err[i] = e.err[i];
  for (int i = 0; i < 9; i++) A[i] = 0;
  for (int i = 0; i < 18; i++) B[i] = 0;
  linearize(P, e, A, B);
}

extern "C" void oracle_se3_exp_mul(const double u[6], const double q[4], const double t[3], double q_out[4],
                                   double t_out[3]) {
  SE3 T;
  T.q = {q[0], q[1], q[2], q[3]};
  for (int i = 0; i < 3; i++) T.t[i] = t[i];
  const SE3 R = se3_mul(se3_exp(u), T);
  q_out[0] = R.q.x;
  q_out[1] = R.q.y;
  q_out[2] = R.q.z;
  q_out[3] = R.q.w;
  for (int i = 0; i < 3; i++) t_out[i] = R.t[i];
}
