// localba.hip -- Optimizer::LocalBundleAdjustment (src/Optimizer.cc:530-885)
// on g2o semantics (BlockSolver<6,3> + LinearSolverEigen + Levenberg, Huber
// kernels, two phases), FP64, device-resident.
//
// Per LM iteration (g2o OptimizationAlgorithmLevenberg::solve):
//   k_ba_errors      computeActiveErrors + robust chi per edge (errors kept per
//                    edge exactly like g2o's _error, including after a pop)
//   k_ba_linearize   linearizeOplus + constructQuadraticForm per active edge:
//                    Hpl_e = B^T W A, point (Hll,bl) and pose (Hpp,bp) terms
//   k_ba_point_sum   Hll, bl per point (fixed edge order)
//   k_ba_cam_sum     Hpp, bp per pose (fixed edge order)
//   per trial:
//   k_ba_point_schur D = Hll + lambda I, Dinv (cofactor inverse), BD_e = Hpl_e Dinv, cf_e = Hpl_e Dinv bl
//   k_ba_pairs       Hschur block (c1,c2) = [c1==c2](Hpp+lambda I) - sum_points BD_e1 Hpl_e2^T
//                    (one wave per block, fixed lane partition + tree: deterministic)
//   k_ba_cam_coef    bschur = bp - sum_e cf_e
//   k_ba_ldlt        dense LDLT of the reduced camera system in LDS, solve
//   k_ba_backsub     x_l = Dinv (bl - sum_e Hpl_e^T x_p), X += x_l; T = exp(x_p) T; scale terms
//   k_ba_errors      new chi -> host LM decision (one 3-double readback per trial)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "../../include/orbx.h"
#include "orbx_device.h"

namespace orbx {

// ------------------------------------------------------------ SE3 numerics
struct Quat {
  double x, y, z, w;
};

__host__ __device__ inline Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - (a.x * b.x + a.y * b.y + a.z * b.z);
  r.x = a.w * b.x + b.w * a.x + (a.y * b.z - a.z * b.y);
  r.y = a.w * b.y + b.w * a.y + (a.z * b.x - a.x * b.z);
  r.z = a.w * b.z + b.w * a.z + (a.x * b.y - a.y * b.x);
  return r;
}

// Eigen Quaternion * Vector3 (_transformVector)
__host__ __device__ inline void qrot(const Quat& q, const double v[3], double out[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] += uv[0];
  uv[1] += uv[1];
  uv[2] += uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  for (int i = 0; i < 3; i++) out[i] = v[i] + q.w * uv[i] + c[i];
}

__host__ __device__ inline void qmat(const Quat& q, double R[9]) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__host__ __device__ inline Quat mat2q(const double m[9]) {
  Quat q;
  double t = m[0] + m[4] + m[8];
  if (t > 0) {
    t = sqrt(t + 1.0);
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
    t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
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

__host__ __device__ inline void qnormalize(Quat& q) {
  if (q.w < 0) {
    q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w;
  }
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

struct SE3d {
  Quat q;
  double t[3];
};

__device__ inline SE3d se3_exp(const double u[6]) {
  const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
  const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double O2[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
  double R[9], V[9];
  if (theta < 0.00001) {
    for (int i = 0; i < 9; i++) R[i] = ((i % 4) == 0 ? 1.0 : 0.0) + O[i] + O2[i];
    for (int i = 0; i < 9; i++) V[i] = R[i];
  } else {
    const double s = sin(theta), c = cos(theta);
    const double a = s / theta, b = (1 - c) / (theta * theta), d = (theta - s) / pow(theta, 3);
    for (int i = 0; i < 9; i++) {
      const double I = (i % 4) == 0 ? 1.0 : 0.0;
      R[i] = I + a * O[i] + b * O2[i];
      V[i] = I + b * O[i] + d * O2[i];
    }
  }
  SE3d T;
  T.q = mat2q(R);
  for (int r = 0; r < 3; r++) T.t[r] = V[3 * r] * up[0] + V[3 * r + 1] * up[1] + V[3 * r + 2] * up[2];
  qnormalize(T.q);
  return T;
}

__device__ inline void inv3(const double m[9], double out[9]) {
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

// ------------------------------------------------------------ device state
struct BaDev {
  int nc, np, ne;
  // cameras
  double* cq;    // nc*4 (x,y,z,w)
  double* ct;    // nc*3
  double* cbak;  // nc*7
  const double* intr;  // nc*5 fx,fy,cx,cy,bf
  int* chidx;    // nc: pose hessian index or -1
  // points
  double* X;     // np*3
  double* Xbak;  // np*3
  // edges (all)
  const int* ept;
  const int* ecam;
  const uint8_t* est;    // stereo flag
  const double* eobs;    // ne*3
  const double* einfo;  // ne
  const double* edelta; // ne
  const float* edsqr;   // ne
  uint8_t* erobust;     // ne
  double* eerr;         // ne*3
  // active edge structure (positions k = 0..na-1, point-major)
  int na;
  int* act;        // na: edge id
  int* pt_off;     // npa+1 over positions
  int* pt_id;      // npa: point id of active point i
  int npa;
  int* cam_pos;    // positions grouped by active pose
  int* cam_off;    // nposes+1
  int* pose_cam;   // nposes: camera id
  int nposes;
  int* blk_off;    // nblk+1 over pair list
  int2* blk_cc;    // nblk: (c1,c2) pose indices
  int2* pairs;     // (k1,k2) positions
  int nblk;
  // per position
  double* Hpl;     // na*18 (6x3)
  double* ptc;     // na*12: Hll 9 + bl 3
  double* cmc;     // na*42: Hpp 36 + bp 6
  double* BD;      // na*18
  double* cf;      // na*6
  double* chi;     // na (robust chi of the edge)
  // per active point
  double* Hll;     // npa*9
  double* bl;      // npa*3
  double* Dinv;    // npa*9
  double* xl;      // npa*3
  double* dmax_p;  // npa
  double* scale_p; // npa
  // per pose
  double* Hpp;     // nposes*36
  double* bp;      // nposes*6
  double* xp;      // nposes*6
  double* bs;      // nposes*6
  double* S;       // (6*nposes)^2
  double* dmax_c;  // nposes
  double* scale_c; // nposes
  double* scal;    // scalars: [0] chi, [1] scale, [2] ok, [3] dmax
};

constexpr int LBS = 256;

__device__ inline void edge_error(const BaDev& D, int e, double err[3], double& chi2) {
  const int c = D.ecam[e], p = D.ept[e];
  Quat q = {D.cq[4 * c], D.cq[4 * c + 1], D.cq[4 * c + 2], D.cq[4 * c + 3]};
  const double Xw[3] = {D.X[3 * p], D.X[3 * p + 1], D.X[3 * p + 2]};
  double Pc[3];
  qrot(q, Xw, Pc);
  for (int i = 0; i < 3; i++) Pc[i] += D.ct[3 * c + i];
  const double fx = D.intr[5 * c], fy = D.intr[5 * c + 1], cx = D.intr[5 * c + 2], cy = D.intr[5 * c + 3];
  const double info = D.einfo[e];
  if (!D.est[e]) {
    const double u = Pc[0] / Pc[2] * fx + cx, v = Pc[1] / Pc[2] * fy + cy;
    err[0] = D.eobs[3 * e] - u;
    err[1] = D.eobs[3 * e + 1] - v;
    err[2] = 0;
    chi2 = err[0] * (info * err[0]) + err[1] * (info * err[1]);
  } else {
    const float invz = (float)(1.0 / Pc[2]);
    const float bff = (float)D.intr[5 * c + 4];
    const double u = Pc[0] * invz * fx + cx, v = Pc[1] * invz * fy + cy;
    const double ur = u - (double)(bff * invz);
    err[0] = D.eobs[3 * e] - u;
    err[1] = D.eobs[3 * e + 1] - v;
    err[2] = D.eobs[3 * e + 2] - ur;
    chi2 = err[0] * (info * err[0]) + err[1] * (info * err[1]) + err[2] * (info * err[2]);
  }
}

__device__ inline void huber(double chi, double delta, float dsqr, double rho[3]) {
  if (chi <= dsqr) {
    rho[0] = chi;
    rho[1] = 1.;
    rho[2] = 0.;
  } else {
    const double sq = sqrt(chi);
    rho[0] = 2 * sq * delta - dsqr;
    rho[1] = delta / sq;
    rho[2] = -0.5 * rho[1] / chi;
  }
}

__global__ __launch_bounds__(LBS) void k_ba_errors(BaDev D, int recompute) {
  const int k = blockIdx.x * LBS + threadIdx.x;
  if (k >= D.na) return;
  const int e = D.act[k];
  double c2;
  if (recompute) {
    double err[3];
    edge_error(D, e, err, c2);
    D.eerr[3 * e] = err[0];
    D.eerr[3 * e + 1] = err[1];
    D.eerr[3 * e + 2] = err[2];
  } else {
    const double info = D.einfo[e];
    c2 = 0;
    for (int i = 0; i < (D.est[e] ? 3 : 2); i++) c2 += D.eerr[3 * e + i] * (info * D.eerr[3 * e + i]);
  }
  double chi = c2;
  if (D.erobust[e]) {
    double rho[3];
    huber(c2, D.edelta[e], D.edsqr[e], rho);
    chi = rho[0];
  }
  D.chi[k] = chi;
}

// Deterministic sum / max of n doubles into *out (one block).
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ in, int n, double* out, int op_max) {
  __shared__ double s[1024];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc = op_max ? fmax(acc, in[i]) : acc + in[i];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) s[threadIdx.x] = op_max ? fmax(s[threadIdx.x], s[threadIdx.x + o]) : s[threadIdx.x] + s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = s[0];
}

// constructQuadraticForm of one edge with DIM-dimensional error (2 mono, 3 stereo)
template <int DIM>
__device__ __forceinline__ void lin_accumulate(const BaDev& D, int k, int e, int c, const double* A, const double* Bm) {
  const double info = D.einfo[e];
  double omr[DIM], W = info;
#pragma unroll
  for (int i = 0; i < DIM; i++) omr[i] = -info * D.eerr[3 * e + i];
  if (D.erobust[e]) {
    double c2 = 0;
#pragma unroll
    for (int i = 0; i < DIM; i++) c2 += D.eerr[3 * e + i] * (info * D.eerr[3 * e + i]);
    double rho[3];
    huber(c2, D.edelta[e], D.edsqr[e], rho);
    W = rho[1] * info;
#pragma unroll
    for (int i = 0; i < DIM; i++) omr[i] *= rho[1];
  }
  double* pc = D.ptc + 12 * (size_t)k;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0;
#pragma unroll
    for (int d = 0; d < DIM; d++) s += A[3 * d + r] * omr[d];
    pc[9 + r] = s;
#pragma unroll
    for (int cc = 0; cc < 3; cc++) {
      double h = 0;
#pragma unroll
      for (int d = 0; d < DIM; d++) h += A[3 * d + r] * W * A[3 * d + cc];
      pc[3 * r + cc] = h;
    }
  }
  if (D.chidx[c] >= 0) {
    double* cm = D.cmc + 42 * (size_t)k;
    double* hp = D.Hpl + 18 * (size_t)k;
#pragma unroll
    for (int r = 0; r < 6; r++) {
      double s = 0;
#pragma unroll
      for (int d = 0; d < DIM; d++) s += Bm[6 * d + r] * omr[d];
      cm[36 + r] = s;
#pragma unroll
      for (int cc = 0; cc < 6; cc++) {
        double h = 0;
#pragma unroll
        for (int d = 0; d < DIM; d++) h += Bm[6 * d + r] * W * Bm[6 * d + cc];
        cm[6 * r + cc] = h;
      }
#pragma unroll
      for (int cc = 0; cc < 3; cc++) {
        double h = 0;
#pragma unroll
        for (int d = 0; d < DIM; d++) h += Bm[6 * d + r] * W * A[3 * d + cc];
        hp[3 * r + cc] = h;
      }
    }
  }
}

__global__ __launch_bounds__(LBS) void k_ba_linearize(BaDev D) {
  const int k = blockIdx.x * LBS + threadIdx.x;
  if (k >= D.na) return;
  const int e = D.act[k];
  const int c = D.ecam[e], p = D.ept[e];
  Quat q = {D.cq[4 * c], D.cq[4 * c + 1], D.cq[4 * c + 2], D.cq[4 * c + 3]};
  const double Xw[3] = {D.X[3 * p], D.X[3 * p + 1], D.X[3 * p + 2]};
  double Pc[3];
  qrot(q, Xw, Pc);
  for (int i = 0; i < 3; i++) Pc[i] += D.ct[3 * c + i];
  const double x = Pc[0], y = Pc[1], z = Pc[2], z_2 = z * z;
  double R[9];
  qmat(q, R);
  const double fx = D.intr[5 * c], fy = D.intr[5 * c + 1], bf = D.intr[5 * c + 4];
  const bool st = D.est[e];
  double A[9], Bm[18] = {};
  if (!st) {
    const double tmp[6] = {fx, 0, -x / z * fx, 0, fy, -y / z * fy};
    for (int r = 0; r < 2; r++)
      for (int cc = 0; cc < 3; cc++)
        A[3 * r + cc] = -1. / z * (tmp[3 * r] * R[cc] + tmp[3 * r + 1] * R[3 + cc] + tmp[3 * r + 2] * R[6 + cc]);
  } else {
    for (int cc = 0; cc < 3; cc++) {
      A[cc] = -fx * R[cc] / z + fx * x * R[6 + cc] / z_2;
      A[3 + cc] = -fy * R[3 + cc] / z + fy * y * R[6 + cc] / z_2;
      A[6 + cc] = A[cc] - bf * R[6 + cc] / z_2;
    }
  }
  Bm[0] = x * y / z_2 * fx;
  Bm[1] = -(1 + (x * x / z_2)) * fx;
  Bm[2] = y / z * fx;
  Bm[3] = -1. / z * fx;
  Bm[4] = 0;
  Bm[5] = x / z_2 * fx;
  Bm[6] = (1 + y * y / z_2) * fy;
  Bm[7] = -x * y / z_2 * fy;
  Bm[8] = -x / z * fy;
  Bm[9] = 0;
  Bm[10] = -1. / z * fy;
  Bm[11] = y / z_2 * fy;
  if (st) {
    Bm[12] = Bm[0] - bf * y / z_2;
    Bm[13] = Bm[1] + bf * x / z_2;
    Bm[14] = Bm[2];
    Bm[15] = Bm[3];
    Bm[16] = 0;
    Bm[17] = Bm[5] - bf / z_2;
  }
  if (st)
    lin_accumulate<3>(D, k, e, c, A, Bm);
  else
    lin_accumulate<2>(D, k, e, c, A, Bm);
}

__global__ __launch_bounds__(LBS) void k_ba_point_sum(BaDev D) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i >= D.npa) return;
  double h[12];
  for (int j = 0; j < 12; j++) h[j] = 0;
  for (int k = D.pt_off[i]; k < D.pt_off[i + 1]; k++) {
    const double* pc = D.ptc + 12 * (size_t)k;
    for (int j = 0; j < 12; j++) h[j] += pc[j];
  }
  for (int j = 0; j < 9; j++) D.Hll[9 * i + j] = h[j];
  for (int j = 0; j < 3; j++) D.bl[3 * i + j] = h[9 + j];
  D.dmax_p[i] = fmax(fmax(fabs(h[0]), fabs(h[4])), fabs(h[8]));
}

// one block per pose; thread j < 42 sums component j over the pose's edges in order
__global__ __launch_bounds__(64) void k_ba_cam_sum(BaDev D) {
  const int ci = blockIdx.x, j = threadIdx.x;
  __shared__ double dg[6];
  if (j < 42) {
    double s = 0;
    for (int t = D.cam_off[ci]; t < D.cam_off[ci + 1]; t++) s += D.cmc[42 * (size_t)D.cam_pos[t] + j];
    if (j < 36) D.Hpp[36 * ci + j] = s; else D.bp[6 * ci + (j - 36)] = s;
    if (j < 36 && (j % 7) == 0) dg[j / 7] = fabs(s);
  }
  __syncthreads();
  if (j == 0) {
    double m = 0;
    for (int r = 0; r < 6; r++) m = fmax(m, dg[r]);
    D.dmax_c[ci] = m;
  }
}

__global__ __launch_bounds__(LBS) void k_ba_point_schur(BaDev D, double lambda) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i >= D.npa) return;
  double Dm[9];
  for (int j = 0; j < 9; j++) Dm[j] = D.Hll[9 * i + j];
  Dm[0] += lambda;
  Dm[4] += lambda;
  Dm[8] += lambda;
  double Di[9];
  inv3(Dm, Di);
  for (int j = 0; j < 9; j++) D.Dinv[9 * i + j] = Di[j];
  const double b0 = D.bl[3 * i], b1 = D.bl[3 * i + 1], b2 = D.bl[3 * i + 2];
  double db[3];
  for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
  for (int k = D.pt_off[i]; k < D.pt_off[i + 1]; k++) {
    if (D.chidx[D.ecam[D.act[k]]] < 0) continue;
    const double* B1 = D.Hpl + 18 * (size_t)k;
    double* bd = D.BD + 18 * (size_t)k;
    for (int r = 0; r < 6; r++) {
      for (int c = 0; c < 3; c++) bd[3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
      D.cf[6 * (size_t)k + r] = B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
    }
  }
}

// One wave per Hschur block (c1 <= c2): lanes take pairs lane, lane+64, ...;
// every lane accumulates the 6x6 block, then a fixed shuffle tree sums lanes.
__global__ __launch_bounds__(64) void k_ba_pairs(BaDev D, double lambda) {
  const int b = blockIdx.x, lane = threadIdx.x;
  double acc[36];
  for (int j = 0; j < 36; j++) acc[j] = 0;
  for (int t = D.blk_off[b] + lane; t < D.blk_off[b + 1]; t += 64) {
    const int2 pr = D.pairs[t];
    const double* bd = D.BD + 18 * (size_t)pr.x;
    const double* h2 = D.Hpl + 18 * (size_t)pr.y;
    double A[18], Bv[18];
    for (int j = 0; j < 18; j++) {
      A[j] = bd[j];
      Bv[j] = h2[j];
    }
    for (int r = 0; r < 6; r++)
      for (int c = 0; c < 6; c++) acc[6 * r + c] += A[3 * r] * Bv[3 * c] + A[3 * r + 1] * Bv[3 * c + 1] + A[3 * r + 2] * Bv[3 * c + 2];
  }
  for (int j = 0; j < 36; j++) {
    double v = acc[j];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    acc[j] = v;
  }
  if (lane < 36) {
    const int2 cc = D.blk_cc[b];
    const int N = 6 * D.nposes;
    const int r = lane / 6, c = lane % 6;
    double v = 0;
#pragma unroll
    for (int j = 0; j < 36; j++)
      if (j == lane) v = acc[j];
    double s;
    if (cc.x == cc.y) {
      s = D.Hpp[36 * cc.x + lane] + (r == c ? lambda : 0.0) - v;
    } else {
      s = -v;
      D.S[(size_t)(6 * cc.y + c) * N + 6 * cc.x + r] = s;
    }
    D.S[(size_t)(6 * cc.x + r) * N + 6 * cc.y + c] = s;
  }
}

__global__ __launch_bounds__(64) void k_ba_cam_coef(BaDev D) {
  const int ci = blockIdx.x, j = threadIdx.x;
  if (j >= 6) return;
  double s = 0;
  for (int t = D.cam_off[ci]; t < D.cam_off[ci + 1]; t++) s += D.cf[6 * (size_t)D.cam_pos[t] + j];
  D.bs[6 * ci + j] = D.bp[6 * ci + j] - s;
}

// Dense LDLT (no pivoting; fails on an exactly zero pivot like Eigen's
// SimplicialLDLT) of the N x N reduced camera system, right-looking: per
// column j, scale the column by 1/d_j then a rank-1 update of the trailing
// lower triangle, all threads; then column-oriented triangular solves.
// A lives in LDS when it fits, else in place in global memory.
__global__ __launch_bounds__(1024) void k_ba_ldlt(BaDev D, int in_lds) {
  extern __shared__ double sm[];
  const int N = 6 * D.nposes, tid = threadIdx.x, nt = blockDim.x;
  double* y = sm;
  double* w = sm + N;
  double* A = in_lds ? sm + 2 * N : D.S;
  if (in_lds)
    for (int i = tid; i < N * N; i += nt) A[i] = D.S[i];
  for (int i = tid; i < N; i += nt) y[i] = D.bs[i];
  __syncthreads();
  for (int j = 0; j < N; j++) {
    const double d = A[(size_t)j * N + j];
    if (d == 0.0) {  // uniform: every thread reads the same value
      if (tid == 0) D.scal[2] = 0.0;
      return;
    }
    for (int i = j + 1 + tid; i < N; i += nt) {
      const double a = A[(size_t)i * N + j];
      w[i] = a;
      A[(size_t)i * N + j] = a / d;
    }
    __syncthreads();
    const int M = N - j - 1;
    for (int t = tid; t < M * M; t += nt) {
      const int i = j + 1 + t / M, k = j + 1 + t % M;
      if (k <= i) A[(size_t)i * N + k] -= A[(size_t)i * N + j] * w[k];
    }
    __syncthreads();
  }
  // L z = b
  for (int i = 0; i < N; i++) {
    const double yi = y[i];
    for (int k = i + 1 + tid; k < N; k += nt) y[k] -= A[(size_t)k * N + i] * yi;
    __syncthreads();
  }
  for (int i = tid; i < N; i += nt) y[i] /= A[(size_t)i * N + i];
  __syncthreads();
  // L^T x = z
  for (int i = N - 1; i >= 0; i--) {
    const double xi = y[i];
    for (int k = tid; k < i; k += nt) y[k] -= A[(size_t)i * N + k] * xi;
    __syncthreads();
  }
  for (int i = tid; i < N; i += nt) D.xp[i] = y[i];
  if (tid == 0) D.scal[2] = 1.0;
}

// back-substitution + update (push first) + LM scale terms
__global__ __launch_bounds__(LBS) void k_ba_update(BaDev D, double lambda) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i < D.npa) {
    double c[3] = {D.bl[3 * i], D.bl[3 * i + 1], D.bl[3 * i + 2]};
    for (int k = D.pt_off[i]; k < D.pt_off[i + 1]; k++) {
      const int ci = D.chidx[D.ecam[D.act[k]]];
      if (ci < 0) continue;
      const double* B = D.Hpl + 18 * (size_t)k;
      for (int j = 0; j < 3; j++)
        for (int r = 0; r < 6; r++) c[j] -= B[3 * r + j] * D.xp[6 * ci + r];
    }
    const double* Di = D.Dinv + 9 * (size_t)i;
    double x[3];
    for (int r = 0; r < 3; r++) x[r] = Di[3 * r] * c[0] + Di[3 * r + 1] * c[1] + Di[3 * r + 2] * c[2];
    const int p = D.pt_id[i];
    double sc = 0;
    for (int r = 0; r < 3; r++) {
      D.Xbak[3 * p + r] = D.X[3 * p + r];
      D.X[3 * p + r] += x[r];
      D.xl[3 * i + r] = x[r];
      sc += x[r] * (lambda * x[r] + D.bl[3 * i + r]);
    }
    D.scale_p[i] = sc;
  } else if (i < D.npa + D.nposes) {
    const int pi = i - D.npa;
    const int c = D.pose_cam[pi];
    double u[6];
    double sc = 0;
    for (int r = 0; r < 6; r++) {
      u[r] = D.xp[6 * pi + r];
      sc += u[r] * (lambda * u[r] + D.bp[6 * pi + r]);
    }
    D.scale_c[pi] = sc;
    for (int r = 0; r < 4; r++) D.cbak[7 * c + r] = D.cq[4 * c + r];
    for (int r = 0; r < 3; r++) D.cbak[7 * c + 4 + r] = D.ct[3 * c + r];
    const SE3d E = se3_exp(u);
    const Quat q = {D.cq[4 * c], D.cq[4 * c + 1], D.cq[4 * c + 2], D.cq[4 * c + 3]};
    const double t[3] = {D.ct[3 * c], D.ct[3 * c + 1], D.ct[3 * c + 2]};
    double rt[3];
    qrot(E.q, t, rt);
    Quat nq = qmul(E.q, q);
    qnormalize(nq);
    D.cq[4 * c] = nq.x;
    D.cq[4 * c + 1] = nq.y;
    D.cq[4 * c + 2] = nq.z;
    D.cq[4 * c + 3] = nq.w;
    for (int r = 0; r < 3; r++) D.ct[3 * c + r] = E.t[r] + rt[r];
  }
}

__global__ __launch_bounds__(LBS) void k_ba_restore(BaDev D) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i < D.npa) {
    const int p = D.pt_id[i];
    for (int r = 0; r < 3; r++) D.X[3 * p + r] = D.Xbak[3 * p + r];
  } else if (i < D.npa + D.nposes) {
    const int c = D.pose_cam[i - D.npa];
    for (int r = 0; r < 4; r++) D.cq[4 * c + r] = D.cbak[7 * c + r];
    for (int r = 0; r < 3; r++) D.ct[3 * c + r] = D.cbak[7 * c + 4 + r];
  }
}

// phase transition (:764-802) and the final erase test (:817-847): per edge
// chi2 of its stored error against th, and depth of the current estimate
__global__ __launch_bounds__(LBS) void k_ba_outliers(BaDev D, uint8_t* flag, int drop_kernel) {
  const int e = blockIdx.x * LBS + threadIdx.x;
  if (e >= D.ne) return;
  const int c = D.ecam[e], p = D.ept[e];
  const double info = D.einfo[e];
  double c2 = 0;
  const int Dm = D.est[e] ? 3 : 2;
  for (int i = 0; i < Dm; i++) c2 += D.eerr[3 * e + i] * (info * D.eerr[3 * e + i]);
  Quat q = {D.cq[4 * c], D.cq[4 * c + 1], D.cq[4 * c + 2], D.cq[4 * c + 3]};
  const double Xw[3] = {D.X[3 * p], D.X[3 * p + 1], D.X[3 * p + 2]};
  double Pc[3];
  qrot(q, Xw, Pc);
  const double z = Pc[2] + D.ct[3 * c + 2];
  const double th = D.est[e] ? 7.815 : 5.991;
  flag[e] = (c2 > th || !(z > 0.0)) ? 1 : 0;
  if (drop_kernel) D.erobust[e] = 0;
}

__global__ __launch_bounds__(LBS) void k_ba_export(BaDev D, float* Tcw, float* Xw, double* Tcw_d, double* Xw_d) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i < D.nc) {
    const Quat q = {D.cq[4 * i], D.cq[4 * i + 1], D.cq[4 * i + 2], D.cq[4 * i + 3]};
    double R[9];
    qmat(q, R);
    for (int r = 0; r < 3; r++) {
      for (int k = 0; k < 3; k++) {
        Tcw[12 * i + 4 * r + k] = (float)R[3 * r + k];
        if (Tcw_d) Tcw_d[12 * i + 4 * r + k] = R[3 * r + k];
      }
      Tcw[12 * i + 4 * r + 3] = (float)D.ct[3 * i + r];
      if (Tcw_d) Tcw_d[12 * i + 4 * r + 3] = D.ct[3 * i + r];
    }
  }
  if (i < D.np) {
    for (int r = 0; r < 3; r++) {
      Xw[3 * i + r] = (float)D.X[3 * i + r];
      if (Xw_d) Xw_d[3 * i + r] = D.X[3 * i + r];
    }
  }
}

// ------------------------------------------------------------------ host

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t count) {
    if (count <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    hipError_t e = hipMalloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T));
    if (e == hipSuccess) n = std::max<size_t>(count, 1);
    return e;
  }
  hipError_t put(const std::vector<T>& v) {
    hipError_t e = alloc(v.size());
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  }
};

struct Ctx {
  DBuf<double> cq, ct, cbak, intr, X, Xbak, eobs, einfo, edelta, eerr, Hpl, ptc, cmc, BD, cf, chi, Hll, bl, Dinv, xl,
      dmax_p, scale_p, Hpp, bp, xp, bs, S, scal;
  DBuf<int> chidx, ept, ecam, act, pt_off, pt_id, cam_pos, cam_off, pose_cam, blk_off;
  DBuf<int2> blk_cc, pairs;
  DBuf<uint8_t> est, erobust, flag;
  DBuf<float> edsqr, Tcw_out, Xw_out;
  DBuf<double> Tcw_d_out, Xw_d_out;
};

#define BA_CHECK(x)                          \
  do {                                       \
    if ((x) != hipSuccess) return ORBX_ERR_HIP; \
  } while (0)

struct LocalBA {
  BaDev D{};
  Ctx c;  // device buffers, kept across calls (grow only)
  std::vector<int> e_pt, e_cam;
  std::vector<uint8_t> e_st, fixed;
  std::vector<uint8_t> level;  // 0/1 per edge
  int trials = 0;

  // Active set of a phase: SparseOptimizer::initializeOptimization(level) +
  // buildIndexMapping; point-major positions, pose groups, Schur pair blocks.
  orbx_status build_structure(int lvl) {
    const int nc = D.nc, np = D.np, ne = D.ne;
    std::vector<int> act;
    std::vector<char> cam_used(nc, 0), pt_used(np, 0);
    std::vector<std::vector<int>> by_pt(np);
    for (int e = 0; e < ne; e++) {
      if (lvl >= 0 && level[e] != lvl) continue;
      by_pt[e_pt[e]].push_back(e);
      cam_used[e_cam[e]] = 1;
      pt_used[e_pt[e]] = 1;
    }
    std::vector<int> chidx(nc, -1), pose_cam;
    for (int c = 0; c < nc; c++)
      if (cam_used[c] && !fixed[c]) {
        chidx[c] = (int)pose_cam.size();
        pose_cam.push_back(c);
      }
    const int nposes = (int)pose_cam.size();
    std::vector<int> pt_off(1, 0), pt_id;
    for (int p = 0; p < np; p++) {
      if (!pt_used[p]) continue;
      for (int e : by_pt[p]) act.push_back(e);
      pt_id.push_back(p);
      pt_off.push_back((int)act.size());
    }
    const int na = (int)act.size(), npa = (int)pt_id.size();
    std::vector<std::vector<int>> by_cam(nposes);
    for (int k = 0; k < na; k++) {
      const int ci = chidx[e_cam[act[k]]];
      if (ci >= 0) by_cam[ci].push_back(k);
    }
    std::vector<int> cam_off(1, 0), cam_pos;
    for (int ci = 0; ci < nposes; ci++) {
      cam_pos.insert(cam_pos.end(), by_cam[ci].begin(), by_cam[ci].end());
      cam_off.push_back((int)cam_pos.size());
    }
    // pair blocks (c1 <= c2), pairs ordered by point then edge order
    std::vector<std::vector<int2>> blk((size_t)nposes * nposes);
    for (int i = 0; i < npa; i++) {
      for (int k1 = pt_off[i]; k1 < pt_off[i + 1]; k1++) {
        const int c1 = chidx[e_cam[act[k1]]];
        if (c1 < 0) continue;
        for (int k2 = pt_off[i]; k2 < pt_off[i + 1]; k2++) {
          const int c2 = chidx[e_cam[act[k2]]];
          if (c2 < 0 || c2 < c1) continue;
          blk[(size_t)c1 * nposes + c2].push_back(make_int2(k1, k2));
        }
      }
    }
    std::vector<int> blk_off(1, 0);
    std::vector<int2> blk_cc, pairs;
    for (int c1 = 0; c1 < nposes; c1++)
      for (int c2 = c1; c2 < nposes; c2++) {
        const auto& v = blk[(size_t)c1 * nposes + c2];
        if (v.empty() && c1 != c2) continue;
        pairs.insert(pairs.end(), v.begin(), v.end());
        blk_off.push_back((int)pairs.size());
        blk_cc.push_back(make_int2(c1, c2));
      }
    BA_CHECK(c.act.put(act));
    BA_CHECK(c.chidx.put(chidx));
    BA_CHECK(c.pose_cam.put(pose_cam));
    BA_CHECK(c.pt_off.put(pt_off));
    BA_CHECK(c.pt_id.put(pt_id));
    BA_CHECK(c.cam_off.put(cam_off));
    BA_CHECK(c.cam_pos.put(cam_pos));
    BA_CHECK(c.blk_off.put(blk_off));
    BA_CHECK(c.blk_cc.put(blk_cc));
    BA_CHECK(c.pairs.put(pairs));
    const size_t N = 6 * (size_t)nposes;
    BA_CHECK(c.Hpl.alloc(18 * (size_t)na));
    BA_CHECK(c.ptc.alloc(12 * (size_t)na));
    BA_CHECK(c.cmc.alloc(42 * (size_t)na));
    BA_CHECK(c.BD.alloc(18 * (size_t)na));
    BA_CHECK(c.cf.alloc(6 * (size_t)na));
    BA_CHECK(c.chi.alloc(na));
    BA_CHECK(c.Hll.alloc(9 * (size_t)npa));
    BA_CHECK(c.bl.alloc(3 * (size_t)npa));
    BA_CHECK(c.Dinv.alloc(9 * (size_t)npa));
    BA_CHECK(c.xl.alloc(3 * (size_t)npa));
    BA_CHECK(c.dmax_p.alloc(npa + nposes));
    BA_CHECK(c.scale_p.alloc(npa + nposes));
    BA_CHECK(c.Hpp.alloc(36 * (size_t)nposes));
    BA_CHECK(c.bp.alloc(N));
    BA_CHECK(c.xp.alloc(N));
    BA_CHECK(c.bs.alloc(N));
    BA_CHECK(c.S.alloc(N * N));
    D.na = na;
    D.npa = npa;
    D.nposes = nposes;
    D.nblk = (int)blk_cc.size();
    D.act = c.act.p;
    D.chidx = c.chidx.p;
    D.pose_cam = c.pose_cam.p;
    D.pt_off = c.pt_off.p;
    D.pt_id = c.pt_id.p;
    D.cam_off = c.cam_off.p;
    D.cam_pos = c.cam_pos.p;
    D.blk_off = c.blk_off.p;
    D.blk_cc = c.blk_cc.p;
    D.pairs = c.pairs.p;
    D.Hpl = c.Hpl.p;
    D.ptc = c.ptc.p;
    D.cmc = c.cmc.p;
    D.BD = c.BD.p;
    D.cf = c.cf.p;
    D.chi = c.chi.p;
    D.Hll = c.Hll.p;
    D.bl = c.bl.p;
    D.Dinv = c.Dinv.p;
    D.xl = c.xl.p;
    D.scale_p = c.scale_p.p;
    D.scale_c = c.scale_p.p + npa;  // contiguous with the point terms for one reduction
    D.Hpp = c.Hpp.p;
    D.bp = c.bp.p;
    D.xp = c.xp.p;
    D.bs = c.bs.p;
    D.S = c.S.p;
    D.dmax_p = c.dmax_p.p;
    D.dmax_c = c.dmax_p.p + npa;  // contiguous: one max-reduction for lambda init
    return ORBX_OK;
  }

  hipError_t errors(hipStream_t st, int recompute = 1) {
    if (D.na > 0) hipLaunchKernelGGL(k_ba_errors, dim3((D.na + LBS - 1) / LBS), dim3(LBS), 0, st, D, recompute);
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, st, D.chi, D.na, D.scal + 0, 0);
    return hipGetLastError();
  }

  hipError_t read_scalars(double out[4], hipStream_t st) {
    hipError_t e = hipMemcpyAsync(out, D.scal, 4 * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
  }

  // OptimizationAlgorithmLevenberg::solve (+ optimize loop); returns iterations
  orbx_status optimize(int iterations, const volatile int* stop, hipStream_t st, int* iters, double* final_chi) {
    double lambda = 0, ni = 2;
    int nBad = 0;
    int it = 0;
    const size_t N = 6 * (size_t)D.nposes;
    const int in_lds = (N * N + 2 * N) * sizeof(double) <= 160 * 1024;
    const size_t ldlt_smem = (in_lds ? N * N + 2 * N : 2 * N) * sizeof(double);
    if (ldlt_smem > 160 * 1024) return ORBX_ERR_SIZE;
    if (hipFuncSetAttribute((const void*)k_ba_ldlt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldlt_smem) !=
        hipSuccess)
      return ORBX_ERR_HIP;
    const int gp = (D.npa + D.nposes + LBS - 1) / LBS;
    double sc[4];
    for (int i = 0; i < iterations && !(stop && *stop); i++) {
      BA_CHECK(errors(st));
      if (D.na > 0) hipLaunchKernelGGL(k_ba_linearize, dim3((D.na + LBS - 1) / LBS), dim3(LBS), 0, st, D);
      if (D.npa > 0) hipLaunchKernelGGL(k_ba_point_sum, dim3((D.npa + LBS - 1) / LBS), dim3(LBS), 0, st, D);
      if (D.nposes > 0) hipLaunchKernelGGL(k_ba_cam_sum, dim3(D.nposes), dim3(64), 0, st, D);
      if (i == 0) hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, st, D.dmax_p, D.npa + D.nposes, D.scal + 3, 1);
      BA_CHECK(hipGetLastError());
      BA_CHECK(read_scalars(sc, st));
      double currentChi = sc[0];
      const double iniChi = currentChi;
      if (i == 0) {
        lambda = 1e-5 * sc[3];  // computeLambdaInit: tau * max |H_jj|
        ni = 2;
        nBad = 0;
      }
      double rho = 0;
      int qmax = 0;
      do {
        if (D.npa > 0) hipLaunchKernelGGL(k_ba_point_schur, dim3((D.npa + LBS - 1) / LBS), dim3(LBS), 0, st, D, lambda);
        if (D.nposes > 0) {
          BA_CHECK(hipMemsetAsync(D.S, 0, N * N * sizeof(double), st));
          hipLaunchKernelGGL(k_ba_pairs, dim3(D.nblk), dim3(64), 0, st, D, lambda);
          hipLaunchKernelGGL(k_ba_cam_coef, dim3(D.nposes), dim3(64), 0, st, D);
          hipLaunchKernelGGL(k_ba_ldlt, dim3(1), dim3(1024), ldlt_smem, st, D, in_lds);
        } else {
          const double one = 1.0;
          BA_CHECK(hipMemcpyAsync(D.scal + 2, &one, sizeof(double), hipMemcpyHostToDevice, st));
        }
        BA_CHECK(hipGetLastError());
        BA_CHECK(read_scalars(sc, st));
        const bool ok2 = sc[2] != 0.0;
        double tempChi, scale = 0;
        trials++;
        if (ok2) {
          hipLaunchKernelGGL(k_ba_update, dim3(std::max(gp, 1)), dim3(LBS), 0, st, D, lambda);
          hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, st, D.scale_p, D.npa + D.nposes, D.scal + 1, 0);
          BA_CHECK(errors(st));
          BA_CHECK(read_scalars(sc, st));
          tempChi = sc[0];
          scale = sc[1];
        } else {
          BA_CHECK(errors(st));
          tempChi = std::numeric_limits<double>::max();
        }
        rho = currentChi - tempChi;
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
          if (ok2) hipLaunchKernelGGL(k_ba_restore, dim3(std::max(gp, 1)), dim3(LBS), 0, st, D);
          BA_CHECK(hipGetLastError());
        }
        qmax++;
      } while (rho < 0 && qmax < 10 && !(stop && *stop));
      ++it;
      if (qmax == 10 || rho == 0) break;
      if ((iniChi - currentChi) * 1e3 < iniChi)
        nBad++;
      else
        nBad = 0;
      if (nBad >= 3) break;
    }
    *iters = it;
    BA_CHECK(errors(st, 0));  // activeRobustChi2 of the stored errors
    BA_CHECK(read_scalars(sc, st));
    if (final_chi) *final_chi = sc[0];
    return ORBX_OK;
  }
};

orbx_status run_local_ba(LocalBA& L, const orbx_ba_problem* pb, orbx_ba_result* res, const volatile int* stop,
                         hipStream_t st) {
  L.trials = 0;
  BaDev& D = L.D;
  Ctx& c = L.c;
  const int nc = pb->n_cams, np = pb->n_points, ne = pb->n_edges;
  D.nc = nc;
  D.np = np;
  D.ne = ne;
  // vertices: Converter::toSE3Quat (float -> double, Quaterniond(R), normalize)
  std::vector<double> cq(4 * (size_t)nc), ct(3 * (size_t)nc), intr(5 * (size_t)nc), X(3 * (size_t)np);
  L.fixed.assign(nc, 0);
  for (int i = 0; i < nc; i++) {
    const float* T = pb->Tcw + 12 * i;
    const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    Quat q = mat2q(R);
    qnormalize(q);
    cq[4 * i] = q.x;
    cq[4 * i + 1] = q.y;
    cq[4 * i + 2] = q.z;
    cq[4 * i + 3] = q.w;
    ct[3 * i] = T[3];
    ct[3 * i + 1] = T[7];
    ct[3 * i + 2] = T[11];
    for (int k = 0; k < 5; k++) intr[5 * i + k] = pb->intr[5 * i + k];
    L.fixed[i] = pb->fixed ? pb->fixed[i] : 0;
  }
  for (int i = 0; i < 3 * np; i++) X[i] = pb->Xw[i];
  L.e_pt.assign(pb->edge_point, pb->edge_point + ne);
  L.e_cam.assign(pb->edge_cam, pb->edge_cam + ne);
  for (int e = 0; e < ne; e++) {
    if (L.e_pt[e] < 0 || L.e_pt[e] >= np || L.e_cam[e] < 0 || L.e_cam[e] >= nc) return ORBX_ERR_ARG;
  }
  std::vector<double> eobs(3 * (size_t)ne), einfo(ne), edelta(ne);
  std::vector<float> edsqr(ne);
  L.e_st.resize(ne);
  std::vector<uint8_t> erob(ne, 1);
  const float thMono = std::sqrt(5.991f), thStereo = std::sqrt(7.815f);  // src/Optimizer.cc:653-654
  for (int e = 0; e < ne; e++) {
    L.e_st[e] = pb->obs[3 * e + 2] >= 0 ? 1 : 0;
    for (int k = 0; k < 3; k++) eobs[3 * e + k] = pb->obs[3 * e + k];
    einfo[e] = pb->inv_sigma2[e];
    edelta[e] = L.e_st[e] ? thStereo : thMono;
    edsqr[e] = (float)(edelta[e] * edelta[e]);
  }
  BA_CHECK(c.cq.put(cq));
  BA_CHECK(c.ct.put(ct));
  BA_CHECK(c.cbak.alloc(7 * (size_t)nc));
  BA_CHECK(c.intr.put(intr));
  BA_CHECK(c.X.put(X));
  BA_CHECK(c.Xbak.alloc(3 * (size_t)np));
  BA_CHECK(c.ept.put(L.e_pt));
  BA_CHECK(c.ecam.put(L.e_cam));
  BA_CHECK(c.est.put(L.e_st));
  BA_CHECK(c.eobs.put(eobs));
  BA_CHECK(c.einfo.put(einfo));
  BA_CHECK(c.edelta.put(edelta));
  BA_CHECK(c.edsqr.put(edsqr));
  BA_CHECK(c.erobust.put(erob));
  BA_CHECK(c.eerr.alloc(3 * (size_t)ne));
  BA_CHECK(hipMemsetAsync(c.eerr.p, 0, 3 * sizeof(double) * std::max(ne, 1), st));
  BA_CHECK(c.flag.alloc(ne));
  BA_CHECK(c.scal.alloc(4));
  D.cq = c.cq.p;
  D.ct = c.ct.p;
  D.cbak = c.cbak.p;
  D.intr = c.intr.p;
  D.X = c.X.p;
  D.Xbak = c.Xbak.p;
  D.ept = c.ept.p;
  D.ecam = c.ecam.p;
  D.est = c.est.p;
  D.eobs = c.eobs.p;
  D.einfo = c.einfo.p;
  D.edelta = c.edelta.p;
  D.edsqr = c.edsqr.p;
  D.erobust = c.erobust.p;
  D.eerr = c.eerr.p;
  D.scal = c.scal.p;
  res->iterations[0] = res->iterations[1] = 0;
  res->trials = 0;
  res->chi2[0] = res->chi2[1] = 0;
  const int ge = (ne + LBS - 1) / LBS;
  bool ran = false;
  if (!(stop && *stop)) {  // src/Optimizer.cc:749-751
    ran = true;
    L.level.assign(ne, 0);
    orbx_status s = L.build_structure(-1);
    if (s != ORBX_OK) return s;
    s = L.optimize(5, stop, st, &res->iterations[0], &res->chi2[0]);
    if (s != ORBX_OK) return s;
    if (!(stop && *stop)) {
      // :764-802 level-1 outliers, drop robust kernels
      if (ne > 0) hipLaunchKernelGGL(k_ba_outliers, dim3(ge), dim3(LBS), 0, st, D, c.flag.p, 1);
      BA_CHECK(hipGetLastError());
      BA_CHECK(hipMemcpyAsync(L.level.data(), c.flag.p, ne, hipMemcpyDeviceToHost, st));
      BA_CHECK(hipStreamSynchronize(st));
      s = L.build_structure(0);
      if (s != ORBX_OK) return s;
      s = L.optimize(10, stop, st, &res->iterations[1], &res->chi2[1]);
      if (s != ORBX_OK) return s;
    }
  }
  res->trials = L.trials;
  if (!ran) {  // src/Optimizer.cc:749-751: return before any write-back
    std::memcpy(res->Tcw, pb->Tcw, sizeof(float) * 12 * nc);
    std::memcpy(res->Xw, pb->Xw, sizeof(float) * 3 * np);
    if (ne > 0) std::memset(res->edge_outlier, 0, ne);
    if (res->Tcw_d)
      for (int i = 0; i < 12 * nc; i++) res->Tcw_d[i] = pb->Tcw[i];
    if (res->Xw_d)
      for (int i = 0; i < 3 * np; i++) res->Xw_d[i] = pb->Xw[i];
    return ORBX_OK;
  }
  // :817-847 vToErase
  if (ne > 0) {
    hipLaunchKernelGGL(k_ba_outliers, dim3(ge), dim3(LBS), 0, st, D, c.flag.p, 0);
    BA_CHECK(hipGetLastError());
    BA_CHECK(hipMemcpyAsync(res->edge_outlier, c.flag.p, ne, hipMemcpyDeviceToHost, st));
  }
  BA_CHECK(c.Tcw_out.alloc(12 * (size_t)nc));
  BA_CHECK(c.Xw_out.alloc(3 * (size_t)np));
  if (res->Tcw_d) BA_CHECK(c.Tcw_d_out.alloc(12 * (size_t)nc));
  if (res->Xw_d) BA_CHECK(c.Xw_d_out.alloc(3 * (size_t)np));
  const int gx = (std::max(nc, np) + LBS - 1) / LBS;
  hipLaunchKernelGGL(k_ba_export, dim3(std::max(gx, 1)), dim3(LBS), 0, st, D, c.Tcw_out.p, c.Xw_out.p,
                     res->Tcw_d ? c.Tcw_d_out.p : nullptr, res->Xw_d ? c.Xw_d_out.p : nullptr);
  BA_CHECK(hipGetLastError());
  BA_CHECK(hipMemcpyAsync(res->Tcw, c.Tcw_out.p, 12 * sizeof(float) * nc, hipMemcpyDeviceToHost, st));
  BA_CHECK(hipMemcpyAsync(res->Xw, c.Xw_out.p, 3 * sizeof(float) * np, hipMemcpyDeviceToHost, st));
  if (res->Tcw_d) BA_CHECK(hipMemcpyAsync(res->Tcw_d, c.Tcw_d_out.p, 12 * sizeof(double) * nc, hipMemcpyDeviceToHost, st));
  if (res->Xw_d) BA_CHECK(hipMemcpyAsync(res->Xw_d, c.Xw_d_out.p, 3 * sizeof(double) * np, hipMemcpyDeviceToHost, st));
  BA_CHECK(hipStreamSynchronize(st));
  return ORBX_OK;
}

}  // namespace orbx

struct orbx_ba {
  int device = 0;
  hipStream_t st = nullptr;
  orbx::LocalBA L;
};

extern "C" {

orbx_status orbx_ba_create(int device, orbx_ba** out) {
  if (!out) return ORBX_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= n) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  orbx_ba* h = new (std::nothrow) orbx_ba();
  if (!h) return ORBX_ERR_HIP;
  h->device = device;
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return ORBX_ERR_HIP;
  }
  *out = h;
  return ORBX_OK;
}

orbx_status orbx_ba_destroy(orbx_ba* h) {
  if (!h) return ORBX_ERR_ARG;
  (void)hipSetDevice(h->device);
  if (h->st) (void)hipStreamDestroy(h->st);
  delete h;
  return ORBX_OK;
}

orbx_status orbx_ba_run(orbx_ba* h, const orbx_ba_problem* p, orbx_ba_result* r, const volatile int* stop_flag) {
  if (!h || !p || !r) return ORBX_ERR_ARG;
  if (p->n_cams < 0 || p->n_points < 0 || p->n_edges < 0) return ORBX_ERR_ARG;
  if (p->n_cams > 0 && (!p->Tcw || !p->intr || !r->Tcw)) return ORBX_ERR_ARG;
  if (p->n_points > 0 && (!p->Xw || !r->Xw)) return ORBX_ERR_ARG;
  if (p->n_edges > 0 && (!p->edge_point || !p->edge_cam || !p->obs || !p->inv_sigma2 || !r->edge_outlier))
    return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  return orbx::run_local_ba(h->L, p, r, stop_flag, h->st);
}

orbx_status orbx_local_ba(const orbx_ba_problem* p, orbx_ba_result* r, const volatile int* stop_flag, int device) {
  orbx_ba* h = nullptr;
  orbx_status s = orbx_ba_create(device, &h);
  if (s != ORBX_OK) return s;
  s = orbx_ba_run(h, p, r, stop_flag);
  orbx_ba_destroy(h);
  return s;
}

}  // extern "C"
