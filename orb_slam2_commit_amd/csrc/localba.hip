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
//   k_ba_cam_sum     Hpp, bp per pose: chunk partials (pose lists split over blocks)
//   k_ba_cam_fin     chunk partials -> Hpp, bp, max |Hpp_jj| (chunk order; batched driver --
//                    the single-problem entry does it inside k_ba_lm_start)
//   per trial:
//   k_ba_point_schur D = Hll + lambda I, Dinv (cofactor inverse), BD_e = Hpl_e Dinv, cf_e = Hpl_e Dinv bl
//   k_ba_pairs       chunk partials of sum_points BD_e1 Hpl_e2^T per Hschur block
//                    (pairs from the per-phase k_ba_pair_table) and of sum_e cf_e per pose
//   k_ba_schur_fin   S block (c1,c2) = [c1==c2](Hpp+lambda I) - pair sum; bschur = bp - sum cf
//   k_ba_ldlt        dense LDLT of the reduced camera system in LDS, solve
//   k_ba_update      x_l = Dinv (bl - sum_e Hpl_e^T x_p), X += x_l; T = exp(x_p) T; scale terms
//   k_ba_errors_ctl  new chi (block partials), then the LM verdict in the launch's last block
//                    (k_ba_lm_control's body): partials summed in block order, accept/reject,
//                    lambda/ni, trial budget, _nBad, stop flag polled through host-mapped
//                    memory; gates the next trial's kernels
// Every reduction has a fixed partition and order: results are run-to-run
// identical.  The one cross-block hand-off (k_ba_errors_ctl) uses write-through
// partials and a relaxed ticket, not an agent-scope release/acquire (per block
// that costs an L2 writeback/invalidate on the multi-XCD part).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/orbx.h"
#include "../../include/orbx_debug.h"
#include "orbx_device.h"

namespace orbx {
// Debug / test options of the solver handle running on this thread (orbx_debug_ba_options); the
// production default is all-off.  Set for the duration of an orbx_ba_run* call (BaOptScope).
inline const orbx_ba_debug_options& ba_opts();
}  // namespace orbx

namespace orbx {

// The reference's pbStopFlag (bool*, src/Optimizer.cc:530, set by LocalMapping::InterruptBA) or an
// int mirror of it; polled before the run and between LM trials (SparseOptimizer::terminate()).
struct StopFlag {
  const volatile int* i = nullptr;
  const volatile bool* b = nullptr;
  bool operator()() const { return (i && *i) || (b && *b); }
};


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
    // the three cases spelled out on named entries: no array indexed at run time (which put the
    // matrix in scratch memory); same arithmetic as c[i], c[j], c[k] with (i, j, k) cyclic
    if (i == 0) {  // (0, 1, 2)
      t = sqrt(m[0] - m[4] - m[8] + 1.0);
      const double ci = 0.5 * t;
      t = 0.5 / t;
      q.w = (m[7] - m[5]) * t;
      q.x = ci;
      q.y = (m[3] + m[1]) * t;
      q.z = (m[6] + m[2]) * t;
    } else if (i == 1) {  // (1, 2, 0)
      t = sqrt(m[4] - m[8] - m[0] + 1.0);
      const double ci = 0.5 * t;
      t = 0.5 / t;
      q.w = (m[2] - m[6]) * t;
      q.y = ci;
      q.z = (m[7] + m[5]) * t;
      q.x = (m[1] + m[3]) * t;
    } else {  // (2, 0, 1)
      t = sqrt(m[8] - m[0] - m[4] + 1.0);
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
constexpr int LBS = 256;

// Levenberg-Marquardt control of one optimize() call kept on the device
// (OptimizationAlgorithmLevenberg::solve + the _nBad rule, Appendix B of
// SURVEY): k_ba_lm_control updates it after every trial, and the trial's
// kernels read lambda and the gates from it, so a phase runs without a host
// round trip per trial.
struct LmState {
  double lambda, ni, currentChi, iniChi;
  int it, qmax, nBad, trials;
  int relin;       // the next trial starts a new iteration: linearise first
  int done;        // the phase has ended: every gated kernel returns at once
  int rejected;    // the last trial was rejected after a successful solve: restore
  int iterations;  // the phase's iteration budget
  int stopped;     // the stop flag was seen
  int refresh;     // an iteration ended on a rejected trial (rho NaN) and the phase goes on: the
                   // phase pauses (done) until the host pops the trial, recomputes the errors at
                   // the restored state and resumes (k_ba_lm_resume), as g2o's next iteration does
  double final_chi;  // batched driver: activeRobustChi2 of the stored errors at the phase end
  unsigned ticket;   // k_ba_errors_ctl: blocks of the current launch that have stored their partial
};

// rho's cube rounded once (std::pow(x, 3) in the reference; glibc's pow is
// within 0.52 ulp): x^2 and x^2*x split exactly with fma, host and device alike
__host__ __device__ inline double lm_cube(double x) {
  const double p = x * x, pe = fma(x, x, -p);
  const double c = p * x, ce = fma(p, x, -c);
  return c + (ce + pe * x);
}

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
  int* pcam;       // na: pose index of position k (-1: fixed camera)
  int* boff;       // nblk+1: block b's slice of ptab (one slot per position of pose c1)
  int* ptab;       // per (block, c1 position): first c2 partner k2 | more<<30, or -1
  int nblk;        // nposes*(nposes+1)/2 upper-triangle Hschur blocks
  // per position
  double* Hpl;     // na*18 (6x3)
  double* ptc;     // na*12: Hll 9 + bl 3
  double* cmc;     // na*kCmc: Hpp upper triangle 21 (row-major, c >= r) + bp 6
  double* BD;      // na*18
  double* cf;      // na*6
  // per active point
  double* Hll;     // npa*9
  double* bl;      // npa*3
  double* Dinv;    // npa*9
  double* dmax_p;  // npa
  // per pose
  double* Hpp;     // nposes*36
  double* bp;      // nposes*6
  double* xp;      // nposes*6
  double* bs;      // nposes*6
  double* S;       // (6*nposes)^2
  double* Sw;      // padded LDLT work matrix when it does not fit LDS
  unsigned long long* dbg;  // optional phase timestamps (debug probe only)
  double* dmax_c;  // nposes
  int* pos_pt;     // na: active point index of position k
  int* pblk;       // nbf+1: first active point of each fused point-side block (k_ba_lin_schur), or null
  int nbf;         // fused point-side blocks (0: the unfused kernels run)
  int fused;       // device-LM launches of a problem with nbf > 0: k_ba_lin_schur does the point side
                   // (3: a phase's entry linearisation -- k_ba_linearize + k_ba_point_sum's outputs only)
                   // of iteration-start trials (k_ba_linearize / point_sum / point_schur skip them)
  int ldlt_pan;    // the reduced system goes through k_ba_ldlt_pan (else the column-step kernel): per
                   // problem, so a batch with both kinds launches both and each skips the other's
  int camfold;     // device-LM trials: k_ba_pairs' rhs blocks also sum the pose terms (k_ba_cam_sum's
                   // partials) and k_ba_schur_fin does k_ba_cam_fin's Hpp / bp (not launched)
  double* gpart;   // chunk partials of the pose-list gathers (summed by the *_fin kernels)
  double* gpose;   // posepart: nbf x nposes x kCmc -- per fused block and pose, the pose terms of the
                   // block's positions on that pose summed in position order (relinearising trials)
  int posepart;    // relinearising device-LM trials: k_ba_lin_schur writes gpose instead of the
                   // per-position pose terms, k_ba_pairs' rhs blocks sum gpose over the fused blocks
  int bdfold;      // device-LM trials of a fused problem: B D^-1 is not stored; k_ba_pairs forms it
                   // from H_pl and the point's D^-1 (the same expression, the same bits)
  int gsplit;      // chunks per pose list in the gather kernels
  int nbe;         // k_ba_errors blocks; scal[8..] holds its block partials (2 slots), then k_ba_update's
  int nbu;         // k_ba_update blocks (its LM-scale partials)
  double* scal;    // scalars: [0] chi at iteration start, [1] chi after the trial, [2] solve ok, [3] max diag, [4] LM scale
  const LmState* lm;  // device LM state: gates the trial's kernels and carries lambda (null: host control)
  // phase-end readout (set on the last k_ba_errors launch of a phase only): the launch also writes
  // its block partials, block 0 the rest of the readback block and *lm_copy, into mapped pinned
  // memory (rb_out, lm_out), so the host reads them after one event with no copy launches
  double* rb_out;
  LmState* lm_out;
  const LmState* lm_copy;
  int nan_trial;      // debug (ORBX_BA_NAN_TRIAL): this trial's chi is NaN; -1 off
  int raise_after;    // debug (ORBX_BA_RAISE_STOP_AFTER): the device raises the stop mirror after this many trials; -1 off
};

// gates of the device LM loop (uniform per launch, checked before any barrier)
__device__ inline bool lm_skip(const BaDev& D) { return D.lm && D.lm->done; }
__device__ inline bool lm_skip_lin(const BaDev& D) { return D.lm && (D.lm->done || !D.lm->relin); }
__device__ inline double lm_lambda(const BaDev& D, double lambda) { return D.lm ? D.lm->lambda : lambda; }
// The phase-2 launches queued speculatively behind phase 1's last trials (k_ba_outliers and the
// structure kernels with D.lm set): they run only if phase 1 has ended on an accepted state -- done,
// no refresh pending, no rejected trial still to pop -- which the host then reads back with phase
// 1's state; otherwise they return at once and the host queues them again after its pop.
__device__ inline bool spec_skip(const BaDev& D) {
  return D.lm && !(D.lm->done && !D.lm->refresh && !D.lm->rejected);
}

// Cross-lane exchange with the partner lane for butterfly level O: xor 32 via
// ds_bpermute, xor 16 via ds_swizzle, and the in-row levels through DPP (no
// LDS traffic): row_mirror (i <-> 15-i), row_half_mirror (i <-> 7-i), quad
// perms.  Each is an involution whose partner differs in bit O of the lane.
template <int O>
__device__ inline int xlane_i(int x) {
  if constexpr (O == 32) return __shfl_xor(x, 32, 64);
  else if constexpr (O == 16) return __builtin_amdgcn_ds_swizzle(x, (0x10 << 10) | 0x1F);
  else if constexpr (O == 8) return __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false);
  else if constexpr (O == 4) return __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);
  else if constexpr (O == 2) return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false);
  else return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
}
template <int O>
__device__ inline double xlane(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = xlane_i<O>((int)x), hi = xlane_i<O>((int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Butterfly sum of one double over the 64 lanes (every lane gets the total).
template <int O = 32>
__device__ inline double wave_sum(double v) {
  v += xlane<O>(v);
  if constexpr (O > 1) return wave_sum<O / 2>(v);
  else return v;
}

// Reduce-scatter of M per-lane values over the wave by recursive halving: at
// level O the lanes with bit O set keep the upper half and send the lower,
// so only M/2 values cross lanes per level (M-1 exchanges in all instead of
// 6M).  On exit w[0] of every lane is the wave total of value idx.
template <int M, int O>
__device__ inline void wave_reduce_scatter(double* w, int lane, int& idx) {
  if constexpr (O > 0) {
    const bool hi = (lane & O) != 0;
    if constexpr (M > 1) {
#pragma unroll
      for (int i = 0; i < M / 2; i++) {
        const double keep = hi ? w[M / 2 + i] : w[i];
        const double send = hi ? w[i] : w[M / 2 + i];
        w[i] = keep + xlane<O>(send);
      }
      if (hi) idx += M / 2;
      wave_reduce_scatter<M / 2, O / 2>(w, lane, idx);
    } else {
      w[0] += xlane<O>(w[0]);
      wave_reduce_scatter<1, O / 2>(w, lane, idx);
    }
  }
}

// Fixed-order block sum of one double per thread (blockDim LBS); every thread gets the result.
__device__ inline double block_sum1(double v, double* red /* LDS [LBS/64] */) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0;
#pragma unroll
  for (int w = 0; w < LBS / 64; w++) s += red[w];
  __syncthreads();
  return s;
}

// Block partial of a grid-wide sum: stored to out[blockIdx.x]; the host adds
// the partials in block order after its one readback per LM trial (fixed
// order, no cross-block synchronisation on the device).
__device__ inline void block_partial(double v, double* out, double* out2 = nullptr) {
  __shared__ double red[LBS / 64];
  const double bs = block_sum1(v, red);
  if (threadIdx.x == 0) {
    out[blockIdx.x] = bs;
    if (out2) out2[blockIdx.x] = bs;
  }
}

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

// Relaxed agent-scope store / load of a double: written through / read past the XCD's L2, so a
// value one block stores is seen by another block of the same launch (k_ba_errors_ctl's partials)
__device__ inline void st_agent(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline double ld_agent(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Returns false where the block did nothing (gated launch, block past the problem): uniform per block.
// coh: the block partial is stored write-through (st_agent) for k_ba_errors_ctl's last block.
template <bool coh = false>
__device__ __forceinline__ bool k_ba_errors_body(const BaDev& D, int recompute, int dst) {
  // recompute == 2: the refresh launch (only while the device LM state asks for it)
  if (recompute == 2 ? !(D.lm && D.lm->refresh) : lm_skip(D)) return false;
  if ((int)blockIdx.x >= D.nbe) return false;  // (a batched grid spans the largest problem)
  const int k = blockIdx.x * LBS + threadIdx.x;
  double chi = 0;
  if (k < D.na) {
    const int e = D.act[k];
    // robust-kernel inputs loaded up front (not behind the eerr stores and the flag's branch)
    const bool rob = D.erobust[e] != 0;
    const double dl = D.edelta[e];
    const float ds = D.edsqr[e];
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
    chi = c2;
    if (rob) {
      double rho[3];
      huber(c2, dl, ds, rho);
      chi = rho[0];
    }
    // debug hook (ORBX_BA_NAN_TRIAL): the given trial's chi is NaN, i.e. rho is NaN
    if (dst == 1 && k == 0 && D.nan_trial >= 0 && D.lm && D.lm->trials == D.nan_trial)
      chi = __builtin_nan("");
  }
  if (coh) {
    __shared__ double red[LBS / 64];
    const double bs = block_sum1(chi, red);
    if (threadIdx.x == 0) st_agent(D.scal + 8 + dst * D.nbe + blockIdx.x, bs);
    return true;
  }
  block_partial(chi, D.scal + 8 + dst * D.nbe, D.rb_out ? D.rb_out + 8 + dst * D.nbe : nullptr);
  if (D.rb_out && blockIdx.x == 0) {
    // the readback block's other entries (written by earlier launches), then the LM state
    const int n_rb = 8 + 2 * D.nbe + D.nbu;
    for (int i = threadIdx.x; i < n_rb; i += LBS)
      if (i < 8 + dst * D.nbe || i >= 8 + (dst + 1) * D.nbe) D.rb_out[i] = D.scal[i];
    if (D.lm_out) {
      constexpr int kW = sizeof(LmState) / 4;
      static_assert(sizeof(LmState) % 4 == 0, "LmState copied as words");
      if (threadIdx.x < kW)
        reinterpret_cast<uint32_t*>(D.lm_out)[threadIdx.x] = reinterpret_cast<const uint32_t*>(D.lm_copy)[threadIdx.x];
    }
  }
  return true;
}
__global__ __launch_bounds__(LBS) void k_ba_errors(BaDev D, int recompute, int dst) { k_ba_errors_body(D, recompute, dst); }
__global__ __launch_bounds__(LBS) void k_ba_errors_many(const BaDev* __restrict__ Ds, int recompute, int dst) {
  k_ba_errors_body(Ds[blockIdx.z], recompute, dst);
}


// constructQuadraticForm of one edge with DIM-dimensional error (2 mono, 3 stereo)
// One staged output array of the linearisation: each thread's NV values go to
// LDS, then the block's contiguous NV doubles per position leave with
// coalesced 8-B stores (position k's values land at out[NV * k + j], as
// before); PARTS > 1 stages the block's positions in that many slices so the
// LDS buffer stays at LBS * 21 doubles.
template <int NV, int PARTS, class F>
__device__ __forceinline__ void lin_stage_store(double* sh, double* out, int k0, int nk, bool act, F f) {
  constexpr int PS = LBS / PARTS;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < PARTS; q++) {
    if (act && t / PS == q) f(sh + NV * (t - q * PS));
    __syncthreads();
    const int n = min(PS, nk - q * PS);
    for (int j = t; j < n * NV; j += LBS) out[NV * ((size_t)k0 + q * PS) + j] = sh[j];
    __syncthreads();
  }
}

constexpr int kCmc = 27;  // pose terms per position (see lin_pose_terms)

// constructQuadraticForm terms of one edge (DIM = 2 mono, 3 stereo); written
// through LDS by the block (positions on fixed cameras get pose terms too:
// nothing reads them).
struct LinTerms {
  double omr[3], W;
};
template <int DIM>
__device__ __forceinline__ LinTerms lin_weights(const BaDev& D, int e) {
  LinTerms T;
  const double info = D.einfo[e];
  const bool rob = D.erobust[e] != 0;
  const double dl = D.edelta[e];
  const float ds = D.edsqr[e];
  T.W = info;
#pragma unroll
  for (int i = 0; i < DIM; i++) T.omr[i] = -info * D.eerr[3 * e + i];
  if (rob) {
    double c2 = 0;
#pragma unroll
    for (int i = 0; i < DIM; i++) c2 += D.eerr[3 * e + i] * (info * D.eerr[3 * e + i]);
    double rho[3];
    huber(c2, dl, ds, rho);
    T.W = rho[1] * info;
#pragma unroll
    for (int i = 0; i < DIM; i++) T.omr[i] *= rho[1];
  }
  return T;
}
template <int DIM>
__device__ __forceinline__ void lin_point_terms(const LinTerms& T, const double* A, double* pc) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double s = 0;
#pragma unroll
    for (int d = 0; d < DIM; d++) s += A[3 * d + r] * T.omr[d];
    pc[9 + r] = s;
#pragma unroll
    for (int cc = 0; cc < 3; cc++) {
      double h = 0;
#pragma unroll
      for (int d = 0; d < DIM; d++) h += A[3 * d + r] * T.W * A[3 * d + cc];
      pc[3 * r + cc] = h;
    }
  }
}
template <int DIM>
__device__ __forceinline__ void lin_pose_terms(const LinTerms& T, const double* Bm, double* cm) {
  // only the upper triangle is ever summed (k_ba_cam_sum, k_ba_pairs; k_ba_schur_fin mirrors it),
  // so only it is formed and stored: kCmc doubles per position instead of 42
  int j = 0;
#pragma unroll
  for (int r = 0; r < 6; r++) {
    double s = 0;
#pragma unroll
    for (int d = 0; d < DIM; d++) s += Bm[6 * d + r] * T.omr[d];
    cm[21 + r] = s;
#pragma unroll
    for (int cc = r; cc < 6; cc++) {
      double h = 0;
#pragma unroll
      for (int d = 0; d < DIM; d++) h += Bm[6 * d + r] * T.W * Bm[6 * d + cc];
      cm[j++] = h;
    }
  }
}
template <int DIM>
__device__ __forceinline__ void lin_cross_terms(const LinTerms& T, const double* A, const double* Bm, double* hp) {
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int cc = 0; cc < 3; cc++) {
      double h = 0;
#pragma unroll
      for (int d = 0; d < DIM; d++) h += Bm[6 * d + r] * T.W * A[3 * d + cc];
      hp[3 * r + cc] = h;
    }
}

// Jacobians (linearizeOplus, types_six_dof_expmap.h:80-141) and robust weights of edge e at the
// current state: point block A (DIM x 3), pose block Bm (DIM x 6), stereo flag.
struct LinEdge {
  double A[9], Bm[18];
  LinTerms T;
  bool st;
};
__device__ __forceinline__ void lin_edge(const BaDev& D, int e, LinEdge& o) {
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
  double* A = o.A;
  double* Bm = o.Bm;
  for (int i = 0; i < 18; i++) Bm[i] = 0.0;
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
  o.st = st;
  o.T = st ? lin_weights<3>(D, e) : lin_weights<2>(D, e);
}

__device__ __forceinline__ void k_ba_linearize_body(const BaDev& D) {
  if (lm_skip_lin(D) || D.fused) return;
  __shared__ double sh[LBS * 21];
  const int k0 = blockIdx.x * LBS, k = k0 + threadIdx.x;
  if (k0 >= D.na) return;  // block-uniform
  const int nk = min(LBS, D.na - k0);
  const bool act = k < D.na;
  const int e = act ? D.act[k] : D.act[k0];
  LinEdge L;
  lin_edge(D, e, L);
  lin_stage_store<12, 1>(sh, D.ptc, k0, nk, act, [&](double* o) {
    if (L.st) lin_point_terms<3>(L.T, L.A, o); else lin_point_terms<2>(L.T, L.A, o);
  });
  lin_stage_store<18, 1>(sh, D.Hpl, k0, nk, act, [&](double* o) {
    if (L.st) lin_cross_terms<3>(L.T, L.A, L.Bm, o); else lin_cross_terms<2>(L.T, L.A, L.Bm, o);
  });
  lin_stage_store<kCmc, 2>(sh, D.cmc, k0, nk, act, [&](double* o) {
    if (L.st) lin_pose_terms<3>(L.T, L.Bm, o); else lin_pose_terms<2>(L.T, L.Bm, o);
  });
}
__global__ __launch_bounds__(LBS) void k_ba_linearize(BaDev D) { k_ba_linearize_body(D); }
__global__ __launch_bounds__(LBS) void k_ba_linearize_many(const BaDev* __restrict__ Ds) {
  k_ba_linearize_body(Ds[blockIdx.z]);
}

__device__ __forceinline__ void k_ba_point_sum_body(const BaDev& D) {
  if (lm_skip_lin(D) || D.fused) return;
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
__global__ __launch_bounds__(LBS) void k_ba_point_sum(BaDev D) { k_ba_point_sum_body(D); }
__global__ __launch_bounds__(LBS) void k_ba_point_sum_many(const BaDev* __restrict__ Ds) {
  k_ba_point_sum_body(Ds[blockIdx.z]);
}

// Fixed-order block sum of NV per-thread partials over a kGB-thread block
// (shuffle tree per wave, then the waves' results summed in wave order by
// thread j < NV): deterministic for a fixed launch shape.  Returns the NV
// totals (in LDS, visible to the whole block).
constexpr int kGB = 256;  // gather-block size (pose lists are split into chunks across blocks)
constexpr int kGW = kGB / 64;
constexpr int kPB = 256;
template <int NV, int NW = kGW>
__device__ inline const double* block_sum_fixed(double (&v)[NV], double* red /* LDS [(NW+1)*NV] */) {
  static_assert(NV <= 64, "one value per lane after the reduce-scatter");
  constexpr int P = NV <= 1 ? 1 : NV <= 2 ? 2 : NV <= 4 ? 4 : NV <= 8 ? 8 : NV <= 16 ? 16 : NV <= 32 ? 32 : 64;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double w[P];
#pragma unroll
  for (int j = 0; j < P; j++) w[j] = j < NV ? v[j] : 0.0;
  int idx = 0;
  wave_reduce_scatter<P, 32>(w, lane, idx);
  if (idx < NV && (lane & ((64 / P) - 1)) == 0) red[wv * NV + idx] = w[0];
  __syncthreads();
  if (threadIdx.x < NV) {
    double t = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) t += red[w * NV + threadIdx.x];
    red[NW * NV + threadIdx.x] = t;
  }
  __syncthreads();
  return red + NW * NV;
}

// Chunk s of S of the range [lo, hi): [lo + n*s/S, lo + n*(s+1)/S).
__device__ inline void chunk_range(int lo, int hi, int s, int S, int& a, int& b) {
  const long long n = hi - lo;
  a = lo + (int)(n * s / S);
  b = lo + (int)(n * (s + 1) / S);
}

// Hpp, bp per pose: grid (pose, chunk); a chunk's threads take its positions
// t, t+kGB, ... ; only the upper triangle (21) + b (6) are summed.  Chunk
// partials -> gpart, summed in chunk order by k_ba_cam_fin.
__device__ __forceinline__ void k_ba_cam_sum_body(const BaDev& D) {
  if (lm_skip_lin(D) || (int)blockIdx.x >= D.nposes || (int)blockIdx.y >= D.gsplit) return;
  __shared__ double red[(kGW + 1) * 27];
  const int ci = blockIdx.x;
  double v[27];
#pragma unroll
  for (int j = 0; j < 27; j++) v[j] = 0;
  int lo, hi;
  chunk_range(D.cam_off[ci], D.cam_off[ci + 1], blockIdx.y, D.gsplit, lo, hi);
  for (int t = lo + threadIdx.x; t < hi; t += kGB) {
    const double* cm = D.cmc + kCmc * (size_t)D.cam_pos[t];
#pragma unroll
    for (int j = 0; j < kCmc; j++) v[j] += cm[j];
  }
  const double* tot = block_sum_fixed<27>(v, red);
  if (threadIdx.x < 27) D.gpart[((size_t)ci * D.gsplit + blockIdx.y) * 27 + threadIdx.x] = tot[threadIdx.x];
}
__global__ __launch_bounds__(kGB) void k_ba_cam_sum(BaDev D) { k_ba_cam_sum_body(D); }
__global__ __launch_bounds__(kGB) void k_ba_cam_sum_many(const BaDev* __restrict__ Ds) {
  k_ba_cam_sum_body(Ds[blockIdx.z]);
}

// One 64-thread block per pose: Hpp (symmetric), bp, max |Hpp_jj|.
__device__ __forceinline__ void k_ba_cam_fin_body(const BaDev& D) {
  if (lm_skip_lin(D) || (int)blockIdx.x >= D.nposes) return;
  __shared__ double tot[27];
  const int ci = blockIdx.x, j = threadIdx.x, S = D.gsplit;
  if (j < 27) {
    double t = 0;
    for (int c = 0; c < S; c++) t += D.gpart[((size_t)ci * S + c) * 27 + j];
    tot[j] = t;
  }
  __syncthreads();
  if (j < 36) {
    int r = j / 6, c = j % 6;
    if (c < r) {
      const int t = r;
      r = c;
      c = t;
    }
    D.Hpp[36 * ci + j] = tot[r * 6 - (r * (r - 1)) / 2 + (c - r)];  // upper-triangle index
  } else if (j < 42) {
    D.bp[6 * ci + (j - 36)] = tot[21 + (j - 36)];
  } else if (j == 42) {
    double m = 0;
    for (int r = 0; r < 6; r++) m = fmax(m, fabs(tot[r * 6 - (r * (r - 1)) / 2]));
    D.dmax_c[ci] = m;
  }
}
__global__ __launch_bounds__(64) void k_ba_cam_fin_many(const BaDev* __restrict__ Ds) {
  k_ba_cam_fin_body(Ds[blockIdx.z]);
}

// One thread per active edge position: D = Hll + lambda I of its point,
// Dinv (stored once per point), BD_e = Hpl_e Dinv, cf_e = Hpl_e Dinv bl.
__device__ __forceinline__ void k_ba_point_schur_body(const BaDev& D, double lambda) {
  if (lm_skip(D) || D.fused == 2 || (D.fused && !lm_skip_lin(D))) return;  // k_ba_lin_schur ran this trial
  lambda = lm_lambda(D, lambda);
  // the block's 256 positions are contiguous: Hpl comes in and BD / cf go out
  // through LDS with coalesced 8-B accesses (per-lane 144-B strides made every
  // load/store instruction touch 64 separate lines)
  __shared__ double sh[LBS * 18];
  __shared__ double scf[LBS * 6];
  const int k0 = blockIdx.x * LBS, t = threadIdx.x, k = k0 + t;
  if (k == 0 && D.nposes == 0) D.scal[2] = 1.0;  // no reduced system to factor
  if (k0 >= D.na) return;  // block-uniform
  const int nk = min(LBS, D.na - k0);
  for (int j = t; j < nk * 18; j += LBS) sh[j] = D.Hpl[18 * (size_t)k0 + j];
  __syncthreads();
  double bdv[18], cfv[6];
  const bool act = k < D.na;
  if (act) {
    const int i = D.pos_pt[k];
    double Dm[9];
    for (int j = 0; j < 9; j++) Dm[j] = D.Hll[9 * i + j];
    Dm[0] += lambda;
    Dm[4] += lambda;
    Dm[8] += lambda;
    double Di[9];
    inv3(Dm, Di);
    if (k == D.pt_off[i])
      for (int j = 0; j < 9; j++) D.Dinv[9 * i + j] = Di[j];
    const double b0 = D.bl[3 * i], b1 = D.bl[3 * i + 1], b2 = D.bl[3 * i + 2];
    double db[3];
    for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
    const double* B1 = sh + 18 * t;
    for (int r = 0; r < 6; r++) {
      for (int c = 0; c < 3; c++) bdv[3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
      cfv[r] = B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
    }
  }
  __syncthreads();
  if (act) {
    for (int j = 0; j < 18; j++) sh[18 * t + j] = bdv[j];
    for (int r = 0; r < 6; r++) scf[6 * t + r] = cfv[r];
  }
  __syncthreads();
  // (positions on fixed cameras get values too; nothing reads them)
  for (int j = t; j < nk * 18; j += LBS) D.BD[18 * (size_t)k0 + j] = sh[j];
  for (int j = t; j < nk * 6; j += LBS) D.cf[6 * (size_t)k0 + j] = scf[j];
}
__global__ __launch_bounds__(LBS) void k_ba_point_schur(BaDev D, double lambda) { k_ba_point_schur_body(D, lambda); }

// ---- the point side of an iteration-start trial in one kernel (device LM, one problem) ----
// k_ba_linearize -> k_ba_point_sum -> k_ba_point_schur fused: block b takes the whole points
// pblk[b] .. pblk[b+1] (positions pt_off[pblk[b]] .. pt_off[pblk[b+1]], fewer than kFuseNT: a
// block's points start inside a kFuseStride-position window and no point has more than
// kFuseMaxDeg positions, checked at intake).  128-thread blocks with 63 KB of LDS: two per CU, so
// a config-4 phase's ~450 blocks are all resident at once.  Per position the same linearisation; the point
// terms stay in LDS and each point's thread sums them in position order (k_ba_point_sum's
// order), then D = Hll + lambda I, D^-1 (once per point) and B D^-1, B D^-1 b_l per position from
// the staged Hpl -- bit-identical to the three kernels, without their global round trips.
constexpr int kFuseNT = 128, kFuseStride = 96, kFuseMaxDeg = 32;
// n (even) doubles between 16-B aligned arrays, one 16-B pair per thread and step (half the
// iterations of 8-B copies: these LDS <-> global loops are a block's tail)
typedef double dpair_t __attribute__((ext_vector_type(2)));
template <int NT>
__device__ __forceinline__ void copy_pairs(double* __restrict__ dst, const double* __restrict__ src, int n, int t) {
  dpair_t* d = reinterpret_cast<dpair_t*>(dst);
  const dpair_t* q = reinterpret_cast<const dpair_t*>(src);
  for (int j = t; j < n / 2; j += NT) d[j] = q[j];
}
// Phase probe (build with -DORBX_LS_PROBE only; tools/ls_probe.py): s_memtime of thread 0 of every
// k_ba_lin_schur block at six points of the last launch, 8 words per block
#ifdef ORBX_LS_PROBE
__device__ unsigned long long g_ls_probe[1024 * 8];
#define LS_TS(k)                                                                                  \
  do {                                                                                            \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_ls_probe[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define LS_TS(k)
#endif
static_assert(kFuseStride - 1 + kFuseMaxDeg <= kFuseNT, "a fused block's positions fit its threads");
__device__ __forceinline__ void k_ba_lin_schur_body(const BaDev& D) {
  if (!D.fused || lm_skip(D) || (int)blockIdx.x >= D.nbf) return;
  // fused == 2: the trials that do not relinearise (a rejected step's new lambda) also come here,
  // for k_ba_point_schur's part: the staged Hpl, D = Hll + lambda I, D^-1 b_l (same bits)
  const bool lin = !lm_skip_lin(D);
  if (!lin && D.fused != 2) return;
  constexpr int NT = kFuseNT;
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  double* sptc = fsm;                // NT x 12 point terms; then with sbuf: BD (18) | cf (6) staging
  double* sbuf = sptc + NT * 12;     // NT x 21; with sdi (before the point sums): the 27 pose terms
  double* sdi = sbuf + NT * 21;      // NT x 12: per point D^-1 (9) and D^-1 b_l (3)
  double* shpl = sdi + NT * 12;      // NT x 18
  double* sout = sptc;               // NT x 24 over sptc + sbuf once the point sums are done
  static_assert(12 + 1 + kCmc <= 12 + 21 + 12, "the pose-term staging fits sbuf + sdi");
  const int b = blockIdx.x, t = threadIdx.x;
  const int p0 = D.pblk[b], p1 = D.pblk[b + 1];
  const int k0 = D.pt_off[p0], nk = D.pt_off[p1] - k0, npt = p1 - p0;
  if (nk <= 0) return;  // block-uniform
  const double lambda = lm_lambda(D, 0.0);
  const bool act = t < nk;
  const int k = k0 + (act ? t : 0);
  LS_TS(0);
  if (!lin) {
    copy_pairs<NT>(shpl, D.Hpl + 18 * (size_t)k0, nk * 18, t);  // (18 k0 doubles: 16-B aligned)
    if (t < npt) {
      const int i = p0 + t;
      double Dm[9];
      for (int j = 0; j < 9; j++) Dm[j] = D.Hll[9 * i + j];
      Dm[0] += lambda;
      Dm[4] += lambda;
      Dm[8] += lambda;
      double Di[9];
      inv3(Dm, Di);
      for (int j = 0; j < 9; j++) D.Dinv[9 * i + j] = Di[j];
      const double b0 = D.bl[3 * i], b1 = D.bl[3 * i + 1], b2 = D.bl[3 * i + 2];
      for (int r = 0; r < 3; r++) sdi[12 * t + 9 + r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
      for (int j = 0; j < 9; j++) sdi[12 * t + j] = Di[j];
    }
  } else {
  LinEdge L;
  lin_edge(D, D.act[k], L);
  if (act) {
    if (L.st) {
      lin_point_terms<3>(L.T, L.A, sptc + 12 * t);
      lin_cross_terms<3>(L.T, L.A, L.Bm, shpl + 18 * t);
    } else {
      lin_point_terms<2>(L.T, L.A, sptc + 12 * t);
      lin_cross_terms<2>(L.T, L.A, L.Bm, shpl + 18 * t);
    }
  }
  LS_TS(1);
  // the 27 pose terms of every position out through LDS in one pass (sbuf + sdi, free until the
  // point sums) and 16-B pair stores; the staging starts at the global block's parity (27 k0 may be
  // odd), so the LDS and the global pairs are aligned alike
  double cm[kCmc];
  if (L.st) lin_pose_terms<3>(L.T, L.Bm, cm); else lin_pose_terms<2>(L.T, L.Bm, cm);
  if (D.posepart && D.fused != 3) {
    // per pose, the block's positions on it summed in position order (the rhs blocks of k_ba_pairs
    // then add the fused blocks' sums in block order): one nposes x kCmc record per block instead
    // of kCmc doubles per position.  Pose c's positions = the set bits of each wave's ballot,
    // walked in ascending order.
    double* scm = sbuf;                                             // NT x kCmc
    uint64_t* pm = reinterpret_cast<uint64_t*>(sbuf + NT * kCmc);   // nposes x (NT / 64) masks
    const int pc = act ? D.pcam[k] : -1;
    if (act) {
#pragma unroll
      for (int j = 0; j < kCmc; j++) scm[kCmc * t + j] = cm[j];
    }
    const int np = D.nposes;
    for (int c = 0; c < np; c++) {
      const uint64_t m = __ballot(pc == c);
      if ((t & 63) == 0) pm[(NT / 64) * c + (t >> 6)] = m;
    }
    __syncthreads();
    double* dst = D.gpose + (size_t)b * np * kCmc;
    for (int it = t; it < np * kCmc; it += NT) {
      const int c = it / kCmc, j = it - c * kCmc;
      double acc = 0.0;
#pragma unroll
      for (int w = 0; w < NT / 64; w++) {
        uint64_t m = pm[(NT / 64) * c + w];
        while (m) {
          acc += scm[kCmc * (64 * w + __builtin_ctzll(m)) + j];
          m &= m - 1;
        }
      }
      dst[it] = acc;
    }
    __syncthreads();  // (sbuf / sdi are written again below)
  } else {
    const int par = (int)((kCmc * (size_t)k0) & 1), n = nk * kCmc;
    double* scm = sbuf + par;
    if (act) {
#pragma unroll
      for (int j = 0; j < kCmc; j++) scm[kCmc * t + j] = cm[j];
    }
    __syncthreads();
    double* dst = D.cmc + kCmc * (size_t)k0;
    if (par && t == 0) dst[0] = scm[0];
    copy_pairs<NT>(dst + par, scm + par, (n - par) & ~1, t);
    if (((n - par) & 1) && t == NT - 1) dst[n - 1] = scm[n - 1];
    __syncthreads();  // (sbuf / sdi are written again below)
  }
  LS_TS(2);
  copy_pairs<NT>(D.Hpl + 18 * (size_t)k0, shpl, nk * 18, t);
  // point sums (k_ba_point_sum's order), D^-1 and D^-1 b_l once per point
  if (t < npt) {
    const int i = p0 + t;
    const int a = D.pt_off[i] - k0, e = D.pt_off[i + 1] - k0;
    double h[12];
    for (int j = 0; j < 12; j++) h[j] = 0;
    for (int kk = a; kk < e; kk++)
      for (int j = 0; j < 12; j++) h[j] += sptc[12 * kk + j];
    for (int j = 0; j < 9; j++) D.Hll[9 * i + j] = h[j];
    for (int j = 0; j < 3; j++) D.bl[3 * i + j] = h[9 + j];
    D.dmax_p[i] = fmax(fmax(fabs(h[0]), fabs(h[4])), fabs(h[8]));
    if (D.fused == 3) return;  // (a phase's entry linearisation: no lambda yet, no Schur terms)
    double Dm[9];
    for (int j = 0; j < 9; j++) Dm[j] = h[j];
    Dm[0] += lambda;
    Dm[4] += lambda;
    Dm[8] += lambda;
    double Di[9];
    inv3(Dm, Di);
    for (int j = 0; j < 9; j++) D.Dinv[9 * i + j] = Di[j];
    const double b0 = h[9], b1 = h[10], b2 = h[11];
    for (int r = 0; r < 3; r++) sdi[12 * t + 9 + r] = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
    for (int j = 0; j < 9; j++) sdi[12 * t + j] = Di[j];
  }
  }  // lin
  if (D.fused == 3) return;  // block-uniform
  LS_TS(3);
  __syncthreads();
  LS_TS(4);
  if (act) {
    const double* Di = sdi + 12 * (D.pos_pt[k] - p0);
    const double* db = Di + 9;
    const double* B1 = shpl + 18 * t;
    for (int r = 0; r < 6; r++) {
      for (int c = 0; c < 3; c++)
        sout[18 * t + 3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
      sout[18 * NT + 6 * t + r] = B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
    }
  }
  __syncthreads();
  if (!D.bdfold) copy_pairs<NT>(D.BD + 18 * (size_t)k0, sout, nk * 18, t);
  copy_pairs<NT>(D.cf + 6 * (size_t)k0, sout + 18 * NT, nk * 6, t);
  LS_TS(5);
}
__global__ __launch_bounds__(kFuseNT) void k_ba_lin_schur(BaDev D) { k_ba_lin_schur_body(D); }
__global__ __launch_bounds__(kFuseNT) void k_ba_lin_schur_many(const BaDev* __restrict__ Ds) {
  k_ba_lin_schur_body(Ds[blockIdx.z]);
}
constexpr size_t kFuseSmem = (size_t)kFuseNT * (12 + 21 + 18 + 12) * sizeof(double);

// Per phase: pblk[b] = the first active point whose first position is >= b * kFuseStride (block b
// then ends where block b+1's first point starts); pblk[nbf] = npa.  One thread per point, run by the
// pair-table launch's extra blocks.
__device__ __forceinline__ void pblk_body(const BaDev& D, int b) {
  const int p = b * LBS + threadIdx.x;
  if (p > D.npa) return;
  const int cur = p < D.npa ? D.pt_off[p] / kFuseStride : D.nbf;
  const int prev = p == 0 ? -1 : D.pt_off[p - 1] / kFuseStride;
  for (int q = prev + 1; q <= min(cur, D.nbf); q++) D.pblk[q] = p;
}
__global__ __launch_bounds__(LBS) void k_ba_point_schur_many(const BaDev* __restrict__ Ds, double lambda) {
  k_ba_point_schur_body(Ds[blockIdx.z], lambda);
}

// Accumulates acc += BD_k1 Hpl_k2^T (6x3 * 3x6), one Hpl row at a time.
__device__ inline void pair_acc(double acc[36], const double A[18], const double* __restrict__ h2) {
#pragma unroll
  for (int c = 0; c < 6; c++) {
    const double b0 = h2[3 * c], b1 = h2[3 * c + 1], b2 = h2[3 * c + 2];
#pragma unroll
    for (int r = 0; r < 6; r++) acc[6 * r + c] += A[3 * r] * b0 + A[3 * r + 1] * b1 + A[3 * r + 2] * b2;
  }
}

__device__ inline int tri_decode(int b, int n, int& c1) {
  c1 = 0;
  while (b >= n - c1) {
    b -= n - c1;
    c1++;
  }
  return c1 + b;
}

// Once per phase (the structure is fixed across its LM trials): for Hschur
// block (c1, c2) and each position k1 of pose c1 (ascending, i.e. point
// order), the first position k2 of the same point on pose c2, flagged when
// the point has more than one.
// grid (nblk [+ the pblk blocks], chunks): blocks past nblk fill pblk (chunk 0 only)
__global__ __launch_bounds__(kPB) void k_ba_pair_table(BaDev D) {
  const int2 bxy = xcd_block2();  // (as k_ba_pairs: one pose chunk's blocks on one XCD)
  if (bxy.x >= D.nblk) {
    if (bxy.y == 0) pblk_body(D, bxy.x - D.nblk);
    return;
  }
  int c1;
  const int c2 = tri_decode(bxy.x, D.nposes, c1);
  int lo, hi;
  chunk_range(D.cam_off[c1], D.cam_off[c1 + 1], bxy.y, gridDim.y, lo, hi);
  int* tab = D.ptab + D.boff[bxy.x] - D.cam_off[c1];
  for (int t = lo + threadIdx.x; t < hi; t += kPB) {
    const int i = D.pos_pt[D.cam_pos[t]];
    const int s = D.pt_off[i], e = D.pt_off[i + 1];
    int first = -1, more = 0;
    for (int k0 = s; k0 < e; k0 += 8) {  // the point's pose indices, eight loads in flight (clamped)
      int pc[8];
#pragma unroll
      for (int u = 0; u < 8; u++) pc[u] = D.pcam[min(k0 + u, e - 1)];
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (k0 + u < e && pc[u] == c2) {
          more |= first >= 0;
          first = first < 0 ? k0 + u : first;
        }
    }
    tab[t] = first < 0 ? -1 : (first | (more << 30));
  }
}

// Grid (nblk + nposes, chunk).  Blocks b < nblk: Hschur block (c1 <= c2)
// pair sum  sum BD_k1 Hpl_k2^T  over the pairs of k_ba_pair_table; thread t of
// a chunk takes pose c1's positions t, t+kPB, ... (each thread's pairs in
// (k1, k2) order).  Blocks b >= nblk: sum of cf over pose b - nblk's positions
// (the Schur rhs correction).  Chunk partials -> gpart; k_ba_schur_fin sums
// them in chunk order (deterministic).
// device-LM trials fold k_ba_cam_sum / k_ba_cam_fin into k_ba_pairs / k_ba_schur_fin (the entry
// linearisation of a phase still launches them)
// device-LM value of BaDev::fused: 2 = k_ba_lin_schur also takes the non-relinearising trials'
// point side and k_ba_point_schur is not launched.  A problem without free poses keeps 1
// (k_ba_point_schur flags its empty reduced system).
static int fused_mode(int nbf, int nposes) {
  if (nbf <= 0) return 0;
  return nposes > 0 ? 2 : 1;
}
// The device-LM trial copy's fold flags (single and batched drivers alike, so a batched problem
// keeps its single run's bits): with k_ba_lin_schur doing every trial's point side (fused == 2),
// B D^-1 is formed inside k_ba_pairs (bdfold) and, where the per-block pose records fit
// (gpose allocated), the pose terms leave k_ba_lin_schur summed per block and pose (posepart).
#ifndef ORBX_BA_BDFOLD
#define ORBX_BA_BDFOLD 1
#endif
#ifndef ORBX_BA_POSEPART
#define ORBX_BA_POSEPART 1
#endif
constexpr int kPosePartMaxPoses = 256;        // the block's per-pose masks fit k_ba_lin_schur's free LDS
constexpr size_t kPosePartMaxDoubles = 1 << 22;  // nbf x nposes x kCmc (32 MB)
__host__ inline void set_trial_folds(BaDev& d) {
  d.bdfold = (ORBX_BA_BDFOLD && d.fused == 2) ? 1 : 0;
  d.posepart = (ORBX_BA_POSEPART && d.fused == 2 && d.gpose) ? 1 : 0;
}

// pose-term chunk partials of a camfold trial, after the pair and rhs partials
__device__ inline size_t cam_part_off(const BaDev& D) { return ((size_t)D.nblk * 36 + (size_t)D.nposes * 6) * D.gsplit; }

// (gx, gy) = the block's (Hschur / rhs block, chunk) in the launch grid, taken XCD-contiguous
// (xcd_block2): the Hschur blocks of one (c1, chunk) share an XCD, so chunk c1's BD rows come from
// one L2 -- 50.7 -> 24.3 MB fetched per launch, 20.0 -> 18.9 us at config 4 (profiles/r05)
__device__ __forceinline__ void k_ba_pairs_body(const BaDev& D, int gx, int gy) {
  if (lm_skip(D) || gx >= D.nblk + D.nposes || gy >= D.gsplit) return;
  __shared__ double red[(kPB / 64 + 1) * 36];
  const int S = D.gsplit, s = gy;
  // dispatch order: the rhs blocks (every position of a pose, the pose terms too) first, then the
  // Schur blocks -- the heaviest blocks leave first and the grid's second round is light ones
  const int bx = gx < D.nposes ? D.nblk + gx : gx - D.nposes;
  if (bx >= D.nblk) {
    const int ci = bx - D.nblk;
    const bool cam = D.camfold && !lm_skip_lin(D);  // block-uniform
    double v[6] = {0, 0, 0, 0, 0, 0};
    double w[27];
#pragma unroll
    for (int j = 0; j < 27; j++) w[j] = 0;
    int lo, hi;
    chunk_range(D.cam_off[ci], D.cam_off[ci + 1], s, S, lo, hi);
    const bool camp = cam && !D.posepart;
    for (int t = lo + threadIdx.x; t < hi; t += kPB) {
      const int k = D.cam_pos[t];
      const double* f = D.cf + 6 * (size_t)k;
#pragma unroll
      for (int r = 0; r < 6; r++) v[r] += f[r];
      if (camp) {  // k_ba_cam_sum's accumulation (same chunks, same per-thread positions)
        const double* cm = D.cmc + kCmc * (size_t)k;
#pragma unroll
        for (int j = 0; j < kCmc; j++) w[j] += cm[j];
      }
    }
    if (cam && D.posepart) {  // the fused blocks' per-pose sums, chunked over the blocks
      int blo, bhi;
      chunk_range(0, D.nbf, s, S, blo, bhi);
      for (int b = blo + threadIdx.x; b < bhi; b += kPB) {
        const double* g = D.gpose + ((size_t)b * D.nposes + ci) * kCmc;
#pragma unroll
        for (int j = 0; j < kCmc; j++) w[j] += g[j];
      }
    }
    const double* tot = block_sum_fixed<6, kPB / 64>(v, red);
    if (threadIdx.x < 6)
      D.gpart[(size_t)D.nblk * S * 36 + ((size_t)ci * S + s) * 6 + threadIdx.x] = tot[threadIdx.x];
    if (cam) {
      static_assert(kPB == kGB, "k_ba_cam_sum's block shape");
      __syncthreads();  // red is reused
      const double* tc = block_sum_fixed<27, kPB / 64>(w, red);
      if (threadIdx.x < 27) D.gpart[cam_part_off(D) + ((size_t)ci * S + s) * 27 + threadIdx.x] = tc[threadIdx.x];
    }
    return;
  }
  int c1;
  const int c2 = tri_decode(bx, D.nposes, c1);
  double acc[36];
#pragma unroll
  for (int j = 0; j < 36; j++) acc[j] = 0;
  int lo, hi;
  chunk_range(D.cam_off[c1], D.cam_off[c1 + 1], s, S, lo, hi);
  const int* tab = D.ptab + D.boff[bx] - D.cam_off[c1];
  for (int t = lo + threadIdx.x; t < hi; t += kPB) {
    const int v = tab[t];
    const int k1 = D.cam_pos[t];
    if (v < 0) continue;
    const int first = v & ((1 << 30) - 1);
    double A[18];
    if (D.bdfold) {  // B D^-1 = H_pl D^-1 of the point (k_ba_lin_schur's expression, the same bits)
      const double* B1 = D.Hpl + 18 * (size_t)k1;
      const double* Di = D.Dinv + 9 * (size_t)D.pos_pt[k1];
      double h[18], di[9];
#pragma unroll
      for (int j = 0; j < 18; j++) h[j] = B1[j];
#pragma unroll
      for (int j = 0; j < 9; j++) di[j] = Di[j];
#pragma unroll
      for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) A[3 * r + c] = h[3 * r] * di[c] + h[3 * r + 1] * di[3 + c] + h[3 * r + 2] * di[6 + c];
    } else {
      const double* bd = D.BD + 18 * (size_t)k1;
#pragma unroll
      for (int j = 0; j < 18; j++) A[j] = bd[j];
    }
    pair_acc(acc, A, D.Hpl + 18 * (size_t)first);
    if (v >> 30) {
      const int e = D.pt_off[D.pos_pt[k1] + 1];
      for (int k2 = first + 1; k2 < e; k2++)
        if (D.pcam[k2] == c2) pair_acc(acc, A, D.Hpl + 18 * (size_t)k2);
    }
  }
  const double* tot = block_sum_fixed<36, kPB / 64>(acc, red);
  if (threadIdx.x < 36) D.gpart[((size_t)bx * S + s) * 36 + threadIdx.x] = tot[threadIdx.x];
}
__global__ __launch_bounds__(kPB) void k_ba_pairs(BaDev D) {
  const int2 b = xcd_block2();
  k_ba_pairs_body(D, b.x, b.y);
}
__global__ __launch_bounds__(kPB) void k_ba_pairs_many(const BaDev* __restrict__ Ds) {
  const int3 b = xcd_block3();
  k_ba_pairs_body(Ds[b.z], b.x, b.y);
}

// Reduced system from the chunk partials: blocks b < nblk write Hschur block
// (c1, c2) = [c1==c2](Hpp + lambda I) - pair sum (both triangles, so every
// entry of S is written); blocks b >= nblk write bs = bp - sum cf.
__device__ inline void schur_fin_block(const BaDev& D, int blk, int j, double lambda) {
  const int S = D.gsplit;
  // sum of the S chunk partials at p, p + stride, ... in chunk order; loads issued in groups of 8
  // (clamped, not predicated) before their adds
  auto psum = [&](const double* p, size_t stride) {
    double t = 0;
    for (int c0 = 0; c0 < S; c0 += 8) {
      double v[8];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const double* q = p + (size_t)min(c0 + e, S - 1) * stride;
        v[e] = *q;
      }
#pragma unroll
      for (int e = 0; e < 8; e++)
        if (c0 + e < S) t += v[e];
    }
    return t;
  };
  const bool cam = D.camfold && !lm_skip_lin(D);  // k_ba_cam_fin's sums (chunk order) done here
  const double* camp = D.gpart + cam_part_off(D);
  if (blk >= D.nblk) {
    const int ci = blk - D.nblk;
    if (j < 6) {
      const double t = psum(D.gpart + (size_t)D.nblk * S * 36 + (size_t)ci * S * 6 + j, 6);
      double bp;
      if (cam) {
        bp = psum(camp + (size_t)ci * S * 27 + 21 + j, 27);
        D.bp[6 * ci + j] = bp;
      } else {
        bp = D.bp[6 * ci + j];
      }
      D.bs[6 * ci + j] = bp - t;
    }
    return;
  }
  if (j >= 36) return;
  int c1;
  const int c2 = tri_decode(blk, D.nposes, c1);
  const double v = psum(D.gpart + (size_t)blk * S * 36 + j, 36);
  const int N = 6 * D.nposes;
  const int r = j / 6, c = j % 6;
  double sv;
  if (c1 == c2) {
    double h;
    if (cam) {
      const int lo = min(r, c), hi = max(r, c);
      h = psum(camp + (size_t)c1 * S * 27 + lo * 6 - (lo * (lo - 1)) / 2 + (hi - lo), 27);
      D.Hpp[36 * c1 + j] = h;
    } else {
      h = D.Hpp[36 * c1 + j];
    }
    sv = h + (r == c ? lambda : 0.0) - v;
  } else {
    sv = -v;
    D.S[(size_t)(6 * c2 + c) * N + 6 * c1 + r] = sv;
  }
  D.S[(size_t)(6 * c1 + r) * N + 6 * c2 + c] = sv;
}
__device__ __forceinline__ void k_ba_schur_fin_body(const BaDev& D, double lambda) {
  if (lm_skip(D) || (int)blockIdx.x >= D.nblk + D.nposes) return;
  schur_fin_block(D, blockIdx.x, threadIdx.x, lm_lambda(D, lambda));
}
__global__ __launch_bounds__(64) void k_ba_schur_fin(BaDev D, double lambda) { k_ba_schur_fin_body(D, lambda); }
__global__ __launch_bounds__(64) void k_ba_schur_fin_many(const BaDev* __restrict__ Ds, double lambda) {
  k_ba_schur_fin_body(Ds[blockIdx.z], lambda);
}

__device__ inline double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int kLdltMaxNp = 1024;                // padded size limit (panel buffer Np x 17 doubles in LDS)
constexpr int kLdltLdsNp = 128;                 // largest padded size kept in LDS
inline int ldlt_np(int N) { return (N + 15) & ~15; }
inline size_t ldlt_smem_bytes(int N, bool lds) {
  const size_t Np = ldlt_np(N);
  return ((lds ? Np * (Np + 1) : 0) + Np * 17) * sizeof(double);
}

// Dense LDLT (no pivoting; fails on an exactly zero pivot like Eigen's
// SimplicialLDLT) of the N x N reduced camera system and the solve, blocked
// by 16-column panels.  The matrix is padded to Np = 16k with an identity
// block (decoupled, never a zero pivot).  Per panel:
//   1. wave 0 factors the 16 x 16 diagonal block in registers (lane r = row
//      r, column values broadcast with readlane);
//   2. each row below it solves its 16 panel entries against L11 (one
//      thread per row) and stores W = L D (in A) and L (in P);
//   3. the trailing lower triangle is updated A22 -= W21 L21^T with FP64
//      MFMA 16x16x4 tiles spread over the 16 waves.
// Then L = W / D in place, and the two triangular solves run on wave 0 with
// the vector in registers.  kLds: A in LDS (row stride Np+1), else in the
// global scratch D.Sw (row stride Np).  A template parameter, not a runtime
// select, so that LDS accesses are ds_* and not FLAT instructions.
#define LDLT_TS(idx)                                                  \
  do {                                                                \
    if (D.dbg && tid == 0 && (idx) < 64) D.dbg[idx] = __builtin_amdgcn_s_memtime(); \
  } while (0)
template <bool kLds>
__global__ __launch_bounds__(1024) void k_ba_ldlt(BaDev D, int stage_limit) {
  if (lm_skip(D)) return;
  extern __shared__ double sm[];
  __shared__ int fail;
  __shared__ double Dinv_p[16];
  const int N = 6 * D.nposes, Np = (N + 15) & ~15, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ld = kLds ? Np + 1 : Np;
  double* A = kLds ? sm : D.Sw;
  double* P = sm + (kLds ? (size_t)Np * ld : 0);  // Np x 16 (stride 17): L of the current panel
  for (int i0 = 0; i0 < Np * Np; i0 += 4 * 1024) {
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int idx = i0 + u * 1024 + tid, r = idx / Np, c = idx - r * Np;
      v[u] = (r < N && c < N) ? D.S[(size_t)r * N + c] : (r == c ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int idx = i0 + u * 1024 + tid, r = idx / Np, c = idx - r * Np;
      if (idx < Np * Np) A[(size_t)r * ld + c] = v[u];
    }
  }
  if (tid == 0) fail = 0;
  __syncthreads();
  LDLT_TS(0);
  if (stage_limit == 1) return;
  for (int j0 = 0; j0 < Np; j0 += 16) {
    if (wv == 0) {
      const int r = lane & 15;
      double row[16];
#pragma unroll
      for (int c = 0; c < 16; c++) row[c] = A[(size_t)(j0 + r) * ld + j0 + c];
      bool bad = false;  // no early exit: the loops must unroll fully (constant register indices)
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double d = readlane_d(row[c], c);
        bad |= d == 0.0;
        const double invd = 1.0 / d;
#pragma unroll
        for (int k = c + 1; k < 16; k++) {
          const double lk = readlane_d(row[c], k) * invd;  // L[k][c]
          if (r >= k) row[k] -= row[c] * lk;
        }
      }
      if (bad) {
        if (lane == 0) fail = 1;
      } else if (lane < 16) {
        const double dr = row[r < 16 ? r : 0];
        double dd[16];
#pragma unroll
        for (int c = 0; c < 16; c++) dd[c] = readlane_d(row[c], c);
#pragma unroll
        for (int c = 0; c < 16; c++) {
          if (c <= r) A[(size_t)(j0 + r) * ld + j0 + c] = row[c];
          if (c < r) P[(j0 + r) * 17 + c] = row[c] / dd[c];
        }
        Dinv_p[r] = 1.0 / dr;
      }
    }
    __syncthreads();
    LDLT_TS(1 + 3 * (j0 >> 4));
    if (fail) {
      if (tid == 0) D.scal[2] = 0.0;
      return;
    }
    const int nrows = Np - j0 - 16;
    for (int t = tid; t < nrows; t += 1024) {
      const int i = j0 + 16 + t;
      double w[16];
#pragma unroll
      for (int c = 0; c < 16; c++) w[c] = A[(size_t)i * ld + j0 + c];
#pragma unroll
      for (int c = 1; c < 16; c++)
#pragma unroll
        for (int m = 0; m < c; m++) w[c] -= w[m] * P[(j0 + c) * 17 + m];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        A[(size_t)i * ld + j0 + c] = w[c];
        P[i * 17 + c] = w[c] * Dinv_p[c];
      }
    }
    __syncthreads();
    LDLT_TS(2 + 3 * (j0 >> 4));
    const int m = nrows >> 4, T = m * (m + 1) / 2;
    for (int t = wv; t < T; t += 16) {
      int ti = (int)((sqrtf(8.f * t + 1.f) - 1.f) * 0.5f);
      while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
      while (ti * (ti + 1) / 2 > t) ti--;
      const int tk = t - ti * (ti + 1) / 2;
      const int R0 = j0 + 16 + 16 * ti, C0 = j0 + 16 + 16 * tk;
      double4_t acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; kk++) {
        const double av = A[(size_t)(R0 + (lane & 15)) * ld + j0 + 4 * kk + (lane >> 4)];  // W[row][k]
        const double bv = P[(C0 + (lane & 15)) * 17 + 4 * kk + (lane >> 4)];              // L[col][k]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        const size_t o = (size_t)(R0 + (lane >> 4) + 4 * rr) * ld + C0 + (lane & 15);
        A[o] -= acc[rr];
      }
    }
    __syncthreads();
    LDLT_TS(3 + 3 * (j0 >> 4));
  }
  if (stage_limit == 2) return;
  for (int i = 1 + (tid >> 5); i < Np; i += 32)
    for (int k = tid & 31; k < i; k += 32) A[(size_t)i * ld + k] /= A[(size_t)k * ld + k];
  __syncthreads();
  LDLT_TS(60);
  if (stage_limit == 3) return;
  // blocked triangular solves with the vector in LDS (the panel buffer P is
  // free now): per 16-row panel wave 0 solves the small triangle in registers
  // (readlane broadcasts), then every thread updates the remaining rows
  double* yv = P;
  for (int i = tid; i < Np; i += 1024) yv[i] = i < N ? D.bs[i] : 0.0;
  __syncthreads();
  for (int j0 = 0; j0 < Np; j0 += 16) {  // L z = b (unit lower)
    if (wv == 0) {
      const int r = lane & 15;
      double Lr[16];
#pragma unroll
      for (int c = 0; c < 16; c++) Lr[c] = A[(size_t)(j0 + r) * ld + j0 + c];
      double val = yv[j0 + r];
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double zc = readlane_d(val, c);
        if (r > c) val -= Lr[c] * zc;
      }
      if (lane < 16) yv[j0 + r] = val;
    }
    __syncthreads();
    for (int i = j0 + 16 + tid; i < Np; i += 1024) {
      double sacc = yv[i];
#pragma unroll
      for (int c = 0; c < 16; c++) sacc -= A[(size_t)i * ld + j0 + c] * yv[j0 + c];
      yv[i] = sacc;
    }
    __syncthreads();
  }
  for (int i = tid; i < Np; i += 1024) yv[i] /= A[(size_t)i * ld + i];
  __syncthreads();
  for (int j0 = Np - 16; j0 >= 0; j0 -= 16) {  // L^T x = z
    if (wv == 0) {
      const int r = lane & 15;
      double Lc[16];
#pragma unroll
      for (int c = 0; c < 16; c++) Lc[c] = A[(size_t)(j0 + c) * ld + j0 + r];
      double val = yv[j0 + r];
#pragma unroll
      for (int c = 15; c >= 0; c--) {
        const double xc = readlane_d(val, c);
        if (r < c) val -= Lc[c] * xc;
      }
      if (lane < 16) yv[j0 + r] = val;
    }
    __syncthreads();
    for (int i = tid; i < j0; i += 1024) {
      double sacc = yv[i];
#pragma unroll
      for (int c = 0; c < 16; c++) sacc -= A[(size_t)(j0 + c) * ld + i] * yv[j0 + c];
      yv[i] = sacc;
    }
    __syncthreads();
  }
  for (int i = tid; i < N; i += 1024) D.xp[i] = yv[i];
  if (tid == 0) D.scal[2] = 1.0;
  LDLT_TS(61);
}

// ---- reduced camera system, small N: column-step LDLT with 4x4 tiles ----
// Right-looking LDL^T of the augmented [S b; b^T .] with one barrier per
// pivot (~780 cycles per pivot on gfx950, latency-bound: LDS round trip +
// reciprocal + barrier; 60 us at N = 120 vs 71 us for the 16-wide blocked
// kernel, whose in-wave panel factorisation is readlane/division bound).  Each thread owns TPT 4x4 tiles of the lower triangle in registers
// (rows up to N, row N = rhs, padded to a multiple of 4).  At pivot j a tile
// reads 4 + 4 entries of column j from LDS (two ds_read_b128 each) and does
// 16 FMAs -- a quarter of the LDS traffic of one element per thread, which
// is what bounds this loop.  After pivot j's update the owners of column
// j+1 publish it (and 1/d_{j+1}) to LDS; nothing else is read from LDS.  The
// augmented row ends as z = L^-1 b (columns are unscaled: entry (i,j) =
// L_ij d_j), so the forward solve is free; wave 0 then applies D^-1 and the
// backward L^T solve, prefetching column entries eight pivots at a time.  A
// zero pivot fails the solve (scal[2] = 0) like the blocked kernel.
//
// LDS column j holds rows (j & ~3) .. Np4-1 at Lc[cbase(j) + i], 32-byte
// aligned for every 4-row group.
__host__ __device__ inline int ldlt_np4(int N) { return (N + 1 + 3) & ~3; }
__host__ __device__ inline int ldlt_cstart(int j, int N) {  // sum_{c<j} (Np4 - (c & ~3))
  const int q = j >> 2, r = j & 3;
  return j * ldlt_np4(N) - (8 * q * (q - 1) + 4 * q * r);
}
__host__ __device__ inline int ldlt_cbase(int j, int N) { return ldlt_cstart(j, N) - (j & ~3); }
inline int ldlt_col_tiles(int N) {
  const int Tr = ldlt_np4(N) / 4, Tc = (N + 3) / 4;
  return Tc * Tr - Tc * (Tc - 1) / 2;
}
inline size_t ldlt_col_smem(int N) { return (size_t)(ldlt_cstart(N, N) + N + 1) * sizeof(double); }
constexpr size_t kLdltColMaxSmem = 160 * 1024 - 256;
inline bool ldlt_col_fits(int N) { return ldlt_col_smem(N) <= kLdltColMaxSmem && ldlt_col_tiles(N) <= 2048; }

typedef double double2_t __attribute__((ext_vector_type(2)));

// 1/d by v_rcp_f64 + two Newton steps (full double accuracy, a third of the
// latency of the IEEE division sequence -- it sits on the per-pivot path).
__device__ inline double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// Pivot j = 4m + U of k_ba_ldlt_col: rank-1 update of the active tiles from
// column j, then the owners of column j+1 publish it and 1/d_{j+1}.  The updates (and the
// back solve's) are explicit FMAs: one FP64 op per link of the chain instead of a multiply and
// a subtract (60 -> 55 us at N = 120).  The solve is tested against numpy (1e-10) and through the
// LM decisions against the oracle; no other path shares its rounding.
template <int TPT, int U>
__device__ __forceinline__ void ldlt_col_step(double* Lc, double* rinv, double (&a)[TPT][4][4], const int (&ti)[TPT],
                                              const int (&tk)[TPT], int m, int N, int& fail) {
  const int j = 4 * m + U;
  if (j >= N) return;  // uniform
  const double* cj = Lc + ldlt_cbase(j, N);
  const double invd = rinv[j];
#pragma unroll
  for (int t = 0; t < TPT; t++) {
    if (tk[t] >= m && !(tk[t] == m && U == 3)) {  // some column of the tile is > j
      const double2_t* pr = reinterpret_cast<const double2_t*>(cj + 4 * ti[t]);
      const double2_t* pk = reinterpret_cast<const double2_t*>(cj + 4 * tk[t]);
      const double2_t r0 = pr[0], r1 = pr[1], k0 = pk[0], k1 = pk[1];
      const double cr[4] = {r0.x, r0.y, r1.x, r1.y}, ckv[4] = {k0.x, k0.y, k1.x, k1.y};
      double ck[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const bool live = (tk[t] > m || q > U) && 4 * tk[t] + q < N;
        ck[q] = live ? ckv[q] * invd : 0.0;  // select: junk never propagates
      }
#pragma unroll
      for (int p = 0; p < 4; p++)
#pragma unroll
        for (int q = 0; q < 4; q++) a[t][p][q] = __builtin_fma(-cr[p], ck[q], a[t][p][q]);  // one op per link
    }
  }
  constexpr int Q = (U + 1) & 3;  // column j+1 within its tile
  const int mn = U == 3 ? m + 1 : m;
  if (j + 1 < N) {
#pragma unroll
    for (int t = 0; t < TPT; t++) {
      if (tk[t] == mn) {
        double2_t* dst = reinterpret_cast<double2_t*>(Lc + ldlt_cbase(j + 1, N) + 4 * ti[t]);
        dst[0] = double2_t{a[t][0][Q], a[t][1][Q]};
        dst[1] = double2_t{a[t][2][Q], a[t][3][Q]};
        if (ti[t] == tk[t]) {
          const double dn = a[t][Q][Q];
          rinv[j + 1] = rcp_nr(dn);
          if (dn == 0.0) fail = 1;
        }
      }
    }
  }
  __syncthreads();
}

template <int TPT, int NT>
__device__ __forceinline__ void k_ba_ldlt_col_body(const BaDev& D) {
  if (lm_skip(D) || D.ldlt_pan) return;
  extern __shared__ __attribute__((aligned(16))) double Lc[];
  __shared__ int fail;
  const int N = 6 * D.nposes, tid = threadIdx.x;
  const int Np4 = ldlt_np4(N), Tr = Np4 / 4, Tc = (N + 3) / 4;
  const int ntiles = Tc * Tr - Tc * (Tc - 1) / 2;
  double* rinv = Lc + ldlt_cstart(N, N);
  double a[TPT][4][4];
  int ti[TPT], tk[TPT];
  if (tid == 0) fail = 0;
#pragma unroll
  for (int t = 0; t < TPT; t++) {
    int x = tid + NT * t, k = 0;
    ti[t] = 0;
    tk[t] = -1;  // inactive
    if (x < ntiles) {
      while (x >= Tr - k) {  // column-major tile order
        x -= Tr - k;
        k++;
      }
      tk[t] = k;
      ti[t] = k + x;
    }
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int i = 4 * ti[t] + p, kk = 4 * tk[t] + q;
        double v = 0.0;
        if (tk[t] >= 0 && kk < N) v = i < N ? D.S[(size_t)i * N + kk] : (i == N ? D.bs[kk] : 0.0);
        a[t][p][q] = v;
      }
    if (tk[t] == 0) {
#pragma unroll
      for (int p = 0; p < 4; p++) Lc[ldlt_cbase(0, N) + 4 * ti[t] + p] = a[t][p][0];
      if (ti[t] == 0) {
        rinv[0] = rcp_nr(a[t][0][0]);
        if (a[t][0][0] == 0.0) fail = 1;
      }
    }
  }
  __syncthreads();
  for (int m = 0; 4 * m < N; m++) {  // pivots j = 4m + U, U unrolled so tile columns index statically
    ldlt_col_step<TPT, 0>(Lc, rinv, a, ti, tk, m, N, fail);
    ldlt_col_step<TPT, 1>(Lc, rinv, a, ti, tk, m, N, fail);
    ldlt_col_step<TPT, 2>(Lc, rinv, a, ti, tk, m, N, fail);
    ldlt_col_step<TPT, 3>(Lc, rinv, a, ti, tk, m, N, fail);
  }
  if (fail) {
    if (tid == 0) D.scal[2] = 0.0;
    return;
  }
  if (tid >= 64) return;
  // y = D^-1 z; L^T x = y (x_k final at step k, rows i < k updated)
  const int lane = tid;
  double y[4], invd[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int i = lane + 64 * r;
    invd[r] = 0.0;
    y[r] = 0.0;
    if (i < N) {
      invd[r] = rinv[i];
      y[r] = Lc[ldlt_cbase(i, N) + N] * invd[r];
    }
  }
  int cb[4];  // column i's base; rows >= N clamp to a valid column (their Lv is zeroed)
#pragma unroll
  for (int r = 0; r < 4; r++) cb[r] = ldlt_cbase(min(lane + 64 * r, N - 1), N);
  for (int kb = N - 1; kb >= 0; kb -= 8) {
    double Lv[8][4];
#pragma unroll
    for (int u = 0; u < 8; u++)
#pragma unroll
      for (int r = 0; r < 4; r++) {  // branchless: all 32 LDS reads issue together
        const int i = lane + 64 * r, k = kb - u;
        const double v = Lc[cb[r] + (i < k ? k : min(i, N - 1))];  // always a finite L entry
        Lv[u][r] = v * (i < k ? invd[r] : 0.0);  // L[k][i]; a multiply, so the load is unconditional
      }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = kb - u;
      if (k >= 0) {
        const int rk = k >> 6;
        const double yk = rk == 0 ? y[0] : rk == 1 ? y[1] : rk == 2 ? y[2] : y[3];
        const double xk = readlane_d(yk, k & 63);
#pragma unroll
        for (int r = 0; r < 4; r++) y[r] = __builtin_fma(-Lv[u][r], xk, y[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++)
    if (lane + 64 * r < N) D.xp[lane + 64 * r] = y[r];
  if (lane == 0) D.scal[2] = 1.0;
}
template <int TPT, int NT>
__global__ __launch_bounds__(NT) void k_ba_ldlt_col(BaDev D) { k_ba_ldlt_col_body<TPT, NT>(D); }
template <int TPT, int NT>
__global__ __launch_bounds__(NT) void k_ba_ldlt_col_many(const BaDev* __restrict__ Ds) {
  k_ba_ldlt_col_body<TPT, NT>(Ds[blockIdx.z]);
}

// ---- reduced camera system: 8-wide panels over the column-step kernel's register tiles ----
// The column-step kernel pays one barrier and one LDS round trip per pivot; its per-pivot chain
// (publish column j+1 and 1/d, barrier, read, scale, update) is what bounds it.  Here the pivots
// go eight at a time.  Per panel M (columns c0 = 8M .. c0+7, tile columns 2M, 2M+1):
//   B  one thread per row i = c0 .. N (the augmented row b^T included) reads the panel's 8x8
//      diagonal block and its own row from LDS, factors the diagonal block in registers (every
//      such thread the same way: no cross-lane broadcast on the pivot chain) and solves its row:
//      L_i (scaled) and V_i = L_i D (unscaled) to LDS, L_i also into the packed factor;
//   C  every register tile right of the next panel takes A -= L_rows V_cols^T (8 FMAs per entry,
//      the tile stays in registers: only the panel rows move through LDS); the tiles of the panel
//      after next publish themselves once updated and leave the registers;
//   A  (before B of panel M+1) panel M's update of panel M+1's eight columns, in LDS, by every
//      thread: two entries of one row each, so it costs ~16 FMAs per thread instead of the
//      128 of a register tile's look-ahead in one wave (1.5k cycles per panel).
// Panel values are double-buffered (panel M+1 in one buffer while panel M+2 is published into the
// other) and so are L / V (panel M's are read by C while B writes panel M+1's).  Every entry sees
// the same updates in the same order as the register path: results are unchanged bit for bit.
// Two barriers per eight pivots.  The augmented row ends as y = D^-1 L^-1 b, and wave 0 solves
// L^T x = y.  Failure rule as the other kernels: an exactly zero pivot fails the solve.
// LDS: packed strictly-lower L (N(N-1)/2), two panel-value, two L and two V arrays ((Np+8) x 8
// each), y (N).
#ifndef ORBX_LDLT_PW
#define ORBX_LDLT_PW 8
#endif
constexpr int kPW = ORBX_LDLT_PW;  // panel width (pivots per panel): 4 or 8
static_assert(kPW == 4 || kPW == 8, "panels of one or two tile columns");
constexpr int kTPP = kPW / 4;      // tile columns per panel
__host__ __device__ inline int ldlt_pan_rows(int N) { return ldlt_np4(N) + 8; }
// panel arrays: rows of kPW doubles in groups of four, each group padded by 2 doubles, so that
// the lanes of a wave reading different row groups spread over the LDS banks
constexpr int kPG = 4 * kPW + 2;
__host__ __device__ inline int ldlt_prow(int i) { return (i >> 2) * kPG + (i & 3) * kPW; }
__host__ __device__ inline int ldlt_pan_arr(int N) { return ldlt_pan_rows(N) / 4 * kPG; }
inline size_t ldlt_pan_smem(int N) {
  return ((size_t)N * (N - 1) / 2 + 6 * (size_t)ldlt_pan_arr(N) + N) * sizeof(double);
}
// (one tile per thread: with two the trailing update doubles and the panel kernel loses to the
// column-step one, e.g. 91 us at N = 126)
inline bool ldlt_pan_fits(int N) { return ldlt_pan_smem(N) <= kLdltColMaxSmem && ldlt_col_tiles(N) <= 512 && N < 128; }
// default where it fits (debug option ldlt = ORBX_BA_LDLT_COLUMN keeps the column-step kernel)
inline bool ldlt_use_pan(int N) { return ldlt_pan_fits(N) && ba_opts().ldlt == ORBX_BA_LDLT_AUTO; }
constexpr int ldlt_tri(int a, int b) { return a * (a + 1) / 2 + b; }

template <int TPT, int NT, int R>  // R: 64-row groups of the back solve (N < 64 R)
__device__ __forceinline__ void k_ba_ldlt_pan_body(const BaDev& D) {
  if (lm_skip(D) || !D.ldlt_pan) return;
  extern __shared__ __attribute__((aligned(16))) double Lpk[];  // row k: Lpk[k(k-1)/2 + c], c < k
  __shared__ int fail;
  const int N = 6 * D.nposes, tid = threadIdx.x;
  const int Np4 = ldlt_np4(N), Tr = Np4 / 4, Tc = (N + 3) / 4;
  const int ntiles = Tc * Tr - Tc * (Tc - 1) / 2;
  const int PA = ldlt_pan_arr(N);
  double* Pn = Lpk + (size_t)N * (N - 1) / 2;  // row i at ldlt_prow(i): current panel values
  double* Lp = Pn + PA;                         // panel L (scaled)
  double* Vp = Lp + PA;                         // panel V = L D (unscaled)
  double* ys = Vp + PA;                         // [N] y = D^-1 L^-1 b
  double* Lp2 = ys + N;                         // the second L / V set
  double* Vp2 = Lp2 + PA;
  double* Pn2 = Vp2 + PA;                       // the second panel-value buffer
  double a[TPT][4][4];
  int ti[TPT], tk[TPT];
  LDLT_TS(0);
  if (tid == 0) fail = 0;
#pragma unroll
  for (int t = 0; t < TPT; t++) {
    int x = tid + NT * t, k = 0;
    ti[t] = 0;
    tk[t] = -1;  // inactive
    if (x < ntiles) {
      while (x >= Tr - k) {  // column-major tile order
        x -= Tr - k;
        k++;
      }
      tk[t] = k;
      ti[t] = k + x;
    }
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int i = 4 * ti[t] + p, kk = 4 * tk[t] + q;
        double v = 0.0;
        if (tk[t] >= 0 && kk < N) v = i < N ? D.S[(size_t)i * N + kk] : (i == N ? D.bs[kk] : 0.0);
        a[t][p][q] = v;
      }
  }
  // (the tile loads above are in flight while the panel arrays are cleared)
  for (int j = tid; j < 3 * PA; j += NT) Pn[j] = 0.0;  // padding rows / columns stay finite
  for (int j = tid; j < 3 * PA; j += NT) Lp2[j] = 0.0;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < TPT; t++) {  // panels 0 and 1 publish and leave the registers
    if (tk[t] >= 0 && tk[t] < 2 * kTPP) {
      double* P = tk[t] < kTPP ? Pn : Pn2;
#pragma unroll
      for (int p = 0; p < 4; p++) {
        double2_t* dst = reinterpret_cast<double2_t*>(P + ldlt_prow(4 * ti[t] + p) + 4 * (tk[t] % kTPP));
        dst[0] = double2_t{a[t][p][0], a[t][p][1]};
        dst[1] = double2_t{a[t][p][2], a[t][p][3]};
      }
    }
  }
  __syncthreads();
  LDLT_TS(1);
  // B: the panel rows of panel M into (Lq, Vq)
  auto panel_rows = [&](int M, const double* Pq, double* Lq, double* Vq) {
    constexpr int W = kPW, H = kPW / 2;  // (H: double2 per panel row)
    const int c0 = W * M, w = min(W, N - c0);
    const int i = c0 + tid;
    if (i <= N) {
      double Dm[W * (W + 1) / 2], u[W];
#pragma unroll
      for (int r = 0; r < W; r++) {
        const double2_t* src = reinterpret_cast<const double2_t*>(Pq + ldlt_prow(c0 + r));
        double row[W];
#pragma unroll
        for (int h = 0; h < H; h++) {
          const double2_t v = src[h];
          row[2 * h] = v.x, row[2 * h + 1] = v.y;
        }
#pragma unroll
        for (int c = 0; c <= r; c++) Dm[ldlt_tri(r, c)] = row[c];
      }
      {
        const double2_t* src = reinterpret_cast<const double2_t*>(Pq + ldlt_prow(i));
#pragma unroll
        for (int h = 0; h < H; h++) {
          const double2_t v = src[h];
          u[2 * h] = v.x, u[2 * h + 1] = v.y;
        }
      }
      double L[W], V[W];
      bool zero = false;
#pragma unroll
      for (int q = 0; q < W; q++) {
        L[q] = 0.0;
        V[q] = 0.0;
        if (q < w) {  // uniform
          const double d = Dm[ldlt_tri(q, q)];
          zero |= d == 0.0;
          const double rq = rcp_nr(d);
          double lq[W];
#pragma unroll
          for (int r = q + 1; r < W; r++) lq[r] = Dm[ldlt_tri(r, q)] * rq;
#pragma unroll
          for (int r = q + 1; r < W; r++)
#pragma unroll
            for (int c = q + 1; c <= r; c++) Dm[ldlt_tri(r, c)] = __builtin_fma(-lq[r], Dm[ldlt_tri(c, q)], Dm[ldlt_tri(r, c)]);
          V[q] = u[q];
          L[q] = u[q] * rq;
#pragma unroll
          for (int c = q + 1; c < W; c++) u[c] = __builtin_fma(-L[q], Dm[ldlt_tri(c, q)], u[c]);
        }
      }
      if (tid == 0 && zero) fail = 1;
      double2_t* lo = reinterpret_cast<double2_t*>(Lq + ldlt_prow(i));
      double2_t* vo = reinterpret_cast<double2_t*>(Vq + ldlt_prow(i));
#pragma unroll
      for (int h = 0; h < H; h++) {
        lo[h] = double2_t{L[2 * h], L[2 * h + 1]};
        vo[h] = double2_t{V[2 * h], V[2 * h + 1]};
      }
      if (i < N) {
        double* lrow = Lpk + (size_t)i * (i - 1) / 2 + c0;
#pragma unroll
        for (int q = 0; q < W; q++)
          if (c0 + q < i && q < w) lrow[q] = L[q];
      } else {
#pragma unroll
        for (int q = 0; q < W; q++)
          if (q < w) ys[c0 + q] = L[q];
      }
    }
  };
  // C: the register tiles right of panel M+1 take A -= L_rows V_cols^T; those of panel M+2 then
  // publish themselves into Pq and retire
  auto trailing = [&](int M, const double* Lq, const double* Vq, double* Pq) {
#pragma unroll
    for (int t = 0; t < TPT; t++) {
      if (tk[t] >= kTPP * (M + 2)) {
        const double* lr = Lq + kPG * ti[t];
        const double* vr = Vq + kPG * tk[t];
#pragma unroll
        for (int h = 0; h < kTPP; h++) {
          double Lv[4][4], Vv[4][4];
#pragma unroll
          for (int p = 0; p < 4; p++) {
            const double2_t* ls = reinterpret_cast<const double2_t*>(lr + kPW * p + 4 * h);
            const double2_t* vs = reinterpret_cast<const double2_t*>(vr + kPW * p + 4 * h);
            const double2_t l0 = ls[0], l1 = ls[1], v0 = vs[0], v1 = vs[1];
            Lv[p][0] = l0.x, Lv[p][1] = l0.y, Lv[p][2] = l1.x, Lv[p][3] = l1.y;
            Vv[p][0] = v0.x, Vv[p][1] = v0.y, Vv[p][2] = v1.x, Vv[p][3] = v1.y;
          }
#pragma unroll
          for (int s = 0; s < 4; s++)
#pragma unroll
            for (int p = 0; p < 4; p++)
#pragma unroll
              for (int q = 0; q < 4; q++) a[t][p][q] = __builtin_fma(-Lv[p][s], Vv[q][s], a[t][p][q]);
        }
        if (tk[t] < kTPP * (M + 3)) {  // panel M+2 publishes itself
#pragma unroll
          for (int p = 0; p < 4; p++) {
            double2_t* dst = reinterpret_cast<double2_t*>(Pq + ldlt_prow(4 * ti[t] + p) + 4 * (tk[t] % kTPP));
            dst[0] = double2_t{a[t][p][0], a[t][p][1]};
            dst[1] = double2_t{a[t][p][2], a[t][p][3]};
          }
        }
      }
    }
  };
  // A: panel M's update of panel M+1's values in Pq (rows c1 = kPW (M+1) .. N, kPW columns):
  // thread -> (row c1 + tid / 4, columns CPT (tid % 4) .. +CPT-1), the s = 0..kPW-1 FMAs in the
  // register path's order
  auto lookahead = [&](const double* Lq, const double* Vq, double* Pq, int c1) {
    constexpr int CPT = kPW / 4;
    const int i = c1 + tid / 4, j0 = CPT * (tid & 3);
    if (i <= N) {
      const double2_t* ls = reinterpret_cast<const double2_t*>(Lq + ldlt_prow(i));
      double* dst = Pq + ldlt_prow(i) + j0;
      double x[CPT];
      const double2_t* vr[CPT];
#pragma unroll
      for (int c = 0; c < CPT; c++) {
        x[c] = dst[c];
        vr[c] = reinterpret_cast<const double2_t*>(Vq + ldlt_prow(c1 + j0 + c));
      }
#pragma unroll
      for (int h = 0; h < kPW / 2; h++) {
        const double2_t l = ls[h];
        double2_t v[CPT];
#pragma unroll
        for (int c = 0; c < CPT; c++) v[c] = vr[c][h];
#pragma unroll
        for (int c = 0; c < CPT; c++) x[c] = __builtin_fma(-l.x, v[c].x, x[c]);
#pragma unroll
        for (int c = 0; c < CPT; c++) x[c] = __builtin_fma(-l.y, v[c].y, x[c]);
      }
#pragma unroll
      for (int c = 0; c < CPT; c++) dst[c] = x[c];
    }
  };
  static_assert(NT / 4 >= 124, "one look-ahead pass covers rows kPW .. N of a panel (N < 128)");
  panel_rows(0, Pn, Lp, Vp);
  __syncthreads();
  for (int M = 0; kTPP * M < Tc; M++) {
    double* Lc = (M & 1) ? Lp2 : Lp;  // panel M's L / V
    double* Vc = (M & 1) ? Vp2 : Vp;
    double* Pnext = (M & 1) ? Pn : Pn2;  // panel M+1's values (then panel M+3's)
    double* Pafter = (M & 1) ? Pn2 : Pn;  // panel M+2's values, published by C below
    const bool more = kTPP * (M + 1) < Tc;
    if (more) lookahead(Lc, Vc, Pnext, kPW * (M + 1));
    __syncthreads();
    LDLT_TS(2 + 2 * M);
    if (more) panel_rows(M + 1, Pnext, (M & 1) ? Lp : Lp2, (M & 1) ? Vp : Vp2);
    LDLT_TS(32 + M);  // (thread 0 is always a panel-row thread: the rows' chain ends here)
    trailing(M, Lc, Vc, Pafter);
    __syncthreads();
    LDLT_TS(3 + 2 * M);
  }
  if (fail) {
    if (tid == 0) D.scal[2] = 0.0;
    return;
  }
  if (tid >= 64) return;
  // L^T x = y one row at a time from the bottom: x_k = y_k (final once every row below is done) is
  // read out of its lane and each lane takes y_i -= L[k][i] x_k for its rows i < k.  Per row the
  // dependent chain is one lane read and one FMA; rows are loaded eight ahead (the lgkmcnt window
  // is 15) and the reads run past row k's k entries into the next rows or the panel arrays
  // (written LDS): they are masked where they are used -- a select right after a load would wait
  // for it there -- and the loops have no branches, so the waits stay per group of eight rows.
  // Two phases by the 64-row group of k, so that each row needs no select of its y register and
  // phase 2 (k < 64) leaves the upper group alone.
  // (The 8-row blocked form -- readlanes of a block, an 8x8 unit triangular solve, two register
  // sets of 44 LDS reads -- took 1.5k cycles per block, 24k of the kernel's 100k at N = 120.)
  const int lane = tid;
  double y[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int i = lane + 64 * r;
    y[r] = i < N ? ys[i] : 0.0;
  }
  static_assert(R == 2, "the two-phase row loop below: rows 64.. then 0..63");
  // Rows are clamped to [1, N-1]: a row k >= N (the 8-row groups round N up) reads row N-1's
  // entries, which are finite and meet x_k = y_k = 0, and no read leaves the kernel's LDS (the
  // lanes past a row's k entries read the next rows or the zero-initialised panel arrays).
  auto row_ptr = [&](int k) {
    const int r = min(max(k, 1), max(N - 1, 1));
    return Lpk + (size_t)r * (r - 1) / 2;
  };
  constexpr int kAhead = 8;  // rows loaded ahead (<= 15 LDS reads in flight)
  LDLT_TS(48);
  // phase 1 (N > 64): rows k = K1 .. 64 (K1 >= N - 1; rows k >= N have x_k = y_k = 0 and change
  // nothing): x_k sits in y[1]; rows i < 64 always take the update, rows i >= 64 only when i < k
  if (N > 64) {
    const int K1 = 64 + 8 * ((N - 64 + 7) / 8) - 1;
    double L0[kAhead], L1[kAhead];
#pragma unroll
    for (int u = 0; u < kAhead; u++) {
      const double* Lk = row_ptr(K1 - u);
      L0[u] = Lk[lane];
      L1[u] = Lk[lane + 64];
    }
    for (int k0 = K1; k0 >= 64; k0 -= kAhead) {
#pragma unroll
      for (int u = 0; u < kAhead; u++) {
        const int k = k0 - u;
        const double xk = readlane_d(y[1], k - 64);
        y[0] = __builtin_fma(-L0[u], xk, y[0]);
        const double y1 = __builtin_fma(-L1[u], xk, y[1]);
        y[1] = lane + 64 < k ? y1 : y[1];  // (rows at or past k keep their value: no 0 * inf)
        const double* Lk = row_ptr(k - kAhead);  // (rows below 64 of the next group: unused)
        L0[u] = Lk[lane];
        L1[u] = Lk[lane + 64];
      }
    }
  }
  // phase 2: rows k = K2 .. 0 (K2 = min(63, N - 1) rounded up to a group of eight), x_k in y[0];
  // rows i >= 64 are final
  {
    const int K2 = min(63, 8 * ((N + 7) / 8) - 1);
    double L0[kAhead];
#pragma unroll
    for (int u = 0; u < kAhead; u++) L0[u] = row_ptr(K2 - u)[lane];
    for (int k0 = K2; k0 >= 0; k0 -= kAhead) {
#pragma unroll
      for (int u = 0; u < kAhead; u++) {
        const int k = k0 - u;
        const double xk = readlane_d(y[0], k);
        const double y0 = __builtin_fma(-L0[u], xk, y[0]);
        y[0] = lane < k ? y0 : y[0];
        L0[u] = row_ptr(k - kAhead)[lane];  // (k - kAhead < 1: unused)
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++)
    if (lane + 64 * r < N) D.xp[lane + 64 * r] = y[r];
  if (lane == 0) D.scal[2] = 1.0;
  LDLT_TS(63);
}
template <int TPT, int NT, int R>
__global__ __launch_bounds__(NT) void k_ba_ldlt_pan(BaDev D) { k_ba_ldlt_pan_body<TPT, NT, R>(D); }
template <int TPT, int NT, int R>
__global__ __launch_bounds__(NT) void k_ba_ldlt_pan_many(const BaDev* __restrict__ Ds) {
  k_ba_ldlt_pan_body<TPT, NT, R>(Ds[blockIdx.z]);
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device), raised only when a larger
// size is asked for: the runtime call costs microseconds and used to sit between the launches of
// every LM phase (the device idled behind it)
inline hipError_t set_smem_attr(const void* fn, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(mu);
  size_t& have = done[{fn, dev}];
  if (bytes <= have) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) have = bytes;
  return e;
}

// Launch plan for the reduced system: the 8-wide panel kernel (N < 128), the column-step kernel while
// the packed factor fits LDS, else the 16-wide blocked MFMA kernel (LDS or global).  The debug options
// (orbx_debug_ba_options) can force the column-step or the blocked kernel where they fit, for tests.
struct LdltPlan {
  int N = 0, tpt = 0, nt = 1024;
  bool col = false, in_lds = false, pan = false;
  size_t smem = 0;
  hipError_t prepare(int n, bool allow_pan = true) {
    N = n;
    pan = allow_pan && ldlt_use_pan(N);
    if (pan) {
      col = false;
      in_lds = true;
      nt = 512;
      tpt = 1;
      smem = ldlt_pan_smem(N);
      return set_smem_attr(kernel_ptr(), smem);
    }
    col = ldlt_col_fits(N) && ba_opts().ldlt != ORBX_BA_LDLT_BLOCKED;
    if (col) {
      nt = 1024;
      const int tiles = ldlt_col_tiles(N);
      tpt = (tiles + nt - 1) / nt;
      if (tpt > 8 || (nt == 1024 && tpt > 2) || (nt == 512 && tpt > 4)) {
        nt = 1024;
        tpt = tiles <= 1024 ? 1 : 2;
      }
      tpt = tpt <= 1 ? 1 : tpt <= 2 ? 2 : tpt <= 4 ? 4 : 8;
      smem = ldlt_col_smem(N);
    } else {
      in_lds = ldlt_np(N) <= kLdltLdsNp;
      smem = ldlt_smem_bytes(N, in_lds);
    }
    return set_smem_attr(kernel_ptr(), smem);
  }
  const void* kernel_ptr() const {
    if (pan) return (const void*)k_ba_ldlt_pan<1, 512, 2>;
    if (col) {
      if (nt == 1024) return tpt == 1 ? (const void*)k_ba_ldlt_col<1, 1024> : (const void*)k_ba_ldlt_col<2, 1024>;
      if (nt == 512)
        return tpt == 1 ? (const void*)k_ba_ldlt_col<1, 512>
                        : tpt == 2 ? (const void*)k_ba_ldlt_col<2, 512> : (const void*)k_ba_ldlt_col<4, 512>;
      return tpt <= 2 ? (const void*)k_ba_ldlt_col<2, 256>
                      : tpt == 4 ? (const void*)k_ba_ldlt_col<4, 256> : (const void*)k_ba_ldlt_col<8, 256>;
    }
    return in_lds ? (const void*)k_ba_ldlt<true> : (const void*)k_ba_ldlt<false>;
  }
  // batched driver: the column-step kernel over K problems (blockIdx.z), sized for the largest
  const void* many_ptr() const {
    if (pan) return (const void*)k_ba_ldlt_pan_many<1, 512, 2>;
    if (nt == 1024) return tpt == 1 ? (const void*)k_ba_ldlt_col_many<1, 1024> : (const void*)k_ba_ldlt_col_many<2, 1024>;
    if (nt == 512)
      return tpt == 1 ? (const void*)k_ba_ldlt_col_many<1, 512>
                      : tpt == 2 ? (const void*)k_ba_ldlt_col_many<2, 512> : (const void*)k_ba_ldlt_col_many<4, 512>;
    return tpt <= 2 ? (const void*)k_ba_ldlt_col_many<2, 256>
                    : tpt == 4 ? (const void*)k_ba_ldlt_col_many<4, 256> : (const void*)k_ba_ldlt_col_many<8, 256>;
  }
  hipError_t prepare_many() const {
    return set_smem_attr(many_ptr(), smem);
  }
  void launch_many(const BaDev* Ds, int K, hipStream_t st) const {
    hipLaunchKernelGGL(reinterpret_cast<void (*)(const BaDev*)>(const_cast<void*>(many_ptr())), dim3(1, 1, K),
                       dim3(nt), smem, st, Ds);
  }
  void launch(const BaDev& D, hipStream_t st, int stage_limit = 99) const {
    if (col || pan) {
      hipLaunchKernelGGL(reinterpret_cast<void (*)(BaDev)>(const_cast<void*>(kernel_ptr())), dim3(1), dim3(nt),
                         smem, st, D);
    } else if (in_lds) {
      hipLaunchKernelGGL(k_ba_ldlt<true>, dim3(1), dim3(1024), smem, st, D, stage_limit);
    } else {
      hipLaunchKernelGGL(k_ba_ldlt<false>, dim3(1), dim3(1024), smem, st, D, stage_limit);
    }
  }
};

constexpr int kUpCh = 2048;  // k_ba_update: positions per LDS chunk (48 KB)
// k_ba_update: points per block (all LBS threads form the position products): 64 points take one
// round of position products per block and four times the blocks (10.8 -> 7.4 us at config 4;
// 32 points: 7.0 us, within the spread)
constexpr int kUpPts = 64;
static_assert(kUpPts <= LBS, "one thread per point");
// back-substitution + update (push first) + LM scale, skipped when the solve failed
// (scal[2] == 0).  Blocks: the active poses first (their se3 exp chains then overlap the point
// blocks), then LBS active points per block; one LM-scale partial per block.
__device__ __forceinline__ void k_ba_update_body(const BaDev& D, double lambda) {
  if (lm_skip(D) || (int)blockIdx.x >= D.nbu) return;
  lambda = lm_lambda(D, lambda);
  // device LM: the previous trial's pop is folded in (same values as k_ba_restore).
  // Every state value is loaded into registers before any store: the X / Xbak (cq, cbak)
  // stores may alias the next loads as far as the compiler knows, which otherwise
  // serialised each load behind the previous store (one memory round trip apiece).
  const bool rej = D.lm && D.lm->rejected;
  const bool ok = D.scal[2] != 0.0;
  const int npb = (D.nposes + LBS - 1) / LBS;
  double sc = 0;
  if ((int)blockIdx.x < npb) {
    const int pi = blockIdx.x * LBS + threadIdx.x;
    if (pi < D.nposes) {
      const int c = D.pose_cam[pi];
      double u[6], bp[6];
      for (int r = 0; r < 6; r++) {
        u[r] = D.xp[6 * pi + r];
        bp[r] = D.bp[6 * pi + r];
      }
      double q4[4], t3[3];
      if (rej) {
        for (int r = 0; r < 4; r++) q4[r] = D.cbak[7 * c + r];
        for (int r = 0; r < 3; r++) t3[r] = D.cbak[7 * c + 4 + r];
      } else {
        for (int r = 0; r < 4; r++) q4[r] = D.cq[4 * c + r];
        for (int r = 0; r < 3; r++) t3[r] = D.ct[3 * c + r];
      }
      if (ok) {
        for (int r = 0; r < 6; r++) sc += u[r] * (lambda * u[r] + bp[r]);
        for (int r = 0; r < 4; r++) D.cbak[7 * c + r] = q4[r];
        for (int r = 0; r < 3; r++) D.cbak[7 * c + 4 + r] = t3[r];
        const SE3d E = se3_exp(u);
        const Quat q = {q4[0], q4[1], q4[2], q4[3]};
        double rt[3];
        qrot(E.q, t3, rt);
        Quat nq = qmul(E.q, q);
        qnormalize(nq);
        D.cq[4 * c] = nq.x;
        D.cq[4 * c + 1] = nq.y;
        D.cq[4 * c + 2] = nq.z;
        D.cq[4 * c + 3] = nq.w;
        for (int r = 0; r < 3; r++) D.ct[3 * c + r] = E.t[r] + rt[r];
      } else if (rej) {
        for (int r = 0; r < 4; r++) D.cq[4 * c + r] = q4[r];
        for (int r = 0; r < 3; r++) D.ct[3 * c + r] = t3[r];
      }
    }
  } else {
    const int i0 = (blockIdx.x - npb) * kUpPts, i = i0 + threadIdx.x, i1 = min(i0 + kUpPts, D.npa);
    const bool pt = (int)threadIdx.x < kUpPts && i < D.npa;
    const int ic = pt ? i : i0;  // (i0 < npa in a point block) loads stay in range
    // everything that depends on neither the solve's flag nor the LM state, issued first
    const int p = D.pt_id[ic];
    const int ka = D.pt_off[ic], kz = pt ? D.pt_off[ic + 1] : ka;
    const int kb = D.pt_off[i0], ke = D.pt_off[i1];
    double c[3], bl[3], Di[9];
    for (int r = 0; r < 3; r++) c[r] = bl[r] = D.bl[3 * ic + r];
    for (int r = 0; r < 9; r++) Di[r] = D.Dinv[9 * (size_t)ic + r];
    const double* from = rej ? D.Xbak : D.X;
    const double X0[3] = {from[3 * p], from[3 * p + 1], from[3 * p + 2]};
    // b_l - sum_k Hpl_k^T x_c(k): the per-position products H_pl^T x_c are formed by all the
    // block's threads at once (4 positions per thread per round, every load issued before the
    // arithmetic) and staged in LDS; each point's thread then subtracts its positions' products
    // in position order.  (A thread per point walking its own positions paid two dependent
    // memory round trips per position.)  Unused when the solve failed.
    __shared__ double sq[kUpCh * 3];
    for (int base = kb; base < ke; base += kUpCh) {  // block-uniform
      const int n = min(kUpCh, ke - base);
      for (int u0 = threadIdx.x; u0 < n; u0 += 4 * LBS) {
        int ci[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
          const int u = u0 + s * LBS;
          ci[s] = u < n ? D.pcam[base + u] : -1;
        }
        double B[4][18], x[4][6];
#pragma unroll
        for (int s = 0; s < 4; s++) {
          const int u = min(u0 + s * LBS, n - 1);
          const double* h = D.Hpl + 18 * (size_t)(base + u);
          const double* xc = D.xp + 6 * max(ci[s], 0);
#pragma unroll
          for (int j = 0; j < 18; j++) B[s][j] = h[j];
#pragma unroll
          for (int r = 0; r < 6; r++) x[s][r] = xc[r];
        }
#pragma unroll
        for (int s = 0; s < 4; s++) {
          const int u = u0 + s * LBS;
          if (u < n) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
              double q = 0;
#pragma unroll
              for (int r = 0; r < 6; r++) q += B[s][3 * r + j] * x[s][r];
              sq[3 * u + j] = ci[s] >= 0 ? q : 0.0;  // fixed camera: no term
            }
          }
        }
      }
      __syncthreads();
      for (int k = max(ka, base); k < min(kz, base + n); k++)
#pragma unroll
        for (int j = 0; j < 3; j++) c[j] -= sq[3 * (k - base) + j];
      __syncthreads();
    }
    if (pt) {
      if (ok) {
        double x[3];
        for (int r = 0; r < 3; r++) x[r] = Di[3 * r] * c[0] + Di[3 * r + 1] * c[1] + Di[3 * r + 2] * c[2];
        for (int r = 0; r < 3; r++) sc += x[r] * (lambda * x[r] + bl[r]);
        for (int r = 0; r < 3; r++) {
          D.Xbak[3 * p + r] = X0[r];
          D.X[3 * p + r] = X0[r] + x[r];
        }
      } else if (rej) {
        for (int r = 0; r < 3; r++) D.X[3 * p + r] = X0[r];
      }
    }
  }
  block_partial(sc, D.scal + 8 + 2 * D.nbe);
}
__global__ __launch_bounds__(LBS) void k_ba_update(BaDev D, double lambda) { k_ba_update_body(D, lambda); }
__global__ __launch_bounds__(LBS) void k_ba_update_many(const BaDev* __restrict__ Ds, double lambda) {
  k_ba_update_body(Ds[blockIdx.z], lambda);
}

__device__ __forceinline__ void k_ba_restore_body(const BaDev& D) {
  if (D.lm && !D.lm->rejected) return;  // (a refresh always follows a rejected trial)
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i < D.npa) {
    const int p = D.pt_id[i];
    const double v[3] = {D.Xbak[3 * p], D.Xbak[3 * p + 1], D.Xbak[3 * p + 2]};  // loads before stores
    for (int r = 0; r < 3; r++) D.X[3 * p + r] = v[r];
  } else if (i < D.npa + D.nposes) {
    const int c = D.pose_cam[i - D.npa];
    double v[7];
    for (int r = 0; r < 7; r++) v[r] = D.cbak[7 * c + r];
    for (int r = 0; r < 4; r++) D.cq[4 * c + r] = v[r];
    for (int r = 0; r < 3; r++) D.ct[3 * c + r] = v[4 + r];
  }
}
__global__ __launch_bounds__(LBS) void k_ba_restore(BaDev D) { k_ba_restore_body(D); }
__global__ __launch_bounds__(LBS) void k_ba_restore_many(const BaDev* __restrict__ Ds) {
  k_ba_restore_body(Ds[blockIdx.z]);
}

// The caller's stop flag as the device sees it (host-mapped pinned pages):
// SparseOptimizer::terminate(), polled where the host loop polls it.
struct DevStop {
  const int* i;
  const bool* b;
  __device__ bool operator()() const {
    return (i && __hip_atomic_load(i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) ||
           (b && __hip_atomic_load(reinterpret_cast<const char*>(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0);
  }
};

// optimize() entry: lambda = tau * max diag(H) (computeLambdaInit), chi of
// the linearised state from errors slot 0 (block partials).
// Sum of n block partials in a fixed order, by one wave: lane l adds p[l], p[l + 64], ... in index
// order (eight loads in flight per round), then a butterfly over the 64 lanes.  Lane 0's value --
// the one the LM verdict uses -- is the same bits on every run and in the batched driver.  (It
// replaced lane 0 adding all partials in sequence through LDS: a ~170-add FP64 chain per sum on the
// trial's critical path, and no barrier is needed now, so any wave of a block may call it.)
template <bool coh = false>  // coh: p is read with ld_agent (partials stored by this launch's other blocks)
__device__ inline double fixed_sum_wave(const double* p, int n) {
  const int lane = threadIdx.x & 63;
  double s = 0;
  for (int base = 0; base < n; base += 512) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {  // clamped, unpredicated loads: all eight in flight at once
      const int i = max(min(base + lane + 64 * u, n - 1), 0);
      v[u] = coh ? ld_agent(p + i) : p[i];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) s += base + lane + 64 * u < n ? v[u] : 0.0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}
__device__ inline double seq_sum_wave(const double* p, int n) { return fixed_sum_wave<false>(p, n); }
// The host readback's order (partials added in index order, lane 0; block = one wave): the batched
// driver's reported final chi, which must equal the single driver's host-side sum bit for bit.
__device__ inline double index_order_sum_wave(const double* p, int n) {
  __shared__ double buf[1024];
  double s = 0;
  for (int base = 0; base < n; base += 1024) {
    const int m = min(1024, n - base);
    for (int i = threadIdx.x; i < m; i += 64) buf[i] = p[base + i];
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 0; i < m; i++) s += buf[i];
    __syncthreads();
  }
  return s;
}
// two such sums (the verdict's chi and LM scale); valid in lane 0 of every calling wave
template <bool coh = false>
__device__ inline void seq_sum2_wave(const double* p, int n, const double* q, int m, double& sp, double& sq) {
  sp = fixed_sum_wave<coh>(p, n);
  sq = fixed_sum_wave<false>(q, m);
}

__device__ __forceinline__ void k_ba_lm_init_body(const BaDev& D, int iterations) {
  LmState* L = const_cast<LmState*>(D.lm);
  const double a = seq_sum_wave(D.scal + 8, D.nbe);
  if (threadIdx.x != 0) return;
  L->lambda = 1e-5 * D.scal[3];
  L->ni = 2;
  L->currentChi = L->iniChi = a;
  L->it = L->qmax = L->nBad = L->trials = 0;
  L->relin = 0;  // linearised by the entry launches
  L->rejected = 0;
  L->iterations = iterations;
  L->stopped = 0;  // the host polled the flag just before this phase
  L->refresh = 0;
  L->done = iterations <= 0 ? 1 : 0;
  L->ticket = 0;
}
// A phase's entry after k_ba_cam_sum (single-problem device LM): k_ba_cam_fin, the lambda init (the
// max of |H_jj| over points and poses -> scal[3], a 1024-wide tree: max is order-free) and the LM
// state init in one launch; the batched driver runs k_ba_cam_fin_many, k_ba_dmax_many and
// k_ba_lm_init_many
__global__ __launch_bounds__(1024) void k_ba_lm_start(BaDev D, int iterations) {
  __shared__ double wmax[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < D.npa; i += 1024) acc = fmax(acc, D.dmax_p[i]);
  // k_ba_cam_fin's finalisation of the entry's pose sums: item (pose, j) sums the chunk partials of
  // its upper-triangle / rhs entry in chunk order (Hpp both triangles, bp); the diagonal entries'
  // |H_jj| join the lambda-init maximum here, and after the barrier each pose's thread takes its own
  // maximum from the six diagonal entries this block just wrote
  const int S = D.gsplit;
  auto csum = [&](int ci, int q) {  // chunk order; loads in groups of 8 (clamped) before their adds
    double t = 0;
    for (int c0 = 0; c0 < S; c0 += 8) {
      double v[8];
#pragma unroll
      for (int e = 0; e < 8; e++) v[e] = D.gpart[((size_t)ci * S + min(c0 + e, S - 1)) * 27 + q];
#pragma unroll
      for (int e = 0; e < 8; e++)
        if (c0 + e < S) t += v[e];
    }
    return t;
  };
  for (int it = threadIdx.x; it < D.nposes * 42; it += 1024) {
    const int ci = it / 42, j = it - ci * 42;
    if (j < 36) {
      const int r = min(j / 6, j % 6), c = max(j / 6, j % 6);
      const double v = csum(ci, r * 6 - (r * (r - 1)) / 2 + (c - r));
      D.Hpp[36 * ci + j] = v;
      if (j / 6 == j % 6) acc = fmax(acc, fabs(v));
    } else {
      D.bp[6 * ci + (j - 36)] = csum(ci, 21 + (j - 36));
    }
  }
  // the maximum over the block: wave maxima by lane exchanges, then the 16 of them (max is order-free)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc = fmax(acc, __shfl_xor(acc, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = acc;
  __syncthreads();  // (also orders the Hpp stores above before the per-pose reads below)
  for (int ci = threadIdx.x; ci < D.nposes; ci += 1024) {
    double m = 0;
    for (int r = 0; r < 6; r++) m = fmax(m, fabs(D.Hpp[36 * ci + 7 * r]));
    D.dmax_c[ci] = m;
  }
  if (threadIdx.x >= 64) return;
  if (threadIdx.x == 0) {
    double m = wmax[0];
    for (int w = 1; w < 16; w++) m = fmax(m, wmax[w]);
    D.scal[3] = m;  // (read back below by the same thread)
  }
  k_ba_lm_init_body(D, iterations);
}
__global__ __launch_bounds__(64) void k_ba_lm_init_many(const BaDev* __restrict__ Ds, int iterations) {
  k_ba_lm_init_body(Ds[blockIdx.z], iterations);
}

// One LM trial's verdict (OptimizationAlgorithmLevenberg::solve, the
// reference's arithmetic in the same order as the host loop of
// LocalBA::optimize): chi and LM scale summed from the block partials in
// block order, accept (lambda *= max(1/3, min(2/3, 1-(2rho-1)^3))) or reject
// (lambda *= ni, ni *= 2, restore), then the iteration bookkeeping: the
// <= 10 trial budget, rho == 0, the _nBad rule and the stop flag.
template <bool coh = false>
__device__ __forceinline__ void k_ba_lm_control_body(const BaDev& D, DevStop stop) {
  LmState* L = const_cast<LmState*>(D.lm);
  const int nbu = D.nbu;
  if (L->done) return;  // uniform; a finished phase keeps `rejected` for the final restore
  // the flag's host-memory read is issued first, so its latency hides behind the sums (one read
  // serves both of the loop's polls below; a flag raised after it is seen at the next trial)
  // (thread 0 alone reads it: the verdict below is thread 0's)
  const bool st = threadIdx.x == 0 && (stop() || (D.raise_after >= 0 && L->trials >= D.raise_after));  // (+ test hook)
  const double* p = D.scal + 8;
  double b, u;
  seq_sum2_wave<coh>(p + D.nbe, D.nbe, p + 2 * D.nbe, nbu, b, u);
  if (threadIdx.x != 0) return;
  L->rejected = 0;
  const bool ok2 = D.scal[2] != 0.0;
  if (L->qmax == 0) L->iniChi = L->currentChi;
  L->trials++;
  const double tempChi = ok2 ? b : 1.7976931348623157e308;
  double rho = L->currentChi - tempChi;
  double scale = ok2 ? u : 0.0;
  scale += 1e-3;
  rho /= scale;
  if (rho > 0 && isfinite(tempChi)) {
    double alpha = 1. - lm_cube(2 * rho - 1);
    alpha = alpha < 2. / 3. ? alpha : 2. / 3.;
    const double scaleFactor = 1. / 3. > alpha ? 1. / 3. : alpha;
    L->lambda *= scaleFactor;
    L->ni = 2;
    L->currentChi = tempChi;
  } else {
    L->lambda *= L->ni;
    L->ni *= 2;
    if (ok2) L->rejected = 1;
  }
  L->qmax++;
  if (rho < 0 && L->qmax < 10 && !st) {  // another trial of this iteration
    L->relin = 0;
    return;
  }
  L->it++;
  bool brk = L->qmax == 10 || rho == 0;
  if (!brk) {
    if ((L->iniChi - L->currentChi) * 1e3 < L->iniChi)
      L->nBad++;
    else
      L->nBad = 0;
    brk = L->nBad >= 3;
  }
  L->qmax = 0;
  const bool st2 = !brk && L->it < L->iterations && st;
  L->stopped = st || st2;
  L->done = (brk || L->it >= L->iterations || st2) ? 1 : 0;
  L->relin = L->done ? 0 : 1;
  if (!L->done && L->rejected) {
    // rho was NaN: the iteration ended on a rejection and the phase goes on.  g2o pops the
    // trial and its next iteration recomputes the errors at the restored state; pause the
    // phase until the host has queued exactly that (restore, errors, k_ba_lm_resume).
    L->refresh = 1;
    L->done = 1;
  }
}

// Resume a phase paused for a refresh: chi of the recomputed errors (slot 0, block order, as
// the host loop's computeActiveErrors + activeRobustChi2) becomes the iteration's starting chi.
__device__ __forceinline__ void k_ba_lm_resume_body(const BaDev& D) {
  LmState* L = const_cast<LmState*>(D.lm);
  if (!L->refresh) return;
  const double a = seq_sum_wave(D.scal + 8, D.nbe);
  if (threadIdx.x != 0) return;
  L->currentChi = a;
  L->rejected = 0;
  L->refresh = 0;
  L->done = 0;
  L->relin = 1;
}
__global__ __launch_bounds__(64) void k_ba_lm_resume(BaDev D) { k_ba_lm_resume_body(D); }
__global__ __launch_bounds__(64) void k_ba_lm_resume_many(const BaDev* __restrict__ Ds) {
  k_ba_lm_resume_body(Ds[blockIdx.z]);
}
// A trial's k_ba_errors(D, 1, 1) and k_ba_lm_control in one launch (single-problem device LM): every
// block's thread 0 stores its chi partial (agent scope) and then takes a ticket with an agent-scope
// acq_rel RMW; the block whose ticket is the last one has thereby acquired every other block's
// release, i.e. every partial store happens-before its reads (the block barrier carries that to the
// rest of the block).  That block runs the verdict (wave 0 works, the other waves only pass the
// barriers).  Same partials, same order, same arithmetic as the two launches k_ba_errors +
// k_ba_lm_control, which are the default (debug option fused_ctl selects this one; tests compare
// the two bit for bit): the per-block release costs more than the dispatch it saves.
__global__ __launch_bounds__(LBS) void k_ba_errors_ctl(BaDev D, DevStop stop) {
  if (!k_ba_errors_body<true>(D, 1, 1)) return;
  __shared__ int last;
  if (threadIdx.x == 0) {
    unsigned* tk = &const_cast<LmState*>(D.lm)->ticket;
    // release RMW in every block (the RMWs form one release sequence); only the block that reads the
    // last ticket needs the acquire, as a fence after its RMW (the other blocks skip the L2 invalidate)
    last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(D.nbe - 1);
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;  // (uniform per block)
  k_ba_lm_control_body<true>(D, stop);
}
// The two-launch form's verdict (the default): after k_ba_errors(D, 1, 1), one wave.
__global__ __launch_bounds__(64) void k_ba_lm_control(BaDev D, DevStop stop) { k_ba_lm_control_body(D, stop); }
__global__ __launch_bounds__(64) void k_ba_lm_control_many(const BaDev* __restrict__ Ds, DevStop stop) {
  k_ba_lm_control_body(Ds[blockIdx.z], stop);
}

// Batched driver helpers (one block per problem, blockIdx.z): the lambda-init
// maximum of |H_jj| (k_ba_lm_start's partition and order) and the phase's final
// chi from errors slot 0 (summed in block order, like the host readback).
__global__ __launch_bounds__(1024) void k_ba_dmax_many(const BaDev* __restrict__ Ds) {
  const BaDev& D = Ds[blockIdx.z];
  __shared__ double sm[1024];
  const int n = D.npa + D.nposes;
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) acc = fmax(acc, D.dmax_p[i]);
  sm[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) sm[threadIdx.x] = fmax(sm[threadIdx.x], sm[threadIdx.x + o]);
    __syncthreads();
  }
  if (threadIdx.x == 0) D.scal[3] = sm[0];
}
__global__ __launch_bounds__(64) void k_ba_lm_final_many(const BaDev* __restrict__ Ds) {
  const BaDev& D = Ds[blockIdx.z];
  const double a = index_order_sum_wave(D.scal + 8, D.nbe);
  if (threadIdx.x == 0) const_cast<LmState*>(D.lm)->final_chi = a;
}

// Block-wide exclusive scan of one int per thread under `op` (identity
// `ident`); *total gets the reduction over the block.  ws: NT/64 ints of LDS.
template <int NT, typename Op>
__device__ inline int ba_block_scan(int v, int ident, Op op, int* ws, int* total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x = op(x, y);
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  if (w == 0) {  // scan of the wave totals: NW lanes of wave 0
    int s = lane < NW ? ws[lane] : ident;
    for (int d = 1; d < NW; d <<= 1) {
      const int y = __shfl_up(s, d, 64);
      if (lane >= d) s = op(s, y);
    }
    if (lane < NW) ws[lane] = s;
  }
  __syncthreads();
  int ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = ident;
  const int r = w ? op(ws[w - 1], ex) : ex;
  *total = ws[NW - 1];
  __syncthreads();  // ws free for the next scan
  return r;
}

// Lanes of the wave holding the same key (keys < 2^nbits): one ballot per bit.
__device__ inline uint64_t ba_match(int key, int nbits) {
  uint64_t m = ~0ull;
  for (int b = 0; b < nbits; b++) {
    const bool s = (key >> b) & 1;
    const uint64_t bal = __ballot(s);
    m &= s ? bal : ~bal;
  }
  return m;
}

// Active-edge structure of a phase on the device: build_structure's one-pass
// (edges grouped by point) path, same arrays, same order, in three launches
// over tiles of kTileE edges (kTileT threads x kStructV contiguous edges, so
// positions keep edge order):
//  k_ba_struct_count  per tile: active edges per camera, active count,
//                     first/last active point, point segments inside the tile;
//  k_ba_struct_scan   one block: camera totals -> pose tables (one camera per
//                     thread, nc <= kStructMaxNc), per (tile, camera) cam_pos
//                     offsets, per tile position/point/segment carries, boff
//                     and the five sizes;
//  k_ba_struct_fill   per tile: act/pos_pt/pcam/pt_off/pt_id, and cam_pos as a
//                     stable per-wave multisplit of the tile's positions by
//                     camera (bitwise match, no atomics), ascending in a pose.
#ifndef ORBX_STRUCT_V
#define ORBX_STRUCT_V 4
#endif
// 4 edges per thread (1,024-edge tiles): at config 4 the three launches take 23.7 µs against 29.5 with
// 8 (k_ba_struct_fill 14.5 -> 9.1, k_ba_struct_scan 8.7 -> 9.8 over twice the tiles; profiles/r05)
constexpr int kTileT = 256, kStructV = ORBX_STRUCT_V, kTileE = kTileT * kStructV;  // kTileE < 2^16: packed scans
constexpr int kStructNT = 1024, kStructMaxNc = 512, kStructMaxTiles = kStructNT;

__device__ inline void ba_tile_load(const BaDev& D, const uint8_t* __restrict__ flag, int lvl, int e0, bool* a,
                                    int* pt, int* cm) {
#pragma unroll
  for (int j = 0; j < kStructV; j++) {
    const int e = e0 + j;
    const bool in = e < D.ne;
    pt[j] = in ? D.ept[e] : -1;
    cm[j] = in ? D.ecam[e] : 0;
    a[j] = in && (lvl < 0 || flag[e] == lvl);
  }
}

struct BaAdd {
  __device__ int operator()(int a, int b) const { return a + b; }
};
struct BaMax {
  __device__ int operator()(int a, int b) const { return a > b ? a : b; }
};
struct BaMin {
  __device__ int operator()(int a, int b) const { return a < b ? a : b; }
};

__global__ __launch_bounds__(kTileT) void k_ba_struct_count(BaDev D, const uint8_t* __restrict__ flag, int lvl,
                                                            int* __restrict__ tcnt, int4* __restrict__ ttot) {
  if (spec_skip(D)) return;  // (block-uniform, before any barrier)
  constexpr int V = kStructV;
  extern __shared__ int sm_sc[];
  const int nc = D.nc, t = threadIdx.x, tile = blockIdx.x;
  int* hc = sm_sc;    // nc
  int* ws = hc + nc;  // kTileT/64
  for (int i = t; i < nc; i += kTileT) hc[i] = 0;
  bool a[V];
  int pt[V], cm[V];
  ba_tile_load(D, flag, lvl, tile * kTileE + t * V, a, pt, cm);
  __syncthreads();
  int nact = 0, lastp = -1, firstp = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < V; j++)
    if (a[j]) {
      atomicAdd(&hc[cm[j]], 1);
      nact++;
      lastp = pt[j];
      firstp = min(firstp, pt[j]);
    }
  int tlast, tot, tfirst;
  // points ascend along the edge list: the max over earlier edges is the
  // point of the last active edge before this thread's (-1: none in the tile)
  const int p = ba_block_scan<kTileT>(lastp, -1, BaMax(), ws, &tlast);
  int nseg = 0;
#pragma unroll
  for (int j = 0, q = p; j < V; j++)
    if (a[j]) {
      nseg += pt[j] != q;
      q = pt[j];
    }
  (void)ba_block_scan<kTileT>(nact | nseg << 16, 0, BaAdd(), ws, &tot);
  (void)ba_block_scan<kTileT>(firstp, 0x7fffffff, BaMin(), ws, &tfirst);
  for (int i = t; i < nc; i += kTileT) tcnt[(size_t)tile * nc + i] = hc[i];
  if (t == 0) ttot[tile] = make_int4(tot & 0xffff, tfirst, tlast, tot >> 16);
}

__global__ __launch_bounds__(kStructNT) void k_ba_struct_scan(BaDev D, const uint8_t* __restrict__ fixed, int ntiles,
                                                              int* __restrict__ tcnt, const int4* __restrict__ ttot,
                                                              int4* __restrict__ tcar, int* __restrict__ out) {
  if (spec_skip(D)) return;
  constexpr int NT = kStructNT;
  extern __shared__ int sm_ss[];
  const int nc = D.nc, t = threadIdx.x;
  int* coff = sm_ss;        // nposes+1
  int* ws = coff + nc + 1;  // NW
  // camera totals; tcnt becomes each tile's offset inside its camera's run
  int cc = 0;
  if (t < nc)
    for (int i0 = 0; i0 < ntiles; i0 += 8) {  // loads of 8 tiles in flight before their stores
      int x[8];
#pragma unroll
      for (int j = 0; j < 8; j++) x[j] = i0 + j < ntiles ? tcnt[(size_t)(i0 + j) * nc + t] : 0;
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (i0 + j < ntiles) tcnt[(size_t)(i0 + j) * nc + t] = cc;
        cc += x[j];
      }
    }
  int nposes, tot, maxc, na, npa, nslots, tmp;
  const bool pose = t < nc && cc > 0 && !fixed[t];
  const int pidx = ba_block_scan<NT>(pose ? 1 : 0, 0, BaAdd(), ws, &nposes);
  const int pofs = ba_block_scan<NT>(pose ? cc : 0, 0, BaAdd(), ws, &tot);
  (void)ba_block_scan<NT>(pose ? cc : 0, 0, BaMax(), ws, &maxc);
  if (t < nc) D.chidx[t] = pose ? pidx : -1;
  if (pose) {
    D.pose_cam[pidx] = t;
    coff[pidx] = pofs;
    D.cam_off[pidx] = pofs;
  }
  // tile carries: first position, last active point before the tile, first segment
  const int4 tt = t < ntiles ? ttot[t] : make_int4(0, 0x7fffffff, -1, 0);
  const int kb = ba_block_scan<NT>(tt.x, 0, BaAdd(), ws, &na);
  const int pv = ba_block_scan<NT>(tt.z, -1, BaMax(), ws, &tmp);
  const int sg = tt.w - (tt.x > 0 && tt.y == pv ? 1 : 0);  // first point continues the previous tile's
  const int sb = ba_block_scan<NT>(sg, 0, BaAdd(), ws, &npa);
  if (t < ntiles) tcar[t] = make_int4(kb, pv, sb, 0);
  if (t == 0) {
    coff[nposes] = tot;
    D.cam_off[nposes] = tot;
    D.pt_off[npa] = na;
  }
  __syncthreads();
  // boff: block (c1, c2 >= c1) holds one slot per position of pose c1
  const int n1 = t < nposes ? coff[t + 1] - coff[t] : 0;
  const int q = ba_block_scan<NT>(t < nposes ? n1 * (nposes - t) : 0, 0, BaAdd(), ws, &nslots);
  if (t < nposes) {
    const int b0 = t * nposes - t * (t - 1) / 2;
    for (int j = 0; j < nposes - t; j++) D.boff[b0 + j] = q + j * n1;
  }
  if (t == 0) {
    D.boff[nposes * (nposes + 1) / 2] = nslots;
    out[0] = na;
    out[1] = npa;
    out[2] = nposes;
    out[3] = maxc;
    out[4] = nslots;
  }
}

__global__ __launch_bounds__(kTileT) void k_ba_struct_fill(BaDev D, const uint8_t* __restrict__ flag, int lvl,
                                                           const int* __restrict__ tcnt,
                                                           const int4* __restrict__ tcar) {
  if (spec_skip(D)) return;
  constexpr int V = kStructV, NW = kTileT / 64;
  extern __shared__ int sm_sf[];
  const int nc = D.nc, t = threadIdx.x, lane = t & 63, w = t >> 6, tile = blockIdx.x;
  int* chl = sm_sf;        // nc: pose index per camera
  int* cw = chl + nc;      // NW*nc: per-wave camera counts, then fill cursors
  int* lpc = cw + NW * nc; // kTileE: camera of each tile position (-1: fixed)
  int* ws = lpc + kTileE;  // NW
  for (int i = t; i < nc; i += kTileT) chl[i] = D.chidx[i];
  for (int i = t; i < NW * nc; i += kTileT) cw[i] = 0;
  const int4 car = tcar[tile];
  bool a[V];
  int pt[V], cm[V];
  const int e0 = tile * kTileE + t * V;
  ba_tile_load(D, flag, lvl, e0, a, pt, cm);
  int nact = 0, lastp = -1;
#pragma unroll
  for (int j = 0; j < V; j++) {
    nact += a[j];
    if (a[j]) lastp = pt[j];
  }
  int tlast, tks;
  int p = max(car.y, ba_block_scan<kTileT>(lastp, -1, BaMax(), ws, &tlast));
  int nseg = 0;
#pragma unroll
  for (int j = 0, q = p; j < V; j++)
    if (a[j]) {
      nseg += pt[j] != q;
      q = pt[j];
    }
  const int ks = ba_block_scan<kTileT>(nact | nseg << 16, 0, BaAdd(), ws, &tks);
  int kl = ks & 0xffff;
  int s = car.z + (ks >> 16) - 1;
#pragma unroll
  for (int j = 0; j < V; j++)
    if (a[j]) {
      if (pt[j] != p) {
        s++;
        D.pt_off[s] = car.x + kl;
        D.pt_id[s] = pt[j];
        p = pt[j];
      }
      const int pc = chl[cm[j]];
      D.act[car.x + kl] = e0 + j;
      D.pos_pt[car.x + kl] = s;
      D.pcam[car.x + kl] = pc;
      lpc[kl] = pc >= 0 ? cm[j] : -1;
      kl++;
    }
  __syncthreads();
  // cam_pos: stable multisplit of the tile's positions by camera
  const int nt = tks & 0xffff, nbits = 32 - __clz(nc);
  const int R = (((nt + NW - 1) / NW) + 63) & ~63;
  const int k0 = min(w * R, nt), k1 = min(k0 + R, nt);
  for (int kb = k0; kb < k1; kb += 64) {
    const int kk = kb + lane;
    const int c = kk < k1 ? lpc[kk] : -1;
    const uint64_t m = ba_match(c >= 0 ? c : nc, nbits);
    if (c >= 0 && __popcll(m & ((1ull << lane) - 1)) == 0) cw[w * nc + c] += __popcll(m);
  }
  __syncthreads();
  for (int c = t; c < nc; c += kTileT)
    if (chl[c] >= 0) {
      int run = D.cam_off[chl[c]] + tcnt[(size_t)tile * nc + c];
      for (int v = 0; v < NW; v++) {
        const int x = cw[v * nc + c];
        cw[v * nc + c] = run;
        run += x;
      }
    }
  __syncthreads();
  for (int kb = k0; kb < k1; kb += 64) {
    const int kk = kb + lane;
    const int c = kk < k1 ? lpc[kk] : -1;
    const uint64_t m = ba_match(c >= 0 ? c : nc, nbits);
    const int r = __popcll(m & ((1ull << lane) - 1));
    const int b = c >= 0 ? cw[w * nc + c] : 0;
    if (c >= 0) D.cam_pos[b + r] = car.x + kk;
    if (c >= 0 && r == 0) cw[w * nc + c] = b + __popcll(m);
  }
}

// Problem intake on the device: the caller's float observations / points
// become the FP64 edge and vertex arrays (Converter / g2o setMeasurement
// casts), the per-edge stereo flag, Huber delta (the float sqrt thresholds of
// src/Optimizer.cc:653-654, passed from the host) and its float square, robust
// flags on, stored errors zero.  Only the raw arrays cross PCIe.
__global__ __launch_bounds__(LBS) void k_ba_prep(int ne, int np, const float* __restrict__ obs,
                                                 const float* __restrict__ isig, const float* __restrict__ Xf,
                                                 double* __restrict__ X, uint8_t* __restrict__ est,
                                                 double* __restrict__ eobs, double* __restrict__ einfo,
                                                 double* __restrict__ edelta, float* __restrict__ edsqr,
                                                 uint8_t* __restrict__ erob, double* __restrict__ eerr, float thMono,
                                                 float thStereo) {
  const int i = blockIdx.x * LBS + threadIdx.x;
  if (i < ne) {
    const float u = obs[3 * i], v = obs[3 * i + 1], ur = obs[3 * i + 2];
    const bool s = ur >= 0;
    est[i] = s ? 1 : 0;
    eobs[3 * i] = u;
    eobs[3 * i + 1] = v;
    eobs[3 * i + 2] = ur;
    einfo[i] = isig[i];
    const double d = s ? thStereo : thMono;
    edelta[i] = d;
    edsqr[i] = (float)(d * d);
    erob[i] = 1;
    eerr[3 * i] = eerr[3 * i + 1] = eerr[3 * i + 2] = 0.0;
  }
  if (i < 3 * np) X[i] = Xf[i];
}

// phase transition (:764-802) and the final erase test (:817-847): per edge
// chi2 of its stored error against th, and depth of the current estimate
__global__ __launch_bounds__(LBS) void k_ba_outliers(BaDev D, uint8_t* flag, int drop_kernel) {
  if (spec_skip(D)) return;
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
  DBuf<double> cbak, Xbak, eerr, Hpl, ptc, cmc, BD, cf, Hll, bl, Dinv, dmax_p, Hpp, bp, xp, bs, S, Sw, scal, gpart, gpose;

  DBuf<int> ptab;
  DBuf<uint8_t> flag;
  DBuf<LmState> lm;
  DBuf<uint8_t> prob;  // k_ba_prep outputs: FP64 points and edge arrays
};

#define HIP_TRY(x)                      \
  do {                                  \
    const hipError_t e_ = (x);          \
    if (e_ != hipSuccess) return e_;    \
  } while (0)
#define BA_CHECK(x)                          \
  do {                                       \
    if ((x) != hipSuccess) return ORBX_ERR_HIP; \
  } while (0)

// Pinned host staging buffer + one device arena: arrays are laid out with
// take(), filled through host(), and sent with one async copy.
// A pinned host block and its device twin, carved by take() in the same offsets.  mapped: no
// twin -- dbuf is the device's view of the pinned block itself, so kernels write results straight
// into host memory (no copy, no copy engine hand-off after the last kernel)
struct Arena {
  uint8_t* hbuf = nullptr;
  uint8_t* dbuf = nullptr;
  size_t cap = 0, off = 0;
  bool mapped = false;
  explicit Arena(bool m = false) : mapped(m) {}
  ~Arena() { release(); }
  void release() {
    if (hbuf) (void)hipHostFree(hbuf);
    if (dbuf && !mapped) (void)hipFree(dbuf);
    hbuf = dbuf = nullptr;
  }
  hipError_t reserve(size_t bytes) {
    off = 0;
    if (bytes <= cap && hbuf) return hipSuccess;
    release();
    cap = bytes + bytes / 4 + 4096;
    hipError_t e = hipHostMalloc((void**)&hbuf, cap, mapped ? hipHostMallocMapped : hipHostMallocDefault);
    if (e == hipSuccess)
      e = mapped ? hipHostGetDevicePointer((void**)&dbuf, hbuf, 0) : hipMalloc((void**)&dbuf, cap);
    if (e != hipSuccess) {
      release();
      cap = 0;
    }
    return e;
  }
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* d = reinterpret_cast<T*>(dbuf + off);
    off += std::max<size_t>(n, 1) * sizeof(T);
    return d;
  }
  template <class T>
  T* host(T* d) {
    return reinterpret_cast<T*>(hbuf + (reinterpret_cast<uint8_t*>(d) - dbuf));
  }
  template <class T>
  T* put(const std::vector<T>& v) {
    T* d = take<T>(v.size());
    if (!v.empty()) std::memcpy(host(d), v.data(), v.size() * sizeof(T));
    return d;
  }
  hipError_t upload(hipStream_t st) {
    return off && !mapped ? hipMemcpyAsync(dbuf, hbuf, off, hipMemcpyHostToDevice, st) : hipSuccess;
  }
};

inline size_t arena_bytes(std::initializer_list<size_t> sizes) {
  size_t t = 0;
  for (size_t x : sizes) t += ((std::max<size_t>(x, 1) + 255) & ~(size_t)255);
  return t + 256;
}

struct LocalBA {
  BaDev D{};
  Ctx c;  // device buffers, kept across calls (grow only)
  Arena prob_arena, struct_arena;
  // result write-back: k_ba_outliers / k_ba_export write the flags, poses and points straight
  // into a mapped pinned block, then host copies into the caller's arrays.  (A device arena read
  // back by one copy measured 81 us of copy-engine hand-off after k_ba_export plus the 11 us copy
  // per call, profiles/r05/localba_timeline_*.txt)
  Arena wb_arena{true};
  struct Wb {
    double *Tcw_d, *Xw_d;
    float *Tcw, *Xw;
    uint8_t* flag;
  } wb{};
  std::vector<int> e_pt, e_cam;
  std::vector<uint8_t> fixed;
  std::vector<uint8_t> level;  // 0/1 per edge
  int trials = 0;
  int nbu = 1, n_rb = 8;           // k_ba_update blocks; doubles in the readback block
  double* rb_host = nullptr;       // pinned readback block (mapped: rb_map is the device's view)
  double* rb_map = nullptr;
  int rb_cap = 0;
  hipEvent_t rb_ev = nullptr;      // recorded after the readback copy (the wait skips later work)
  // the linearisation outputs the LM trials read
  struct LinSet {
    double *Hpl, *Hll, *bl, *dmax_p, *Hpp, *bp;
  };
  LinSet lin0 = {};
  LocalBA() = default;
  LocalBA(const LocalBA&) = delete;
  LocalBA& operator=(const LocalBA&) = delete;
  ~LocalBA() {
    if (rb_host) (void)hipHostFree(rb_host);
    if (rb_ev) (void)hipEventDestroy(rb_ev);
    if (sint_host) (void)hipHostFree(sint_host);
    if (lm_host) (void)hipHostFree(lm_host);
    if (own_stop) (void)hipHostFree(own_stop);
    if (mirror) (void)hipHostFree(mirror);
  }
  int* own_stop = nullptr;  // orbx_ba_stop_flag: pinned, device-readable
  bool hook_stopped = false;  // ORBX_BA_RAISE_STOP_AFTER fired (the host then stops as for a raised flag)
  static void use_lin(BaDev& D, const LinSet& L) {
    D.Hpl = L.Hpl;
    D.Hll = L.Hll;
    D.bl = L.bl;
    D.Hpp = L.Hpp;
    D.bp = L.bp;
    D.dmax_p = L.dmax_p;
    D.dmax_c = L.dmax_p + D.npa;  // contiguous: one max-reduction for lambda init
  }
  // computeActiveErrors is not repeated: the errors/chi stored by the trial
  // (recompute, slot 1) are the ones at the state being linearised
  static void lin_points(const BaDev& Dl, hipStream_t st) {
    const int ga = std::max((Dl.na + LBS - 1) / LBS, 1);
    if (Dl.na > 0) hipLaunchKernelGGL(k_ba_linearize, dim3(ga), dim3(LBS), 0, st, Dl);
    if (Dl.npa > 0) hipLaunchKernelGGL(k_ba_point_sum, dim3((Dl.npa + LBS - 1) / LBS), dim3(LBS), 0, st, Dl);
  }
  // fused point side (k_ba_lin_schur): edges grouped by point with at most kFuseMaxDeg per point
  bool fuse_ok = false;
  DBuf<int> pblk;
  // host scratch, reused across calls
  std::vector<int> act, pos_pt, chidx, pose_cam, pt_off, pt_id, cam_off, cam_pos, cnt, pcam, ccnt, ccnt4, boff;

  // Active set of a phase: SparseOptimizer::initializeOptimization(level) +
  // buildIndexMapping; point-major positions, pose groups (positions
  // ascending within each pose).  Edges arriving grouped by point (the
  // reference adds them per MapPoint, Optimizer.cc:659-745) take the one-pass
  // path; otherwise a stable counting sort by point.  Schur pairs are found on
  // the device (k_ba_pairs), not listed here.
  double t_struct[4] = {0, 0, 0, 0};  // host ms: index/CSR, pose groups, device build, upload+alloc
  bool dev_struct = false;  // k_ba_struct_* build the arrays (edges grouped by point, nc <= kStructMaxNc)
  const uint8_t* dfix = nullptr;  // device copy of the fixed flags
  DBuf<int> sbuf;                 // k_ba_struct_* tiles and outputs, sized for the whole edge list
  int* sint_host = nullptr;       // pinned, mapped: k_ba_struct_scan's five sizes (written there directly)
  int* sint_map = nullptr;
  int sizes1[5] = {0, 0, 0, 0, 0};  // phase-1 sizes (all edges active), counted on the host
  orbx_status build_structure(int lvl, hipStream_t st) {
    if (dev_struct) return build_structure_dev(lvl, st, lvl < 0 ? sizes1 : nullptr);
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto T0 = now();
    const int nc = D.nc, np = D.np, ne = D.ne;
    const uint8_t* lv = level.data();
    ccnt.assign(nc, 0);
    int na = 0;
    bool sorted = true;
    for (int e = 0, last = -1; e < ne; e++)
      if (lvl < 0 || lv[e] == lvl) {
        ccnt[e_cam[e]]++;
        na++;
        sorted &= e_pt[e] >= last;
        last = e_pt[e];
      }
    chidx.assign(nc, -1);
    pose_cam.clear();
    cam_off.assign(1, 0);
    for (int c = 0; c < nc; c++)
      if (ccnt[c] && !fixed[c]) {
        chidx[c] = (int)pose_cam.size();
        pose_cam.push_back(c);
        cam_off.push_back(cam_off.back() + ccnt[c]);
      }
    const int nposes = (int)pose_cam.size();
    int maxc = 0;
    for (int ci = 0; ci < nposes; ci++) maxc = std::max(maxc, cam_off[ci + 1] - cam_off[ci]);
    act.resize(na);
    pos_pt.resize(na);
    pcam.resize(na);
    pt_off.clear();
    pt_id.clear();
    if (sorted) {
      int k = 0;
      for (int e = 0; e < ne; e++)
        if (lvl < 0 || lv[e] == lvl) {
          const int p = e_pt[e];
          if (pt_id.empty() || pt_id.back() != p) {
            pt_off.push_back(k);
            pt_id.push_back(p);
          }
          act[k] = e;
          pos_pt[k] = (int)pt_id.size() - 1;
          pcam[k] = chidx[e_cam[e]];
          k++;
        }
      pt_off.push_back(na);
    } else {
      cnt.assign(np + 1, 0);
      for (int e = 0; e < ne; e++)
        if (lvl < 0 || lv[e] == lvl) cnt[e_pt[e] + 1]++;
      pt_off.push_back(0);
      for (int p = 0; p < np; p++) {
        const int n = cnt[p + 1];
        cnt[p + 1] = cnt[p] + n;  // start of point p's positions
        if (n) {
          pt_id.push_back(p);
          pt_off.push_back(cnt[p + 1]);
        }
      }
      for (int e = 0; e < ne; e++)
        if (lvl < 0 || lv[e] == lvl) act[cnt[e_pt[e]]++] = e;  // stable: ascending edge order per point
      for (int i = 0; i < (int)pt_id.size(); i++)
        for (int k = pt_off[i]; k < pt_off[i + 1]; k++) pos_pt[k] = i;
      for (int k = 0; k < na; k++) pcam[k] = chidx[e_cam[act[k]]];
    }
    const int npa = (int)pt_id.size();
    const auto T1 = now();
    cam_pos.resize(cam_off[nposes]);
    {
      std::vector<int>& fill = cnt;  // reuse
      fill.assign(cam_off.begin(), cam_off.end());
      for (int k = 0; k < na; k++)
        if (pcam[k] >= 0) cam_pos[fill[pcam[k]]++] = k;
    }
    const auto T2 = now();
    const auto T3 = T2;
    boff.assign(1, 0);
    for (int c1 = 0; c1 < nposes; c1++)
      for (int c2 = c1; c2 < nposes; c2++) boff.push_back(boff.back() + cam_off[c1 + 1] - cam_off[c1]);
    // one upload
    hipError_t he = struct_arena.reserve(arena_bytes({4 * (size_t)na, 4 * (size_t)na, 4 * (size_t)nc,
                                                      4 * (size_t)nposes, 4 * (size_t)(npa + 1), 4 * (size_t)npa,
                                                      4 * (size_t)(nposes + 1), 4 * cam_pos.size(), 4 * (size_t)na,
                                                      4 * boff.size()}));
    if (he != hipSuccess) return ORBX_ERR_HIP;
    Arena& A = struct_arena;
    D.act = A.put(act);
    D.pos_pt = A.put(pos_pt);
    D.chidx = A.put(chidx);
    D.pose_cam = A.put(pose_cam);
    D.pt_off = A.put(pt_off);
    D.pt_id = A.put(pt_id);
    D.cam_off = A.put(cam_off);
    D.cam_pos = A.put(cam_pos);
    D.pcam = A.put(pcam);
    D.boff = A.put(boff);
    BA_CHECK(A.upload(st));
    const orbx_status fs = finish_structure(na, npa, nposes, maxc, boff.back(), st);
    const auto T4 = now();
    t_struct[0] += ms(T0, T1);
    t_struct[1] += ms(T1, T2);
    t_struct[2] += ms(T2, T3);
    t_struct[3] += ms(T3, T4);
    return fs;
  }

  // The same arrays built by k_ba_struct_* from the device-resident edge list
  // and phase flags (no host copy of the flags, no upload); one readback of
  // the five sizes the launch grids and allocations need (none when the
  // sizes are known: phase 1, every edge active).
  orbx_status build_structure_dev(int lvl, hipStream_t st, const int* known) {
    const auto T0 = std::chrono::steady_clock::now();
    BA_CHECK(launch_structure_dev(lvl, st, known, nullptr));
    const int* sz = known;
    if (!sz) {
      BA_CHECK(hipStreamSynchronize(st));
      sz = sint_host;
    }
    const orbx_status fs = finish_structure(sz[0], sz[1], sz[2], sz[3], sz[4], st);
    t_struct[2] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
    return fs;
  }
  // The structure kernels alone (sizes to the mapped sint_host unless known); gate: the device LM
  // state that gates them (spec_skip), or null.  The host reads the sizes after the stream's next
  // synchronisation point and calls finish_structure.
  hipError_t launch_structure_dev(int lvl, hipStream_t st, const int* known, const LmState* gate) {
    const int nc = D.nc, ne = D.ne;
    const int ntiles = (ne + kTileE - 1) / kTileE;
    const size_t nb = (size_t)nc * (nc + 1) / 2 + 1;
    HIP_TRY(sbuf.alloc(8 * (size_t)ntiles + (size_t)ntiles * nc + 6 * (size_t)ne + 1 + 3 * (size_t)nc + 1 + nb + 8));
    if (!sint_host) {
      HIP_TRY(hipHostMalloc((void**)&sint_host, 8 * sizeof(int), hipHostMallocMapped));
      HIP_TRY(hipHostGetDevicePointer((void**)&sint_map, sint_host, 0));
    }
    int* p = sbuf.p;
    int4* ttot = reinterpret_cast<int4*>(p);  // first: 16-byte aligned
    p += 4 * (size_t)ntiles;
    int4* tcar = reinterpret_cast<int4*>(p);
    p += 4 * (size_t)ntiles;
    int* tcnt = p;
    p += (size_t)ntiles * nc;
    D.act = p, p += ne;
    D.pos_pt = p, p += ne;
    D.pcam = p, p += ne;
    D.cam_pos = p, p += ne;
    D.pt_id = p, p += ne;
    D.pt_off = p, p += ne + 1;
    D.chidx = p, p += nc;
    D.pose_cam = p, p += nc;
    D.cam_off = p, p += nc + 1;
    D.boff = p, p += nb;
    const uint8_t* fl = lvl < 0 ? nullptr : (const uint8_t*)c.flag.p;
    BaDev Ds = D;
    Ds.lm = gate;
    if (ntiles > 0)
      hipLaunchKernelGGL(k_ba_struct_count, dim3(ntiles), dim3(kTileT), sizeof(int) * (nc + kTileT / 64), st, Ds, fl,
                         lvl, tcnt, ttot);
    hipLaunchKernelGGL(k_ba_struct_scan, dim3(1), dim3(kStructNT), sizeof(int) * (nc + 1 + kStructNT / 64), st, Ds,
                       dfix, ntiles, tcnt, ttot, tcar, known ? p : sint_map);
    if (ntiles > 0)
      hipLaunchKernelGGL(k_ba_struct_fill, dim3(ntiles), dim3(kTileT),
                         sizeof(int) * ((1 + kTileT / 64) * (size_t)nc + kTileE + kTileT / 64), st, Ds, fl, lvl, tcnt,
                         tcar);
    return hipGetLastError();
  }

  // Sizes known: scratch allocations, readback block, Schur pair table.
  orbx_status finish_structure(int na, int npa, int nposes, int maxc, int nslots, hipStream_t st) {
#ifndef ORBX_GSPLIT_PPT
#define ORBX_GSPLIT_PPT 2
#endif
    constexpr int kPpt = ORBX_GSPLIT_PPT;  // ~positions per thread of a pose chunk
    const int gsplit = std::min(std::max((maxc + kPpt * kGB - 1) / (kPpt * kGB), 1), 64);
    const size_t N = 6 * (size_t)nposes;
    BA_CHECK(c.Hpl.alloc(18 * (size_t)na));
    BA_CHECK(c.ptc.alloc(12 * (size_t)na));
    BA_CHECK(c.cmc.alloc(kCmc * (size_t)na));
    BA_CHECK(c.BD.alloc(18 * (size_t)na));
    BA_CHECK(c.cf.alloc(6 * (size_t)na));
    BA_CHECK(c.Hll.alloc(9 * (size_t)npa));
    BA_CHECK(c.bl.alloc(3 * (size_t)npa));
    BA_CHECK(c.Dinv.alloc(9 * (size_t)npa));
    BA_CHECK(c.dmax_p.alloc(npa + nposes));
    BA_CHECK(c.Hpp.alloc(36 * (size_t)nposes));
    BA_CHECK(c.bp.alloc(N));
    if (!rb_ev) BA_CHECK(hipEventCreateWithFlags(&rb_ev, hipEventDisableTiming));
    BA_CHECK(c.xp.alloc(N));
    BA_CHECK(c.bs.alloc(N));
    BA_CHECK(c.S.alloc(N * N));
    D.na = na;
    D.npa = npa;
    D.nposes = nposes;
    D.nblk = nposes * (nposes + 1) / 2;
    D.gsplit = gsplit;
    BA_CHECK(c.gpart.alloc((size_t)(D.nblk * 36 + nposes * 6 + nposes * 27) * gsplit));  // pairs | rhs | camfold pose terms
    D.gpart = c.gpart.p;
    // readback block: scal[0..7], then errors partials (2 slots of nbe), then update partials
    D.nbe = std::max((na + LBS - 1) / LBS, 1);
    nbu = std::max((nposes + LBS - 1) / LBS + (npa + kUpPts - 1) / kUpPts, 1);  // k_ba_update: pose blocks, then point blocks
    D.nbu = nbu;
    n_rb = 8 + 2 * D.nbe + nbu;
    BA_CHECK(c.scal.alloc(n_rb));
    D.scal = c.scal.p;
    if (rb_cap < n_rb) {
      if (rb_host) (void)hipHostFree(rb_host);
      rb_host = nullptr;
      rb_cap = 0;
      BA_CHECK(hipHostMalloc((void**)&rb_host, n_rb * sizeof(double), hipHostMallocMapped));
      BA_CHECK(hipHostGetDevicePointer((void**)&rb_map, rb_host, 0));
      rb_cap = n_rb;
    }
    BA_CHECK(c.ptab.alloc(nslots));
    D.ptab = c.ptab.p;
    D.nbf = 0;
    D.pblk = nullptr;
    D.fused = 0;  // set on the device-LM copies only
    D.camfold = 0;
    D.posepart = D.bdfold = 0;
    D.gpose = nullptr;
    int npb = 0;  // the pblk blocks, run inside the pair-table launch
    if (fuse_ok && na > 0) {
      D.nbf = (na - 1) / kFuseStride + 1;
      BA_CHECK(pblk.alloc((size_t)D.nbf + 1));
      D.pblk = pblk.p;
      npb = npa / LBS + 1;
      const size_t ng = (size_t)D.nbf * nposes * kCmc;
      if (nposes > 0 && nposes <= kPosePartMaxPoses && ng <= kPosePartMaxDoubles) {
        BA_CHECK(c.gpose.alloc(ng));
        D.gpose = c.gpose.p;
      }
    }
    static_assert(kPB == LBS, "pblk blocks inside k_ba_pair_table");
    if (D.nblk + npb > 0) hipLaunchKernelGGL(k_ba_pair_table, dim3(D.nblk + npb, gsplit), dim3(kPB), 0, st, D);
    BA_CHECK(hipGetLastError());
    D.ptc = c.ptc.p;
    D.cmc = c.cmc.p;
    D.BD = c.BD.p;
    D.cf = c.cf.p;
    D.Dinv = c.Dinv.p;
    D.xp = c.xp.p;
    D.bs = c.bs.p;
    D.S = c.S.p;
    lin0 = LinSet{c.Hpl.p, c.Hll.p, c.bl.p, c.dmax_p.p, c.Hpp.p, c.bp.p};
    use_lin(D, lin0);
    return ORBX_OK;
  }

  hipError_t errors(hipStream_t st, int recompute, int dst) {
    hipLaunchKernelGGL(k_ba_errors, dim3(std::max((D.na + LBS - 1) / LBS, 1)), dim3(LBS), 0, st, D, recompute, dst);
    return hipGetLastError();
  }

  // One readback: out[2] ok flag, out[3] lambda-init max; out[0], out[1]
  // (chi of the two error slots) and out[4] (LM scale) are the block
  // partials added in block order.
  hipError_t read_scalars(double out[5], hipStream_t st) {
    hipError_t e = start_read(st);
    return e == hipSuccess ? finish_read(out) : e;
  }
  hipError_t start_read(hipStream_t st) {
    hipError_t e = hipMemcpyAsync(rb_host, D.scal, n_rb * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipEventRecord(rb_ev, st);
    return e;
  }
  hipError_t finish_read(double out[5]) {
    hipError_t e = wait_event(rb_ev);
    if (e != hipSuccess) return e;
    out[2] = rb_host[2];
    out[3] = rb_host[3];
    const double* p = rb_host + 8;
    double a = 0, b = 0, u = 0;
    for (int i = 0; i < D.nbe; i++) a += p[i];
    for (int i = 0; i < D.nbe; i++) b += p[D.nbe + i];
    for (int i = 0; i < nbu; i++) u += p[2 * D.nbe + i];
    out[0] = a;
    out[1] = b;
    out[4] = u;
    return hipSuccess;
  }

  // SparseOptimizer::optimize + OptimizationAlgorithmLevenberg::solve with the LM control on the
  // device: the entry linearisation and lambda init, then trials queued back to back --
  // (gated) linearisation, Schur, solve, update (which first pops a rejected
  // trial), errors, k_ba_lm_control -- with no host round trip between them,
  // and one gated restore when the phase ends on a rejection.  The host
  // queues as many trials as iterations remain (every trial ends at most one
  // iteration), reads the state back once, and queues more only after
  // rejections; a finished phase turns the queued rest into empty launches.
  LmState* lm_host = nullptr;  // pinned, mapped (lm_map: the device's view)
  LmState* lm_map = nullptr;
  // spec (optional): launches queued behind every readback of the phase (before its event), gated on
  // the device LM state (spec_skip) -- phase 1 queues phase 2's outlier marking and structure there
  orbx_status optimize_dev(int iterations, const StopFlag& stop, const DevStop& dstop, hipStream_t st, int* iters,
                           double* final_chi, const std::function<hipError_t()>& spec = nullptr) {
    const size_t N = 6 * (size_t)D.nposes;
    if (ldlt_np((int)N) > kLdltMaxNp) return ORBX_ERR_SIZE;
    LdltPlan ldlt;
    BA_CHECK(ldlt.prepare((int)N));
    D.ldlt_pan = ldlt.pan ? 1 : 0;
    if (!ldlt.col && !ldlt.in_lds) {
      BA_CHECK(c.Sw.alloc((size_t)ldlt_np((int)N) * ldlt_np((int)N)));
      D.Sw = c.Sw.p;
    }
    BA_CHECK(c.lm.alloc(1));
    if (!lm_host) {
      BA_CHECK(hipHostMalloc((void**)&lm_host, sizeof(LmState), hipHostMallocMapped));
      BA_CHECK(hipHostGetDevicePointer((void**)&lm_map, lm_host, 0));
    }
    const int gp = std::max((D.npa + D.nposes + LBS - 1) / LBS, 1);
    const int ga = std::max((D.na + LBS - 1) / LBS, 1);
    const int ge = std::max((D.na + LBS - 1) / LBS, 1);
    double sc[5] = {0, 0, 0, 0, 0};
    BaDev D0 = D;  // ungated: the entry launches and the final chi
    D0.lm = nullptr;
    BaDev Dg = D;
    Dg.lm = c.lm.p;
    Dg.fused = fused_mode(D.nbf, D.nposes);
    Dg.camfold = 1;
    set_trial_folds(Dg);
    int it = 0;
    if (!(stop())) {  // the loop head's first poll (i = 0)
      const bool fused = Dg.nbf > 0;
      if (fused) BA_CHECK(set_smem_attr((const void*)k_ba_lin_schur, kFuseSmem));
      // entry: errors, linearisation (point side through k_ba_lin_schur's entry mode when the
      // edges are point-grouped), pose sums, then cam_fin + lambda init + LM init in one launch
      hipLaunchKernelGGL(k_ba_errors, dim3(ge), dim3(LBS), 0, st, D0, 1, 0);
      if (fused) {
        BaDev De = D0;
        De.fused = 3;
        hipLaunchKernelGGL(k_ba_lin_schur, dim3(De.nbf), dim3(kFuseNT), kFuseSmem, st, De);
      } else {
        lin_points(D0, st);
      }
      if (D0.nposes > 0) hipLaunchKernelGGL(k_ba_cam_sum, dim3(D0.nposes, D0.gsplit), dim3(kGB), 0, st, D0);
      hipLaunchKernelGGL(k_ba_lm_start, dim3(1), dim3(1024), 0, st, Dg, iterations);
      BA_CHECK(hipGetLastError());
      const bool psfold = Dg.fused == 2;
      // a trial's errors and LM verdict: two launches by default.  The one-launch form
      // (k_ba_errors_ctl, debug option fused_ctl) pays an agent-scope release per block -- an L2
      // write-back on this multi-XCD part -- and measured 1.5-2.5 % slower per call (profiles/r06)
      const bool split_ctl = ba_opts().fused_ctl == 0;
      auto trial = [&](bool lin) {
        // linearisation gated on the device: only at the start of a new iteration
        if (fused && (lin || psfold)) hipLaunchKernelGGL(k_ba_lin_schur, dim3(Dg.nbf), dim3(kFuseNT), kFuseSmem, st, Dg);
        if (lin && !fused) lin_points(Dg, st);
        // (returns at once after k_ba_lin_schur: the point side of an iteration-start trial is done)
        if (!psfold) hipLaunchKernelGGL(k_ba_point_schur, dim3(ga), dim3(LBS), 0, st, Dg, 0.0);
        if (Dg.nposes > 0) {
          hipLaunchKernelGGL(k_ba_pairs, dim3(Dg.nblk + Dg.nposes, Dg.gsplit), dim3(kPB), 0, st, Dg);
          hipLaunchKernelGGL(k_ba_schur_fin, dim3(Dg.nblk + Dg.nposes), dim3(64), 0, st, Dg, 0.0);
          ldlt.launch(Dg, st);
        }
        hipLaunchKernelGGL(k_ba_update, dim3(Dg.nbu), dim3(LBS), 0, st, Dg, 0.0);
        if (split_ctl) {
          hipLaunchKernelGGL(k_ba_errors, dim3(ge), dim3(LBS), 0, st, Dg, 1, 1);
          hipLaunchKernelGGL(k_ba_lm_control, dim3(1), dim3(64), 0, st, Dg, dstop);
        } else {
          hipLaunchKernelGGL(k_ba_errors_ctl, dim3(Dg.nbe), dim3(LBS), 0, st, Dg, dstop);
        }
      };
      // (capturing the trial as a HIP graph and launching that instead measured slower on this
      // stack: 2.81 vs 2.76 ms per config-4 call)
      for (int budget = iterations, first = 1;; first = 0) {
        for (int t = 0; t < budget; t++) trial(!(first && t == 0));  // t = 0: linearised by the entry launches
        // the phase's final activeRobustChi2 of the stored errors rides on the same readback
        // (slot 0 is not read by the trials; a batch that did not finish recomputes it later); the
        // launch writes the readback block and the LM state into mapped memory itself
        BaDev Dr = D0;
        Dr.rb_out = rb_map;
        Dr.lm_out = lm_map;
        Dr.lm_copy = c.lm.p;
        hipLaunchKernelGGL(k_ba_errors, dim3(ge), dim3(LBS), 0, st, Dr, 0, 0);
        BA_CHECK(hipGetLastError());
        if (spec) BA_CHECK(spec());
        BA_CHECK(hipEventRecord(rb_ev, st));
        BA_CHECK(finish_read(sc));
        if (lm_host->refresh) {  // paused on a NaN-rho rejection: pop, errors at the restored state, resume
          hipLaunchKernelGGL(k_ba_restore, dim3(gp), dim3(LBS), 0, st, Dg);
          hipLaunchKernelGGL(k_ba_errors, dim3(ge), dim3(LBS), 0, st, Dg, 2, 0);
          hipLaunchKernelGGL(k_ba_lm_resume, dim3(1), dim3(64), 0, st, Dg);
          BA_CHECK(hipGetLastError());
        } else if (lm_host->done) {
          break;
        }
        budget = std::max(1, iterations - lm_host->it);
      }
      it = lm_host->it;
      trials += lm_host->trials;
      hook_stopped |= lm_host->stopped && D.raise_after >= 0;
      if (lm_host->rejected) {  // ended on a rejected trial: its pop (chi above reads errors only)
        hipLaunchKernelGGL(k_ba_restore, dim3(gp), dim3(LBS), 0, st, Dg);
        BA_CHECK(hipGetLastError());
      }
    } else {
      hipLaunchKernelGGL(k_ba_errors, dim3(ge), dim3(LBS), 0, st, D0, 0, 0);  // activeRobustChi2 of the stored errors
      BA_CHECK(hipGetLastError());
      BA_CHECK(read_scalars(sc, st));
    }
    *iters = it;
    if (final_chi) *final_chi = sc[0];
    return ORBX_OK;
  }

  // The stop flag as k_ba_lm_control sees it.  The handle's own flag (orbx_ba_stop_flag:
  // pinned, mapped) is read by the device directly.  Any other caller flag is never mapped or
  // registered: the device polls a pinned per-handle MIRROR, and the calling thread -- blocked
  // in the call anyway -- copies the caller's flag into it while it waits for the device
  // (wait_event).  So the device never holds an address whose page the caller may free or
  // remap, and no registration outlives the call (or is shared between handles).
  int* mirror = nullptr;  // pinned, mapped
  StopFlag mirror_src;    // the caller flag the mirror follows during a call (empty: none)
  bool map_stop(const StopFlag& s, DevStop* ds) {
    ds->i = nullptr;
    ds->b = nullptr;
    mirror_src = StopFlag{};
    if (!s.i && !s.b) return true;
    void* dp = nullptr;
    if (s.i && own_stop && (const void*)s.i == (const void*)own_stop) {
      if (hipHostGetDevicePointer(&dp, own_stop, 0) != hipSuccess) {
        (void)hipGetLastError();
        return false;
      }
      ds->i = (const int*)dp;
      return true;
    }
    if (!mirror) {
      if (hipHostMalloc((void**)&mirror, sizeof(int), hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        mirror = nullptr;
        return false;
      }
    }
    if (hipHostGetDevicePointer(&dp, mirror, 0) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    mirror_src = s;
    *(volatile int*)mirror = s() ? 1 : 0;
    ds->i = (const int*)dp;
    return true;
  }
  void unmap_stop() { mirror_src = StopFlag{}; }
  // hipEventSynchronize that keeps the device's view of the caller's stop flag current
  hipError_t wait_event(hipEvent_t ev) {
    if (!mirror_src.i && !mirror_src.b) return hipEventSynchronize(ev);
    for (;;) {
      const int v = mirror_src() ? 1 : 0;
      if (*(volatile int*)mirror != v) *(volatile int*)mirror = v;
      const hipError_t q = hipEventQuery(ev);
      if (q != hipErrorNotReady) return q;
      std::this_thread::yield();
    }
  }
};

// Problem intake: validation, the phase-1 sizes, one pinned-arena upload of
// the raw arrays and k_ba_prep (src/Optimizer.cc:603-745's graph assembly).
orbx_status ba_intake(LocalBA& L, const orbx_ba_problem* pb, hipStream_t st) {
  L.trials = 0;
  for (double& t : L.t_struct) t = 0;
  BaDev& D = L.D;
  // test hooks (off unless orbx_debug_ba_options set them): a NaN trial, a device-raised stop flag
  D.nan_trial = ba_opts().nan_trial;
  D.raise_after = ba_opts().raise_stop_after;
  Ctx& c = L.c;
  const int nc = pb->n_cams, np = pb->n_points, ne = pb->n_edges;
  D.nc = nc;
  D.np = np;
  D.ne = ne;
  // Index checks, point order and point count in one branch-free (vectorisable) pass; the camera
  // histogram in four interleaved counter sets (a run of one camera's edges does not serialise on one
  // counter).  The host pass sits on the call's critical path: the device waits for its upload.
  const int* ep = pb->edge_point;
  const int* ec = pb->edge_cam;
  int pmin = ne > 0 ? ep[0] : 0, pmax = pmin, cmin = ne > 0 ? ec[0] : 0, cmax = cmin, ord = 1, npts = ne > 0;
  for (int e = 1; e < ne; e++) {
    const int p = ep[e], q = ep[e - 1], c = ec[e];
    pmin = std::min(pmin, p);
    pmax = std::max(pmax, p);
    cmin = std::min(cmin, c);
    cmax = std::max(cmax, c);
    ord &= p >= q;
    npts += p != q;
  }
  if (ne > 0 && (pmin < 0 || pmax >= np || cmin < 0 || cmax >= nc)) return ORBX_ERR_ARG;
  const bool grouped = ord != 0;  // edges ordered by point (the reference adds them per MapPoint)
  // grouped: some point has more than kFuseMaxDeg positions <=> ep[e] == ep[e - kFuseMaxDeg] somewhere
  int long_run = 0;
  if (grouped)
    for (int e = kFuseMaxDeg; e < ne; e++) long_run |= ep[e] == ep[e - kFuseMaxDeg];
  L.ccnt.assign(nc, 0);
  L.ccnt4.assign(4 * (size_t)nc, 0);
  int* h = L.ccnt4.data();
  int e4 = 0;
  for (; e4 + 4 <= ne; e4 += 4) {
    h[ec[e4]]++;
    h[nc + ec[e4 + 1]]++;
    h[2 * nc + ec[e4 + 2]]++;
    h[3 * nc + ec[e4 + 3]]++;
  }
  for (; e4 < ne; e4++) h[ec[e4]]++;
  for (int i = 0; i < nc; i++) L.ccnt[i] = h[i] + h[nc + i] + h[2 * nc + i] + h[3 * nc + i];
  // the fused point side needs every point's positions inside one block (else the three kernels)
  L.fuse_ok = grouped && !long_run;
  // the structure on the device when the edges arrive grouped by point (else the host build)
  L.dev_struct = grouped && nc <= kStructMaxNc && (ne + kTileE - 1) / kTileE <= kStructMaxTiles;
  if (L.dev_struct) {  // phase-1 sizes: the launches need no readback
    int nposes = 0, maxc = 0;
    for (int i = 0; i < nc; i++)
      if (L.ccnt[i] && !(pb->fixed && pb->fixed[i])) {
        nposes++;
        maxc = std::max(maxc, L.ccnt[i]);
      }
    int nslots = 0;
    for (int i = 0, j = 0; i < nc; i++)
      if (L.ccnt[i] && !(pb->fixed && pb->fixed[i])) nslots += L.ccnt[i] * (nposes - j++);
    const int s1[5] = {ne, npts, nposes, maxc, nslots};
    std::memcpy(L.sizes1, s1, sizeof s1);
  }
  if (!L.dev_struct) {  // the host structure build reads them
    L.e_pt.assign(pb->edge_point, pb->edge_point + ne);
    L.e_cam.assign(pb->edge_cam, pb->edge_cam + ne);
  }
  L.fixed.assign(nc, 0);
  Arena& A = L.prob_arena;
  if (A.reserve(arena_bytes({32 * (size_t)nc, 24 * (size_t)nc, 40 * (size_t)nc, 12 * (size_t)np, 4 * (size_t)ne,
                             4 * (size_t)ne, 12 * (size_t)ne, 4 * (size_t)ne, (size_t)nc})) != hipSuccess)
    return ORBX_ERR_HIP;
  double* cq = A.take<double>(4 * (size_t)nc);
  double* ct = A.take<double>(3 * (size_t)nc);
  double* intr = A.take<double>(5 * (size_t)nc);
  float* Xf = A.take<float>(3 * (size_t)np);
  int* ept = A.take<int>(ne);
  int* ecam = A.take<int>(ne);
  float* obs_f = A.take<float>(3 * (size_t)ne);
  float* isig_f = A.take<float>(ne);
  uint8_t* dfix = A.take<uint8_t>(nc);
  L.dfix = dfix;
  // device-only FP64 / flag arrays, filled by k_ba_prep
  const size_t al = 256;
  auto rnd = [&](size_t b) { return (std::max<size_t>(b, 1) + al - 1) / al * al; };
  const size_t o_X = 0, o_eobs = o_X + rnd(24 * (size_t)np), o_einfo = o_eobs + rnd(24 * (size_t)ne),
               o_edelta = o_einfo + rnd(8 * (size_t)ne), o_edsqr = o_edelta + rnd(8 * (size_t)ne),
               o_est = o_edsqr + rnd(4 * (size_t)ne), o_erob = o_est + rnd(ne), o_end = o_erob + rnd(ne);
  BA_CHECK(c.prob.alloc(o_end));
  double* X = reinterpret_cast<double*>(c.prob.p + o_X);
  double* eobs = reinterpret_cast<double*>(c.prob.p + o_eobs);
  double* einfo = reinterpret_cast<double*>(c.prob.p + o_einfo);
  double* edelta = reinterpret_cast<double*>(c.prob.p + o_edelta);
  float* edsqr = reinterpret_cast<float*>(c.prob.p + o_edsqr);
  uint8_t* est = c.prob.p + o_est;
  uint8_t* erob = c.prob.p + o_erob;
  // vertices: Converter::toSE3Quat (float -> double, Quaterniond(R), normalize)
  {
    double* hq = A.host(cq);
    double* ht = A.host(ct);
    double* hi = A.host(intr);
    for (int i = 0; i < nc; i++) {
      const float* T = pb->Tcw + 12 * i;
      const double R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
      Quat q = mat2q(R);
      qnormalize(q);
      hq[4 * i] = q.x;
      hq[4 * i + 1] = q.y;
      hq[4 * i + 2] = q.z;
      hq[4 * i + 3] = q.w;
      ht[3 * i] = T[3];
      ht[3 * i + 1] = T[7];
      ht[3 * i + 2] = T[11];
      for (int k = 0; k < 5; k++) hi[5 * i + k] = pb->intr[5 * i + k];
      L.fixed[i] = pb->fixed ? pb->fixed[i] : 0;
      A.host(dfix)[i] = L.fixed[i];
    }
    if (np) std::memcpy(A.host(Xf), pb->Xw, 12 * (size_t)np);
    if (ne) {
      std::memcpy(A.host(ept), pb->edge_point, 4 * (size_t)ne);
      std::memcpy(A.host(ecam), pb->edge_cam, 4 * (size_t)ne);
      std::memcpy(A.host(obs_f), pb->obs, 12 * (size_t)ne);
      std::memcpy(A.host(isig_f), pb->inv_sigma2, 4 * (size_t)ne);
    }
  }
  BA_CHECK(A.upload(st));
  BA_CHECK(c.cbak.alloc(7 * (size_t)nc));
  BA_CHECK(c.Xbak.alloc(3 * (size_t)np));
  BA_CHECK(c.eerr.alloc(3 * (size_t)ne));
  {
    const float thMono = std::sqrt(5.991f), thStereo = std::sqrt(7.815f);  // src/Optimizer.cc:653-654
    const int gpre = (std::max(ne, 3 * np) + LBS - 1) / LBS;
    if (gpre > 0)
      hipLaunchKernelGGL(k_ba_prep, dim3(gpre), dim3(LBS), 0, st, ne, np, obs_f, isig_f, Xf, X, est, eobs, einfo,
                         edelta, edsqr, erob, c.eerr.p, thMono, thStereo);
    BA_CHECK(hipGetLastError());
  }
  BA_CHECK(c.flag.alloc(ne));
  BA_CHECK(c.scal.alloc(8));
  D.cq = cq;
  D.ct = ct;
  D.cbak = c.cbak.p;
  D.intr = intr;
  D.X = X;
  D.Xbak = c.Xbak.p;
  D.ept = ept;
  D.ecam = ecam;
  D.est = est;
  D.eobs = eobs;
  D.einfo = einfo;
  D.edelta = edelta;
  D.edsqr = edsqr;
  D.erobust = erob;
  D.eerr = c.eerr.p;
  D.scal = c.scal.p;
  return ORBX_OK;
}

// Write-back (src/Optimizer.cc:817-885): the erase list, poses and points, issued on st into the
// write-back arena; the caller syncs st, then ba_writeback_finish fills its arrays.
orbx_status ba_writeback(LocalBA& L, const orbx_ba_problem* pb, orbx_ba_result* res, bool ran, hipStream_t st) {
  BaDev& D = L.D;
  const int nc = pb->n_cams, np = pb->n_points, ne = pb->n_edges;
  const int ge = (ne + LBS - 1) / LBS;
  res->trials = L.trials;
  res->ran = ran ? 1 : 0;
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
  // :817-847 vToErase, then the poses and points; everything lands in the mapped write-back arena
  // (ba_writeback_finish moves it into the caller's arrays after the sync)
  Arena& A = L.wb_arena;
  BA_CHECK(A.reserve(arena_bytes({res->Tcw_d ? 12 * sizeof(double) * nc : 0, res->Xw_d ? 3 * sizeof(double) * np : 0,
                                  12 * sizeof(float) * nc, 3 * sizeof(float) * np, (size_t)ne})));
  LocalBA::Wb& w = L.wb;
  w.Tcw_d = res->Tcw_d ? A.take<double>(12 * (size_t)nc) : nullptr;
  w.Xw_d = res->Xw_d ? A.take<double>(3 * (size_t)np) : nullptr;
  w.Tcw = A.take<float>(12 * (size_t)nc);
  w.Xw = A.take<float>(3 * (size_t)np);
  w.flag = A.take<uint8_t>((size_t)ne);
  if (ne > 0) hipLaunchKernelGGL(k_ba_outliers, dim3(ge), dim3(LBS), 0, st, D, w.flag, 0);
  const int gx = (std::max(nc, np) + LBS - 1) / LBS;
  hipLaunchKernelGGL(k_ba_export, dim3(std::max(gx, 1)), dim3(LBS), 0, st, D, w.Tcw, w.Xw, w.Tcw_d, w.Xw_d);
  BA_CHECK(hipGetLastError());
  return ORBX_OK;
}

// After the stream has synchronised: the write-back arena's pinned copy into the caller's arrays.
void ba_writeback_finish(LocalBA& L, const orbx_ba_problem* pb, orbx_ba_result* res, bool ran) {
  if (!ran) return;
  const int nc = pb->n_cams, np = pb->n_points, ne = pb->n_edges;
  Arena& A = L.wb_arena;
  const LocalBA::Wb& w = L.wb;
  if (ne > 0) std::memcpy(res->edge_outlier, A.host(w.flag), ne);
  std::memcpy(res->Tcw, A.host(w.Tcw), 12 * sizeof(float) * nc);
  std::memcpy(res->Xw, A.host(w.Xw), 3 * sizeof(float) * np);
  if (res->Tcw_d) std::memcpy(res->Tcw_d, A.host(w.Tcw_d), 12 * sizeof(double) * nc);
  if (res->Xw_d) std::memcpy(res->Xw_d, A.host(w.Xw_d), 3 * sizeof(double) * np);
}

orbx_status run_local_ba(LocalBA& L, const orbx_ba_problem* pb, orbx_ba_result* res, const StopFlag& stop,
                         hipStream_t st) {
  double host_build_ms = 0;
  const auto t_start = std::chrono::steady_clock::now();
  // host-side marks for the trace line: intake, phase-1 structure, phase 1, phase-2 structure, phase 2
  std::chrono::steady_clock::time_point tm[5];
  for (auto& t : tm) t = t_start;
  orbx_status s0 = ba_intake(L, pb, st);
  if (s0 != ORBX_OK) return s0;
  tm[0] = std::chrono::steady_clock::now();
  BaDev& D = L.D;
  Ctx& c = L.c;
  const int ne = pb->n_edges;
  res->iterations[0] = res->iterations[1] = 0;
  res->trials = 0;
  res->chi2[0] = res->chi2[1] = 0;
  const int ge = (ne + LBS - 1) / LBS;
  bool ran = false;
  // LM control on the device; the stop flag it polls lives in pinned, device-mapped memory
  DevStop dstop{nullptr, nullptr};
  L.unmap_stop();
  L.hook_stopped = false;
  if (!L.map_stop(stop, &dstop)) return ORBX_ERR_HIP;
  auto optimize = [&](int iterations, int* iters, double* chi, const std::function<hipError_t()>& spec = nullptr) {
    return L.optimize_dev(iterations, stop, dstop, st, iters, chi, spec);
  };
  // phase 2's outlier marking and structure, queued behind phase 1's readback and gated on its LM
  // state (spec_skip): when phase 1 ends on an accepted state the one readback also brings phase
  // 2's sizes, so the call pays one host round trip between the phases instead of two
#ifndef ORBX_BA_SPEC2
#define ORBX_BA_SPEC2 1
#endif
  const bool spec2 = ORBX_BA_SPEC2 && L.dev_struct && ne > 0;
  BaDev Dspec = D;  // (filled below, after the phase-1 structure)
  auto spec = [&]() -> hipError_t {
    // the gate is read here, not when Dspec is filled: optimize_dev allocates the LM state on a
    // handle's first call, after the phase-1 structure (an ungated launch would run mid-phase)
    if (!c.lm.p) return hipErrorInvalidValue;
    Dspec.lm = c.lm.p;
    hipLaunchKernelGGL(k_ba_outliers, dim3(ge), dim3(LBS), 0, st, Dspec, c.flag.p, 1);
    HIP_TRY(hipGetLastError());
    return L.launch_structure_dev(0, st, nullptr, c.lm.p);
  };
  if (!(stop())) {  // src/Optimizer.cc:749-751
    ran = true;
    if (!L.dev_struct) L.level.assign(ne, 0);
    const auto tb0 = std::chrono::steady_clock::now();
    orbx_status s = L.build_structure(-1, st);
    const auto tb1 = std::chrono::steady_clock::now();
    host_build_ms += std::chrono::duration<double, std::milli>(tb1 - tb0).count();
    tm[1] = tb1;
    if (s != ORBX_OK) return s;
    Dspec = D;
    s = optimize(5, &res->iterations[0], &res->chi2[0], spec2 ? std::function<hipError_t()>(spec) : nullptr);
    if (s != ORBX_OK) return s;
    // did the speculative phase-2 launches run (phase 1 ended done, nothing to pop or refresh)?
    const bool spec_ran = spec2 && L.lm_host->done && !L.lm_host->refresh && !L.lm_host->rejected;
    tm[2] = tm[3] = tm[4] = std::chrono::steady_clock::now();
    if (!(stop()) && !L.hook_stopped) {
      // :764-802 level-1 outliers, drop robust kernels (already done on the device when spec_ran)
      if (ne > 0 && !spec_ran) hipLaunchKernelGGL(k_ba_outliers, dim3(ge), dim3(LBS), 0, st, D, c.flag.p, 1);
      BA_CHECK(hipGetLastError());
      if (!L.dev_struct) {
        BA_CHECK(hipMemcpyAsync(L.level.data(), c.flag.p, ne, hipMemcpyDeviceToHost, st));
        BA_CHECK(hipStreamSynchronize(st));
      }
      const auto tb2 = std::chrono::steady_clock::now();
      if (spec_ran) {
        const int* sz = L.sint_host;  // written by the speculative k_ba_struct_scan before the readback's event
        s = L.finish_structure(sz[0], sz[1], sz[2], sz[3], sz[4], st);
      } else {
        s = L.build_structure(0, st);
      }
      tm[3] = std::chrono::steady_clock::now();
      host_build_ms += std::chrono::duration<double, std::milli>(tm[3] - tb2).count();
      if (s != ORBX_OK) return s;
      s = optimize(10, &res->iterations[1], &res->chi2[1]);
      if (s != ORBX_OK) return s;
      tm[4] = std::chrono::steady_clock::now();
    }
  }
  BA_CHECK(ba_writeback(L, pb, res, ran, st));
  L.unmap_stop();
  if (!ran) return ORBX_OK;
  BA_CHECK(hipStreamSynchronize(st));
  ba_writeback_finish(L, pb, res, ran);
  if (ba_opts().trace) {
    const auto t_end = std::chrono::steady_clock::now();
    auto d = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    std::fprintf(stderr,
                 "[orbx_ba] total %.3f ms, structure %.3f ms (host index %.3f, host poses %.3f, device %.3f, upload %.3f), "
                 "iterations %d+%d, trials %d; host marks: intake %.3f, struct1 %.3f, phase1 %.3f, struct2 %.3f, "
                 "phase2 %.3f, writeback %.3f ms\n",
                 d(t_start, t_end), host_build_ms, L.t_struct[0], L.t_struct[1], L.t_struct[2], L.t_struct[3],
                 res->iterations[0], res->iterations[1], res->trials, d(t_start, tm[0]), d(tm[0], tm[1]),
                 d(tm[1], tm[2]), d(tm[2], tm[3]), d(tm[3], tm[4]), d(tm[4], t_end));
  }
  return ORBX_OK;
}

// ---- batched driver: K independent problems through the same launches ----
// Every trial kernel runs once for all K problems (blockIdx.z), each block on
// its own problem's arrays and LM state; grids span the largest problem and
// the smaller ones' extra blocks return at once.  Per problem the arithmetic,
// partitions and reduction orders are those of the single-problem device LM
// loop, so every problem's result is bit-identical to running it alone.
struct BaBatch {
  DBuf<BaDev> dev;       // [Dg_0..Dg_K-1, D0_0..D0_K-1]
  DBuf<LmState> lm;      // K
  LmState* lm_host = nullptr;
  int cap = 0;
  std::vector<BaDev> hostD;
  ~BaBatch() {
    if (lm_host) (void)hipHostFree(lm_host);
  }
};

orbx_status optimize_many(LocalBA* const* Ls, int K, BaBatch& B, int iterations, const StopFlag& stop,
                          const DevStop& dstop, hipStream_t st, int* iters, double* chis) {
  int Nmax = 0, gaM = 1, gpM = 1, geM = 1, gnpM = 1, nbpM = 0, gsM = 1, nposM = 0, nbfM = 0, n_unfused = 0;
  for (int i = 0; i < K; i++) {
    const BaDev& D = Ls[i]->D;
    nbfM = std::max(nbfM, D.nbf);
    n_unfused += D.nbf > 0 ? 0 : 1;
    Nmax = std::max(Nmax, 6 * D.nposes);
    gaM = std::max(gaM, (D.na + LBS - 1) / LBS);
    gpM = std::max(gpM, D.nbu);
    geM = std::max(geM, D.nbe);
    gnpM = std::max(gnpM, (D.npa + LBS - 1) / LBS);
    nbpM = std::max(nbpM, D.nblk + D.nposes);
    gsM = std::max(gsM, D.gsplit);
    nposM = std::max(nposM, D.nposes);
  }
  // each problem takes the LDLT kernel a single call would (bit-identical results): the panel
  // kernel for the small systems, the column-step one (or the MFMA-blocked opt-in) for the rest
  int Npan = 0, Ncol = 0;
  for (int i = 0; i < K; i++) {
    const int Ni = 6 * Ls[i]->D.nposes;
    if (ldlt_use_pan(Ni)) Npan = std::max(Npan, Ni); else Ncol = std::max(Ncol, Ni);
  }
  LdltPlan ldlt, lpan;
  if (Ncol > 0 || Npan == 0) {
    BA_CHECK(ldlt.prepare(std::max(Ncol, 6), false));
    if (!ldlt.col) return ORBX_ERR_SIZE;  // the caller runs the problems one by one
    BA_CHECK(ldlt.prepare_many());
  }
  if (Npan > 0) {
    BA_CHECK(lpan.prepare(Npan));
    if (!lpan.pan) return ORBX_ERR_SIZE;
    BA_CHECK(lpan.prepare_many());
  }
  const bool camfold = true;
  int n_ps = 0, n_psfold = 0;  // problems that launch k_ba_point_schur / whose k_ba_lin_schur takes it
  if (B.cap < K) {
    if (B.lm_host) (void)hipHostFree(B.lm_host);
    B.lm_host = nullptr;
    B.cap = 0;
    BA_CHECK(hipHostMalloc((void**)&B.lm_host, sizeof(LmState) * K, hipHostMallocDefault));
    B.cap = K;
  }
  BA_CHECK(B.lm.alloc(K));
  BA_CHECK(B.dev.alloc(2 * (size_t)K));
  B.hostD.resize(2 * (size_t)K);
  for (int i = 0; i < K; i++) {
    B.hostD[i] = Ls[i]->D;
    B.hostD[i].lm = B.lm.p + i;
    B.hostD[i].fused = fused_mode(B.hostD[i].nbf, B.hostD[i].nposes);
    n_ps += B.hostD[i].fused == 2 ? 0 : 1;
    n_psfold += B.hostD[i].fused == 2 ? 1 : 0;
    B.hostD[i].camfold = camfold ? 1 : 0;
    set_trial_folds(B.hostD[i]);
    B.hostD[i].ldlt_pan = ldlt_use_pan(6 * B.hostD[i].nposes) ? 1 : 0;
    B.hostD[K + i] = Ls[i]->D;
    B.hostD[K + i].lm = nullptr;
  }
  BA_CHECK(hipMemcpyAsync(B.dev.p, B.hostD.data(), sizeof(BaDev) * 2 * K, hipMemcpyHostToDevice, st));
  const BaDev* Dg = B.dev.p;
  const BaDev* D0 = B.dev.p + K;
  if (nbfM > 0)
    BA_CHECK(set_smem_attr((const void*)k_ba_lin_schur_many, kFuseSmem));
  // the entry launches (D0: no LM state, nothing fused) and the gated trials: per problem either
  // k_ba_lin_schur or the three separate kernels do the point side (each returns for the other)
  auto linearize = [&](const BaDev* Ds) {
    const bool gated = Ds == Dg;
    if (gated && nbfM > 0) hipLaunchKernelGGL(k_ba_lin_schur_many, dim3(nbfM, 1, K), dim3(kFuseNT), kFuseSmem, st, Ds);
    if (!gated || n_unfused > 0) {
      hipLaunchKernelGGL(k_ba_linearize_many, dim3(gaM, 1, K), dim3(LBS), 0, st, Ds);
      hipLaunchKernelGGL(k_ba_point_sum_many, dim3(gnpM, 1, K), dim3(LBS), 0, st, Ds);
    }
    if (nposM > 0 && !(gated && camfold)) {
      hipLaunchKernelGGL(k_ba_cam_sum_many, dim3(nposM, gsM, K), dim3(kGB), 0, st, Ds);
      hipLaunchKernelGGL(k_ba_cam_fin_many, dim3(nposM, 1, K), dim3(64), 0, st, Ds);
    }
  };
  for (int i = 0; i < K; i++) iters[i] = 0;
  if (!(stop())) {
    hipLaunchKernelGGL(k_ba_errors_many, dim3(geM, 1, K), dim3(LBS), 0, st, D0, 1, 0);
    linearize(D0);
    hipLaunchKernelGGL(k_ba_dmax_many, dim3(1, 1, K), dim3(1024), 0, st, D0);
    hipLaunchKernelGGL(k_ba_lm_init_many, dim3(1, 1, K), dim3(64), 0, st, Dg, iterations);
    BA_CHECK(hipGetLastError());
    for (int budget = iterations, first = 1;; first = 0) {
      for (int t = 0; t < budget; t++) {
        if (!(first && t == 0))
          linearize(Dg);  // gated per problem
        else if (n_psfold > 0)
          hipLaunchKernelGGL(k_ba_lin_schur_many, dim3(nbfM, 1, K), dim3(kFuseNT), kFuseSmem, st, Dg);
        if (n_ps > 0) hipLaunchKernelGGL(k_ba_point_schur_many, dim3(gaM, 1, K), dim3(LBS), 0, st, Dg, 0.0);
        if (nposM > 0) {
          hipLaunchKernelGGL(k_ba_pairs_many, dim3(nbpM, gsM, K), dim3(kPB), 0, st, Dg);
          hipLaunchKernelGGL(k_ba_schur_fin_many, dim3(nbpM, 1, K), dim3(64), 0, st, Dg, 0.0);
          if (Npan > 0) lpan.launch_many(Dg, K, st);
          if (Ncol > 0) ldlt.launch_many(Dg, K, st);
        }
        hipLaunchKernelGGL(k_ba_update_many, dim3(gpM, 1, K), dim3(LBS), 0, st, Dg, 0.0);
        hipLaunchKernelGGL(k_ba_errors_many, dim3(geM, 1, K), dim3(LBS), 0, st, Dg, 1, 1);
        hipLaunchKernelGGL(k_ba_lm_control_many, dim3(1, 1, K), dim3(64), 0, st, Dg, dstop);
      }
      hipLaunchKernelGGL(k_ba_errors_many, dim3(geM, 1, K), dim3(LBS), 0, st, D0, 0, 0);
      hipLaunchKernelGGL(k_ba_lm_final_many, dim3(1, 1, K), dim3(64), 0, st, Dg);
      BA_CHECK(hipGetLastError());
      BA_CHECK(hipMemcpyAsync(B.lm_host, B.lm.p, sizeof(LmState) * K, hipMemcpyDeviceToHost, st));
      BA_CHECK(hipEventRecord(Ls[0]->rb_ev, st));
      BA_CHECK(Ls[0]->wait_event(Ls[0]->rb_ev));  // keeps the device's stop mirror current
      int left = 0;
      bool refresh = false;
      for (int i = 0; i < K; i++) {
        if (!B.lm_host[i].done || B.lm_host[i].refresh) left = std::max(left, iterations - B.lm_host[i].it);
        refresh |= B.lm_host[i].refresh != 0;
      }
      if (left == 0) break;
      if (refresh) {  // problems paused on a NaN-rho rejection (all three launches gated per problem)
        hipLaunchKernelGGL(k_ba_restore_many, dim3(gpM, 1, K), dim3(LBS), 0, st, Dg);
        hipLaunchKernelGGL(k_ba_errors_many, dim3(geM, 1, K), dim3(LBS), 0, st, Dg, 2, 0);
        hipLaunchKernelGGL(k_ba_lm_resume_many, dim3(1, 1, K), dim3(64), 0, st, Dg);
        BA_CHECK(hipGetLastError());
      }
      budget = std::max(1, left);
    }
    bool rej = false;
    for (int i = 0; i < K; i++) {
      iters[i] = B.lm_host[i].it;
      Ls[i]->trials += B.lm_host[i].trials;
      chis[i] = B.lm_host[i].final_chi;
      rej |= B.lm_host[i].rejected != 0;
    }
    if (rej) {  // the pops of problems that ended on a rejected trial (gated per problem)
      hipLaunchKernelGGL(k_ba_restore_many, dim3(gpM, 1, K), dim3(LBS), 0, st, Dg);
      BA_CHECK(hipGetLastError());
    }
  } else {
    hipLaunchKernelGGL(k_ba_errors_many, dim3(geM, 1, K), dim3(LBS), 0, st, D0, 0, 0);
    hipLaunchKernelGGL(k_ba_lm_final_many, dim3(1, 1, K), dim3(64), 0, st, Dg);
    BA_CHECK(hipGetLastError());
    BA_CHECK(hipMemcpyAsync(B.lm_host, B.lm.p, sizeof(LmState) * K, hipMemcpyDeviceToHost, st));
    BA_CHECK(hipStreamSynchronize(st));
    for (int i = 0; i < K; i++) chis[i] = B.lm_host[i].final_chi;
  }
  return ORBX_OK;
}

// K LocalBundleAdjustment calls at once: per-problem intake and structure,
// each LM phase batched, per-problem write-back.  Problems that need the host
// structure build or a reduced system beyond the column-step kernel run one
// by one instead (same results).
orbx_status run_local_ba_many(LocalBA* const* Ls, int K, BaBatch& B, const orbx_ba_problem* pbs,
                              orbx_ba_result* ress, const StopFlag& stop, hipStream_t st) {
  for (int i = 0; i < K; i++) {
    orbx_status s = ba_intake(*Ls[i], &pbs[i], st);
    if (s != ORBX_OK) return s;
  }
  DevStop dstop{nullptr, nullptr};
  for (int i = 0; i < K; i++) Ls[i]->unmap_stop();
  if (!Ls[0]->map_stop(stop, &dstop)) return ORBX_ERR_HIP;
  bool batch = true;
  for (int i = 0; i < K; i++) batch &= Ls[i]->dev_struct;
  if (!batch) {  // one by one (intake again inside: the arenas are reused)
    for (int i = 0; i < K; i++) {
      orbx_status s = run_local_ba(*Ls[i], &pbs[i], &ress[i], stop, st);
      if (s != ORBX_OK) return s;
    }
    return ORBX_OK;
  }
  std::vector<int> it(K);
  std::vector<double> chi(K);
  for (int i = 0; i < K; i++) {
    ress[i].iterations[0] = ress[i].iterations[1] = 0;
    ress[i].trials = 0;
    ress[i].chi2[0] = ress[i].chi2[1] = 0;
  }
  bool ran = false;
  if (!(stop())) {  // src/Optimizer.cc:749-751
    ran = true;
    for (int i = 0; i < K; i++) BA_CHECK(Ls[i]->build_structure(-1, st));
    orbx_status s = optimize_many(Ls, K, B, 5, stop, dstop, st, it.data(), chi.data());
    if (s == ORBX_ERR_SIZE) {  // reduced system beyond the column-step kernel: one by one
      for (int i = 0; i < K; i++) {
        s = run_local_ba(*Ls[i], &pbs[i], &ress[i], stop, st);
        if (s != ORBX_OK) return s;
      }
      return ORBX_OK;
    }
    if (s != ORBX_OK) return s;
    bool hook = false;
    for (int i = 0; i < K; i++) {
      ress[i].iterations[0] = it[i];
      ress[i].chi2[0] = chi[i];
      hook |= B.lm_host[i].stopped && Ls[i]->D.raise_after >= 0;
    }
    if (!(stop()) && !hook) {
      for (int i = 0; i < K; i++) {  // :764-802 level-1 outliers, drop robust kernels
        const int ne = pbs[i].n_edges;
        if (ne > 0)
          hipLaunchKernelGGL(k_ba_outliers, dim3((ne + LBS - 1) / LBS), dim3(LBS), 0, st, Ls[i]->D, Ls[i]->c.flag.p, 1);
        BA_CHECK(hipGetLastError());
      }
      for (int i = 0; i < K; i++) BA_CHECK(Ls[i]->build_structure(0, st));
      s = optimize_many(Ls, K, B, 10, stop, dstop, st, it.data(), chi.data());
      if (s != ORBX_OK) return s;
      for (int i = 0; i < K; i++) {
        ress[i].iterations[1] = it[i];
        ress[i].chi2[1] = chi[i];
      }
    }
  }
  for (int i = 0; i < K; i++) BA_CHECK(ba_writeback(*Ls[i], &pbs[i], &ress[i], ran, st));
  Ls[0]->unmap_stop();
  BA_CHECK(hipStreamSynchronize(st));
  for (int i = 0; i < K; i++) ba_writeback_finish(*Ls[i], &pbs[i], &ress[i], ran);
  return ORBX_OK;
}

}  // namespace orbx

namespace orbx {
constexpr orbx_ba_debug_options kBaOptsDefault = {ORBX_BA_LDLT_AUTO, -1, -1, 0, 0};
thread_local const orbx_ba_debug_options* t_ba_opts = nullptr;
inline const orbx_ba_debug_options& ba_opts() { return t_ba_opts ? *t_ba_opts : kBaOptsDefault; }
struct BaOptScope {  // the handle's options for this call on this thread
  const orbx_ba_debug_options* prev;
  explicit BaOptScope(const orbx_ba_debug_options* o) : prev(t_ba_opts) { t_ba_opts = o; }
  ~BaOptScope() { t_ba_opts = prev; }
};
}  // namespace orbx

struct orbx_ba {
  int device = 0;
  hipStream_t st = nullptr;
  orbx_ba_debug_options opts = orbx::kBaOptsDefault;
  orbx::LocalBA L;
  std::vector<std::unique_ptr<orbx::LocalBA>> more;  // orbx_ba_run_many: problems 1..K-1
  orbx::BaBatch batch;
};

extern "C" {

orbx_status orbx_ba_create_priority(int device, int priority, orbx_ba** out) {
  if (!out) return ORBX_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= n) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  orbx_ba* h = new (std::nothrow) orbx_ba();
  if (!h) return ORBX_ERR_HIP;
  h->device = device;
  hipError_t e;
  if (priority == 0) {
    e = hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking);
  } else {
    int least = 0, greatest = 0;
    e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e == hipSuccess) {
      const int p = std::min(std::max(priority, std::min(least, greatest)), std::max(least, greatest));
      e = hipStreamCreateWithPriority(&h->st, hipStreamNonBlocking, p);
    }
  }
  if (e != hipSuccess) {
    delete h;
    return ORBX_ERR_HIP;
  }
  *out = h;
  return ORBX_OK;
}

orbx_status orbx_ba_create(int device, orbx_ba** out) { return orbx_ba_create_priority(device, 0, out); }

orbx_status orbx_stream_create(int device, const uint32_t* cu_mask, int cu_mask_words, void** stream) {
  if (!stream || cu_mask_words < 0 || (cu_mask_words > 0 && !cu_mask)) return ORBX_ERR_ARG;
  *stream = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ORBX_ERR_NODEV;
  if (device < 0 || device >= n) return ORBX_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return ORBX_ERR_HIP;
  hipStream_t st = nullptr;
  const hipError_t e = cu_mask_words > 0 ? hipExtStreamCreateWithCUMask(&st, (uint32_t)cu_mask_words, cu_mask)
                                         : hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e != hipSuccess) return ORBX_ERR_HIP;
  *stream = (void*)st;
  return ORBX_OK;
}

void orbx_stream_destroy(void* stream) {
  if (!stream) return;
  (void)hipStreamSynchronize((hipStream_t)stream);
  (void)hipStreamDestroy((hipStream_t)stream);
}

orbx_status orbx_ba_create_masked(int device, const uint32_t* cu_mask, int cu_mask_words, orbx_ba** out) {
  if (!out) return ORBX_ERR_ARG;
  *out = nullptr;
  void* st = nullptr;
  const orbx_status s = orbx_stream_create(device, cu_mask, cu_mask_words, &st);
  if (s != ORBX_OK) return s;
  orbx_ba* h = new (std::nothrow) orbx_ba();
  if (!h) {
    orbx_stream_destroy(st);
    return ORBX_ERR_HIP;
  }
  h->device = device;
  h->st = (hipStream_t)st;
  *out = h;
  return ORBX_OK;
}

orbx_status orbx_ba_run_many(orbx_ba* h, int n, const orbx_ba_problem* problems, orbx_ba_result* results,
                             const volatile int* stop_flag) {
  if (!h || n < 0 || (n > 0 && (!problems || !results))) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  for (int i = 0; i < n; i++) {
    const orbx_ba_problem* p = &problems[i];
    const orbx_ba_result* r = &results[i];
    if (p->n_cams < 0 || p->n_points < 0 || p->n_edges < 0 || (p->n_cams > 0 && (!p->Tcw || !p->intr)) ||
        (p->n_points > 0 && !p->Xw) ||
        (p->n_edges > 0 && (!p->edge_point || !p->edge_cam || !p->obs || !p->inv_sigma2 || !r->edge_outlier)) ||
        (p->n_cams > 0 && !r->Tcw) || (p->n_points > 0 && !r->Xw))
      return ORBX_ERR_ARG;
  }
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  while ((int)h->more.size() < n - 1) {
    h->more.emplace_back(new (std::nothrow) orbx::LocalBA());
    if (!h->more.back()) {
      h->more.pop_back();
      return ORBX_ERR_HIP;
    }
  }
  std::vector<orbx::LocalBA*> Ls(n);
  Ls[0] = &h->L;
  for (int i = 1; i < n; i++) Ls[i] = h->more[i - 1].get();
  orbx::BaOptScope scope(&h->opts);
  orbx::StopFlag sf;
  sf.i = stop_flag;
  return orbx::run_local_ba_many(Ls.data(), n, h->batch, problems, results, sf, h->st);
}

int orbx_debug_ba_options(orbx_ba* h, const orbx_ba_debug_options* o) {
  if (!h) return ORBX_ERR_ARG;
  if (o && (o->ldlt < ORBX_BA_LDLT_AUTO || o->ldlt > ORBX_BA_LDLT_BLOCKED)) return ORBX_ERR_ARG;
  h->opts = o ? *o : orbx::kBaOptsDefault;
  return ORBX_OK;
}

orbx_status orbx_ba_stop_flag(orbx_ba* h, volatile int** flag) {
  if (!h || !flag) return ORBX_ERR_ARG;
  if (!h->L.own_stop) {
    (void)hipSetDevice(h->device);
    if (hipHostMalloc((void**)&h->L.own_stop, sizeof(int), hipHostMallocMapped) != hipSuccess) {
      h->L.own_stop = nullptr;
      return ORBX_ERR_HIP;
    }
    *h->L.own_stop = 0;
  }
  *flag = h->L.own_stop;
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
  orbx::BaOptScope scope(&h->opts);
  orbx::StopFlag f;
  f.i = stop_flag;
  return orbx::run_local_ba(h->L, p, r, f, h->st);
}

orbx_status orbx_ba_run_bool(orbx_ba* h, const orbx_ba_problem* p, orbx_ba_result* r, const volatile bool* stop_flag) {
  if (!h || !p || !r) return ORBX_ERR_ARG;
  if (p->n_cams < 0 || p->n_points < 0 || p->n_edges < 0) return ORBX_ERR_ARG;
  if (p->n_cams > 0 && (!p->Tcw || !p->intr || !r->Tcw)) return ORBX_ERR_ARG;
  if (p->n_points > 0 && (!p->Xw || !r->Xw)) return ORBX_ERR_ARG;
  if (p->n_edges > 0 && (!p->edge_point || !p->edge_cam || !p->obs || !p->inv_sigma2 || !r->edge_outlier))
    return ORBX_ERR_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return ORBX_ERR_HIP;
  orbx::BaOptScope scope(&h->opts);
  orbx::StopFlag f;
  f.b = stop_flag;
  return orbx::run_local_ba(h->L, p, r, f, h->st);
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

// Debug/benchmark probe (include/orbx_debug.h): solve S x = b (N = 6 * nposes)
// with the LocalBA LDLT kernel; ms = average kernel time over reps launches.
#ifdef ORBX_LS_PROBE
extern "C" int orbx_debug_ls_probe(unsigned long long* out) {  // 1024 x 8 words (probe build only)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_ls_probe), sizeof(unsigned long long) * 1024 * 8) == hipSuccess ? 0 : -3;
}
#endif
extern "C" int orbx_debug_ldlt(const double* S, const double* b, int N, double* x, int reps, float* ms) {
  return orbx_debug_ldlt_ex(S, b, N, x, reps, ms, ORBX_BA_LDLT_AUTO, nullptr);
}

extern "C" int orbx_debug_ldlt_ex(const double* S, const double* b, int N, double* x, int reps, float* ms, int kind,
                                  unsigned long long* stamps) {
  if (!S || !b || !x || N <= 0 || N % 6 || reps < 1) return ORBX_ERR_ARG;
  if (kind < ORBX_BA_LDLT_AUTO || kind > ORBX_BA_LDLT_BLOCKED) return ORBX_ERR_ARG;
  orbx_ba_debug_options o = orbx::kBaOptsDefault;
  o.ldlt = kind;
  orbx::BaOptScope scope(&o);
  const int stage_limit = 99;
  orbx::BaDev D{};
  D.nposes = N / 6;
  double *dS = nullptr, *dS0 = nullptr, *db = nullptr, *dx = nullptr, *dscal = nullptr;
  const size_t nn = (size_t)N * N * sizeof(double);
  hipEvent_t e0, e1;
  hipError_t e = hipMalloc((void**)&dS, nn);
  if (e == hipSuccess) e = hipMalloc((void**)&dS0, nn);
  if (e == hipSuccess) e = hipMalloc((void**)&db, N * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&dx, N * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&dscal, 8 * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dS0, S, nn, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(db, b, N * sizeof(double), hipMemcpyHostToDevice);
  D.S = dS;
  D.bs = db;
  D.xp = dx;
  D.scal = dscal;
  unsigned long long* ddbg = nullptr;
  const bool want_ts = stamps != nullptr;
  if (e == hipSuccess && want_ts) {
    e = hipMalloc((void**)&ddbg, 64 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(ddbg, 0, 64 * sizeof(unsigned long long));
  }
  D.dbg = ddbg;
  if (orbx::ldlt_np(N) > orbx::kLdltMaxNp) e = hipErrorInvalidValue;
  orbx::LdltPlan plan;
  if (e == hipSuccess) e = plan.prepare(N);
  D.ldlt_pan = plan.pan ? 1 : 0;
  double* dSw = nullptr;
  if (e == hipSuccess && !plan.col && !plan.in_lds)
    e = hipMalloc((void**)&dSw, (size_t)orbx::ldlt_np(N) * orbx::ldlt_np(N) * sizeof(double));
  D.Sw = dSw;
  float total = 0;
  if (e == hipSuccess) {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int r = 0; r < reps && e == hipSuccess; r++) {
      e = hipMemcpy(dS, dS0, nn, hipMemcpyDeviceToDevice);
      (void)hipEventRecord(e0, nullptr);
      plan.launch(D, nullptr, stage_limit);
      (void)hipEventRecord(e1, nullptr);
      if (e == hipSuccess) e = hipEventSynchronize(e1);
      float t = 0;
      (void)hipEventElapsedTime(&t, e0, e1);
      total += t;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  double ok = 0;
  if (e == hipSuccess) e = hipMemcpy(x, dx, N * sizeof(double), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(&ok, dscal + 2, sizeof(double), hipMemcpyDeviceToHost);
  if (ms) *ms = total / reps;
  (void)hipFree(dS);
  (void)hipFree(dS0);
  (void)hipFree(db);
  (void)hipFree(dx);
  (void)hipFree(dscal);
  if (dSw) (void)hipFree(dSw);
  if (ddbg) {
    // the kernel's s_memtime stamps (LDLT_TS points; 0 = not reached) of the last launch
    if (hipMemcpy(stamps, ddbg, 64 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
      e = hipErrorUnknown;
    (void)hipFree(ddbg);
  }
  if (e != hipSuccess) return ORBX_ERR_HIP;
  return ok != 0.0 ? ORBX_OK : ORBX_ERR_STATE;
}
