/*
 * orb_oracle.h -- C ABI of the CPU ORACLE (test infrastructure only).
 *
 * THIS IS NOT THE PRODUCT.  It is a single-threaded C++ restatement of the
 * reference's hot path used as the parity checker by tests/, by
 * __graft_entry__.smoke() and as the `cpu_baseline` leg of bench.py.  Nothing
 * under orb_slam2_commit_amd/ may include, link or call it.
 *
 * Parity status: the reference (qpc001/ORB_SLAM2_Commit) needs OpenCV, Eigen
 * and the missing g2o/DBoW2 .cpp sources and cannot be built here, and it
 * ships no tests, fixtures or golden vectors.  The
 * oracle is therefore "parity unpinned" against the genuine binary; it is
 * pinned instead by independent known-answer tests in tests/ (FAST-9 segment
 * test by brute force, Gaussian kernel integers, resize coefficients,
 * fastAtan2 vs atan2, popcount vs numpy) and by the committed fixtures it
 * generated (tests/golden/).
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint layout (28 bytes). */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} oracle_keypoint;

typedef struct {
  int nfeatures;
  float scale_factor;
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
} oracle_params;

/* Scale tables (ORBextractor ctor, src/ORBextractor.cc:416-490). Arrays of nlevels. */
int oracle_scale_tables(const oracle_params* p, float* scale, float* inv_scale,
                        float* sigma2, float* inv_sigma2, int* features_per_level);

/* Full ORBextractor::operator() (src/ORBextractor.cc:1138-1211).
 * pyramid_out (optional): concatenation of the nlevels level images, each
 * w_l*h_l bytes, row-major, no padding; level sizes written to level_wh (2*nlevels).
 * Returns number of keypoints, or <0 on error (-2: cap too small). */
int oracle_extract(const oracle_params* p, const uint8_t* img, int w, int h, size_t stride,
                   oracle_keypoint* kps, int cap, uint8_t* desc,
                   uint8_t* pyramid_out, size_t pyramid_cap, int* level_wh);

/* Stage probes for unit tests. */
int oracle_resize_linear(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh);
int oracle_gaussian_blur7(const uint8_t* src, int w, int h, uint8_t* dst);
/* FAST-9 with NMS on a window (OpenCV FAST_t<16> semantics). Writes packed
 * (score<<24 | y<<12 | x) in emission order; returns count. */
int oracle_fast_window(const uint8_t* img, int w, int h, size_t stride, int threshold,
                       uint32_t* out, int cap);
int oracle_fast_score(const uint8_t* img, size_t stride, int x, int y);
float oracle_fast_atan2(float y, float x);
float oracle_cosf(float x);
float oracle_sinf(float x);

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1844-1860). */
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);
void oracle_hamming_pairs(const uint8_t* a, const uint8_t* b, int n, int32_t* d);

/* Frame::ComputeStereoMatches (src/Frame.cc:547-788).
 * pyrL/pyrR: pyramids in oracle_extract's pyramid_out layout. */
int oracle_stereo_match(const oracle_params* p,
                        const oracle_keypoint* kpsL, const uint8_t* descL, int nL,
                        const oracle_keypoint* kpsR, const uint8_t* descR, int nR,
                        const uint8_t* pyrL, const uint8_t* pyrR, const int* level_wh,
                        float bf, float baseline, float* uRight, float* depth);

/* One side of SearchByBoW: descriptors, keypoint angles, MapPoint validity
 * (NULL = all valid) and its DBoW2::FeatureVector as CSR (ascending node ids). */
typedef struct {
  int n;
  const uint8_t* desc;
  const float* angle;
  const uint8_t* valid;
  int n_nodes;
  const uint32_t* node_id;
  const int32_t* node_off;
  const int32_t* feat;
} oracle_bow_side;

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&), src/ORBmatcher.cc:175-325.
 * match_f[f->n] = KF feature index matched to each frame feature, or -1. Returns nmatches. */
int oracle_search_by_bow_kf_f(const oracle_bow_side* kf, const oracle_bow_side* f, float nnratio, int check_ori,
                              int32_t* match_f);
/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&), src/ORBmatcher.cc:589-736.
 * match12[kf1->n] = KF2 feature index or -1. Returns nmatches. */
int oracle_search_by_bow_kf_kf(const oracle_bow_side* kf1, const oracle_bow_side* kf2, float nnratio, int check_ori,
                               int32_t* match12);
/* ORBmatcher::ComputeThreeMaxima, src/ORBmatcher.cc:1797-1839 (on bin counts). */
void oracle_three_maxima(const int* counts, int L, int* ind1, int* ind2, int* ind3);

/* Optimizer::LocalBundleAdjustment (src/Optimizer.cc:530-885) on g2o semantics.
 * Cameras: Tcw row-major 3x4 float (KeyFrame::GetPose), fixed flag (local KF
 * with mnId==0 or fixed camera), intrinsics fx,fy,cx,cy,bf (float).  Points:
 * world positions float.  Edges: point, camera, obs (u, v, ur; ur < 0 ->
 * monocular EdgeSE3ProjectXYZ, else EdgeStereoSE3ProjectXYZ) and invSigma2 of
 * the keypoint octave. */
typedef struct {
  int n_cams;
  const float* Tcw;
  const uint8_t* fixed;
  const float* intr;
  int n_points;
  const float* Xw;
  int n_edges;
  const int32_t* edge_point;
  const int32_t* edge_cam;
  const float* obs;
  const float* inv_sigma2;
} oracle_ba_problem;

typedef struct {
  float* Tcw;             /* n_cams x 12 */
  float* Xw;              /* n_points x 3 */
  uint8_t* edge_outlier;  /* n_edges: (KF, MapPoint) pair to erase (:817-847) */
  double* Tcw_d;          /* optional double copies (NULL to skip) */
  double* Xw_d;
  int iterations[2];      /* LM iterations of optimize(5) / optimize(10) */
  int trials;             /* LM inner trials in total */
  double chi2[2];         /* active robust chi2 at the end of each phase */
} oracle_ba_result;

int oracle_local_ba(const oracle_ba_problem* p, oracle_ba_result* r, const volatile int* stop_flag);

/* Test probes: EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ computeError +
 * linearizeOplus at (q xyzw, t, X); A = d err/d X (rows of 3), B = d err/d
 * pose (rows of 6, pose update exp(u) * T, u = (omega, upsilon)). */
void oracle_ba_edge_probe(const double q[4], const double t[3], const double X[3], const double intr[5], int stereo,
                          const double obs[3], double err[3], double A[9], double B[18]);
/* exp(u) * T (SE3Quat::exp, operator*, normalizeRotation). */
void oracle_se3_exp_mul(const double u[6], const double q[4], const double t[3], double q_out[4], double t_out[3]);

/* PnPsolver (src/PnPsolver.cc:67-1101).  Correspondences in ctor gather
 * order; SetRansacParameters(probability, minInliers, maxIterations, minSet,
 * epsilon, th2) applied at creation. */
typedef struct oracle_pnp oracle_pnp;
oracle_pnp* oracle_pnp_create(int n, const float* p3d, const float* p2d, const float* sigma2, float fx, float fy,
                              float cx, float cy, double probability, int min_inliers, int max_iterations,
                              int min_set, float epsilon, float th2);
void oracle_pnp_destroy(oracle_pnp* h);
void oracle_pnp_params(const oracle_pnp* h, int* min_inliers, int* max_its, float* epsilon);
/* iterate(nIterations, bNoMore, vbInliers, nInliers) over caller rand() values
 * (consumed count in *used); returns 1 if a pose is returned, 0 if not, -1
 * if rand_vals ran out. */
int oracle_pnp_iterate(oracle_pnp* h, int nIterations, const int32_t* rand_vals, int n_rand, int* used,
                       int* bNoMore, float Tcw[16], uint8_t* inliers, int* nInliers);
/* EPnP compute_pose probe; returns the reprojection error. */
double oracle_epnp(const double* pws, const double* us, int n, double fu, double fv, double uc, double vc, double* R,
                   double* t);
/* cvSVD probe on an m x n matrix (m >= n): left vectors as rows, w, Vt. */
void oracle_svd(const double* A, int m, int n, double* Ut, double* w, double* Vt);

/* SearchByProjection (src/ORBmatcher.cc:46-142, 1489-1646, 1648-1795); layout
 * identical to orbx_proj_frame / orbx_proj_problem in include/orbx.h. */
typedef struct {
  int n;
  const oracle_keypoint* keys_un;
  const uint8_t* desc;
  const float* u_right;
  const int8_t* occ;
  float min_x, max_x, min_y, max_y;
  float grid_inv_w, grid_inv_h;
  int nlevels;
  float scale_factors[16];
  float inv_level_sigma2[16];
  float log_scale_factor;
  float fx, fy, cx, cy, bf, b;
  float Tcw[16];
  float grid_min_x, grid_min_y;  /* the grid's bounds when grid_min_set (a KeyFrame: the Frame's float
                                    mnMinX/mnMinY, while min_x/min_y are its integer copies) */
  int grid_min_set;
} oracle_proj_frame;

typedef struct {
  int kind, frustum;
  oracle_proj_frame f;
  int n_points;
  const uint8_t* desc;
  const uint8_t* flags;
  const float* pos;
  const float* normal;
  const float* dist_minmax;
  const float* angle;
  const int32_t* octave;
  float* track;
  int32_t* track_level;
  float th, nnratio, view_cos_limit;
  int check_ori, mono, orb_dist;
  float last_Tcw[16];
  int32_t* frame_out;
  int32_t* point_match;
  int32_t* nmatches;
} oracle_proj_problem;

int oracle_search_by_projection(const oracle_proj_problem* p);

/* ORBmatcher::SearchBySim3 (src/ORBmatcher.cc:1238-1487); layout identical to orbx_sim3_problem. */
typedef struct {
  oracle_proj_frame kf1, kf2;
  const uint8_t* desc1;
  const float* pos1;
  const float* dist_minmax1;
  const uint8_t* flags1;
  const uint8_t* desc2;
  const float* pos2;
  const float* dist_minmax2;
  const uint8_t* flags2;
  float s12;
  float R12[9];
  float t12[3];
  float th;
  int32_t* match12;
  int32_t* nfound;
} oracle_sim3_problem;

int oracle_search_by_sim3(const oracle_sim3_problem* p);

/* ORBmatcher::SearchForInitialization (src/ORBmatcher.cc:442-587); layout identical to
 * orbx_init_problem. */
typedef struct {
  oracle_proj_frame f1, f2;
  float* prev_matched;
  int window;
  float nnratio;
  int check_ori;
  int32_t* match12;
  int32_t* nmatches;
} oracle_init_problem;

int oracle_search_for_initialization(const oracle_init_problem* p);

/* Optimizer::PoseOptimization (src/Optimizer.cc:287-528); layout identical to
 * orbx_pose_problem in include/orbx.h. */
typedef struct {
  int n;
  const float* obs;
  const float* Xw;
  const float* inv_sigma2;
  float fx, fy, cx, cy, bf;
  float Tcw[16];
  float* Tcw_out;
  uint8_t* outlier;
  int32_t* ngood;
  int32_t* iterations;
} oracle_pose_problem;
int oracle_pose_optimization(const oracle_pose_problem* p);

/* ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:738-925); layout
 * identical to orbx_tri_problem in include/orbx.h. */
typedef struct {
  int n;
  const oracle_keypoint* keys_un;
  const uint8_t* desc;
  const float* u_right;
  const uint8_t* has_mp;
  int n_nodes;
  const uint32_t* node_id;
  const int32_t* node_off;
  const int32_t* feat;
} oracle_tri_kf;
typedef struct {
  oracle_tri_kf kf1, kf2;
  float F12[9];
  float C1w[3];
  float T2w[16];
  float fx, fy, cx, cy;
  float scale_factors2[16];
  float level_sigma2_2[16];
  int only_stereo, check_ori;
  int32_t* match12;
  int32_t* nmatches;
} oracle_tri_problem;
int oracle_search_for_triangulation(const oracle_tri_problem* p);
/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:249-320), batched:
 * point p's observed descriptors are desc[obs_off[p] .. obs_off[p+1]). */
void oracle_distinctive_descriptors(const uint8_t* desc, const int32_t* obs_off, int n_points, int32_t* best,
                                    uint8_t* out_desc);
/* Frame::UndistortKeyPoints (src/Frame.cc:471-506) via cvUndistortPoints (OpenCV 3.2). */
void oracle_undistort_point(const float K[9], const float* dist, int n_dist, float x, float y, float* xo, float* yo);
void oracle_undistort_keypoints(const oracle_keypoint* keys, int n, const float K[9], const float* dist, int n_dist,
                                oracle_keypoint* keys_un);
void oracle_pose_edge_probe(const double q[4], const double t[3], const double X[3], const double intr[5], int stereo,
                            const double obs[3], double err[3], double J[18]);
int oracle_ldlt6(const double* H, const double* b, double* x);
float oracle_log_det(float x);
int oracle_predict_scale(float max_distance, float dist, float log_sf, int nlevels);
int oracle_features_in_area(const oracle_proj_frame* f, float x, float y, float r, int minLevel, int maxLevel,
                            int32_t* out, int cap);

#ifdef __cplusplus
}
#endif
#endif
